"""CPU tier: guards on the gfx950 code the hot kernels compile to.

Throughput of these kernels depends on code generation as much as on the
source: in round 3 the same two-quad ACL source ran 0.62 ms in one build and
0.83 ms in the next (profiles/r03_ab_acl_quads.txt), and the kernel then
carried a 96-byte private segment -- the ACL context struct spilled to
scratch because it was indexed with a runtime list number.  This test reads
the code objects `make` builds (build/obj/device/*.o: the .hip_fatbin
section, unbundled for gfx950 with clang-offload-bundler) and checks, per
hot kernel, from the AMDGPU metadata and the disassembly:

- private segment size 0 and no VGPR spills: no scratch traffic (SGPR
  spills go to VGPR lanes through v_writelane / v_readlane, which the
  private segment size would show if they reached memory);
- VGPRs within what the launch keeps resident (4 waves per SIMD for the
  1024-thread pipeline workgroup and two 512-thread ACL workgroups per CU);
- the hint / DNS / DNS drain-loop kernels make no call (no `s_swappc`):
  their rare paths run in follow-up kernels;
- the two-quad ACL kernel's lockstep search loop issues its 8 LDS reads
  (two quads of four tuples) per step with one branch, and the one-quad
  loop 4 (acl_v4_four in device/classify.hip).
No GPU is needed: hipcc cross-compiles for gfx950 here.
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "build", "obj", "device")
LLVM = "/opt/rocm/lib/llvm/bin"


def _code_object(name, tmp_path):
    subprocess.check_call(["make", "-s", "-j8", "-C", os.path.join(ROOT, "vproxy_amd", "csrc")])
    fb, co = tmp_path / (name + ".fatbin"), tmp_path / (name + ".co")
    subprocess.check_call([LLVM + "/llvm-objcopy", "--dump-section", ".hip_fatbin=%s" % fb,
                           os.path.join(OBJ, name + ".o"), str(tmp_path / (name + ".tmp"))])
    subprocess.check_call([LLVM + "/clang-offload-bundler", "--unbundle", "--type=o",
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--input=%s" % fb,
                           "--output=%s" % co])
    return str(co)


def _kernels(co):
    """kernel name -> metadata fields"""
    notes = subprocess.check_output([LLVM + "/llvm-readelf", "--notes", co], text=True)
    out = {}
    for blk in notes.split("  - .agpr_count")[1:]:
        get = lambda k: re.search(r"\.%s:\s+(\S+)" % k, blk).group(1)
        out[get("name")] = {k: int(get(k)) for k in (
            "private_segment_fixed_size", "vgpr_count", "vgpr_spill_count", "sgpr_spill_count",
            "group_segment_fixed_size")}
    return out


def _functions(co):
    """kernel name -> list of (address, instruction text)"""
    dis = subprocess.check_output([LLVM + "/llvm-objdump", "-d", "--no-show-raw-insn", co],
                                  text=True)
    funcs = {}
    for part in re.split(r"\n(?=[0-9a-f]+ <)", dis):
        m = re.match(r"[0-9a-f]+ <([^>]+)>:", part)
        if not m:
            continue
        ins = []
        for line in part.split("\n")[1:]:
            a = re.search(r"//\s*([0-9A-Fa-f]{8,}):", line)
            if a:
                ins.append((int(a.group(1), 16), line.split("//")[0].strip()))
        funcs[m.group(1)] = ins
    return funcs


def _loops(ins):
    """(first address, last address) of every backward branch's body"""
    loops = []
    for addr, text in ins:
        m = re.match(r"s_(?:cbranch_\w+|branch)\s+(\d+)", text)
        if m:
            simm = int(m.group(1))
            if simm >= 0x8000:
                loops.append((addr + 4 + 4 * (simm - 0x10000), addr))
    return loops


def _one(d, part):
    hits = [k for k in d if part in k]
    assert len(hits) == 1, (part, hits)
    return hits[0]


HOT = {   # kernel (mangled-name fragment) -> VGPR ceiling of its launch
    "pipeline_v4_kernelILb1ELb1ELb1E": 128,   # C5: LDS ACL, vector, counting
    "pipeline_v4_kernelILb1ELb1ELb0E": 128,
    "pipeline_mix_kernelILb1ELb1ELb1ELb0E": 128,
    "pipeline_mix_kernelILb1ELb1ELb1ELb1E": 128,   # compact IPv6 rows
    "acl_v4_kernelILb1ELi2E": 128,            # C2 (two quads per lane)
    "acl_v4_kernelILb1ELi1E": 128,
    "13acl_v6_kernelE": 128,
    "15route_v4_kernelE": 128,
    "route_v6_kernel_x4": 128,
    "bucket_scatter_kernelILb1E": 128,
    "bucket_hist_kernel": 128,
    "bucket_count_kernelILb1E": 128,
    "hist_kernelILb1E": 128,
}

# string kernels without a call in their loops (device/hint.hip: rare lanes
# go to a follow-up kernel); a call site there brought back a private
# segment, scratch spills of the loop state and SGPR spills on every chunk
# (VGPR bound, spilled dwords allowed)
HOT_STRING = {
    "hint_kernelILb1ELb1ELb0E": (72, 0),      # 7 waves per SIMD
    "hint_kernelILb1ELb1ELb1E": (72, 3),      # the uri-aware instance (c4uri)
    "dns_kernelILb1ELb1E": (80, 0),           # 6
    "dnsd_kernelILb1ELb1E": (96, 0),          # 5 waves per SIMD, in-place qnames
}


# frame and mirror kernels of round 6 (bind-port ACL image, bit-set mirrors)
HOT_FRAME = {
    "switch_kernelILb1ELb1EE": 128,
    "switch_kernelILb1ELb0EE": 128,
    "mirror_switch_kernelILb1ELb1ELb1EE": 128,
    "mirror_match_kernelILb1ELb1EE": 128,
}


def test_hot_kernels_use_no_scratch(tmp_path):
    k = _kernels(_code_object("classify", tmp_path))
    k.update(_kernels(_code_object("counters", tmp_path)))
    f = _kernels(_code_object("packet", tmp_path))
    f.update(_kernels(_code_object("mirror", tmp_path)))
    for part, vmax in HOT_FRAME.items():
        m = f[_one(f, part)]
        assert m["private_segment_fixed_size"] == 0, (part, m)
        assert m["vgpr_spill_count"] == 0, (part, m)
        assert m["vgpr_count"] <= vmax, (part, m)
        # LDS within the 5 workgroups per CU these latency-bound kernels keep
        assert m["group_segment_fixed_size"] <= 160 * 1024 // 5, (part, m)
    for part, vmax in HOT.items():
        name = _one(k, part)
        m = k[name]
        assert m["private_segment_fixed_size"] == 0, (part, m)
        assert m["vgpr_spill_count"] == 0, (part, m)
        assert m["vgpr_count"] <= vmax, (part, m)


def test_string_kernels_have_no_call_in_their_loops(tmp_path):
    co = _code_object("hint", tmp_path)
    k = _kernels(co)
    f = _functions(co)
    for part, (vmax, spill) in HOT_STRING.items():
        name = _one(k, part)
        m = k[name]
        assert m["private_segment_fixed_size"] <= 4 * spill + 4 * bool(spill), (part, m)
        assert m["vgpr_spill_count"] <= spill, (part, m)
        assert m["vgpr_count"] <= vmax, (part, m)
        ins = f[_one(f, part)]
        assert not any(t.startswith("s_swappc") for _, t in ins), part


@pytest.mark.parametrize("quads", [1, 2])
def test_acl_lockstep_loop_shape(tmp_path, quads):
    co = _code_object("classify", tmp_path)
    f = _functions(co)
    ins = f[_one(f, "acl_v4_kernelILb1ELi%dE" % quads)]
    assert not any(t.startswith("scratch_") for _, t in ins)
    loops = []
    for lo, hi in _loops(ins):
        body = [t for a, t in ins if lo <= a <= hi]
        loops.append((sum(t.startswith("ds_read") for t in body),
                      sum(t.startswith("s_cbranch") for t in body),
                      sum(t.startswith(("global_load", "flat_load")) for t in body)))
    # the lockstep search: 4 LDS reads per quad per step, one branch, no
    # memory loads (the record loads follow the loop)
    assert (4 * quads, 1, 0) in loops, loops
