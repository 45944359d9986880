"""The JNI shim (jni/) against the C ABI and its Java class, CPU tier.

No JDK is in this image: jni/Makefile builds the shim where JAVA_HOME is
set.  Here the C file is compiled (gcc -Wall -Wextra -Werror) against
tests/native/jni_spec/jni.h, the subset of the JNI specification's types
and function table it uses, and run under a fake JNIEnv
(tests/native/jni_harness.c): without a GPU, create throws IOException,
buffers shorter than their batch throw IllegalArgumentException before the
library is called, and compileUpstream leaves the caller's buffer as it was
(the GPU tier runs the same harness against the C ABI,
tests/test_gpu_abi_c.py).  These checks also keep the three files
consistent: every native method GpuClassifier.java declares has its
Java_..._<name> export in the C file and vice versa, and every vc_* function
the shim calls is declared in include/vclassify.h (and exported by
libvclassify.so, test_capi_symbols.py).
"""
import os
import re
import subprocess

from vproxy_amd._lib import header_symbols

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JNI = os.path.join(ROOT, "jni")


def _read(name):
    with open(os.path.join(JNI, name)) as f:
        return f.read()


def test_java_natives_match_c_exports():
    java = _read("GpuClassifier.java")
    c = _read("vproxy_component_secure_GpuClassifier.c")
    natives = set(re.findall(r"public static native [\w\[\]]+ (\w+)\(", java))
    exports = set(re.findall(r"Java_vproxy_component_secure_GpuClassifier_(\w+)", c))
    assert natives and natives == exports


def test_shim_calls_only_header_functions():
    c = _read("vproxy_component_secure_GpuClassifier.c")
    called = set(re.findall(r"\b(vc_[a-z0-9_]+)\s*\(", c))
    assert called <= set(header_symbols()), called - set(header_symbols())
    # the shim's sequence for the drain-loop batch and the metrics endpoint
    assert {"vc_create", "vc_pipeline", "vc_counters_prometheus", "vc_host_register"} <= called


def test_shim_compiles_and_runs_under_fake_jnienv():
    native = os.path.join(ROOT, "tests", "native")
    subprocess.check_call(["make", "-s", "-C", native, "build/jni_harness"])
    r = subprocess.run([os.path.join(native, "build", "jni_harness"), "cpu"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "JNI OK" in r.stdout, r.stdout + r.stderr


def _java_consts(name, keys):
    src = _read(name)
    out = {}
    for k in keys:
        m = re.search(r"\b%s = (-?\d+)" % k, src)
        assert m, (name, k)
        out[k] = int(m.group(1))
    return out


def test_java_layouts_and_statuses_match_the_header():
    """The Java side packs vclassify.h structs and switches on its status
    codes by number (jni/GpuContext.java, DnsDrainBatcher.java,
    SwitchDrainBatcher.java): the numbers must be the C ones."""
    import ctypes as C
    from vproxy_amd import _lib as L
    sizes = _java_consts("GpuContext.java", ["NET_BYTES", "ACL_RULE_BYTES", "ANNOS_BYTES",
                                             "GROUP_ANNOS_BYTES"])
    assert sizes == {"NET_BYTES": C.sizeof(L.VcNet), "ACL_RULE_BYTES": C.sizeof(L.VcAclRule),
                     "ANNOS_BYTES": C.sizeof(L.VcAnnos),
                     "GROUP_ANNOS_BYTES": C.sizeof(L.VcGroupAnnos)}
    hdr = open(os.path.join(ROOT, "include", "vclassify.h")).read()
    cdef = lambda k: int(re.search(r"#define %s\s+\(?(-?\d+)" % k, hdr).group(1))
    dns = _java_consts("DnsDrainBatcher.java", ["ANSWER", "RECURSIVE", "RESPONSE", "REJECTED",
                                                "EMPTY", "MALFORMED", "HOST", "MAXQ"])
    for k, v in dns.items():
        assert v == cdef("VC_DNSD_" + k), k
    sw = _java_consts("SwitchDrainBatcher.java", ["PKT_OK", "PKT_EXCEPTION", "PKT_LOOP",
                                                  "LAYER_VXLAN"])
    assert sw == {"PKT_OK": cdef("VC_PKT_OK"), "PKT_EXCEPTION": cdef("VC_PKT_EXCEPTION"),
                  "PKT_LOOP": cdef("VC_PKT_LOOP"), "LAYER_VXLAN": cdef("VC_LAYER_VXLAN")}


def test_fallback_contract_in_java_matches_the_shim():
    """GpuContext.call keys its fallback on the exceptions the shim throws:
    IOException (VC_EDEVICE / VC_ENOMEM) marks the context dead,
    IllegalStateException (VC_ESTATE) is per call; the shim maps them so
    (tests/native/jni_harness.c injects each status)."""
    ctx = _read("GpuContext.java")
    body = ctx[ctx.index("public boolean call("):]
    body = body[:body.index("\n    }\n")]
    assert "catch (IllegalStateException" in body and "catch (IOException" in body
    assert body.index("catch (IOException") < body.index("dead = true")
    shim = _read("vproxy_component_secure_GpuClassifier.c")
    assert 'VC_ESTATE    ? "java/lang/IllegalStateException"' in shim
    # -Dclassifier=gpu selection, loaded as PosixFDs loads vfdposix
    cfg = _read("ClassifierConfig.java")
    assert 'getSystemProperty("classifier", "java")' in cfg
    assert "System.loadLibrary(lib)" in _read("GpuClassifier.java")
