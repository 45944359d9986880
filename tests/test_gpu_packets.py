"""GPU tier: header extraction (device/packet.hip) through the C ABI against
the oracle (vo_parse_packet, the vpacket parsers' restatement), bit-exact on
every output field; the reference's TestPacket vectors; host and device
entry points; and parse -> SecurityGroup composition on the outputs."""
import json
import os

import numpy as np
import pytest

import oracle_ffi as O
import vproxy_amd as V
from cases import gen_frames

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def clf():
    c = V.Classifier(0)
    yield c
    c.close()


def _rows(res, i):
    l3 = int(res["l3"][i])
    if l3 == 6:
        src, dst = bytes(res["src6"][i]).hex(), bytes(res["dst6"][i]).hex()
    else:
        src = int(res["src4"][i]).to_bytes(4, "big").hex()
        dst = int(res["dst4"][i]).to_bytes(4, "big").hex()
    return {"status": int(res["status"][i]), "l3": l3, "l4": int(res["l4"][i]),
            "proto": int(res["proto"][i]), "vni": int(res["vni"][i]),
            "ether_type": int(res["ether_type"][i]), "src": src, "dst": dst,
            "sport": int(res["sport"][i]), "dport": int(res["dport"][i])}


def test_testpacket_vectors_on_gpu(clf):
    with open(os.path.join(G, "packets.json")) as f:
        cases = json.load(f)["cases"]
    for c in cases:
        res = clf.parse_packets([bytes.fromhex(c["hex"])], c["layer"])
        got = _rows(res, 0)
        for k, v in c["want"].items():
            assert got[k] == v, (c["name"], k, got[k], v)


@pytest.mark.parametrize("layer,cut", [(0, 0), (1, 8), (4, 22), (6, 22)])
def test_frames_vs_oracle(clf, layer, cut):
    import torch
    frames = [f[cut:] for f in gen_frames(np.random.default_rng(17 + layer), 30000)]
    res = clf.parse_packets(frames, layer)
    want = [O.parse_packet(f, layer) for f in frames]
    for i, w in enumerate(want):
        assert _rows(res, i) == w, (i, frames[i].hex())
    # device entry point on a device blob: same bytes
    lens = np.array([len(f) for f in frames], np.int64)
    off = np.zeros(len(frames) + 1, np.int64)
    off[1:] = np.cumsum(lens)
    blob = torch.from_numpy(np.frombuffer(b"".join(frames), np.uint8).copy()).cuda()
    dres = clf.parse_packets((blob, torch.from_numpy(off.astype(np.int32)).cuda()), layer)
    torch.cuda.synchronize()
    for k in res:
        np.testing.assert_array_equal(dres[k].cpu().numpy().view(res[k].dtype), res[k], err_msg=k)


def test_parse_then_classify(clf):
    """Frames -> (proto, src4, dport) -> SecurityGroup.allow: the parse
    outputs feed the ACL entry point directly."""
    from vproxy_amd import workloads as W
    tcp, udp = W.gen_sg_rules(300, 33)
    a, na, ka = W.as_ctypes(tcp, V._lib.VcAclRule)
    b, nb, kb = W.as_ctypes(udp, V._lib.VcAclRule)
    V.check(V.lib().vc_compile_acl(clf.h, a, na, b, nb, 0))
    frames = gen_frames(np.random.default_rng(99), 20000)
    res = clf.parse_packets(frames, 0)
    ok = (res["status"] == 0) & (res["l3"] == 4) & (res["l4"] == 6)
    assert ok.sum() > 1000
    idx, allow = clf.acl_v4(res["proto"][ok], res["src4"][ok], res["dport"][ok])
    want, wv = O.sg_batch_v4_np(tcp, udp, False, res["proto"][ok], res["src4"][ok],
                                res["dport"][ok])
    np.testing.assert_array_equal(idx, want)
    np.testing.assert_array_equal(allow, wv)


@pytest.mark.parametrize("shift,pad", [(1, 0), (0, 1400), (3, 1400)])
def test_unstaged_paths(clf, shift, pad):
    """The kernel's global-memory parse: an unaligned blob (no LDS stage) and
    waves of jumbo frames whose span exceeds the per-wave stage."""
    import torch
    rng = np.random.default_rng(70 + shift + pad)
    frames = [f + bytes(int(rng.integers(0, pad + 1))) if pad else f
              for f in gen_frames(rng, 5000)]
    want = [O.parse_packet(f, 0) for f in frames]
    lens = np.array([len(f) for f in frames], np.int64)
    off = np.zeros(len(frames) + 1, np.int64)
    off[1:] = np.cumsum(lens)
    b = np.concatenate([np.zeros(shift, np.uint8), np.frombuffer(b"".join(frames), np.uint8)])
    blob = torch.from_numpy(b).cuda()[shift:]
    res = clf.parse_packets((blob, torch.from_numpy(off.astype(np.int32)).cuda()), 0)
    torch.cuda.synchronize()
    res = {k: v.cpu().numpy() for k, v in res.items()}
    for k in ("src6", "dst6"):
        res[k] = res[k].view(np.uint8)
    for k in ("src4", "dst4", "vni"):
        res[k] = res[k].view(np.uint32)
    for k in ("sport", "dport", "ether_type"):
        res[k] = res[k].view(np.uint16)
    for i, w in enumerate(want):
        assert _rows(res, i) == w, (i, frames[i][:80].hex())


def test_ragged_batch_sizes(clf):
    """Chunk boundaries of the staged kernels: each wave takes the next
    chunk's offsets one chunk ahead and the span's end from the last live
    lane (stage.h span_of), so batches of 1, 63, 64, 65, 127, 129 frames and
    one that leaves a partial chunk after a full grid stride are checked
    against the oracle (the switch, mirror and DNS-datagram kernels share
    the loop)."""
    frames_all = gen_frames(np.random.default_rng(123), 70000)
    for n in (1, 2, 63, 64, 65, 127, 128, 129, 4097, 65536 + 65):
        frames = frames_all[:n]
        res = clf.parse_packets(frames, 0)
        for i in list(range(min(n, 200))) + list(range(max(0, n - 200), n)):
            assert _rows(res, i) == O.parse_packet(frames[i], 0), (n, i)


@pytest.mark.parametrize("shift", [0, 1])
def test_blob_at_allocation_end(clf, shift):
    """The frames' last byte is the last byte of a device allocation (a
    32 MiB torch block -- above 10 MiB the caching allocator gives a request
    its own segment -- filled from its end) and the offsets array ends one
    element past n likewise: staged (aligned) and unstaged (shift 1) parse
    kernels must read nothing beyond [0, off[n]) and off[0..n]."""
    import torch
    frames = gen_frames(np.random.default_rng(131 + shift), 9000)
    raw = np.frombuffer(b"".join(frames), np.uint8)
    cap = 32 << 20
    assert len(raw) + shift <= cap
    block = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    start = cap - len(raw)           # the blob's last byte is the block's last byte
    if (start % 4 == 0) != (shift == 0):
        # trailing padding frame of 1-3 bytes moves the start to the wanted alignment
        pad = (start % 4) if shift == 0 else 1
        frames = frames + [bytes(pad)]
        raw = np.frombuffer(b"".join(frames), np.uint8)
        start = cap - len(raw)
    block[start:start + len(raw)] = torch.from_numpy(raw.copy()).cuda()
    blob = block[start:]
    if shift == 0:
        assert blob.data_ptr() % 4 == 0
    else:
        assert blob.data_ptr() % 4 != 0
    lens = np.array([len(f) for f in frames], np.int64)
    off = np.zeros(len(frames) + 1, np.int32)
    off[1:] = np.cumsum(lens)
    obuf = torch.zeros(cap // 4, dtype=torch.int32, device="cuda")
    doff = obuf[cap // 4 - len(off):]
    doff.copy_(torch.from_numpy(off).cuda())
    res = clf.parse_packets((blob, doff), 0)
    torch.cuda.synchronize()
    res = {k: v.cpu().numpy() for k, v in res.items()}
    for k in ("src6", "dst6"):
        res[k] = res[k].view(np.uint8)
    for k in ("src4", "dst4", "vni"):
        res[k] = res[k].view(np.uint32)
    for k in ("sport", "dport", "ether_type"):
        res[k] = res[k].view(np.uint16)
    for i in list(range(300)) + list(range(len(frames) - 300, len(frames))):
        assert _rows(res, i) == O.parse_packet(frames[i], 0), i
