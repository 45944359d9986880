"""The string and frame kernels hand each wave a static block of the chunks
before the work tickets (chunks.h ChunksT: hint 60 %, DNS 50 %, SNI and
mirror 25 %, the DNS drain loop 60 %).  A block exists only once a batch has
more chunks than the resident waves can split, so the ordinary GPU tests
(at most a few hundred thousand items) never reach it.  Here each kernel
runs one batch large enough for blocks of several chunks -- a small case
tiled -- and its every result must equal the same items classified in
batches too small for any static block (tickets only), which the other GPU
tests check against the oracle."""
import numpy as np
import pytest

import vproxy_amd as V
from vproxy_amd import workloads as W
from cases import gen_mirror_case, mirror_frames, hint_cases_shapes

pytestmark = pytest.mark.gpu

BIG = 40          # tiles: ~2M names, ~1.2M frames
PIECE = 20000     # the small batches (no static block)


@pytest.fixture(scope="module")
def clf():
    c = V.Classifier(0)
    yield c
    c.close()


def _dev_strings(items):
    import torch
    blob, off, nul = V.pack_strings(items)
    return (torch.from_numpy(blob).cuda(), torch.from_numpy(off.astype(np.int32)).cuda(),
            torch.from_numpy(nul).cuda() if nul is not None else None)


def _pieces(fn, items):
    return np.concatenate([np.asarray(fn(items[i:i + PIECE]))
                           for i in range(0, len(items), PIECE)])


def test_hint_static_blocks(clf):
    import torch
    groups, names = hint_cases_shapes(np.random.default_rng(101), 50000)
    clf.compile_upstream(groups)
    names = names * BIG
    got = clf.hint_search(_dev_strings(names))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.cpu().numpy(), _pieces(clf.hint_search, names))


def test_dns_static_blocks(clf):
    import torch
    groups, ghosts = W.gen_groups(20000, 102)
    clf.compile_upstream(groups)
    clf.compile_hosts([(h + ".", i) for i, h in enumerate(ghosts[:300])])
    names = W.gen_hostnames(ghosts, 50000, 103, dns=True)
    names += [b"1.2.3.4.", b"::1.", b"caf\xe9.com.", b"a.vproxy.local."] * 10
    names = names * BIG
    qb, qo, _ = _dev_strings(names)
    kind, val = clf.dns_classify((qb, qo))
    torch.cuda.synchronize()
    pk = [clf.dns_classify(names[i:i + PIECE]) for i in range(0, len(names), PIECE)]
    np.testing.assert_array_equal(kind.cpu().numpy(), np.concatenate([k for k, _ in pk]))
    np.testing.assert_array_equal(val.cpu().numpy(), np.concatenate([v for _, v in pk]))


def test_sni_static_blocks(clf):
    import torch
    _, hosts = W.gen_groups(20000, 104, wildcard=False)
    holders = [[hosts[i], "*." + hosts[i + 1]] for i in range(0, len(hosts), 2)]
    clf.compile_certs(holders)
    snis = [n.split(b":")[0] for n in W.gen_hostnames(hosts, 50000, 105)] * BIG
    snis[::37] = [None] * len(snis[::37])
    got = clf.cert_choose(_dev_strings(snis))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.cpu().numpy(), _pieces(clf.cert_choose, snis))


def test_mirror_static_blocks(clf):
    import torch
    rng = np.random.default_rng(106)
    filters, _ = gen_mirror_case(rng, 40, 0, origins=("switch", "other"))
    clf.compile_mirror(filters)
    frames = mirror_frames(rng, 30000) * BIG
    lens = np.array([len(f) for f in frames], np.int64)
    off = np.zeros(len(frames) + 1, np.int64)
    off[1:] = np.cumsum(lens)
    blob = torch.from_numpy(np.frombuffer(b"".join(frames), np.uint8).copy()).cuda()
    got = clf.mirror_switch("switch", (blob, torch.from_numpy(off.astype(np.int32)).cuda()))
    torch.cuda.synchronize()
    want = _pieces(lambda f: clf.mirror_switch("switch", f), frames)
    np.testing.assert_array_equal(got.cpu().numpy().view(np.uint64), want.astype(np.uint64))
