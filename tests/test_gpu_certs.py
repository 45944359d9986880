"""GPU tier: SSLContextHolder.choose (device/hint.hip cert_kernel) through the
C ABI against the oracle (vo_cert_choose, SSLContextHolder.java:51-186),
bit-exact: the hand-derived vectors, random holder sets hitting every
compare() branch, a large table (20k holders) with 200k SNIs from the
staged (aligned) and unstaged (unaligned blob) kernels, and the 0/1-holder
cases."""
import numpy as np
import pytest

import oracle_ffi as O
import vproxy_amd as V
from vproxy_amd import workloads as W
from test_certs_cpu import HOLDERS, VECTORS, _random_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def clf():
    c = V.Classifier(0)
    yield c
    c.close()


def test_vectors(clf):
    clf.compile_certs(HOLDERS)
    got = clf.cert_choose([s for s, _ in VECTORS])
    np.testing.assert_array_equal(got, [w for _, w in VECTORS])


@pytest.mark.parametrize("seed,n_holders", [(11, 0), (12, 1), (13, 5), (14, 300)])
def test_random_vs_oracle(clf, seed, n_holders):
    holders, snis = _random_case(np.random.default_rng(seed), n_holders, 20000)
    clf.compile_certs(holders)
    got = clf.cert_choose(snis)
    c = O.Certs(holders)
    want = np.array([c.choose(s) for s in snis], np.int32)
    np.testing.assert_array_equal(got, want)


def test_large_table_device_paths(clf):
    import torch
    from vproxy_amd import workloads as W
    rng = np.random.default_rng(15)
    _, hosts = W.gen_groups(40000, 16, wildcard=False)
    holders = []
    for i in range(0, len(hosts), 2):           # 20k holders: CN + "*." SAN + a shared name
        holders.append([hosts[i], "*." + hosts[i + 1], "shared%d.example" % (i % 97)])
    clf.compile_certs(holders)
    names = W.gen_hostnames(hosts, 200000, 17)
    snis = [n.split(b":")[0] for n in names]
    snis[::41] = [None] * len(snis[::41])
    got = clf.cert_choose(snis)
    c = O.Certs(holders)
    samp = rng.integers(0, len(snis), 4000)
    np.testing.assert_array_equal(got[samp], [c.choose(snis[i]) for i in samp])
    assert (got > 0).mean() > 0.3                   # the table is really hit
    blob, off, nul = V.pack_strings(snis)
    for shift in (0, 1):                            # staged kernel / unaligned blob
        b = np.concatenate([np.zeros(shift, np.uint8), blob])
        db = torch.from_numpy(b).cuda()[shift:]
        dev = clf.cert_choose((db, torch.from_numpy(off.astype(np.int32)).cuda(),
                               torch.from_numpy(nul).cuda()))
        torch.cuda.synchronize()
        np.testing.assert_array_equal(dev.cpu().numpy(), got)


def test_sni_bench_batch(clf):
    """The `sni` sub-bench's batch exactly as bench.py builds it
    (bench.sni_workload: 100k holders = 200k names, 16M seeded draws from
    1M SNIs) through vc_cert_choose_dev: every one of the 16M results equal
    to exact.CertChecker (SSLContextHolder.choose, SSLContextHolder.java:
    50-79,171-186), with an oracle sample."""
    import torch
    import bench as B
    from exact import CertChecker
    n = 16 << 20
    holders, names, pidx = B.sni_workload(n)
    clf.compile_certs(holders)
    nblob, noff = W.pack(names)
    blob, off, _ = B.gather_strings_dev(nblob, noff, pidx, "cuda")
    got = clf.cert_choose((blob, off, None))
    torch.cuda.synchronize()
    want = torch.from_numpy(CertChecker(holders).batch(nblob, noff)).cuda()[
        torch.from_numpy(pidx).cuda()]
    assert torch.equal(got, want), int((got != want).sum())
    c = O.Certs(holders)
    s = np.random.default_rng(3).integers(0, n, 300)
    np.testing.assert_array_equal(got.cpu().numpy()[s], [c.choose(names[pidx[i]]) for i in s])
    assert (want > 0).float().mean() > 0.3


def test_errors(clf):
    with pytest.raises(V.IllegalArgumentException):
        V.check(V.lib().vc_compile_certs(clf.h, None, None, None, 1, 1))
    clf.compile_certs([["a.com"], ["b.com"]])
    assert clf.cert_choose([]).shape == (0,)


def test_reference_cert_kats(clf):
    """kats.json certs: TestSSL.TEST_CERT's CN (decoded from the reference's
    PEM) and the certificates SSLContextHolder.checkSNI documents, through
    vc_compile_certs / vc_cert_choose (no SNI, one holder, no holders,
    wildcard depth, case, first holder in add() order)."""
    import json
    import os
    G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    with open(os.path.join(G, "kats.json")) as f:
        cases = json.load(f)["certs"]
    for case in cases:
        clf.compile_certs(case["holders"])
        got = clf.cert_choose([s for s, _ in case["queries"]])
        assert got.tolist() == [w for _, w in case["queries"]], case["source"]
