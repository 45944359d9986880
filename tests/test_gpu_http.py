"""HTTP/1 request heads -> the upstream group (vc_http_hint[_dev]): the
request line and headers as HttpSubContext reads them
(/root/reference/base/src/main/java/vproxybase/processor/http1/
HttpSubContext.java:394-534), HttpContext.connectionHint (HttpContext.java:
55-71) and Upstream.searchForGroup, against the oracle (vo_http_hint)."""
import json
import os

import numpy as np
import pytest

import oracle_ffi as O
import vproxy_amd as V
from cases import _HOSTS, _URIS, hint_cases_random, http_heads_random

pytestmark = pytest.mark.gpu

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def clf():
    c = V.Classifier(0)
    yield c
    c.close()


def _oracle(groups, heads):
    blob = np.frombuffer(b"".join(heads) or b"\0", np.uint8)
    off = np.cumsum([0] + [len(h) for h in heads]).astype(np.uint32)
    kind, grp = O.http_batch_np(groups, blob, off, nthreads=8)
    return grp, kind


def test_golden_heads(clf):
    """TestHttp1Parser's request heads and the state-machine KATs
    (tests/golden/http1.json), against groups keyed on their hosts / uris."""
    with open(os.path.join(G, "http1.json")) as f:
        heads = [bytes.fromhex(c["head"]) for c in json.load(f)["cases"]]
    groups = [({"host": "example.com"}, {}), ({}, {"uri": "/hello"}), ({"host": "h"}, {}),
              ({"host": "two"}, {}), ({"uri": "/a"}, {"host": "ab.c"}),
              ({"host": "￤.example"}, {}), ({"host": "*"}, {"uri": "/ab"})]
    clf.compile_upstream(groups)
    got, kind = clf.http_hint(heads)
    want, wkind = _oracle(O.Groups(groups), heads)
    np.testing.assert_array_equal(kind, wkind)
    np.testing.assert_array_equal(got, want)
    assert (got >= 0).sum() >= 15


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_heads(clf, seed):
    rng = np.random.default_rng(700 + seed)
    groups, _, _ = hint_cases_random(rng, 300, 0)
    uris = [u for u in _URIS if u is not None] + ["/a/b/c?x=1", "/a/", "/z/", "/b?q", "*", ""]
    hosts = [h for h in _HOSTS if h] + ["q.w.a.com", "[::1]", "::1", "1.2.3.4"]
    heads = http_heads_random(rng, 30000, hosts, uris)
    clf.compile_upstream(groups)
    got, kind = clf.http_hint(heads)
    want, wkind = _oracle(O.Groups(groups), heads)
    np.testing.assert_array_equal(kind, wkind)
    np.testing.assert_array_equal(got, want)
    assert (got >= 0).mean() > 0.3 and set(np.unique(kind)) == {0, 1, 3}


def test_device_blob_unaligned(clf):
    """The _dev entry point over a device blob at an odd offset equals the
    host entry point (16-byte block reads around every head)."""
    import torch
    rng = np.random.default_rng(77)
    groups, _, _ = hint_cases_random(rng, 200, 0)
    heads = http_heads_random(rng, 20000, [h for h in _HOSTS if h], ["/", "/a", "/a/b", "*"])
    clf.compile_upstream(groups)
    want, wkind = clf.http_hint(heads)
    raw = b"".join(heads)
    buf = torch.zeros(len(raw) + 3, dtype=torch.uint8, device="cuda")
    buf[3:] = torch.frombuffer(bytearray(raw), dtype=torch.uint8).cuda()
    off = torch.tensor(np.cumsum([0] + [len(h) for h in heads]), dtype=torch.int32, device="cuda")
    got, kind = clf.http_hint((buf[3:], off))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.cpu().numpy(), want)
    np.testing.assert_array_equal(kind.cpu().numpy(), wkind)


def test_edges(clf):
    clf.compile_upstream([({"host": "a.com"}, {})])
    g, k = clf.http_hint([])
    assert len(g) == 0 and len(k) == 0
    g, k = clf.http_hint([b"", b"G", b"GET /x HTTP/1.1\r\nHost: a.com\r\n\r\n"])
    assert list(g) == [-1, -1, 0] and list(k) == [0, 0, 3]


def test_http_bench_batch_whole(clf):
    """The `http` sub-bench's whole batch (bench.http_workload: 8M draws of
    262k request heads over the C4 groups, a fifth with hint-uris): every
    group and kind equal to the oracle's extraction (vo_http_extract) scored
    by exact.HintLevelChecker (Hint.matchLevel + searchForGroup's strict
    '>', Upstream.java:187-198), itself checked against vo_http_hint on a
    sample of the heads."""
    import torch
    import bench as B
    from exact import HintLevelChecker
    n = 8 << 20
    groups, heads, pidx = B.http_workload(n)
    clf.compile_upstream(groups)
    tb, to = B.W.pack(heads)
    blob, off, nbytes = B.gather_strings_dev(tb, to, pidx, "cuda")
    grp, kind = clf.http_hint((blob, off))
    torch.cuda.synchronize()
    og = O.Groups(groups)
    chk = HintLevelChecker(groups)
    want_g = np.empty(len(heads), np.int32)
    want_k = np.empty(len(heads), np.uint8)
    for t, h in enumerate(heads):
        u, host = O.http_extract(h)
        want_k[t] = (2 if host is not None else 0) | (1 if u is not None else 0)
        want_g[t] = chk(host, 0, u) if want_k[t] else -1
    rng = np.random.default_rng(5)
    for t in rng.integers(0, len(heads), 200):
        assert O.http_hint(og, heads[t]) == (want_g[t], want_k[t])
    np.testing.assert_array_equal(grp.cpu().numpy(), want_g[pidx])
    np.testing.assert_array_equal(kind.cpu().numpy(), want_k[pidx])
    assert (want_g >= 0).mean() > 0.5


def test_dev_span_past_blob_bytes(clf):
    """vc_http_hint_dev with blob_bytes short of off[n]: the heads reaching
    past it come back VC_HTTP_BAD_SPAN (0xFF, group -1) and nothing is
    written past the 3 * blob_bytes scratch; the others are classified."""
    import ctypes as C
    import torch
    clf.compile_upstream([({"host": "a.com"}, {})])
    heads = [b"GET /x HTTP/1.1\r\nHost: a.com\r\n\r\n", b"GET /\xe4 HTTP/1.1\r\nHost: a.com\r\n\r\n"]
    raw = b"".join(heads)
    blob = torch.frombuffer(bytearray(raw), dtype=torch.uint8).cuda()
    off = torch.tensor([0, len(heads[0]), len(raw)], dtype=torch.int32, device="cuda")
    grp = torch.empty(2, dtype=torch.int32, device="cuda")
    kind = torch.empty(2, dtype=torch.uint8, device="cuda")
    V.check(V.lib().vc_http_hint_dev(clf.h, C.c_void_p(blob.data_ptr()), len(heads[0]) + 3,
                                     C.c_void_p(off.data_ptr()), 2, C.c_void_p(grp.data_ptr()),
                                     C.c_void_p(kind.data_ptr()), None))
    torch.cuda.synchronize()
    assert grp.tolist() == [0, -1] and kind.tolist() == [3, 0xFF]


def test_heads_past_the_stage(clf):
    """Chunks of 64 heads longer than a wave's 10 KiB stage (kilobyte
    cookies) take the global-memory path inside the staged kernel; mixed
    with chunks that stage, every result equals the oracle."""
    rng = np.random.default_rng(91)
    groups, _, _ = hint_cases_random(rng, 200, 0)
    base = http_heads_random(rng, 6000, [h for h in _HOSTS if h], ["/", "/a", "/a/b?x", "*"])
    heads = []
    for k, h in enumerate(base):
        if (k // 64) % 3 == 0:                       # every third chunk: big heads
            cut = h.find(b"\r\n") + 2 if b"\r\n" in h else len(h)
            h = h[:cut] + b"Cookie: " + b"c" * int(rng.integers(200, 2000)) + b"\r\n" + h[cut:]
        heads.append(h)
    clf.compile_upstream(groups)
    got, kind = clf.http_hint(heads)
    want, wkind = _oracle(O.Groups(groups), heads)
    np.testing.assert_array_equal(kind, wkind)
    np.testing.assert_array_equal(got, want)


def test_http_hint_device_argument_checks():
    """classifier.http_hint refuses device arguments the kernel would
    misread, before the library is called: an int64 offsets tensor (read as
    uint32 pairs), a non-uint8 blob (numel() undercounts its bytes), an
    empty offsets tensor."""
    import torch
    clf = V.Classifier(0)
    try:
        clf.compile_upstream([({}, {"host": "a.com"})])
        head = b"GET / HTTP/1.1\r\nHost: a.com\r\n\r\n"
        hb = torch.tensor(list(head), dtype=torch.uint8, device="cuda")
        ok = torch.tensor([0, len(head)], dtype=torch.int32, device="cuda")
        g, k = clf.http_hint((hb, ok))
        assert g.cpu().tolist() == [0] and k.cpu().tolist() == [3]      # Hint.ofHostUri
        for bad in ((hb, ok.to(torch.int64)), (hb.to(torch.int32), ok),
                    (hb, torch.empty(0, dtype=torch.int32, device="cuda"))):
            with pytest.raises(V.IllegalArgumentException):
                clf.http_hint(bad)
    finally:
        clf.close()
