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
