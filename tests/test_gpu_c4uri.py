"""GPU tier: Upstream.searchForGroup for the hints the L7 callers send,
Hint.ofHostUri(Host, uri) with port 0 (HttpContext.java:63-69,
httpbin/Stream.java:50), scored by the whole Hint.matchLevel
(Hint.java:100-160) and the strict '>' of Upstream.java:187-198.

- The `c4uri` sub-bench's whole batch (bench.c4uri_workload: 100k C4
  groups, a fifth with hint-uris, 200 uri-only and 5,000 path-routed groups;
  16M hints, 80 % with a uri): every result equal to
  exact.HintLevelChecker.table, the per-pair restatement validated against
  the per-item checker and the oracle on the CPU tier.
- Random groups whose hint-hosts overlap (long member lists, keys with and
  without hint-uris, several matching suffix keys, wildcards shared by
  several groups, no wildcard), port-0 uri hints, null hosts and hints with
  ports: equal to the oracle, from the host entry point and from an
  unaligned device blob (the unstaged kernel).
"""
import numpy as np
import pytest

import bench
import oracle_ffi as O
import vproxy_amd as V
from vproxy_amd import workloads as W

pytestmark = pytest.mark.gpu


def test_c4uri_bench_batch_exact():
    import torch
    from exact import HintLevelChecker
    groups, names, uris, nidx, uidx = bench.c4uri_workload()
    clf = V.Classifier(0)
    try:
        clf.compile_upstream(groups)
        hb, ho, ub, uo, un, _ = bench.c4uri_batch(names, uris, nidx, uidx, "cuda")
        n = len(nidx)
        og = O.Groups(groups)
        chk = HintLevelChecker(groups)
        tab = chk.table(names, uris + [None])
        want = tab[nidx, np.where(uidx < 0, len(uris), uidx)]
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        for _ in range(2):                         # and a second launch on the same slots
            out.fill_(-7)
            V.check(V.lib().vc_hint_search_dev(
                clf.h, hb.data_ptr(), ho.data_ptr(), None, None, ub.data_ptr(), uo.data_ptr(),
                un.data_ptr(), n, out.data_ptr(), None))
            torch.cuda.synchronize()
            got = out.cpu().numpy()
            np.testing.assert_array_equal(got, want)
        s = np.random.default_rng(5).integers(0, n, 400)
        np.testing.assert_array_equal(got[s], [O.search_for_group(
            og, names[nidx[i]], 0, uris[uidx[i]] if uidx[i] >= 0 else None) for i in s])
        # the uri decides for some hints: the same name answers differently by uri
        assert (tab[:, :-1] != tab[:, -1:]).any(axis=1).mean() > 0.02
        assert (got >= 0).mean() > 0.9 and len(np.unique(got)) > 50000
    finally:
        clf.close()


def _split_groups(rng, hosts, ng, wildcards):
    """Groups over a few hint-hosts: keys with one or many members, with and
    without hint-uris, and (wildcards) several "*" groups."""
    uris = ["/", "/a", "/a/b", "/a/b/c", "*", "/b", "/a/b/c/d/e"]
    out = []
    for _ in range(ng):
        a = {}
        r = rng.random()
        if r < 0.85:
            a["host"] = hosts[int(rng.integers(0, len(hosts)))]
        elif r < 0.85 + wildcards:
            a["host"] = "*"
        if rng.random() < 0.35:
            a["uri"] = uris[int(rng.integers(0, len(uris)))]
        if rng.random() < 0.05:
            a["port"] = 8080
        out.append(({}, a))
    return out


@pytest.mark.parametrize("wildcards", [0.0, 0.02])
def test_uri_hints_vs_oracle(wildcards):
    import torch
    rng = np.random.default_rng(17 + int(wildcards * 100))
    hosts = ["a.com", "b.a.com", "c.b.a.com", "x.org", "y.x.org", "z.net", "com", "org"]
    groups = _split_groups(rng, hosts, 300, wildcards)
    # hosts no group lists alone, too: misses, deep names under several keys
    qhosts = hosts + ["d.c.b.a.com", "q.z.net", "nope.io", "www.a.com:80", "a.com:8080", ":80",
                      "[::1]:80", "m.y.x.org"]
    quris = ["/a/b/c/x", "/a/b", "/a/", "/a?x=1", "/", "/b/q", "/zz", "*", "/a/b/c/d/e/f?g"]
    n = 60000
    hs = [None if rng.random() < 0.03 else qhosts[int(rng.integers(0, len(qhosts)))]
          for _ in range(n)]
    us = [None if rng.random() < 0.15 else quris[int(rng.integers(0, len(quris)))]
          for _ in range(n)]
    ps = np.where(rng.random(n) < 0.9, 0, rng.choice(np.array([80, 8080]), n)).astype(np.uint16)
    clf = V.Classifier(0)
    try:
        clf.compile_upstream(groups)
        og = O.Groups(groups)
        want = np.array([O.search_for_group(og, h, int(p), u) for h, p, u in zip(hs, ps, us)],
                        np.int32)
        np.testing.assert_array_equal(clf.hint_search(hs, ps, us), want)
        # unaligned device blobs: the unstaged kernel, general path inline
        hb, ho = W.pack([b"" if h is None else h.encode() for h in hs])
        ub, uo = W.pack([b"" if u is None else u.encode() for u in us])
        raw = torch.zeros(len(hb) + 1, dtype=torch.uint8, device="cuda")
        raw[1:] = torch.from_numpy(hb.astype(np.uint8)).cuda()
        hn = torch.from_numpy(np.array([h is None for h in hs], np.uint8)).cuda()
        unl = torch.from_numpy(np.array([u is None for u in us], np.uint8)).cuda()
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt)).cuda()
        ho_d, ub_d, uo_d = t(ho.astype(np.uint32), np.int32), t(ub.astype(np.uint8), np.uint8), \
            t(uo.astype(np.uint32), np.int32)
        pd = t(ps, np.int16)
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        V.check(V.lib().vc_hint_search_dev(clf.h, raw.data_ptr() + 1, ho_d.data_ptr(),
                                           hn.data_ptr(), pd.data_ptr(), ub_d.data_ptr(),
                                           uo_d.data_ptr(), unl.data_ptr(), n, out.data_ptr(),
                                           None))
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy(), want)
        assert len(np.unique(want)) > 50
    finally:
        clf.close()
