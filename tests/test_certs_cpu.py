"""CPU tier: SSLContextHolder.choose.

The oracle (vo_cert_choose, the literal holder/name scan of
SSLContextHolder.java:51-186) against hand-derived vectors.  The certificate
names are the SAN lists quoted in SSLContextHolder.java:119-121 (pixiv,
youtube, google); no reference test pins choose() (parity pinned by these
hand-derived vectors).  Then the compiled certificate table, walked on the
host by the kernel's own cert_one (tests/native/imgcheck.hip, plain pointer
and staged copies at every alignment), against the oracle on random holder
sets built to hit every compare() branch.
"""
import numpy as np
import pytest

import imgcheck_ffi as I
import oracle_ffi as O

PIXIV = ["pixiv.net", "*.pixiv.net", "pixiv.net", "*.pixiv.org", "pixiv.org", "*.pximg.net",
         "pximg.net", "*.ads-pixiv.net", "ads-pixiv.net"]
YOUTUBE = ["youtube.com", "*.youtube.com", "youtube.com", "*.ytimg.com", "ytimg.com",
           "*.ggpht.com", "ggpht.com", "*.googlevideo.com", "googlevideo.com",
           "*.googleapis.com", "googleapis.com", "*.googlesyndication.com",
           "googlesyndication.com"]
GOOGLE = ["google.com", "*.google.com", "google.com", "*.google.com.hk", "google.com.hk"]
HOLDERS = [PIXIV, YOUTUBE, GOOGLE]

VECTORS = [
    ("pixiv.net", 0), ("www.pixiv.net", 0), ("i.pximg.net", 0), ("pixiv.org", 0),
    ("www.youtube.com", 1), ("youtube.com", 1), ("i.ytimg.com", 1),
    ("r3---sn-a.googlevideo.com", 1), ("www.googleapis.com", 1),
    ("google.com", 2), ("maps.google.com", 2), ("google.com.hk", 2), ("www.google.com.hk", 2),
    ("a.b.youtube.com", 0),       # two extra labels: no wildcard match -> default
    ("YouTube.com", 0),           # String.equals is case-sensitive
    (".youtube.com", 0),          # prefix empty: sni.length() > suffix.length() fails
    ("youtube.com.", 0), ("", 0), (None, 0), ("example.org", 0),
]


@pytest.mark.parametrize("sni,want", VECTORS)
def test_oracle_vectors(sni, want):
    assert O.Certs(HOLDERS).choose(sni) == want


def test_oracle_holder_rules():
    # the first holder with any matching name wins, plain or wildcard
    c = O.Certs([["a.com"], ["*.a.com", "a.com"]])
    assert [c.choose(s) for s in ("a.com", "x.a.com", "y.x.a.com")] == [0, 1, 0]
    c = O.Certs([["*.b.com"], ["x.b.com"]])
    assert c.choose("x.b.com") == 0
    c = O.Certs([[], ["x.b.com"], ["*.b.com"]])
    assert [c.choose(s) for s in ("x.b.com", "y.b.com", "b.com")] == [1, 2, 0]
    # one holder: always it; none: null
    assert O.Certs([["only.com"]]).choose("other.org") == 0
    assert O.Certs([]).choose("x") == -1
    # odd names: "*." (suffix "."), "*" and "*x" are plain, "*.*.a" a wildcard
    c = O.Certs([["z"], ["*."], ["*"], ["*x.com"], ["*.*.a"]])
    assert [c.choose(s) for s in ("abc.", ".", "*", "ax.com", "*x.com", "q.*.a", "q.r.a")] == \
        [1, 0, 2, 0, 3, 4, 0]


def test_table_matches_oracle_vectors():
    snis = [s for s, _ in VECTORS]
    np.testing.assert_array_equal(I.certs(HOLDERS, snis), [w for _, w in VECTORS])


def _random_case(rng, n_holders, n_snis):
    labels = ["a", "b", "ab", "c", "x1", "www", "q" * 53, "*", ""]   # one label > 48 B
    def name(k):
        return ".".join(labels[int(rng.integers(0, len(labels) - 2))] for _ in range(k))
    holders = []
    for _ in range(n_holders):
        hs = []
        for _ in range(int(rng.integers(0, 6))):
            r = rng.random()
            base = name(int(rng.integers(1, 4)))
            if r < 0.4:
                hs.append("*." + base)
            elif r < 0.45:
                hs.append(rng.choice(["*.", "*", "*" + base, "*.*." + base, "." + base, ""]))
            else:
                hs.append(base)
        holders.append(hs)
    flat = [s for hs in holders for s in hs] or ["a"]
    snis = []
    for _ in range(n_snis):
        r = rng.random()
        s = flat[int(rng.integers(0, len(flat)))]
        if r < 0.35:
            s = s[2:] if s.startswith("*.") else s
        elif r < 0.7:
            pre = labels[int(rng.integers(0, len(labels)))]
            if rng.random() < 0.2:
                pre += "." + labels[int(rng.integers(0, len(labels)))]
            s = pre + (s[1:] if s.startswith("*.") else "." + s)
        elif r < 0.8:
            s = s.upper()
        elif r < 0.85:
            s = None
        else:
            s = name(int(rng.integers(1, 5)))
        snis.append(s)
    return holders, snis


@pytest.mark.parametrize("seed,n_holders", [(1, 0), (2, 1), (3, 2), (4, 7), (5, 40), (6, 300)])
def test_table_vs_oracle_random(seed, n_holders):
    rng = np.random.default_rng(seed)
    holders, snis = _random_case(rng, n_holders, 3000)
    got = I.certs(holders, snis)
    c = O.Certs(holders)
    want = np.array([c.choose(s) for s in snis], np.int32)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, [(snis[i], int(got[i]), int(want[i])) for i in bad[:5]]
