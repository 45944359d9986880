"""CPU tier: the word-based Network.maskMatch (common/netmatch.h, used by the
host control plane and the mirror-filter kernels) against the oracle's
byte-wise restatement (Network.java:183-278) for every length combination,
with random bytes and the IPv4-compatible / IPv4-mapped prefixes that
lowBitsV6V4 accepts; and the compiled per-input-family form the mirror
kernels use (NetMatch), run on the host."""
import ctypes as C

import numpy as np

import imgcheck_ffi as I
import oracle_ffi as O
import vproxy_amd as V


def _net(rule, mask):
    n = V._lib.VcNet()
    n.ip[:len(rule)] = list(rule)
    n.mask[:len(mask)] = list(mask)
    n.ip_len, n.mask_len = len(rule), len(mask)
    return n


def test_mask_match_all_length_cases():
    rng = np.random.default_rng(5)
    L = V.lib()
    specials = [bytes(10) + b"\0\0", bytes(10) + b"\xff\xff", bytes(10) + b"\0\xff",
                bytes(9) + b"\1\0\0"]
    checked = 0
    for inl in (4, 16):
        for rl in (4, 16):
            for ml in (4, 16):
                for _ in range(3000):
                    inp = bytearray(rng.integers(0, 256, inl).astype(np.uint8).tobytes())
                    rule = bytearray(rng.integers(0, 256, rl).astype(np.uint8).tobytes())
                    m = int(rng.integers(0, ml * 8 + 1))
                    mask = (((1 << (ml * 8)) - 1) ^ ((1 << (ml * 8 - m)) - 1)).to_bytes(ml, "big")
                    r = rng.random()
                    if r < 0.4:          # rule inside the mask -> matches are likely
                        if rl == inl:
                            rule = bytearray(a & b for a, b in zip(inp, mask)) if ml == inl \
                                else rule
                        elif rl == 16 and inl == 4:
                            rule[:12] = specials[int(rng.integers(0, 4))]
                            rule[12:] = bytes(a & b for a, b in zip(inp, mask[-4:]))
                        else:
                            inp[:12] = specials[int(rng.integers(0, 4))]
                            rule = bytearray(a & b for a, b in zip(inp[12:], mask[-4:]))
                    want = O.mask_match(bytes(inp), bytes(rule), mask)
                    net = _net(rule, mask)
                    buf = (C.c_uint8 * 16).from_buffer_copy(bytes(inp).ljust(16, b"\0"))
                    got = bool(L.vc_net_contains_ip(C.byref(net), buf, inl))
                    assert got == want, (inp.hex(), rule.hex(), mask.hex())
                    # the mirror kernels' compiled per-family form
                    got2 = bool(I.lib().ic_net_match(bytes(inp), inl, bytes(rule), rl, mask, ml))
                    assert got2 == want, ("matcher", inp.hex(), rule.hex(), mask.hex())
                    checked += want
    assert checked > 1000
