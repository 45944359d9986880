"""ctypes face of tests/native/dnsd_loop.c (the C replay of
jni/DnsDrainBatcher.java) and the reference loop's action trace.

reference_trace restates DNSServer's drain loop
(core/src/main/java/vproxy/dns/DNSServer.java:457-500) one datagram at a
time, from the per-datagram outcome of the oracle (vo_dnsd_batch): what the
loop does with datagram i, and where a `return` ends the readable event.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
NATIVE = os.path.join(HERE, "native")

ANSWER, RECURSIVE, RESPONSE, REJECTED, EMPTY, MALFORMED, HOST = range(7)
EINVAL, EDEVICE, ENOMEM, ESTATE = -1, -5, -6, -7
_lib = None


def lib():
    global _lib
    if _lib is None:
        subprocess.check_call(["make", "-s", "-C", NATIVE, "build/libdnsd_loop.so"])
        _lib = C.CDLL(os.path.join(NATIVE, "build", "libdnsd_loop.so"))
        _lib.dnsd_loop_trace.restype = C.c_int
        _lib.dnsd_loop_trace.argtypes = [C.c_void_p] + [C.c_void_p] * 2 + [C.c_int64] + \
            [C.c_void_p] * 4 + [C.c_int, C.c_void_p, C.c_int, C.c_char_p, C.c_int64]
    return _lib


def trace(ctx, blob, off, fam, r4, r6, port, batch, inject=()):
    """The batcher's action trace over the datagram queue (list of tokens)."""
    n = len(off) - 1
    keep = [np.ascontiguousarray(blob, np.uint8), np.ascontiguousarray(off, np.uint32),
            np.ascontiguousarray(fam, np.uint8), np.ascontiguousarray(r4, np.uint32),
            np.ascontiguousarray(r6, np.uint8), np.ascontiguousarray(port, np.uint16)]
    inj = (C.c_int * max(1, len(inject)))(*inject)
    cap = 96 * n + 4096
    out = C.create_string_buffer(cap)
    p = lambda a: C.c_void_p(a.ctypes.data)
    rc = lib().dnsd_loop_trace(ctx, p(keep[0]), p(keep[1]), n, p(keep[2]), p(keep[3]),
                               p(keep[4]), p(keep[5]), batch, inj, len(inject), out, cap)
    assert rc == 0, rc
    return out.value.decode().split()


def reference_trace(want):
    """DNSServer.java:457-500 over the queue, datagram by datagram."""
    out = []
    for i, st in enumerate(want["status"]):
        if st == REJECTED:                       # :469-472 not allowed -> continue
            out += ["S", str(i)]
        elif st in (EMPTY, MALFORMED):           # :473-476 read == 0, :481-486 parse threw -> return
            out += ["E", str(i), "|"]            # the selector fires again for the rest
        elif st == HOST:                         # shapes the library hands back: the Java body
            out += ["J", str(i)]
        elif st == RESPONSE:                     # :489-492 logged, continue
            out += ["P", str(i)]
        elif st == RECURSIVE:                    # :493-496 opcode, or handleRequest's runRecursive
            out += ["R", str(i)]
        else:                                    # :497 handleRequest answers every question
            nq = int(want["nq"][i])
            out += ["A", str(i), str(nq)] + ["%d:%d" % (want["kind"][i][q], want["value"][i][q])
                                             for q in range(nq)]
    return out
