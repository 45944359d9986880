"""ctypes face of tests/native/switch_loop.c (the C replay of
jni/SwitchDrainBatcher.java) and the reference loop's action trace.

reference_trace restates Switch.PacketHandler.readable
(core/src/main/java/vswitch/Switch.java:744-776) with
handleNetworkAndGetVXLanPacket (:643-731) one datagram at a time, from
per-datagram outcomes the oracle computes: VProxyEncryptedPacket.from
(`decrypt`, a test stub), bareVXLanAccess.allow (vo_sg_allow, UDP, the
bind port), VXLanPacket.from (vo_parse) and the inner route
(vo_rt_lookup).
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
NATIVE = os.path.join(HERE, "native")

PKT_OK, PKT_EXCEPTION, PKT_LOOP = 0, 4, 5
EINVAL, EDEVICE, ENOMEM, ESTATE = -1, -5, -6, -7
_lib = None


def lib():
    global _lib
    if _lib is None:
        subprocess.check_call(["make", "-s", "-C", NATIVE, "build/libswitch_loop.so"])
        _lib = C.CDLL(os.path.join(NATIVE, "build", "libswitch_loop.so"))
        _lib.switch_loop_trace.restype = C.c_int
        _lib.switch_loop_trace.argtypes = [C.c_void_p] + [C.c_void_p] * 2 + [C.c_int64] + \
            [C.c_void_p] * 4 + [C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_char_p, C.c_int64]
    return _lib


def trace(ctx, blob, off, decrypt, fam, r4, r6, bind_port, batch, inject=()):
    """The batcher's action trace over the datagram queue (list of tokens)."""
    n = len(off) - 1
    keep = [np.ascontiguousarray(blob, np.uint8), np.ascontiguousarray(off, np.uint32),
            np.ascontiguousarray(decrypt, np.uint8), np.ascontiguousarray(fam, np.uint8),
            np.ascontiguousarray(r4, np.uint32), np.ascontiguousarray(r6, np.uint8)]
    inj = (C.c_int * max(1, len(inject)))(*inject)
    cap = 32 * n + 4096
    out = C.create_string_buffer(cap)
    p = lambda a: C.c_void_p(a.ctypes.data)
    rc = lib().switch_loop_trace(ctx, p(keep[0]), p(keep[1]), n, p(keep[2]), p(keep[3]),
                                 p(keep[4]), p(keep[5]), bind_port, batch, inj, len(inject), out,
                                 cap)
    assert rc == 0, rc
    return out.value.decode().split()


def reference_trace(lens, decrypt, allow, status, route):
    """Switch.java:744-776 over the queue, datagram by datagram: a read of 0
    bytes ends the readable event (:757-759; the level-triggered selector
    fires again while datagrams remain)."""
    out = []
    for i, ln in enumerate(lens):
        if ln == 0:
            out.append("|")
        elif decrypt[i]:                         # packet.from(data) == null: user iface
            out += ["E", str(i)]
        elif not allow[i]:                       # :711-714 not in allowed security-group
            out += ["S", str(i)]
        elif status[i] in (PKT_EXCEPTION, PKT_LOOP):   # VXLanPacket.from throws / loops
            out += ["J", str(i)]
        elif status[i] != PKT_OK:                # :684-687 invalid packet for vxlan
            out += ["X", str(i)]
        else:                                    # :688-731 then inputVXLan -> L3 route
            out += ["B", str(i), str(int(route[i]))]
    if not out or out[-1] != "|":
        out.append("|")
    return out
