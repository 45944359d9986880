"""Traffic-mirror filters over libvclassify.

`MirrorFilters` parses filter configs the way Mirror.parseAndLoadFilter
does (base/src/main/java/vmirror/Mirror.java:545-601: "mac2" only with
"mac", "network2" only with "network", "port2" only with "port", min > max
rejected) and interns the origin / protocol strings to the ids the C ABI
takes (equal strings <-> equal ids).  Matching runs in the HIP kernels
(vc_mirror_match / vc_mirror_switch); there is no CPU path.
"""
import ctypes as C

import numpy as np

from . import _lib
from ._lib import VcMirrorFilter, VcMirrorItems, check, lib


def parse_mac(s):
    """MacAddress(String) (vfd/MacAddress.java:21-44): 17 chars, 6 parts of 2,
    each Integer.parseInt(part, 16) cast to a byte (a sign is allowed)."""
    if len(s) != 17:
        raise _lib.IllegalArgumentException("invalid mac %r" % s)
    parts = s.split(":")
    if len(parts) != 6 or any(len(p) != 2 for p in parts):
        raise _lib.IllegalArgumentException("invalid mac %r" % s)
    out = []
    for p in parts:
        body = p[1:] if p[0] in "+-" else p
        if not body or any(c not in "0123456789abcdefABCDEF" for c in body):
            raise _lib.IllegalArgumentException("invalid mac %r" % s)
        out.append(int(p, 16) & 0xFF)
    return bytes(out)


class MirrorFilters:
    """A compiled FilterConfig list plus the string interning it was built with."""

    def __init__(self):
        self.ids = {}

    def id_of(self, s, create=True):
        """-1 for null; a fresh id for a string no filter names (matches none)."""
        if s is None:
            return -1
        if s not in self.ids:
            if not create:
                return -2
            self.ids[s] = len(self.ids)
        return self.ids[s]

    def build(self, filters):
        """filters: list of dicts {"origin", "mirror", "mac", "mac2", "network",
        "network2", "transportLayerProtocol", "port", "port2",
        "applicationLayerProtocol"} in list order -> vc_mirror_filter array."""
        from .classifier import Network
        arr = (VcMirrorFilter * max(1, len(filters)))()
        for i, f in enumerate(filters):
            r = arr[i]
            r.origin = self.id_of(f["origin"])
            r.mirror = int(f["mirror"])
            if "mac" in f:
                r.has_mac_x = 1
                r.mac_x[:] = list(parse_mac(f["mac"]))
                if "mac2" in f:
                    r.has_mac_y = 1
                    r.mac_y[:] = list(parse_mac(f["mac2"]))
            if "network" in f:
                r.has_net_x = 1
                r.net_x = Network(f["network"]).c
                if "network2" in f:
                    r.has_net_y = 1
                    r.net_y = Network(f["network2"]).c
            r.transport = self.id_of(f.get("transportLayerProtocol"))
            if "port" in f:
                r.has_port_x = 1
                r.port_x[:] = [int(f["port"][0]), int(f["port"][1])]
                if "port2" in f:
                    r.has_port_y = 1
                    r.port_y[:] = [int(f["port2"][0]), int(f["port2"][1])]
            r.app = self.id_of(f.get("applicationLayerProtocol"))
        return arr, len(filters)


def _ptr(a):
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        return C.c_void_p(a.data_ptr())
    return C.c_void_p(a.ctypes.data)


def items_struct(cols):
    """cols: dict of arrays (numpy or torch CUDA) keyed like vc_mirror_items."""
    it = VcMirrorItems()
    for k, _ in VcMirrorItems._fields_:
        setattr(it, k, _ptr(cols.get(k)))
    return it
