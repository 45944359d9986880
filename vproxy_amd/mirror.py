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


class MirrorSettings:
    """A parsed mirror config file: `enabled`, the mirrors as (tap, mtu) in
    list order, the origins some filter names, and the flattened filter list
    (each filter dict carries its origin and its mirror's index) that
    Classifier.compile_mirror takes."""

    def __init__(self, enabled, mirrors, origins, filters):
        self.enabled = enabled
        self.mirrors = mirrors
        self.origins = origins
        self.filters = filters

    def is_enabled(self, origin):
        """Mirror.isEnabled (Mirror.java:66-71): nothing is mirrored while the
        config is disabled, and only origins named in it are checked."""
        return self.enabled and origin in self.origins


def load_config(cfg):
    """Mirror.parseAndLoad (base/src/main/java/vmirror/Mirror.java:345-374,
    503-601) over a parsed JSON document: `enabled` a boolean, `mirrors` an
    array of {"tap": string, "mtu": int in [0, 1500], "origins": [{"origin":
    string, "filters": [object, ...]}]}.  A value of the wrong JSON type is a
    type error, an absent field a missing field, a bad value (mtu range, a
    port range with min > max, a mac or network that does not parse) an
    invalid value -- all IllegalArgumentException here, naming the field
    being handled as the Java messages do.  Filters keep their list order
    across mirrors and origins.  The tap devices themselves are not opened
    (no tap I/O on this path)."""
    where = ["input"]

    def bad(kind):
        raise _lib.IllegalArgumentException("%s when handling %s" % (kind, ".".join(where)))

    def get(obj, key, types, kind_missing="missing field"):
        if not isinstance(obj, dict):
            bad("type error")
        if key not in obj:
            bad(kind_missing)
        v = obj[key]
        # JSON true/false are not numbers (vjson getInt on a bool: a cast error)
        if isinstance(v, bool) and bool not in types:
            bad("type error")
        if not isinstance(v, types):
            bad("type error")
        return v

    where[:] = ["enabled"]
    enabled = get(cfg, "enabled", (bool,))
    where[:] = ["mirrors"]
    mirrors_j = get(cfg, "mirrors", (list,))
    mirrors, origins, filters = [], set(), []
    for mi, m in enumerate(mirrors_j):
        where[:] = ["mirrors[%d]" % mi]
        if not isinstance(m, dict):
            bad("type error")
        where.append("tap")
        tap = get(m, "tap", (str,))
        where[-1] = "packetSize"                  # Mirror.java:509 names mtu so
        mtu = get(m, "mtu", (int,))
        if mtu < 0 or mtu > 1500:
            bad("invalid value")
        where[-1] = "origins"
        for oi, o in enumerate(get(m, "origins", (list,))):
            where[1:] = ["origins[%d]" % oi]
            if not isinstance(o, dict):
                bad("type error")
            where.append("origin")
            origin = get(o, "origin", (str,))
            origins.add(origin)
            where[-1] = "filters"
            for fi, f in enumerate(get(o, "filters", (list,))):
                where[2:] = ["filters[%d]" % fi]
                if not isinstance(f, dict):
                    bad("type error")
                flt = {"origin": origin, "mirror": mi}
                # Mirror.parseAndLoadFilter (Mirror.java:545-600) field by
                # field, each value checked before the next field is read, so
                # the first bad field is the one reported
                from .classifier import Network

                def parsed(key, check):
                    where[3:] = [key]
                    v = get(f, key, (str,))
                    try:
                        check(v)
                    except _lib.IllegalArgumentException:
                        bad("invalid value")
                    flt[key] = v

                def port_range(key):
                    where[3:] = [key]
                    arr = get(f, key, (list,))
                    if len(arr) < 2:                  # getInt(1): IndexOutOfBounds
                        bad("invalid value")
                    if any(isinstance(x, bool) or not isinstance(x, int) for x in arr[:2]):
                        bad("type error")
                    if arr[0] > arr[1]:
                        bad("invalid value")
                    flt[key] = [arr[0], arr[1]]

                for first, second, check in (("mac", "mac2", parse_mac),
                                             ("network", "network2", Network)):
                    if first in f:
                        parsed(first, check)
                        if second in f:
                            parsed(second, check)
                if "transportLayerProtocol" in f:
                    where[3:] = ["transportLayerProtocol"]
                    flt["transportLayerProtocol"] = get(f, "transportLayerProtocol", (str,))
                if "port" in f:
                    port_range("port")
                    if "port2" in f:
                        port_range("port2")
                if "applicationLayerProtocol" in f:
                    where[3:] = ["applicationLayerProtocol"]
                    flt["applicationLayerProtocol"] = get(f, "applicationLayerProtocol", (str,))
                del where[3:]
                filters.append(flt)
            del where[2:]
        mirrors.append((tap, mtu))
    return MirrorSettings(enabled, mirrors, origins, filters)


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
