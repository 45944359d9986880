"""ctypes binding of libvclassify.so (include/vclassify.h).

The library is built in-tree by `make -C vproxy_amd/csrc` (or
__graft_entry__.build()).  There is no fallback: if the shared library is
missing, importing the classifier raises.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# VCLASSIFY_LIB: another in-tree build of the same library (A/B measurements)
LIB_PATH = os.environ.get("VCLASSIFY_LIB") or os.path.join(HERE, "libvclassify.so")

VC_OK, VC_EINVAL, VC_EEXIST, VC_ENOTFOUND, VC_EXEXC, VC_EDEVICE, VC_ENOMEM, VC_ESTATE = \
    0, -1, -2, -3, -4, -5, -6, -7
PROTO_TCP, PROTO_UDP = 6, 17
DNS_HOSTS, DNS_GROUP, DNS_IP_LITERAL, DNS_INTERNAL, DNS_RECURSIVE = 1, 2, 3, 4, 5
COUNTERS_ACL, COUNTERS_ROUTE, COUNTERS_GROUP = 0, 1, 2
# vc_dns_datagrams status codes (VC_DNSD_*)
(DNSD_ANSWER, DNSD_RECURSIVE, DNSD_RESPONSE, DNSD_REJECTED, DNSD_EMPTY, DNSD_MALFORMED,
 DNSD_HOST) = range(7)
DNSD_MAXQ = 4
SOURCE_ALL, SOURCE_IPV4, SOURCE_IPV6 = 0, 4, 6
LAYER_VXLAN, LAYER_ETHER, LAYER_IPV4, LAYER_IPV6 = 0, 1, 4, 6
SWITCH_NO_TABLE = -2           # vc_switch_classify: the packet's VNI has no table
# snapshot kinds of vc_pin_acquire / vc_generation (VC_SNAP_*)
(SNAP_ACL, SNAP_ROUTE, SNAP_UPSTREAM, SNAP_HOSTS, SNAP_SERVERS, SNAP_CERTS, SNAP_MIRROR,
 SNAP_VNI) = range(8)
SNAP_ALL = 0xFF


class VcNet(C.Structure):
    _fields_ = [("ip", C.c_uint8 * 16), ("mask", C.c_uint8 * 16),
                ("ip_len", C.c_int32), ("mask_len", C.c_int32)]


class VcAclRule(C.Structure):
    _fields_ = [("net", VcNet), ("min_port", C.c_int32), ("max_port", C.c_int32),
                ("allow", C.c_int32)]


class VcAnnos(C.Structure):
    _fields_ = [("host", C.c_char_p), ("host_len", C.c_int32), ("port", C.c_int32),
                ("uri", C.c_char_p), ("uri_len", C.c_int32)]


class VcGroupAnnos(C.Structure):
    _fields_ = [("handle", VcAnnos), ("group", VcAnnos)]


class VcPktOut(C.Structure):
    _fields_ = [("status", C.c_void_p), ("l3", C.c_void_p), ("l4", C.c_void_p),
                ("proto", C.c_void_p), ("vni", C.c_void_p), ("ether_type", C.c_void_p),
                ("src4", C.c_void_p), ("dst4", C.c_void_p), ("src6", C.c_void_p),
                ("dst6", C.c_void_p), ("sport", C.c_void_p), ("dport", C.c_void_p)]


class VcDnsdOut(C.Structure):
    """vc_dnsd_out: per-datagram status / rule / question count, and per
    question [n][VC_DNSD_MAXQ] qtype / kind / value."""
    _fields_ = [("status", C.c_void_p), ("acl", C.c_void_p), ("nq", C.c_void_p),
                ("qtype", C.c_void_p), ("kind", C.c_void_p), ("value", C.c_void_p)]


class VcPackets(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("family", "proto", "src4", "dst4", "src6", "dst6",
                                          "dport", "host_id")]


class VcPipelineOut(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("acl", "route", "group", "allow")]


class VcServer(C.Structure):
    _fields_ = [("ip", C.c_uint8 * 16), ("ip_len", C.c_int32), ("port", C.c_int32),
                ("weight", C.c_int32), ("healthy", C.c_int32)]


class VcMirrorFilter(C.Structure):
    _fields_ = [("origin", C.c_int32), ("mirror", C.c_int32), ("has_mac_x", C.c_int32),
                ("has_mac_y", C.c_int32), ("mac_x", C.c_uint8 * 6), ("mac_y", C.c_uint8 * 6),
                ("has_net_x", C.c_int32), ("has_net_y", C.c_int32), ("net_x", VcNet),
                ("net_y", VcNet), ("transport", C.c_int32), ("has_port_x", C.c_int32),
                ("has_port_y", C.c_int32), ("port_x", C.c_int32 * 2), ("port_y", C.c_int32 * 2),
                ("app", C.c_int32)]


class VcMirrorItems(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("mac_src", "mac_dst", "ip_src_len", "ip_dst_len",
                                          "ip_src", "ip_dst", "transport", "port_src",
                                          "port_dst", "app")]


class VcMetric(C.Structure):
    _fields_ = [("metric", C.c_char_p), ("type", C.c_int32), ("n_labels", C.c_int32),
                ("label_keys", C.POINTER(C.c_char_p)), ("label_values", C.POINTER(C.c_char_p)),
                ("value", C.c_int64)]


METRIC_COUNTER, METRIC_GAUGE = 0, 1


# ---- exceptions mirroring the reference's (vproxybase.util.exception.*) ----
class VcError(Exception):
    code = None


class IllegalArgumentException(VcError, ValueError):
    code = VC_EINVAL


class AlreadyExistException(VcError):
    code = VC_EEXIST


class NotFoundException(VcError):
    code = VC_ENOTFOUND


class XException(VcError):
    code = VC_EXEXC


class DeviceError(VcError, RuntimeError):
    code = VC_EDEVICE


class StateError(VcError, RuntimeError):
    code = VC_ESTATE


_EXC = {c.code: c for c in (IllegalArgumentException, AlreadyExistException, NotFoundException,
                            XException, DeviceError, StateError)}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("libvclassify.so not built (run `make -C vproxy_amd/csrc` or "
                              "__graft_entry__.build()); there is no CPU fallback")
        # One HIP runtime per process.  PyTorch-ROCm ships its own
        # libamdhip64.so.7; if libvclassify loaded the system copy first,
        # torch would bring up a second runtime that sees no GPU.  Loading
        # torch first makes the dynamic linker bind libvclassify's
        # libamdhip64.so.7 dependency to the already-loaded runtime.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        P = C.POINTER
        vp, i64, i32 = C.c_void_p, C.c_int64, C.c_int
        L.vc_version.restype = C.c_char_p
        L.vc_last_error.restype = C.c_char_p
        L.vc_create.argtypes = [i32, P(vp)]
        L.vc_destroy.argtypes = [vp]
        L.vc_net_parse.argtypes = [C.c_char_p, P(VcNet)]
        L.vc_net_from_prefix.argtypes = [vp, i32, i32, P(VcNet)]
        L.vc_net_contains_ip.argtypes = [P(VcNet), vp, i32]
        L.vc_ip_parse.argtypes = [C.c_char_p, vp]
        L.vc_compile_acl.argtypes = [vp, P(VcAclRule), i32, P(VcAclRule), i32, i32]
        for f in ("vc_acl_classify_v4_dev", "vc_acl_classify_v6_dev"):
            getattr(L, f).argtypes = [vp, vp, vp, vp, i64, vp, vp, vp]
        for f in ("vc_acl_classify_v4", "vc_acl_classify_v6"):
            getattr(L, f).argtypes = [vp, vp, vp, vp, i64, vp, vp]
        L.vc_compile_routes.argtypes = [vp, P(VcNet), i32, P(VcNet), i32]
        for f in ("vc_route_lookup_v4_dev", "vc_route_lookup_v6_dev"):
            getattr(L, f).argtypes = [vp, vp, i64, vp, vp]
        for f in ("vc_route_lookup_v4", "vc_route_lookup_v6"):
            getattr(L, f).argtypes = [vp, vp, i64, vp]
        if hasattr(L, "vc_compile_vni_routes"):    # (A/B runs load older builds without it)
            L.vc_compile_vni_routes.argtypes = [vp, vp, vp, vp, vp, vp, i32]
            L.vc_routetables_compile_vni.argtypes = [vp, vp, i32]
        L.vc_compile_upstream.argtypes = [vp, P(VcGroupAnnos), i32]
        L.vc_hint_search_dev.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, i64, vp, vp]
        L.vc_hint_search.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, i64, vp]
        L.vc_compile_hosts.argtypes = [vp, P(C.c_char_p), vp, vp, i32]
        L.vc_compile_hosts_text.argtypes = [vp, C.c_char_p, i64]
        L.vc_dns_classify_dev.argtypes = [vp, vp, vp, i64, vp, vp, vp]
        L.vc_dns_classify.argtypes = [vp, vp, vp, i64, vp, vp]
        L.vc_http_hint_dev.argtypes = [vp, vp, i64, vp, i64, vp, vp, vp]
        L.vc_http_hint.argtypes = [vp, vp, vp, i64, vp, vp]
        L.vc_pipeline_v4_dev.argtypes = [vp, vp, vp, vp, vp, vp, vp, i64, i64, vp, vp, vp, vp, vp]
        L.vc_pipeline_v4_dev_ex.argtypes = [vp, vp, vp, vp, vp, vp, vp, i64, i64, vp, vp, vp, vp,
                                            vp, vp]
        L.vc_pipeline_dev.argtypes = [vp, P(VcPackets), i64, vp, i64, P(VcPipelineOut), vp, vp,
                                      vp]
        L.vc_pipeline_c6_dev.argtypes = [vp, P(VcPackets), i64, i64, vp, i64, P(VcPipelineOut), vp,
                                         vp, vp]
        L.vc_pipeline.argtypes = [vp, P(VcPackets), i64, vp, i64, P(VcPipelineOut)]
        L.vc_pipeline_c6.argtypes = [vp, P(VcPackets), i64, i64, vp, i64, P(VcPipelineOut)]
        L.vc_compile_servers.argtypes = [vp, P(VcServer), vp, i32]
        L.vc_servers_set_health.argtypes = [vp, vp, i64]
        for f in ("vc_source_select_v4_dev", "vc_source_select_v6_dev"):
            getattr(L, f).argtypes = [vp, vp, vp, i64, i32, vp, vp]
        for f in ("vc_source_select_v4", "vc_source_select_v6"):
            getattr(L, f).argtypes = [vp, vp, vp, i64, i32, vp]
        L.vc_compile_certs.argtypes = [vp, P(C.c_char_p), vp, vp, i32, i32]
        L.vc_cert_choose_dev.argtypes = [vp, vp, vp, vp, i64, vp, vp]
        L.vc_cert_choose.argtypes = [vp, vp, vp, vp, i64, vp]
        L.vc_host_register.argtypes = [vp, i64]
        L.vc_host_unregister.argtypes = [vp]
        L.vc_compile_mirror.argtypes = [vp, P(VcMirrorFilter), i32]
        L.vc_mirror_match_dev.argtypes = [vp, i32, P(VcMirrorItems), i64, vp, vp]
        L.vc_mirror_match.argtypes = [vp, i32, P(VcMirrorItems), i64, vp]
        L.vc_mirror_switch_dev.argtypes = [vp, i32, vp, vp, i64, i32, vp, vp]
        L.vc_mirror_switch.argtypes = [vp, i32, vp, vp, i64, i32, vp]
        L.vc_parse_packets_dev.argtypes = [vp, vp, vp, i64, i32, P(VcPktOut), vp]
        L.vc_parse_packets.argtypes = [vp, vp, vp, i64, i32, P(VcPktOut)]
        L.vc_switch_classify_dev.argtypes = [vp, vp, vp, i64, i32, vp, vp, vp, i32, P(VcPktOut),
                                             vp, vp, vp, vp]
        L.vc_switch_classify.argtypes = [vp, vp, vp, i64, i32, vp, vp, vp, i32, P(VcPktOut), vp,
                                         vp, vp]
        if hasattr(L, "vc_dns_datagrams"):     # (A/B runs load older builds without it)
            L.vc_dns_datagrams_dev.argtypes = [vp, vp, vp, i64, vp, vp, vp, vp, P(VcDnsdOut), vp]
            L.vc_dns_datagrams.argtypes = [vp, vp, vp, i64, vp, vp, vp, vp, P(VcDnsdOut)]
        L.vc_counters_enable.argtypes = [vp, i32]
        L.vc_counters_device.argtypes = [vp, i32, P(vp), P(C.c_int64)]
        L.vc_counters_read.argtypes = [vp, i32, vp, i64]
        L.vc_counters_reset.argtypes = [vp]
        L.vc_counters_add_dev.argtypes = [vp, i32, vp, vp, i32, i64, vp]
        u64p = P(C.c_uint64)
        L.vc_table_digest.argtypes = [vp, i32, u64p]
        if hasattr(L, "vc_pin_acquire"):       # (A/B runs load older builds without it)
            L.vc_pin_acquire.argtypes = [vp, C.c_uint32, P(vp)]
            L.vc_pin_bind.argtypes = [vp, vp]
            L.vc_pin_generation.argtypes = [vp, i32, u64p]
            L.vc_pin_release.argtypes = [vp]
            L.vc_pin_release.restype = None
            L.vc_generation.argtypes = [vp, i32, u64p]
        L.vc_digest_acl.argtypes = [P(VcAclRule), i32, P(VcAclRule), i32, i32, u64p]
        L.vc_digest_routes.argtypes = [P(VcNet), i32, P(VcNet), i32, u64p]
        L.vc_digest_upstream.argtypes = [P(VcGroupAnnos), i32, u64p]
        cpp = P(C.c_char_p)
        L.vc_prometheus_format.argtypes = [P(VcMetric), i32, cpp, cpp, i32, vp, i64, P(i64)]
        L.vc_prometheus_hits.argtypes = [vp, i32, i32, vp, i32, i32, vp, i32, C.c_char_p, vp, i64,
                                         P(i64)]
        L.vc_counters_prometheus.argtypes = [vp, C.c_char_p, vp, i64, P(i64)]
        L.vc_secgroup_new.argtypes = [C.c_char_p, i32, P(vp)]
        L.vc_secgroup_free.argtypes = [vp]
        L.vc_secgroup_set_default.argtypes = [vp, i32]
        L.vc_secgroup_add_rule.argtypes = [vp, C.c_char_p, P(VcNet), i32, i32, i32, i32]
        L.vc_secgroup_remove_rule.argtypes = [vp, C.c_char_p]
        L.vc_secgroup_rules.argtypes = [vp, i32, P(VcAclRule), i32]
        L.vc_secgroup_compile.argtypes = [vp, vp]
        L.vc_routetable_new.argtypes = [P(VcNet), P(VcNet), i32, P(vp)]
        L.vc_routetable_free.argtypes = [vp]
        L.vc_routetable_add_rule.argtypes = [vp, C.c_char_p, P(VcNet), i32, vp, i32]
        L.vc_routetable_add_rules.argtypes = [vp, C.c_char_p, P(VcNet), i32, i32]
        L.vc_routetable_del_rule.argtypes = [vp, C.c_char_p]
        L.vc_routetable_rules.argtypes = [vp, i32, P(VcNet), i32]
        L.vc_routetable_compile.argtypes = [vp, vp]
        _lib = L
    return _lib


def check(rc):
    """Raise the reference-style exception for a negative status."""
    if rc is not None and rc < 0:
        msg = lib().vc_last_error().decode(errors="replace")
        raise _EXC.get(rc, VcError)(msg)
    return rc


# every symbol include/vclassify.h declares (checked by tests/test_capi_symbols.py)
def header_symbols(header=None):
    import re
    header = header or os.path.join(os.path.dirname(HERE), "include", "vclassify.h")
    with open(header) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(vc_[a-z0-9_]+)\s*\(", text)))
