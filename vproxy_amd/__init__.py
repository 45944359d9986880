"""vproxy_amd -- MI355X-native batched classifier for vproxy's hot path.

SecurityGroup first-match ACL, vswitch RouteTable lookup, Upstream Host/SNI
hint matching and DNSServer record classification, evaluated by hand-written
HIP kernels for gfx950 behind the C ABI in include/vclassify.h.
"""
from ._lib import (AlreadyExistException, DeviceError, IllegalArgumentException,  # noqa: F401
                   NotFoundException, StateError, VcError, XException, check, lib,
                   COUNTERS_ACL, COUNTERS_ROUTE, COUNTERS_GROUP, PROTO_TCP, PROTO_UDP,
                   DNS_HOSTS, DNS_GROUP, DNS_IP_LITERAL, DNS_INTERNAL, DNS_RECURSIVE,
                   DNSD_ANSWER, DNSD_RECURSIVE, DNSD_RESPONSE, DNSD_REJECTED, DNSD_EMPTY,
                   DNSD_MALFORMED, DNSD_HOST, DNSD_MAXQ,
                   SOURCE_ALL, SOURCE_IPV4, SOURCE_IPV6,
                   LAYER_VXLAN, LAYER_ETHER, LAYER_IPV4, LAYER_IPV6, SWITCH_NO_TABLE,
                   SNAP_ACL, SNAP_ROUTE, SNAP_UPSTREAM, SNAP_HOSTS, SNAP_SERVERS, SNAP_CERTS,
                   SNAP_MIRROR, SNAP_VNI, SNAP_ALL)
from .classifier import (Annotations, Classifier, Network, Pin, RouteTable, SecurityGroup,  # noqa: F401
                         acl_rule_array, group_array, net_array, pack_strings, parse_ip,
                         server_array, cn_of_dn, digest_acl, digest_routes, digest_upstream)

__all__ = ["Classifier", "Network", "SecurityGroup", "RouteTable", "Annotations", "parse_ip"]
