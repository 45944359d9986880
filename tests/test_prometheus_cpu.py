"""CPU tier: Prometheus text exposition through the
C ABI (vc_prometheus_format / vc_prometheus_hits; host code, no GPU).

Pinned by the reference's own known answers,
test/src/test/java/vproxy/test/cases/TestPrometheus.java:13-69 (counter and
gauge expositions); the quoting, extra-label and hit-counter cases follow
Metric.java:15-25, GlobalInspection.java:95-125 and JSON string escaping.
"""
import numpy as np
import pytest

from vproxy_amd import _lib
from vproxy_amd import prometheus as P


def test_reference_counter_vector():
    """TestPrometheus.counter (TestPrometheus.java:13-40)."""
    metrics = P.Metrics()
    c1 = P.Counter("vproxy_test_case_counter", {"class": "TestPrometheus", "method": "counter"})
    metrics.add(c1)
    c2 = P.Counter("vproxy_connections_total", {"type": "tcp-lb", "alias": "tl0"})
    metrics.add(c2)
    c3 = P.Counter("vproxy_connections_total", {"type": "tcp-lb", "alias": "tl1"})
    metrics.add(c3)
    metrics.registerHelpMessage("vproxy_test_case_counter", "Some description messages")
    c1.incr(7)
    c2.incr(19)
    c3.incr(91)
    assert metrics.toString() == (
        "# TYPE vproxy_connections_total counter\n"
        "vproxy_connections_total{alias=\"tl0\",type=\"tcp-lb\"} 19\n"
        "vproxy_connections_total{alias=\"tl1\",type=\"tcp-lb\"} 91\n"
        "# HELP vproxy_test_case_counter Some description messages\n"
        "# TYPE vproxy_test_case_counter counter\n"
        "vproxy_test_case_counter{class=\"TestPrometheus\",method=\"counter\"} 7\n")


def test_reference_gauge_vector():
    """TestPrometheus.gauge (TestPrometheus.java:42-69)."""
    metrics = P.Metrics()
    g1 = P.Gauge("vproxy_test_case_gauge", {"class": "TestPrometheus", "method": "gauge"})
    metrics.add(g1)
    g2 = P.Gauge("vproxy_connections_current", {"type": "tcp-lb", "alias": "tl0"})
    metrics.add(g2)
    g3 = P.Gauge("vproxy_connections_current", {"type": "tcp-lb", "alias": "tl1"})
    metrics.add(g3)
    metrics.registerHelpMessage("vproxy_test_case_gauge", "Some description messages")
    g1.incr(7)
    g2.incr(19)
    g3.incr(91)
    assert str(metrics) == (
        "# TYPE vproxy_connections_current gauge\n"
        "vproxy_connections_current{alias=\"tl0\",type=\"tcp-lb\"} 19\n"
        "vproxy_connections_current{alias=\"tl1\",type=\"tcp-lb\"} 91\n"
        "# HELP vproxy_test_case_gauge Some description messages\n"
        "# TYPE vproxy_test_case_gauge gauge\n"
        "vproxy_test_case_gauge{class=\"TestPrometheus\",method=\"gauge\"} 7\n")


def test_order_removal_and_negative_gauge():
    """Same-name metrics keep creation order even when added out of order;
    removed metrics vanish; a gauge below zero prints as a signed long;
    an empty set prints nothing."""
    m = P.Metrics()
    assert m.toString() == ""
    a = P.Gauge("b", {"k": "1"})
    b = P.Gauge("b", {"k": "2"})
    c = P.Counter("a", {})
    m.add(b)
    m.add(c)
    m.add(a)
    a.decr(5)
    assert m.toString() == ("# TYPE a counter\na{} 0\n"
                            "# TYPE b gauge\nb{k=\"1\"} -5\nb{k=\"2\"} 0\n")
    m.remove(a)
    assert m.toString() == "# TYPE a counter\na{} 0\n# TYPE b gauge\nb{k=\"2\"} 0\n"


def test_label_quoting():
    """Label values are JSON string literals (SimpleString.stringify)."""
    v = "a\"b\\c\b\f\n\r\t\x01\x1f\x7f~ \xe9"
    text = P.format_metrics([P.Counter("m", {"z": v, "a": ""})])
    assert text == ("# TYPE m counter\n"
                    "m{a=\"\",z=\"a\\\"b\\\\c\\b\\f\\n\\r\\t\\u0001\\u001f\\u007f~ \\u00e9\"} 0\n")


def _hits(**kw):
    return P.hits_text(**kw)


def test_hit_counter_layout():
    acl = np.array([5, 0, 7, 1, 2], np.uint64)       # 2 tcp, 1 udp, tcp default, udp default
    route = np.array([3, 4, 9, 10], np.uint64)       # 1 v4, 1 v6, v4 none, v6 none
    group = np.array([11, 12, 13], np.uint64)        # 2 groups, none
    text = _hits(acl=acl, n_tcp=2, n_udp=1, route=route, n4=1, n6=1, group=group, n_groups=2)
    lines = text.splitlines()
    assert lines[0] == "# HELP route_table_rule_hit_count " \
        "Lookups matched per RouteTable rule (list index, or none)"
    assert lines[1] == "# TYPE route_table_rule_hit_count counter"
    assert lines[2:6] == [
        'route_table_rule_hit_count{family="v4",rule="0"} 3',
        'route_table_rule_hit_count{family="v6",rule="0"} 4',
        'route_table_rule_hit_count{family="v4",rule="none"} 9',
        'route_table_rule_hit_count{family="v6",rule="none"} 10']
    assert lines[7] == "# TYPE security_group_rule_hit_count counter"
    assert lines[8:13] == [
        'security_group_rule_hit_count{protocol="TCP",rule="0"} 5',
        'security_group_rule_hit_count{protocol="TCP",rule="1"} 0',
        'security_group_rule_hit_count{protocol="UDP",rule="0"} 7',
        'security_group_rule_hit_count{protocol="TCP",rule="default"} 1',
        'security_group_rule_hit_count{protocol="UDP",rule="default"} 2']
    assert lines[14] == "# TYPE upstream_server_group_hit_count counter"
    assert lines[15:] == ['upstream_server_group_hit_count{group="0"} 11',
                          'upstream_server_group_hit_count{group="1"} 12',
                          'upstream_server_group_hit_count{group="none"} 13']
    assert _hits(group=group, n_groups=2).count("\n") == 5
    big = _hits(group=np.arange(2001, dtype=np.uint64), n_groups=2000)   # > first 4 KiB buffer
    assert big.count("\n") == 2003 and big.endswith('{group="none"} 2000\n')


def test_extra_labels():
    """getExtraLabels: blank pieces skipped, key before the first '=', later
    keys win, extra labels override the metric's own (putAll order)."""
    group = np.array([1, 2], np.uint64)
    text = _hits(group=group, n_groups=1,
                 extra_labels=" ,zone=a=b,, host=h1,zone=eu,group=X,\t")
    assert text.splitlines()[2:] == [
        'upstream_server_group_hit_count{ host="h1",group="X",zone="eu"} 1',
        'upstream_server_group_hit_count{ host="h1",group="X",zone="eu"} 2']
    with pytest.raises(_lib.IllegalArgumentException):
        _hits(group=group, n_groups=1, extra_labels="a=1,broken")
    assert _hits(group=group, n_groups=1, extra_labels="") == _hits(group=group, n_groups=1)


def test_buffer_too_small_reports_length():
    import ctypes as C
    L = _lib.lib()
    need = C.c_int64(0)
    buf = C.create_string_buffer(8)
    g = np.array([1, 2], np.uint64)
    rc = L.vc_prometheus_hits(None, 0, 0, None, 0, 0, C.c_void_p(g.ctypes.data), 1, None, buf, 8,
                              C.byref(need))
    assert rc == _lib.VC_ENOMEM
    assert need.value == len(_hits(group=g, n_groups=1))
    rc = L.vc_prometheus_hits(None, 0, 0, None, 0, 0, C.c_void_p(g.ctypes.data), 1, None, None, 0,
                              C.byref(need))
    assert rc == _lib.VC_ENOMEM
