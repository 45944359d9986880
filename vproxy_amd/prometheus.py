"""Prometheus text exposition over libvclassify.

Mirrors vproxybase.prometheus (Metrics / Counter / Gauge,
base/src/main/java/vproxybase/prometheus/*.java) so a caller that keeps
its own counters renders them exactly as vproxy does; the formatting runs
in the library (vc_prometheus_format).  `hits_text` and
`Classifier.counters_prometheus` render the per-rule hit counters the GPU
paths keep (vc_prometheus_hits / vc_counters_prometheus).
"""
import ctypes as C
import itertools

from . import _lib
from ._lib import METRIC_COUNTER, METRIC_GAUGE, VcMetric, check, lib

_index = itertools.count(1)   # Metric.indexes (Metric.java:9,16)


def _b(s):
    return s.encode("latin-1") if isinstance(s, str) else bytes(s)


def _call_text(fn, *args):
    """Run a vc text function, growing the buffer once if it was too small."""
    need = C.c_int64(0)
    cap = 4096
    while True:
        buf = C.create_string_buffer(cap)
        rc = fn(*args, buf, cap, C.byref(need))
        if rc == _lib.VC_ENOMEM and need.value >= cap:
            cap = need.value + 1
            continue
        check(rc)
        return buf.raw[:need.value].decode("latin-1")


class Metric:
    """Metric.java: name + labels, creation index for the output order."""
    type_code = None

    def __init__(self, metric, labels):
        self.index = next(_index)
        self.metric = metric
        self.labels = dict(labels)

    def value(self):
        raise NotImplementedError


class Counter(Metric):
    """Counter.java (LongAdder)."""
    type_code = METRIC_COUNTER

    def __init__(self, metric, labels):
        super().__init__(metric, labels)
        self._v = 0

    def incr(self, n):
        self._v += int(n)

    def longValue(self):
        return self._v

    def clear(self):
        self._v = 0

    def value(self):
        return self._v


class Gauge(Counter):
    """Gauge.java: same value semantics, type "gauge"."""
    type_code = METRIC_GAUGE

    def decr(self, n):
        self._v -= int(n)


class Metrics:
    """Metrics.java: add / remove / registerHelpMessage / toString."""

    def __init__(self):
        self._metrics = {}
        self._help = {}

    def add(self, metric):
        self._metrics[id(metric)] = metric

    def remove(self, metric):
        self._metrics.pop(id(metric), None)

    def registerHelpMessage(self, metric, message):
        self._help[metric] = message

    def toString(self):
        ms = sorted(self._metrics.values(), key=lambda m: m.index)
        return format_metrics(ms, self._help)

    __str__ = toString


def format_metrics(metrics, help_messages=None):
    """vc_prometheus_format over Metric objects given in creation order."""
    metrics = list(metrics)
    keep = []
    arr = (VcMetric * max(1, len(metrics)))()
    for i, m in enumerate(metrics):
        keys = (C.c_char_p * max(1, len(m.labels)))(*[_b(k) for k in m.labels])
        vals = (C.c_char_p * max(1, len(m.labels)))(*[_b(v) for v in m.labels.values()])
        keep += [keys, vals]
        arr[i].metric = _b(m.metric)
        arr[i].type = m.type_code
        arr[i].n_labels = len(m.labels)
        arr[i].label_keys = keys
        arr[i].label_values = vals
        arr[i].value = m.value()
    help_messages = help_messages or {}
    hk = (C.c_char_p * max(1, len(help_messages)))(*[_b(k) for k in help_messages])
    hv = (C.c_char_p * max(1, len(help_messages)))(*[_b(v) for v in help_messages.values()])
    return _call_text(lib().vc_prometheus_format, arr, len(metrics), hk, hv, len(help_messages))


def hits_text(acl=None, n_tcp=0, n_udp=0, route=None, n4=0, n6=0, group=None, n_groups=0,
              extra_labels=None):
    """vc_prometheus_hits over host uint64 counter arrays (VC_COUNTERS_* layouts)."""
    import numpy as np

    def arr(a, n):
        if a is None:
            return None, None
        a = np.ascontiguousarray(a, dtype=np.uint64)
        if len(a) < n:
            raise _lib.IllegalArgumentException("counter array shorter than its layout")
        return a, C.c_void_p(a.ctypes.data)

    a, pa = arr(acl, n_tcp + n_udp + 2)
    r, pr = arr(route, n4 + n6 + 2)
    g, pg = arr(group, n_groups + 1)
    return _call_text(lib().vc_prometheus_hits, pa, n_tcp, n_udp, pr, n4, n6, pg, n_groups,
                      None if extra_labels is None else _b(extra_labels))
