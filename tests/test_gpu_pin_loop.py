"""GPU tier: readers never wait for a recompile at the Java boundary.

jni/GpuContext.java pins each published state (a View: vc_pin_acquire's
snapshots + the Java lists their indices refer to) and maps every batch
through the view it ran on, with no lock across the native compile, as the
reference's copy-on-write swaps never block a reader
(core/src/main/java/vproxy/component/secure/SecurityGroup.java:56-103,
core/.../svrgroup/Upstream.java:146-157).  tests/native/pin_loop.c replays
that protocol through the JNI shim's pin natives: three event-loop threads
classify 64K-lookup route batches (RouteTable.lookup on registered direct
buffers, as the drain-loop batchers do) while the control thread recompiles
a C3-size route table (980,848 IPv4 + 200,000 IPv6 rules) ten times,
alternating the RouteTable's list and its reverse, so almost every lookup
changes its answer at each swap.  Every batch's outputs must equal its own
view's table, every pin must report its view's generation, and the p99
batch latency during the recompiles must stay near the quiet one.  The
round-5 protocol (a read-write lock around compile and batch) is run beside
it as the contrast the verdict measured: there a batch waits for a compile.
"""
import ctypes as C
import json
import os
import subprocess

import numpy as np
import pytest

import vproxy_amd as V
from vproxy_amd import workloads as W

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
NATIVE = os.path.join(HERE, "native")
ROOT = os.path.dirname(HERE)


class Cfg(C.Structure):
    _fields_ = [(k, C.c_int) for k in ("threads", "batch", "think_us", "quiet_ms", "tail_ms",
                                       "recompiles", "mode")]


class Stats(C.Structure):
    _fields_ = ([(k, C.c_int64) for k in ("batches_quiet", "batches_during", "batches_after")] +
                [(k, C.c_double) for k in ("p50_quiet", "p99_quiet", "max_quiet", "p50_during",
                                           "p99_during", "max_during", "compile_ms_mean",
                                           "compile_ms_max")] +
                [(k, C.c_int64) for k in ("mismatches", "gen_mismatches", "errors",
                                          "views_used")] +
                [("table_batches", C.c_int64 * 2)] +
                [(k, C.c_int64) for k in ("retries", "differ", "slow_quiet", "slow_during")])


def _lib():
    subprocess.check_call(["make", "-s", "-C", NATIVE, "build/libpin_loop.so"])
    lib = C.CDLL(os.path.join(NATIVE, "build", "libpin_loop.so"))
    lib.pin_loop_run.restype = C.c_int
    lib.pin_loop_run.argtypes = ([C.c_int] + [C.c_void_p, C.c_int] * 4 +
                                 [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                                  C.POINTER(Cfg), C.POINTER(Stats)])
    return lib


@pytest.fixture(scope="module")
def tables():
    net, plen = W.gen_v4_prefixes(1_000_000, W.SEED + 3)
    hi, lo, p6 = W.gen_v6_prefixes(200_000, W.SEED + 4)
    rt = V.RouteTable()
    allnets = np.concatenate([W.v4_nets(net, plen), W.v6_nets(hi, lo, p6)])
    arr, n_all, keep = W.as_ctypes(allnets, V._lib.VcNet)
    rt.add_rules("bgp", arr, n=n_all)
    a4, n4 = rt.rules_raw(4)
    a6, n6 = rt.rules_raw(6)
    t4 = np.frombuffer(bytes(a4)[:n4 * 40], np.uint8).reshape(n4, 40).copy()
    t6 = np.frombuffer(bytes(a6)[:n6 * 40], np.uint8).reshape(n6, 40).copy()
    keys = W.v4_lookups(net, plen, 4 << 20, W.SEED + 61)
    del rt
    return t4, t6, t4[::-1].copy(), t6[::-1].copy(), keys


def _run(tables, mode):
    t4a, t6a, t4b, t6b, keys = tables
    exp_a = np.empty(len(keys), np.int32)
    exp_b = np.empty(len(keys), np.int32)
    cfg = Cfg(threads=3, batch=65536, think_us=200, quiet_ms=1500, tail_ms=300, recompiles=10,
              mode=mode)
    st = Stats()
    p = lambda a: C.c_void_p(a.ctypes.data)
    rc = _lib().pin_loop_run(0, p(t4a), len(t4a), p(t6a), len(t6a), p(t4b), len(t4b), p(t6b),
                             len(t6b), p(keys), len(keys), p(exp_a), p(exp_b), C.byref(cfg),
                             C.byref(st))
    assert rc == 0, rc
    d = {k: getattr(st, k) for k, _ in Stats._fields_ if k != "table_batches"}
    d["table_batches"] = list(st.table_batches)
    d["mode"] = "views+pins" if mode == 0 else "rwlock (round 5)"
    return d, exp_a, exp_b


def test_batches_never_wait_for_a_recompile(tables):
    pins, exp_a, exp_b = _run(tables, 0)
    lock, _, _ = _run(tables, 1)
    print("PINLOOP", json.dumps(pins))
    print("PINLOOP", json.dumps(lock))
    out = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "r06_pin_loop.jsonl"), "w") as f:
            f.write(json.dumps(pins) + "\n" + json.dumps(lock) + "\n")
    # the two tables answer differently almost everywhere, so a batch mapped
    # through the wrong view's lists could not pass
    assert pins["differ"] > 0.9 * len(exp_a)
    for d in (pins, lock):
        assert d["errors"] == 0 and d["mismatches"] == 0, d
        assert d["table_batches"][0] > 0 and d["table_batches"][1] > 0, d
        assert d["batches_quiet"] > 100 and d["batches_during"] > 0, d
    assert pins["batches_during"] > 1000, pins    # the event loops kept going
    assert pins["gen_mismatches"] == 0
    assert pins["views_used"] >= 8, pins          # batches ran on most of the 11 views
    # a compile (~150 ms) never shows in a batch's latency
    assert pins["compile_ms_mean"] > 50, pins
    assert pins["p99_during"] < pins["p99_quiet"] + 10.0, pins
    assert pins["max_during"] < 0.5 * pins["compile_ms_mean"], pins
    # the round-5 protocol: a batch that meets a recompile waits it out
    assert lock["max_during"] > 0.5 * lock["compile_ms_mean"], lock
