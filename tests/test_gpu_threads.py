"""GPU tier: classify calls from several threads while the control thread
recompiles (SURVEY.md §8(b) "Threading": classify is reentrant across
event-loop threads; a recompile publishes a new immutable snapshot and a
call classifies against the tables it started with).  Every result of every
call must equal the oracle over ONE of the two alternating rule sets --
never a mix -- including host calls that span several 4M-item chunks."""
import threading

import numpy as np
import pytest

import oracle_ffi as O
import vproxy_amd as V
from vproxy_amd import workloads as W

pytestmark = pytest.mark.gpu


def test_concurrent_classify_and_recompile():
    clf = V.Classifier(0)
    sets = [W.gen_sg_rules(400, 91), W.gen_sg_rules(400, 92)]
    ctypes_sets = []
    for tcp, udp in sets:
        a, na, ka = W.as_ctypes(tcp, V._lib.VcAclRule)
        b, nb, kb = W.as_ctypes(udp, V._lib.VcAclRule)
        ctypes_sets.append((a, na, b, nb, ka, kb))
    compile_ = lambda k: V.check(V.lib().vc_compile_acl(clf.h, ctypes_sets[k][0], ctypes_sets[k][1],
                                                        ctypes_sets[k][2], ctypes_sets[k][3], 0))
    compile_(0)
    n = 9_000_001                                   # three host chunks
    proto, src, port = W.gen_acl_queries(sets[0][0], sets[0][1], n, 93)
    samp = np.random.default_rng(94).integers(0, n, 20000)
    want = [O.sg_batch_v4_np(t, u, False, proto[samp], src[samp], port[samp])[0] for t, u in sets]
    assert (want[0] != want[1]).mean() > 0.3
    full = []
    for k in range(2):                              # full expected outputs, from the GPU itself
        compile_(k)
        full.append(clf.acl_v4(proto, src, port)[0])
        np.testing.assert_array_equal(full[k][samp], want[k])
    errors, stop, calls = [], threading.Event(), []

    def worker():
        try:
            while not stop.is_set():
                got, _ = clf.acl_v4(proto, src, port)
                calls.append(1)
                if not (np.array_equal(got, full[0]) or np.array_equal(got, full[1])):
                    errors.append("mixed snapshot result")
                    return
        except Exception as e:             # noqa: BLE001
            errors.append(repr(e))

    threads = [threading.Thread(target=worker) for _ in range(3)]
    for t in threads:
        t.start()
    for i in range(12):
        compile_(i % 2)
    for _ in range(400):                          # classify calls overlapped the recompiles
        if len(calls) >= 6 or errors:
            break
        compile_(len(calls) % 2)
    stop.set()
    for t in threads:
        t.join(timeout=120)
    clf.close()
    assert not errors, errors[:3]
