"""CPU tier: the DNS drain-loop batcher's fallback (tests/native/dnsd_loop.c,
the C replay of jni/DnsDrainBatcher.java) with injected call statuses: no
GPU is touched.  VC_ESTATE (IllegalStateException: nothing compiled yet)
answers that batch with the Java loop body and tries the GPU again on the
next; VC_EDEVICE / VC_ENOMEM (IOException) marks the context dead and every
later batch takes the Java path; any other status is a caller bug and is
returned, not swallowed."""
import numpy as np
import pytest

import dnsd_loop as L
from vproxy_amd import workloads as W


def _queue(n):
    blob, off = W.pack([b"\x00" * (12 + i % 5) for i in range(n)])
    return blob, off, np.full(n, 4, np.uint8), np.zeros(n, np.uint32), \
        np.zeros((n, 16), np.uint8), np.full(n, 53, np.uint16)


def test_state_is_per_batch_device_is_sticky():
    q = _queue(10)
    t = L.trace(None, *q, batch=3, inject=[L.ESTATE, L.ESTATE, L.EDEVICE])
    js = lambda a, b: sum((["J", str(i)] for i in range(a, b)), [])
    assert t == ["F"] + js(0, 3) + ["F"] + js(3, 6) + ["D"] + js(6, 10)


@pytest.mark.parametrize("rc", [L.EDEVICE, L.ENOMEM])
def test_device_errors_kill_the_context(rc):
    q = _queue(7)
    assert L.trace(None, *q, batch=2, inject=[rc]) == ["D"] + sum(
        (["J", str(i)] for i in range(7)), [])


def test_caller_bug_is_not_a_fallback():
    q = _queue(4)
    with pytest.raises(AssertionError):
        L.trace(None, *q, batch=2, inject=[L.ESTATE])   # 2nd call reaches the library: EINVAL
