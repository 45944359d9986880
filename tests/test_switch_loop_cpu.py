"""CPU tier: the vswitch drain-loop batcher's fallback and receive rule
(tests/native/switch_loop.c, the C replay of jni/SwitchDrainBatcher.java)
with injected call statuses: no GPU is touched.  Decrypted (user-iface)
datagrams never reach the library; VC_ESTATE sends that batch's bare
datagrams down the Java body and retries the GPU on the next batch;
VC_EDEVICE / VC_ENOMEM mark the context dead for good; a batch size of 1
still makes progress (the blob holds at least one largest datagram); an
empty datagram ends the readable event as a 0-byte read does in
Switch.java:757-759."""
import numpy as np
import pytest

import switch_loop as L
from vproxy_amd import workloads as W


def _queue(n, decrypt_every=0, empty_at=()):
    dg = [b"" if i in empty_at else b"\x08" + b"\x00" * (15 + i % 7) for i in range(n)]
    blob, off = W.pack(dg)
    dec = np.array([decrypt_every and i % decrypt_every == 0 for i in range(n)], np.uint8)
    return blob, off, dec, np.full(n, 4, np.uint8), np.zeros(n, np.uint32), np.zeros((n, 16), np.uint8)


def _js(idx):
    return sum((["J", str(i)] for i in idx), [])


def test_state_is_per_batch_device_is_sticky():
    q = _queue(10)
    t = L.trace(None, *q, 4789, batch=3, inject=[L.ESTATE, L.ESTATE, L.EDEVICE])
    assert t == ["F"] + _js(range(0, 3)) + ["F"] + _js(range(3, 6)) + ["D"] + _js(range(6, 10)) + ["|"]


@pytest.mark.parametrize("rc", [L.EDEVICE, L.ENOMEM])
def test_device_errors_kill_the_context(rc):
    q = _queue(7)
    assert L.trace(None, *q, 4789, batch=2, inject=[rc]) == ["D"] + _js(range(7)) + ["|"]


def test_decrypted_never_reach_the_library():
    # every datagram decrypts: no call is made, so no injected status is used
    q = _queue(9, decrypt_every=1)
    t = L.trace(None, *q, 4789, batch=4, inject=[L.EDEVICE])
    assert t == sum((["E", str(i)] for i in range(9)), []) + ["|"]
    # mixed: the bare ones take the Java body after the failure, in arrival order
    q = _queue(8, decrypt_every=3)
    t = L.trace(None, *q, 4789, batch=8, inject=[L.EDEVICE])
    want = ["D"] + sum(((["E", str(i)] if i % 3 == 0 else ["J", str(i)]) for i in range(8)), [])
    assert t == want + ["|"]


def test_batch_of_one_progresses_and_empty_reads_end_events():
    q = _queue(6, empty_at=(2,))
    t = L.trace(None, *q, 4789, batch=1, inject=[L.EDEVICE])
    assert t == ["D", "J", "0", "J", "1", "|", "J", "3", "J", "4", "J", "5", "|"]


def test_caller_bug_is_not_a_fallback():
    q = _queue(4)
    with pytest.raises(AssertionError):
        L.trace(None, *q, 4789, batch=2, inject=[L.ESTATE])   # 2nd call reaches the library
