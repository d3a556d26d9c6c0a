"""Failure paths a healthy GPU never takes, driven by the library's fault
hook (crc32c_test_inject, api_internal.h pech_fault_site):

* the drop-in crc32c() stays total: a failed GPU leg is recomputed on the
  host, exactly (SURVEY.md §8(b) "Errors": the reference cannot fail,
  include/crc32c.h:88-96);
* the async layer: a failed launch or payload DMA fails the
  payloads of that slot through their callbacks (err < 0), makes the
  context's error sticky, wakes the eventfd, and never strands a later
  callback; a submission that returns an error gets no callback.
Run on the GPU box (-m gpu)."""
import ctypes
import select

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

SITE_DROPIN_GPU, SITE_ASYNC_LAUNCH, SITE_ASYNC_DMA = 0, 1, 2


def inject(site, countdown):
    from pech_amd import _lib

    L = _lib.lib()
    L.crc32c_test_inject.argtypes = [ctypes.c_int, ctypes.c_int]
    assert L.crc32c_test_inject(site, countdown) == 0


@pytest.fixture(autouse=True)
def disarm():
    yield
    for s in (SITE_DROPIN_GPU, SITE_ASYNC_LAUNCH, SITE_ASYNC_DMA):
        inject(s, 0)


def test_dropin_gpu_failure_recomputed_on_host():
    import pech_amd as P

    rng = np.random.default_rng(41)
    prev = P.set_cpu_max(0)
    try:
        before = P.stats()
        d = rng.integers(0, 256, 100000, dtype=np.uint8)
        inject(SITE_DROPIN_GPU, 2)  # the second GPU call fails
        assert P.crc32c(1, d) == O.crc(1, d)
        assert P.crc32c(2, d) == O.crc(2, d)
        assert P.crc32c(3, d) == O.crc(3, d)
        after = P.stats()
        assert after["gpu_fallbacks"] == before["gpu_fallbacks"] + 1
        assert after["gpu_calls"] == before["gpu_calls"] + 2
    finally:
        P.set_cpu_max(prev)


def _wait(ac, timeout=60.0):
    fd = ac.fd()
    while ac.pending():
        r, _, _ = select.select([fd], [], [], timeout)
        assert r, f"eventfd never became readable, {ac.pending()} pending"
        ac.complete()


def test_async_launch_failure_fails_its_slot_then_sticky():
    import pech_amd as P

    rng = np.random.default_rng(42)
    ac = P.AsyncCrc()
    got = {}
    bufs = [rng.integers(0, 256, 5000 + i, dtype=np.uint8) for i in range(6)]
    cb = lambda i: (lambda crc, err: got.__setitem__(i, (crc, err)))  # noqa: E731
    # batch 1 (payloads 0, 1) launches normally
    for i in (0, 1):
        ac.submit(bufs[i].ctypes.data, bufs[i].size, i, cb(i), keep=bufs[i])
    ac.flush()
    # batch 2 (payloads 2, 3): its launch fails
    for i in (2, 3):
        ac.submit(bufs[i].ctypes.data, bufs[i].size, i, cb(i), keep=bufs[i])
    inject(SITE_ASYNC_LAUNCH, 1)
    with pytest.raises(P.Crc32cError):
        ac.flush()
    # the context's error is sticky: later submissions are refused (no callback)
    with pytest.raises(P.Crc32cError):
        ac.submit(bufs[4].ctypes.data, bufs[4].size, 4, cb(4), keep=bufs[4])
    _wait(ac)  # the eventfd woke the loop; every accepted payload completed
    assert got[0] == (O.crc(0, bufs[0]), 0)
    assert got[1] == (O.crc(1, bufs[1]), 0)
    assert got[2][1] < 0 and got[3][1] < 0
    assert 4 not in got
    assert list(got) == [0, 1, 2, 3]  # submission order
    ac.close()


def test_async_dma_failure_mid_slot():
    import pech_amd as P

    rng = np.random.default_rng(43)
    ac = P.AsyncCrc()  # DMA mode: crc32c_pages payloads are DMA'd to the slot
    pages = [P.Pages(3) for _ in range(4)]
    for pg in pages:
        pg.view[:] = rng.integers(0, 256, pg.nbytes, dtype=np.uint8)
    got = {}
    cb = lambda i: (lambda crc, err: got.__setitem__(i, (crc, err)))  # noqa: E731
    ac.submit(pages[0].ptr, pages[0].nbytes, 0, cb(0))
    ac.flush()  # payload 0 in flight in its own slot
    ac.submit(pages[1].ptr, pages[1].nbytes, 1, cb(1))  # slot 2, DMA'd
    inject(SITE_ASYNC_DMA, 1)
    with pytest.raises(P.Crc32cError):  # payload 2's DMA fails: no callback for it
        ac.submit(pages[2].ptr, pages[2].nbytes, 2, cb(2))
    with pytest.raises(P.Crc32cError):  # drain reports the sticky error after the callbacks ran
        ac.drain()
    assert got[0] == (O.crc(0, pages[0].view), 0)
    assert got[1][1] < 0  # shared the failed slot
    assert 2 not in got
    assert ac.pending() == 0
    ac.close()
    for pg in pages:
        pg.free()


def test_async_context_after_failure_is_replaceable():
    # a fresh context works after one failed (the failure is per context)
    import pech_amd as P

    d = np.random.default_rng(44).integers(0, 256, 70000, dtype=np.uint8)
    ac = P.AsyncCrc()
    got = []
    ac.submit(d.ctypes.data, d.size, 9, lambda crc, err: got.append((crc, err)), keep=d)
    ac.drain()
    assert got == [(O.crc(9, d), 0)]
    ac.close()
