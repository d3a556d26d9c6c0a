"""Failure paths a healthy GPU never takes, driven by the fault-injection
hook (crc32c_test_inject, api_internal.h pech_fault_site).  The hook exists
only in the test build, build/lib_test.so (`make`, -DPECH_TEST_HOOKS): the
release library cannot be armed.  So every scenario runs in ONE child
process (this file run as a script, PECH_CRC32C_LIB=build/lib_test.so) and
each test below checks its scenario's outcome:

* the drop-in crc32c() stays total: a failed GPU leg is recomputed on the
  host, exactly (SURVEY.md §8(b) "Errors": the reference cannot fail,
  include/crc32c.h:88-96);
* the async layer: a failed launch or payload DMA fails the
  payloads of that slot through their callbacks (err < 0), makes the
  context's error sticky, wakes the eventfd, and never strands a later
  callback; a submission that returns an error gets no callback -- also the
  one whose own submit filled the slot and whose launch failed (under the
  messenger adapter too: no callback reaches a freed verify-queue entry);
* a batch whose stream fails after its launch never signals the eventfd;
  complete() finds it by asking the stream and fails its payloads;
* a flat launch whose waves gave up waiting for out[]'s initialisation, or
  whose async results publication is missing, never hands out a CRC: the
  drop-in recomputes, crc32c_batch fails, the async slot fails (-EIO) or
  copies the results, the adapter recomputes; all counted.
Run on the GPU box (-m gpu)."""
import ctypes
import json
import os
import select
import subprocess
import sys
import traceback

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TEST_LIB = os.path.join(REPO, "build", "lib_test.so")
SITE_DROPIN_GPU, SITE_ASYNC_LAUNCH, SITE_ASYNC_DMA, SITE_ASYNC_STREAM = 0, 1, 2, 3
SITE_FLAT_TIMEOUT, SITE_FLAT_NOPUB = 4, 5  # the flat kernel's fault bits (layout.h PECH_FLAT_T_*)
SLOT_DESCS, SLOT_BYTES = 8192, 32 << 20  # crc32c_async.cpp kSlotDescs / kSlotBytes


# ---- scenarios (run in the child, on build/lib_test.so) ---------------------
def inject(site, countdown):
    from pech_amd import _lib

    L = _lib.lib()
    L.crc32c_test_inject.argtypes = [ctypes.c_int, ctypes.c_int]
    assert L.crc32c_test_inject(site, countdown) == 0


def disarm():
    for s in (SITE_DROPIN_GPU, SITE_ASYNC_LAUNCH, SITE_ASYNC_DMA, SITE_ASYNC_STREAM, SITE_FLAT_TIMEOUT,
              SITE_FLAT_NOPUB):
        inject(s, 0)


def sc_dropin_gpu_failure_recomputed_on_host():
    import oracle_lib as O
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


def sc_async_launch_failure_fails_its_slot_then_sticky():
    import oracle_lib as O
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
    try:
        ac.flush()
        raise AssertionError("flush after an injected launch failure returned 0")
    except P.Crc32cError:
        pass
    # the context's error is sticky: later submissions are refused (no callback)
    try:
        ac.submit(bufs[4].ctypes.data, bufs[4].size, 4, cb(4), keep=bufs[4])
        raise AssertionError("submit on a failed context returned 0")
    except P.Crc32cError:
        pass
    _wait(ac)  # the eventfd woke the loop; every accepted payload completed
    assert got[0] == (O.crc(0, bufs[0]), 0)
    assert got[1] == (O.crc(1, bufs[1]), 0)
    assert got[2][1] < 0 and got[3][1] < 0
    assert 4 not in got and ac.stray == 0
    assert list(got) == [0, 1, 2, 3]  # submission order
    ac.close()


def sc_async_dma_failure_mid_slot():
    # CRC32C_ASYNC_DMA records the payload copies at submit and issues them
    # when the slot launches: a failed copy fails that slot's payloads
    # through their callbacks (the submits themselves made no HIP call and
    # succeeded), makes the error sticky, and drain reports it
    import oracle_lib as O
    import pech_amd as P

    rng = np.random.default_rng(43)
    ac = P.AsyncCrc(dma=True)
    pages = [P.Pages(3) for _ in range(4)]
    for pg in pages:
        pg.view[:] = rng.integers(0, 256, pg.nbytes, dtype=np.uint8)
    got = {}
    cb = lambda i: (lambda crc, err: got.__setitem__(i, (crc, err)))  # noqa: E731
    ac.submit(pages[0].ptr, pages[0].nbytes, 0, cb(0))
    ac.flush()  # payload 0 in flight in its own slot, its copy issued
    ac.submit(pages[1].ptr, pages[1].nbytes, 1, cb(1))  # slot 2: copies recorded
    ac.submit(pages[2].ptr, pages[2].nbytes, 2, cb(2))
    inject(SITE_ASYNC_DMA, 1)
    try:  # the slot's copies fail at its launch
        ac.drain()
        raise AssertionError("drain after a failed slot returned 0")
    except P.Crc32cError:
        pass
    assert got[0] == (O.crc(0, pages[0].view), 0)
    assert got[1][1] < 0 and got[2][1] < 0  # the failed slot's payloads
    try:  # sticky: later submissions are refused, no callback
        ac.submit(pages[3].ptr, pages[3].nbytes, 3, cb(3))
        raise AssertionError("submit on a failed context returned 0")
    except P.Crc32cError:
        pass
    assert 3 not in got and ac.stray == 0
    assert ac.pending() == 0
    ac.close()
    for pg in pages:
        pg.free()


def sc_submit_that_fills_the_slot_fails_without_callback():
    # the payload whose own submit filled the slot
    # (kSlotDescs pieces) and whose launch failed gets an error return and
    # NO callback; the slot's earlier payloads get err < 0 callbacks
    import pech_amd as P

    rng = np.random.default_rng(45)
    data = rng.integers(0, 256, 64, dtype=np.uint8)
    ac = P.AsyncCrc()
    got = {}
    cb = lambda i: (lambda crc, err: got.__setitem__(i, (crc, err)))  # noqa: E731
    for i in range(SLOT_DESCS - 1):
        ac.submit(data.ctypes.data, 64, i, cb(i), keep=data)
    inject(SITE_ASYNC_LAUNCH, 1)
    try:
        ac.submit(data.ctypes.data, 64, SLOT_DESCS - 1, cb(SLOT_DESCS - 1), keep=data)
        raise AssertionError("the submit that filled the failed slot returned 0")
    except P.Crc32cError:
        pass
    _wait(ac)
    assert SLOT_DESCS - 1 not in got and ac.stray == 0
    assert len(got) == SLOT_DESCS - 1 and all(e < 0 for _, e in got.values())
    ac.close()


def sc_msgr_submit_that_fills_the_slot_is_recomputed_once():
    # the same failure under the messenger adapter (crc32c_msgr.c): the
    # refused payload is recomputed on the host at once, and since no
    # callback follows, rx_next may free its entry before complete() runs
    import oracle_lib as O
    import pech_amd as P
    from pech_amd import _lib

    L = _lib.lib()
    prev = L.crc32c_msgr_set_host_max(0)  # every checked payload to the GPU
    released = []
    REL = ctypes.CFUNCTYPE(None, ctypes.c_void_p)
    rel = REL(lambda m: released.append(m))
    ac = P.AsyncCrc()
    conn = L.crc32c_msgr_conn_create(ac.handle, 16, None, None, ctypes.cast(rel, ctypes.c_void_p))
    assert conn
    try:
        rng = np.random.default_rng(46)
        big = rng.integers(0, 256, SLOT_BYTES, dtype=np.uint8)  # fills a staging slot by itself
        want = O.crc(0, big)
        inject(SITE_ASYNC_LAUNCH, 1)
        assert L.crc32c_msgr_rx_queue(conn, ctypes.c_void_p(7), big.ctypes.data, big.size, 1, want) == 0
        msg, crc = ctypes.c_void_p(), ctypes.c_uint32()
        assert L.crc32c_msgr_rx_next(conn, ctypes.byref(msg), ctypes.byref(crc)) == 1  # recomputed, entry freed
        assert msg.value == 7 and crc.value == want
        for _ in range(3):  # no callback may reach the freed entry
            L.crc32c_async_complete(ac.handle)
        assert ac.pending() == 0
        st = _lib.CMsgrStats()
        L.crc32c_msgr_get_stats(ctypes.byref(st))
        assert st.rx_host >= 1 and st.rx_verified >= 1 and st.rx_bad == 0
        assert released == []
    finally:
        L.crc32c_msgr_conn_destroy(conn)
        L.crc32c_msgr_set_host_max(prev)
        ac.close()


def sc_failed_stream_found_by_complete():
    # a batch whose stream fails after the launch never runs
    # its host function, so the eventfd stays quiet; complete() (called from
    # the loop's timer) asks the stream and fails the batch's payloads
    import oracle_lib as O
    import pech_amd as P

    rng = np.random.default_rng(47)
    d = rng.integers(0, 256, 10000, dtype=np.uint8)
    ac = P.AsyncCrc()
    got = []
    ac.submit(d.ctypes.data, d.size, 3, lambda crc, err: got.append((crc, err)), keep=d)
    ac.flush()
    ac.drain()
    assert got == [(O.crc(3, d), 0)]
    inject(SITE_ASYNC_STREAM, 1)
    ac.submit(d.ctypes.data, d.size, 4, lambda crc, err: got.append((crc, err)), keep=d)
    ac.flush()
    r, _, _ = select.select([ac.fd()], [], [], 1.0)
    assert not r, "the eventfd fired for a batch whose host function never ran"
    for _ in range(200):  # the timer
        ac.complete()
        if len(got) == 2:
            break
        select.select([], [], [], 0.01)
    assert len(got) == 2 and got[1][1] < 0
    assert ac.pending() == 0
    ac.close()


def sc_failed_stream_found_by_drain():
    # the BLOCKING wait (drain, destroy) on a batch whose
    # stream failed -- its host function never runs, so `finished` is never
    # set -- must see the failure from the stream query and end
    import pech_amd as P

    d = np.random.default_rng(48).integers(0, 256, 10000, dtype=np.uint8)
    ac = P.AsyncCrc()
    got = []
    inject(SITE_ASYNC_STREAM, 1)
    ac.submit(d.ctypes.data, d.size, 5, lambda crc, err: got.append((crc, err)), keep=d)
    ac.flush()
    try:
        ac.drain()
        raise AssertionError("drain over a failed stream returned 0")
    except P.Crc32cError:
        pass
    assert len(got) == 1 and got[0][1] < 0
    assert ac.pending() == 0 and ac.stray == 0
    ac.close()


def sc_failed_stream_found_by_blocked_submit():
    # ... and the submit that must wait for a free slot while every slot is
    # in flight and the oldest one's stream failed: an error return for it
    # (no callback), err < 0 for the failed slot's payload, exact CRCs for
    # the slots that ran
    import oracle_lib as O
    import pech_amd as P

    rng = np.random.default_rng(49)
    bufs = [rng.integers(0, 256, 3000 + i, dtype=np.uint8) for i in range(5)]
    ac = P.AsyncCrc()
    got = {}
    cb = lambda i: (lambda crc, err: got.__setitem__(i, (crc, err)))  # noqa: E731
    inject(SITE_ASYNC_STREAM, 1)  # the first launch's stream "fails"
    for i in range(4):  # four slots in flight (kMaxSlots)
        ac.submit(bufs[i].ctypes.data, bufs[i].size, i, cb(i), keep=bufs[i])
        ac.flush()
    try:
        ac.submit(bufs[4].ctypes.data, bufs[4].size, 4, cb(4), keep=bufs[4])
        raise AssertionError("a submit blocked on a failed slot returned 0")
    except P.Crc32cError:
        pass
    try:
        ac.drain()
    except P.Crc32cError:
        pass  # the context's error is sticky
    assert got[0][1] < 0
    for i in (1, 2, 3):
        assert got[i] == (O.crc(i, bufs[i]), 0), (i, got.get(i))
    assert 4 not in got and ac.pending() == 0 and ac.stray == 0
    ac.close()


# ---- flat launches that void or miss their results ---------
# The test library arms the flat kernel's own fault bits (layout.h
# PECH_FLAT_T_*): every wave that waits for out[]'s initialisation times out
# at once (its results are void and the kernel reports PECH_FLAT_ERR), or the
# async slot's in-kernel publication is skipped.  No wrong CRC may reach a
# caller: the drop-in recomputes on the host, crc32c_batch fails loudly, the
# async layer fails the slot's payloads (-EIO, not sticky) or copies the
# results from the GPU, the adapter recomputes on the host; every event is
# counted.
def _big_payloads(rng, k, size=1 << 20):
    return [rng.integers(0, 256, size + 977 * i, dtype=np.uint8) for i in range(k)]


def sc_flat_timeout_dropin_recomputed_on_host():
    import oracle_lib as O
    import pech_amd as P

    rng = np.random.default_rng(51)
    prev = P.set_cpu_max(0)  # every call through the GPU: > 64 KiB is one flat launch
    try:
        d = rng.integers(0, 256, 300000, dtype=np.uint8)
        before = P.stats()
        assert P.crc32c(5, d) == O.crc(5, d)
        inject(SITE_FLAT_TIMEOUT, 1)
        assert P.crc32c(6, d) == O.crc(6, d)  # voided on the GPU, recomputed on the host
        assert P.crc32c(7, d) == O.crc(7, d)
        after = P.stats()
        assert after["gpu_faults"] == before["gpu_faults"] + 1, (before, after)
        assert after["gpu_fallbacks"] == before["gpu_fallbacks"] + 1, (before, after)
        assert after["gpu_calls"] == before["gpu_calls"] + 2, (before, after)
    finally:
        P.set_cpu_max(prev)


def sc_flat_timeout_batch_fails_loudly():
    import oracle_lib as O
    import pech_amd as P

    rng = np.random.default_rng(52)
    bufs = _big_payloads(rng, 5)
    want = [O.crc(0, b) for b in bufs]
    assert P.crc32c_batch([b.tobytes() for b in bufs]) == want
    before = P.stats()
    inject(SITE_FLAT_TIMEOUT, 1)
    try:
        P.crc32c_batch([b.tobytes() for b in bufs])
        raise AssertionError("crc32c_batch returned results of a voided flat launch")
    except P.Crc32cError:
        pass
    assert P.crc32c_batch([b.tobytes() for b in bufs]) == want  # the next call is exact
    # a device entry point's caller reads the fault from the counters (device
    # memory from the library's own HIP runtime: this child process has
    # initialised it before torch could)
    from pech_amd import _lib
    L = _lib.lib()
    hip = ctypes.CDLL("libamdhip64.so.7")
    total = sum(b.size for b in bufs)
    dbuf, ddesc, dout, dws = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    wsb = L.crc32c_dev_workspace_bytes(len(bufs))
    for p, nb in ((dbuf, total), (ddesc, 16 * len(bufs)), (dout, 4 * len(bufs)), (dws, wsb)):
        assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(nb)) == 0
    try:
        descs = np.zeros(len(bufs), dtype=[("addr", "<u8"), ("len", "<u4"), ("seed", "<u4")])
        off = 0
        for i, b in enumerate(bufs):
            assert hip.hipMemcpy(ctypes.c_void_p(dbuf.value + off), b.ctypes.data_as(ctypes.c_void_p),
                                 ctypes.c_size_t(b.size), 1) == 0
            descs[i] = (dbuf.value + off, b.size, 0)
            off += b.size
        assert hip.hipMemcpy(ddesc, descs.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(descs.nbytes), 1) == 0
        res = np.zeros(len(bufs), dtype=np.uint32)
        for armed in (True, False):
            if armed:
                inject(SITE_FLAT_TIMEOUT, 1)
            assert L.crc32c_dev_batch_ws_async(ddesc, dout, len(bufs), dws, wsb, None) == 0
            assert hip.hipDeviceSynchronize() == 0
            if armed:
                mid = P.stats()
                assert mid["gpu_faults"] == before["gpu_faults"] + 2, (before, mid)
        assert hip.hipMemcpy(res.ctypes.data_as(ctypes.c_void_p), dout, ctypes.c_size_t(res.nbytes), 2) == 0
        assert res.tolist() == want
        assert P.stats()["gpu_faults"] == mid["gpu_faults"]
    finally:
        for p in (dbuf, ddesc, dout, dws):
            hip.hipFree(p)


def sc_flat_timeout_async_slot_fails_not_sticky():
    import oracle_lib as O
    import pech_amd as P

    rng = np.random.default_rng(53)
    bufs = _big_payloads(rng, 6)
    ac = P.AsyncCrc()
    got = {}
    cb = lambda i: (lambda crc, err: got.__setitem__(i, (crc, err)))  # noqa: E731
    for i in (0, 1):  # one flat batch, exact
        ac.submit(bufs[i].ctypes.data, bufs[i].size, i, cb(i), keep=bufs[i])
    ac.drain()
    s0 = ac.stats()
    inject(SITE_FLAT_TIMEOUT, 1)
    for i in (2, 3):  # its batch is voided by the kernel: err < 0, no CRC
        ac.submit(bufs[i].ctypes.data, bufs[i].size, i, cb(i), keep=bufs[i])
    try:
        ac.drain()
    except P.Crc32cError:
        pass
    for i in (4, 5):  # not sticky: the next batch is exact
        ac.submit(bufs[i].ctypes.data, bufs[i].size, i, cb(i), keep=bufs[i])
    ac.drain()
    s1 = ac.stats()
    for i in (0, 1, 4, 5):
        assert got[i] == (O.crc(i, bufs[i]), 0), (i, got.get(i))
    assert got[2][1] < 0 and got[3][1] < 0, got
    assert s1["faults"] == s0["faults"] + 1 and s1["pub_missing"] == s0["pub_missing"], (s0, s1)
    assert ac.pending() == 0 and ac.stray == 0
    ac.close()


def sc_flat_missing_publication_never_stale():
    # the slot's host array still holds the previous batch's results when
    # the publication is skipped: the callbacks must get THIS batch's CRCs
    import oracle_lib as O
    import pech_amd as P

    rng = np.random.default_rng(54)
    bufs = _big_payloads(rng, 4)
    ac = P.AsyncCrc()
    got = {}
    cb = lambda i: (lambda crc, err: got.__setitem__(i, (crc, err)))  # noqa: E731
    for i in (0, 1):
        ac.submit(bufs[i].ctypes.data, bufs[i].size, i, cb(i), keep=bufs[i])
    ac.drain()
    s0 = ac.stats()
    inject(SITE_FLAT_NOPUB, 1)
    for i in (2, 3):  # same slot, same piece count: h_out holds batch 1's words
        ac.submit(bufs[i].ctypes.data, bufs[i].size, i, cb(i), keep=bufs[i])
    ac.drain()
    s1 = ac.stats()
    for i in range(4):
        assert got[i] == (O.crc(i, bufs[i]), 0), (i, got.get(i))
    assert s1["pub_missing"] == s0["pub_missing"] + 1 and s1["faults"] == s0["faults"], (s0, s1)
    assert s1["host_out"] >= s0["host_out"] + 1, (s0, s1)  # it was a publishing flat launch
    ac.close()


def sc_flat_timeout_under_the_adapter_is_recomputed():
    # the messenger adapter (crc32c_msgr.c) gets err < 0 for a voided batch
    # and checksums the payload on the host: the footer compare still sees
    # the exact CRC (rx_verified, no rx_bad)
    import oracle_lib as O
    import pech_amd as P
    from pech_amd import _lib

    L = _lib.lib()
    prev = L.crc32c_msgr_set_host_max(0)
    released = []
    REL = ctypes.CFUNCTYPE(None, ctypes.c_void_p)
    rel = REL(lambda m: released.append(m))
    ac = P.AsyncCrc()
    conn = L.crc32c_msgr_conn_create(ac.handle, 16, None, None, ctypes.cast(rel, ctypes.c_void_p))
    assert conn
    try:
        rng = np.random.default_rng(55)
        big = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
        want = O.crc(0, big)
        st0 = _lib.CMsgrStats()
        L.crc32c_msgr_get_stats(ctypes.byref(st0))
        inject(SITE_FLAT_TIMEOUT, 1)
        assert L.crc32c_msgr_rx_queue(conn, ctypes.c_void_p(9), big.ctypes.data, big.size, 1, want) == 0
        L.crc32c_async_flush(ac.handle)
        msg, crc = ctypes.c_void_p(), ctypes.c_uint32()
        for _ in range(2000):
            L.crc32c_async_complete(ac.handle)
            if L.crc32c_msgr_rx_next(conn, ctypes.byref(msg), ctypes.byref(crc)) == 1:
                break
            select.select([ac.fd()], [], [], 0.01)
        else:
            raise AssertionError("the voided payload never completed")
        assert msg.value == 9 and crc.value == want
        st = _lib.CMsgrStats()
        L.crc32c_msgr_get_stats(ctypes.byref(st))
        assert st.rx_verified == st0.rx_verified + 1 and st.rx_bad == st0.rx_bad, (st0.rx_verified, st.rx_verified)
        assert ac.stats()["faults"] >= 1
    finally:
        L.crc32c_msgr_conn_destroy(conn)
        L.crc32c_msgr_set_host_max(prev)
        ac.close()


def sc_context_after_failure_is_replaceable():
    # a fresh context works after one failed (the failure is per context)
    import oracle_lib as O
    import pech_amd as P

    d = np.random.default_rng(44).integers(0, 256, 70000, dtype=np.uint8)
    ac = P.AsyncCrc()
    got = []
    ac.submit(d.ctypes.data, d.size, 9, lambda crc, err: got.append((crc, err)), keep=d)
    ac.drain()
    assert got == [(O.crc(9, d), 0)]
    ac.close()


SCENARIOS = [n for n in list(globals()) if n.startswith("sc_")]


def child_main():
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    res = {}
    for name in SCENARIOS:
        try:
            globals()[name]()
            res[name] = "ok"
        except Exception:  # noqa: BLE001 -- reported to the parent test
            res[name] = traceback.format_exc()
        finally:
            disarm()
    print("FAULT_RESULTS " + json.dumps(res), flush=True)


# ---- the tests (parent process) ---------------------------------------------
@pytest.fixture(scope="module")
def results():
    assert os.path.exists(TEST_LIB), "build/lib_test.so is built by `make` (__graft_entry__.build())"
    env = dict(os.environ, PECH_CRC32C_LIB=TEST_LIB)
    r = subprocess.run([sys.executable, "-u", os.path.abspath(__file__)], capture_output=True, text=True,
                       timeout=300, env=env)
    line = [l for l in r.stdout.splitlines() if l.startswith("FAULT_RESULTS ")]
    assert r.returncode == 0 and line, (r.returncode, r.stdout[-3000:], r.stderr[-3000:])
    return json.loads(line[-1][len("FAULT_RESULTS "):])


@pytest.mark.gpu
@pytest.mark.parametrize("name", SCENARIOS)
def test_fault_scenario(results, name):
    assert results[name] == "ok", results[name]


def test_release_library_has_no_fault_hook():
    # failure injection is not exported by the release library
    out = subprocess.check_output(["nm", "-D", "--defined-only", os.path.join(REPO, "pech_amd", "libpech_crc32c.so")],
                                  text=True)
    assert "crc32c_test_" not in out  # no test hook at all (inject, cpu variants, stack switch)
    if os.path.exists(TEST_LIB):
        assert "crc32c_test_inject" in subprocess.check_output(["nm", "-D", "--defined-only", TEST_LIB], text=True)


if __name__ == "__main__":
    child_main()
