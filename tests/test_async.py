"""The messenger-facing layer (include/pech_crc32c_async.h, SURVEY §8f rows
1-3): eventfd-completed payload batches, pinned payload pages, CRC reuse by
concatenation.  CPU tests: the algebra and the C test program's build; GPU
tests: every callback bit-exact against the oracle (the reference loop)."""
import os
import re
import select
import subprocess

import numpy as np
import pytest

import oracle_lib as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ---- CPU -----------------------------------------------------------------
def test_concat_matches_oracle():
    # crc32c(seed, S0||S1||...) from zero-seeded segment CRCs: the REPOP
    # fan-out case (osd_server.c:1119 nested cursors, :1972 per replica)
    from pech_amd import crc32c_concat

    rng = np.random.default_rng(11)
    for trial in range(50):
        k = int(rng.integers(1, 8))
        segs = [rng.integers(0, 256, int(rng.integers(0, 5000)), dtype=np.uint8) for _ in range(k)]
        seed = int(rng.integers(0, 1 << 32)) if trial % 2 else 0
        crcs = [O.crc(0, s) for s in segs]
        want = O.crc(seed, np.concatenate(segs) if sum(len(s) for s in segs) else np.zeros(0, np.uint8))
        assert crc32c_concat(seed, crcs, [len(s) for s in segs]) == want
    assert crc32c_concat(0x1234, [], []) == 0x1234
    # lengths beyond 4 GiB (algebra only): concat == combine chain
    o = O.oracle()
    a, b, c = 0x11111111, 0x22222222, 0x33333333
    la, lb = (5 << 32) + 7, (1 << 33) + 3
    assert crc32c_concat(a, [b, c], [la, lb]) == o.oracle_combine(o.oracle_combine(a, b, la), c, lb)


def test_msgr_sim_builds_as_pech_c():
    # the test program is gnu89 C against the installed headers, -Werror
    exe = os.path.join(REPO, "build", "msgr_sim")
    r = subprocess.run(["make", "-s", "-C", REPO, "build/msgr_sim"], capture_output=True)
    assert r.returncode == 0, r.stderr.decode()
    assert os.path.exists(exe)


# ---- GPU -----------------------------------------------------------------
def _wait_all(ac, timeout=60.0):
    fd = ac.fd()
    while ac.pending():
        r, _, _ = select.select([fd], [], [], timeout)
        assert r, f"eventfd never became readable, {ac.pending()} pending"
        ac.complete()


@pytest.mark.gpu
@pytest.mark.parametrize("dma", [False, True])
def test_async_payloads_bit_exact(dma):
    # zero-copy (the default) and CRC32C_ASYNC_DMA (copies issued at launch)
    import pech_amd as P

    rng = np.random.default_rng(21 + dma)
    ac = P.AsyncCrc(dma=dma)
    sizes = [0, 1, 15, 16, 17, 4095, 4096, 4097, 65536, 1 << 20, (4 << 20) + 5, 123457]
    sizes = sizes * 6 + [int(x) for x in rng.integers(0, 300000, 100)]
    results, expect, keep = {}, {}, []
    for i, n in enumerate(sizes):
        seed = int(rng.integers(0, 1 << 32)) if i % 3 == 0 else 0
        if i % 2:
            pg = P.Pages(max(0, int(np.ceil(np.log2(max(n, 1) / 4096)))) if n > 4096 else 0)
            pg.view[:n] = rng.integers(0, 256, n, dtype=np.uint8)
            data, addr = pg.view[:n], pg.ptr
            keep.append(pg)
        else:
            data = rng.integers(0, 256, max(n, 1), dtype=np.uint8)[:n]
            addr = data.ctypes.data if n else data.ctypes.data
            keep.append(data)
        expect[i] = O.crc(seed, data)

        def cb(crc, err, i=i):
            assert err == 0
            results[i] = crc

        ac.submit(addr, n, seed, cb, keep=data)
        if i % 10 == 9:
            ac.flush()
    ac.flush()
    _wait_all(ac)
    assert results == expect
    order = list(results)
    assert order == sorted(order), "callbacks must run in submission order"
    ac.close()
    for k in keep:
        if isinstance(k, P.Pages):
            k.free()


@pytest.mark.gpu
def test_async_payload_larger_than_slots():
    # 70 MiB payloads are cut into pieces across 32 MiB staging slots and
    # folded back with crc32c_combine; more bytes than all slots in flight
    import pech_amd as P

    rng = np.random.default_rng(5)
    ac = P.AsyncCrc()
    bufs = [rng.integers(0, 256, (70 << 20) + 3 * i, dtype=np.uint8) for i in range(3)]
    got = {}
    for i, b in enumerate(bufs):
        ac.submit(b.ctypes.data, b.size, 0xFFFFFFFF, lambda crc, err, i=i: got.__setitem__(i, (crc, err)), keep=b)
    ac.drain()
    for i, b in enumerate(bufs):
        assert got[i] == (O.crc(0xFFFFFFFF, b), 0)
    ac.close()


@pytest.mark.gpu
def test_async_dma_wait_launches_the_next_slot():
    # CRC32C_ASYNC_DMA keeps one slot's copies in flight; a submit that waits
    # for a free slot harvests the oldest AND launches the next queued one
    # (it stayed queued until complete() or the next blocking
    # submit, so copy engine and GPU idled while the caller filled slots)
    import pech_amd as P

    rng = np.random.default_rng(8)
    ac = P.AsyncCrc(dma=True)
    pages = [P.Pages(11) for _ in range(17)]  # 8 MiB each: four fill a 32 MiB slot
    got, want = {}, {}
    for i, pg in enumerate(pages):
        pg.view[:] = rng.integers(0, 256, pg.nbytes, dtype=np.uint8)
        want[i] = O.crc(i, pg.view)
        ac.submit(pg.ptr, pg.nbytes, i, lambda crc, err, i=i: got.__setitem__(i, (crc, err)))
        st = ac.stats()
        if i == 15:  # four slots filled: the first launched, three queued behind it
            assert st["launches"] == 1 and st["inflight"] == 1 and st["queued"] == 3, st
    # the 17th submit waited for the first slot: the second is launched now
    assert st["launches"] == 2 and st["inflight"] == 1 and st["queued"] == 2, st
    assert st["submitted"] == 17
    ac.drain()
    assert got == {i: (want[i], 0) for i in range(17)}
    ac.close()
    for pg in pages:
        pg.free()


@pytest.mark.gpu
def test_async_context_per_device(monkeypatch):
    # one context per GPU of the PECH_DEVICES list (two on one GPU here), each
    # with its own counters; payloads spread over them complete bit-exact
    import pech_amd as P

    monkeypatch.setenv("PECH_DEVICES", "0,0")
    devs = P.async_devices()
    assert devs == [0, 0]
    ctxs = [P.AsyncCrc(device=d) for d in devs]
    rng = np.random.default_rng(9)
    got, want, keep = {}, {}, []
    for i in range(40):
        b = rng.integers(0, 256, int(rng.integers(1, 3 << 20)), dtype=np.uint8)
        keep.append(b)
        want[i] = O.crc(0, b)
        ctxs[i % 2].submit(b.ctypes.data, b.size, 0, lambda crc, err, i=i: got.__setitem__(i, (crc, err)), keep=b)
    for ac in ctxs:
        ac.drain()
    assert got == {i: (want[i], 0) for i in range(40)}
    for ac in ctxs:
        st = ac.stats()
        assert st["device"] == 0 and st["submitted"] == 20 and st["launches"] >= 1, st
        ac.close()
    monkeypatch.setenv("PECH_DEVICES", "0,99")
    with pytest.raises(P.Crc32cError):
        P.async_devices()


@pytest.mark.gpu
@pytest.mark.parametrize("host_out", ["1", "0"])
def test_async_results_stored_by_the_kernel(monkeypatch, host_out):
    """Flat and direct launches store a slot's results in its pinned host
    array themselves (no copy after the kernel; PECH_ASYNC_HOST_OUT=0 keeps
    the copy, as planned batches of more than 4,096 pieces always do), and a
    lone small batch is polled by the context's thread.  Lone payloads one at
    a time: 64 KiB and 1 MiB (flat), 4 KiB and 20 KiB pieces (direct), with
    and without seeds, a zero-length one; then slots of 300 x 40 KiB
    (plan + main at a flat limit of 256; pech_crc32c_flatg, stored by the
    kernel, at 4,096, the default), then one of 4,200 pieces, one
    of them 40 KiB (plan + main, results copied)."""
    import pech_amd as P

    monkeypatch.setenv("PECH_ASYNC_HOST_OUT", host_out)
    rng = np.random.default_rng(12)
    ac = P.AsyncCrc()
    got, want, keep = {}, {}, []
    sizes = [65536, 1 << 20, 4096, 20000, 0, 65536 + 3, 777]
    k = 0
    for rep in range(3):
        for L in sizes:
            b = rng.integers(0, 256, L, dtype=np.uint8)
            seed = int(rng.integers(0, 1 << 32)) if k % 2 else 0
            keep.append(b)
            want[k] = O.crc(seed, b)
            ac.submit(b.ctypes.data, L, seed, lambda crc, err, k=k: got.__setitem__(k, (crc, err)), keep=b)
            ac.drain()  # one batch in flight at a time: a lone batch
            k += 1
    st = ac.stats()
    assert got == {i: (want[i], 0) for i in range(k)}
    lone = st["launches"]
    assert lone >= 3 * (len(sizes) - 1), st
    assert st["polled"] == lone, st  # every lone batch of <= 8 MiB polled
    assert st["host_out"] == (lone if host_out == "1" else 0), st
    # 300 pieces in one slot: plan + main at a flat limit of 256,
    # pech_crc32c_flatg with results stored by the kernel at 4,096 (the default)
    base = dict(got)
    prev = P.set_flat_max(256)
    try:
        for fm, stored in ((256, 0), (4096, 1 if host_out == "1" else 0)):
            P.set_flat_max(fm)
            st1 = ac.stats()
            for i in range(300):
                b = rng.integers(0, 256, 40000, dtype=np.uint8)
                keep.append(b)
                want[k] = O.crc(i, b)
                ac.submit(b.ctypes.data, b.size, i, lambda crc, err, k=k: got.__setitem__(k, (crc, err)), keep=b)
                k += 1
            ac.drain()
            assert got == {i: (want[i], 0) for i in range(k)}
            st2 = ac.stats()
            assert st2["launches"] == st1["launches"] + 1, (st1, st2)
            assert st2["host_out"] - st1["host_out"] == stored, (fm, st1, st2)
    finally:
        P.set_flat_max(prev)
    # more than 4,096 pieces in one slot: plan + main, results copied
    P.set_flat_max(4096)
    for i in range(4200):
        b = rng.integers(0, 256, 40000 if i == 77 else 4096, dtype=np.uint8)
        keep.append(b)
        want[k] = O.crc(i, b)
        ac.submit(b.ctypes.data, b.size, i, lambda crc, err, k=k: got.__setitem__(k, (crc, err)), keep=b)
        k += 1
    ac.drain()
    assert got == {i: (want[i], 0) for i in range(k)}
    st3 = ac.stats()
    P.set_flat_max(prev)
    assert st3["launches"] == st2["launches"] + 1 and st3["host_out"] == st2["host_out"], (st2, st3)
    assert base.items() <= got.items()
    ac.close()


@pytest.mark.gpu
def test_pages_allocator():
    import pech_amd as P
    from pech_amd import _lib

    L = _lib.lib()
    a = P.Pages(0)
    b = P.Pages(4)
    assert a.ptr % 4096 == 0 and b.ptr % 4096 == 0
    assert L.crc32c_pages_is_pinned(a.ptr, 4096) == 1
    assert L.crc32c_pages_is_pinned(a.ptr + 100, 10) == 1
    assert L.crc32c_pages_is_pinned(a.ptr, 4097) == 0
    assert L.crc32c_pages_is_pinned(b.ptr, 4096 << 4) == 1
    host = np.zeros(8192, np.uint8)
    assert L.crc32c_pages_is_pinned(host.ctypes.data, 10) == 0
    pa = a.ptr
    a.free()
    assert L.crc32c_pages_is_pinned(pa, 4096) == 0  # freed (cached) pages are not live
    c = P.Pages(0)
    assert c.ptr == pa  # the per-order free list hands it back (src/page.c fast path)
    c.free()
    b.free()
    L.crc32c_pages_trim()


@pytest.mark.gpu
@pytest.mark.parametrize("zerocopy,contexts", [("0", "1"), ("1", "1"), ("1", "3")])
def test_msgr_sim_event_loop(zerocopy, contexts):
    # contexts > 1: one context per GPU in turn (several per GPU on a 1-GPU
    # box), all driven from one thread on one epoll set
    exe = os.path.join(REPO, "build", "msgr_sim")
    assert os.path.exists(exe), "build/msgr_sim is built by `make` (__graft_entry__.build())"
    r = subprocess.run([exe, "200", zerocopy, contexts], capture_output=True, timeout=120)
    assert r.returncode == 0, (r.stdout.decode(), r.stderr.decode())
    assert b"0 bad" in r.stdout


def test_msgr_conn_sim_builds_as_pech_c():
    r = subprocess.run(["make", "-s", "-C", REPO, "build/msgr_conn_sim"], capture_output=True)
    assert r.returncode == 0, r.stderr.decode()


@pytest.mark.gpu
@pytest.mark.parametrize("mode,corrupt,host_max", [("crc", "7", None), ("crc", "7", "0"), ("crc", "0", None),
                                                   ("nocrc", "0", None)])
def test_msgr_connection_state_machine(mode, corrupt, host_max):
    # tests/c/msgr_conn_sim.c: send-side held footers (a6), receive verify
    # queue with in-order dispatch and acks only after verification (a5, f1),
    # corruption -> -EBADMSG -> fault -> resend (no corrupted dispatch),
    # REPOP footers by CRC reuse / crc32c_concat of per-op GPU CRCs (f3),
    # NO_DATA_CRC / header-CRC gates (a10); every footer vs the reference chain
    exe = os.path.join(REPO, "build", "msgr_conn_sim")
    assert os.path.exists(exe), "build/msgr_conn_sim is built by `make`"
    # host_max: the adapter's size routing (crc32c_msgr_set_host_max): by
    # default payloads <= 8 KiB are checksummed on the host and the larger
    # ones on the GPU; "0" sends every checked payload to the GPU
    env = dict(os.environ)
    if host_max is not None:
        env["PECH_CRC32C_MSGR_HOST_MAX"] = host_max
    r = subprocess.run([exe, mode, "150", corrupt], capture_output=True, timeout=240, env=env)
    out = r.stdout.decode() + r.stderr.decode()
    assert r.returncode == 0, out[-4000:]
    assert " 0 errors" in out
    if mode == "crc" and corrupt != "0":
        assert "corrupted 0 " not in out  # the run did inject and catch corruption
    if mode == "crc":
        m = re.search(r"rx submitted (\d+) .* tx submitted (\d+) .*host-routed rx (\d+) tx (\d+)", out)
        rx_gpu, tx_gpu, rx_host, tx_host = map(int, m.groups())
        assert rx_gpu > 0 and tx_gpu > 0  # sizes above the cutoff went to the GPU
        if host_max == "0":
            assert rx_host == 0 and tx_host == 0
        else:  # 0/1/100/4096/4097-byte payloads stayed on the host
            assert rx_host > 0 and tx_host > 0


@pytest.mark.gpu
def test_msgr_lone_payloads_route_to_the_host():
    """Routing by queue depth (VERDICT r05 #4, crc32c_msgr.c route_host): a
    payload of at most crc32c_msgr_set_lone_max() bytes that finds its
    context idle, the first since the last flush, is checksummed on the host
    (rx_lone / tx_lone); the rest of a burst read in the same pass goes to
    the GPU; payloads above the cutoff always do; host_max 0 sends
    everything to the GPU.  Every CRC checked against the oracle."""
    import ctypes

    import pech_amd as P
    from pech_amd import _lib

    L = _lib.lib()
    released = []
    REL = ctypes.CFUNCTYPE(None, ctypes.c_void_p)
    rel = REL(lambda m: released.append(m))
    ac = P.AsyncCrc()
    conn = L.crc32c_msgr_conn_create(ac.handle, 64, None, None, ctypes.cast(rel, ctypes.c_void_p))
    assert conn
    rng = np.random.default_rng(61)
    bufs = [rng.integers(0, 256, n, dtype=np.uint8) for n in (65536, 65536, 65536, 65536, 200000, 1 << 20, 65536)]
    want = [O.crc(0, b) for b in bufs]

    def st():
        s = _lib.CMsgrStats()
        L.crc32c_msgr_get_stats(ctypes.byref(s))
        return {k: int(getattr(s, k)) for k, _ in _lib.CMsgrStats._fields_}

    def queue(i):
        assert L.crc32c_msgr_rx_queue(conn, ctypes.c_void_p(0x1000 + i), bufs[i].ctypes.data, bufs[i].size, 1,
                                      want[i]) == 0

    def take(n):
        got = []
        for _ in range(4000):
            L.crc32c_async_complete(ac.handle)
            m, c = ctypes.c_void_p(), ctypes.c_uint32()
            while len(got) < n:
                rc = L.crc32c_msgr_rx_next(conn, ctypes.byref(m), ctypes.byref(c))
                if rc != 1:
                    assert rc == 0, rc
                    break
                got.append((m.value - 0x1000, c.value))
            if len(got) == n:
                return got
            select.select([ac.fd()], [], [], 0.005)
        raise AssertionError(f"{n - len(got)} payload(s) never completed")

    prev_host = L.crc32c_msgr_set_host_max(8192)
    prev_lone = L.crc32c_msgr_set_lone_max(256 << 10)
    try:
        L.crc32c_async_flush(ac.handle)
        s0 = st()
        queue(0)  # queue depth 1: lone -> host
        assert take(1) == [(0, want[0])]
        L.crc32c_async_flush(ac.handle)
        s1 = st()
        assert s1["rx_lone"] == s0["rx_lone"] + 1 and s1["rx_host"] == s0["rx_host"] + 1
        assert s1["rx_submitted"] == s0["rx_submitted"]
        for i in (1, 2, 3, 4):  # a burst in one pass: the first lone, the rest batch on the GPU
            queue(i)
        L.crc32c_async_flush(ac.handle)
        assert take(4) == [(i, want[i]) for i in (1, 2, 3, 4)]
        s2 = st()
        assert s2["rx_lone"] == s1["rx_lone"] + 1 and s2["rx_submitted"] == s1["rx_submitted"] + 3, (s1, s2)
        queue(5)  # 1 MiB: above the lone cutoff, GPU even when idle
        L.crc32c_async_flush(ac.handle)
        assert take(1) == [(5, want[5])]
        s3 = st()
        assert s3["rx_lone"] == s2["rx_lone"] and s3["rx_submitted"] == s2["rx_submitted"] + 1
        L.crc32c_msgr_set_host_max(0)  # everything to the GPU, lone payloads too
        queue(6)
        L.crc32c_async_flush(ac.handle)
        assert take(1) == [(6, want[6])]
        s4 = st()
        assert s4["rx_lone"] == s3["rx_lone"] and s4["rx_submitted"] == s3["rx_submitted"] + 1
        L.crc32c_msgr_set_host_max(8192)
        # send side: a lone message's footer is ready at once (host), the
        # next one in the same pass is submitted
        crc = ctypes.c_uint32()
        assert L.crc32c_msgr_tx_submit(conn, ctypes.c_void_p(0x77), bufs[0].ctypes.data, bufs[0].size, 0) == 0
        assert L.crc32c_msgr_tx_submit(conn, ctypes.c_void_p(0x78), bufs[1].ctypes.data, bufs[1].size, 0) == 0
        s5 = st()
        assert s5["tx_lone"] == s4["tx_lone"] + 1 and s5["tx_submitted"] == s4["tx_submitted"] + 1
        assert L.crc32c_msgr_tx_footer(conn, ctypes.c_void_p(0x77), ctypes.byref(crc)) == 1 and crc.value == want[0]
        L.crc32c_async_flush(ac.handle)
        for _ in range(4000):
            L.crc32c_async_complete(ac.handle)
            if L.crc32c_msgr_tx_footer(conn, ctypes.c_void_p(0x78), ctypes.byref(crc)) == 1:
                break
            select.select([ac.fd()], [], [], 0.005)
        assert crc.value == want[1]
    finally:
        L.crc32c_msgr_set_host_max(prev_host)
        L.crc32c_msgr_set_lone_max(prev_lone)
        L.crc32c_msgr_conn_destroy(conn)
        ac.close()
    assert released == []


@pytest.mark.gpu
@pytest.mark.parametrize("il", ["1", "0"])
@pytest.mark.parametrize("k,size,off", [(8, 4 << 20, 0), (30, (1 << 20) - 100, 0), (64, 200 << 10, 17), (5, 131072, 0),
                                        (3, 131072 - 1, 64), (40, 1 << 20, 4095)])
def test_zero_copy_slots_interleaved_rows(monkeypatch, il, k, size, off):
    """Zero-copy slots of uniform payloads of >= 128 KiB (pinned crc32c_pages
    memory read in place) run the flat kernel on interleaved rows
    (PECH_FLAT_F_IL, crc32c_kernels.hip prologue_flat): the workgroup's 128
    lane groups over one portion, A_16384 Horner steps, the last line's bytes
    kept below kb, every byte offset within the line; PECH_FLAT_IL=0 keeps the
    static slices.  Every CRC against the oracle, seeds included."""
    import pech_amd as P

    monkeypatch.setenv("PECH_FLAT_IL", il)  # (read at each zero-copy flat launch)
    rng = np.random.default_rng(k * 1000 + size % 997 + off)
    order = max(0, int(np.ceil(np.log2((size + off) / 4096))))
    pages = [P.Pages(order) for _ in range(k)]
    ac = P.AsyncCrc()
    got, want = {}, {}
    try:
        for i, pg in enumerate(pages):
            pg.view[off:off + size] = rng.integers(0, 256, size, dtype=np.uint8)
            seed = int(rng.integers(0, 1 << 32)) if i % 3 == 1 else 0
            want[i] = O.crc(seed, pg.view[off:off + size])
            ac.submit(pg.ptr + off, size, seed, lambda crc, err, i=i: got.__setitem__(i, (crc, err)))
        ac.flush()
        _wait_all(ac)
        assert got == {i: (want[i], 0) for i in range(k)}
    finally:
        ac.close()
        for pg in pages:
            pg.free()
