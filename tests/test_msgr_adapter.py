"""The messenger adapter's queue logic (include/pech_crc32c_msgr.h,
pech_amd/csrc/crc32c_msgr.c) on its host-only paths, in the build container:
unchecked messages, skip markers and payloads at or below the host cutoff
never reach the async layer, so the connection is created over a stand-in
context pointer that is never dereferenced.  The GPU paths of the same queue
are tests/c/msgr_conn_sim.c and tests/c/msgr_loopback.c (-m gpu).

Seq semantics follow the reference's read_partial_message / process_message
(/root/reference/src/ceph/messenger.c:2737-2770, :2858-2883): every message,
skipped or not, takes one place in arrival order; in_seq moves by one per
place returned by rx_next."""
import ctypes

import numpy as np
import pytest

import oracle_lib as O
from pech_amd import _lib

EAGAIN, EBADMSG = 11, 74
FAKE_CTX = ctypes.c_void_p(0x1000)  # never dereferenced on these paths
REL = ctypes.CFUNCTYPE(None, ctypes.c_void_p)


@pytest.fixture
def conn(request):
    L = _lib.lib()
    max_pending = getattr(request, "param", 4)
    prev = L.crc32c_msgr_set_host_max(1 << 20)  # every checked payload here is host-routed
    released = []
    rel = REL(lambda m: released.append(m))
    c = L.crc32c_msgr_conn_create(FAKE_CTX, max_pending, None, None, ctypes.cast(rel, ctypes.c_void_p))
    assert c
    yield L, c, released
    L.crc32c_msgr_conn_destroy(c)
    L.crc32c_msgr_set_host_max(prev)
    del rel


def nxt(L, c):
    m, crc = ctypes.c_void_p(), ctypes.c_uint32()
    rc = L.crc32c_msgr_rx_next(c, ctypes.byref(m), ctypes.byref(crc))
    return rc, m.value, crc.value


@pytest.mark.parametrize("conn", [2048], indirect=True)
def test_markers_coalesce_and_keep_arrival_order(conn):
    L, c, released = conn
    rng = np.random.default_rng(3)
    d = rng.integers(0, 256, 5000, dtype=np.uint8)
    good = O.crc(0, d)
    assert L.crc32c_msgr_rx_queue(c, ctypes.c_void_p(0x11), None, 0, 0, 0) == 0
    for _ in range(1000):  # skipped messages: one shared entry, 1000 places
        assert L.crc32c_msgr_rx_queue(c, None, None, 0, 0, 0) == 0
    assert L.crc32c_msgr_rx_queue(c, ctypes.c_void_p(0x22), d.ctypes.data, d.size, 1, good) == 0
    assert L.crc32c_msgr_rx_queue(c, None, None, 0, 0, 0) == 0
    assert L.crc32c_msgr_rx_queue(c, ctypes.c_void_p(0x33), d.ctypes.data, d.size, 1, good ^ 1) == 0
    assert L.crc32c_msgr_rx_pending(c) == 1004
    assert nxt(L, c) == (1, 0x11, 0)
    for k in range(1000):
        assert nxt(L, c) == (1, None, 0), k
        assert L.crc32c_msgr_rx_pending(c) == 1002 - k
    assert nxt(L, c) == (1, 0x22, good)
    assert nxt(L, c) == (1, None, 0)
    assert nxt(L, c) == (-EBADMSG, 0x33, good)
    assert nxt(L, c)[0] == 0 and L.crc32c_msgr_rx_pending(c) == 0
    assert released == []  # messages returned by rx_next are the messenger's


def test_queue_full_refuses_messages_not_markers(conn):
    L, c, released = conn
    for k in range(4):  # max_pending = 4
        assert L.crc32c_msgr_rx_queue(c, ctypes.c_void_p(0x100 + k), None, 0, 0, 0) == 0
    assert L.crc32c_msgr_rx_queue(c, ctypes.c_void_p(0x200), None, 0, 0, 0) == -EAGAIN
    for _ in range(50):
        assert L.crc32c_msgr_rx_queue(c, None, None, 0, 0, 0) == 0
    assert L.crc32c_msgr_rx_pending(c) == 54
    assert nxt(L, c) == (1, 0x100, 0)
    assert L.crc32c_msgr_rx_queue(c, ctypes.c_void_p(0x200), None, 0, 0, 0) == -EAGAIN  # still 53 pending
    L.crc32c_msgr_conn_reset(c)  # con_fault: queued messages released, markers dropped
    assert sorted(released) == [0x101, 0x102, 0x103]
    assert L.crc32c_msgr_rx_pending(c) == 0
    assert L.crc32c_msgr_rx_queue(c, ctypes.c_void_p(0x200), None, 0, 0, 0) == 0


def test_marker_after_message_is_a_new_entry(conn):
    # a marker never merges into a message entry, and a marker queued after
    # the shared one was partly consumed extends it
    L, c, _ = conn
    assert L.crc32c_msgr_rx_queue(c, None, None, 0, 0, 0) == 0
    assert L.crc32c_msgr_rx_queue(c, None, None, 0, 0, 0) == 0
    assert nxt(L, c) == (1, None, 0)
    assert L.crc32c_msgr_rx_queue(c, None, None, 0, 0, 0) == 0
    assert L.crc32c_msgr_rx_queue(c, ctypes.c_void_p(0x44), None, 0, 0, 0) == 0
    assert L.crc32c_msgr_rx_queue(c, None, None, 0, 0, 0) == 0
    assert [nxt(L, c) for _ in range(5)] == [(1, None, 0), (1, None, 0), (1, 0x44, 0), (1, None, 0), (0, None, 0)]


def test_host_routed_send_footer(conn):
    L, c, released = conn
    d = np.random.default_rng(4).integers(0, 256, 3000, dtype=np.uint8)
    assert L.crc32c_msgr_tx_submit(c, ctypes.c_void_p(0x55), d.ctypes.data, d.size, 7) == 0
    assert L.crc32c_msgr_tx_has(c, ctypes.c_void_p(0x55)) == 1
    assert L.crc32c_msgr_tx_submit(c, ctypes.c_void_p(0x55), d.ctypes.data, d.size, 7) == 1  # resend
    crc = ctypes.c_uint32()
    assert L.crc32c_msgr_tx_footer(c, ctypes.c_void_p(0x55), ctypes.byref(crc)) == 1
    assert crc.value == O.crc(7, d)
    assert L.crc32c_msgr_tx_has(c, ctypes.c_void_p(0x55)) == 0
    assert L.crc32c_msgr_tx_submit(c, ctypes.c_void_p(0x66), d.ctypes.data, d.size, 0) == 0
    assert L.crc32c_msgr_tx_cancel(c, None) == 1 and released == [0x66]  # revoke: the adapter's reference
