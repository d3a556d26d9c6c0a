"""Pin the oracle (oracle/crc32c_oracle.c) before trusting it: against the
reference's own table and golden vectors generated from the compiled
reference header (tests/golden/kat.json), and against
the compiled reference itself when oracle/_ref is present.  CPU only."""
import json
import os

import numpy as np
import pytest

import oracle_lib as O
from gen import splitmix_bytes, xorshift_bytes

KAT = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "kat.json")))


def test_table_regenerates_reference_table():
    # include/crc32c.h:16-81 regenerated from 0x82F63B78
    t = np.zeros(256, dtype=np.uint32)
    O.oracle().oracle_table_copy(t.ctypes.data)
    assert [int(x) for x in t] == KAT["table"]
    assert KAT["table"][1] == 0xF26B8303 and KAT["table"][128] == 0x82F63B78


def test_appendix_a_known_answers():
    for row in KAT["appendix_a"]:
        if row["len"] > 65536:
            continue  # covered by test_appendix_a_large
        d = xorshift_bytes(row["len"])
        for s, want in row["crc"].items():
            assert O.crc(int(s, 16), d) == want, (row["len"], s)


@pytest.mark.slow
def test_appendix_a_large():
    for row in KAT["appendix_a"]:
        if row["len"] <= 65536:
            continue
        d = xorshift_bytes(row["len"])
        for s, want in row["crc"].items():
            assert O.crc(int(s, 16), d) == want, (row["len"], s)


def test_offset_length_seed_vectors():
    stream = np.frombuffer(splitmix_bytes(0xC0FFEE, 3 * 65536 + 4096), dtype=np.uint8)
    v = KAT["vectors"]
    got = O.crcs(stream, [x["off"] for x in v], [x["len"] for x in v], [x["seed"] for x in v])
    want = np.array([x["crc"] for x in v], dtype=np.uint32)
    assert np.array_equal(got, want)


def test_checks():
    c = KAT["checks"]
    assert O.crc(0, b"123456789") == c["123456789_seed0"] == 0x58E3FA20
    assert (~O.crc(0xFFFFFFFF, b"123456789")) & 0xFFFFFFFF == c["123456789_std"] == 0xE3069283
    assert O.crc(0, bytes(4096)) == c["zeros4096_seed0"] == 0
    assert O.crc(0, b"\xff" * 4096) == c["ff4096_seed0"]
    assert O.crc(0xFFFFFFFF, bytes(4096)) == c["zeros4096_seedffffffff"]


def test_oracle_matches_compiled_reference_random():
    R = O.ref()
    if R is None:
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    rng = np.random.default_rng(7)
    data = rng.integers(0, 256, 1 << 18, dtype=np.uint8)
    for _ in range(300):
        off = int(rng.integers(0, 1000))
        n = int(rng.integers(0, 5000))
        s = int(rng.integers(0, 1 << 32))
        p = data.ctypes.data + off
        assert O.oracle().oracle_crc32c(s, p, n) == R.ref_crc32c(s, p, n)
    t = np.zeros(256, dtype=np.uint32)
    R.ref_table_copy(t.ctypes.data)
    assert [int(x) for x in t] == KAT["table"]


def test_chaining_matches_page_piece_walk():
    # ceph_crc32c_iov (messenger.c:1734) chains <=4 KiB pieces through the seed
    rng = np.random.default_rng(3)
    d = rng.integers(0, 256, 3 * 4096 + 123, dtype=np.uint8)
    for s in (0, 0xFFFFFFFF, 0x1234567):
        whole = O.crc(s, d)
        for piece in (1, 7, 4096, 1 << 20):
            assert O.oracle().oracle_crc32c_pieces(s, d.ctypes.data, d.nbytes, piece) == whole


def test_algebra_shift_combine():
    o = O.oracle()
    rng = np.random.default_rng(11)
    a = rng.integers(0, 256, 777, dtype=np.uint8)
    b = rng.integers(0, 256, 1234, dtype=np.uint8)
    for s in (0, 0xDEADBEEF):
        ab = O.crc(s, np.concatenate([a, b]))
        assert o.oracle_combine(O.crc(s, a), O.crc(0, b), b.nbytes) == ab
        # shift == zero bytes
        assert o.oracle_shift(s, 100) == O.crc(s, bytes(100))
        # seed-in-data identity: R(s, D) == R(0, D ^ s) for |D| >= 4
        d = a.copy()
        d[:4] ^= np.frombuffer(np.uint32(s).tobytes(), dtype=np.uint8)
        assert O.crc(0, d) == O.crc(s, a)


def test_sse42_context_baseline_matches_oracle():
    """bench.py's SSE4.2 CPU row (oracle/crc32c_hw.c) is bit-exact with the
    reference loop: golden vectors, then random lengths around its 3-stream
    threshold at every alignment, random seeds, and the threaded batch."""
    H = O.hw()
    if H is None:
        pytest.skip("no SSE4.2 on this host")
    for row in KAT["appendix_a"]:
        if row["len"] > 65536:
            continue
        d = np.frombuffer(bytes(xorshift_bytes(row["len"])), dtype=np.uint8).copy()
        for s, want in row["crc"].items():
            assert H.hw_crc32c(int(s, 16), d.ctypes.data, d.nbytes) == want, (row["len"], s)
    rng = np.random.default_rng(7)
    buf = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    for _ in range(400):
        n = int(rng.choice([rng.integers(0, 64), rng.integers(1000, 1100), rng.integers(0, 200000)]))
        off = int(rng.integers(0, 16))
        seed = int(rng.integers(0, 1 << 32))
        assert H.hw_crc32c(seed, buf.ctypes.data + off, n) == O.crc(seed, buf[off:off + n]), (n, off)
    lens = rng.integers(0, 70000, 300).astype(np.uint32)
    offs = np.cumsum(np.concatenate([[3], lens[:-1].astype(np.uint64) + 5])).astype(np.uint64)
    big = rng.integers(0, 256, int(offs[-1] + lens[-1] + 8), dtype=np.uint8)
    out = np.zeros(len(lens), dtype=np.uint32)
    assert H.hw_crc32c_batch_mt(big.ctypes.data, offs.ctypes.data, lens.ctypes.data, out.ctypes.data, len(lens), 4,
                                2) == 0
    assert np.array_equal(out, O.crcs(big, offs, lens))
