"""GPU parity: the gfx950 kernel (through the C-ABI) against the oracle and
the golden vectors, bit-exact.  Run on an MI355X: pytest -m gpu."""
import ctypes
import json
import os

import numpy as np
import pytest

import oracle_lib as O
from gen import splitmix_bytes, xorshift_bytes

pytestmark = pytest.mark.gpu

KAT = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "kat.json")))


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    return torch, torch.device("cuda:0")


@pytest.fixture(scope="module")
def P():
    import pech_amd

    return pech_amd


@pytest.fixture
def gpu_route(P):
    """Route every non-empty drop-in crc32c() call to the GPU for the test and
    check afterwards that the kernels computed them (no host fallback)."""
    prev = P.set_cpu_max(0)
    before = P.stats()
    yield
    P.set_cpu_max(prev)
    after = P.stats()
    assert after["gpu_fallbacks"] == before["gpu_fallbacks"], after
    assert after["gpu_calls"] > before["gpu_calls"], after
    assert after["cpu_calls"] == before["cpu_calls"], after


def dev_crcs(torch, P, dbuf, offs, lens, seeds=None):
    """kernel CRCs of dbuf[off:off+len] (dbuf: device uint8 tensor)."""
    base = dbuf.data_ptr()
    addrs = [base + int(o) for o in offs]
    descs = P.make_descs(addrs, lens, seeds, device=dbuf.device)
    out = torch.full((len(lens),), 0x5A5A5A5A, dtype=torch.int32, device=dbuf.device)
    P.dev_batch_async(descs, out)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


def to_dev(torch, host_u8, dev):
    return torch.from_numpy(np.ascontiguousarray(host_u8)).to(dev)


def test_perm_lane_layout_known_answer(torch_dev, P):
    torch, dev = torch_dev
    d = b"123456789"
    buf = to_dev(torch, np.frombuffer(d, dtype=np.uint8), dev)
    got = dev_crcs(torch, P, buf, [0], [9], [0])
    assert got[0] == 0x58E3FA20
    got = dev_crcs(torch, P, buf, [0], [9], [0xFFFFFFFF])
    assert (~int(got[0])) & 0xFFFFFFFF == 0xE3069283


def test_appendix_a_device(torch_dev, P):
    torch, dev = torch_dev
    for row in KAT["appendix_a"]:
        n = row["len"]
        d = np.frombuffer(xorshift_bytes(n), dtype=np.uint8) if n else np.zeros(1, np.uint8)
        buf = to_dev(torch, d, dev)
        seeds = [int(s, 16) for s in row["crc"]]
        got = dev_crcs(torch, P, buf, [0] * 3, [n] * 3, seeds)
        assert [int(x) for x in got] == [row["crc"][f"{s:08x}"] for s in seeds], n


def test_golden_vectors_unaligned_device(torch_dev, P):
    torch, dev = torch_dev
    stream = np.frombuffer(splitmix_bytes(0xC0FFEE, 3 * 65536 + 4096), dtype=np.uint8)
    buf = to_dev(torch, stream, dev)
    v = KAT["vectors"]
    got = dev_crcs(torch, P, buf, [x["off"] for x in v], [x["len"] for x in v], [x["seed"] for x in v])
    want = np.array([x["crc"] for x in v], dtype=np.uint32)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(v[i], hex(got[i])) for i in bad[:10]]


def test_each_vector_alone(torch_dev, P):
    # single-buffer launches (one group, whole-buffer store path)
    torch, dev = torch_dev
    stream = np.frombuffer(splitmix_bytes(0xC0FFEE, 3 * 65536 + 4096), dtype=np.uint8)
    buf = to_dev(torch, stream, dev)
    for x in KAT["vectors"][::7]:
        got = dev_crcs(torch, P, buf, [x["off"]], [x["len"]], [x["seed"]])
        assert int(got[0]) == x["crc"], x


def test_random_mixed_batch(torch_dev, P):
    torch, dev = torch_dev
    rng = np.random.default_rng(1234)
    n = 4000
    lens = rng.integers(0, 20000, n)
    lens[rng.random(n) < 0.1] = 0
    tiny = rng.random(n) < 0.1
    lens[tiny] = rng.integers(0, 40, int(tiny.sum()))
    offs = np.zeros(n, dtype=np.int64)
    pos = 0
    for i in range(n):
        pos += int(rng.integers(0, 64))
        offs[i] = pos
        pos += int(lens[i])
    host = rng.integers(0, 256, pos + 64, dtype=np.uint8)
    seeds = rng.integers(0, 1 << 32, n, dtype=np.uint64)
    seeds[rng.random(n) < 0.5] = 0
    got = dev_crcs(torch, P, to_dev(torch, host, dev), offs, lens, seeds)
    want = O.crcs(host, offs, lens, seeds)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(offs[i]), int(lens[i]), int(seeds[i]), hex(got[i]), hex(want[i])) for i in bad[:10]]


def test_overlapping_and_repeated_buffers(torch_dev, P):
    # descriptors may alias the same bytes; buffers are read only
    torch, dev = torch_dev
    rng = np.random.default_rng(99)
    host = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    offs = rng.integers(0, 1 << 19, 500)
    lens = rng.integers(1, 1 << 19, 500)
    got = dev_crcs(torch, P, to_dev(torch, host, dev), offs, lens)
    assert np.array_equal(got, O.crcs(host, offs, lens))


def test_c2_shape_full_parity(torch_dev, P):
    # BASELINE config 2: 65,536 x 4 KiB device-resident buffers, every output checked
    torch, dev = torch_dev
    n, L = 65536, 4096
    g = torch.Generator(device=dev)
    g.manual_seed(2)
    buf = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev, generator=g)
    offs = np.arange(n, dtype=np.int64) * L
    got = dev_crcs(torch, P, buf, offs, [L] * n)
    host = buf.cpu().numpy()
    assert np.array_equal(got, O.crcs(host, offs, [L] * n))


def test_c3_shape_parity(torch_dev, P):
    # BASELINE config 3 shape: 4 MiB buffers (64 of them = 256 MiB), every output checked
    torch, dev = torch_dev
    n, L = 64, 4 << 20
    buf = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev)
    offs = np.arange(n, dtype=np.int64) * L
    got = dev_crcs(torch, P, buf, offs, [L] * n)
    host = buf.cpu().numpy()
    assert np.array_equal(got, O.crcs(host, offs, [L] * n))


@pytest.mark.parametrize("config", ["c3", "c4", "c2-odd"])
def test_full_size_batch_parity(torch_dev, P, config):
    """BASELINE configs at their full per-GPU size, every output checked
    against the oracle: C3 = 256 x 4 MiB (1 GiB, the bench's batch), C4 =
    65,536 x 4 KiB + 4,096 x 64 KiB + 256 x 1 MiB + 64 x 4 MiB shuffled with
    seed 42 (1 GiB, bench.py's c4_sizes), and bench.py's unaligned c2-odd
    (65,536 x 4,100 B back to back), random seeds."""
    torch, dev = torch_dev
    if config == "c3":
        sizes = [4 << 20] * 256
    elif config == "c2-odd":
        sizes = [4100] * 65536
    else:
        sizes = [4096] * 65536 + [65536] * 4096 + [1 << 20] * 256 + [4 << 20] * 64
        np.random.default_rng(42).shuffle(sizes)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    total = int(np.sum(sizes))
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    buf = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=g)
    seeds = [int(x) for x in np.random.default_rng(8).integers(0, 1 << 32, len(sizes))]
    got = dev_crcs(torch, P, buf, offs, sizes, seeds)
    host = buf.cpu().numpy()
    del buf
    want = O.crcs(host, offs, sizes, seeds)
    assert np.array_equal(got, want), int(np.sum(got != want))


def test_c4_mixed_sizes_parity(torch_dev, P):
    # config 4 mix (4 KiB / 64 KiB / 1 MiB / 4 MiB), shuffled, scaled to 128 MiB
    torch, dev = torch_dev
    rng = np.random.default_rng(42)
    sizes = [4096] * 8192 + [65536] * 512 + [1 << 20] * 32 + [4 << 20] * 8
    rng.shuffle(sizes)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    total = int(np.sum(sizes))
    buf = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev)
    got = dev_crcs(torch, P, buf, offs, sizes)
    assert np.array_equal(got, O.crcs(buf.cpu().numpy(), offs, sizes))


@pytest.mark.parametrize("case", ["uniform-odd-n", "uniform-unaligned", "uniform-with-holes", "empty-first-chunk",
                                  "many-chunks", "fewer-buffers-than-waves"])
def test_prologue_start_search(torch_dev, P, case):
    """The main kernel's prologue speculates each wave's start position and
    checks it exactly (uniform batches start there; others fall back to the
    row-offset scan).  Batches around that check: uniform sizes at batch
    sizes that are no multiple of a chunk, unaligned buffers (virtual
    leading pieces), uniform batches with tiny/empty buffers sprinkled in
    (compacted positions shift the guess), a first chunk with no core rows at
    all, more than 16 chunks (the chunk scan spans lanes), and fewer
    buffers than waves."""
    torch, dev = torch_dev
    rng = np.random.default_rng(sum(map(ord, case)))
    gap = 0
    if case == "uniform-odd-n":
        sizes = [12288] * 5001
    elif case == "uniform-unaligned":
        sizes, gap = [4096 + 7] * 3001, 9
    elif case == "uniform-with-holes":
        sizes = [8192] * 6000
        for i in rng.choice(6000, 300, replace=False):
            sizes[i] = int(rng.integers(0, 31))
    elif case == "empty-first-chunk":
        sizes = [int(x) for x in rng.integers(0, 16, 1024)] + [65536] * 1500
    elif case == "many-chunks":
        sizes = [2048] * 40000 + [int(x) for x in rng.integers(0, 100000, 500)]
    else:
        sizes = [1 << 20] * 37 + [333333] * 5
    n = len(sizes)
    offs = np.zeros(n, dtype=np.int64)
    pos = 3
    for i, L in enumerate(sizes):
        offs[i] = pos
        pos += L + gap
    buf = torch.randint(0, 256, (pos + 64,), dtype=torch.uint8, device=dev)
    seeds = [int(x) for x in rng.integers(0, 1 << 32, n)] if case in ("uniform-odd-n", "many-chunks") else None
    got = dev_crcs(torch, P, buf, offs, sizes, seeds)
    host = buf.cpu().numpy()
    want = O.crcs(host, offs, sizes, seeds)
    assert np.array_equal(got, want), int(np.sum(got != want))


def test_single_huge_buffer_split_over_all_groups(torch_dev, P):
    torch, dev = torch_dev
    L = (96 << 20) + 12345
    buf = torch.randint(0, 256, (L + 16,), dtype=torch.uint8, device=dev)
    host = buf.cpu().numpy()
    for off, seed in ((0, 0), (3, 0xFFFFFFFF), (11, 0x12345678)):
        got = dev_crcs(torch, P, buf, [off], [L], [seed])
        assert int(got[0]) == O.crc(seed, host[off:off + L])


def test_near_4gib_buffer(torch_dev, P):
    """One buffer of 2^32 - 100 bytes, unaligned: its split runs end up to 2^25
    rows before the buffer's end, past the row-power table's 2^18 rows (the
    digits above it, v0.25) and at the rows-after bit 25.  The
    check is the SSE4.2 oracle (cross-checked against the compiled reference in
    test_oracle.py), or the byte loop without SSE4.2."""
    torch, dev = torch_dev
    L = (1 << 32) - 100
    blk = torch.randint(0, 256, (64 << 20,), dtype=torch.uint8, device=dev)
    buf = torch.empty(64 * (64 << 20) + 64, dtype=torch.uint8, device=dev)
    body = buf[:64 * (64 << 20)].view(64, -1)
    body.copy_(blk.expand(64, -1))
    body += torch.arange(64, dtype=torch.uint8, device=dev).view(64, 1)  # (uint8 wraps)
    buf[64 * (64 << 20):] = 7
    host = buf.cpu().numpy()
    H = O.hw()
    ref = (lambda s, a: H.hw_crc32c(s, a.ctypes.data, a.nbytes)) if H else O.crc
    for off, seed in ((3, 0x9E3779B9), (0, 0)):
        got = dev_crcs(torch, P, buf, [off], [L], [seed])
        assert int(got[0]) == ref(seed, host[off:off + L]), (off, seed)


def test_sensitivity_constant_data(torch_dev, P):
    torch, dev = torch_dev
    for val in (0x00, 0xFF):
        buf = torch.full((64 * 4096,), val, dtype=torch.uint8, device=dev)
        got = dev_crcs(torch, P, buf, np.arange(64) * 4096, [4096] * 64)
        want = KAT["checks"]["zeros4096_seed0" if val == 0 else "ff4096_seed0"]
        assert all(int(x) == want for x in got)


def test_chaining_and_linearity_at_full_size(torch_dev, P):
    # size-independent properties on a 1 GiB buffer (no oracle needed):
    #   crc(s, A||B) == combine(crc(s, A), crc(0, B), |B|)
    #   crc(0, X ^ Y) == crc(0, X) ^ crc(0, Y)          (equal lengths)
    torch, dev = torch_dev
    L = 1 << 30
    x = torch.randint(0, 256, (L,), dtype=torch.uint8, device=dev)
    y = torch.randint(0, 256, (L,), dtype=torch.uint8, device=dev)
    cut = 123456789
    whole, a, b = dev_crcs(torch, P, x, [0, 0, cut], [L, cut, L - cut], [7, 7, 0])
    assert P.crc32c_combine(int(a), int(b), L - cut) == int(whole)
    xy = torch.bitwise_xor(x, y)
    cx, cy, cxy = (int(dev_crcs(torch, P, t, [0], [L])[0]) for t in (x, y, xy))
    assert cx ^ cy == cxy


def test_empty_and_tiny(torch_dev, P):
    torch, dev = torch_dev
    host = np.arange(256, dtype=np.uint8)
    buf = to_dev(torch, host, dev)
    offs, lens, seeds = [], [], []
    for off in range(0, 20):
        for n in range(0, 6):
            for s in (0, 0xA5A5A5A5):
                offs.append(off)
                lens.append(n)
                seeds.append(s)
    got = dev_crcs(torch, P, buf, offs, lens, seeds)
    assert np.array_equal(got, O.crcs(host, offs, lens, seeds))
    # all-empty batch: every output is its seed
    got = dev_crcs(torch, P, buf, [0] * 10, [0] * 10, list(range(10)))
    assert [int(x) for x in got] == list(range(10))


def test_more_than_one_launch_of_buffers(torch_dev, P):
    # > 2^20 descriptors: the library splits into several plan/main launches
    torch, dev = torch_dev
    n = (1 << 20) + 777
    host = np.random.default_rng(5).integers(0, 256, n + 64, dtype=np.uint8)
    offs = np.arange(n, dtype=np.int64)
    lens = (np.arange(n) % 33).astype(np.int64)
    got = dev_crcs(torch, P, to_dev(torch, host, dev), offs, lens)
    assert np.array_equal(got, O.crcs(host, offs, lens))


def test_dropin_crc32c_host_memory(P, gpu_route):
    rng = np.random.default_rng(8)
    for n in (1, 3, 4, 49, 4096, 100000):
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        for s in (0, 0xFFFFFFFF):
            assert P.crc32c(s, d) == O.crc(s, d)
    assert P.crc32c(0x1234, b"") == 0x1234


def test_dropin_small_path_boundaries(P, gpu_route):
    # On the GPU route, crc32c() up to PECH_SMALL_MAX (64 KiB) is one
    # zero-copy launch; above it the staged batch path.  Sizes around both paths' edges, unaligned
    # sources, random seeds
    rng = np.random.default_rng(18)
    big = rng.integers(0, 256, (1 << 17) + 64, dtype=np.uint8)
    for n in (1, 2, 15, 16, 17, 63, 64, 65, 1023, 1024, 1025, 4097, 65535, 65536, 65537, 70001):
        for off in (0, 1, 13):
            d = big[off:off + n].tobytes()
            s = int(rng.integers(0, 1 << 32))
            assert P.crc32c(s, d) == O.crc(s, d), (n, off)


def test_dropin_crc32c_larger_than_staging(P, gpu_route):
    # > 64 MiB staging slot: chained through the seed inside the library
    d = np.random.default_rng(9).integers(0, 256, (64 << 20) + 4097, dtype=np.uint8)
    assert P.crc32c(0xFFFFFFFF, d) == O.crc(0xFFFFFFFF, d)


def test_batch_host_pinned_device_flags(torch_dev, P):
    torch, dev = torch_dev
    from pech_amd import _lib

    rng = np.random.default_rng(10)
    lens = [int(x) for x in rng.integers(0, 300000, 64)] + [0, 1, 2, 70000]
    bufs = [rng.integers(0, 256, n, dtype=np.uint8) for n in lens]
    seeds = [int(x) for x in rng.integers(0, 1 << 32, len(lens))]
    want = [O.crc(s, b) for s, b in zip(seeds, bufs)]
    assert P.crc32c_batch([b.tobytes() for b in bufs], seeds) == want
    L = _lib.lib()
    n = len(lens)
    # pinned host memory: DMA'd in place
    pinned = [torch.from_numpy(b).pin_memory() if b.size else torch.zeros(1, dtype=torch.uint8).pin_memory()
              for b in bufs]
    ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() for t in pinned])
    cl = (ctypes.c_uint * n)(*lens)
    cs = (ctypes.c_uint32 * n)(*seeds)
    out = (ctypes.c_uint32 * n)()
    assert L.crc32c_batch(ptrs, cl, cs, out, n, 2) == 0
    assert list(out) == want
    # device memory through the synchronous batch call
    dts = [t.to(dev) for t in pinned]
    ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() for t in dts])
    out = (ctypes.c_uint32 * n)()
    assert L.crc32c_batch(ptrs, cl, cs, out, n, 1) == 0
    assert list(out) == want
    # invalid flags
    assert L.crc32c_batch(ptrs, cl, cs, out, n, 3) < 0


@pytest.mark.parametrize("devices", [None, "0,0", ",".join(["0"] * 8)])
def test_batch_pinned_all_devices(torch_dev, P, monkeypatch, devices):
    # CRC32C_F_PINNED | CRC32C_F_ALL_DEVICES: byte-balanced shards, one per GPU,
    # all issued before any wait.  "0,0" = two shards on GPU 0 (both slots,
    # one stream): the split/gather path on a 1-GPU box.  Sub-batches of
    # 65,536 descriptors: n > that takes several rounds per shard.
    torch, dev = torch_dev
    from pech_amd import _lib

    if devices:
        monkeypatch.setenv("PECH_DEVICES", devices)
    rng = np.random.default_rng(12)
    lens = np.concatenate([rng.integers(0, 5000, 140000), rng.integers(1 << 20, 3 << 20, 12), [0, 7, 4096]])
    rng.shuffle(lens)
    host = torch.empty(int(lens.sum()) + 64, dtype=torch.uint8).pin_memory()
    data = rng.integers(0, 256, host.numel(), dtype=np.uint8)
    host.copy_(torch.from_numpy(data))
    offs = np.concatenate([[3], 3 + np.cumsum(lens)[:-1]])
    seeds = rng.integers(0, 1 << 32, len(lens), dtype=np.uint64)
    n = len(lens)
    ptrs = (ctypes.c_void_p * n)(*[host.data_ptr() + int(o) for o in offs])
    cl = (ctypes.c_uint * n)(*[int(x) for x in lens])
    cs = (ctypes.c_uint32 * n)(*[int(x) for x in seeds])
    out = (ctypes.c_uint32 * n)()
    L = _lib.lib()
    assert L.crc32c_batch(ptrs, cl, cs, out, n, P.F_PINNED | P.F_ALL_DEVICES) == 0, L.crc32c_last_error()
    assert np.array_equal(np.frombuffer(out, dtype=np.uint32), O.crcs(data, offs, lens, seeds))
    # pageable memory has no device mapping: refused before anything launches
    page = np.zeros(1 << 16, np.uint8)
    p1 = (ctypes.c_void_p * 1)(page.ctypes.data)
    l1 = (ctypes.c_uint * 1)(1000)
    assert L.crc32c_batch(p1, l1, None, out, 1, P.F_PINNED | P.F_ALL_DEVICES) == -22


@pytest.mark.parametrize("devices", ["0,0", "0,0,0", ",".join(["0"] * 8), ",".join(["0"] * 17)])
def test_batch_pinned_all_devices_splits_huge_buffer(torch_dev, P, monkeypatch, devices):
    """A buffer larger than one device's share (>= 16 MiB) is cut into
    per-device segments whose CRCs combine on the host (SURVEY 8e's optional
    split).  G shards on one GPU rehearse G GPUs (G = 8, the
    100 MiB buffer cut into 8 page-aligned segments); they share the device's
    descriptor slots, so more than 16 on one device are refused."""
    torch, dev = torch_dev
    from pech_amd import _lib

    monkeypatch.setenv("PECH_DEVICES", devices)
    rng = np.random.default_rng(31)
    lens = np.array([(100 << 20) + 12345, 5000, 0, 17, (20 << 20) + 3, 4096], dtype=np.int64)
    host = torch.empty(int(lens.sum()) + 64, dtype=torch.uint8).pin_memory()
    data = rng.integers(0, 256, host.numel(), dtype=np.uint8)
    host.copy_(torch.from_numpy(data))
    offs = np.concatenate([[5], 5 + np.cumsum(lens)[:-1]])
    seeds = rng.integers(0, 1 << 32, len(lens), dtype=np.uint64)
    n = len(lens)
    ptrs = (ctypes.c_void_p * n)(*[host.data_ptr() + int(o) for o in offs])
    cl = (ctypes.c_uint * n)(*[int(x) for x in lens])
    cs = (ctypes.c_uint32 * n)(*[int(x) for x in seeds])
    out = (ctypes.c_uint32 * n)()
    L = _lib.lib()
    rc = L.crc32c_batch(ptrs, cl, cs, out, n, P.F_PINNED | P.F_ALL_DEVICES)
    if devices.count(",") + 1 > 16:
        assert rc == -22
        return
    assert rc == 0, L.crc32c_last_error()
    assert np.array_equal(np.frombuffer(out, dtype=np.uint32), O.crcs(data, offs, lens, seeds))


def test_batch_device_aliasing_beyond_launch_limit(torch_dev, P):
    # 60,000 descriptors over ONE 5 MiB device buffer: 293 GiB of payload,
    # past the 256 GiB per-launch cap (rows are counted in 32 bits), so
    # crc32c_batch splits it into two launches
    torch, dev = torch_dev
    from pech_amd import _lib

    rng = np.random.default_rng(14)
    L5 = 5 << 20
    host = rng.integers(0, 256, L5, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    n = 60000
    ptrs = (ctypes.c_void_p * n)(*([d.data_ptr()] * n))
    lens = (ctypes.c_uint * n)(*([L5] * n))
    out = (ctypes.c_uint32 * n)()
    L = _lib.lib()
    assert L.crc32c_batch(ptrs, lens, None, out, n, P.F_DEVICE) == 0, L.crc32c_last_error()
    got = np.frombuffer(out, dtype=np.uint32)
    assert np.all(got == O.crc(0, host))


def test_concurrent_streams_explicit_workspaces(torch_dev, P):
    # bench.py's pipelined pass: independent batches alternate over streams,
    # one workspace per stream, launches overlapping on the device
    torch, dev = torch_dev
    shapes = [([4096] * 8192, 0), ([4 << 20] * 16, 1), ([65536] * 512, 0xFFFFFFFF), ([1 << 20] * 32, 5)]
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    wss = [torch.empty(P.workspace_bytes(8192), dtype=torch.uint8, device=dev) for _ in range(2)]
    jobs = []
    for sizes, seed in shapes:
        offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
        buf = torch.randint(0, 256, (int(np.sum(sizes)),), dtype=torch.uint8, device=dev)
        descs = P.make_descs(buf.data_ptr() + offs, sizes, [seed] * len(sizes), device=dev)
        out = torch.zeros(len(sizes), dtype=torch.int32, device=dev)
        jobs.append((buf, offs, sizes, seed, descs, out))
    torch.cuda.synchronize()
    for rep in range(3):
        for i, (_, _, _, _, descs, out) in enumerate(jobs):
            P.dev_batch_ws_async(descs, out, wss[i % 2], stream=streams[i % 2])
    torch.cuda.synchronize()
    for buf, offs, sizes, seed, _, out in jobs:
        want = O.crcs(buf.cpu().numpy(), offs, sizes, [seed] * len(sizes))
        assert np.array_equal(out.cpu().numpy().view(np.uint32), want)


def test_graph_capture_and_replay(torch_dev, P):
    # the device batch enqueues no host sync / allocation: capturable with
    # its own workspace; the internal workspace is refused inside a capture
    # (a replay would use it outside the library's stream ordering)
    torch, dev = torch_dev
    n, L = 256, 65536
    buf = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev)
    offs = np.arange(n) * L
    descs = P.make_descs([buf.data_ptr() + int(o) for o in offs], [L] * n, device=dev)
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    ws = torch.empty(P.workspace_bytes(n), dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        P.dev_batch_ws_async(descs, out, ws, stream=s)  # warm-up outside capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        with pytest.raises(P.Crc32cError, match="graph"):
            P.dev_batch_async(descs, out, stream=s)
        P.dev_batch_ws_async(descs, out, ws, stream=s)
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), O.crcs(buf.cpu().numpy(), offs, [L] * n))


def test_dropin_default_route(P):
    # default routing: headers / front sections / <=4 KiB pieces (and every
    # call up to 4 MiB) on the host routine, larger calls on the GPU
    rng = np.random.default_rng(31)
    before = P.stats()
    for n in (49, 4096, 65536, 4 << 20):
        d = rng.integers(0, 256, n, dtype=np.uint8)
        assert P.crc32c(5, d) == O.crc(5, d)
    mid = P.stats()
    assert mid["cpu_calls"] - before["cpu_calls"] == 4 and mid["gpu_calls"] == before["gpu_calls"]
    d = rng.integers(0, 256, (4 << 20) + 1, dtype=np.uint8)
    assert P.crc32c(6, d) == O.crc(6, d)
    after = P.stats()
    assert after["gpu_calls"] == mid["gpu_calls"] + 1 and after["gpu_fallbacks"] == before["gpu_fallbacks"]


def test_dropin_concurrent_with_device_batch(torch_dev, P, gpu_route):
    # a drop-in / host batch call while a device batch is in
    # flight on another stream must not share its workspace
    torch, dev = torch_dev
    n, L = 4096, 65536
    buf = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev)
    offs = np.arange(n) * L
    descs = P.make_descs([buf.data_ptr() + int(o) for o in offs], [L] * n, device=dev)
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    host = np.random.default_rng(32).integers(0, 256, 1 << 20, dtype=np.uint8)
    s = torch.cuda.Stream(dev)
    want_host = O.crc(3, host)
    for _ in range(3):
        P.dev_batch_async(descs, out, stream=s)  # 256 MiB in flight
        assert P.crc32c(3, host) == want_host    # staged host path meanwhile
        assert P.crc32c_batch([host.tobytes()], [3]) == [want_host]
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), O.crcs(buf.cpu().numpy(), offs, [L] * n))


def test_internal_workspace_two_streams(torch_dev, P):
    # two device batches on the INTERNAL workspace from two streams: the
    # second waits for the first instead of overwriting its workspace
    torch, dev = torch_dev
    jobs = []
    for k, (n, L) in enumerate(((2048, 65536), (64, 4 << 20))):
        buf = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev)
        offs = np.arange(n) * L
        descs = P.make_descs([buf.data_ptr() + int(o) for o in offs], [L] * n, [k] * n, device=dev)
        out = torch.zeros(n, dtype=torch.int32, device=dev)
        jobs.append((buf, offs, L, k, descs, out, torch.cuda.Stream(dev)))
    torch.cuda.synchronize()
    for _ in range(4):
        for buf, offs, L, k, descs, out, st in jobs:
            P.dev_batch_async(descs, out, stream=st)
    torch.cuda.synchronize()
    for buf, offs, L, k, descs, out, st in jobs:
        want = O.crcs(buf.cpu().numpy(), offs, [L] * len(offs), [k] * len(offs))
        assert np.array_equal(out.cpu().numpy().view(np.uint32), want)


def test_max_length_buffer(torch_dev, P):
    # the longest buffer the C-ABI can describe (unsigned int length:
    # 2^32 - 1 bytes) at an odd address, beside an empty and a 1-byte buffer;
    # 33.5 M rows in one buffer, split over every wave of the chip
    torch, dev = torch_dev
    n = (1 << 32) - 1
    buf = torch.randint(0, 256, (n + 64,), dtype=torch.uint8, device=dev)
    base = buf.data_ptr()
    seeds = [0x9E3779B9, 7, 0xFFFFFFFF]
    descs = P.make_descs([base + 5, base + 3, base + n + 10], [n, 0, 1], seeds, device=dev)
    out = torch.zeros(3, dtype=torch.int32, device=dev)
    P.dev_batch_async(descs, out)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    host = buf.cpu().numpy()
    H = O.hw()
    if H is not None:  # SSE4.2 restatement (bit-exact vs the reference, tests/test_oracle.py)
        want0 = H.hw_crc32c(seeds[0], host.ctypes.data + 5, n)
        # and the byte-loop oracle on the last 64 MiB, through the chaining law
        head = H.hw_crc32c(seeds[0], host.ctypes.data + 5, n - (64 << 20))
        tail = O.crc(0, host[5 + n - (64 << 20):5 + n])
        assert P.crc32c_combine(head, tail, 64 << 20) == want0
    else:
        want0 = O.crc(seeds[0], host[5:5 + n])
    assert int(got[0]) == want0
    assert int(got[1]) == seeds[1]
    assert int(got[2]) == O.crc(seeds[2], host[n + 10:n + 11])
