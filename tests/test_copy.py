"""Fused CRC + copy (crc32c_dev_copy_batch_*, SURVEY §8f row 4: the copies
memstore makes of the same bytes, src/ceph/memstore.c:306, :445): every CRC
bit-exact against the oracle, every destination byte equal to its source,
and not one byte outside the destination ranges written (guard pattern)."""
import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

GUARD = 0xA5


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    return torch, torch.device("cuda:0")


def run_copy(torch, dev, host_src, src_offs, lens, dst_offs, dst_bytes, seeds=None, small=False):
    import pech_amd as P
    from pech_amd import _lib

    src = torch.from_numpy(host_src).to(dev)
    dst = torch.full((dst_bytes,), GUARD, dtype=torch.uint8, device=dev)
    descs = P.make_descs(src.data_ptr() + np.asarray(src_offs, dtype=np.int64), lens, seeds, device=dev)
    dsts = torch.from_numpy((dst.data_ptr() + np.asarray(dst_offs, dtype=np.int64)).astype(np.int64)).to(dev)
    out = torch.zeros(len(lens), dtype=torch.int32, device=dev)
    fn = "crc32c_dev_copy_batch_small_async" if small else "crc32c_dev_copy_batch_async"
    if small:  # the direct kernel stores its results: out must need no initialisation
        out.fill_(-1)
    rc = getattr(_lib.lib(), fn)(descs.data_ptr(), dsts.data_ptr(), out.data_ptr(), len(lens),
                                 torch.cuda.current_stream(dev).cuda_stream)
    _lib.check(rc, fn)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32), dst.cpu().numpy()


def check_copy(host_src, src_offs, lens, dst_offs, got_dst):
    mask = np.zeros(got_dst.size, dtype=bool)
    for so, n, do in zip(src_offs, lens, dst_offs):
        so, n, do = int(so), int(n), int(do)
        assert np.array_equal(got_dst[do:do + n], host_src[so:so + n]), (so, n, do)
        mask[do:do + n] = True
    outside = got_dst[~mask]
    assert np.all(outside == GUARD), f"{int(np.count_nonzero(outside != GUARD))} bytes written outside destinations"


@pytest.mark.parametrize("small", [False, True])
def test_copy_random_unaligned(torch_dev, small):
    # random lengths (tiny ones included), sources and destinations at
    # unrelated byte alignments, gaps between destinations to catch stray
    # writes; small: the one-launch direct copy (crc32c_dev_copy_batch_small_async)
    torch, dev = torch_dev
    rng = np.random.default_rng(77)
    n = 1500
    lens = rng.integers(0, 70000 if not small else 40000, n)
    tiny = rng.random(n) < 0.15
    lens[tiny] = rng.integers(0, 40, int(tiny.sum()))
    src_offs, dst_offs = np.zeros(n, np.int64), np.zeros(n, np.int64)
    sp = dp = 0
    for i in range(n):
        sp += int(rng.integers(0, 48))
        dp += int(rng.integers(1, 48))
        src_offs[i], dst_offs[i] = sp, dp
        sp += int(lens[i])
        dp += int(lens[i])
    host = rng.integers(0, 256, sp + 64, dtype=np.uint8)
    seeds = rng.integers(0, 1 << 32, n, dtype=np.uint64)
    got, dst = run_copy(torch, dev, host, src_offs, lens, dst_offs, dp + 64, seeds, small=small)
    assert np.array_equal(got, O.crcs(host, src_offs, lens, seeds))
    check_copy(host, src_offs, lens, dst_offs, dst)


@pytest.mark.parametrize("n,maxlen", [(1, 5), (7, 33), (300, 200), (4097, 4200), (70000, 5000)])
def test_copy_small_api_shapes(torch_dev, n, maxlen):
    # the direct copy over tiny to messenger-sized buffers, every length mod
    # 16 and every source/destination alignment mix, counts across the
    # workgroup and 128-position steps
    torch, dev = torch_dev
    rng = np.random.default_rng(n * 31 + maxlen)
    lens = rng.integers(0, maxlen + 1, n)
    src_offs, dst_offs = np.zeros(n, np.int64), np.zeros(n, np.int64)
    sp = dp = 0
    for i in range(n):
        sp += int(rng.integers(0, 33))
        dp += int(rng.integers(1, 33))
        src_offs[i], dst_offs[i] = sp, dp
        sp += int(lens[i])
        dp += int(lens[i])
    host = rng.integers(0, 256, sp + 64, dtype=np.uint8)
    seeds = np.where(rng.random(n) < 0.5, 0, rng.integers(0, 1 << 32, n)).astype(np.uint64)
    got, dst = run_copy(torch, dev, host, src_offs, lens, dst_offs, dp + 64, seeds, small=True)
    assert np.array_equal(got, O.crcs(host, src_offs, lens, seeds))
    check_copy(host, src_offs, lens, dst_offs, dst)


@pytest.mark.parametrize("shape", ["c2", "c3", "c4"])
def test_copy_bench_shapes(torch_dev, shape):
    torch, dev = torch_dev
    rng = np.random.default_rng(3)
    if shape == "c2":
        lens = [4096] * 16384
    elif shape == "c3":
        lens = [4 << 20] * 16
    else:
        lens = [4096] * 4096 + [65536] * 256 + [1 << 20] * 16 + [4 << 20] * 4
        rng.shuffle(lens)
    lens = np.asarray(lens, np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    host = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    dst_offs = offs + 4096 * np.arange(len(lens))  # a guard page between destinations
    got, dst = run_copy(torch, dev, host, offs, lens, dst_offs, int(dst_offs[-1] + lens[-1] + 4096))
    assert np.array_equal(got, O.crcs(host, offs, lens))
    check_copy(host, offs, lens, dst_offs, dst)


def test_copy_huge_buffer_misaligned(torch_dev):
    torch, dev = torch_dev
    rng = np.random.default_rng(4)
    L = (40 << 20) + 12345
    host = rng.integers(0, 256, L + 64, dtype=np.uint8)
    got, dst = run_copy(torch, dev, host, [3], [L], [11], L + 64, [0x12345678])
    assert int(got[0]) == O.crc(0x12345678, host[3:3 + L])
    check_copy(host, [3], [L], [11], dst)


@pytest.mark.parametrize("size,n,soff,doff", [
    (4 << 20, 37, 0, 0),                 # interleaved rows, ranges cut mid-buffer (37 over 256 workgroups)
    ((1 << 17) + 5, 300, 3, 11),         # 1,025 rows each, unaligned sources and destinations
    ((1 << 17) - 16, 513, 16, 1),        # just below and around the threshold of the mode
    ((6 << 20) + 99, 3, 7, 0),           # few buffers, many workgroups each
    (1025 * 128 - 100, 300, 0, 0),       # workgroup ranges that start 4 rows before a buffer's end (round 6)
    (1025 * 128 - 100, 3, 64, 5),        # ... and the small-launch ranges of 3 buffers
])
def test_copy_uniform_large_buffers(torch_dev, size, n, soff, doff):
    # uniform batches of large buffers take the fused copy's interleaved mode
    # (the workgroup's 128 lane groups walk rows 128 apart, plan_il): every
    # CRC and every destination byte, guards intact
    torch, dev = torch_dev
    rng = np.random.default_rng(size + n)
    # strides that are whole lines: every buffer has the same alignment, so
    # the same rows -- a uniform batch (until round 6 the strides were size +
    # 4 KiB, which left only the first case uniform)
    stride_s, stride_d = (size + 4096 + 127) // 128 * 128, size + 8192
    src_offs = soff + stride_s * np.arange(n, dtype=np.int64)  # the same alignment for every buffer: uniform
    dst_offs = doff + stride_d * np.arange(n, dtype=np.int64)
    lens = np.full(n, size, np.int64)
    host = rng.integers(0, 256, int(src_offs[-1] + size + 64), dtype=np.uint8)
    seeds = rng.integers(0, 1 << 32, n, dtype=np.uint64)
    got, dst = run_copy(torch, dev, host, src_offs, lens, dst_offs, int(dst_offs[-1] + size + 4096), seeds)
    assert np.array_equal(got, O.crcs(host, src_offs, lens, seeds))
    check_copy(host, src_offs, lens, dst_offs, dst)
