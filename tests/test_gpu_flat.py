"""GPU parity of the one-launch device batch (pech_crc32c_flat: batches of at
most 256 buffers with no plan kernel; pech_crc32c_flatg: up to 4,096, its
prologue scanning over the workgroup and its steps reading the descriptors
in place; crc32c_set_flat_max) against the oracle, bit-exact, and against
the two-launch plan + main path on the same batch.  Cases particular to this kernel: its rows cover ALL of a buffer's
bytes (last-line pieces kept below kb bytes, x^(-8T) at the end), empty
buffers kept in place in descriptor order (runs of them before large ones),
seeds added by the wave that initialises out[], out[] zeroed in the launch
and published by a per-launch tag (garbage in out[], back-to-back launches
on one workspace, two and four streams at once, whose workgroups interleave
on the CUs), the uniform pool, one buffer split over many workgroups, and
the 256 / 257 boundary between the two flat kernels and 4,096 / 4,097 to the
planned path."""
import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

FLAT_MAX = 4096  # PECH_FLATG_MAX: pech_crc32c_flat up to 256 buffers, pech_crc32c_flatg above


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    return torch, torch.device("cuda:0")


@pytest.fixture(scope="module")
def P():
    import pech_amd

    return pech_amd


@pytest.fixture(params=["flat", "planned"])
def route(request, P):
    """Run the test on the flat kernel (default) and on plan + main."""
    prev = P.set_flat_max(FLAT_MAX if request.param == "flat" else 0)
    yield request.param
    P.set_flat_max(prev)


def dev_crcs(torch, P, buf, offs, lens, seeds=None, ws=None, stream=None, sync=True):
    descs = P.make_descs(buf.data_ptr() + np.asarray(offs, dtype=np.int64), lens, seeds, device=buf.device)
    out = torch.full((len(lens),), 0x5A5A5A5A, dtype=torch.int32, device=buf.device)  # garbage must not leak
    if ws is None:
        ws = torch.empty(P.workspace_bytes(len(lens)), dtype=torch.uint8, device=buf.device)
    P.dev_batch_ws_async(descs, out, ws, stream=stream)
    if not sync:
        return out, descs
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


def rand_buf(torch, dev, nbytes, seed):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    return torch.randint(0, 256, (max(nbytes, 1),), dtype=torch.uint8, device=dev, generator=g)


def layout(sizes, rng, max_gap=200):
    offs = np.zeros(len(sizes), dtype=np.int64)
    pos = int(rng.integers(0, 128))
    for i, L in enumerate(sizes):
        offs[i] = pos
        pos += int(L) + int(rng.integers(0, max_gap))
    return offs, pos + 64


def check(torch, P, buf, offs, lens, seeds=None):
    got = dev_crcs(torch, P, buf, offs, lens, seeds)
    want = O.crcs(buf.cpu().numpy(), offs, lens, seeds)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(offs[i]), int(lens[i]), hex(got[i]), hex(want[i])) for i in bad[:8]]


def test_known_answer(torch_dev, P, route):
    torch, dev = torch_dev
    buf = torch.from_numpy(np.frombuffer(b"123456789", dtype=np.uint8).copy()).to(dev)
    got = dev_crcs(torch, P, buf, [0, 0, 0], [9, 9, 0], [0, 0xFFFFFFFF, 0x1234])
    assert got[0] == 0x58E3FA20
    assert (~int(got[1])) & 0xFFFFFFFF == 0xE3069283
    assert got[2] == 0x1234


@pytest.mark.parametrize("n", [1, 2, 7, 8, 9, 63, 64, 65, 255, 256, 257, 300, 511, 512, 1023, 1024, 1025, 2049, 4095,
                               4096, 4097])
def test_random_sizes(torch_dev, P, route, n):
    # sizes from 0 to 5 MiB (at most ~2 GiB a batch) at random byte offsets,
    # random seeds, empties
    torch, dev = torch_dev
    rng = np.random.default_rng(1000 + n)
    lens = rng.integers(0, min(5 << 20, (2 << 30) // n), n)
    lens[rng.random(n) < 0.15] = 0
    small = rng.random(n) < 0.3
    lens[small] = rng.integers(1, 300, int(small.sum()))
    seeds = rng.integers(0, 1 << 32, n, dtype=np.uint64)
    seeds[rng.random(n) < 0.5] = 0
    offs, total = layout(lens, rng)
    buf = rand_buf(torch, dev, total, n)
    check(torch, P, buf, offs, lens, seeds)


@pytest.mark.parametrize("copies", [1, 8])
@pytest.mark.parametrize("L", [1, 15, 16, 17, 113, 127, 128, 129, 255, 4096, 4100, 65537])
def test_last_line_masks(torch_dev, P, route, L, copies):
    # every start offset within a line: head and tail in one line (small L),
    # T from 0 to 127, a buffer ending exactly on a line (T = 0); 8 copies:
    # 1,024 buffers (pech_crc32c_flatg)
    torch, dev = torch_dev
    m = 128 * copies
    offs = np.arange(m, dtype=np.int64) * (L + 128 + 37) + np.arange(m) % 128
    buf = rand_buf(torch, dev, int(offs[-1]) + L + 64, L)
    check(torch, P, buf, offs, [L] * m)


@pytest.mark.parametrize("cap", [256, 3000])
def test_empty_runs_before_large_buffers(torch_dev, P, route, cap):
    # runs of 8 and more empty buffers (no rows: skipped in place) between
    # large ones, and a batch that ends in empties; whole workgroup-scan
    # threads (4 positions each) without rows in the large batch
    torch, dev = torch_dev
    rng = np.random.default_rng(5)
    lens = []
    while len(lens) < cap - 9:
        lens += [0] * int(rng.integers(1, 20 if cap <= 256 else 60))
        lens += [int(rng.integers(100000, 3 << 20 if cap <= 256 else 1 << 20))]
    lens = np.asarray(lens[:cap - 9] + [0] * 9)
    seeds = rng.integers(0, 1 << 32, len(lens), dtype=np.uint64)
    offs, total = layout(lens, rng)
    buf = rand_buf(torch, dev, total, 5)
    check(torch, P, buf, offs, lens, seeds)


@pytest.mark.parametrize("n", [40, 2000])
def test_all_empty(torch_dev, P, route, n):
    torch, dev = torch_dev
    buf = rand_buf(torch, dev, 64, 1)
    got = dev_crcs(torch, P, buf, [0] * n, [0] * n, list(range(n)))
    assert [int(x) for x in got] == list(range(n))


@pytest.mark.parametrize("L,off", [((64 << 20) + 12345, 3), (33 << 20, 0), (4 << 20, 0), (300 * 128 + 5, 77)])
def test_one_buffer_over_many_workgroups(torch_dev, P, route, L, off):
    # one buffer split over every wave that walks rows (XORs from many
    # workgroups into one out[] word zeroed in the same launch)
    torch, dev = torch_dev
    buf = rand_buf(torch, dev, L + off + 64, L)
    host = buf.cpu().numpy()
    for seed in (0, 0xFFFFFFFF):
        got = dev_crcs(torch, P, buf, [off], [L], [seed])
        assert int(got[0]) == O.crc(seed, host[off:off + L])


@pytest.mark.parametrize("n,L,gap", [(256, 4 << 20, 0), (200, (1 << 20) + 3, 5), (256, 65536, 0), (16, 16 << 20, 128),
                                     (4096, 65536, 0), (1024, 1 << 20, 0), (600, (1 << 20) + 3, 5), (300, 4 << 20, 0)])
def test_uniform_pool(torch_dev, P, route, n, L, gap):
    # every buffer the same rows: the workgroup pool (positions by division)
    torch, dev = torch_dev
    offs = np.arange(n, dtype=np.int64) * (L + gap) + (7 if gap % 128 else 0)
    buf = rand_buf(torch, dev, int(offs[-1]) + L + 64, n + L)
    seeds = [int(x) for x in np.random.default_rng(n).integers(0, 1 << 32, n)]
    check(torch, P, buf, offs, [L] * n, seeds)


def test_back_to_back_launches_one_workspace(torch_dev, P):
    # each launch publishes its zeroed out[] under a fresh tag: a stale tag
    # from the previous launch on the same workspace must not let a wave XOR
    # into an out[] that is not zeroed yet
    torch, dev = torch_dev
    ws = torch.empty(P.workspace_bytes(FLAT_MAX), dtype=torch.uint8, device=dev)
    rng = np.random.default_rng(77)
    bufs, outs = [], []
    for k in range(40):
        n = int(rng.integers(1, 300)) if k % 2 else int(rng.integers(1, FLAT_MAX + 1))
        lens = rng.integers(0, min(1 << 20, (512 << 20) // n), n)
        offs, total = layout(lens, rng, 64)
        buf = rand_buf(torch, dev, total, 100 + k)
        out, descs = dev_crcs(torch, P, buf, offs, lens, ws=ws, sync=False)
        bufs.append((buf, offs, lens, descs))
        outs.append(out)
    torch.cuda.synchronize()
    for (buf, offs, lens, _), out in zip(bufs, outs):
        got = out.cpu().numpy().view(np.uint32)
        assert np.array_equal(got, O.crcs(buf.cpu().numpy(), offs, lens))


def test_two_streams_two_workspaces(torch_dev, P):
    torch, dev = torch_dev
    streams = [torch.cuda.Stream(device=dev) for _ in range(2)]
    wss = [torch.empty(P.workspace_bytes(FLAT_MAX), dtype=torch.uint8, device=dev) for _ in range(2)]
    rng = np.random.default_rng(3)
    jobs = []
    for k in range(16):
        lens = [int(x) for x in rng.integers(1 << 16, 4 << 20, 64)]
        offs, total = layout(lens, rng, 16)
        buf = rand_buf(torch, dev, total, 300 + k)
        torch.cuda.synchronize()
        out, descs = dev_crcs(torch, P, buf, offs, lens, ws=wss[k % 2], stream=streams[k % 2], sync=False)
        jobs.append((buf, offs, lens, out, descs))
    torch.cuda.synchronize()
    for buf, offs, lens, out, _ in jobs:
        assert np.array_equal(out.cpu().numpy().view(np.uint32), O.crcs(buf.cpu().numpy(), offs, lens))


@pytest.mark.parametrize("n,L", [(256, 4 << 20), (4096, 64 << 10)])
def test_flat_and_planned_agree_on_c3(torch_dev, P, n, L):
    # BASELINE C3 (256 x 4 MiB) and C4's 64 KiB class (4,096 x 64 KiB) through
    # both paths, every output vs the oracle
    torch, dev = torch_dev
    buf = rand_buf(torch, dev, n * L, 33)
    offs = np.arange(n, dtype=np.int64) * L
    want = O.crcs(buf.cpu().numpy(), offs, [L] * n)
    prev = P.set_flat_max(FLAT_MAX)
    try:
        flat = dev_crcs(torch, P, buf, offs, [L] * n)
        P.set_flat_max(0)
        planned = dev_crcs(torch, P, buf, offs, [L] * n)
    finally:
        P.set_flat_max(prev)
    assert np.array_equal(flat, want) and np.array_equal(planned, want)


def test_set_flat_max_clamps(P):
    prev = P.set_flat_max(10 ** 6)
    assert P.set_flat_max(prev) == FLAT_MAX


@pytest.mark.parametrize("n,L", [(128, 1 << 20), (1024, 256 << 10)])
def test_concurrent_flat_launches_on_four_streams(torch_dev, P, n, L):
    """Flat launches on four streams at once, each large enough to fill the
    chip: their workgroups interleave on the CUs, so one launch's workgroup 0
    may wait for a CU while its other workgroups reach their first XOR.
    Those may not wait for workgroup 0 (two such launches deadlocked each
    other, each holding the CUs the other's workgroup 0 needed): a running
    wave claims out[]'s initialisation instead (flat_init)."""
    torch, dev = torch_dev
    streams = [torch.cuda.Stream(device=dev) for _ in range(4)]
    wss = [torch.empty(P.workspace_bytes(FLAT_MAX), dtype=torch.uint8, device=dev) for _ in range(8)]
    rng = np.random.default_rng(44)
    bufs = [rand_buf(torch, dev, n * L + 64, 500 + k) for k in range(4)]
    torch.cuda.synchronize()
    jobs = []
    for k in range(32):
        off = np.sort(rng.integers(0, 64, n)) + np.arange(n, dtype=np.int64) * L
        lens = rng.integers(L // 2, L - 64, n)
        seeds = rng.integers(0, 1 << 32, n, dtype=np.uint64) if k % 3 == 0 else None
        b = bufs[k % 4]
        out, descs = dev_crcs(torch, P, b, off, lens, seeds, ws=wss[k % 8], stream=streams[k % 4], sync=False)
        jobs.append((b, off, lens, seeds, out, descs))
    torch.cuda.synchronize()
    hosts = [b.cpu().numpy() for b in bufs]
    for k, (b, off, lens, seeds, out, _) in enumerate(jobs):
        want = O.crcs(hosts[k % 4], off, lens, seeds)
        assert np.array_equal(out.cpu().numpy().view(np.uint32), want), k


def test_one_huge_buffer_among_many(torch_dev, P, route):
    # pech_crc32c_flatg with one 64 MiB buffer among 700 small ones: shares of
    # many waves inside one position, the workgroup scan's thread holding it
    torch, dev = torch_dev
    rng = np.random.default_rng(9)
    lens = rng.integers(0, 40000, 701)
    lens[350] = (64 << 20) + 999
    seeds = rng.integers(0, 1 << 32, 701, dtype=np.uint64)
    offs, total = layout(lens, rng)
    buf = rand_buf(torch, dev, total, 9)
    check(torch, P, buf, offs, lens, seeds)
