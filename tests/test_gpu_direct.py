"""GPU parity of the small-buffer device batch (crc32c_dev_batch_small_async:
the direct kernel, no plan launch, no workspace) against the oracle,
bit-exact.  The cases follow the reference's own coverage of the messenger
path (empty, ragged, seeded, unaligned pieces) plus what is
particular to this kernel: positions split per wave, 16-position
interleave, tails / seeds / in-block buffers on the slow path, idle groups,
batches beyond one launch (2^20 descriptors), and buffers above the 32 KiB
contract (correct, only unbalanced)."""
import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    return torch, torch.device("cuda:0")


@pytest.fixture(scope="module")
def P():
    import pech_amd

    return pech_amd


def run_small(torch, P, buf, offs, lens, seeds=None, stream=None):
    descs = P.make_descs(buf.data_ptr() + np.asarray(offs, dtype=np.int64), lens, seeds, device=buf.device)
    # stored results: garbage in out[] must not leak into them
    out = torch.full((len(lens),), 0x5A5A5A5A, dtype=torch.int32, device=buf.device)
    P.dev_batch_small_async(descs, out, stream=stream)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


def rand_buf(torch, dev, nbytes, seed):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    return torch.randint(0, 256, (max(nbytes, 1),), dtype=torch.uint8, device=dev, generator=g)


def packed(sizes, align=1, skew=0):
    sizes = np.asarray(sizes, dtype=np.int64)
    step = (sizes + align - 1) // align * align + skew
    offs = np.concatenate([[0], np.cumsum(step)[:-1]]).astype(np.int64)
    return offs, int(offs[-1] + sizes[-1]) if len(sizes) else 0


def test_known_answer(torch_dev, P):
    torch, dev = torch_dev
    buf = torch.from_numpy(np.frombuffer(b"123456789", dtype=np.uint8).copy()).to(dev)
    got = run_small(torch, P, buf, [0, 0], [9, 9], [0, 0xFFFFFFFF])
    assert got[0] == 0x58E3FA20
    assert (~int(got[1])) & 0xFFFFFFFF == 0xE3069283


@pytest.mark.parametrize("size,skew", [(4096, 0), (4100, 1), (512, 0), (32767, 3), (128, 0), (1000, 7)])
def test_uniform_batches(torch_dev, P, size, skew):
    # the messenger's shapes: C2 (4 KiB aligned), C2-odd (4,100 B at odd offsets)
    torch, dev = torch_dev
    n = 8192 if size <= 4100 else 1024
    offs, total = packed([size] * n, 1, skew)
    buf = rand_buf(torch, dev, total, size + skew)
    got = run_small(torch, P, buf, offs, [size] * n)
    assert np.array_equal(got, O.crcs(buf.cpu().numpy(), offs, [size] * n))


@pytest.mark.parametrize("n", [1, 2, 7, 8, 9, 15, 16, 17, 31, 33, 255, 256, 257, 4095, 4097, 32767, 32769,
                               65537, 98309])
def test_position_splits(torch_dev, P, n):
    # n below, at and across the workgroup count (256), the workgroup step
    # (128 positions per workgroup: 32,768 over the chip), the wave count and
    # the 8-position steps
    torch, dev = torch_dev
    rng = np.random.default_rng(n)
    sizes = rng.integers(1, 9000, n)
    offs, total = packed(sizes, 1, 5)
    seeds = rng.integers(0, 1 << 32, n, dtype=np.uint64)
    buf = rand_buf(torch, dev, total, n)
    got = run_small(torch, P, buf, offs, sizes, seeds)
    assert np.array_equal(got, O.crcs(buf.cpu().numpy(), offs, sizes, seeds))


def test_tiny_and_empty_buffers(torch_dev, P):
    # every length 0..48 at every offset mod 16, seeded and not: buffers
    # inside one 16-byte block take the slow path alone
    torch, dev = torch_dev
    lens, offs = [], []
    for off in range(16):
        for ln in range(49):
            lens.append(ln)
            offs.append(4096 + 64 * len(offs) + off)
    n = len(lens)
    buf = rand_buf(torch, dev, offs[-1] + 128, 3)
    host = buf.cpu().numpy()
    for seeds in (None, [0xFFFFFFFF] * n, list(range(1, n + 1))):
        got = run_small(torch, P, buf, offs, lens, seeds)
        assert np.array_equal(got, O.crcs(host, offs, lens, seeds))


def test_ragged_fuzz(torch_dev, P):
    # ragged sizes below the contract, any alignment, mixed seeds, overlap
    torch, dev = torch_dev
    rng = np.random.default_rng(2024)
    buf = rand_buf(torch, dev, 64 << 20, 11)
    host = buf.cpu().numpy()
    for trial in range(6):
        n = int(rng.integers(1, 30000))
        sizes = np.where(rng.random(n) < 0.1, rng.integers(0, 64, n), rng.integers(0, 32768, n))
        offs = rng.integers(0, (64 << 20) - 32768, n)
        seeds = np.where(rng.random(n) < 0.5, 0, rng.integers(0, 1 << 32, n)).astype(np.uint64)
        got = run_small(torch, P, buf, offs, sizes, seeds)
        assert np.array_equal(got, O.crcs(host, offs, sizes, seeds)), trial


def test_buffers_above_the_contract(torch_dev, P):
    # larger buffers are walked by one group alone: slower, still exact, and
    # the idle groups beside them stay within valid memory
    torch, dev = torch_dev
    sizes = [4096] * 40 + [1 << 20, 3, (2 << 20) + 5, 0, 40000] + [100] * 37
    offs, total = packed(sizes, 16, 0)
    offs = offs + 1
    buf = rand_buf(torch, dev, total + 64, 5)
    got = run_small(torch, P, buf, offs, sizes, [7] * len(sizes))
    assert np.array_equal(got, O.crcs(buf.cpu().numpy(), offs, sizes, [7] * len(sizes)))


def test_batch_beyond_one_launch(torch_dev, P):
    # 2^20 + 1000 descriptors: two launches, the second's slots offset
    torch, dev = torch_dev
    n = (1 << 20) + 1000
    rng = np.random.default_rng(9)
    sizes = rng.integers(0, 200, n)
    offs = rng.integers(0, (8 << 20) - 256, n)
    buf = rand_buf(torch, dev, 8 << 20, 13)
    got = run_small(torch, P, buf, offs, sizes)
    assert np.array_equal(got, O.crcs(buf.cpu().numpy(), offs, sizes))


def test_matches_the_planned_batch(torch_dev, P):
    # the two device entry points agree on a C2-odd batch
    torch, dev = torch_dev
    n, size = 4096, 4100
    offs, total = packed([size] * n, 1, 1)
    buf = rand_buf(torch, dev, total, 17)
    descs = P.make_descs(buf.data_ptr() + offs, [size] * n, device=dev)
    a = torch.zeros(n, dtype=torch.int32, device=dev)
    b = torch.zeros(n, dtype=torch.int32, device=dev)
    P.dev_batch_async(descs, a)
    P.dev_batch_small_async(descs, b)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


def test_concurrent_streams_share_nothing(torch_dev, P):
    # no workspace: batches on several streams may overlap freely
    torch, dev = torch_dev
    streams = [torch.cuda.Stream(dev) for _ in range(4)]
    jobs = []
    for i, s in enumerate(streams):
        n, size = 2048, 4096 + 13 * i
        offs, total = packed([size] * n, 1, i)
        buf = rand_buf(torch, dev, total, 40 + i)
        descs = P.make_descs(buf.data_ptr() + offs, [size] * n, [i] * n, device=dev)
        out = torch.zeros(n, dtype=torch.int32, device=dev)
        jobs.append((buf, offs, n, size, i, descs, out, s))
    torch.cuda.synchronize()
    for rep in range(3):
        for buf, offs, n, size, i, descs, out, s in jobs:
            P.dev_batch_small_async(descs, out, stream=s)
    torch.cuda.synchronize()
    for buf, offs, n, size, i, descs, out, s in jobs:
        assert np.array_equal(out.cpu().numpy().view(np.uint32), O.crcs(buf.cpu().numpy(), offs, [size] * n, [i] * n))


def test_graph_capture(torch_dev, P):
    torch, dev = torch_dev
    n, size = 1024, 4100
    offs, total = packed([size] * n, 1, 1)
    buf = rand_buf(torch, dev, total, 23)
    descs = P.make_descs(buf.data_ptr() + offs, [size] * n, device=dev)
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        P.dev_batch_small_async(descs, out, stream=s)
    out.fill_(-1)
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), O.crcs(buf.cpu().numpy(), offs, [size] * n))
