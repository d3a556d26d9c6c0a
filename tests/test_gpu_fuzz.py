"""Seeded fuzz of the gfx950 kernels against the oracle: random batch
shapes (counts across the chunk and wave boundaries, a mixture of sizes from
empty to several MiB, random byte offsets, overlapping and repeated buffers,
random seeds) through the device API, and the same shapes through the fused
CRC + copy with every destination byte and the bytes around the destinations
checked.  Bit-exact or fail."""
import numpy as np
import pytest

import oracle_lib as O
from test_copy import check_copy, run_copy

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    return torch, torch.device("cuda:0")


def random_sizes(rng, n):
    kind = rng.choice(5, n, p=[0.2, 0.35, 0.3, 0.13, 0.02])
    sizes = np.where(kind == 0, rng.integers(0, 64, n),
             np.where(kind == 1, rng.integers(64, 8192, n),
              np.where(kind == 2, rng.integers(8192, 200000, n),
               np.where(kind == 3, rng.integers(200000, 1 << 20, n), rng.integers(1 << 20, 5 << 20, n)))))
    return sizes.astype(np.int64)


def random_batch(rng):
    n = int(rng.choice([1, 7, 63, 64, 65, 1023, 1024, 1025, 2049, 4097, int(rng.integers(1, 6000))]))
    sizes = random_sizes(rng, n)
    while sizes.sum() > (96 << 20):  # bound the oracle's work
        sizes = sizes // 2
    gaps = rng.integers(0, 256, n)
    offs = int(rng.integers(0, 128)) + np.concatenate([[0], np.cumsum(sizes + gaps)[:-1]])
    total = int(offs[-1] + sizes[-1] + 256)
    if n > 4 and rng.random() < 0.3:  # some buffers alias others (repeated and overlapping ranges)
        k = int(rng.integers(1, n // 4 + 1))
        src = rng.integers(0, n, k)
        dst = rng.integers(0, n, k)
        offs[dst] = offs[src] + rng.integers(0, 64, k)
        sizes[dst] = np.minimum(sizes[src], total - 256 - offs[dst])
    seeds = [int(x) for x in rng.integers(0, 1 << 32, n)] if rng.random() < 0.5 else None
    return offs.astype(np.int64), sizes.astype(np.int64), seeds, total


@pytest.mark.parametrize("case", range(24))
def test_fuzz_device_batch(torch_dev, case):
    import pech_amd as P

    torch, dev = torch_dev
    rng = np.random.default_rng(1000 + case)
    offs, sizes, seeds, total = random_batch(rng)
    host = rng.integers(0, 256, total, dtype=np.uint8)
    buf = torch.from_numpy(host).to(dev)
    descs = P.make_descs(buf.data_ptr() + offs, sizes, seeds, device=dev)
    out = torch.full((len(sizes),), 0x5A5A5A5A, dtype=torch.int32, device=dev)
    P.dev_batch_async(descs, out)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    want = O.crcs(host, offs, sizes, seeds)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(i), int(offs[i]), int(sizes[i])) for i in bad[:5]]


@pytest.mark.parametrize("case", range(8))
def test_fuzz_fused_copy(torch_dev, case):
    torch, dev = torch_dev
    rng = np.random.default_rng(2000 + case)
    offs, sizes, seeds, total = random_batch(rng)
    # destinations never overlap each other; random byte alignment against the source
    dgap = rng.integers(0, 200, len(sizes))
    doffs = int(rng.integers(0, 64)) + np.concatenate([[0], np.cumsum(sizes + dgap)[:-1]])
    dst_bytes = int(doffs[-1] + sizes[-1] + 256)
    host = rng.integers(0, 256, total, dtype=np.uint8)
    got, got_dst = run_copy(torch, dev, host, offs, sizes, doffs, dst_bytes, seeds)
    assert np.array_equal(got, O.crcs(host, offs, sizes, seeds))
    check_copy(host, offs, sizes, doffs, got_dst)
