"""The bounds-checked kernel build (build/lib_dbg.so, -DPECH_DEBUG_BOUNDS,
built by `make`) on C4- and C2-shaped batches with unaligned starts and
ragged ends: every ring load (plan + main kernels, the direct kernel of the
small-buffer API, and the flat kernels of batches of up to 256 and 4,096
buffers) is
checked against its buffer's rows on the GPU (a violation prints "PECH OOB" and is redirected instead of faulting),
and every result must still equal the oracle.  Runs in a subprocess so the
release library stays the one this test process loads."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import sys
import numpy as np
import torch
sys.path.insert(0, "tests")
import oracle_lib as O
import pech_amd as P
assert P._lib.LIB_PATH.endswith("lib_dbg.so"), P._lib.LIB_PATH
dev = torch.device("cuda:0")
rng = np.random.default_rng(int(sys.argv[1]))
shape = sys.argv[2]
if shape == "c4":
    lens = np.array([4096] * 2048 + [65536] * 128 + [1 << 20] * 8 + [4 << 20] * 2, dtype=np.int64)
    lens = lens + rng.integers(-15, 16, lens.size)       # ragged ends
elif shape in ("flat", "flatg"):  # <= 256 / <= 4,096 buffers: the one-launch flat kernels
    m = 200 if shape == "flat" else 1500
    lens = rng.integers(0, 3 << 20 if shape == "flat" else 600 << 10, m)
    small = rng.random(m) < 0.3
    lens[small] = rng.integers(0, 300, int(small.sum()))
    lens[rng.random(m) < 0.1] = 0
else:
    lens = np.array([4096] * 8192, dtype=np.int64) + rng.integers(-33, 34, 8192)
rng.shuffle(lens)
offs = np.cumsum(np.concatenate([[7], lens[:-1] + rng.integers(1, 40, lens.size - 1)]))
host = rng.integers(0, 256, int(offs[-1] + lens[-1] + 64), dtype=np.uint8)
seeds = rng.integers(0, 1 << 32, lens.size, dtype=np.uint64)
buf = torch.from_numpy(host).to(dev)
descs = P.make_descs(buf.data_ptr() + offs, lens, seeds, device=dev)
out = torch.zeros(lens.size, dtype=torch.int32, device=dev)
if sys.argv[3] == "small":  # the direct kernel (no plan), C2 shapes and the over-contract C4 mix
    out.fill_(-1)
    P.dev_batch_small_async(descs, out)
else:  # "planned": plan + main at any size; "flat": the flat kernels up to their 4,096 buffers
    P.set_flat_max(0 if sys.argv[3] == "planned" else 4096)
    P.dev_batch_async(descs, out)
torch.cuda.synchronize()
got = out.cpu().numpy().view(np.uint32)
assert np.array_equal(got, O.crcs(host, offs, lens, seeds)), "parity"
print("ok", lens.size, int(lens.sum()))
"""


@pytest.mark.parametrize("seed,shape,api", [(1, "c4", "planned"), (2, "c2", "planned"), (3, "c4", "planned"),
                                            (4, "c2", "small"), (5, "c4", "small"), (6, "flat", "flat"),
                                            (7, "flat", "flat"), (8, "flatg", "flat"), (9, "flatg", "flat"),
                                            (10, "c4", "flat")])
def test_bounds_checked_build(seed, shape, api):
    lib = os.path.join(REPO, "build", "lib_dbg.so")
    assert os.path.exists(lib), "build/lib_dbg.so is built by `make`"
    env = dict(os.environ, PECH_CRC32C_LIB=lib)
    r = subprocess.run([sys.executable, "-c", SCRIPT, str(seed), shape, api], cwd=REPO, env=env, capture_output=True,
                       timeout=300)
    out = r.stdout.decode() + r.stderr.decode()
    assert "PECH OOB" not in out, out[-3000:]
    assert r.returncode == 0, out[-3000:]
    assert "ok" in r.stdout.decode()
