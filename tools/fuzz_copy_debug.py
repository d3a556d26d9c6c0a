"""GPU box: per-buffer mismatch report of the fused-copy fuzz cases (tests/test_gpu_fuzz.py)."""
import sys, os, numpy as np
sys.path.insert(0, 'tests'); sys.path.insert(0, '.')
import torch
import test_gpu_fuzz as F
from test_copy import run_copy
import oracle_lib as O
dev = torch.device('cuda:0')
for case in range(8):
    rng = np.random.default_rng(2000 + case)
    offs, sizes, seeds, total = F.random_batch(rng)
    dgap = rng.integers(0, 200, len(sizes))
    doffs = int(rng.integers(0, 64)) + np.concatenate([[0], np.cumsum(sizes + dgap)[:-1]])
    dst_bytes = int(doffs[-1] + sizes[-1] + 256)
    host = rng.integers(0, 256, total, dtype=np.uint8)
    got, gd = run_copy(torch, dev, host, offs, sizes, doffs, dst_bytes, seeds)
    crc_ok = np.array_equal(got, O.crcs(host, offs, sizes, seeds))
    bad = []
    for j, (so, n, do) in enumerate(zip(offs, sizes, doffs)):
        so, n, do = int(so), int(n), int(do)
        g = gd[do:do+n]; w = host[so:so+n]
        if not np.array_equal(g, w):
            idx = np.nonzero(g != w)[0]
            bad.append((j, so, n, do, int(idx[0]), int(idx[-1]), len(idx), (so + int(idx[0])) % 16, (so+n) % 16))
    print(os.environ.get('PECH_CRC32C_LIB','cur'), 'case', case, 'n', len(sizes), 'crc_ok', crc_ok, 'bad', len(bad), bad[:4])
