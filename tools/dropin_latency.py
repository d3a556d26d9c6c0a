"""Latency of the drop-in crc32c() (one synchronous call per buffer, pageable
host memory, as messenger.c calls it per <=4 KiB piece) on the GPU box."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch  # noqa: F401  (load torch's HIP runtime first)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pech_amd import _lib  # noqa: E402

L = _lib.lib()
res = {}
for n in (49, 4096, 65536, 1 << 20):
    buf = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8)
    p = buf.ctypes.data
    for _ in range(20):
        L.crc32c(0, p, n)
    reps = 2000 if n <= 65536 else 200
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        L.crc32c(0, p, n)
        t.append(time.perf_counter() - t0)
    t = np.asarray(t) * 1e6
    res[n] = {"p50_us": round(float(np.median(t)), 2), "p90_us": round(float(np.percentile(t, 90)), 2)}
print(json.dumps({"dropin_crc32c_latency": res}))
