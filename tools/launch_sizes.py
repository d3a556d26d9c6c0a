"""Diagnostic (GPU box): main-kernel µs per launch (HIP events) for launches
of chosen shapes, e.g. odd launch sizes whose rows per wave are not a
multiple of 8:

    python tools/launch_sizes.py 8x4m 7x4m 5x4m+3x1m 40x700k 12x3m ...

<n>x<size>[+<n>x<size>...], sizes in bytes or with k/m suffixes (KiB/MiB).
Every launch is checked against the oracle once (first region)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import pech_amd as P  # noqa: E402
import oracle_lib as O  # noqa: E402


def parse(spec):
    sizes = []
    for part in spec.split("+"):
        n, s = part.split("x")
        mult = {"k": 1 << 10, "m": 1 << 20}.get(s[-1], 1)
        sizes += [int(s.rstrip("km")) * mult] * int(n)
    return np.asarray(sizes, dtype=np.int64)


def main():
    dev = torch.device("cuda:0")
    pool = torch.randint(0, 256, (2 << 30,), dtype=torch.uint8, device=dev)
    for spec in sys.argv[1:]:
        sizes = parse(spec)
        tot = int(sizes.sum())
        offs = np.concatenate([[0], np.cumsum(sizes)[:-1]])
        regions = max(1, min(64, (2 << 30) // tot))
        descs = [P.make_descs(pool.data_ptr() + r * tot + offs, sizes, device=dev) for r in range(regions)]
        out = torch.zeros(len(sizes), dtype=torch.int32, device=dev)
        ws = torch.empty(P.workspace_bytes(len(sizes)), dtype=torch.uint8, device=dev)
        P.dev_batch_ws_async(descs[0], out, ws)
        torch.cuda.synchronize()
        host = pool[:tot].cpu().numpy()
        ok = np.array_equal(out.cpu().numpy().view(np.uint32), O.crcs(host, offs, sizes))
        assert ok or os.environ.get("LS_NOCHECK") == "1", spec  # (LS_NOCHECK: diagnostic builds with wrong CRCs)
        for i in range(8):
            P.dev_batch_ws_async(descs[i % regions], out, ws)
        torch.cuda.synchronize()
        P.timing(True)
        P.timing_read()
        k = max(regions, 30)
        for i in range(k):
            P.dev_batch_ws_async(descs[i % regions], out, ws)
        torch.cuda.synchronize()
        P.timing_read()
        us = np.asarray(P.timing_samples(), dtype=np.float64) * 1e3
        P.timing(False)
        rows = int(sum((int(s) + 127) // 128 for s in sizes))
        print(f"{spec}: {tot / 2**20:.1f} MiB, {len(sizes)} buffers, ~{rows} rows (rows/1024 = {rows / 1024:.1f}): "
              f"main {np.mean(us):.2f} us (p50 {np.median(us):.2f}), parity {'ok' if ok else 'WRONG (diagnostic)'}")


if __name__ == "__main__":
    main()
