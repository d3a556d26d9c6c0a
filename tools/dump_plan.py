"""Debug helper (GPU box): run one batch through the explicit-workspace API
and dump the plan kernel's outputs (cores, lrs, partials, nzs)."""
import json, os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
import pech_amd as P
from pech_amd import _lib
from gen import splitmix_bytes
K = json.load(open(os.path.join(REPO, "tests", "golden", "kat.json")))
dev = torch.device("cuda:0")
stream = torch.from_numpy(np.frombuffer(splitmix_bytes(0xC0FFEE, 3 * 65536 + 4096), dtype=np.uint8).copy()).to(dev)
v = K["vectors"]
descs = P.make_descs([stream.data_ptr() + x["off"] for x in v], [x["len"] for x in v], [x["seed"] for x in v], device=dev)
n = len(v)
L = _lib.lib()
wsb = L.crc32c_dev_workspace_bytes(n)
ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
out = torch.zeros(n, dtype=torch.int32, device=dev)
rc = L.crc32c_dev_batch_ws_async(descs.data_ptr(), out.data_ptr(), n, ws.data_ptr(), wsb, torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
w = ws.cpu().numpy()
slots = 1024
cores = w[:slots * 16].view(np.uint32).reshape(slots, 4)
lrs = w[slots * 16: slots * 20].view(np.uint32)
part = w[slots * 20: slots * 20 + 4096].view(np.uint32)
nzs = w[slots * 20 + 4096: slots * 20 + 8192].view(np.uint32)
nz = int(nzs[0])
rows = cores[:nz, 2]
exp = np.concatenate([[0], np.cumsum(rows)])[:nz]
print("rc", rc, "nz", nz, "partial", part[0], "sum rows", rows.sum())
bad = np.nonzero(lrs[:nz] != exp)[0]
print("lrs mismatches", len(bad), "first", bad[:10])
print("lrs[150:180]", lrs[150:180].tolist())
print("exp[150:180]", exp[150:180].tolist())
print("rows[150:180]", rows[150:180].tolist())
print("monotone", bool(np.all(np.diff(lrs[:nz].astype(np.int64)) >= 0)))
