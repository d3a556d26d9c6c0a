"""Diagnostic (GPU box): per-wave entry/start/end s_memrealtime of the main kernel for
one c3-shaped batch, using the PECH_STAMPS build (PECH_CRC32C_LIB)."""
import ctypes, os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import pech_amd as P
from pech_amd import _lib
cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
if os.environ.get("PECH_FLAT_MAX"):  # 0: the planned path (plan + main) for batches of <= 256 buffers
    P.set_flat_max(int(os.environ["PECH_FLAT_MAX"]))
dev = torch.device("cuda:0")
if cfg == "c3":
    sizes = np.full(256, 4 << 20, dtype=np.int64)
elif cfg.endswith("x4m"):  # launch-size series: <n> x 4 MiB
    sizes = np.full(int(cfg[:-3]), 4 << 20, dtype=np.int64)
elif "x" in cfg and cfg.split("x")[0].isdigit():  # <n>x<bytes>[k|m] (tools/launch_sizes.py shapes)
    n, sz = cfg.split("x")
    sizes = np.full(int(n), int(sz.rstrip("km")) * {"k": 1 << 10, "m": 1 << 20}.get(sz[-1], 1), dtype=np.int64)
elif cfg == "c4":  # bench.py's c4_sizes: equal bytes per class, shuffled with seed 42
    sizes = [4096] * 65536 + [65536] * 4096 + [1 << 20] * 256 + [4 << 20] * 64
    np.random.default_rng(42).shuffle(sizes)
    sizes = np.asarray(sizes, dtype=np.int64)
elif cfg == "c2-1g":
    sizes = np.full(262144, 4096, dtype=np.int64)
elif cfg == "c2-odd":  # bench.py's c2-odd: 4,100-byte buffers back to back (unaligned starts and ends)
    sizes = np.full(65536, 4100, dtype=np.int64)
else:
    sizes = np.full(65536, 4096, dtype=np.int64)
offs = np.concatenate([[0], np.cumsum(sizes)[:-1]])
buf = torch.randint(0, 256, (int(sizes.sum()),), dtype=torch.uint8, device=dev)
descs = P.make_descs(buf.data_ptr() + offs, sizes, device=dev)
out = torch.zeros(len(sizes), dtype=torch.int32, device=dev)
for _ in range(3):
    P.dev_batch_async(descs, out)
torch.cuda.synchronize()
P.timing(True)  # the main kernel's packet-level duration (HIP events) for the same launch
P.timing_read()
P.dev_batch_async(descs, out)
torch.cuda.synchronize()
P.timing_read()
event_us = float(np.asarray(P.timing_samples())[-1]) * 1e3
P.timing(False)
L = _lib.lib()
L.pech_read_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
W = 4096
NS = 12
st = np.zeros(NS * W, dtype=np.uint64)
assert L.pech_read_stamps(st.ctypes.data, W) == 0
s, e, tag, ent, tscan, tfind, tplan, tfill, q1, q2, q3, tiss = (st[k::NS].astype(np.int64) for k in range(NS))
ok = (s > 0) & (e > 0)
s, e, tag, ent = s[ok], e[ok], tag[ok], ent[ok]
tscan, tfind, tplan, tfill, tiss = tscan[ok], tfind[ok], tplan[ok], tfill[ok], tiss[ok]
q1, q2, q3 = q1[ok], q2[ok], q3[ok]
xcc, blk = tag & 0xF, tag >> 8
# s_memrealtime: 100 MHz chip-wide clock (10 ns ticks)
t0 = ent.min()
s -= t0; e -= t0; ent -= t0; tscan -= t0; tfind -= t0; tplan -= t0; tfill -= t0; tiss -= t0
q1 -= t0; q2 -= t0; q3 -= t0
pro = s - ent
span = e.max()
pct = lambda a, q: float(np.percentile(a, q))
print(f"{cfg}: waves {ok.sum()}, span {span*10/1000:.1f} us (entry of the first wave to end of the last); "
      f"main-kernel event duration {event_us:.1f} us")
print("entry us p50/p99/max: %.1f %.1f %.1f" % (pct(ent,50)/100, pct(ent,99)/100, ent.max()/100))
print("prologue (entry->first row) us p10/p50/p90/max: %.1f %.1f %.1f %.1f" % (pct(pro,10)/100, pct(pro,50)/100, pct(pro,90)/100, pro.max()/100))
for nm, a, b in (("entry->issued", ent, tiss), ("issued->scan", tiss, tscan), ("scan->find", tscan, tfind), ("find->plan", tfind, tplan),
                 ("plan->fill", tplan, tfill), ("fill->start(barrier)", tfill, s)):
    d = b - a
    print("  %-22s us p10/p50/p90: %.2f %.2f %.2f" % (nm, pct(d, 10) / 100, pct(d, 50) / 100, pct(d, 90) / 100))
print("start us p50/p99/max: %.1f %.1f %.1f" % (pct(s,50)/100, pct(s,99)/100, s.max()/100))
print("end   us p1/p10/p50/p90/max: %.1f %.1f %.1f %.1f %.1f" % (pct(e,1)/100, pct(e,10)/100, pct(e,50)/100, pct(e,90)/100, e.max()/100))
print("mean wave busy / span: %.3f" % float(((e - s) / span).mean()))
busy = (e - s) / 100
print("busy us p1/p10/p50/p90/p99/max: %.1f %.1f %.1f %.1f %.1f %.1f" % (pct(busy, 1), pct(busy, 10), pct(busy, 50),
                                                                        pct(busy, 90), pct(busy, 99), busy.max()))
if os.environ.get("PECH_STAMP_FIN") == "1":  # stamps built with -DPECH_STAMP_FIN: q3/q2 bracket the last finish_run
    fin, flush = (q2 - q3) / 100, (e - q2) / 100
    print("last step's fold+shift us p10/p50/p90/max: %.2f %.2f %.2f %.2f" % (pct(fin, 10), pct(fin, 50), pct(fin, 90), fin.max()))
    print("after it (deferral flush) us p50/p90/max: %.2f %.2f %.2f" % (pct(flush, 50), pct(flush, 90), flush.max()))
    print("start->last fold us p10/p50/p90/max: %.1f %.1f %.1f %.1f" % tuple(x / 100 for x in (pct(q3 - s, 10), pct(q3 - s, 50), pct(q3 - s, 90), (q3 - s).max())))
    plan = (q1 + t0) / 100  # (a sum of durations, not a time stamp: undo the shift)
    print("steps planned in the loop, us per wave p10/p50/p90/max: %.2f %.2f %.2f %.2f" % (pct(plan, 10), pct(plan, 50), pct(plan, 90), plan.max()))
hist, edges = np.histogram(e / 100, bins=12)
print("end-time histogram (us):", [(round(float(edges[i]),1), int(hist[i])) for i in range(len(hist))])

print("workgroups on XCC blockIdx %% 8: %.3f" % float(((blk % 8) == xcc).mean()))
for x in range(8):
    m = xcc == x
    print(f"xcc{x}: waves {int(m.sum())} end p10 {pct(e[m],10)/100:.1f} p50 {pct(e[m],50)/100:.1f} max {e[m].max()/100:.1f} us")
# within-CU spread: per block, max-min of end
per = {}
for b, t in zip(blk, e):
    per.setdefault(int(b), []).append(int(t))
spread = np.array([max(v) - min(v) for v in per.values()]) / 100
bmax = np.array([max(v) for v in per.values()]) / 100
print("per-CU end spread us p50/p90/max: %.1f %.1f %.1f" % (pct(spread,50), pct(spread,90), spread.max()))
print("per-CU last-wave end us p10/p50/p90: %.1f %.1f %.1f" % (pct(bmax,10), pct(bmax,50), pct(bmax,90)))

# by wave slot inside the workgroup (wid % waves-per-WG): systematic arbitration bias?
wpg = int(os.environ.get("PECH_WAVES", "16"))
wid = np.nonzero(ok)[0]
slot = wid % wpg
print("end p50 by wave slot (us):", [round(pct(e[slot == k], 50) / 100, 1) for k in range(wpg)])
print("busy p50 by wave slot (us):", [round(pct((e - s)[slot == k], 50) / 100, 1) for k in range(wpg)])
# bytes-over-time profile: each wave's rows are piecewise linear between its
# start, 25/50/75% stamps (first step; c3 waves have one) and end
if cfg == "c3" and (q1 > 0).all():
    per_wave = int(sizes.sum()) / len(s)
    bins = np.arange(0, int(e.max()) + 500, 500)  # 5 us
    prog = np.zeros(len(bins))
    for k, (a, b) in enumerate(((s, q1), (q1, q2), (q2, q3), (q3, e))):
        for i in range(len(s)):
            lo, hi = a[i], b[i]
            if hi <= lo:
                continue
            ov = np.clip(np.minimum(bins[1:], hi) - np.maximum(bins[:-1], lo), 0, None)
            prog[:-1] += ov / (hi - lo) * per_wave / 4
    rate = prog[:-1] / 5e-6 / 1e9
    print("HBM read rate by 5 us bin (GB/s):", [int(x) for x in rate])
# C4: each wave's size class (host replica of the plan kernel's order: chunks of
# 1,024 buffers, stably sorted by class, smallest first; static shares of the
# row space as wave_share's proportional split) -> busy / end by class
if cfg == "c4":
    G = 256
    rows = (sizes // 128).astype(np.int64)  # (aligned: whole lines)
    order = []
    for c0 in range(0, len(rows), 1024):
        ch = np.arange(c0, min(c0 + 1024, len(rows)))
        order.append(ch[np.argsort(np.minimum(rows[ch], 2048), kind="stable")])  # class cap PECH_LARGE_ROWS
    order = np.concatenate(order)
    rcum = np.concatenate([[0], np.cumsum(rows[order])])
    Rtot = int(rcum[-1])
    cls_of = {32: "4k", 512: "64k", 8192: "1m", 32768: "4m"}
    lab = []
    for w in wid:
        b, wv = divmod(int(w), wpg)
        wg0 = b * Rtot // G
        wgr = (b + 1) * Rtot // G - wg0
        r0, r1 = wg0 + wgr * wv // wpg, wg0 + wgr * (wv + 1) // wpg
        i0 = np.searchsorted(rcum, r0, side="right") - 1
        i1 = np.searchsorted(rcum, r1 - 1, side="right") - 1
        got = {}
        for i in range(i0, i1 + 1):
            ov = min(r1, rcum[i + 1]) - max(r0, rcum[i])
            k = cls_of.get(int(rows[order[i]]), "?")
            got[k] = got.get(k, 0) + ov
        lab.append(max(got, key=got.get))
    lab = np.asarray(lab)
    for k in ("4k", "64k", "1m", "4m"):
        m = lab == k
        if m.any():
            print(f"class {k}: waves {int(m.sum())} busy p50 {pct(busy[m], 50):.1f} p90 {pct(busy[m], 90):.1f} "
                  f"end p50 {pct(e[m], 50) / 100:.1f} p90 {pct(e[m], 90) / 100:.1f} max {e[m].max() / 100:.1f} us")
    # per workgroup: its last wave's end against its share of small-class rows
    wgl = {}
    for w, t, k in zip(wid, e, lab):
        d = wgl.setdefault(int(w) // wpg, [0, 0])
        d[0] = max(d[0], int(t))
        d[1] += k in ("4k", "64k")
    arr = np.array(list(wgl.values()))
    for lo, hi in ((0, 0), (1, 8), (9, 15), (16, 16)):
        m = (arr[:, 1] >= lo) & (arr[:, 1] <= hi)
        if m.any():
            print(f"workgroups with {lo}-{hi} small-class waves: {int(m.sum())}, last end p50 {pct(arr[m, 0], 50) / 100:.1f} "
                  f"max {arr[m, 0].max() / 100:.1f} us")
out_dir = os.path.join(REPO, "gpurun_out")
os.makedirs(out_dir, exist_ok=True)
np.savez(os.path.join(out_dir, f"stamps_{cfg}.npz"), start=s, end=e, entry=ent, tag=tag, wid=wid, q1=q1, q2=q2, q3=q3,
         tplan=tplan, tfill=tfill, tfind=tfind)
