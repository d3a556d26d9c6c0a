"""Per-class wave busy times of a C4 stamps run (gpurun_out/stamps_c4.npz from tools/wave_stamps.py c4): maps every wave's row share onto the plan's buffer order (tests/kernel_model.py) and reports busy time by the size class it walked."""
import sys, numpy as np
sys.path.insert(0, 'tests')
import kernel_model as KM
d = np.load('gpurun_out/stamps_c4.npz')
s, e, wid = d['start'], d['end'], d['wid']
busy = (e - s) / 100.0
sizes = [4096] * 65536 + [65536] * 4096 + [1 << 20] * 256 + [4 << 20] * 64
np.random.default_rng(42).shuffle(sizes)
# torch buffers are 256-aligned; back-to-back offsets (bench layout)
offs = np.concatenate([[0], np.cumsum(sizes)[:-1]])
base = 1 << 30
descs = [(base + int(o), int(l)) for o, l in zip(offs, sizes)]
cores, lrs, partials, nzs = KM.plan(descs)
pref = np.concatenate([[0], np.cumsum(partials)])
Rtot = int(pref[-1])
ranges = KM.wave_ranges(Rtot, 256)
# map each row range to the classes it touches (rows per class)
rows_of = []
for c in range(len(partials)):
    for k in range(nzs[c]):
        cd = cores[c * 1024 + k]
        rows_of.append((int(pref[c] + lrs[c * 1024 + k]), cd['rows'], sizes[cd['orig']]))
starts = np.array([r[0] for r in rows_of]); rws = np.array([r[1] for r in rows_of]); szs = np.array([r[2] for r in rows_of])
cls_names = {4096: '4K', 65536: '64K', 1 << 20: '1M', 4 << 20: '4M'}
frac = {k: np.zeros(len(ranges)) for k in cls_names}
nbuf = np.zeros(len(ranges))
for w, (r0, r1) in enumerate(ranges):
    i0 = np.searchsorted(starts, r0, side='right') - 1
    i1 = np.searchsorted(starts, r1, side='left')
    for i in range(max(i0, 0), i1):
        a, b = max(r0, starts[i]), min(r1, starts[i] + rws[i])
        if b > a:
            frac[szs[i]][w] += (b - a) / (r1 - r0)
            nbuf[w] += 1
order = np.argsort(wid)
b = np.zeros(len(ranges)); b[wid] = busy
dom = np.array([max(cls_names, key=lambda k: frac[k][w]) for w in range(len(ranges))])
for k, nm in cls_names.items():
    m = dom == k
    print(nm, 'waves', int(m.sum()), 'busy p50 %.1f p90 %.1f max %.1f' % (np.percentile(b[m], 50), np.percentile(b[m], 90), b[m].max()), 'bufs/wave p50', np.percentile(nbuf[m], 50))
slot = np.arange(len(ranges)) % 16
for sl in (0, 15):
    print('slot', sl, {cls_names[k]: round(float(np.median(b[(dom == k) & (slot == sl)])), 1) for k in cls_names if ((dom == k) & (slot == sl)).any()})
