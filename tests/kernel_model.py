"""Host-side shadow model of the work decomposition of
pech_amd/csrc/crc32c_kernels.hip (plan + main kernels), statement by
statement, used by tests/test_kernel_model.py to check -- on the CPU, before a
kernel ever runs on a GPU -- that

  * every 16-byte load the main kernel issues lies inside the lines holding
    the buffer it is working on, from its first (aligned) piece on (no read
    before/after a buffer: a GPU fault),
  * the first row's bytes before the buffer are zeroed (whole pieces, and
    the head's first addr%16 bytes),
  * every core row of every buffer is consumed by exactly one lane-group,
  * every run's final shift targets the right buffer end.

Keep in sync with the kernel: constants come from layout.h by parsing.
"""
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _consts():
    src = open(os.path.join(REPO, "pech_amd", "csrc", "layout.h")).read()
    out = {}
    for m in re.finditer(r"#define (PECH_\w+) (\d+)u", src):
        out[m.group(1)] = int(m.group(2))
    ksrc = open(os.path.join(REPO, "pech_amd", "csrc", "crc32c_kernels.hip")).read()
    out["PECH_U"] = int(re.search(r"#define PECH_U (\d+)", ksrc).group(1))
    out["PECH_U_COPY"] = int(re.search(r"#define PECH_U_COPY (\d+)", ksrc).group(1))
    out["PECH_MAIN_WAVES"] = int(re.search(r"#define PECH_MAIN_WAVES (\d+)", ksrc).group(1))
    out["PECH_SPLIT_MIN"] = int(re.search(r"#define PECH_SPLIT_MIN (\d+)u", ksrc).group(1))
    out["PECH_DEAL_BLOCKS"] = int(re.search(r"#define PECH_DEAL_BLOCKS (\d+)u", ksrc).group(1))
    out["PECH_SLOT_W"] = [1, 1, 1, 1]  # the kernel splits a workgroup's rows equally over its waves
    return out


C = _consts()
ROW = C["PECH_ROW_BYTES"]
CHUNK = C["PECH_CHUNK"]
SPLIT = C["PECH_SPLIT_ROWS"]
SPLIT_MIN = C["PECH_SPLIT_MIN"]
DEAL_BLOCKS = C["PECH_DEAL_BLOCKS"]
LARGE = C["PECH_LARGE_ROWS"]
WAVES_PER_WG = C["PECH_MAIN_WAVES"]
ITEM = C["PECH_ITEM_ROWS"]
POOL = C.get("PECH_POOL_ROWS", 0xFFFFFFFF)
POOL_MIN = C.get("PECH_POOL_MIN_SHARE", 0)


def share_head(a, b, item=None, pool=None):
    """kernel share_head: end of the head of share [a, b) its owner walks first"""
    item, pool = item or ITEM, pool or POOL
    return min(b, max(a + item, b - min(pool, b - a)))
NZ_UNIFORM = 0x80000000
NZ_MASK = 0x7FF            # nzs[c] bits 0-10: non-empty cores of chunk c
NS_SHIFT = 11              # bits 11-21: of them, small ones (< PECH_SPLIT_ROWS rows), sorted first


def core_rows(addr, ln):
    """rows (128-byte lines) holding the core [addr, align16_down(addr + len))
    (layout.h pech_core_rows, v0.16: the head is part of the core, masked)"""
    ce = (addr + ln) & ~15
    if ce <= addr:
        return 0
    return ((addr & 127) + (ce - addr) + 127) >> 7


def encode_m(ra, zt, tail):
    """kernel mp_bits / ra_bit: (Step.mp, Step.oz bit) of a run with `ra` rows
    of its buffer after it, in 32-bit words"""
    return ((ra << 7) | (zt << 4) | tail) & 0xFFFFFFFF, ((ra >> 25) & 1) << 29


def decode_m(mp, oz):
    """kernel STEP_M: bytes from the run's end to the buffer's end"""
    ra = (mp >> 7) | ((oz & (1 << 29)) >> 4)
    return ra * ROW + (mp & 15) - (mp & 0x70)


def size_class(rows):
    if rows >= LARGE:
        return 12
    c = 0
    while (2 << c) <= rows:
        c += 1
    return c


def plan(descs, rng=None):
    """descs: list of (addr, len).  Returns per-slot cores, lrs, partials,
    nzs.  Without `rng`, the plan kernel's order (stable by class, 16-blocks
    interleaved below the split size); with `rng`, an arbitrary order inside
    each class (the main kernel must not depend on it)."""
    n = len(descs)
    nch = (n + CHUNK - 1) // CHUNK
    cores = [None] * (nch * CHUNK)
    lrs = [0] * (nch * CHUNK)
    partials, nzs = [], []
    for c in range(nch):
        items = []
        for b in range(c * CHUNK, min(n, (c + 1) * CHUNK)):
            addr, ln = descs[b]
            rows = core_rows(addr, ln)
            if rows == 0:
                continue
            ce = (addr + ln) & ~15
            vbase = addr & ~127  # rows on the line grid
            lb = addr - vbase    # leading bytes of row 0 before the buffer
            vp, zh = lb >> 4, lb & 15
            zt = rows * 8 - ((ce - vbase) >> 4)
            t = addr + ln - ce
            items.append(dict(vbase=vbase, rows=rows, orig=b, vp=vp, zh=zh, zt=zt, tail=t, addr=addr, ce=ce,
                              a0=vbase + 16 * vp, cls=size_class(rows)))
        order = []
        for cls in range(13):
            group = [it for it in items if it["cls"] == cls]
            if rng is not None:
                rng.shuffle(group)
            elif group and group[0]["rows"] < SPLIT:
                # the plan kernel's order: stable inside the class, and inside
                # every full block of 16 ranks 0,2,..,14 then 1,3,..,15
                g2 = list(group)
                for k in range(0, len(group) - 15, 16):
                    blk = group[k:k + 16]
                    g2[k:k + 16] = blk[0::2] + blk[1::2]
                group = g2
            order += group
        acc = 0
        for pos in range(CHUNK):
            lrs[c * CHUNK + pos] = acc
            if pos < len(order):
                cores[c * CHUNK + pos] = order[pos]
                acc += order[pos]["rows"]
        partials.append(acc)
        # uniform chunk (plan kernel): every buffer has a core, all of the
        # largest one's rows -> flag bit in nzs
        cnt = min(n, (c + 1) * CHUNK) - c * CHUNK
        rmax = max((it["rows"] for it in order), default=0)
        uni = len(order) == cnt and len(order) * rmax == acc and acc != 0
        nsmall = sum(1 for it in order if it["rows"] < SPLIT)
        assert all(it["rows"] < SPLIT for it in order[:nsmall])  # the small ones come first
        nzs.append(len(order) | (nsmall << NS_SHIFT) | (NZ_UNIFORM if uni else 0))
    return cores, lrs, partials, nzs


def run_rows_loads(U, nl, nu, zoff, T, nmin):
    """Row indices (and whether the zoff redirect applies) loaded by one
    lane for one step, in issue order, and the rows it consumes (r < nu).

    Ring discipline of the kernel: row k lives in slot k % U; priming loads
    rows 0..U-2; the iteration consuming row k first loads row k+U-1 into
    slot (k-1) % U.  The last block's iterations 1..U-1 load the NEXT step's
    rows 0..U-2 (modelled as that step's priming).  Slot contents are
    simulated and every consumed row is checked to be the row in its slot."""
    last = nl - 1
    loads = []
    slots = {}

    def load(row, clamp, zo):
        r = min(row, last) if clamp else row
        loads.append((r, zo and r == 0 and zoff != 0))
        slots[row % U] = (row, r)

    for i in range(U - 1):
        load(i, True, True)
    nblk = (T + U - 1) // U
    consumed = []

    def consume(k):
        want, got = slots[k % U]
        assert want == k, ("ring slot holds row", want, "consuming", k)
        if k < nu:
            assert got == k, ("consumed row was clamped", k, got)
            consumed.append(k)

    blk = 0
    while blk + 1 < nblk and (blk + 2) * U <= nmin:
        for i in range(U):
            load(blk * U + i + U - 1, False, False)
            consume(blk * U + i)
        blk += 1
    while blk + 1 < nblk:
        r = blk * U
        for i in range(U):
            load(r + i + U - 1, True, True)
            consume(r + i)
        blk += 1
    r = blk * U
    load(r + U - 1, True, True)
    consume(r)
    for i in range(1, U):
        slots[(i - 1) % U] = ("next step row", i - 1)  # overwritten by the next step's priming
        consume(r + i)
    return loads, consumed


def find_start(lrs, pref, nzs, r):
    """find_start_wave: chunk by binary search of the prefix, then the count
    of the chunk's row offsets <= the chunk-local row (one wave-wide read of
    all PECH_CHUNK offsets, entries past nz excluded)."""
    nzs = [z & NZ_MASK for z in nzs]
    nchunks = len(nzs)
    clo, chi = 0, nchunks
    while chi - clo > 1:
        mid = (clo + chi) >> 1
        if pref[mid] <= r:
            clo = mid
        else:
            chi = mid
    rr = r - pref[clo]
    ok = [lrs[clo * CHUNK + i] for i in range(CHUNK) if i < nzs[clo] and lrs[clo * CHUNK + i] <= rr]
    assert ok, "row offset 0 always qualifies"
    return clo * CHUNK + len(ok) - 1, rr - max(ok)


def slot_cw(k, weights):
    """Cumulative share weight of workgroup waves 0..k-1 (kernel slot_cw)."""
    return sum(weights[g] * min(4, max(0, k - 4 * g)) for g in range(4))


def wave_ranges(Rtot, ncu, rpw_min=None, weights=None, waves=None, il=False, by_wg=False):
    """Kernel wave_share: [r0, r1) of every wave, workgroup by workgroup.
    Large launches (Rtot >= W * rpw): proportional workgroup ranges, equal
    contiguous pieces inside (by age-rank weight in the model's A/B
    variants).  Small ones: shares of rpw rows -- rpw from rpw_min up to 4
    rpw_min, aiming at four live waves per CU -- dealt over Gd = min(ncu,
    ceil(shares / 4)) workgroups, in blocks of 4 S shares (a workgroup's live
    shares S apart) when Gd is a multiple of S, else wave-major (k = wave *
    Gd + workgroup), except in the fused copy's interleaved mode,
    which walks each workgroup's contiguous range.  by_wg: a list per live
    workgroup, and whether the launch is proportional."""
    rpw_min = rpw_min or C["PECH_RPW_MIN"]
    weights = weights or C["PECH_SLOT_W"]
    waves = waves or WAVES_PER_WG
    W = ncu * waves
    G4 = 4 * ncu
    rpw = min(max((Rtot + G4 - 1) // G4, rpw_min), 4 * rpw_min)
    prop = Rtot >= W * rpw
    tot = slot_cw(waves, weights)
    out = []
    for b in range(ncu):
        if not prop and not il:
            nsh = (Rtot + rpw - 1) // rpw
            Gd = min(ncu, (nsh + 3) // 4)  # just enough workgroups for four live waves each
            S = DEAL_BLOCKS
            blocks = S and Gd % S == 0
            first = (b // S) * 4 * S + b % S if blocks else b
            if b >= Gd or first * rpw >= Rtot:
                continue
            ks = [(b // S) * 4 * S + b % S + S * w if blocks and w < 4 else w * Gd + b for w in range(waves)]
            out.append([(min(k * rpw, Rtot), min(k * rpw + rpw, Rtot)) for k in ks])
            continue
        wg0 = b * Rtot // ncu if prop else b * waves * rpw
        if wg0 >= Rtot:
            continue
        wg_rows = (b + 1) * Rtot // ncu - wg0 if prop else min(waves * rpw, Rtot - wg0)
        out.append([(wg0 + wg_rows * slot_cw(w, weights) // tot, wg0 + wg_rows * slot_cw(w + 1, weights) // tot)
                     for w in range(waves)])
    if by_wg:
        return out, prop
    return [r for wg in out for r in wg]


IL = C["PECH_IL_GROUPS"]
IL_MIN = C["PECH_IL_MIN_ROWS"]


def walk_il(cores, pos, lr, rem, U, events):
    """Fused copy, interleaved rows (kernel plan_il): the workgroup's 128 lane
    groups walk each portion [lr, lr + P) of a buffer together, group j taking
    rows lr + j, lr + j + 128, ..."""
    guard = 0
    while rem:
        guard += 1
        assert guard < 10 ** 6
        cd = cores[pos]
        rows0 = cd["rows"]
        P = min(rows0 - lr, rem)
        for wave in range(WAVES_PER_WG):
            j0 = 8 * wave
            counts = [(P - j0 - g + IL - 1) // IL if P > j0 + g else 0 for g in range(8)]
            T = counts[0]
            nmin = min([c for c in counts if c] or [0])
            for grp in range(8):
                j, nn = j0 + grp, counts[grp]
                st = lr + j
                last = st + IL * (nn - 1)
                for g8 in range(8):
                    if nn:
                        zoff = 16 * (cd["vp"] - g8) if (st == 0 and g8 < cd["vp"]) else 0
                        loads, used = run_rows_loads(U, nn, nn, zoff, T, nmin)
                        for row, z in loads:
                            events.append(("load", cd, cd["vbase"] + (st + IL * row) * ROW + 16 * g8 + (zoff if z else 0)))
                        zl = last == rows0 - 1 and g8 >= 8 - cd["zt"]
                        zh = cd["zh"] if (st == 0 and g8 == cd["vp"]) else 0
                        for row in used:
                            events.append(("use", cd["orig"], st + IL * row, g8,
                                           (zoff != 0 and row == 0) or (zl and row == nn - 1), zh if row == 0 else 0))
                    else:  # idle group: the portion's first row, state ignored
                        zoff = 16 * (cd["vp"] - g8) if (lr == 0 and g8 < cd["vp"]) else 0
                        loads, _ = run_rows_loads(U, 1, 0, zoff, T, nmin)
                        for row, z in loads:
                            events.append(("load", cd, cd["vbase"] + (lr + IL * row) * ROW + 16 * g8 + (zoff if z else 0)))
                if nn:
                    events.append(("finish", cd["orig"], last + 1, (rows0 - last - 1) * ROW + cd["tail"] - 16 * cd["zt"]))
        rem -= P
        if lr + P == rows0:
            pos += 1
            lr = 0
        else:
            lr += P


def main(cores, lrs, partials, nzs, ncu, rpw_min=None, U=None, weights=None, copy=False):
    """Yield events: ("load", buf, lane_piece_addr), ("use", orig, row, g8,
    virtual) and ("finish", orig, run_end_row, m) over every wave's range."""
    U = U or C["PECH_U"]
    pref = [0]
    for p in partials:
        pref.append(pref[-1] + p)
    Rtot = pref[-1]
    events = []
    # uniform batch (kernel prologue): every chunk flagged, all with chunk 0's
    # rows per buffer -> items of ITEM rows: each wave's share's first item by
    # its owner, the rest from the workgroup pool (claim c: item 1 + c//16 of
    # share c%16; which wave takes a claim does not matter for coverage)
    nz = [z & NZ_MASK for z in nzs]
    U0 = partials[0] // nz[0] if nz and nz[0] else 0
    uniform = bool(U0) and all((z & NZ_UNIFORM) and n * U0 == p for z, n, p in zip(nzs, nz, partials))
    il = copy and uniform and U0 >= IL_MIN
    wgs, prop = wave_ranges(Rtot, ncu, rpw_min, weights, il=il, by_wg=True)
    if il:  # fused copy: interleaved rows over each workgroup's range
        for shares in wgs:
            wg0, wg_rows = shares[0][0], shares[-1][1] - shares[0][0]
            if wg_rows:
                walk_il(cores, wg0 // U0, wg0 % U0, wg_rows, U, events)
        return events
    for shares in wgs:
        wg_rows = shares[-1][1] - shares[0][0]
        # (shares below POOL_MIN rows keep static shares; wave-major small
        # launches never pool)
        jmax = (1 + (min(POOL, (wg_rows + WAVES_PER_WG - 1) // WAVES_PER_WG) + ITEM - 1) // ITEM
                if prop and uniform and wg_rows >= WAVES_PER_WG * POOL_MIN else 0)
        for r0, r1 in shares:
            if r1 > r0:
                pos, lr = find_start(lrs, pref, nzs, r0)
                if jmax:
                    walk(cores, nzs, pos, lr, share_head(r0, r1) - r0, U, events)
                else:
                    pos, lr, rem = snap_to_grid(lrs, pref, nzs, pos, lr, r0, r1)
                    if rem:
                        walk(cores, nzs, pos, lr, rem, U, events, grid=True)
        if jmax > 1:
            for c in range(WAVES_PER_WG * (jmax - 1)):
                j, sh = 1 + c // WAVES_PER_WG, c % WAVES_PER_WG
                a, b = shares[sh]
                st = share_head(a, b) + (j - 1) * ITEM
                if st < b:
                    pos, lr = st // U0, st % U0
                    assert (pos, lr) == find_start(lrs, pref, nzs, st), (st, pos, lr)
                    walk(cores, nzs, pos, lr, min(ITEM, b - st), U, events)
    return events


def snap_to_grid(lrs, pref, nzs, pos, lr, r0, r1):
    """Kernel prologue, non-uniform batches: small buffers (< PECH_SPLIT_ROWS
    rows, the first nsmall positions of a chunk) are walked in whole steps of
    8 positions on a grid from the chunk start; a step belongs to the wave
    whose share holds its middle row (the first row of its position
    cnt/2).  A wave starting inside a small step k walks it if it owns it
    (from the step's start, before r0), else starts at the next grid point."""
    c, local = pos >> 10, pos & 1023
    nz, ns = nzs[c] & NZ_MASK, (nzs[c] >> NS_SHIFT) & NZ_MASK

    def roff(l):
        return pref[c] + (lrs[c * CHUNK + l] if l < nz else pref[c + 1] - pref[c])
    if local < ns:
        k0 = local & ~7
        cnt = min(8, ns - k0)
        start = k0 if roff(k0 + cnt // 2) >= r0 else min(ns, k0 + 8)
        pos = c * CHUNK + start if start < nz else (c + 1) * CHUNK
        return pos, 0, max(0, r1 - roff(start))
    return pos, lr, r1 - r0


def walk(cores, nzs, pos, lr, rem, U, events, grid=False):
    """plan_step + run of one sub-range (pos, lr, rem).  grid: a step of
    small buffers that starts inside the range is walked whole."""
    nzs = [z & NZ_MASK for z in nzs]
    if True:
        guard = 0
        while rem:
            guard += 1
            assert guard < 10 ** 6, "wave loop does not terminate"
            c = pos >> 10
            if (pos & 1023) >= nzs[c]:
                pos = (c + 1) << 10
                continue
            cd = cores[pos]
            rows0 = cd["rows"]
            avail0 = rows0 - lr
            assert avail0 > 0
            # a large buffer (or what is left of it) goes to 8 slices when at
            # least SPLIT_MIN (8) of its rows are to be walked: a remainder
            # walked by group 0 alone left 7 groups idle
            if rows0 >= SPLIT and min(avail0, rem) >= SPLIT_MIN:
                P = min(avail0, rem)
                q, rm = P >> 3, P & 7
                T = q + (1 if rm else 0)
                for grp in range(8):
                    st = lr + grp * q + min(grp, rm)
                    nn = q + (1 if grp < rm else 0)
                    for g8 in range(8):
                        zoff = 16 * (cd["vp"] - g8) if (st == 0 and g8 < cd["vp"]) else 0
                        loads, used = run_rows_loads(U, nn, nn, zoff, T, q)
                        for row, z in loads:
                            events.append(("load", cd, cd["vbase"] + (st + row) * ROW + 16 * g8 + (zoff if z else 0)))
                        zl = st + nn == rows0 and g8 >= 8 - cd["zt"]
                        zh = cd["zh"] if (st == 0 and g8 == cd["vp"]) else 0
                        for row in used:
                            events.append(("use", cd["orig"], st + row, g8,
                                           (zoff != 0 and row == 0) or (zl and row == nn - 1), zh if row == 0 else 0))
                    events.append(("finish", cd["orig"], st + nn,
                                   (rows0 - st - nn) * ROW + cd["tail"] - 16 * cd["zt"]))
                rem -= P
                if P == avail0:
                    pos += 1
                    lr = 0
                else:
                    lr += P
            else:
                nzc = nzs[c]
                mys, cut = [], []
                for grp in range(8):
                    myp = pos + grp
                    inchunk = (myp & 1023) < nzc and (myp >> 10) == c
                    my = cores[myp] if (grp and inchunk) else cd
                    myrows = my["rows"] if inchunk else 0
                    cut.append(grp > 0 and (not inchunk or myrows >= SPLIT))
                    mys.append((my, myrows))
                kcut = next((g for g in range(8) if cut[g]), 8)
                avails = [(mys[g][1] - (lr if g == 0 else 0)) if g < kcut else 0 for g in range(8)]
                pres = [sum(avails[:g]) for g in range(8)]
                whole = grid and rows0 < SPLIT
                if whole:  # a grid step of small buffers whose middle lies in the range: all of it
                    assert lr == 0 and (pos & 7) == 0, (pos, lr)
                    nus = list(avails) if pres[kcut // 2] < rem else [0] * 8
                else:
                    nus = [0 if pres[g] >= rem else min(avails[g], rem - pres[g]) for g in range(8)]
                if whole and not any(nus):
                    break  # the step is the next wave's: this range is done (kernel: S.T == 0)
                T = max(nus)
                nmin = min(x for x in nus if x) if any(nus) else 0xFFFFFFFF
                used_rows = sum(nus) if whole else min(pres[7] + avails[7], rem)
                assert used_rows == sum(nus)
                n0 = min(avail0, rem)
                for grp in range(8):
                    my, myrows = mys[grp]
                    nu = nus[grp]
                    mylr = 0 if grp else lr
                    for g8 in range(8):
                        if nu:
                            zoff = 16 * (my["vp"] - g8) if (mylr == 0 and g8 < my["vp"]) else 0
                            base, buf, nl = my["vbase"] + mylr * ROW + 16 * g8, my, nu
                        else:
                            zoff = 16 * (cd["vp"] - g8) if (lr == 0 and g8 < cd["vp"]) else 0
                            base, buf, nl = cd["vbase"] + lr * ROW + 16 * g8, cd, n0
                        loads, used = run_rows_loads(U, nl, nu, zoff, T, nmin)
                        for row, z in loads:
                            events.append(("load", buf, base + row * ROW + (zoff if z else 0)))
                        zl = nu != 0 and mylr + nu == myrows and g8 >= 8 - my["zt"]
                        zh = my["zh"] if (mylr == 0 and g8 == my["vp"]) else 0
                        for row in used:
                            events.append(("use", my["orig"], mylr + row, g8,
                                           (zoff != 0 and row == 0) or (zl and row == nu - 1), zh if row == 0 else 0))
                    if nu:
                        events.append(("finish", my["orig"], mylr + nu,
                                       (myrows - mylr - nu) * ROW + my["tail"] - 16 * my["zt"]))
                rem = 0 if whole and not used_rows else rem - min(used_rows, rem)
                if rem:
                    pos += kcut
                    lr = 0
    return events


def direct_positions(n, ncu, waves=None):
    """The direct kernel's schedule (v0.21, workgroup-interleaved): workgroup
    b owns positions [b n / ncu, (b+1) n / ncu); step k of its wave w takes
    positions wb + 128 k + 8 w + g (g < 8, below the range end), one per
    lane group.  Yields (workgroup, wave, step, group, position)."""
    waves = waves or WAVES_PER_WG
    for b in range(ncu):
        wb, we = b * n // ncu, (b + 1) * n // ncu
        for w in range(waves):
            k = 0
            while True:
                e0 = min(wb + 128 * k + 8 * w + 8, we)
                p = min(wb + 128 * k + 8 * w, e0)
                if p >= e0:  # the kernel's S.T == 0: no later step has positions either
                    assert wb + 128 * (k + 1) + 8 * w >= we
                    break
                for g in range(min(8, e0 - p)):
                    yield b, w, k, g, p + g
                k += 1
