"""CPU checks of the main kernel's work decomposition through the shadow
model (tests/kernel_model.py): loads stay inside the lines holding each
buffer's core (never before its first piece), every row piece is consumed
exactly once, the pieces and head bytes outside the core count as zeros,
and shifts target the buffer end."""
import collections
import random

import pytest

import kernel_model as KM


def check(descs, ncu=4, seed=0, weights=None, U=None, copy=False):
    rng = random.Random(seed)
    cores, lrs, partials, nzs = KM.plan(descs, rng)
    ev = KM.main(cores, lrs, partials, nzs, ncu, weights=weights, U=U, copy=copy)
    used = collections.Counter()
    byorig = {}
    for c in cores:
        if c is not None:
            byorig[c["orig"]] = c
    for e in ev:
        if e[0] == "load":
            _, buf, a = e
            # from the aligned piece holding the buffer's first byte; past ce
            # only inside the core's last line (trailing virtual pieces)
            assert buf["a0"] <= a and a + 16 <= buf["vbase"] + buf["rows"] * KM.ROW, (buf, a)
            assert a % KM.ROW // 16 == (a - buf["vbase"]) % KM.ROW // 16  # rows on the line grid
        elif e[0] == "use":
            _, orig, row, g8, virt, zh = e
            c = byorig[orig]
            used[(orig, row, g8)] += 1
            piece = row * 8 + g8
            assert virt == (piece < c["vp"] or piece >= c["rows"] * 8 - c["zt"]), (orig, row, g8)
            # bytes of the piece before the buffer's first byte, zeroed in place
            assert zh == (c["addr"] - c["a0"] if piece == c["vp"] else 0), (orig, row, g8, zh)
        elif e[0] == "finish":
            _, orig, endrow, m = e
            c = byorig[orig]
            assert m == (c["rows"] - endrow) * KM.ROW + c["tail"] - 16 * c["zt"]
            assert KM.decode_m(*KM.encode_m(c["rows"] - endrow, c["zt"], c["tail"])) == m  # the kernel's packing
    for orig, c in byorig.items():
        for row in range(c["rows"]):
            for g8 in range(8):
                assert used[(orig, row, g8)] == 1, (orig, row, g8, used[(orig, row, g8)])
    assert sum(used.values()) == 8 * sum(c["rows"] for c in byorig.values())


def test_uniform_4k():
    check([(0x10000 + 4096 * i, 4096) for i in range(300)])


def test_uniform_4m_like():
    # 4 MiB-style large buffers, fewer of them (model cost)
    check([(0x100000 * (i + 1), 300000) for i in range(6)], ncu=2)


def test_uniform_pool_4k_many_chunks():
    # uniform batch over 3 chunks (the last partial): items of PECH_ITEM_ROWS
    # from the workgroup pool, each located by division (checked against the
    # row-offset search inside the model)
    descs = [(0x10000 + 4096 * i, 4096) for i in range(2500)]
    cores, lrs, partials, nzs = KM.plan(descs)
    assert all(z & KM.NZ_UNIFORM for z in nzs)
    check(descs, ncu=2)


def test_uniform_pool_large_buffers():
    check([(0x100000 * (i + 1), 1 << 20) for i in range(5)], ncu=1)


def test_not_uniform_when_chunks_differ():
    # each chunk uniform on its own, different rows per buffer: static shares
    descs = [(0x10000 + 8192 * i, 4096 if i < 1024 else 8192) for i in range(2048)]
    cores, lrs, partials, nzs = KM.plan(descs)
    assert all(z & KM.NZ_UNIFORM for z in nzs) and partials[0] // 1024 != partials[1] // 1024
    check(descs, ncu=1)


def test_tiny_and_unaligned():
    rng = random.Random(1)
    descs = []
    base = 1 << 20
    for i in range(500):
        ln = rng.choice([0, 1, 5, 15, 16, 17, 31, 32, 33, 64, 100, 127, 128, 129, 1000, 4095, 4097, 20000])
        off = rng.randrange(0, 64)
        descs.append((base + off, ln))
        base += off + ln + rng.randrange(0, 32)
    check(descs, ncu=3)


@pytest.mark.parametrize("U", [None, KM.C["PECH_U_COPY"]])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_mixed_sizes(seed, U):
    rng = random.Random(seed)
    sizes = [4096] * 200 + [65536] * 20 + [300000] * 3 + [16] * 30 + [7] * 10
    rng.shuffle(sizes)
    descs, base = [], 4096
    for s in sizes:
        descs.append((base, s))
        base += s
    # U: the fused-copy kernel's shallower ring too.  Its stores are exactly
    # the non-virtual consumed pieces, so "used once" covers them
    check(descs, ncu=2, seed=seed, U=U)


def test_many_chunks_and_empty_chunks():
    descs = [(4096 * (i + 1), 0 if (i // 1024) == 1 else 256) for i in range(3000)]
    check(descs, ncu=1)


def test_one_buffer_many_waves():
    check([(1 << 30, 4 << 20)], ncu=1)


@pytest.mark.parametrize("weights", [[16, 12, 9, 8], [16, 1, 1, 1], [1, 1, 1, 16]])
def test_weighted_shares(weights):
    # any contiguous split of a workgroup's rows is valid (the kernel uses equal shares)
    sizes = [4096] * 300 + [300000] * 2 + [100] * 40
    random.Random(5).shuffle(sizes)
    descs, base = [], 1 << 16
    for sz in sizes:
        descs.append((base, sz))
        base += sz + 48
    check(descs, ncu=3, weights=weights)


@pytest.mark.parametrize("Rtot", [0, 1, 63, 64, 1000, 65536, 8 << 20])
@pytest.mark.parametrize("ncu", [1, 7, 256])
def test_wave_ranges_partition_row_space(Rtot, ncu):
    # (small launches deal their shares wave-major: sorted, they tile the rows)
    pos = 0
    for r0, r1 in sorted(KM.wave_ranges(Rtot, ncu)):
        if r1 == r0:
            continue
        assert r0 == pos and r1 > r0
        pos = r1
    assert pos == Rtot


@pytest.mark.parametrize("item,pool", [(64, 200), (256, 1024), (512, 0xFFFFFFFF), (32, 32)])
def test_pool_item_and_tail_sizes(monkeypatch, item, pool):
    # the A/B sizes of the pooled share tails: every row still consumed once
    monkeypatch.setattr(KM, "ITEM", item)
    monkeypatch.setattr(KM, "POOL", pool)
    check([(0x10000 + 4096 * i, 4096) for i in range(1500)], ncu=1)
    check([(0x100000 * (i + 1), 1 << 20) for i in range(3)], ncu=1)


@pytest.mark.parametrize("pool_min", [0, 1024])
def test_pool_min_share(monkeypatch, pool_min):
    # 512-row shares (the 256 MiB launches of 64 KiB-4 MiB buffers, scaled
    # down): pooled below the kernel's PECH_POOL_MIN_SHARE only when it is 0,
    # static shares otherwise; every row consumed once either way
    monkeypatch.setattr(KM, "POOL_MIN", pool_min)
    check([(0x100000 * (i + 1), 1 << 16) for i in range(32)], ncu=2)
    check([(0x100000 * (i + 1), 1 << 20) for i in range(2)], ncu=2)


@pytest.mark.parametrize("ncu,descs", [
    (2, [(0x100000 * (i + 1), 1 << 20) for i in range(5)]),             # 8192-row buffers, ranges cut mid-buffer
    (3, [(0x40000 * (i + 1) + 48, (1 << 17) - 48) for i in range(7)]),   # 1,024 rows, unaligned start, ragged portions
    (1, [(0x1000 + 5, (3 << 20) + 777)]),                                 # one misaligned buffer over one workgroup
])
def test_fused_copy_interleaved_rows(ncu, descs):
    # the fused copy's interleaved mode (plan_il): every core row consumed
    # once by the lane group it belongs to, loads inside the buffer's lines,
    # every run shifted to its buffer's end
    cores, lrs, partials, nzs = KM.plan(descs)
    assert all(z & KM.NZ_UNIFORM for z in nzs)
    assert min(c["rows"] for c in cores if c is not None) >= KM.IL_MIN  # the interleaved mode, not the slices
    check(descs, ncu=ncu, copy=True, U=12)


@pytest.mark.parametrize("n,ncu", [(1, 256), (7, 256), (255, 256), (256, 256), (257, 256), (4097, 256),
                                   (32767, 256), (32769, 256), (65536, 256), (98309, 256), (1000, 3)])
def test_direct_kernel_positions_once(n, ncu):
    # the direct kernel's workgroup-interleaved schedule: every position of
    # the batch taken by exactly one lane group, in steps of <= 8 per wave
    seen = collections.Counter(p for *_, p in KM.direct_positions(n, ncu))
    assert sorted(seen) == list(range(n)) and set(seen.values()) == {1}


def test_final_shift_packing_at_maximum_length():
    # a buffer within 255 bytes of 4 GiB has a core of 2^25 + 1
    # rows; a 1-row run at its start has 2^25 rows after it, which wraps the
    # 32-bit Step.mp after its << 7 -- bit 25 rides in Step.oz bit 29
    for addr in (127, 0x1000 + 113, 0x7F):
        for ln in ((1 << 32) - 1, (1 << 32) - 17, (1 << 32) - 128):
            rows = KM.core_rows(addr, ln)
            ce = (addr + ln) & ~15
            zt = rows * 8 - ((ce - (addr & ~127)) >> 4)
            tail = addr + ln - ce
            for ra in (0, 1, (1 << 25) - 1, rows - 1):
                mp, oz = KM.encode_m(ra, zt, tail)
                assert mp < 1 << 32
                assert KM.decode_m(mp, oz) == ra * KM.ROW + tail - 16 * zt, (addr, ln, ra)
    assert KM.core_rows(127, (1 << 32) - 1) == (1 << 25) + 1  # the case exists


def test_small_launch_live_workgroups_count():
    """The flat kernel's in-launch publication (flat_publish, the async
    layer's host array) waits for st.nlive workgroups: the count must equal
    the workgroups wave_share keeps live for every launch size, and their
    shares must cover each share exactly once -- the blocked dealing's first
    count missed that past 4 G shares the waves beyond the fourth take the
    rest (a 32 MiB + 256-row launch counted 257 live workgroups of 256, so no
    workgroup published and the host read stale results)."""
    G, LW, S = 256, 4, KM.DEAL_BLOCKS
    W = G * KM.WAVES_PER_WG
    for Rtot in list(range(1, 70000, 7)) + list(range(70000, 1100000, 997)):
        rpw = min(max((Rtot + LW * G - 1) // (LW * G), 64), 256)
        if Rtot >= W * rpw:
            continue
        nsh = (Rtot + rpw - 1) // rpw
        Gd = min(G, (nsh + LW - 1) // LW)
        blocks = S and Gd % S == 0
        nl = min(Gd, nsh // (LW * S) * S + min(nsh % (LW * S), S)) if blocks else min(G, nsh, Gd)
        live, cov = 0, [0] * nsh
        for b in range(Gd):
            first = (b // S) * LW * S + b % S if blocks else b
            if (first >= nsh) if blocks else (b * rpw >= Rtot):
                continue
            live += 1
            for w in range(KM.WAVES_PER_WG):
                k = (b // S) * LW * S + b % S + S * w if blocks and w < LW else w * Gd + b
                if k < nsh:
                    cov[k] += 1
        assert live == nl and all(c == 1 for c in cov), (Rtot, rpw, nsh, Gd, nl, live)
