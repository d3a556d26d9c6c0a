#!/usr/bin/env python3
"""bench.py -- CRC32C GiB/s on device-resident object buffers (BASELINE.json).

One "step" = one pass of the hot path (libpech_crc32c.so's kernels: one
flat launch for batches of up to 4,096 buffers, plan + main beyond) over one
batch of device-resident synthetic buffers.
Default workload = BASELINE config 3 / per-GPU shard of config 5:
256 x 4 MiB buffers (1 GiB) per GPU, rotating between 2 distinct batches
(2 GiB resident) so the 256 MiB Infinity Cache cannot serve a step.

    python bench.py                       # N=1, defaults
    python bench.py --config c2           # 65,536 x 4 KiB (parity-sized line)
    torchrun --nproc-per-node N bench.py --gpus N   # one process per GPU

Multi-GPU: batches are independent, so each rank checksums its own shard
(weak scaling); no collective touches the data path -- the only
communication is the timing barrier and a MAX all-reduce of the elapsed time.

Two timed passes of K steps each, both bracketed by barrier + synchronize:
a one-stream pass (batches back to back; `serial`, and the roofline), then
the `value` pass with consecutive batches alternating over two streams (own
workspace each), so one batch's plan kernel, launch boundaries, prologue and
tail overlap its neighbour's streaming -- how a server drives the library.

Prints ONE JSON line (rank 0).  `roofline` is for the main kernel: HIP
events around every main-kernel launch of the one-stream pass give the
average launch duration; achieved = algorithmic bytes per launch (sum of
buffer lengths) / that duration, against 8.0 TB/s HBM3E peak
(/opt/skills/guides/MI355X_MICROARCH.md).  `cpu_baseline` times the
reference crc32c() (oracle/_ref, compiled from the reference header) on
rank 0's host cores over a bounded sample of the same buffers, and checks
the GPU outputs for that sample bit-exact.
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak, GB/s (MI355X_MICROARCH.md)

CONFIGS = {
    # name: (list of buffer sizes per GPU, rotate, description)
    "c2": ([4096] * 65536, 4, "c2: 65,536 x 4 KiB device-resident buffers per GPU, 4 rotating batches (1 GiB)"),
    "c3": ([4 << 20] * 256, 2, "c3: 256 x 4 MiB device-resident buffers per GPU, 2 rotating batches (2 GiB)"),
    "c4": (None, 2, "c4: mixed 4 KiB/64 KiB/1 MiB/4 MiB, equal bytes per class (1 GiB) per GPU, shuffled seed 42, "
                    "2 rotating batches"),
    # C4's size classes as separate launches (per-size GiB/s), 256 MiB each, 4 rotating batches
    "c4-4k": ([4096] * 65536, 4, "c4 class 4 KiB: 65,536 x 4 KiB per launch"),
    "c4-64k": ([65536] * 4096, 4, "c4 class 64 KiB: 4,096 x 64 KiB per launch"),
    "c4-1m": ([1 << 20] * 256, 4, "c4 class 1 MiB: 256 x 1 MiB per launch"),
    "c4-4m": ([4 << 20] * 64, 4, "c4 class 4 MiB: 64 x 4 MiB per launch"),
    # C2's 4 KiB buffers in a 1 GiB launch (the size class of C4 that costs most, at C3's launch size)
    "c2-1g": ([4096] * 262144, 2, "c2-1g: 262,144 x 4 KiB (1 GiB) per launch, 2 rotating batches"),
    # small launches (the launch curve's points as configs, for PMC passes): 4 MiB and 32 MiB of 4 MiB buffers
    "l4m": ([4 << 20], 8, "l4m: one 4 MiB buffer per launch, 8 rotating batches"),
    "l32m": ([4 << 20] * 8, 8, "l32m: 8 x 4 MiB per launch, 8 rotating batches"),
    # unaligned payloads (messenger lengths are arbitrary): every buffer has a head and/or a tail
    "c2-odd": ([4100] * 65536, 4, "c2-odd: 65,536 x 4,100 B back to back (unaligned heads and tails), 4 rotating batches"),
}


def c4_sizes():
    rng = np.random.default_rng(42)
    sizes = [4096] * 65536 + [65536] * 4096 + [1 << 20] * 256 + [4 << 20] * 64
    rng.shuffle(sizes)
    return sizes


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline work (rank 0, N=1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-path", action="store_true", help="skip the PCIe-inclusive pinned-host leg")
    ap.add_argument("--host-passes", type=int, default=4)
    ap.add_argument("--op", default="crc", choices=["crc", "copy"],
                    help="crc: the checksum path; copy: fused CRC + copy to a second buffer (SURVEY 8f row 4)")
    ap.add_argument("--streams", type=int, default=2,
                    help="HIP streams that consecutive batches alternate over (own workspace each) in the timed "
                         "pass that gives `value`; a one-stream pass always gives the per-launch roofline")
    ap.add_argument("--api", choices=["auto", "planned", "small"], default="auto",
                    help="device entry point: planned = crc32c_dev_batch_ws_async (plan + main kernel), small = "
                         "crc32c_dev_batch_small_async (direct kernel, one launch); auto = small when every buffer "
                         "is below 32 KiB, as the async layer routes its slots")
    ap.add_argument("--flat-max", type=int, default=4096,
                    help="device batches of at most this many buffers run as one launch with no plan kernel "
                         "(crc32c_set_flat_max; 0 = always plan + main, the A/B against the planned path)")
    ap.add_argument("--no-kernel-events", action="store_true",
                    help="diagnostic: no HIP events around the main kernel (roofline unavailable)")
    ap.add_argument("--data", choices=["random", "zeros", "ones"], default="random",
                    help="payload bytes: uniform random (default) or the constant sensitivity rows of SURVEY 8(d)")
    ap.add_argument("--profile-json", default=None, help="PMC summary (profiles/*.json) to fill roofline.traffic")
    ap.add_argument("--rotate", type=int, default=None,
                    help="distinct resident batches to rotate over (default per config; a multiple of --streams)")
    ap.add_argument("--sustain-seconds", type=float, default=6.0,
                    help="before the warm-up and the K timed steps, run the value pass this long and report its "
                         "rate as `sustained` (seconds of GPU work: clocks/thermals settle before the timed steps, a "
                         "sampling monitor sees the GPU busy); 0 = skip")
    ap.add_argument("--single-thread", action="store_true",
                    help="pech's model: ONE process drives --gpus devices (hipSetDevice + crc32c_dev_batch_ws_async "
                         "per device, own streams and workspaces), instead of one process per GPU")
    ap.add_argument("--curve-only", action="store_true",
                    help="diagnostic (A/B of kernel builds): print only the launch-size curve (launch_curve) of "
                         "the c3 batches and exit")
    ap.add_argument("--devices", default=None,
                    help="with --single-thread: comma-separated device list (default 0..gpus-1); a repeated id "
                         "puts several shards on one GPU (rehearsal on a 1-GPU box)")
    return ap.parse_args()


def main():
    args = parse()
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # PECH_BENCH_BACKEND=gloo rehearses the N>1 bench on a box with fewer
    # GPUs than ranks (ranks share devices round-robin; timing all-reduce on
    # the host).  The driver's N>1 runs use the default: RCCL, one GPU per rank.
    backend = os.environ.get("PECH_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local %= max(1, torch.cuda.device_count())
    # PECH_BENCH_FORCE_DIST=1: the process-group path at world size 1 too (a
    # one-GPU rehearsal of the N>1 code on RCCL: init, barriers, MAX timing,
    # device gather, per-rank parity)
    if world > 1 or os.environ.get("PECH_BENCH_FORCE_DIST") == "1":
        import torch.distributed as dist

        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    if args.single_thread:
        if world > 1:
            raise SystemExit("--single-thread is one process: do not launch it under torchrun")
        devids = [int(x) for x in args.devices.split(",")] if args.devices else list(range(args.gpus))
    else:
        devids = [local]
    dev = torch.device("cuda", devids[0])
    torch.cuda.set_device(dev)

    import pech_amd as P
    from pech_amd import _lib

    P.set_flat_max(args.flat_max)
    sizes, rotate, desc = CONFIGS[args.config]
    if args.rotate:
        rotate = args.rotate
        desc = desc.split(",")[0] + f", {rotate} rotating batches"
    if sizes is None:
        sizes = c4_sizes()
    sizes = np.asarray(sizes, dtype=np.int64)
    n = len(sizes)
    batch_bytes = int(sizes.sum())
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    maxs = max(1, args.streams)
    small_api = args.api == "small" or (args.api == "auto" and int(sizes.max()) < (32 << 10))
    flat = not small_api and args.op == "crc" and n <= min(args.flat_max, 4096)

    class Shard:
        """One device's batches: `rotate` distinct resident batches of random
        bytes + descriptors, outputs, streams and a workspace per stream."""

        def __init__(self, d, seed):
            self.dev = torch.device("cuda", d)
            with torch.cuda.device(self.dev):
                gen = torch.Generator(device=self.dev)
                gen.manual_seed(seed)
                self.bufs, self.descs = [], []
                for r in range(rotate):
                    if args.data == "random":
                        b = torch.randint(0, 256, (batch_bytes,), dtype=torch.uint8, device=self.dev, generator=gen)
                    else:  # SURVEY 8(d) sensitivity rows: constant bytes (every lane looks up the same entries)
                        b = torch.full((batch_bytes,), 0 if args.data == "zeros" else 0xFF, dtype=torch.uint8,
                                       device=self.dev)
                    self.bufs.append(b)
                    self.descs.append(P.make_descs(b.data_ptr() + offs, sizes, device=self.dev))
                self.outs = [torch.zeros(n, dtype=torch.int32, device=self.dev) for _ in range(rotate)]
                self.dsts = []
                if args.op == "copy":  # a destination buffer per rotating batch, same layout
                    for r in range(rotate):
                        dd = torch.empty(batch_bytes, dtype=torch.uint8, device=self.dev)
                        self.dsts.append((dd, torch.from_numpy((dd.data_ptr() + offs).astype(np.int64)).to(self.dev)))
                assert _lib.lib().crc32c_dev_reserve(n) == 0
                self.streams = [torch.cuda.current_stream(self.dev) if not args.single_thread
                                else torch.cuda.Stream(self.dev)] + \
                               [torch.cuda.Stream(self.dev) for _ in range(maxs - 1)]
                wsb = P.workspace_bytes(n)
                self.wss = [torch.empty(wsb, dtype=torch.uint8, device=self.dev) for _ in range(maxs)]

        def step(self, i, k):
            with torch.cuda.device(self.dev):
                if self.dsts and small_api:
                    P.dev_copy_batch_small_async(self.descs[i % rotate], self.dsts[i % rotate][1],
                                                 self.outs[i % rotate], stream=self.streams[k])
                elif self.dsts:
                    P.dev_copy_batch_ws_async(self.descs[i % rotate], self.dsts[i % rotate][1],
                                              self.outs[i % rotate], self.wss[k], stream=self.streams[k])
                elif small_api:
                    P.dev_batch_small_async(self.descs[i % rotate], self.outs[i % rotate], stream=self.streams[k])
                else:
                    P.dev_batch_ws_async(self.descs[i % rotate], self.outs[i % rotate], self.wss[k],
                                         stream=self.streams[k])

    shards = [Shard(d, 1000 + rank * 64 + j) for j, d in enumerate(devids)]
    bufs, outs, dsts = shards[0].bufs, shards[0].outs, shards[0].dsts
    if args.curve_only:
        print(json.dumps({"kernel": P.version(), "lib": _lib.LIB_PATH, "launch_curve": launch_curve(shards[0], P, torch)}))
        return

    def sync_all():
        for d in sorted(set(devids)):
            torch.cuda.synchronize(torch.device("cuda", d))

    def timed(nstreams, steps, warmup, events=False):
        """Warm-up, then `steps` batches bracketed by barrier + synchronize;
        batch i on stream i % nstreams (own workspace) of every shard.  A
        batch's output buffer is only ever written from one stream, so steps
        never race.  Returns (elapsed seconds, max over ranks; per-launch
        main-kernel us; this rank's own elapsed seconds; seconds its host
        thread spent issuing the K steps)."""
        if rotate % nstreams:
            raise SystemExit(f"{nstreams} streams must divide the {rotate} rotating batches")

        def step(i):
            for sh in shards:  # one host thread issues every device's batch, then the next
                sh.step(i, i % nstreams)

        for i in range(warmup):
            step(i)
        sync_all()
        P.timing(events)
        P.timing_read()  # discard warm-up launches
        if dist is not None:
            dist.barrier()
        sync_all()
        t0 = time.perf_counter()
        for i in range(steps):
            step(i)
        issue = time.perf_counter() - t0  # (the host thread's issue time: no wait inside a step)
        sync_all()
        if dist is not None:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        own = elapsed
        P.timing_read()
        samples = np.asarray(P.timing_samples(), dtype=np.float64) * 1e3  # us per main-kernel launch
        P.timing(False)
        if dist is not None:
            t = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        return elapsed, samples, own, issue

    # Pass 1, one stream, every launch stamped by HIP events: its per-launch
    # kernel durations (dispatch-packet events, non-overlapping) give the
    # roofline.  Pass 2, one stream, no events: batches back to back (`serial`,
    # pech's one batch in flight).  Pass 3, `--streams` streams (default 2):
    # consecutive batches alternate over them, so one batch's plan kernel,
    # launch boundaries, prologue and tail overlap its neighbour's streaming --
    # how a server runs the library (the async layer keeps four batches in
    # flight).  Pass 3 is `value`.
    nstreams = max(1, args.streams)
    # The sustained pass runs first: seconds of the value pass, so clocks and
    # thermals have settled before the K timed steps (a 20-step pass lasts
    # ~4 ms), and a sampling GPU monitor sees the device busy.
    sustained = None
    if args.sustain_seconds > 0:
        sustained = sustain(shards, nstreams, args.sustain_seconds, sync_all, dist, backend, dev, torch)
    # The roofline pass stamps every launch with HIP events (hipExtLaunchKernel
    # start/stop: ~5 us of extra gap per launch, measured on C2); the serial
    # and value passes run as a server does, without them.
    samples = timed(1, args.steps, args.warmup, events=True)[1] if not args.no_kernel_events else np.zeros(0)
    serial_el, _, serial_own, serial_issue = timed(1, args.steps, args.warmup)
    elapsed, _, own_el, issue_s = ((serial_el, None, serial_own, serial_issue) if nstreams == 1 else
                                   timed(nstreams, args.steps, args.warmup))
    launches = len(samples)
    kernel_ms = float(samples.sum()) / 1e3

    total_bytes = batch_bytes * args.steps * world * len(shards)
    value = total_bytes / elapsed / (1 << 30)
    avg_kernel_s = kernel_ms / 1e3 / max(launches, 1)
    # algorithmic HBM bytes per launch: each payload byte read once (+ written
    # once by the fused copy)
    algo_bytes = batch_bytes * (2 if dsts else 1)
    achieved_gbs = algo_bytes / avg_kernel_s / 1e9 if launches else 0.0

    # HBM bytes per launch from the committed rocprofv3 PMC pass of this
    # config (tools/pmc_traffic.py: FETCH_SIZE x 2, the gfx950 correction of
    # MI355X_MICROARCH.md), used only when it was taken on this kernel build.
    traffic = None
    tag = args.config + ("-copy" if dsts else "")
    for pj in ([args.profile_json] if args.profile_json else
               [os.path.join(REPO, "profiles", r, f"{tag}_traffic.json") for r in ("r06", "r05", "r04", "r03", "r02", "r01")]):
        if os.path.exists(pj):
            prof = json.load(open(pj))
            if prof.get("kernel") == P.version():
                traffic = prof.get("hbm_bytes_per_launch")
                break

    # distinct devices over all ranks (a gloo rehearsal puts several ranks on one GPU)
    ndev = len(set(devids))
    if dist is not None:
        alldev = [None] * world
        dist.all_gather_object(alldev, [(socket.gethostname(), d) for d in devids])
        ndev = len({x for r in alldev for x in r})
    line = {
        "metric": "CRC32C GiB/s on device-resident object buffers (4 KiB–4 MiB), 1/2/4/8 GPUs",
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": ndev,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": ("synthetic (uniform random bytes, torch.randint on device), seed 0 per buffer" if args.data == "random"
                 else f"synthetic constant bytes ({'0x00' if args.data == 'zeros' else '0xFF'}), seed 0 per buffer"),
        "config": {"workload": desc + ("; fused CRC + copy to a second buffer (read + write)" if dsts else ""),
                   "buffers_per_gpu": n, "bytes_per_gpu_per_step": batch_bytes,
                   "parallelism": (f"single-thread: one process drives {len(shards)} shard(s) on device(s) "
                                   f"{','.join(map(str, devids))}, no collective" if args.single_thread else
                                   f"shard{world} (independent buffers per GPU, no collective)"),
                   "streams": nstreams,
                   "api": ("crc32c_dev_copy_batch_small_async" if dsts else "crc32c_dev_batch_small_async")
                          if small_api else ("crc32c_dev_copy_batch_ws_async" if dsts else "crc32c_dev_batch_ws_async"),
                   "kernel": P.version()},
        "roofline": {"bound": "hbm", "achieved": round(achieved_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved_gbs / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel": ("pech_crc32c_direct_copy" if dsts else "pech_crc32c_direct") if small_api else
                               ("pech_crc32c_flat" if n <= 256 else "pech_crc32c_flatg") if flat else
                               ("pech_crc32c_main_copy" if dsts else "pech_crc32c_main"),
                     "bytes_per_launch": algo_bytes, "avg_launch_us": round(avg_kernel_s * 1e6, 2),
                     "launch_us_p10_p50_p90": [round(float(np.percentile(samples, q)), 2) for q in (10, 50, 90)]
                     if len(samples) else None,
                     "launches": launches, "pass": "one stream, K launches, HIP events on each"},
        "serial": {"streams": 1, "value": round(total_bytes / serial_el / (1 << 30), 2), "unit": "GiB/s",
                   "ms_per_step": round(serial_el / args.steps * 1e3, 4)},
    }
    if rank == 0 and world == 1 and len(shards) == 1 and not args.no_host_path and not dsts:
        line["pcie_inclusive"] = host_path(args, bufs[0], offs, sizes, outs, P)
        line["dropin_crc32c"] = dropin_latency(P)
        # uniform payloads: the C adapter benchmark (no Python per submit);
        # mixed batches through ctypes, where payloads are few enough for the
        # Python loop not to be the bound
        if len(set(sizes.tolist())) == 1:
            line["msgr_async"] = msgr_c_bench(args, int(sizes[0]), n)
            try:  # auxiliary legs: a failure is reported in the line, not fatal to it
                line["msgr_cpu"] = msgr_cpu_sizes(args)
            except (SystemExit, Exception) as e:  # noqa: BLE001
                line["msgr_cpu"] = {"error": str(e)[:500]}
            try:
                line["msgr_latency"] = msgr_latency(args)
            except (SystemExit, Exception) as e:  # noqa: BLE001
                line["msgr_latency"] = {"error": str(e)[:500]}
        else:
            line["msgr_async"] = msgr_path(args, bufs[0], offs, sizes, outs, P) if n <= 4096 else None
    if rank == 0 and world == 1 and len(shards) == 1 and not args.no_host_path and not dsts and args.config == "c3":
        line["launch_curve"] = launch_curve(shards[0], P, torch)
    if rank == 0 and world == 1 and len(shards) == 1 and not args.no_cpu_baseline and not dsts:
        line["cpu_baseline"] = cpu_baseline(args, bufs[0], offs, sizes, outs, rotate, P)

    if sustained:
        sec, steps_done = sustained
        line["sustained"] = {"seconds": round(sec, 2), "steps": steps_done, "streams": nstreams,
                             "value": round(batch_bytes * steps_done * world * len(shards) / sec / (1 << 30), 2),
                             "unit": "GiB/s"}
    # The host thread's issue time per step beside the kernel time per step
    # (VERDICT r4 #3): one thread driving several devices (--single-thread)
    # is host-bound once issuing a step's launches takes longer than a
    # device's kernel for it.
    line["host_issue"] = {"issue_us_per_step": round(serial_issue / args.steps * 1e6, 2),
                          "launches_per_step": len(shards),
                          "kernel_us_per_launch": round(avg_kernel_s * 1e6, 2) if launches else None,
                          "pass": "serial (one stream per shard): wall time of the issue loop / K"}
    if dist is not None:
        # per-rank evidence: a straggling GPU or a slow XCD
        # pairing on one rank shows here, not only in the MAX-over-ranks value
        mine = {"rank": rank, "host": socket.gethostname(), "device": devids[0],
                "value": round(batch_bytes * args.steps * len(shards) / own_el / (1 << 30), 2),
                "serial": round(batch_bytes * args.steps * len(shards) / serial_own / (1 << 30), 2),
                "avg_launch_us": round(avg_kernel_s * 1e6, 2) if launches else None}
        allr = [None] * world
        dist.all_gather_object(allr, mine)
        line["per_rank"] = allr
        for key, tgt in (("avg_launch_us", line["roofline"]), ("value", line)):
            vals = [r[key] for r in allr if r[key] is not None]
            if vals:
                arg = max(range(len(allr)), key=lambda k: allr[k][key] or 0)
                tgt[f"{key}_per_rank"] = {"min": min(vals), "max": max(vals), "argmax_rank": allr[arg]["rank"],
                                          "spread": round(max(vals) / min(vals) - 1, 4)}
    if len(shards) > 1 and dist is None:
        line["shards_checked"], line["buffers_checked"] = shard_parity(shards, offs, sizes, rotate, P)
    if dist is not None:
        # every rank checks its own shard against the oracle (outside the
        # timed region); rank 0 reports how many shards passed
        try:
            ok, nbuf = shard_parity(shards, offs, sizes, rotate, P)
            bad = 0
        except SystemExit as e:
            print(f"rank {rank}: {e}", file=sys.stderr, flush=True)
            ok, nbuf, bad = 0, 0, 1
        t = torch.tensor([ok, bad, nbuf], dtype=torch.int64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        if int(t[1]):
            raise SystemExit(f"PARITY FAILURE: {int(t[1])} rank(s) computed CRCs that differ from the reference")
        line["shards_checked"] = int(t[0])
        line["buffers_checked"] = int(t[2])
        line["ranks"] = world
    if rank == 0 and world == 1 and len(shards) == 1 and launches:
        probe = stream_probe("copy" if dsts else "read", max(1, batch_bytes >> 20))
        if probe:
            line["roofline"]["probe"] = dict(probe, frac_of_probe=round(achieved_gbs / probe["GBps"], 4))
            if "best_shape" in probe:
                line["roofline"]["probe"]["best_shape"]["frac"] = round(achieved_gbs / probe["best_shape"]["GBps"], 4)

    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def host_path(args, buf0, offs, sizes, outs, P):
    """PCIe-inclusive rate (reported beside `value`, never as it): the same
    batch in pinned host memory through crc32c_batch(..., CRC32C_F_PINNED) --
    the kernel reads the pinned buffers in place over the host link
    (zero-copy), plan + main kernels, D2H of the results.  Outputs are
    checked bit-exact against the device-resident run."""
    import torch
    from pech_amd import _lib

    n = len(sizes)
    host = torch.empty(int(buf0.numel()), dtype=torch.uint8, pin_memory=True)
    host.copy_(buf0)
    P.dev_batch_async(P.make_descs(buf0.data_ptr() + offs, sizes, device=buf0.device), outs[0])
    torch.cuda.synchronize()
    want = outs[0].cpu().numpy().view(np.uint32)
    ptrs = (ctypes.c_void_p * n)(*[host.data_ptr() + int(o) for o in offs])
    lens = (ctypes.c_uint * n)(*[int(x) for x in sizes])
    out = (ctypes.c_uint32 * n)()
    lib = _lib.lib()
    _lib.check(lib.crc32c_batch(ptrs, lens, None, out, n, P.F_PINNED), "crc32c_batch")  # warm-up
    t0 = time.perf_counter()
    for _ in range(args.host_passes):
        _lib.check(lib.crc32c_batch(ptrs, lens, None, out, n, P.F_PINNED), "crc32c_batch")
    dt = time.perf_counter() - t0
    got = np.frombuffer(out, dtype=np.uint32)
    if not np.array_equal(got, want):
        raise SystemExit("PARITY FAILURE: pinned-host path differs from the device-resident path")
    nbytes = int(sizes.sum())
    res = {"value": round(nbytes * args.host_passes / dt / (1 << 30), 2), "unit": "GiB/s",
           "path": "crc32c_batch(CRC32C_F_PINNED): pinned host buffers of >= 1 MiB DMA'd on two copy streams, "
                   "smaller ones read in place by the kernel (zero-copy over the host link), plan+main kernels, "
                   "D2H results; synchronous call",
           "bytes_per_pass": nbytes, "passes": args.host_passes, "matches_device_path": True}
    ndev = torch.cuda.device_count()
    if ndev > 1:
        # the same call sharded over every visible GPU from this one thread
        # (CRC32C_F_ALL_DEVICES: each GPU reads its shard over its own host link)
        flags = P.F_PINNED | P.F_ALL_DEVICES
        rc = lib.crc32c_batch(ptrs, lens, None, out, n, flags)
        if rc != 0:
            res["all_devices"] = {"devices": ndev, "error": lib.crc32c_last_error().decode()}
        else:
            t0 = time.perf_counter()
            for _ in range(args.host_passes):
                _lib.check(lib.crc32c_batch(ptrs, lens, None, out, n, flags), "crc32c_batch")
            dt = time.perf_counter() - t0
            if not np.array_equal(np.frombuffer(out, dtype=np.uint32), want):
                raise SystemExit("PARITY FAILURE: all-devices pinned-host path differs from the device path")
            res["all_devices"] = {"devices": ndev, "value": round(nbytes * args.host_passes / dt / (1 << 30), 2),
                                  "unit": "GiB/s", "path": "crc32c_batch(CRC32C_F_PINNED | CRC32C_F_ALL_DEVICES) "
                                  "from one host thread", "matches_device_path": True}
    return res


def dropin_latency(P):
    """Per-call latency of the drop-in crc32c() from C (build/dropin_bench,
    tools/c/dropin_bench.c): pageable host memory, one synchronous call per
    buffer as messenger.c calls it per header / section / <=4 KiB piece.
    Columns: "host" = default routing (host routine up to 4 MiB, GPU above),
    "gpu" = every call through the gfx950 kernels, "ref" = the reference
    byte loop.  The tool checks every route against the reference."""
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "build", "dropin_bench")
    r = subprocess.run([exe, "0.1"], capture_output=True, timeout=300)
    if r.returncode != 0:
        raise SystemExit("PARITY FAILURE (drop-in): " + r.stdout.decode() + r.stderr.decode())
    res = json.loads(r.stdout.decode().strip().splitlines()[-1])
    res["path"] = ("crc32c(0, buf, n) from pageable memory, synchronous, called from C; host = default "
                   "routing (<= 4 MiB on the host routine), gpu = crc32c_set_cpu_max(0), ref = reference loop")
    # BASELINE config 1 (fio 4 KiB OP_WRITE against a pech-osd) needs fio and a
    # Ceph monitor, absent here.  Its checksum work per operation, from the
    # per-call latencies above: the request's header (49 B, messenger.c:2714),
    # front (~200 B, :2641) and 4 KiB data (:2677 via :1729), and the reply's
    # header (:1403) and front (:1412); a write reply carries no data.
    sz = res.get("sizes", {})
    if all(k in sz for k in ("49", "200", "4096")):
        per_op = {k: round(2 * sz["49"][k] + 2 * sz["200"][k] + sz["4096"][k], 4) for k in ("host", "ref")}
        res["c1_per_op"] = {"calls": "2 x header 49 B + 2 x front 200 B + data 4096 B", "unit": "us",
                            "drop_in": per_op["host"], "reference": per_op["ref"],
                            "note": "derived from the per-call latencies; the fio plumbing itself is not run"}
    return res


def msgr_path(args, buf0, offs, sizes, outs, P):
    """The messenger adapter's rate, PCIe-inclusive: the
    batch's payloads in crc32c_pages memory (pinned payload pages, carved
    from 8 MiB order-11 blocks), one crc32c_async_submit per payload, flush,
    then drain (eventfd completion).  Two modes: DMA into device staging
    slots, and zero-copy (the kernel reads the pinned pages in place).
    Results are checked bit-exact against the device-resident run."""
    import torch

    P.dev_batch_async(P.make_descs(buf0.data_ptr() + offs, sizes, device=buf0.device), outs[0])
    torch.cuda.synchronize()
    want = outs[0].cpu().numpy().view(np.uint32)
    host = buf0.cpu().numpy()
    blocks, addrs, fill = [], [], None
    for o, n in zip(offs, sizes):
        n = int(n)
        if fill is None or fill + n > blocks[-1].nbytes:
            blocks.append(P.Pages(11))
            fill = 0
        blocks[-1].view[fill:fill + n] = host[int(o):int(o) + n]
        addrs.append(blocks[-1].ptr + fill)
        fill = (fill + n + 4095) & ~4095
    nbytes = int(sizes.sum())
    res = {}
    for mode, dma in (("dma", True), ("zerocopy", False)):
        ac = P.AsyncCrc(dma=dma)
        got = np.zeros(len(sizes), dtype=np.uint32)

        def one_pass():
            for i, (a, n) in enumerate(zip(addrs, sizes)):
                ac.submit(a, int(n), 0, lambda crc, err, i=i: got.__setitem__(i, crc if err == 0 else 0))
            ac.drain()

        one_pass()  # warm-up (slot allocation)
        t0 = time.perf_counter()
        for _ in range(args.host_passes):
            one_pass()
        dt = time.perf_counter() - t0
        ac.close()
        if not np.array_equal(got, want):
            raise SystemExit(f"PARITY FAILURE: async {mode} path differs from the device-resident path")
        res[mode] = round(nbytes * args.host_passes / dt / (1 << 30), 2)
    for b in blocks:
        b.free()
    return {"dma": res["dma"], "zerocopy": res["zerocopy"], "unit": "GiB/s",
            "path": "crc32c_async_submit per payload from crc32c_pages memory, flush, drain (eventfd); "
                    "dma: CRC32C_ASYNC_DMA, H2D into 32 MiB device slots at launch; zerocopy (the default): "
                    "kernel reads pinned pages in place",
            "bytes_per_pass": nbytes, "passes": args.host_passes, "matches_device_path": True}


def msgr_c_bench(args, size, count, modes=(("dma", 0), ("zerocopy", 1), ("adapter", 2), ("host", 3)), passes=None,
                 env=None):
    """The messenger-side rate and CPU cost from C (build/msgr_sim bench):
    `count` payloads of `size` bytes in crc32c_pages memory per pass, flushed
    every 64 and completed from an epoll loop, through the async layer (DMA
    and zero-copy), the messenger adapter (its size routing at the default),
    and the drop-in's host routine.  Reported per mode: GiB/s, payloads/s,
    CPU microseconds per payload of the calling thread (pech's one OS thread)
    and of the process, submit -> result latency p50/p99.  The C program
    checks every result against the oracle."""
    import subprocess

    exe = os.path.join(REPO, "build", "msgr_sim")
    count = max(1, min(count, (256 << 20) // max(size, 1)))
    res = {}
    for mode, m in modes:
        r = subprocess.run([exe, "bench", str(size), str(count), str(m), str(passes or args.host_passes)],
                           capture_output=True, text=True, timeout=300, env=dict(os.environ, **(env or {})))
        if r.returncode != 0:
            raise SystemExit(f"msgr_sim bench failed ({r.returncode}): {r.stdout} {r.stderr}")
        d = json.loads(r.stdout.strip().splitlines()[-1])
        res[mode] = {k: d[k] for k in ("GiBps", "payloads_per_s", "thread_cpu_us_per_payload",
                                       "process_cpu_us_per_payload", "latency_us_p50", "latency_us_p99")}
    if "zerocopy" not in res:
        return res
    return {"payload_bytes": size, "modes": res, "zerocopy": res["zerocopy"]["GiBps"], "dma": res["dma"]["GiBps"],
            "unit": "GiB/s",
            "path": f"C: {size}-byte payloads in crc32c_pages memory, flush every 64, epoll loop on the eventfd "
                    "(build/msgr_sim bench); dma/zerocopy: crc32c_async_submit per payload; adapter: "
                    "crc32c_msgr_rx_queue/rx_next (host routine up to its cutoff); host: the drop-in crc32c()",
            "payloads": count, "passes": args.host_passes, "matches_oracle": True}


def msgr_cpu_sizes(args):
    """What the messenger's thread pays per payload at the rados.fio sizes
    (C1/C4: 4 KiB, 64 KiB, 1 MiB, 4 MiB): the adapter (host routine up to its
    cutoff, the GPU above it) against checksumming on the host with the
    drop-in, in CPU microseconds per payload of the calling thread and of
    the process (the HIP runtime's threads included), plus the adapter's
    submit -> result latency."""
    out = {}
    for size in (4096, 65536, 1 << 20, 4 << 20):
        r = msgr_c_bench(args, size, 16384, modes=(("adapter", 2), ("host", 3)))
        out[str(size)] = {"adapter_thread_us": r["adapter"]["thread_cpu_us_per_payload"],
                          "adapter_process_us": r["adapter"]["process_cpu_us_per_payload"],
                          "host_thread_us": r["host"]["thread_cpu_us_per_payload"],
                          "adapter_latency_us_p50_p99": [r["adapter"]["latency_us_p50"], r["adapter"]["latency_us_p99"]],
                          "adapter_GiBps": r["adapter"]["GiBps"], "host_GiBps": r["host"]["GiBps"]}
    return {"unit": "CPU us per payload", "sizes": out,
            "path": "build/msgr_sim bench: crc32c_pages payloads, flush every 64, epoll loop; adapter = "
                    "crc32c_msgr_rx_queue/rx_next, host = drop-in crc32c()"}


def msgr_latency(args):
    """Unloaded submit -> verified latency of ONE payload in flight (pech at
    low queue depth: one read_partial_msg_data -> footer compare per message,
    messenger.c:2649-2684, :2836-2842), against checksumming it on the host.
    build/msgr_sim bench with one payload per pass: rx_queue (or the drop-in
    for "host"), flush, epoll_wait on the eventfd, complete, rx_next.
    adapter = its default routing (host routine up to 8 KiB); adapter_gpu =
    PECH_CRC32C_MSGR_HOST_MAX=0, every payload through the GPU (zero-copy
    read of the pinned page, the direct or plan + main kernels, D2H of the
    result, host function, eventfd)."""
    out = {}
    for size in (4096, 65536, 1 << 20, 4 << 20):
        r = msgr_c_bench(args, size, 1, modes=(("adapter", 2), ("host", 3)), passes=300)
        g = msgr_c_bench(args, size, 1, modes=(("adapter_gpu", 2),), passes=300,
                         env={"PECH_CRC32C_MSGR_HOST_MAX": "0"})
        out[str(size)] = {k: [v["latency_us_p50"], v["latency_us_p99"], v["thread_cpu_us_per_payload"]]
                          for k, v in (("adapter", r["adapter"]), ("adapter_gpu", g["adapter_gpu"]),
                                       ("host", r["host"]))}
    return {"columns": "[latency p50 us, latency p99 us, calling-thread CPU us] per payload", "sizes": out,
            "path": "one payload in flight (300 in sequence): crc32c_pages payload, rx_queue, flush, epoll_wait "
                    "on the eventfd, complete, rx_next; host = drop-in crc32c() on the same bytes"}


def launch_curve(shard, P, torch):
    """Per-launch cost of the device batch path (the flat kernel for up to
    4,096 buffers, plan + main kernels beyond) against launch size, for 4 MiB and 64 KiB buffers: 4 / 32 (the async layer's
    slot) / 128 / 256 / 1024 MiB per launch, carved from the shard's resident
    batches and cycled over distinct regions of them (2 GiB in all, so the
    256 MB Infinity Cache cannot serve a launch).  main_us: HIP events around
    each main kernel (its roofline fraction beside it); step_us: wall time
    per launch of back-to-back serial steps (plan kernel and launch gaps
    included)."""
    pool = shard.bufs
    per = int(pool[0].numel())
    stream = shard.streams[0]
    res = {}
    for bsz in (4 << 20, 64 << 10):
        row = {}
        for mib in (4, 32, 128, 256, 1024):
            tot = mib << 20
            n = tot // bsz
            regions = min(512, (per * len(pool)) // tot)
            descs = []
            for r in range(regions):
                b = pool[(r * tot) // per]
                base = b.data_ptr() + (r * tot) % per
                descs.append(P.make_descs(base + np.arange(n, dtype=np.int64) * bsz, np.full(n, bsz, np.int64),
                                          device=shard.dev))
            out = torch.zeros(n, dtype=torch.int32, device=shard.dev)
            ws = torch.empty(P.workspace_bytes(n), dtype=torch.uint8, device=shard.dev)
            k = max(regions, 20)
            with torch.cuda.device(shard.dev):
                for i in range(min(k, 8)):  # warm-up
                    P.dev_batch_ws_async(descs[i % regions], out, ws, stream=stream)
                torch.cuda.synchronize(shard.dev)
                P.timing(True)
                P.timing_read()
                for i in range(k):
                    P.dev_batch_ws_async(descs[i % regions], out, ws, stream=stream)
                torch.cuda.synchronize(shard.dev)
                P.timing_read()
                main_us = float(np.mean(np.asarray(P.timing_samples(), dtype=np.float64))) * 1e3
                P.timing(False)
                t0 = time.perf_counter()
                for i in range(k):
                    P.dev_batch_ws_async(descs[i % regions], out, ws, stream=stream)
                torch.cuda.synchronize(shard.dev)
                step_us = (time.perf_counter() - t0) / k * 1e6
            row[str(mib)] = {"main_us": round(main_us, 2), "frac": round(tot / main_us / 1e3 / HBM_PEAK_GBS, 4),
                             "step_us": round(step_us, 2), "launches": k}
        res["4MiB" if bsz == 4 << 20 else "64KiB"] = row
    return {"unit": "us per launch; frac = launch bytes / main_us / 8 TB/s", "by_buffer_size_then_MiB": res,
            "path": "crc32c_dev_batch_ws_async, one stream: the flat kernels for up to 4,096 buffers (--flat-max), "
                    "plan + main kernels beyond"}


def sustain(shards, nstreams, seconds, sync_all, dist, backend, dev, torch):
    """The value pass kept running for `seconds` (batch i on stream i % nstreams
    of every shard), in rounds of 64 steps; returns (elapsed, steps), elapsed
    max over ranks and every rank running the same number of rounds."""
    sync_all()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    steps = 0
    while True:
        for i in range(64):
            for sh in shards:
                sh.step(steps + i, (steps + i) % nstreams)
        steps += 64
        sync_all()
        go = time.perf_counter() - t0 < seconds
        if dist is not None:  # all ranks stop after the same round
            t = torch.tensor([1 if go else 0], dtype=torch.int32, device=dev if backend == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            go = bool(t.item())
        if not go:
            break
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, steps


def stream_probe(kind, mib):
    """The same box's streaming ceiling for the kernel's access shape, at the
    batch's size (build/sched_probe, tools/sched_probe.hip: `mib` MiB per
    launch, 8-lane groups over 128-byte rows, 8 rows in flight per lane,
    nontemporal, one 1024-thread workgroup per CU, equal static shares):
    "read" for the CRC kernel, "copy" (read + write) for the fused CRC + copy.
    None if the probe is missing."""
    exe = os.path.join(REPO, "build", "sched_probe")
    if not os.path.exists(exe):
        return None
    r = subprocess.run([exe, "10", kind, str(mib)], capture_output=True, timeout=120)
    if r.returncode != 0:
        return None
    res = json.loads(r.stdout.decode())["results"][0]
    gbs = res.get("GBps_read_plus_write", res.get("GBps"))
    out = {"kind": kind, "GBps": gbs, "us_per_launch": res["us"],
           "what": f"tools/sched_probe.hip: same access shape, nontemporal, static shares, {mib} MiB" +
                   (f" read + {mib} MiB written" if kind == "copy" else " read") + " per launch"}
    # The fastest shape measured for the same bytes (a non-persistent grid,
    # one 16-byte nontemporal element per thread): a stricter denominator
    # that no table-driven persistent kernel reaches (profiles/r02/shape_probes.txt).
    r = subprocess.run([exe, "10", "grid", str(mib)], capture_output=True, timeout=120)
    if r.returncode == 0:
        res = json.loads(r.stdout.decode())["results"][1 if kind == "copy" else 0]
        out["best_shape"] = {"GBps": res["GBps"], "us_per_launch": res["us"], "what": res["probe"] +
                             ": non-persistent grid, one 16-byte element per thread"}
    return out


def shard_parity(shards, offs, sizes, rotate, P):
    """Multi-shard runs (single-thread, or one rank of a torchrun job): EVERY
    buffer of every shard's rotating batches against the oracle, outside the
    timed region -- the SSE4.2 batch oracle (oracle/crc32c_hw.c, bit-exact
    against the compiled reference in tests/test_oracle.py) on 16 host
    threads, or, on a host without SSE4.2, the reference loop on each batch's
    first and last buffer.  Returns (shards, buffers) checked."""
    import torch

    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib as O

    H = O.hw()
    offs64 = np.ascontiguousarray(offs, dtype=np.uint64)
    lens32 = np.ascontiguousarray(sizes, dtype=np.uint32)
    n = len(sizes)
    checked = 0
    for sh in shards:
        torch.cuda.synchronize(sh.dev)
        for r in range(rotate):
            got = sh.outs[r].cpu().numpy().view(np.uint32)
            host = sh.bufs[r].cpu().numpy()
            if H is not None:
                want = np.zeros(n, dtype=np.uint32)
                if H.hw_crc32c_batch_mt(host.ctypes.data, offs64.ctypes.data, lens32.ctypes.data, want.ctypes.data,
                                        n, 16, 1):
                    raise SystemExit("shard parity: oracle threads failed to start")
                bad = np.nonzero(got != want)[0]
                if len(bad):
                    raise SystemExit(f"PARITY FAILURE: shard on {sh.dev}, batch {r}, {len(bad)} buffer(s), first {bad[0]}")
                checked += n
            else:
                for i in (0, n - 1):
                    lo, hi = int(offs[i]), int(offs[i] + sizes[i])
                    if int(got[i]) != O.crc(0, host[lo:hi]):
                        raise SystemExit(f"PARITY FAILURE: shard on {sh.dev}, batch {r}, buffer {i}")
                    checked += 1
            del host
    return len(shards), checked


def cpu_baseline(args, buf0, offs, sizes, outs, rotate, P):
    """Reference crc32c() on this host's cores over a bounded sample of the
    same batch; also checks the GPU's outputs for the sampled buffers."""
    import torch

    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib as O

    # recompute batch 0 on the GPU (outputs of the last timed step may be batch 1)
    P.dev_batch_async(P.make_descs(buf0.data_ptr() + offs, sizes, device=buf0.device),
                      outs[0])
    torch.cuda.synchronize()
    gpu = outs[0].cpu().numpy().view(np.uint32)
    # sample: leading buffers of batch 0, about 256 MiB
    k = int(np.searchsorted(np.cumsum(sizes), 256 << 20, side="right"))
    k = max(1, min(k, len(sizes)))
    nbytes = int(offs[k - 1] + sizes[k - 1])
    host = buf0[:nbytes].cpu().numpy()
    ref = O.ref()
    kind = "reference" if ref is not None else "port"
    fn = ref.ref_crc32c if ref is not None else O.oracle().oracle_crc32c
    base = host.ctypes.data
    res = np.zeros(k, dtype=np.uint32)
    done_bytes = 0
    t0 = time.perf_counter()
    reps = 0
    while True:
        for i in range(k):
            res[i] = fn(0, base + int(offs[i]), int(sizes[i]))
        done_bytes += nbytes
        reps += 1
        if time.perf_counter() - t0 >= args.cpu_seconds:
            break
    dt = time.perf_counter() - t0
    if not np.array_equal(res, gpu[:k]):
        bad = int(np.count_nonzero(res != gpu[:k]))
        raise SystemExit(f"PARITY FAILURE: {bad}/{k} sampled buffers differ between GPU and reference")
    cpu_model = ""
    try:
        for l in open("/proc/cpuinfo"):
            if l.startswith("model name"):
                cpu_model = l.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    rate1 = done_bytes / dt / (1 << 30)
    line = {"value": round(rate1, 4), "unit": "GiB/s", "cores": 1, "kind": kind,
            "sample": f"{k} leading buffers ({nbytes / (1 << 20):.0f} MiB) of batch 0, {reps} pass(es), "
                      f"{dt:.1f} s, 1 thread, {cpu_model}; GPU outputs for the sample matched bit-exact"}
    # the same reference loop on this GPU's share of host cores (16 per GPU on
    # the box), independent buffers split over POSIX threads
    if ref is not None and hasattr(ref, "ref_crc32c_batch_mt"):
        threads = max(1, min(16, os.cpu_count() or 1))
        c_offs = np.ascontiguousarray(offs[:k], dtype=np.uint64)
        c_lens = np.ascontiguousarray(sizes[:k], dtype=np.uint32)
        mres = np.zeros(k, dtype=np.uint32)
        mreps = max(1, int(args.cpu_seconds / 3 * threads * rate1 * (1 << 30) / nbytes))
        t0 = time.perf_counter()
        rc = ref.ref_crc32c_batch_mt(base, c_offs.ctypes.data, c_lens.ctypes.data, mres.ctypes.data, k, threads,
                                     mreps)
        mdt = time.perf_counter() - t0
        if rc == 0 and np.array_equal(mres, res):
            line["multi_thread"] = {"value": round(nbytes * mreps / mdt / (1 << 30), 3), "unit": "GiB/s",
                                    "threads": threads, "passes": mreps, "seconds": round(mdt, 2)}
    # context row: the fastest CPU alternative, SSE4.2 `crc32` (3 streams;
    # oracle/crc32c_hw.c, bit-exact with the reference), same sample
    H = O.hw()
    if H is not None:
        threads = max(1, min(16, os.cpu_count() or 1))
        c_offs = np.ascontiguousarray(offs[:k], dtype=np.uint64)
        c_lens = np.ascontiguousarray(sizes[:k], dtype=np.uint32)
        hres = np.zeros(k, dtype=np.uint32)
        sse = {"unit": "GiB/s", "path": "x86 SSE4.2 crc32 instruction, 3 interleaved streams per buffer"}
        for nt in (1, threads):
            reps, el = 1, 0.0
            while True:  # about 1 s per thread count
                t0 = time.perf_counter()
                rc = H.hw_crc32c_batch_mt(base, c_offs.ctypes.data, c_lens.ctypes.data, hres.ctypes.data, k, nt,
                                          reps)
                el = time.perf_counter() - t0
                if rc != 0 or el >= 1.0 or reps >= 1 << 16:
                    break
                reps = max(reps * 2, int(reps * 1.2 / max(el, 1e-6)))
            if rc != 0 or not np.array_equal(hres, res):
                raise SystemExit("PARITY FAILURE: SSE4.2 context baseline differs from the reference")
            sse["value" if nt == 1 else "multi_thread"] = round(nbytes * reps / el / (1 << 30), 3)
        sse["threads"] = threads
        line["sse42"] = sse
    return line


if __name__ == "__main__":
    main()
