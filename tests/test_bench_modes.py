"""bench.py's two multi-GPU drivers emit the same JSON schema (GPU box):
torchrun's one process per GPU (here N=1) and pech's model, one host thread
driving every device (--single-thread), including two shards on one GPU
(--devices 0,0, the 1-GPU rehearsal of the loop)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMMON = ["--steps", "6", "--warmup", "2", "--no-cpu-baseline", "--no-host-path", "--sustain-seconds", "0.5"]


def run(*extra):
    r = subprocess.run([sys.executable, "bench.py", *COMMON, *extra], cwd=REPO, capture_output=True, timeout=240)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    return json.loads(r.stdout.decode().strip().splitlines()[-1])


def test_single_thread_matches_process_per_gpu_schema():
    # 30-step passes for the agreement check below (6-step passes are ~1 ms
    # of GPU time, where the Python loop's jitter shows)
    a = run("--steps", "30")
    b = run("--single-thread", "--gpus", "1", "--steps", "30")
    c = run("--single-thread", "--devices", "0,0")
    assert set(a) == set(b) and set(a["roofline"]) == set(b["roofline"])
    assert set(c) - set(a) == {"shards_checked", "buffers_checked"} and c["shards_checked"] == 2
    # every buffer of both shards' rotating batches checked
    assert c["buffers_checked"] == 2 * c["config"]["buffers_per_gpu"] * 2
    assert a["n_gpus"] == b["n_gpus"] == c["n_gpus"] == 1
    assert "single-thread" in b["config"]["parallelism"] and "single-thread" in c["config"]["parallelism"]
    # same work on one GPU: the two drivers agree within 10 % (VERDICT r05 #7,
    # ADVICE r5): per launch (the same kernels) and on the one-stream pass
    # (the host's issue loop included), each over 30 steps
    ka, kb = a["roofline"]["avg_launch_us"], b["roofline"]["avg_launch_us"]
    assert abs(ka - kb) / ka < 0.10, (ka, kb)
    sa, sb = a["serial"]["value"], b["serial"]["value"]
    assert abs(sa - sb) / sa < 0.10, (sa, sb)
    # two shards on one GPU share its HBM: about one GPU's rate in aggregate
    assert 0.7 < c["value"] / a["value"] < 1.3, (a["value"], c["value"])


def test_torchrun_two_ranks_real_kernels():
    """bench.py's N>1 driver under torchrun with the real kernels: two ranks
    share GPU 0 over gloo (PECH_BENCH_BACKEND=gloo; the driver's N>1 runs use
    RCCL with one GPU per rank).  Rendezvous, barriers, MAX-over-ranks timing
    and rank 0's single JSON line; each rank checksums its own shard and
    checks it against the oracle (shards_checked)."""
    env = dict(os.environ, PECH_BENCH_BACKEND="gloo")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29531", "bench.py", "--gpus", "2", *COMMON],
                       cwd=REPO, capture_output=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    lines = [l for l in r.stdout.decode().splitlines() if l.startswith("{")]
    assert len(lines) == 1, lines  # rank 0 only
    d = json.loads(lines[0])
    # n_gpus counts distinct devices: both ranks are on GPU 0
    assert d["n_gpus"] == 1 and d["ranks"] == 2 and d["scaling"] == "weak" and d["value"] > 0
    # each rank checked every buffer of its own shard against the oracle
    assert d["shards_checked"] == 2 and d["buffers_checked"] == 2 * d["config"]["buffers_per_gpu"] * 2
    assert d["config"]["parallelism"].startswith("shard2")
    assert "cpu_baseline" not in d  # rank 0 at N=1 only
    # per-rank evidence: every rank's own rate and launch
    # time, and which rank is slowest
    pr = d["per_rank"]
    assert sorted(r["rank"] for r in pr) == [0, 1] and all(r["value"] > 0 and r["avg_launch_us"] > 0 for r in pr)
    a = d["roofline"]["avg_launch_us_per_rank"]
    assert a["min"] <= a["max"] and a["argmax_rank"] in (0, 1)
    assert a["max"] == max(r["avg_launch_us"] for r in pr)
    v = d["value_per_rank"]
    assert v["min"] == min(r["value"] for r in pr) and v["max"] == max(r["value"] for r in pr)


def test_torchrun_rccl_process_group_one_rank():
    """The driver's N>1 runs use RCCL (backend "nccl") with one GPU per rank,
    which a one-GPU box cannot host for two ranks.  PECH_BENCH_FORCE_DIST=1
    runs the same process-group code at world size 1 on RCCL: init with the
    rank's device, barriers, the MAX all-reduce of the timing, the device
    gather behind n_gpus and the per-rank parity reduction."""
    env = dict(os.environ, PECH_BENCH_FORCE_DIST="1")
    env.pop("PECH_BENCH_BACKEND", None)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                        "--master-addr", "127.0.0.1", "--master-port", "29533", "bench.py", "--gpus", "1", *COMMON],
                       cwd=REPO, capture_output=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    lines = [l for l in r.stdout.decode().splitlines() if l.startswith("{")]
    assert len(lines) == 1, lines
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["ranks"] == 1 and d["shards_checked"] == 1 and d["value"] > 0
    assert d["buffers_checked"] == d["config"]["buffers_per_gpu"] * 2


def test_single_thread_eight_shards_on_one_gpu():
    """The 1-GPU rehearsal of pech's one thread driving 8 GPUs (VERDICT r3
    #4): --single-thread with 8 shards on device 0, every buffer of every
    shard checked against the oracle."""
    d = run("--single-thread", "--devices", ",".join(["0"] * 8))
    assert d["shards_checked"] == 8 and d["n_gpus"] == 1
    assert d["buffers_checked"] == 8 * d["config"]["buffers_per_gpu"] * 2
    assert d["value"] > 0
    # the one thread's issue time per step of 8 launches, beside the kernel time
    h = d["host_issue"]
    assert h["launches_per_step"] == 8 and h["issue_us_per_step"] > 0 and h["kernel_us_per_launch"] > 0
