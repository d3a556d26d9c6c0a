#!/bin/bash
# Messenger-side CPU cost per payload (GPU box): build/msgr_sim bench at the
# C1/C4 payload sizes, async DMA / zero-copy, the adapter, the host routine.
# One JSON line per (size, mode) -> gpurun_out/msgr_cpu.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/msgr_cpu.jsonl
for size in ${SIZES:-4096 16384 65536 262144 1048576 4194304}; do
  count=$(( ${BYTES_PER_PASS:-268435456} / size )); [ $count -gt 16384 ] && count=16384
  for mode in ${MODES:-0 1 2 3}; do
    timeout -k 10 120 build/msgr_sim bench $size $count $mode ${PASSES:-3} >> gpurun_out/msgr_cpu.jsonl || { echo "msgr_sim rc=$? size $size mode $mode"; exit 1; }
  done
done
python3 - <<'PY'
import json
rows=[json.loads(l) for l in open("gpurun_out/msgr_cpu.jsonl")]
print("%9s %-15s %9s %12s %10s %10s %9s %9s" % ("bytes","mode","GiB/s","payloads/s","thr us/p","proc us/p","lat p50","lat p99"))
for r in rows:
    print("%9d %-15s %9.2f %12.0f %10.3f %10.3f %9.1f %9.1f" % (r["payload_bytes"], r["mode"], r["GiBps"], r["payloads_per_s"],
          r["thread_cpu_us_per_payload"], r["process_cpu_us_per_payload"], r["latency_us_p50"], r["latency_us_p99"]))
PY
