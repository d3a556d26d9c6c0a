#!/bin/bash
# SURVEY 8(d) per-size lines: the C4 classes as separate 256 MiB launches and the mixed 1 GiB launch
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/c4_classes.jsonl
for cfg in c4-4k c4-64k c4-1m c4-4m c4; do
  timeout -k 10 240 python bench.py --config $cfg --steps 30 --no-cpu-baseline --no-host-path > gpurun_out/cls_$cfg.log 2>&1 \
    || { tail -5 gpurun_out/cls_$cfg.log; exit 1; }
  tail -1 gpurun_out/cls_$cfg.log >> gpurun_out/c4_classes.jsonl
  echo "$cfg: $(tail -1 gpurun_out/cls_$cfg.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], r["kernel"], r["avg_launch_us"], r["frac"], d["serial"]["value"])')"
done
