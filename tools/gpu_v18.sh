#!/bin/bash
# v0.18 check: GPU suite (release, bounds-checked), C4 per-class lines, async zero-copy threshold A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop() { echo "stopping after rc=$1 ($2)"; exit "$1"; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_rel.log 2>&1 || { tail -30 gpurun_out/pytest_rel.log; stop $? rel; }
echo "rel: $(tail -1 gpurun_out/pytest_rel.log)"
PECH_CRC32C_LIB=build/lib_dbg.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_dbg.log 2>&1 || { tail -30 gpurun_out/pytest_dbg.log; stop $? dbg; }
echo "dbg: $(tail -1 gpurun_out/pytest_dbg.log) oob=$(grep -c 'PECH OOB' gpurun_out/pytest_dbg.log)"
grep -q "PECH OOB" gpurun_out/pytest_dbg.log && stop 1 oob
: > gpurun_out/c4_classes.jsonl
for cfg in c4-4k c4-64k c4-1m c4-4m c4; do
  timeout -k 10 240 python bench.py --config $cfg --steps 30 --no-cpu-baseline --no-host-path > gpurun_out/cls_$cfg.log 2>&1 \
    || { tail -5 gpurun_out/cls_$cfg.log; stop $? "bench $cfg"; }
  tail -1 gpurun_out/cls_$cfg.log >> gpurun_out/c4_classes.jsonl
  echo "$cfg: $(tail -1 gpurun_out/cls_$cfg.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], r["kernel"], r["avg_launch_us"], r["frac"], d["serial"]["value"])')"
done
for zc in default 4294967295 default 4294967295; do
  env $([ $zc != default ] && echo PECH_ASYNC_ZC_MAX=$zc) SIZES="1048576 4194304" MODES="1 2" bash tools/gpu_msgr_cpu.sh \
    > gpurun_out/zc_$zc.txt 2>&1 || { tail -5 gpurun_out/zc_$zc.txt; stop 1 msgr; }
  echo "zc_max=$zc"; tail -4 gpurun_out/zc_$zc.txt
done
exit 0
