#!/bin/bash
# Round-end validation on one box: the GPU suite on the bounds-checked and the release builds, smoke(), and the driver's
# bench command with its wall time (each step time-limited; the first failure ends the script)
# PART=dbg / PART=release: one half per gpurun call (each call is capped at 20 minutes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${PART:-dbg}" = dbg ]; then
PECH_CRC32C_LIB=build/lib_dbg.so timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread \
  > gpurun_out/pytest_dbg.log 2>&1 || { tail -30 gpurun_out/pytest_dbg.log; exit 1; }
echo "dbg: $(tail -1 gpurun_out/pytest_dbg.log) oob=$(grep -c 'PECH OOB' gpurun_out/pytest_dbg.log)"
grep -q "PECH OOB" gpurun_out/pytest_dbg.log && exit 1
[ -z "${PART:-}" ] || exit 0
fi
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
  || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
echo "release: $(tail -1 gpurun_out/pytest_gpu.log)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log | cut -c1-200
t0=$(date +%s)
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2> gpurun_out/bench_driver.err \
  || { tail -20 gpurun_out/bench_driver.err; exit 1; }
echo "bench wall $(( $(date +%s) - t0 )) s"
tail -1 gpurun_out/bench_driver.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], r['avg_launch_us'], r['frac'], r['traffic'], d['serial']['value'], d['sustained']['value'], d['cpu_baseline']['value'])"
