#!/bin/bash
# GPU box: release and bounds-checked GPU suites, then bench A/B of
# build/lib_HEAD.so against the current library on aligned and unaligned batches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
echo "release: $(tail -1 gpurun_out/pytest_gpu.log)"
PECH_CRC32C_LIB=build/lib_dbg.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_dbg.log 2>&1 || { tail -40 gpurun_out/pytest_dbg.log; exit 2; }
echo "dbg: $(tail -1 gpurun_out/pytest_dbg.log) oob=$(grep -c 'PECH OOB' gpurun_out/pytest_dbg.log)"
for pass in 1 2; do for cfg in ${CFGS:-c2-odd c2 c3 c4}; do for lib in build/lib_HEAD.so pech_amd/libpech_crc32c.so; do
  PECH_CRC32C_LIB=$lib timeout -k 10 150 python3 bench.py --config $cfg --steps 30 --no-cpu-baseline --no-host-path --sustain-seconds 2 > gpurun_out/ab_lg.log 2>&1 || { tail -5 gpurun_out/ab_lg.log; exit 3; }
  grep '^{' gpurun_out/ab_lg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$lib $cfg', d['value'], d['serial']['value'], r['avg_launch_us'], r['frac'], d['sustained']['value'])"
done; done; done
