#!/bin/bash
# GPU box: GPU tests, then plan/main kernel durations (rocprofv3 stats) on
# unaligned (c2-odd) and aligned (c2) batches for build/lib_HEAD.so vs the
# current library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for cfg in ${CFGS:-c2-odd c2}; do for lib in build/lib_HEAD.so pech_amd/libpech_crc32c.so; do
  o=gpurun_out/prof_plan_${cfg}_$(basename $lib .so)
  PECH_CRC32C_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o -o run \
    -- python3 bench.py --config $cfg --no-cpu-baseline --no-host-path --steps 30 --sustain-seconds 2 > $o.log 2>&1 || { tail -5 $o.log; exit 2; }
  tail -1 $o.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$cfg $lib', 'value', d['value'], 'serial', d['serial']['value'], 'main_us', r['avg_launch_us'])"
  grep -h "pech_crc32c" $(find $o -name "*kernel_stats.csv") | cut -d, -f1-4
done; done
