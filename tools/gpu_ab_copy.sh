#!/bin/bash
# GPU box: fused CRC + copy A/B over kernel revisions (build/lib_<rev>.so vs
# the current library), two interleaved passes, C3 shape.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for pass in 1 2; do for lib in ${AB_LIBS:-build/lib_86747c5.so build/lib_588d846.so pech_amd/libpech_crc32c.so}; do
  PECH_CRC32C_LIB=$lib timeout -k 10 150 python3 bench.py --config ${CFG:-c3} --op copy --steps 30 --no-cpu-baseline --no-host-path --sustain-seconds 2 \
    ${AB_EXTRA:-} > gpurun_out/ab_copy.log 2>&1 || { tail -5 gpurun_out/ab_copy.log; exit 3; }
  tail -1 gpurun_out/ab_copy.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$lib', d['value'], d['serial']['value'], r['avg_launch_us'], r['frac'], r.get('probe', {}).get('us_per_launch'))"
done; done
