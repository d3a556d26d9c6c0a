#!/bin/bash
# GPU box: A/B of kernel builds on the sustained two-stream rate (bench.py's
# `sustained`, seconds of the value pass: less noisy than the 30-step value),
# passes interleaved.  AB_LIBS, AB_CONFIGS, PASSES, SUSTAIN.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for p in $(seq 1 ${PASSES:-2}); do for cfg in ${AB_CONFIGS:-c3}; do for lib in ${AB_LIBS:-pech_amd/libpech_crc32c.so}; do
  PECH_CRC32C_LIB=$lib timeout -k 10 200 python3 bench.py --config $cfg --steps 30 --no-cpu-baseline --no-host-path \
    --sustain-seconds ${SUSTAIN:-4} > gpurun_out/ab_sustain.log 2>&1 || { tail -5 gpurun_out/ab_sustain.log; exit 3; }
  tail -1 gpurun_out/ab_sustain.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$lib $cfg sustained', d['sustained']['value'], 'value', d['value'], 'serial', d['serial']['value'], 'launch_us', r['avg_launch_us'])"
done; done; done
