#!/bin/bash
# GPU box: parity on the bounds-checked + release builds, stamps of the new
# prologue (c2, c3), then bench A/B of build/lib_HEAD.so (previous commit)
# against the current library over c2/c4/c3, two passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for c in c2 c3; do
  PECH_CRC32C_LIB=build/lib_stamps.so timeout -k 10 120 python tools/wave_stamps.py $c > gpurun_out/stamps_$c.txt 2>&1 || exit 2
  grep -E "span|prologue|start us|end   us|entry->|scan->|find->|plan->|fill->" gpurun_out/stamps_$c.txt
done
for pass in 1 2; do for lib in build/lib_HEAD.so pech_amd/libpech_crc32c.so; do for c in c2 c4 c3; do
 PECH_CRC32C_LIB=$lib timeout -k 10 150 python3 bench.py --config $c --steps 50 --no-cpu-baseline --no-host-path --sustain-seconds 2 > gpurun_out/ab_$c.log 2>&1 || exit 3
 tail -1 gpurun_out/ab_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$lib $c', d['value'], d['serial']['value'], r['avg_launch_us'], r['frac'], d['sustained']['value'])"
done; done; done
