#!/bin/bash
# One GPU-box validation + A/B session: bounds-checked debug build over the
# GPU tests (OOB loads print instead of faulting), the release GPU tests,
# stamps, then bench A/B.  Each GPU step time-limited; stop on fault.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop() { echo "stopping after rc=$1 ($2)"; exit "$1"; }
if [ -z "${SKIP_TESTS:-}" ]; then
env ${TEST_ENV:-} PECH_CRC32C_LIB=build/lib_dbg.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_dbg.log 2>&1 || { tail -30 gpurun_out/pytest_dbg.log; stop $? dbg; }
echo "dbg: $(tail -1 gpurun_out/pytest_dbg.log) oob=$(grep -c 'PECH OOB' gpurun_out/pytest_dbg.log)"
grep -q "PECH OOB" gpurun_out/pytest_dbg.log && stop 1 oob
env ${TEST_ENV:-} timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; stop $? pytest; }
echo "release: $(tail -1 gpurun_out/pytest_gpu.log)"
fi
for cfg in ${STAMP_CONFIGS:-}; do
  PECH_CRC32C_LIB=${STAMP_LIB:-build/lib_stamps.so} timeout -k 10 120 python tools/wave_stamps.py $cfg > gpurun_out/stamps_$cfg.txt 2>&1 \
    || stop $? "stamps $cfg"
  grep -v "amdgpu.ids\|^xcc\|histogram" gpurun_out/stamps_$cfg.txt
done
# columns: value (2-stream pass) GiB/s, main GB/s, roofline frac, main us, serial (1-stream) GiB/s,
# sustained GiB/s (with AB_EXTRA="--sustain-seconds 4"); AB_EXTRA="--op copy" A/Bs the fused copy
# AB_ENVS: space-separated variants, each a comma-separated VAR=value list ("-" = none)
for pass in $(seq 1 ${PASSES:-1}); do
for ev in ${AB_ENVS:--}; do
for lib in ${AB_LIBS:-pech_amd/libpech_crc32c.so}; do
  for cfg in ${AB_CONFIGS:-c3}; do
    o=gpurun_out/ab_$(basename $lib .so)_${ev//[=,]/_}_$cfg.log
    envs=""; [ "$ev" != - ] && envs=${ev//,/ }
    env $envs PECH_CRC32C_LIB=$lib timeout -k 10 240 python bench.py --config $cfg --steps 30 --no-cpu-baseline --no-host-path \
      ${AB_EXTRA:-} > $o 2>&1 || { tail -5 $o; stop $? "bench $lib $cfg"; }
    echo "$(basename $lib) $ev $cfg: $(tail -1 $o | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], r["achieved"], r["frac"], r["avg_launch_us"], d.get("serial", {}).get("value"), d.get("sustained", {}).get("value"))')"
  done
done
done
done
exit 0
