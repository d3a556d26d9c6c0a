#!/bin/bash
# Perf session on the GPU box: HBM probes, bench A/B over library builds,
# rocprofv3 kernel-trace stats.  Each GPU step time-limited; stop on fault.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
stop() { echo "stopping after rc=$1 ($2)"; exit "$1"; }
if [ -x build/hbm_probe ]; then
  timeout -k 10 120 build/hbm_probe > gpurun_out/hbm_probe.json 2>&1 || stop $? probe
  cat gpurun_out/hbm_probe.json
fi
for lib in ${AB_LIBS:-}; do
  for cfg in ${AB_CONFIGS:-c3}; do
    PECH_CRC32C_LIB=$lib timeout -k 10 240 python bench.py --config $cfg --steps 30 --no-cpu-baseline \
      > gpurun_out/ab_$(basename $lib .so)_$cfg.log 2>&1 || stop $? "bench $lib $cfg"
    echo "$lib $cfg: $(tail -1 gpurun_out/ab_$(basename $lib .so)_$cfg.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["achieved"], d["roofline"]["frac"], d["ms_per_step"])')"
  done
done
if [ -n "${PROF_CONFIGS:-}" ]; then
  for cfg in $PROF_CONFIGS; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$cfg -o run \
      -- python3 bench.py --config $cfg --steps 20 --no-cpu-baseline > gpurun_out/prof_$cfg.log 2>&1 || stop $? "rocprof $cfg"
    find gpurun_out/prof_$cfg -name "*stats*" | head
  done
fi
exit 0
