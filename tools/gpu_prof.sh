#!/bin/bash
# rocprofv3 passes for the committed profiles (GPU box): kernel-trace stats of
# the serial bench pass, then PMC passes -- each its own run, --pmc never
# combined with sys/runtime traces.  FETCH_SIZE -> gpurun_out/<cfg>_traffic.json
# (tools/pmc_traffic.py) for bench.py's roofline.traffic.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
BENCH="bench.py --no-cpu-baseline --no-host-path --pipeline-streams 0"
stop() { echo "stopping after rc=$1 ($2)"; exit "$1"; }
for CFG in ${CFGS:-c3}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${CFG}_trace -o run \
    -- python3 $BENCH --config $CFG --steps 20 > gpurun_out/prof_${CFG}_trace.log 2>&1 || stop $? "trace $CFG"
  tail -1 gpurun_out/prof_${CFG}_trace.log
  grep -h "pech_crc32c" $(find gpurun_out/prof_${CFG}_trace -name "*kernel_stats.csv") || true
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_${CFG}_fetch -o run \
    -- python3 $BENCH --config $CFG --steps 10 --warmup 2 > gpurun_out/prof_${CFG}_fetch.log 2>&1 || stop $? "pmc $CFG"
  TAG=$(python3 -c "import sys; sys.path.insert(0,'.'); import pech_amd as P; print(P.version())")
  python3 tools/pmc_traffic.py $(find gpurun_out/prof_${CFG}_fetch -name "*counter_collection.csv" | head -1) \
    $CFG "$TAG" gpurun_out/${CFG}_traffic.json || echo "traffic json failed"
  for PMC in ${EXTRA_PMC:-}; do
    timeout -s KILL 120 rocprofv3 --pmc ${PMC//,/ } --output-format csv -d gpurun_out/prof_${CFG}_${PMC%%,*} -o run \
      -- python3 $BENCH --config $CFG --steps 10 --warmup 2 > gpurun_out/prof_${CFG}_${PMC%%,*}.log 2>&1 \
      || stop $? "pmc $PMC"
  done
done
exit 0
