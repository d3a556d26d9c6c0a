#!/bin/bash
# rocprofv3 passes for the committed profiles: kernel-trace stats, then PMC
# passes (each its own run; --pmc never combined with sys/runtime traces).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CFG=${CFG:-c3}
stop() { echo "stopping after rc=$1 ($2)"; exit "$1"; }
if [ -x build/hbm_probe ]; then
  timeout -k 10 120 build/hbm_probe > gpurun_out/hbm_probe.json 2>&1 || stop $? probe
  cat gpurun_out/hbm_probe.json
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${CFG}_trace -o run \
  -- python3 bench.py --config $CFG --steps 20 --no-cpu-baseline > gpurun_out/prof_${CFG}_trace.log 2>&1 || stop $? trace
for PMC in "${PMC1:-FETCH_SIZE}" "${PMC2:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU}" "${PMC3:-SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE}"; do
  tag=$(echo $PMC | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $PMC --output-format csv -d gpurun_out/prof_${CFG}_$tag -o run \
    -- python3 bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_${CFG}_$tag.log 2>&1 \
    || echo "pmc pass '$PMC' rc=$? (see log)"
done
ls -R gpurun_out | grep -i csv | head -20
exit 0
