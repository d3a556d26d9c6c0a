#!/bin/bash
# SQ-level PMC passes of the main kernel (GPU box), each its own rocprofv3 run
# (<= 8 SQ counters per pass; never combined with trace domains), then a
# per-dispatch summary (tools/pmc_summary.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CFG=${CFG:-c3}
BENCH="bench.py --no-cpu-baseline --no-host-path --streams 1 --config $CFG --op ${OP:-crc} --steps 10 --warmup 2 --sustain-seconds 0"
i=0
for PMC in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
           ${SALU_PASS:+"SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_WAVES"}; do
  timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv -d gpurun_out/pmc_sq_${CFG}_$i -o run \
    -- python3 $BENCH > gpurun_out/pmc_sq_${CFG}_$i.log 2>&1 || { echo "pmc pass $i rc=$?"; exit 1; }
  i=$((i+1))
done
python3 tools/pmc_summary.py $(find gpurun_out/pmc_sq_${CFG}_* -name "*counter_collection.csv")
