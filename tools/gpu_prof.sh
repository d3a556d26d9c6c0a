#!/bin/bash
# rocprofv3 passes for the committed profiles (GPU box): kernel-trace stats of
# the serial bench pass, then PMC passes -- each its own run, --pmc never
# combined with sys/runtime traces.  FETCH_SIZE (+ WRITE_SIZE for the fused
# copy) -> gpurun_out/<cfg>_traffic.json (tools/pmc_traffic.py).
# CFGS entries: c3, c2, c4 ... or <cfg>-copy for the fused CRC + copy.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
stop() { echo "stopping after rc=$1 ($2)"; exit "$1"; }
TAG=$(python3 -c "import sys; sys.path.insert(0,'.'); import pech_amd as P; print(P.version())")
for C in ${CFGS:-c3}; do
  CFG=${C%-copy}; OP=crc; [ "$C" != "$CFG" ] && OP=copy
  BENCH="bench.py --no-cpu-baseline --no-host-path --streams 1 --config $CFG --op $OP"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${C}_trace -o run \
    -- python3 $BENCH --steps 20 > gpurun_out/prof_${C}_trace.log 2>&1 || stop $? "trace $C"
  tail -1 gpurun_out/prof_${C}_trace.log
  grep -h "pech_crc32c" $(find gpurun_out/prof_${C}_trace -name "*kernel_stats.csv") || true
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_${C}_fetch -o run \
    -- python3 $BENCH --steps 10 --warmup 2 > gpurun_out/prof_${C}_fetch.log 2>&1 || stop $? "pmc fetch $C"
  W=""
  if [ $OP = copy ]; then
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_${C}_write -o run \
      -- python3 $BENCH --steps 10 --warmup 2 > gpurun_out/prof_${C}_write.log 2>&1 || stop $? "pmc write $C"
    W=$(find gpurun_out/prof_${C}_write -name "*counter_collection.csv" | head -1)
  fi
  python3 tools/pmc_traffic.py $(find gpurun_out/prof_${C}_fetch -name "*counter_collection.csv" | head -1) \
    $C "$TAG" gpurun_out/${C}_traffic.json $W || echo "traffic json failed"
  python3 tools/trim_prof.py gpurun_out/prof_${C}_trace gpurun_out/prof_${C}_fetch gpurun_out/prof_${C}_write
  if [ -n "${SQ:-}" ]; then # SQ counter passes (one run each: VALU / LDS instructions, bank conflicts, waits;
    # SALU=1 adds the scalar pass) -> tools/pmc_summary.py; PECH_PMC_KERNEL picks the kernel
    i=0
    for PMC in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU" \
               "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
               ${SALU:+"SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_WAVES"}; do
      timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv -d gpurun_out/pmc_sq_${C}_$i -o run \
        -- python3 $BENCH --steps 10 --warmup 2 --sustain-seconds 0 > gpurun_out/pmc_sq_${C}_$i.log 2>&1 || stop $? "pmc sq $C $i"
      i=$((i+1))
    done
    python3 tools/pmc_summary.py $(find gpurun_out/pmc_sq_${C}_* -name "*counter_collection.csv") > gpurun_out/${C}_pmc_sq.json \
      && cat gpurun_out/${C}_pmc_sq.json
  fi
done
exit 0
