#!/bin/bash
# v0.30c A/B: share divisions in double precision on the VALU against 64-bit integer ones (build/lib_divint.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_flat.py tests/test_gpu_parity.py tests/test_gpu_direct.py > gpurun_out/t_div.log 2>&1 || { tail -30 gpurun_out/t_div.log; exit 1; }
tail -1 gpurun_out/t_div.log
LIBS="pech_amd/libpech_crc32c.so build/lib_divint.so" REPS=3 bash tools/gpu_ab_curve.sh 2>&1 | grep -v amdgpu | tail -6 || exit 1
SKIP_TESTS=1 AB_LIBS="pech_amd/libpech_crc32c.so build/lib_divint.so" AB_CONFIGS="c3 c4 c2" PASSES=2 bash tools/gpu_round.sh > gpurun_out/round_div.txt 2>&1 || { tail -5 gpurun_out/round_div.txt; exit 1; }
grep "^lib" gpurun_out/round_div.txt
for L in pech_amd/libpech_crc32c.so build/lib_divint.so; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVES --output-format csv -d gpurun_out/pmc_div_$(basename $L .so) -o run \
    -- python3 bench.py --no-cpu-baseline --no-host-path --streams 1 --config l4m --steps 10 --warmup 2 --sustain-seconds 0 > /dev/null 2>&1 || { echo "pmc failed"; exit 1; }
  echo "$L $(PECH_PMC_KERNEL=pech_crc32c_flat python3 tools/pmc_summary.py $(find gpurun_out/pmc_div_$(basename $L .so) -name '*counter_collection.csv') | tr -d '\n ')"
done
