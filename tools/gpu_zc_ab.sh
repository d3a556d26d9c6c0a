#!/bin/bash
# zero-copy threshold A/B with 1 GiB passes (DMA mode, zero-copy default 1 MiB, zero-copy for all), plus the window probes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 180 build/sched_probe 10 window > gpurun_out/probe_window2.json 2>&1 || { cat gpurun_out/probe_window2.json; exit 1; }
cat gpurun_out/probe_window2.json
for rep in 1 2; do for zc in default 4294967295; do
  env $([ $zc != default ] && echo PECH_ASYNC_ZC_MAX=$zc) BYTES_PER_PASS=1073741824 SIZES="1048576 4194304" MODES="0 1 2" bash tools/gpu_msgr_cpu.sh \
    > gpurun_out/zc1g_${zc}_$rep.txt 2>&1 || { tail -5 gpurun_out/zc1g_${zc}_$rep.txt; exit 1; }
  echo "zc_max=$zc rep $rep"; tail -6 gpurun_out/zc1g_${zc}_$rep.txt
done; done
timeout -k 10 240 python bench.py --config c2 --steps 30 --no-cpu-baseline --no-host-path > gpurun_out/bench_c2.log 2>&1 || { tail -5 gpurun_out/bench_c2.log; exit 1; }
tail -1 gpurun_out/bench_c2.log
CFG=c2 PECH_PMC_KERNEL=pech_crc32c_direct bash tools/gpu_pmc_sq.sh > gpurun_out/pmc_sq_c2_direct.json 2>&1; cat gpurun_out/pmc_sq_c2_direct.json
