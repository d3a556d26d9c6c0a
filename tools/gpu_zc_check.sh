cd "${GRAFT_REPO_ROOT}"
bash tools/gpu_async_check.sh && BYTES_PER_PASS=1073741824 SIZES="1048576 4194304" MODES="0 1 2" bash tools/gpu_msgr_cpu.sh > gpurun_out/msgr_cpu_1g.txt 2>&1; tail -7 gpurun_out/msgr_cpu_1g.txt
