cd "${GRAFT_REPO_ROOT}"
V=norot AB_CONFIGS="c3 c4-1m c4-4m c4" bash tools/gpu_round.sh && \
SKIP_TESTS=1 AB_LIBS="pech_amd/libpech_crc32c.so build/lib_norot.so pech_amd/libpech_crc32c.so build/lib_norot.so" AB_CONFIGS="c3" bash tools/gpu_round.sh && \
bash tools/gpu_msgr_cpu.sh > gpurun_out/msgr_cpu_v17.txt 2>&1; tail -30 gpurun_out/msgr_cpu_v17.txt
