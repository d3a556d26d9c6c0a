mkdir -p gpurun_out
PECH_CRC32C_LIB=build/lib_dbgnew.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_dbgnew.log 2>&1 || { tail -20 gpurun_out/pytest_dbgnew.log; exit 1; }
echo "dbg: $(tail -1 gpurun_out/pytest_dbgnew.log) oob=$(grep -c 'PECH OOB' gpurun_out/pytest_dbgnew.log)"
grep -q "PECH OOB" gpurun_out/pytest_dbgnew.log && exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/pytest_gpu.log; exit 1; }
echo "release: $(tail -1 gpurun_out/pytest_gpu.log)"
SKIP_TESTS=1 AB_LIBS="build/lib_HEAD.so pech_amd/libpech_crc32c.so build/lib_HEAD.so pech_amd/libpech_crc32c.so" AB_CONFIGS="c3 c4 c4-4m c2" bash tools/gpu_round.sh
