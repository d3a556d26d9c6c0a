#!/bin/bash
# Where a lone payload's latency goes (GPU box): the unloaded msgr_sim bench at
# 64 KiB and 1 MiB under rocprofv3's kernel and memory-copy traces, and the
# same bench with the runtime's copies on blit kernels (HSA_ENABLE_SDMA=0).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
for size in ${SIZES:-65536 1048576}; do
  PECH_CRC32C_MSGR_HOST_MAX=0 timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats \
    -d "$R/gpurun_out/latprof_$size" -o run --output-format csv -- build/msgr_sim bench $size 1 2 300 \
    > gpurun_out/latprof_$size.log 2>&1 || { tail -20 gpurun_out/latprof_$size.log; exit 1; }
  for sd in 1 0; do
    r=$(HSA_ENABLE_SDMA=$sd PECH_CRC32C_MSGR_HOST_MAX=0 timeout -k 10 120 build/msgr_sim bench $size 1 2 300) || { echo "rc=$? $r"; exit 1; }
    echo "size $size sdma $sd: $(echo "$r" | tail -1)"
  done
done
