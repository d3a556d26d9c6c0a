#!/bin/bash
# A/B of the uniform pool on small shares (256 MiB launches of 64 KiB-4 MiB buffers: 512-row shares)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SKIP_TESTS=1 AB_LIBS="pech_amd/libpech_crc32c.so build/lib_pmin1k.so build/lib_nopool.so pech_amd/libpech_crc32c.so build/lib_pmin1k.so build/lib_nopool.so" \
  AB_CONFIGS="${AB_CONFIGS:-c4-64k c4-1m c4-4m c3}" bash tools/gpu_round.sh
