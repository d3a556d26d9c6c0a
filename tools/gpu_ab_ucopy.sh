#!/bin/bash
# fused copy block size A/B in the interleaved mode (v0.20: 12 rows)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SKIP_TESTS=1 AB_EXTRA="--op copy" AB_LIBS="pech_amd/libpech_crc32c.so build/lib_uc10.so build/lib_uc8.so build/lib_uc14.so pech_amd/libpech_crc32c.so build/lib_uc10.so build/lib_uc8.so build/lib_uc14.so" \
  AB_CONFIGS="c3" bash tools/gpu_round.sh
