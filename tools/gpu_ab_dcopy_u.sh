#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SKIP_TESTS=1 AB_EXTRA="--op copy --api small" AB_LIBS="pech_amd/libpech_crc32c.so build/lib_dc6.so build/lib_dc10.so pech_amd/libpech_crc32c.so build/lib_dc6.so build/lib_dc10.so" \
  AB_CONFIGS="c2 c2-odd" bash tools/gpu_round.sh
