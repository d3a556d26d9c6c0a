#!/bin/bash
# A/B of kernel variants by rocprofv3 kernel-trace stats (GPU box): for every
# library in AB_LIBS and config in AB_CONFIGS, the serial bench pass under
# rocprofv3 --kernel-trace --stats; prints the plan / main average durations.
# A variant with wrong results (timing probes) ends with a parity failure
# (rc 1), which is tolerated; any other non-zero rc stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
# configs outer, libraries inner (alternating): clocks drift over minutes of
# load, so running one library's configs after the other's biased the A/B
for cfg in ${AB_CONFIGS:-c3}; do
  for lib in ${AB_LIBS:-pech_amd/libpech_crc32c.so}; do
    tag=$(basename $lib .so)_$cfg
    d=gpurun_out/abprof_$tag
    PECH_CRC32C_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run \
      -- python3 bench.py --config $cfg --streams 1 --steps ${AB_STEPS:-20} --no-cpu-baseline --no-host-path \
      --sustain-seconds ${AB_SUSTAIN:-0} ${AB_EXTRA:-} > $d.log 2>&1
    rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc ($tag)"; tail -5 $d.log; exit $rc; fi
    f=$(find $d -name "*kernel_stats.csv" | head -1)
    echo "$tag rc=$rc $(grep -h pech_crc32c_plan $f | cut -d, -f1,4) $(grep -h 'pech_crc32c_main' $f | cut -d, -f1,4 | tr '\n' ' ')"
  done
done
exit 0
