t0=$(date +%s); timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2> gpurun_out/bench_driver.err; rc=$?; echo "wall $(( $(date +%s) - t0 )) s rc=$rc"; [ $rc = 0 ] || exit $rc
for c in c4 c3 l32m l4m; do
  k=pech_crc32c_flat; [ $c = c4 ] && k=pech_crc32c_main
  SALU_PASS=1 CFG=$c PECH_PMC_KERNEL=$k bash tools/gpu_pmc_sq.sh > gpurun_out/pmc_$c.json 2> gpurun_out/pmc_$c.err || { echo "pmc $c failed"; tail -5 gpurun_out/pmc_$c.err; cat gpurun_out/pmc_$c.json | tail -5; exit 1; }
  echo "== $c"; cat gpurun_out/pmc_$c.json
done
