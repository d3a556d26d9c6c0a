cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for cfg in 1x4m 8x4m 64x4m c3; do
  PECH_CRC32C_LIB=build/lib_stamps.so timeout -k 10 120 python tools/wave_stamps.py $cfg > gpurun_out/st_flat_$cfg.txt 2>&1 || { cat gpurun_out/st_flat_$cfg.txt; exit 1; }
  echo "== flat $cfg"; grep -v "amdgpu.ids\|^xcc\|histogram" gpurun_out/st_flat_$cfg.txt
done
for cfg in 1x4m 8x4m; do
  PECH_FLAT_MAX=0 PECH_CRC32C_LIB=build/lib_stamps.so timeout -k 10 120 python tools/wave_stamps.py $cfg > gpurun_out/st_plan_$cfg.txt 2>&1 || { cat gpurun_out/st_plan_$cfg.txt; exit 1; }
  echo "== planned $cfg"; grep -v "amdgpu.ids\|^xcc\|histogram" gpurun_out/st_plan_$cfg.txt
done
for cfg in 1x4m 8x4m c3; do
  PECH_STAMP_FIN=1 PECH_CRC32C_LIB=build/lib_stfin.so timeout -k 10 120 python tools/wave_stamps.py $cfg > gpurun_out/stfin_flat_$cfg.txt 2>&1 || { cat gpurun_out/stfin_flat_$cfg.txt; exit 1; }
  echo "== stfin flat $cfg"; grep -v "amdgpu.ids\|^xcc\|histogram" gpurun_out/stfin_flat_$cfg.txt
done
