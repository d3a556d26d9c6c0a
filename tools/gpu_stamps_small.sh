cd "${GRAFT_REPO_ROOT}"
for cfg in 1x4m 8x4m; do
  PECH_CRC32C_LIB=build/lib_stamps.so timeout -k 10 120 python tools/wave_stamps.py $cfg > gpurun_out/st_$cfg.txt 2>&1 || { cat gpurun_out/st_$cfg.txt; exit 1; }
  echo "== $cfg"; grep -v "amdgpu.ids\|^xcc\|histogram" gpurun_out/st_$cfg.txt
  PECH_STAMP_FIN=1 PECH_CRC32C_LIB=build/lib_stfin.so timeout -k 10 120 python tools/wave_stamps.py $cfg > gpurun_out/stfin_$cfg.txt 2>&1 || { cat gpurun_out/stfin_$cfg.txt; exit 1; }
  echo "== fin $cfg"; grep -i "fold\|flush\|planned\|start->" gpurun_out/stfin_$cfg.txt
done
