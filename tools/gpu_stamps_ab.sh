cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for c in c2-1g c4; do
  PECH_CRC32C_LIB=build/lib_stamps.so timeout -k 10 120 python tools/wave_stamps.py $c > gpurun_out/stamps_new_$c.txt 2>&1 || exit 2
  echo "== new $c"; grep -E "span|busy us|end   us|prologue|slot" gpurun_out/stamps_new_$c.txt
  PECH_CRC32C_LIB=build/lib_stamps_HEAD.so timeout -k 10 120 python tools/wave_stamps.py $c > gpurun_out/stamps_old_$c.txt 2>&1 || exit 3
  echo "== old $c"; grep -E "span|busy us|end   us|prologue|slot" gpurun_out/stamps_old_$c.txt
done
