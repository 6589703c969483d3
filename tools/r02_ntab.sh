export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
bash tools/r02_ab.sh r02zf "ntall cur" "cant cant-perturbed mac_econ_fwd500 GAP-road cop20k_A" 3 || exit 1
for v in ntall cur; do
  MHS_LIB=$PWD/tools/var/$v/libmhspgemm.so timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/r02zf/w_$v -o run -- python3 tools/sweep.py cant --reps 2 > gpurun_out/r02zf/w_$v.log 2>&1 || exit 1
done
echo NTDONE
