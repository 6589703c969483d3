# usage: bash tools/diag/cmp_wpe.sh lib_dir... (sweeps the non-FEM matrices with each library build)
for v in "$@"; do
  timeout -k 10 250 python -u tools/sweep.py cant cop20k_A mac_econ_fwd500 scircuit webbase-1M cage15 --reps 10 --lib $v > gpurun_out/cmp_$(basename $v).log 2>&1 || exit 1
done
