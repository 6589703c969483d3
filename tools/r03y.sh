# Parity of the count-ranked hash rows and the split block-bin launches, then their A/B.
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
mkdir -p gpurun_out/r03y
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03y/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r03y/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r03y/pytest_gpu.log
bash tools/r02_ab.sh r03y_ab "base rk split" "webbase-1M wb-edu cage15 cop20k_A scircuit cant-s1 pdb1HYS offshore cage12 mac_econ_fwd500" 5 || exit 1
