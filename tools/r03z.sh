# Parity + A/B: count-ranked hash rows, block bins split by LDS need (off: MHS_NO_SPLIT=1),
# near union runs of B (A*A; off with MHS_NO_NEAR=1 together with the near groups).
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
mkdir -p gpurun_out/r03z
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03z/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r03z/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r03z/pytest_gpu.log
bash tools/r02_ab.sh r03z_ab "base cur2 cur2@MHS_NO_SPLIT=1" "cant-perturbed cant webbase-1M wb-edu cage15 cop20k_A scircuit cant-s1 pdb1HYS offshore" 5 || exit 1
