# Parity + A/B after reverting the rank change and dropping the per-group verified atomics.
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
mkdir -p gpurun_out/r03za
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03za/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r03za/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r03za/pytest_gpu.log
for m in cant-perturbed cant; do
  timeout -k 10 300 python bench.py --matrix $m --no-cpu > gpurun_out/r03za/bench_$m.json 2> gpurun_out/r03za/bench_$m.err || { tail -20 gpurun_out/r03za/bench_$m.err; exit 1; }
  cut -c1-260 gpurun_out/r03za/bench_$m.json
done
bash tools/r02_ab.sh r03za_ab "base cur3" "cant-perturbed cant webbase-1M wb-edu cop20k_A pdb1HYS pwtk hood" 5 || exit 1
