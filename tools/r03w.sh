# HEAD validation after the container re-creation: GPU suite, bench lines, a sweep of the
# BASELINE configs + the FEM variants, and the near-group A/B.
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
mkdir -p gpurun_out/r03w
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03w/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r03w/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r03w/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03w/smoke.log 2>&1 || { tail -20 gpurun_out/r03w/smoke.log; exit 1; }; tail -1 gpurun_out/r03w/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r03w/bench_default.json 2> gpurun_out/r03w/bench_default.err || { tail -20 gpurun_out/r03w/bench_default.err; exit 1; }
cat gpurun_out/r03w/bench_default.json | cut -c1-600
for m in cant-perturbed cant-s1; do
  timeout -k 10 300 python bench.py --matrix $m --no-cpu > gpurun_out/r03w/bench_$m.json 2> gpurun_out/r03w/bench_$m.err || { tail -20 gpurun_out/r03w/bench_$m.err; exit 1; }
  cut -c1-300 gpurun_out/r03w/bench_$m.json
done
timeout -k 10 600 python tools/sweep.py cant cant-s1 cant-perturbed webbase-1M mac_econ_fwd500 scircuit cop20k_A cage15 pdb1HYS pwtk cage12 hood rma10 shipsec1 offshore wb-edu GAP-road delaunay_n24 --reps 5 > gpurun_out/r03w/sweep.jsonl 2> gpurun_out/r03w/sweep.err || { tail -20 gpurun_out/r03w/sweep.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/r03w/sweep.jsonl'):
    d=json.loads(l); print('%-16s e2e %9.4f num %9.4f sym %8.4f gflops %8.1f'%(d['matrix'],d['total_e2e'],d['Numeric'],d['Calculate_C_nnz'],d['gflops_e2e']))
"
bash tools/r02_ab.sh r03w_near "base base@MHS_NO_NEAR=1" "cant-perturbed cant pwtk hood shipsec1" 5 || exit 1
