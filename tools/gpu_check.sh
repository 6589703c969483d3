#!/bin/bash
# GPU suite + smoke + default bench line of the current tree, under gpurun_out/<tag>/.
# usage: tools/gpu_check.sh <tag> [pytest -k expression]
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
tag=$1; kexpr=$2; out=gpurun_out/$tag; mkdir -p $out
if [ -n "$kexpr" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$kexpr" > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
fi
tail -1 $out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 400 python bench.py > $out/bench_default.json 2> $out/bench_default.err || { echo "bench failed"; tail $out/bench_default.err; exit 1; }
cut -c1-1500 $out/bench_default.json
echo CHECKDONE
