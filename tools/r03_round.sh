#!/bin/bash
# Round-3 evidence of HEAD: part 1 = GPU suite + smoke, then tools/r02_round.sh part 1 (bench
# lines, rocprofv3 stats + FETCH/WRITE of the bench command); part 2 = r02_round.sh part 2
# (18-matrix sweep with rocSPARSE, per-config kernel traces + FETCH/WRITE passes).
# usage: tools/r03_round.sh <tag> <part>
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
tag=$1; part=$2; out=gpurun_out/$tag; mkdir -p $out
if [ "$part" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
  tail -1 $out/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
  tail -1 $out/smoke.log
fi
bash tools/r02_round.sh $tag $part
