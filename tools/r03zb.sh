# Multi-stream timelines (webbase-1M, wb-edu, cant-perturbed: default streams) and SQ counter
# passes of the bench command (cant, cant-perturbed) on HEAD.
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
out=gpurun_out/r03zb; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
for m in webbase-1M cant-perturbed wb-edu; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/tl_$m -o run -- python3 tools/sweep.py $m --reps 5 > $out/tl_$m.log 2>&1 || { echo "trace $m failed"; tail -5 $out/tl_$m.log; exit 1; }
  echo "== $m trace"
done
bash tools/prof_sq.sh r03zb/sq_cant cant || exit 1
bash tools/prof_sq.sh r03zb/sq_cant-perturbed cant-perturbed || exit 1

bash tools/r02_ab.sh r03zb_ab "cur3 cur5 cur6" "webbase-1M wb-edu cage15 GAP-road cant cant-perturbed scircuit cant-s1" 5 || exit 1
