#!/bin/bash
# A/B of variant libraries (ablib/<name>/libmhspgemm.so; "new" = the package's) on pipelined steps,
# two interleaved rounds.  usage: tools/ab_libs.sh <tag> "<variants>" "<matrices>" [suite]
#   suite: run the GPU test suite on the package's library first
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
tag=$1; V=$2; M=$3
out=gpurun_out/$tag; mkdir -p $out
if [ "$4" = suite ]; then
  timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -30 $out/pytest_gpu.log; exit 1; }
  tail -1 $out/pytest_gpu.log
fi
for r in 1 2; do
  for v in $V; do
    lib=""; [ $v != new ] && lib="--lib ablib/$v"
    timeout -k 10 400 python tools/pipe.py $M --reps 3 $lib > $out/${v}_$r.jsonl 2>> $out/err.log || { tail -5 $out/err.log; exit 1; }
  done
done
python3 tools/ab_pipe.py $out
for v in $V; do echo "$v numeric: $(cat $out/${v}_*.jsonl | python3 -c "
import sys, json, collections
d = collections.defaultdict(list)
for l in sys.stdin: j = json.loads(l); d[j['matrix']].append(j['numeric_ms'])
print(' '.join(f'{k[:8]} {min(x):.4f}' for k, x in d.items()))")"; done
echo ABDONE
