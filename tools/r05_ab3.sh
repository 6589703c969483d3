#!/bin/bash
# A/B of per-wave pieces in the 1024-thread kernels and 4 tiles a lane per batch: pipelined step
# times (two interleaved rounds) + per-kernel durations (rocprofv3 stats, one matrix a run)
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
out=gpurun_out/r05ab3; mkdir -p $out
M="webbase-1M scircuit cop20k_A cant-s1 wb-edu"
for r in 1 2; do
  for v in base pieces tu4; do
    lib=""; [ $v != base ] && lib="--lib ablib/$v"
    timeout -k 10 300 python tools/pipe.py $M --reps 3 $lib > $out/${v}_$r.jsonl 2>> $out/err.log || { tail -5 $out/err.log; exit 1; }
  done
done
python3 tools/ab_pipe.py $out
for m in webbase-1M wb-edu; do
  for v in base pieces; do
    lib=""; [ $v != base ] && lib="--lib ablib/$v"
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/tr_${v}_$m -o run -- python3 tools/pipe.py $m --reps 1 --steps 10 $lib > $out/tr_${v}_$m.log 2>&1 || { echo "trace failed"; exit 1; }
    echo "== $v $m"; python3 tools/timeline.py "$(find $out/tr_${v}_$m -name '*kernel_trace.csv' | head -1)" | tail -22
  done
done
echo AB3DONE
