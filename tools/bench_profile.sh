#!/bin/bash
# Round evidence of the bench command: rocprofv3 --kernel-trace --stats of the default
# `python3 bench.py` (its stats split into the headline and configs parts by
# tools/bench_kernel_stats.py), then FETCH_SIZE and WRITE_SIZE of the headline's launches in
# separate --pmc passes (bench.py --no-cpu --no-configs: the same headline calls).
# usage: tools/bench_profile.sh <tag>
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
tag=$1; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $out/bench_trace -o run -- python3 bench.py > $out/bench_trace.log 2>&1 || { echo "bench trace failed"; tail -5 $out/bench_trace.log; exit 1; }
grep '^{' $out/bench_trace.log | tail -1 | cut -c1-600
tr=$(find $out/bench_trace -name '*kernel_trace.csv' | head -1)
python3 tools/bench_kernel_stats.py "$tr" $out/bench_trace 3 20
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $out/bench_$c -o run -- python3 bench.py --no-cpu --no-configs > $out/bench_$c.log 2>&1 || { echo "bench $c failed"; exit 1; }
  echo "== $c ok"
done
echo BENCHPROFDONE
