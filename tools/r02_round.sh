#!/bin/bash
# Round-2 evidence of HEAD: bench lines, all-matrix sweep, rocprofv3 stats + PMC of the
# bench command, per-config kernel traces + FETCH/WRITE passes.  usage: tools/r02_round.sh <tag> <part>
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
tag=$1; part=$2; out=gpurun_out/$tag; mkdir -p $out
if [ "$part" = "1" ]; then
  timeout -k 10 240 python bench.py > $out/bench_default.json 2> $out/bench_default.err || { echo "bench failed"; tail $out/bench_default.err; exit 1; }
  cat $out/bench_default.json
  for m in cant-s1 cant-perturbed; do
    timeout -k 10 240 python bench.py --matrix $m > $out/bench_$m.json 2> $out/bench_$m.err || { echo "bench $m failed"; exit 1; }
    cut -c1-300 $out/bench_$m.json
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/bench_trace -o run -- python3 bench.py --no-cpu > $out/bench_trace.log 2>&1 || { echo "bench trace failed"; exit 1; }
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $out/bench_fetch -o run -- python3 bench.py --no-cpu > $out/bench_fetch.log 2>&1 || { echo "bench fetch failed"; exit 1; }
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $out/bench_write -o run -- python3 bench.py --no-cpu > $out/bench_write.log 2>&1 || { echo "bench write failed"; exit 1; }
  echo PART1DONE
fi
if [ "$part" = "2" ]; then
  timeout -k 10 700 python tools/sweep.py cant cant-s1 cant-perturbed webbase-1M mac_econ_fwd500 scircuit cop20k_A cage15 pdb1HYS pwtk cage12 hood rma10 shipsec1 offshore wb-edu GAP-road delaunay_n24 --reps 5 --vendor > $out/sweep_all.jsonl 2> $out/sweep_all.err || { echo "sweep failed"; tail -5 $out/sweep_all.err; exit 1; }
  echo SWEEPDONE
  MHS_NUM_STREAMS=1 bash tools/prof_r02.sh $tag "cant webbase-1M mac_econ_fwd500 scircuit cop20k_A cage15" pmc || exit $?
  echo PART2DONE
fi
