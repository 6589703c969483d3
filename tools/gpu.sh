#!/bin/bash
# One parametrised GPU driver (replaces the per-round tools/r05_*.sh scratch scripts).
#   tools/gpu.sh check <tag> [pytest -k expr]     GPU suite, smoke, default bench line
#   tools/gpu.sh ab <tag> "<matrices>" "<ENV=..>|<ENV=..>" [reps]
#                                                  pipelined steps (tools/pipe.py) per env variant,
#                                                  two interleaved rounds; "-" = the default env
#   tools/gpu.sh bench <tag> [bench.py args]      one bench.py line
#   tools/gpu.sh trace <tag> "<matrices>" ["ENV=.."]  kernel timelines of pipelined steps (rocprofv3)
#   tools/gpu.sh prof <tag> <matrix> [passes]     rocprofv3 kernel stats + FETCH/WRITE passes of
#                                                  bench.py --matrix <matrix> (tools/bench_profile.sh)
#   tools/gpu.sh sweep <tag> ["<matrices>"]       synchronised calls with per-phase events, median of 5,
#                                                  rocSPARSE beside them (tools/sweep.py), every stand-in
#   tools/gpu.sh hbm <tag>                        the HBM peak shapes of mhs_hbm.hip (per-shape rates)
# Every GPU step runs under its own timeout; the first failure ends the script.
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
mode=$1; tag=$2; out=gpurun_out/$tag; mkdir -p $out
case $mode in
check)
  bash tools/gpu_check.sh $tag "$3" || exit 1 ;;
ab)
  mats=$3; IFS='|' read -ra vars <<< "$4"; reps=${5:-3}
  for r in 1 2; do
    i=0
    for v in "${vars[@]}"; do
      envs=(); [ "$v" != "-" ] && read -ra envs <<< "$v"
      env "${envs[@]}" timeout -k 10 400 python tools/pipe.py $mats --reps $reps > $out/v${i}_$r.jsonl 2>> $out/err.log \
        || { tail -20 $out/err.log; exit 1; }
      i=$((i+1))
    done
  done
  python3 tools/pipe_table.py $out "$4" | tee $out/table.txt ;;
bench)
  shift 2
  timeout -k 10 600 python bench.py "$@" > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
  cut -c1-3000 $out/bench.json ;;
trace)
  # kernel timelines of pipelined steps: tools/gpu.sh trace <tag> "<matrices>" ["ENV=.. ENV=.."]
  envs=(); [ -n "$4" ] && read -ra envs <<< "$4"
  for m in $3; do
    env "${envs[@]}" timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $out/$m -o run -- python3 tools/pipe.py $m --reps 1 --steps 10 > $out/$m.log 2>&1 \
      || { echo "trace $m failed"; tail -5 $out/$m.log; exit 1; }
    python3 tools/timeline.py "$(find $out/$m -name '*kernel_trace.csv' | head -1)" > $out/$m/timeline.txt 2>&1
    echo "== $m $4"; cat $out/$m/timeline.txt
  done ;;
prof)
  bash tools/bench_profile.sh $tag "$3" "$4" > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
  tail -8 $out/prof.log ;;
sweep)
  mats=${3:-"cant cant-s1 cant-perturbed webbase-1M mac_econ_fwd500 scircuit cop20k_A cage15 pdb1HYS pwtk cage12 hood rma10 shipsec1 offshore wb-edu GAP-road delaunay_n24"}
  for m in $mats; do
    timeout -k 10 300 python3 tools/sweep.py $m --reps 5 --vendor >> $out/sweep_all.jsonl 2>> $out/sweep.err \
      || { echo "$m failed"; tail -5 $out/sweep.err; exit 1; }
    echo "$m done"
  done
  python3 tools/baseline_table.py $out/sweep_all.jsonl ;;
hbm)
  MHS_HBM_VERBOSE=1 timeout -k 10 200 python3 -c "
import sys; sys.path[:0]=['.','mh-spgemm_amd']
import mhspgemm; t=mhspgemm.Tool(0); print(t.hbm_peak(2<<30, 10)); t.close()" > $out/hbm.log 2>&1 || { tail -5 $out/hbm.log; exit 1; }
  grep -v amdgpu $out/hbm.log ;;
*)
  echo "usage: tools/gpu.sh check|ab|bench|trace|prof|sweep|hbm <tag> ..."; exit 2 ;;
esac
echo GPUDONE $mode $tag
