#!/bin/bash
# Round-3 profiling of one or more stand-ins on one GPU box, under gpurun_out/<tag>/<matrix>/:
#   trace/      kernel trace + stats of tools/sweep.py (numeric bins on ONE stream: attribution)
#   stamps.txt  per-row phase cycles of the numeric rows (tools/diag/v9, MHS_ROW_STAMPS build)
#   pmc_<k>/    counter passes (one rocprofv3 run per group, each under its own kill timer)
# usage: tools/prof_r03.sh <tag> "<matrices>" [stamps] [pmc groups "A,B;C,D" ...]
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth MHS_NUM_STREAMS=1
tag=$1; mats=$2; stamps=$3; groups=$4
out=gpurun_out/$tag; mkdir -p $out
for m in $mats; do
  d=$out/$m; mkdir -p $d
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d/trace -o run -- python3 tools/sweep.py $m --reps 5 > $d/sweep.log 2>&1 || { echo "trace $m failed"; exit 1; }
  echo "== $m trace"; tail -1 $d/sweep.log | cut -c1-400
  if [ "$stamps" = "stamps" ]; then
    timeout -k 10 300 python3 tools/diag/stamps2.py $m > $d/stamps.txt 2>&1 || { echo "stamps $m failed"; exit 1; }
    echo "== $m stamps"; head -30 $d/stamps.txt
  fi
  i=0
  IFS=';' read -ra G <<< "$groups"
  for g in "${G[@]}"; do
    [ -z "$g" ] && continue
    i=$((i+1))
    ctr=${g//,/ }
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d $d/pmc_$i -o run -- python3 tools/sweep.py $m --reps 2 > $d/pmc_$i.log 2>&1 || { echo "pmc $g $m failed"; exit 1; }
    echo "== $m pmc $g"
  done
done
echo ALLDONE
