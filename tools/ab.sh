#!/bin/bash
# A/B of library variants (tools/var/<v>/libmhspgemm.so): sweep lines per matrix, two interleaved rounds.
# usage: tools/ab.sh <tag> "<variants>" "<matrices>" [reps]
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
tag=$1; vs=$2; ms=$3; reps=${4:-7}
out=gpurun_out/$tag; mkdir -p $out
# a variant is <dir>[@VAR=value[,VAR=value]]: tools/var/<dir>/libmhspgemm.so (or <dir> itself when it
# holds a '/', e.g. abvar/base or mh-spgemm_amd/mhspgemm for the tree's own) run under those env vars
for r in 1 2; do for spec in $vs; do
  lib=${spec%%@*}; envs=""; [ "$spec" != "$lib" ] && envs=$(echo ${spec#*@} | tr ',' ' ')
  libdir=$lib; [[ "$lib" != */* ]] && libdir=tools/var/$lib
  v=$(echo $spec | tr '@=,/' '____')
  env $envs timeout -k 10 300 python tools/sweep.py $ms --reps $reps --lib $libdir > $out/ab_${v}_$r.jsonl 2>$out/ab_${v}_$r.err || { echo "sweep $v failed"; tail -5 $out/ab_${v}_$r.err; exit 1; }
  python -c "
import json,sys
for l in open('$out/ab_${v}_$r.jsonl'):
    d=json.loads(l); print('%-8s r$r %-16s e2e %9.4f num %9.4f sym %8.4f gflops %8.1f'%('$v',d['matrix'],d['total_e2e'],d['Numeric'],d['Calculate_C_nnz'],d['gflops_e2e']))
"
done; done
echo ABDONE
