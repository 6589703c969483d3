#!/bin/bash
# A/B of bench.py lines (stream-ordered calls, the bench's own timing) under env settings.
# usage: tools/la_ab.sh <tag> "<settings>" "<matrices>" [steps]
#   a setting is VAR=value[,VAR=value] ("-" = none), e.g. "MHS_LAUNCH_AHEAD=0 MHS_LAUNCH_AHEAD=1"
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
tag=$1; sets=$2; ms=$3; steps=${4:-30}
out=gpurun_out/$tag; mkdir -p $out
for r in 1 2; do for m in $ms; do for st in $sets; do
  envs=""; [ "$st" != "-" ] && envs=$(echo $st | tr ',' ' ')
  v=$(echo $st | tr '@=,/' '____')
  env $envs timeout -k 10 300 python bench.py --no-cpu --steps $steps --warmup 3 --matrix $m > $out/${v}_${m}_$r.json 2>$out/${v}_${m}_$r.err || { echo "bench $v $m failed"; tail -5 $out/${v}_${m}_$r.err; exit 1; }
  python -c "
import json
d=json.loads(open('$out/${v}_${m}_$r.json').read().strip().splitlines()[-1])
print('%-28s r$r %-16s %9.1f %s  ms/step %.4f  numeric %.4f'%('$v','$m',d['value'],d['unit'],d['ms_per_step'],d.get('numeric_ms_avg') or -1))
"
done; done; done
echo ABDONE
