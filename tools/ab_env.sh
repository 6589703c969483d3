#!/bin/bash
# A/B of runtime switches on the package's library, pipelined steps, two interleaved rounds.
# usage: tools/ab_env.sh <tag> "<name>:<VAR=V[,VAR=V]> ..." "<matrices>"   (name "base": no switch)
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
tag=$1; V=$2; M=$3
out=gpurun_out/$tag; mkdir -p $out
for r in 1 2; do
  for v in $V; do
    name=${v%%:*}; envs=${v#*:}; [ "$name" = "$v" ] && envs=""
    ( [ -n "$envs" ] && export $(echo $envs | tr ',' ' ')
      timeout -k 10 400 python tools/pipe.py $M --reps 3 > $out/${name}_$r.jsonl 2>> $out/err.log ) || { tail -5 $out/err.log; exit 1; }
  done
done
python3 tools/ab_pipe.py $out
names=""; for v in $V; do names="$names ${v%%:*}"; done
for n in $names; do echo "$n numeric: $(cat $out/${n}_*.jsonl | python3 -c "
import sys, json, collections
d = collections.defaultdict(list)
for l in sys.stdin: j = json.loads(l); d[j['matrix']].append(j['numeric_ms'])
print(' '.join(f'{k[:8]} {min(x):.4f}' for k, x in d.items()))")"; done
echo ABDONE
