#!/bin/bash
# A/B: numeric-first without the probe (MHS_NFT_AUTO_AVG) and the direct-mapped preference
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
out=gpurun_out/r05ab1; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -30 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
M="mac_econ_fwd500 scircuit cop20k_A webbase-1M cant cant-perturbed cage12 offshore"
for r in 1 2; do
  MHS_NFT_AUTO_AVG=0 timeout -k 10 300 python tools/pipe.py $M --reps 3 > $out/base_$r.jsonl 2>> $out/err.log || exit 1
  timeout -k 10 300 python tools/pipe.py $M --reps 3 > $out/nft_$r.jsonl 2>> $out/err.log || exit 1
  timeout -k 10 300 python tools/pipe.py $M --reps 3 --lib ablib/dirpref > $out/dir_$r.jsonl 2>> $out/err.log || exit 1
done
python3 - <<'PY'
import json,glob
out="gpurun_out/r05ab1"
res={}
for f in sorted(glob.glob(out+"/*_?.jsonl")):
    tag=f.split("/")[-1].rsplit("_",1)[0]
    for l in open(f):
        d=json.loads(l); res.setdefault(d["matrix"],{}).setdefault(tag,[]).append(d["ms"])
for m,v in res.items():
    print(f"{m:18s}", "  ".join(f"{k} {min(x):.4f}" for k,x in sorted(v.items())))
PY
echo AB1DONE
