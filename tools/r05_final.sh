#!/bin/bash
# Round-5 evidence (1/2): GPU suite, smoke, default bench line, N=2 gloo rehearsal, and the bench
# command's rocprofv3 stats + FETCH/WRITE passes.
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
tag=$1; out=gpurun_out/$tag; mkdir -p $out
bash tools/gpu_check.sh $tag || exit 1
MHS_BENCH_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 \
  > $out/bench_n2_gloo.json 2> $out/bench_n2_gloo.err || { tail -20 $out/bench_n2_gloo.err; exit 1; }
cut -c1-600 $out/bench_n2_gloo.json
bash tools/bench_profile.sh $tag > $out/bench_profile.log 2>&1 || { tail -20 $out/bench_profile.log; exit 1; }
tail -8 $out/bench_profile.log
echo FINAL1DONE
