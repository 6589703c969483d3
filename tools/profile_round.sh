#!/bin/bash
# rocprofv3 evidence for one round: kernel trace + stats of the bench command, then
# separate PMC passes (FETCH_SIZE, WRITE_SIZE) of the same command.  Writes under gpurun_out/<tag>/.
# usage: tools/profile_round.sh <tag> [bench args]
export TMPDIR=/tmp
tag=$1; shift
args=${*:-"--steps 10 --warmup 2 --no-cpu"}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py $args > $out/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- python3 bench.py $args > $out/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- python3 bench.py $args > $out/write.log 2>&1 || exit $?
echo done
