#!/bin/bash
# PMC passes (one group per pass) on kernels matching $1 in `python tools/diag/run.py`.
# usage: tools/prof_pmc2.sh <kernel-regex> <tag> [groups-file]
export TMPDIR=/tmp
re=$1; tag=$2; gf=${3:-tools/pmc_groups_num.txt}
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "$re" --output-format csv \
     -d gpurun_out/pmc_${tag}_$i -o run -- python3 tools/diag/run.py mh-spgemm_amd/mhspgemm ${MATRIX:-cant} > gpurun_out/pmc_${tag}_$i.log 2>&1 || exit $?
done < "$gf"
