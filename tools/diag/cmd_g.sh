timeout -k 10 400 python -m pytest tests -q -m gpu -x > gpurun_out/t_grp.log 2>&1; tail -1 gpurun_out/t_grp.log
for m in cant; do MATRIX=$m RUNPY=tools/diag/run_phases.py tools/diag/ab.sh "grp||mh-spgemm_amd/mhspgemm" "nogrp|MHS_NO_GROUPS=1|mh-spgemm_amd/mhspgemm" | sed "s/^/$m /" >> gpurun_out/ab_grp.log 2>&1 || exit $?; done
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu > gpurun_out/b_grp.log 2>&1
