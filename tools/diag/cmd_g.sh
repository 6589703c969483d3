timeout -k 10 400 python -m pytest tests -q -m gpu -x > gpurun_out/t_side.log 2>&1; tail -1 gpurun_out/t_side.log
for m in cant cop20k_A webbase-1M; do MATRIX=$m RUNPY=tools/diag/run_phases.py tools/diag/ab.sh "side||mh-spgemm_amd/mhspgemm" "noside|MHS_NO_SIDE_STREAM=1|mh-spgemm_amd/mhspgemm" | sed "s/^/$m /" >> gpurun_out/ab_side.log 2>&1 || exit $?; done
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu > gpurun_out/b_side.log 2>&1
MHS_NO_SIDE_STREAM=1 timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu > gpurun_out/b_noside.log 2>&1
