timeout -k 10 400 python -m pytest tests -q -m gpu -x > gpurun_out/t_tiny.log 2>&1; tail -1 gpurun_out/t_tiny.log
for m in cant cop20k_A webbase-1M scircuit mac_econ_fwd500; do MATRIX=$m RUNPY=tools/diag/run_phases.py tools/diag/ab.sh "new||mh-spgemm_amd/mhspgemm" | sed "s/^/$m /" >> gpurun_out/ab_tiny.log 2>&1 || exit $?; done
