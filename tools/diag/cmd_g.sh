for m in cant cop20k_A webbase-1M; do MATRIX=$m tools/diag/ab.sh "head||tools/diag/vHEAD" "new||mh-spgemm_amd/mhspgemm" | sed "s/^/$m /" >> gpurun_out/ab_fuse.log 2>&1 || exit $?; done
