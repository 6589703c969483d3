# Parity of the multi-block split partition, its A/B, then stochastic PC sampling of cage15-like.
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
out=gpurun_out/r03zc; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
bash tools/r02_ab.sh r03zc_ab "cur5 cur7" "webbase-1M wb-edu cant-s1 scircuit" 5 || exit 1
bash tools/pcsample.sh r03zc_pc "cage15" || exit 1
