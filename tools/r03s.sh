set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "near or launch_ahead or group or bin_zoo or cant" > gpurun_out/r03s_pytest.log 2>&1 || { tail -30 gpurun_out/r03s_pytest.log; exit 1; }
tail -2 gpurun_out/r03s_pytest.log
bash tools/r02_ab.sh r03s_near "base base@MHS_NO_NEAR=1" "cant-perturbed cant pwtk hood shipsec1" 5 || exit 1
mkdir -p gpurun_out/r03s_la
bash tools/r02_ab.sh r03s_scan "base scan4" "cant cop20k_A mac_econ_fwd500 scircuit rma10 pdb1HYS" 5 || exit 1
bash tools/r02_ab.sh r03s_mc "base base@MHS_NO_MCACHE=1" "cage15 webbase-1M" 3 || exit 1
