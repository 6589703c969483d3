set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "near or group or bin_zoo or cant or repeat or unsynced" > gpurun_out/r03v_pytest.log 2>&1 || { tail -30 gpurun_out/r03v_pytest.log; exit 1; }
tail -2 gpurun_out/r03v_pytest.log
bash tools/r02_ab.sh r03v_near "base base@MHS_NO_NEAR=1" "cant-perturbed cant pwtk hood shipsec1 cop20k_A scircuit pdb1HYS rma10" 5 || exit 1
