export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
mkdir -p gpurun_out/fork
for r in 1 2 3; do for f in 0 1; do
  MHS_SYM_FORK=$f timeout -k 10 200 python bench.py --no-cpu > gpurun_out/fork/b_${f}_$r.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/fork/b_${f}_$r.json')); print('fork=$f r$r', d['value'], d['ms_per_step'], d.get('cold_call_ms'))"
done; done
bash tools/r02_ab.sh fork "cur@MHS_SYM_FORK=0 cur@MHS_SYM_FORK=1" "cant mac_econ_fwd500 scircuit cop20k_A cage12 webbase-1M pwtk" 3
