# Stochastic PC sampling of one stand-in's sweep (numeric bins on one stream), one run per
# matrix under its own kill timer.  usage: tools/pcsample.sh <tag> "<matrices>"
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth MHS_NUM_STREAMS=1
tag=$1; mats=$2
out=gpurun_out/$tag; mkdir -p $out
for m in $mats; do
  timeout -s KILL 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
      --pc-sampling-interval 1048576 --kernel-trace --output-format csv -d $out/$m -o run -- python3 tools/sweep.py $m --reps 3 \
      > $out/$m.log 2>&1 || { echo "pc sampling $m failed"; tail -20 $out/$m.log; exit 1; }
  ls $out/$m
  echo "== $m done"
done
echo PCDONE
