# Per-kernel traces (numeric bins on one stream) + L2 hit/miss and FETCH/WRITE passes of
# the stand-ins furthest below the roofline, on HEAD.
set -o pipefail
bash tools/prof_r03.sh r03x "cage15 webbase-1M wb-edu cant-perturbed" nostamps "TCC_HIT_sum,TCC_MISS_sum;FETCH_SIZE;WRITE_SIZE" || exit 1
