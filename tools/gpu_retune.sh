# after making the small-shard schedule the default below SHARD_SMALL: GPU suite, smoke, bench, and
# the A/B against the previous default (PRAOS_V_MAIN=3 PRAOS_MISS_PRIO=1) at 54k
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/retune5
export STEPS=40
bash tools/ab.sh rt5_54 54000 "-" "PRAOS_V_MAIN=3 PRAOS_MISS_PRIO=1" 2>&1 | tee gpurun_out/retune5/ab54.txt || exit 1
bash tools/gpu_full.sh
