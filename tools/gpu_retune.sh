# join placement below SHARD_SMALL with the uncached verifies at normal priority (the default there)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/retune7
export STEPS=40
bash tools/ab.sh rt7_54 54000 "-" "PRAOS_V_MAIN=2" 2>&1 | tee gpurun_out/retune7/ab54.txt
bash tools/ab.sh rt7_40 40000 "-" "PRAOS_V_MAIN=2" 2>&1 | tee gpurun_out/retune7/ab40.txt
bash tools/ab.sh rt7_20 20000 "-" "PRAOS_V_MAIN=2" 2>&1 | tee gpurun_out/retune7/ab20.txt
