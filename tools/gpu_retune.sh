# join placement A/Bs (PRAOS_V_MAIN) at the shard sizes; see DESIGN §15 "Small-shard schedule"
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/retune9
export STEPS=30
bash tools/ab.sh rt9_216 216000 "-" "PRAOS_V_MAIN=2" 2>&1 | tee gpurun_out/retune9/ab216.txt
