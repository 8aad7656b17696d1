# re-tune after the GCD inversion: the KES leaf-key cache cut (KES_NOCACHE_BATCH) at 54k / 64k
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/retune
bash tools/ab.sh rt54 54000 "-" "PRAOS_KES_NOCACHE=0" 2>&1 | tee gpurun_out/retune/ab54.txt
bash tools/ab.sh rt64 64000 "-" "PRAOS_KES_NOCACHE=70000" 2>&1 | tee gpurun_out/retune/ab64.txt
bash tools/ab.sh rt40 40000 "-" "PRAOS_KES_NOCACHE=0" 2>&1 | tee gpurun_out/retune/ab40.txt
