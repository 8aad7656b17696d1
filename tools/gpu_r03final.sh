# final round-3 pass: full -m gpu suite + smoke + default bench, then rocprof trace + PMC of the same build
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_full.sh && bash tools/profile.sh ${PTAG:-r03e}
