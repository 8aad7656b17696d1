# final pass of this build: rocprof kernel trace + PMC (r03c), then the full -m gpu suite, smoke and the default bench
set -o pipefail
export TMPDIR=/tmp
bash tools/profile.sh r03c || { echo PROFFAIL; exit 1; }
bash tools/gpu_full.sh
