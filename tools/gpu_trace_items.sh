# kernel trace of the C5 step at a given shard size: bash tools/gpu_trace_items.sh <tag> <items> [bench args]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; ITEMS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- \
  python3 bench.py --no-cpu --no-e2e --no-proxy --steps 5 --warmup 1 --items $ITEMS "$@" > $OUT/kt_bench.json 2> $OUT/kt.err || { echo KTFAIL; tail $OUT/kt.err; exit 1; }
python3 tools/trace_timeline.py $OUT/kt > $OUT/timeline.txt && tail -60 $OUT/timeline.txt
