#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box via gpurun).
# Kernel trace/stats in one pass; each PMC group in its own pass (no tracing
# domains combined with --pmc).  Outputs under gpurun_out/prof_<tag>.
#   usage: bash tools/profile.sh <tag> [bench args...]
set -u
export TMPDIR=/tmp
TAG=${1:-r02}
shift || true
ARGS=${*:-"--config c5"}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- \
  python3 bench.py $ARGS --no-cpu --no-e2e --no-proxy --steps 5 --warmup 1 > $OUT/kt_bench.json 2> $OUT/kt.err || exit 1
n=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  n=$((n+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp -d $OUT/pmc$n -o pmc$n --output-format csv -- \
    python3 bench.py $ARGS --no-cpu --no-e2e --no-proxy --steps 1 --warmup 0 > /dev/null 2> $OUT/pmc$n.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc pass $n rc=$rc, stopping"; tail -5 $OUT/pmc$n.err; exit 1; fi
  echo "pmc pass $n ok"
done
python3 tools/prof_summary.py $OUT $TAG > $OUT/summary.txt && cp profiles/${TAG}_* $OUT/ && echo summary written
