#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box via gpurun).
# Kernel trace/stats in one pass; each PMC group in its own pass (no tracing
# domains combined with --pmc).  Outputs under gpurun_out/prof_<tag>.
set -u
export TMPDIR=/tmp
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- \
  python3 bench.py --no-cpu --steps 5 --warmup 1 > $OUT/kt_bench.json 2> $OUT/kt.err || exit 1
n=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INST_CYCLES_VALU" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  n=$((n+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d $OUT/pmc$n -o pmc$n --output-format csv -- \
    python3 bench.py --no-cpu --headers 131072 --steps 1 --warmup 0 > /dev/null 2> $OUT/pmc$n.err
  rc=$?
  if [ $rc -ge 124 ]; then echo "pmc pass $n rc=$rc, stopping"; exit $rc; fi
done
python3 tools/prof_summary.py $OUT $TAG > $OUT/summary.txt && echo summary written
