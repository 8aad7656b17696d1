#!/bin/bash
# quick GPU pass: a list of test files, then the default bench (both time-limited)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread > gpurun_out/t_quick.log 2>&1 \
  || { echo TESTFAIL; tail -40 gpurun_out/t_quick.log; exit 1; }
tail -3 gpurun_out/t_quick.log
timeout -k 10 400 python bench.py --cpu-seconds 4 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err \
  || { echo BENCHFAIL; tail gpurun_out/bench_quick.err; exit 1; }
cat gpurun_out/bench_quick.json
