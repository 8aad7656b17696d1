#!/bin/bash
# A subset of the -m gpu suite (test files as arguments), time-limited; log under gpurun_out/some/.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/some
timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/some/t_gpu.log 2>&1 \
  || { echo TESTFAIL; tail -60 gpurun_out/some/t_gpu.log; exit 1; }
tail -5 gpurun_out/some/t_gpu.log
