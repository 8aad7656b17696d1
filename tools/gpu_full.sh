#!/bin/bash
# Full GPU pass: -m gpu suite, smoke(), default bench line (each time-limited, chained).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/full
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/full/t_gpu.log 2>&1 \
  || { echo TESTFAIL; tail -40 gpurun_out/full/t_gpu.log; exit 1; }
tail -3 gpurun_out/full/t_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/full/smoke.log 2>&1 \
  || { echo SMOKEFAIL; tail -20 gpurun_out/full/smoke.log; exit 1; }
tail -1 gpurun_out/full/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/full/bench.json 2> gpurun_out/full/bench.err \
  || { echo BENCHFAIL; tail gpurun_out/full/bench.err; exit 1; }
cat gpurun_out/full/bench.json
