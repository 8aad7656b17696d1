#!/bin/bash
# All BASELINE.json configs on one GPU (c5 = the metric's workload).
set -u
TAG=${1:-r01}
mkdir -p gpurun_out/bench_$TAG
for c in ${CONFIGS:-c5 c2 c3 c4 c1}; do
  timeout -k 10 500 python3 bench.py --config $c ${EXTRA_ARGS:-} > gpurun_out/bench_$TAG/$c.json 2> gpurun_out/bench_$TAG/$c.err
  rc=$?
  echo "$c rc=$rc"; tail -c 600 gpurun_out/bench_$TAG/$c.json
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench_$TAG/$c.err; fi
  if [ $rc -ge 124 ]; then exit $rc; fi
done
