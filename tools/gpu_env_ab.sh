#!/bin/bash
# A/B of an environment knob over the default bench workload: VAR=name VALS="a b a b".
set -o pipefail
mkdir -p gpurun_out/envab
for v in ${VALS:-1 0 1 0}; do
  env $VAR=$v timeout -k 10 240 python3 bench.py --no-cpu --no-e2e --steps 10 --warmup 2 \
    > gpurun_out/envab/$VAR$v.json 2> gpurun_out/envab/$VAR$v.err || { echo "$VAR=$v failed"; tail gpurun_out/envab/$VAR$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/envab/$VAR$v.json')); print('$VAR=$v', round(d['value']), d['ms_per_step'], d['roofline']['kernel_ms_serial'])"
done
