#!/bin/bash
# A/B of side-stream priorities (PRAOS_SIDE_PRIO: OCert, KES, VRF; 1 = high), default bench workload.
set -o pipefail
mkdir -p gpurun_out/prio
for p in ${PRIOS:-000 001 110 000 001}; do
  PRAOS_SIDE_PRIO=$p timeout -k 10 240 python3 bench.py --no-cpu --no-e2e --steps 10 --warmup 2 \
    > gpurun_out/prio/p$p.json 2> gpurun_out/prio/p$p.err || { echo "prio $p failed"; tail gpurun_out/prio/p$p.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/prio/p$p.json')); print('$p', round(d['value']), d['ms_per_step'], d['roofline']['kernel_ms_serial'])"
done
