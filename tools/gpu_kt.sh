#!/bin/bash
# Kernel trace + stats only (one rocprofv3 pass over the default bench workload).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/kt_${TAG:-x}
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT -o kt --output-format csv -- \
  python3 bench.py ${ARGS:-} --no-cpu --no-e2e --steps 5 --warmup 1 > $OUT/bench.json 2> $OUT/kt.err || { tail $OUT/kt.err; exit 1; }
f=$(find $OUT -name '*kernel_stats.csv' | head -1)
python3 -c "
import csv,sys
r=list(csv.DictReader(open('$f')))
for x in sorted(r,key=lambda x:-float(x['TotalDurationNs']))[:14]:
    print(f\"{x['Name'][:40]:40s} calls={x['Calls']:>5s} avg_ms={float(x['AverageNs'])/1e6:8.3f} total_ms={float(x['TotalDurationNs'])/1e6:9.2f}\")
"
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['roofline']['kernel_ms_serial'], d['roofline']['pipeline_ms'])"
