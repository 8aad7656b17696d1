#!/bin/bash
# Round evidence: every BASELINE config's bench line, block-integrity bench, replay bench.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r02e}
mkdir -p gpurun_out/ev_$TAG
CONFIGS="c5 c1 c2 c3 c4" bash tools/bench_all.sh ev_$TAG || exit 1
timeout -k 10 300 python3 -u tools/bench_blocks.py > gpurun_out/ev_$TAG/blocks.json 2> gpurun_out/ev_$TAG/blocks.err || { echo BLOCKFAIL; tail -5 gpurun_out/ev_$TAG/blocks.err; exit 1; }
tail -c 400 gpurun_out/ev_$TAG/blocks.json
timeout -k 10 400 python3 -u tools/replay_bench.py > gpurun_out/ev_$TAG/replay.jsonl 2> gpurun_out/ev_$TAG/replay.err || { echo REPLAYFAIL; tail -5 gpurun_out/ev_$TAG/replay.err; exit 1; }
tail -c 600 gpurun_out/ev_$TAG/replay.jsonl
