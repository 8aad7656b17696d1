# C5-shaped replay: 3000 pools, 432k headers per epoch (f = 1, round-robin forgers), 3 epochs
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03s
mkdir -p $O
timeout -k 10 1000 python -u tools/replay_bench.py --round-robin --pools 3000 --epochs 3 --epoch-length 432000 --reps 2 --batch-sizes 432000,216000,1296000 > $O/replay_c5.jsonl 2> $O/replay_c5.err || { echo RBFAIL; tail $O/replay_c5.err; exit 1; }
cat $O/replay_c5.jsonl
