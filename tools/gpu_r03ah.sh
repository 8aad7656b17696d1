# C5-shaped replay (3000 pools, 432k headers/epoch, 3 epochs): Praos and TPraos on the final build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ah
mkdir -p $O
timeout -k 10 540 python -u tools/replay_bench.py --round-robin --pools 3000 --epochs 3 --epoch-length 432000 --reps 2 --batch-sizes 96000,144000 > $O/replay_c5.jsonl 2> $O/replay_c5.err || { echo RBFAIL; tail $O/replay_c5.err; exit 1; }
cat $O/replay_c5.jsonl | cut -c1-420
timeout -k 10 540 python -u tools/replay_bench.py --tpraos --round-robin --pools 3000 --epochs 3 --epoch-length 432000 --reps 2 --batch-sizes 96000,144000 > $O/replay_c5_tpraos.jsonl 2> $O/replay_c5_tpraos.err || { echo RBFAIL; tail $O/replay_c5_tpraos.err; exit 1; }
cat $O/replay_c5_tpraos.jsonl | cut -c1-420
