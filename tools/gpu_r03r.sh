# threaded replay driver: replay GPU tests, the round-2 replay bench shape, then the C5 shape (3000 pools, 432k/epoch, 3 epochs)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03r
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_replay.py > $O/tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u tools/replay_bench.py --epochs 5 --pools 200 --reps 3 --batch-sizes 32768,131072 > $O/replay_small.jsonl 2> $O/replay_small.err || { echo RBFAIL; tail $O/replay_small.err; exit 1; }
cat $O/replay_small.jsonl
