# fast linker: linked-chain GPU tests, then the C5-shaped replay (3000 pools, 432k headers/epoch, 3 epochs)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03t
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_replay.py tests/test_gpu_chain.py > $O/tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 900 python -u tools/replay_bench.py --round-robin --pools 3000 --epochs 3 --epoch-length 432000 --reps 2 --batch-sizes 432000,216000,1296000 > $O/replay_c5.jsonl 2> $O/replay_c5.err || { echo RBFAIL; tail $O/replay_c5.err; exit 1; }
cat $O/replay_c5.jsonl
