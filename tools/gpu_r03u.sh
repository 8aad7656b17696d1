# replay batches kept in the context, lighter nonce chain: replay tests, C5-shaped replay sweep, bench regression
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03u
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_replay.py > $O/tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 900 python -u tools/replay_bench.py --round-robin --pools 3000 --epochs 3 --epoch-length 432000 --reps 3 --batch-sizes 108000,144000,216000,432000 > $O/replay_c5.jsonl 2> $O/replay_c5.err || { echo RBFAIL; tail $O/replay_c5.err; exit 1; }
cat $O/replay_c5.jsonl
timeout -k 10 400 python -u bench.py --no-cpu --steps 10 > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'],d['e2e']['value'],d['e2e']['bit_exact_vs_resident'])"
