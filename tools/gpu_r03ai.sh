# TPraos: the two certificates' stage V on two streams -- tests, tp bench, TPraos replay at the C5 shape
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ai
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tpraos.py tests/test_gpu_replay.py > $O/tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u bench.py --config tp --steps 10 > $O/tp.json 2> $O/tp.err || { echo BENCHFAIL; tail $O/tp.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/tp.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['frac'],json.dumps(d['self_check']))"
timeout -k 10 540 python -u tools/replay_bench.py --tpraos --round-robin --pools 3000 --epochs 3 --epoch-length 432000 --reps 2 --batch-sizes 96000,144000 > $O/replay_c5_tpraos.jsonl 2> $O/replay_c5_tpraos.err || { echo RBFAIL; tail $O/replay_c5_tpraos.err; exit 1; }
cat $O/replay_c5_tpraos.jsonl | cut -c1-420
