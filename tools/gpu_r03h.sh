set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03h
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_group.py tests/test_gpu_decode.py tests/test_gpu_tpraos.py > gpurun_out/r03h/tests.log 2>&1 || { echo TESTFAIL; tail -60 gpurun_out/r03h/tests.log; exit 1; }
tail -3 gpurun_out/r03h/tests.log
timeout -k 10 400 python -u bench.py --no-cpu --steps 10 > gpurun_out/r03h/bench.json 2> gpurun_out/r03h/bench.err || { echo BENCHFAIL; tail gpurun_out/r03h/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r03h/bench.json'));print(d['value'],d['ms_per_step'],json.dumps(d['e2e']))"
