set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03g
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_replay.py tests/test_gpu_ffi.py tests/test_gpu_tpraos.py tests/test_gpu_group.py > gpurun_out/r03g/tests.log 2>&1 || { echo TESTFAIL; tail -60 gpurun_out/r03g/tests.log; exit 1; }
tail -3 gpurun_out/r03g/tests.log
timeout -k 10 400 python -u bench.py --no-cpu --steps 10 > gpurun_out/r03g/bench.json 2> gpurun_out/r03g/bench.err || { echo BENCHFAIL; tail gpurun_out/r03g/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r03g/bench.json'));print(d['value'],d['ms_per_step'],json.dumps(d['e2e']))"
