set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03c
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_group.py tests/test_gpu_headers.py > gpurun_out/r03c/tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r03c/tests.log; exit 1; }
tail -3 gpurun_out/r03c/tests.log
timeout -k 10 400 python -u bench.py --no-cpu --no-e2e > gpurun_out/r03c/bench.json 2> gpurun_out/r03c/bench.err || { echo BENCHFAIL; tail gpurun_out/r03c/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r03c/bench.json'));print(d['value'],d['ms_per_step'],d['strong_proxy'])"
bash tools/gpu_trace_items.sh r03c/t54 54000
