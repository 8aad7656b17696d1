set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03d
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_headers.py tests/test_gpu_chain.py tests/test_gpu_group.py tests/test_gpu_replay.py tests/test_gpu_decode.py tests/test_gpu_tpraos.py > gpurun_out/r03d/tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r03d/tests.log; exit 1; }
tail -3 gpurun_out/r03d/tests.log
timeout -k 10 400 python -u bench.py --no-cpu --no-e2e > gpurun_out/r03d/bench.json 2> gpurun_out/r03d/bench.err || { echo BENCHFAIL; tail gpurun_out/r03d/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r03d/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms_serial'],d['strong_proxy'])"
bash tools/gpu_trace_items.sh r03d/t54 54000
