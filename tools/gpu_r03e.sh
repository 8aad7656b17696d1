set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03e
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tpraos.py tests/test_gpu_verify.py tests/test_gpu_block.py > gpurun_out/r03e/tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r03e/tests.log; exit 1; }
tail -3 gpurun_out/r03e/tests.log
timeout -k 10 400 python -u bench.py --no-cpu --no-e2e > gpurun_out/r03e/bench.json 2> gpurun_out/r03e/bench.err || { echo BENCHFAIL; tail gpurun_out/r03e/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r03e/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms_serial'],d['strong_proxy'])"
bash tools/gpu_trace_items.sh r03e/t54 54000
