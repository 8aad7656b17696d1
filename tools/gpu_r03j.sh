# twin-engine e2e pipeline + 1-wave blocks for small batches: tests, bench, e2e chunk sweep, 54k timeline
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_headers.py tests/test_gpu_chain.py tests/test_gpu_group.py tests/test_gpu_decode.py tests/test_gpu_ffi.py > $O/tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for K in 0 2 3 6 8; do
timeout -k 10 400 python -u bench.py --no-cpu --steps 10 --pipeline $K > $O/bench_k$K.json 2> $O/bench_k$K.err || { echo BENCHFAIL; tail $O/bench_k$K.err; exit 1; }
python3 -c "import json,sys;d=json.load(open('$O/bench_k$K.json'));r=d['roofline'];e=d['e2e'];print('K=$K',d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'],'e2e',e['value'],e['ms'],e['bit_exact_vs_resident'],json.dumps({k:v['per_gpu_vs_full'] for k,v in d['strong_proxy'].items() if k!='note'}))"
done
bash tools/gpu_trace_items.sh r03j/t54 54000 > /dev/null && tail -42 $O/t54/timeline.txt
