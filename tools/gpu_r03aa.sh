# registered host buffers (direct DMA) for e2e; TPraos through the shared OCert/KES pipeline
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03aa
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tpraos.py tests/test_gpu_replay.py tests/test_gpu_group.py tests/test_gpu_decode.py tests/test_gpu_ffi.py tests/test_gpu_block.py > $O/tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u bench.py --no-cpu --steps 10 > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));e=d['e2e'];print(d['value'],e['value'],e['ms'],e['bit_exact_vs_resident'],e['pageable'])"
timeout -k 10 400 python -u bench.py --config tp --steps 10 > $O/tp.json 2> $O/tp.err || { echo BENCHFAIL; tail $O/tp.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/tp.json'));print('tp',d['value'],d['ms_per_step'],d['roofline']['frac'],json.dumps(d['self_check']),json.dumps(d['keycache']))"
