# VRF as V | U | join: GPU tests of the header path, A/B bench (PRAOS_VRF3), 54k timeline
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03i
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_headers.py tests/test_gpu_chain.py tests/test_gpu_group.py tests/test_gpu_decode.py tests/test_gpu_replay.py > $O/tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u bench.py --no-cpu --no-e2e --steps 10 > $O/bench3.json 2> $O/bench3.err || { echo BENCHFAIL; tail $O/bench3.err; exit 1; }
PRAOS_VRF3=0 timeout -k 10 400 python -u bench.py --no-cpu --no-e2e --steps 10 > $O/bench2.json 2> $O/bench2.err || { echo BENCHFAIL; tail $O/bench2.err; exit 1; }
for f in bench3 bench2; do python3 -c "import json,sys;d=json.load(open('$O/$f.json'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'],json.dumps({k:v['per_gpu_vs_full'] for k,v in d['strong_proxy'].items() if k!='note'}))"; done
bash tools/gpu_trace_items.sh r03i/t54 54000 > /dev/null && tail -45 $O/t54/timeline.txt
