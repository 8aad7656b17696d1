# e2e with the VRF outputs' D2H under the KES tail; key-precompute wave priority A/B (e2e and the 54k proxy)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03q
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_group.py tests/test_gpu_decode.py > $O/tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for P in 0 1; do
PRAOS_KEY_PRIO=$P timeout -k 10 300 python -u tools/e2e_pipe_probe.py 4 6 8 > $O/probe_p$P.txt 2>&1 || { echo PROBEFAIL; tail $O/probe_p$P.txt; exit 1; }
echo "KEY_PRIO=$P"; cat $O/probe_p$P.txt
PRAOS_KEY_PRIO=$P timeout -k 10 400 python -u bench.py --no-cpu --no-e2e --steps 10 > $O/bench_p$P.json 2> $O/bench_p$P.err || { echo BENCHFAIL; tail $O/bench_p$P.err; exit 1; }
python3 -c "import json,sys;d=json.load(open('$O/bench_p$P.json'));r=d['roofline'];print('P=$P',d['value'],d['ms_per_step'],r['kernel_ms'],json.dumps({k:v['per_gpu_vs_full'] for k,v in d['strong_proxy'].items() if k!='note'}))"
done
