# per-chunk KES under the e2e upload + TPraos concurrency: tests, e2e probe, configs TPraos and C1-C4
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03x
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tpraos.py tests/test_gpu_replay.py tests/test_gpu_group.py tests/test_gpu_decode.py > $O/tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/e2e_pipe_probe.py 4 6 8 > $O/probe.txt 2>&1 || { echo PROBEFAIL; tail $O/probe.txt; exit 1; }
cat $O/probe.txt
for C in tp c2 c3 c4 c1; do
timeout -k 10 400 python -u bench.py --config $C --steps 10 > $O/$C.json 2> $O/$C.err || { echo BENCHFAIL $C; tail $O/$C.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/$C.json'));r=d['roofline'];print('$C',d['value'],d['unit'],d['ms_per_step'],r['kernel'],r['frac'],json.dumps(d['self_check']),json.dumps(d.get('keycache')))"
done
