# staged TPraos VRF (V / U with the VRF key cache / join per certificate): tests, then tp bench A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03af
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tpraos.py tests/test_gpu_replay.py tests/test_gpu_block.py tests/test_gpu_ffi.py > $O/tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for st in 1 0; do
  PRAOS_TP_STAGED=$st timeout -k 10 400 python -u bench.py --config tp --steps 10 > $O/tp$st.json 2> $O/tp$st.err || { echo BENCHFAIL; tail $O/tp$st.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/tp$st.json'));print('staged=$st',d['value'],d['ms_per_step'],d['roofline']['kernel_ms_serial'],json.dumps(d['self_check']),json.dumps(d['keycache']))"
done
