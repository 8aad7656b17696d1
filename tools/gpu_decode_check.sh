set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_headers.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_dec.log 2>&1; rc=$?
tail -25 gpurun_out/t_dec.log; exit $rc
