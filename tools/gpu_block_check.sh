set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_block.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_block.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/t_block.log; exit 1; }
tail -8 gpurun_out/t_block.log
