set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03n
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_group.py tests/test_gpu_decode.py > $O/tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/e2e_pipe_probe.py 2 3 4 6 8 > $O/probe.txt 2>&1 || { echo PROBEFAIL; tail $O/probe.txt; exit 1; }
cat $O/probe.txt
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/kt4 -o kt --output-format csv -- python3 tools/e2e_pipe_probe.py 4 > $O/kt4.txt 2>&1 || { echo KT4FAIL; tail $O/kt4.txt; exit 1; }
