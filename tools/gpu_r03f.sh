set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03f
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r03f/tests.log 2>&1 || { echo TESTFAIL; tail -60 gpurun_out/r03f/tests.log; exit 1; }
tail -3 gpurun_out/r03f/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03f/smoke.log 2>&1 || { echo SMOKEFAIL; tail gpurun_out/r03f/smoke.log; exit 1; }
cat gpurun_out/r03f/smoke.log
