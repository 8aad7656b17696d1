set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/t_gpu.log; exit 1; }
tail -3 gpurun_out/t_gpu.log
grep -E "PASSED|FAILED" gpurun_out/t_gpu.log | awk '{print $1}' | sed 's/.*:://' | tr '\n' ' ' | head -c 3000; echo
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKEFAIL; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCHFAIL; tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
