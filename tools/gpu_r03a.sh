# r03 baseline at HEAD: bench (with the strong-scaling proxy) + kernel trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03a
timeout -k 10 400 python -u bench.py --no-cpu > gpurun_out/r03a/bench.json 2> gpurun_out/r03a/bench.err || { echo BENCHFAIL; tail gpurun_out/r03a/bench.err; exit 1; }
cat gpurun_out/r03a/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r03a/kt -o kt --output-format csv -- \
  python3 bench.py --no-cpu --no-e2e --no-proxy --steps 5 --warmup 1 > gpurun_out/r03a/kt_bench.json 2> gpurun_out/r03a/kt.err || { echo KTFAIL; tail gpurun_out/r03a/kt.err; exit 1; }
python3 tools/prof_summary.py gpurun_out/r03a r03a > gpurun_out/r03a/summary.txt 2>&1; head -40 gpurun_out/r03a/summary.txt
