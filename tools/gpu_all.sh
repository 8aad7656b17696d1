set -o pipefail
bash tools/gpu_check.sh || exit 1
timeout -k 10 300 python -u tools/bench_blocks.py > gpurun_out/blk/bench.json 2> gpurun_out/blk/bench.err || { echo BENCHFAIL; tail gpurun_out/blk/bench.err; exit 1; }
cat gpurun_out/blk/bench.json
