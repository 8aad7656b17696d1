set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/blk
timeout -k 10 300 python -u -m pytest tests/test_gpu_block.py tests/test_gpu_decode.py -x -v --timeout 120 --timeout-method thread > gpurun_out/blk/t.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/blk/t.log; exit 1; }
tail -3 gpurun_out/blk/t.log
timeout -k 10 120 python -u tools/bench_blocks.py --blocks 2048 --payload 1024 > gpurun_out/blk/small.json 2>&1 || { echo SMALLFAIL; tail -20 gpurun_out/blk/small.json; exit 1; }
cat gpurun_out/blk/small.json
timeout -k 10 300 python -u tools/bench_blocks.py > gpurun_out/blk/bench.json 2> gpurun_out/blk/bench.err || { echo BENCHFAIL; tail gpurun_out/blk/bench.err; exit 1; }
cat gpurun_out/blk/bench.json
timeout -k 10 300 python -u tools/bench_blocks.py --blocks 65536 > gpurun_out/blk/bench64k.json 2> gpurun_out/blk/bench64k.err || { echo BENCH64FAIL; tail gpurun_out/blk/bench64k.err; exit 1; }
cat gpurun_out/blk/bench64k.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/blk/kt -o kt --output-format csv -- python3 tools/bench_blocks.py --steps 5 --warmup 1 > gpurun_out/blk/kt.json 2> gpurun_out/blk/kt.err || { echo PROFFAIL; tail gpurun_out/blk/kt.err; exit 1; }
find gpurun_out/blk/kt -name "*kernel_stats.csv" | head -1 | xargs cat
