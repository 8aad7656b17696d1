# hardware queues per process (GPU_MAX_HW_QUEUES, default 4): bench + e2e probe at 4 / 8 / 16
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03o
mkdir -p $O
for Q in 4 8 16; do
GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python -u tools/e2e_pipe_probe.py 2 4 8 > $O/probe_q$Q.txt 2>&1 || { echo PROBEFAIL; tail $O/probe_q$Q.txt; exit 1; }
echo "Q=$Q"; cat $O/probe_q$Q.txt
GPU_MAX_HW_QUEUES=$Q timeout -k 10 400 python -u bench.py --no-cpu --no-e2e --steps 10 > $O/bench_q$Q.json 2> $O/bench_q$Q.err || { echo BENCHFAIL; tail $O/bench_q$Q.err; exit 1; }
python3 -c "import json,sys;d=json.load(open('$O/bench_q$Q.json'));r=d['roofline'];print('Q=$Q',d['value'],d['ms_per_step'],r['kernel_ms'],json.dumps({k:v['per_gpu_vs_full'] for k,v in d['strong_proxy'].items() if k!='note'}))"
done
