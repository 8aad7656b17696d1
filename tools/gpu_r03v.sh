# full -m gpu suite, replay sweep (C5 shape) with the launcher thread, default bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03v
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/t_gpu.log 2>&1 || { echo TESTFAIL; tail -60 $O/t_gpu.log; exit 1; }
tail -2 $O/t_gpu.log
timeout -k 10 900 python -u tools/replay_bench.py --round-robin --pools 3000 --epochs 3 --epoch-length 432000 --reps 3 --batch-sizes 96000,144000,216000 > $O/replay_c5.jsonl 2> $O/replay_c5.err || { echo RBFAIL; tail $O/replay_c5.err; exit 1; }
python3 -c "
import json
for l in open('$O/replay_c5.jsonl'): d=json.loads(l); print(d['batch_max'], d['value'], d['wall_ms'], d['stages_ms'])"
timeout -k 10 400 python -u bench.py --no-cpu --steps 10 > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'],d['e2e']['value'],d['e2e']['bit_exact_vs_resident'],json.dumps({k:v['per_gpu_vs_full'] for k,v in d['strong_proxy'].items() if k!='note'}))"
