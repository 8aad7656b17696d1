# ILP-4 field multiply at 1-3 waves/SIMD; 2-rank bench rehearsal (gloo, both ranks on device 0)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03z
mkdir -p $O
timeout -k 10 120 ./tools/microbench/femul4 > $O/femul4.txt 2>&1 || { echo FEMULFAIL; cat $O/femul4.txt; exit 1; }
cat $O/femul4.txt
PRAOS_BENCH_REHEARSAL=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu --no-e2e > $O/rehearsal.json 2> $O/rehearsal.err || { echo REHFAIL; tail -20 $O/rehearsal.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/rehearsal.json'));print('rehearsal N=2',d['value'],d['ms_per_step'],d['n_gpus'],d['config']['items_total'])"
