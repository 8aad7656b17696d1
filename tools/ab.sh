#!/bin/bash
# A/B of library build variants (PRAOS_HIP_LIB) x stream concurrency, 432k headers.
set -u
mkdir -p gpurun_out/ab
for lib in ${LIBS:-libpraos_hip.so}; do
  for conc in ${CONCS:-0 1}; do
    PRAOS_HIP_LIB=$PWD/ouroboros-consensus_amd/$lib timeout -k 10 240 python3 bench.py --no-cpu --steps 5 --warmup 1 \
      --concurrent $conc ${ABARGS:---no-e2e} > gpurun_out/ab/${lib}_c$conc.json 2> gpurun_out/ab/${lib}_c$conc.err
    rc=$?
    if [ $rc -ge 124 ]; then echo "$lib c$conc rc=$rc"; exit $rc; fi
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/${lib}_c$conc.json')); print('$lib', 'conc=$conc', round(d['value']), d['ms_per_step'], d['roofline']['kernel_ms_serial'], d['self_check'].get('clean_ok'), {k: v['per_gpu_vs_full'] for k, v in (d.get('strong_proxy') or {}).items() if isinstance(v, dict)})"
  done
done
