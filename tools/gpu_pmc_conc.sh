#!/bin/bash
# one PMC pass (wait-state counters) with the crypto kernels concurrent and serial
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcq
for conc in 1 0; do
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU -d gpurun_out/pmcq/c$conc -o p --output-format csv -- \
    python3 bench.py --no-cpu --no-e2e --steps 1 --warmup 0 --concurrent $conc > /dev/null 2> gpurun_out/pmcq/c$conc.err || { echo "pmc rc=$?"; tail -5 gpurun_out/pmcq/c$conc.err; exit 1; }
  echo "== concurrent=$conc"
  python3 tools/pmc_quick.py gpurun_out/pmcq/c$conc _ck k_kes k_vrf k_ocert
done
