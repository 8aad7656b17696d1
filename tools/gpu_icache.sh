# instruction-cache PMC pass of the C5 step (concurrent streams, then serial)
set -u
export TMPDIR=/tmp
OUT=gpurun_out/icache
mkdir -p $OUT
n=0
for conc in 1 0; do
  timeout -s KILL 240 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU \
    -d $OUT/c$conc -o pmc --output-format csv -- \
    python3 bench.py --no-cpu --no-e2e --no-proxy --steps 1 --warmup 0 --concurrent $conc > /dev/null 2> $OUT/c$conc.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc rc=$rc"; tail -5 $OUT/c$conc.err; exit 1; fi
  python3 tools/icache_summary.py $OUT/c$conc | tee $OUT/c$conc.txt
done
