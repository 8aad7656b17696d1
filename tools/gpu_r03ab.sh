# 54k strong-proxy A/B: stage V / join wave priority, key precompute wave priority
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ab
mkdir -p $O
for v in "0 0" "1 0" "1 1" "0 1"; do
  set -- $v
  PRAOS_VRF_PRIO=$1 PRAOS_KEY_PRIO=$2 timeout -k 10 300 python -u bench.py --no-cpu --no-e2e --steps 20 > $O/p$1$2.json 2> $O/p$1$2.err || { echo BENCHFAIL $v; tail $O/p$1$2.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/p$1$2.json'));p=d['strong_proxy'];print('vrf_prio=$1 key_prio=$2',d['value'],d['ms_per_step'],[(k,p[k]['ms_per_step'],p[k]['per_gpu_vs_full']) for k in ('n2','n4','n8')])"
done
