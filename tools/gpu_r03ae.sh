# stream-priority A/B for the stored-bytes pipeline and the resident step
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ae
mkdir -p $O
for v in "1 001" "0 001" "0 111" "1 111" "0 110"; do
  set -- $v
  PRAOS_V_PRIO=$1 PRAOS_SIDE_PRIO=$2 timeout -k 10 300 python -u bench.py --no-cpu --no-proxy --steps 10 > $O/v$1_s$2.json 2> $O/v$1_s$2.err || { echo BENCHFAIL $v; tail $O/v$1_s$2.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/v$1_s$2.json'));e=d['e2e'];print('v_prio=$1 side=$2',d['value'],d['ms_per_step'],'e2e',e['value'],e['ms'],e['bit_exact_vs_resident'],'pageable',e['pageable']['ms'])"
done
