#!/bin/bash
# A/B of library knobs on the C5 workload at one batch size (one GPU, resident step only).
#   tools/ab.sh TAG ITEMS "ENV1" "ENV2" ...      (ENV = space-separated VAR=value, or "-" for defaults)
#   E2E=1: the stored-bytes (PCIe-inclusive) line as well; STEPS, EXTRA_ARGS: bench.py
# Each setting runs twice, interleaved (A B A B ...), so box drift shows up as spread.
# Writes gpurun_out/ab/TAG/<i>_<round>.json and prints one line per run.
set -u
TAG=$1; ITEMS=$2; shift 2
OUT=gpurun_out/ab/$TAG
mkdir -p "$OUT"
for r in 0 1; do
  i=0
  for setting in "$@"; do
    envs=()
    [ "$setting" != "-" ] && read -r -a envs <<< "$setting"
    timeout -k 10 300 env "${envs[@]}" python3 bench.py --items "$ITEMS" --steps ${STEPS:-20} --warmup 3 --no-cpu $([ -n "${E2E:-}" ] || echo --no-e2e) \
      --no-proxy ${EXTRA_ARGS:-} > "$OUT/${i}_${r}.json" 2> "$OUT/${i}_${r}.err"
    rc=$?
    if [ $rc -ne 0 ]; then echo "[$setting] rc=$rc"; tail -5 "$OUT/${i}_${r}.err"; exit $rc; fi
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d.get('e2e') or {}; print(f'[{sys.argv[2]}] {d[\"ms_per_step\"]:.3f} ms  {d[\"value\"]/1e6:.2f} M/s  clean_ok {d[\"self_check\"][\"clean_ok\"]}/{d[\"self_check\"][\"clean\"]}' + (f'  e2e {e[\"ms\"]:.2f} ms {e[\"value\"]/1e6:.2f} M/s exact {e[\"bit_exact_vs_resident\"]}' if e else ''))" \
      "$OUT/${i}_${r}.json" "$setting"
    i=$((i + 1))
  done
done
