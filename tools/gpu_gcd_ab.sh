# A/B of the field inversion builds: binary GCD (default), its VGPR-mask inner step
# (libpraos_hip_mask.so: make BUILD=build_mask OUT=../libpraos_hip_mask.so EXTRA=-DFEG_INNER_MASK=1),
# Fermat (libpraos_hip_fermat.so: EXTRA=-DPRAOS_INV_GCD=0)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/gcd2
D=$PWD/ouroboros-consensus_amd
for v in "" _mask _fermat; do
  echo "lib$v"; PRAOS_HIP_LIB=$D/libpraos_hip$v.so timeout -k 10 200 python -u tools/microbench/inv_bench.py 2097152 2>&1 | tee gpurun_out/gcd2/inv_bench$v.txt || exit 1
done
PRAOS_HIP_LIB=$D/libpraos_hip_mask.so timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gcd2/prim_mask.log 2>&1 || { tail -30 gpurun_out/gcd2/prim_mask.log; exit 1; }
tail -1 gpurun_out/gcd2/prim_mask.log
bash tools/ab.sh gm54 54000 "-" "PRAOS_HIP_LIB=$D/libpraos_hip_mask.so" 2>&1 | tee gpurun_out/gcd2/ab54.txt
bash tools/ab.sh gm432 432000 "-" "PRAOS_HIP_LIB=$D/libpraos_hip_mask.so" 2>&1 | tee gpurun_out/gcd2/ab432.txt
