# A/B of the field inversion: binary GCD (default build), its 32-bit inner-step form, Fermat
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/gcd
D=$PWD/ouroboros-consensus_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gcd/prim.log 2>&1 || { tail -30 gpurun_out/gcd/prim.log; exit 1; }
tail -2 gpurun_out/gcd/prim.log
for v in "" _i32 _fermat; do
  echo "lib$v"; PRAOS_HIP_LIB=$D/libpraos_hip$v.so timeout -k 10 200 python -u tools/microbench/inv_bench.py 2097152 2>&1 | tee gpurun_out/gcd/inv_bench$v.txt || exit 1
done
bash tools/ab.sh gcd54 54000 "-" "PRAOS_HIP_LIB=$D/libpraos_hip_i32.so" "PRAOS_HIP_LIB=$D/libpraos_hip_fermat.so" 2>&1 | tee gpurun_out/gcd/ab54.txt
bash tools/ab.sh gcd432 432000 "-" "PRAOS_HIP_LIB=$D/libpraos_hip_i32.so" "PRAOS_HIP_LIB=$D/libpraos_hip_fermat.so" 2>&1 | tee gpurun_out/gcd/ab432.txt
