# launch-bound A/B of the staged VRF kernels: V and U/join at 3 or 2 waves per SIMD
set -o pipefail
export TMPDIR=/tmp
LIBS="libpraos_hip.so lib_f2.so lib_v2f2.so libpraos_hip.so lib_f2.so" CONCS=1 bash tools/ab.sh
