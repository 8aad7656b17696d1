set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/profile.sh ${TAG:-r02} ${ARGS:---config c5} && grep -A22 -E "^-- k_(vrf_ck|kes|ocert_ck) " gpurun_out/prof_${TAG:-r02}/summary.txt | grep -E "^--|WAIT|ACTIVE_INST_ANY|WAVE_CYCLES|HBM|VALU wave" ; sed -n 3,30p gpurun_out/prof_${TAG:-r02}/summary.txt
