set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCHFAIL; tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
bash tools/profile.sh ${TAG:-r02} --config c5 && tail -60 gpurun_out/prof_${TAG:-r02}/summary.txt
