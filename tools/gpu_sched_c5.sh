set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u tools/make_schedule.py c5 --window 400000 --out gpurun_out/c5_schedule.npz > gpurun_out/sched_c5.log 2>&1 || { echo SCHEDFAIL; tail -20 gpurun_out/sched_c5.log; exit 1; }
tail -3 gpurun_out/sched_c5.log
