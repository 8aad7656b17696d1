set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/make_schedule.py c5 --blocks 3000 --window 20000 --out gpurun_out/c5_probe.npz > gpurun_out/sched_probe.log 2>&1 || { echo SCHEDFAIL; tail -20 gpurun_out/sched_probe.log; exit 1; }
tail -4 gpurun_out/sched_probe.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "not c5" > gpurun_out/t_gpu.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/t_gpu.log; exit 1; }
tail -5 gpurun_out/t_gpu.log
