#!/bin/bash
# Replay throughput of the C5 chain (tools/replay_bench.py --chain c5) under host thread-placement
# variants; saves the searched epoch-1 schedule so later runs skip the search.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/replay
mkdir -p $O
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null; \
  python3 -c "import os; print(len(os.sched_getaffinity(0)))"; } > $O/host_cpus.txt 2>&1
SIN=""
[ -f ouroboros-consensus_amd/praos_hip/data/c5_epoch1_schedule.npz ] && SIN="--schedule-in 1=ouroboros-consensus_amd/praos_hip/data/c5_epoch1_schedule.npz"
cat /sys/fs/cgroup/cpu.stat > $O/cpu_stat_before.txt 2>/dev/null
timeout -k 10 1100 python3 -u tools/replay_bench.py --chain c5 --epochs 2 --pools 3000 --epoch-length 8640000 \
  --batch-sizes ${BATCHES:-48000,96000} --members ${MEMBERS:-1,2} --reps ${REPS:-3} --schedule-out $O/sched $SIN \
  --env-variants "${VARIANTS:-PRAOS_REPLAY_PIN=0,PRAOS_COPY_THREADS=16;PRAOS_REPLAY_PIN=1,PRAOS_COPY_THREADS=16;PRAOS_REPLAY_PIN=0,PRAOS_COPY_THREADS=8;PRAOS_REPLAY_PIN=1,PRAOS_COPY_THREADS=8;PRAOS_REPLAY_PIN=1,PRAOS_COPY_THREADS=4}" \
  > $O/replay.jsonl 2> $O/replay.err || { echo REPLAYFAIL; tail -30 $O/replay.err; exit 1; }
cat /sys/fs/cgroup/cpu.stat > $O/cpu_stat_after.txt 2>/dev/null
cat $O/host_cpus.txt
paste $O/cpu_stat_before.txt $O/cpu_stat_after.txt 2>/dev/null
python3 -c "
import json
for l in open('$O/replay.jsonl'):
    d = json.loads(l); print(d['host_settings'], d['members'], d['batch_max'], d['value'], d['wall_ms'], d.get('walls_ms'), d['stages_ms'])
"
