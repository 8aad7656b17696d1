"""Per-batch stage timeline of a replay (PRAOS_REPLAY_TRACE output): one block per replay call,
the stages of each batch (read / decode on the reader thread, chain, launch, wait / fold) with
start, end and duration in ms from the call's start.  usage: replay_trace.py <trace> [call ...]"""
import sys

runs, cur = [], []
for line in open(sys.argv[1]):
    p = line.split()
    if p[0] == "end":
        runs.append((cur, float(p[3])))
        cur = []
        continue
    cur.append((int(p[0]), p[1], float(p[2]), float(p[3]), int(p[4])))
sel = [int(x) for x in sys.argv[2:]] or range(len(runs))
for ri in sel:
    ev, end = runs[ri]
    print(f"call {ri}: {end:.2f} ms")
    for k, what, t0, t1, n in sorted(ev, key=lambda e: (e[0], e[2])):
        print(f"  {k:3d} {what:7s} {t0:8.2f} {t1:8.2f} ({t1 - t0:6.2f}) n={n}")
