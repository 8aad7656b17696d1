"""Per-step kernel timeline from a rocprofv3 kernel trace (bench.py steps): for the
last step, each launch's start / end relative to the step's first kernel, in ms.
usage: trace_timeline.py <kt dir>"""
import csv
import glob
import sys

rows = []
for f in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0],
                     int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)))
rows.sort()
# steps start at the first k_key_insert / k_ocert_dedup after a k_leader
steps, cur = [], []
for r in rows:
    cur.append(r)
    if r[2] == "k_leader":
        steps.append(cur)
        cur = []
last = steps[-1]
# the step begins after the previous k_leader
t0 = min(r[0] for r in last if not r[2].startswith("k_synth"))
print(f"{len(steps)} steps; last step: {(max(r[1] for r in last) - t0) / 1e6:.3f} ms")
for s, e, k, g in sorted(last):
    if s < t0:
        continue
    print(f"{k:24s} grid {g:8d}  {(s - t0) / 1e6:8.3f} -> {(e - t0) / 1e6:8.3f}  ({(e - s) / 1e6:7.3f} ms)")
