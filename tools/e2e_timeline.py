"""Kernel + memory-copy timeline of the last praos_verify_header_bytes call in a rocprofv3
trace directory (--kernel-trace --memory-copy-trace): every event that ends within the last
`window` ms, times relative to the first of them.  usage: e2e_timeline.py <dir> [window_ms]"""
import csv
import glob
import sys

d = sys.argv[1]
win = float(sys.argv[2]) if len(sys.argv) > 2 else 22.0
ev = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:26],
                   f"q{r.get('Queue_Id', '?')}", r.get("Grid_Size_X", r.get("Grid_Size", ""))))
for f in glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", "copy"), "copy",
                   r.get("Size", "")))
ev.sort()
end = max(e[1] for e in ev)
sel = [e for e in ev if e[1] >= end - win * 1e6]
t0 = sel[0][0]
for s, e, name, q, g in sel:
    print(f"{name:26s} {q:6s} {g:>10s} {(s - t0) / 1e6:8.3f} -> {(e - t0) / 1e6:8.3f}  ({(e - s) / 1e6:7.3f} ms)")
