"""Sum rocprofv3 counter values per kernel from a counter_collection.csv (one --pmc pass).
usage: python3 tools/pmc_quick.py <dir> [kernel-substring ...]"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
want = sys.argv[2:]
tot = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if want and not any(w in k for w in want):
            continue
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
for k, c in sorted(tot.items()):
    wc = c.get("SQ_WAVE_CYCLES")
    s = " ".join(f"{n}={v:.3e}" + (f"({v / wc:.0%})" if wc and n.startswith("SQ_WAIT") else "") for n, v in sorted(c.items()))
    print(f"{k:20s} n={len(disp[k])} {s}")
