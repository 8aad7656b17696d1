"""Per-kernel sums of the counters in a rocprofv3 --pmc csv directory (tools/gpu_icache.sh)."""
import collections
import csv
import glob
import sys

rows = []
for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
acc = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.Counter()
for r in rows:
    k = r["Kernel_Name"].split("(")[0][:28]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    calls[(k, r["Counter_Name"])] += 1
names = ["SQC_ICACHE_REQ", "SQC_ICACHE_HITS", "SQC_ICACHE_MISSES", "SQC_ICACHE_MISSES_DUPLICATE", "SQ_IFETCH",
         "SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES", "SQ_INSTS_VALU"]
print(f"{'kernel':28s} " + " ".join(f"{n[-14:]:>14s}" for n in names) + "  miss/req  waitinst/wavecyc")
for k, d in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:14]:
    req = d.get("SQC_ICACHE_REQ", 0) or 1
    wc = d.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{k:28s} " + " ".join(f"{d.get(n, 0):14.4g}" for n in names) +
          f"  {d.get('SQC_ICACHE_MISSES', 0) / req:8.4f}  {d.get('SQ_WAIT_INST_ANY', 0) / wc:8.4f}")
