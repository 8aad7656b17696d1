#!/usr/bin/env python3
"""Summarise a tools/profile.sh run (rocprofv3 kernel stats + PMC passes) into
profiles/<tag>_rocprof.txt and profiles/<tag>_pmc.json.

FETCH_SIZE / WRITE_SIZE are reported by rocprofv3 in KiB.  Per
/opt/skills/guides/MI355X_MICROARCH.md (HBM section) gfx950 FETCH_SIZE counts half the
bytes of wide streaming reads, so HBM read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE is
taken as is.  Per-lane (per header) figures divide by Grid_Size.

usage: prof_summary.py <prof dir> <tag>
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNELS = ("k_ocert", "k_ocert_ck", "k_kes", "k_kes_ck", "k_kes_leafkeys", "k_vrf", "k_vrf_ck", "k_vrf_v", "k_vrf_fin",
           "k_vrf_fin_nc", "k_vrf_tp", "k_leader", "k_key_precompute", "k_key_tables", "k_decode_praos", "k_synth_headers")


def short(name):
    return name.split("(")[0]


def main():
    d, tag = sys.argv[1], sys.argv[2]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lines = [f"rocprofv3 summary {tag}  (source: {d}, produced by tools/profile.sh + tools/prof_summary.py)", ""]
    stats = glob.glob(os.path.join(d, "kt", "*kernel_stats.csv"))
    if stats:
        lines.append("== kernel trace stats (rocprofv3 --kernel-trace --stats; bench.py --no-cpu --steps 5 --warmup 1) ==")
        lines.append(f"{'kernel':28s} {'calls':>6s} {'avg ms':>10s} {'min ms':>10s} {'max ms':>10s} {'%':>7s}")
        with open(stats[0]) as f:
            for r in csv.DictReader(f):
                lines.append(f"{short(r['Name'])[:28]:28s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e6:10.3f} "
                             f"{float(r['MinNs'])/1e6:10.3f} {float(r['MaxNs'])/1e6:10.3f} {float(r['Percentage']):7.2f}")
        lines.append("")
    trace = glob.glob(os.path.join(d, "kt", "*kernel_trace.csv"))
    if trace:
        # bench.py times each crypto kernel alone (serial launches after the timed
        # region) for the roofline; the timed steps run them concurrently on three
        # streams, which stretches each launch.  Split the trace the same way.
        with open(trace[0]) as f:
            rows = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                    for r in csv.DictReader(f)]
        crypto = [r for r in rows if r[0] in KERNELS and not r[0].startswith("k_synth") and r[2] - r[1] > 100_000]
        iso, conc = defaultdict(list), defaultdict(list)
        iso_avg = {}
        for k, s, e in crypto:
            overl = any(o is not None and o[1] < e and s < o[2] for o in crypto if o != (k, s, e))
            (conc if overl else iso)[k].append((e - s) / 1e6)
        lines.append("== per-launch durations split by overlap (launches > 0.1 ms) ==")
        lines.append(f"{'kernel':16s} {'isolated n':>10s} {'avg ms':>8s} {'concurrent n':>12s} {'avg ms':>8s}")
        for k in sorted(set(iso) | set(conc)):
            a = iso.get(k, [])
            b = conc.get(k, [])
            lines.append(f"{k:16s} {len(a):10d} {sum(a)/max(1,len(a)):8.3f} {len(b):12d} {sum(b)/max(1,len(b)):8.3f}")
            if a:
                iso_avg[k] = sum(a) / len(a)
        lines.append("")
    bench = os.path.join(d, "kt_bench.json")
    if os.path.exists(bench):
        lines.append("bench line of the traced run:")
        lines.append(open(bench).read().strip())
        lines.append("")
    acc = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> [(value, grid, vgpr, scratch)]
    meta = {}
    for fn in sorted(glob.glob(os.path.join(d, "pmc*", "*counter_collection.csv"))):
        with open(fn) as f:
            for r in csv.DictReader(f):
                k = short(r["Kernel_Name"])
                if k not in KERNELS:
                    continue
                acc[k][r["Counter_Name"]].append((float(r["Counter_Value"]), int(r["Grid_Size"])))
                meta[k] = {"vgpr": int(r["VGPR_Count"]), "agpr": int(r["Accum_VGPR_Count"]),
                           "sgpr": int(r["SGPR_Count"]), "scratch_per_lane": int(r["Scratch_Size"]),
                           "lds": int(r["LDS_Block_Size"])}
    out = {}
    if acc:
        lines.append("== PMC (one counter group per pass; bench.py <args> --no-cpu --steps 1 --warmup 0) ==")
        lines.append("per dispatch (mean over dispatches), and per lane = per header / signature")
        for k in KERNELS:
            if k not in acc:
                continue
            lines.append(f"-- {k}  {meta[k]}")
            o = {"meta": meta[k]}
            for c, vals in sorted(acc[k].items()):
                v = sum(x for x, _ in vals) / len(vals)
                g = sum(gg for _, gg in vals) / len(vals)
                o[c] = {"per_dispatch": v, "per_lane": v / g, "grid": g}
                lines.append(f"   {c:24s} {v:16.4e}  per lane {v / g:12.2f}")
            if "FETCH_SIZE" in o:
                rb = 2 * 1024 * o["FETCH_SIZE"]["per_lane"]
                o["hbm_read_bytes_per_lane"] = rb
                lines.append(f"   HBM read bytes/lane (2 x FETCH_SIZE KiB, gfx950 correction): {rb:.0f}")
            if "WRITE_SIZE" in o:
                wb = 1024 * o["WRITE_SIZE"]["per_lane"]
                o["hbm_write_bytes_per_lane"] = wb
                lines.append(f"   HBM write bytes/lane (WRITE_SIZE KiB): {wb:.0f}")
            if "SQ_INSTS_VALU" in o:
                lines.append(f"   VALU wave-instructions per wave (one item per lane): "
                             f"{o['SQ_INSTS_VALU']['per_lane'] * 64:.0f}")
            out[k] = o
    # per-launch HBM traffic for bench.py's roofline.traffic (FETCH x2 gfx950 read correction)
    workload = None
    if os.path.exists(bench):
        try:
            workload = json.loads(open(bench).read().strip().splitlines()[-1])["config"]["workload"]
        except (ValueError, KeyError, IndexError):
            workload = None
    traffic = {}
    if not trace:
        iso_avg = {}
    for k, o in out.items():
        if "FETCH_SIZE" in o and "WRITE_SIZE" in o:
            rd = 2 * 1024 * o["FETCH_SIZE"]["per_dispatch"]
            wr = 1024 * o["WRITE_SIZE"]["per_dispatch"]
            traffic[k] = {"bytes_per_launch": rd + wr, "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                          "items_per_launch": o["FETCH_SIZE"]["grid"], "bytes_per_item": (rd + wr) / o["FETCH_SIZE"]["grid"],
                          "rocprof_isolated_avg_ms": iso_avg.get(k)}
    os.makedirs(os.path.join(root, "profiles"), exist_ok=True)
    if traffic and workload:
        with open(os.path.join(root, "profiles", f"{tag}_traffic.json"), "w") as f:
            json.dump({"workload": workload, "source": f"profiles/{tag}_rocprof.txt (tools/profile.sh)",
                       "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                                 "bytes = 2 x FETCH_SIZE KiB x 1024 (gfx950 half-count correction) + WRITE_SIZE KiB x 1024",
                       "kernels": traffic}, f, indent=1)
    with open(os.path.join(root, "profiles", f"{tag}_rocprof.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
    if out:
        with open(os.path.join(root, "profiles", f"{tag}_pmc.json"), "w") as f:
            json.dump(out, f, indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
