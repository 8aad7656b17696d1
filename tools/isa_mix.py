"""VALU instruction-class mix of a kernel from its gfx950 assembly, priced with the measured
issue-cost table (tools/microbench/intrate.hip, profiles/r05/intrate_issue_table.txt).

  python3 tools/isa_mix.py <file.s> <kernel symbol substring> [W]

Prints the static (unweighted) and loop-weighted class counts and the issue cost per VALU
instruction the mix implies at W waves per SIMD.  Loop weighting: every basic block inside a
backward branch's range counts `--trip` times per nesting level (a rough executed-mix proxy;
the rolled chains of the verify kernels are loops of 64 / 255 / 4 iterations)."""
import re
import sys

# SIMD cycles per wave64 instruction at W = 1, 2, 3, 4 (profiles/r05/intrate_issue_table.txt)
COST = {
    "vop2_simple": (5.02, 2.51, 2.79, 2.38),     # v_add_u32 class: plain 32-bit VOP2 ALU, no SGPR write
    "vop3": (5.39, 4.49, 4.37, 4.27),            # v_add3 / v_lshl_add / v_cndmask_e64 / v_fma_f64 class
    "mul32": (4.95, 4.38, 4.27, 4.20),           # v_mul_lo/hi_u32, 24-bit multiplies
    "mad64": (6.27, 5.22, 4.99, 4.87),           # v_mad_u64_u32 with per-chain operands
    "carry": (6.39, 4.80, 4.61, 4.45),           # v_add_co / v_addc_co / v_sub_co / v_subb_co (SGPR or VCC carry)
}
SIMPLE = re.compile(r"^v_(add|sub|subrev|and|or|xor|lshlrev|lshrrev|ashrrev|mov|not|max|min|bfe|alignbit|bfi|perm|"
                    r"cndmask)_(u32|i32|b32)(_e32)?$")


def classify(op, line):
    if op.startswith("v_mad_u64_u32") or op.startswith("v_mad_i64_i32"):
        return "mad64"
    if re.match(r"^v_(mul_lo|mul_hi|mul|mad|mul_hi)_(u32|i32)(_u24|_i24)?", op) or "u24" in op or "i24" in op:
        return "mul32"
    if re.match(r"^v_(add|sub|subrev)(c)?_co_u32", op) or op.startswith("v_addc") or op.startswith("v_subb"):
        return "carry"
    if op.endswith("_e64") or op.startswith("v_add3") or op.startswith("v_lshl_add") or op.startswith("v_lshl_or") \
            or op.startswith("v_and_or") or op.startswith("v_or3") or op.startswith("v_xad") or op.startswith("v_mad") \
            or "b64" in op or op.startswith("v_fma") or op.startswith("v_alignbyte") or op.startswith("v_bfe") \
            or op.startswith("v_perm") or op.startswith("v_bfi") or op.startswith("v_alignbit") \
            or op.startswith("v_cndmask_b32") and re.search(r"\bs\[\d+:\d+\]", line):
        return "vop3"
    if SIMPLE.match(op):
        return "vop2_simple"
    return "vop3"


def kernel_lines(path, sym):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sym in l.split(":")[0] and ":" in l)
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    return lines[start:end]


def main():
    path, sym = sys.argv[1], sys.argv[2]
    W = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    trip = 16
    body = kernel_lines(path, sym)
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = i
    depth = [0] * len(body)
    for i, l in enumerate(body):
        m = re.match(r"^\s+s_cbranch_\w+\s+(\.LBB\w+)", l) or re.match(r"^\s+s_branch\s+(\.LBB\w+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            for j in range(labels[m.group(1)], i + 1):
                depth[j] += 1
    static, weighted = {}, {}
    for i, l in enumerate(body):
        m = re.match(r"^\s+(v_\w+)", l)
        if not m or m.group(1).startswith("v_readfirstlane") or m.group(1).startswith("v_readlane") \
                or m.group(1).startswith("v_writelane"):
            continue
        c = classify(m.group(1), l)
        static[c] = static.get(c, 0) + 1
        weighted[c] = weighted.get(c, 0) + trip ** min(depth[i], 3)
    for name, cnt in (("static", static), ("loop-weighted", weighted)):
        tot = sum(cnt.values())
        cyc = sum(v * COST[k][W - 1] for k, v in cnt.items())
        mix = ", ".join(f"{k} {100.0 * v / tot:.1f}%" for k, v in sorted(cnt.items(), key=lambda kv: -kv[1]))
        print(f"{sym} {name}: {tot} VALU instructions; {mix}; issue cost at W={W}: {cyc / tot:.3f} SIMD cycles / instr")


if __name__ == "__main__":
    main()
