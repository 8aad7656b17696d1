#!/usr/bin/env python3
"""Generate ouroboros-consensus_amd/csrc/fe_cols.hpp: the field products of fe25519.hpp with
the MACs of each product-scanning column software-pipelined so no carry needs s_nop padding.

fe25519.hpp's FE_MAC reads the carry a mad wrote with `s_nop 1` in between (gfx950 wants two
wait states between a VALU carry write and a VALU carry read); FE_MAC2 interleaves two products
and pads with `s_nop 0`.  Here every column is one asm block whose carry reads sit >= 2
instructions after their writes:

  one product  (m MACs, carries rotate over VCC and two SGPR pairs):
      M0 M1 M2 A0 M3 A1 M4 A2 ... M(m-1) A(m-3) A(m-2) A(m-1)
  two products (carries rotate over two registers each: VCC / s1 and s2 / s3):
      M'0 M"0 M'1 M"1  A'0 A"0 M'2 M"2  A'1 A"1 M'3 M"3 ...  A'(m-2) A"(m-2) A'(m-1) A"(m-1)

(M = v_mad_u64_u32 acc += a*b with carry-out, A = v_addc_co_u32 top += carry; the first A of a
column starts top from zero.)  Only columns with one MAC (one product) or fewer than three (one
product) keep a nop.  A two-product column longer than PAIR_CHUNK MACs is split into two asm
blocks at a point where no carry is in flight (the asm operand count stays below 30).

Issue cost, profiles/r05/intrate_issue_table.txt at 3 waves per SIMD: FE_MAC 5.14, FE_MAC2 4.71,
no-nop SGPR-carry MACs 4.47 SIMD cycles per VALU instruction.

Usage: python3 tools/gen_fe_cols.py > ouroboros-consensus_amd/csrc/fe_cols.hpp
"""

PAIR_CHUNK = 5


def mul_cols():
    """[(k, [(i, j), ...])] of an 8x8 product, columns 1..13 (0 and 14 need no carry)."""
    return [(k, [(i, k - i) for i in range(8) if 0 <= k - i <= 7]) for k in range(1, 14)]


def sq_cols():
    """cross products a_i a_j, i < j; columns 3..13 (1 and 2 need no carry: see fe_sq_g)."""
    return [(k, [(i, k - i) for i in range(8) if i < k - i <= 7]) for k in range(3, 14)]


def single_col_asm(m):
    """asm text of one column of one product with m MACs.
    operands: %0 acc, %1 top, %2 cA, %3 cB, %4 zero, a_j = %(5+2j), b_j = %(6+2j)"""
    car = ["vcc", "%2", "%3"]

    def M(j):
        return f"v_mad_u64_u32 %0, {car[j % 3]}, %{5 + 2 * j}, %{6 + 2 * j}, %0"

    def A(j):
        c = car[j % 3]
        if j == 0:
            return "v_addc_co_u32 %1, vcc, 0, %4, vcc"
        return f"v_addc_co_u32 %1, {c}, 0, %1, {c}"

    if m == 1:
        seq = [M(0), "s_nop 1", A(0)]
    elif m == 2:
        seq = [M(0), M(1), "s_nop 0", A(0), A(1)]
    else:
        seq = [M(0), M(1), M(2)]
        for j in range(3, m):
            seq += [A(j - 3), M(j)]
        seq += [A(m - 3), A(m - 2), A(m - 1)]
    return seq


def pair_chunk_asm(m, first):
    """asm text of m MACs of a column of each of two products.
    operands: %0 acc1, %1 acc2, %2 top1, %3 top2, %4 s1, %5 s2, %6 s3, %7 zero,
    a1_j = %(8+4j), b1_j = %(9+4j), a2_j = %(10+4j), b2_j = %(11+4j)"""
    c1 = ["vcc", "%4"]
    c2 = ["%5", "%6"]

    def M1(j):
        return f"v_mad_u64_u32 %0, {c1[j % 2]}, %{8 + 4 * j}, %{9 + 4 * j}, %0"

    def M2(j):
        return f"v_mad_u64_u32 %1, {c2[j % 2]}, %{10 + 4 * j}, %{11 + 4 * j}, %1"

    def A1(j):
        c = c1[j % 2]
        if j == 0 and first:
            return "v_addc_co_u32 %2, vcc, 0, %7, vcc"
        return f"v_addc_co_u32 %2, {c}, 0, %2, {c}"

    def A2(j):
        c = c2[j % 2]
        if j == 0 and first:
            return f"v_cndmask_b32_e64 %3, 0, 1, {c}"
        return f"v_addc_co_u32 %3, {c}, 0, %3, {c}"

    if m == 1:
        return [M1(0), M2(0), "s_nop 0", A1(0), A2(0)]
    seq = [M1(0), M2(0), M1(1), M2(1)]
    for j in range(2, m):
        seq += [A1(j - 2), A2(j - 2), M1(j), M2(j)]
    seq += [A1(m - 2), A2(m - 2), A1(m - 1), A2(m - 1)]
    return seq


def asm_text(seq):
    return '"' + "\\n\\t".join(seq) + '"'


def emit_single(name, cols, a, b, out):
    for k, ij in cols:
        m = len(ij)
        ins = ", ".join(f'"v"({a}.v[{i}]), "v"({b}.v[{j}])' for i, j in ij)
        out.append(f"  {{  // column {k}: {m} MAC{'s' if m > 1 else ''}")
        out.append("    uint64_t cA_, cB_;")
        out.append(f"    asm({asm_text(single_col_asm(m))}")
        out.append('        : "+v"(acc), "=&v"(top), "=&s"(cA_), "=&s"(cB_)')
        out.append(f'        : "v"(0u), {ins}')
        out.append('        : "vcc");')
        out.append("  }")
        out.append(f"  t[{k}] = (uint32_t)acc;")
        out.append("  acc = (acc >> 32) | ((uint64_t)top << 32);")


def chunks(m):
    if m <= PAIR_CHUNK:
        return [m]
    h = (m + 1) // 2
    return [h, m - h]


def emit_pair(cols, a1, b1, a2, b2, out):
    for k, ij in cols:
        m = len(ij)
        out.append(f"  {{  // column {k}: {m} MAC{'s' if m > 1 else ''} per product")
        out.append("    uint64_t s1_, s2_, s3_;")
        pos = 0
        for ci, cm in enumerate(chunks(m)):
            part = ij[pos:pos + cm]
            pos += cm
            first = ci == 0
            ins = ", ".join(f'"v"({a1}.v[{i}]), "v"({b1}.v[{j}]), "v"({a2}.v[{i}]), "v"({b2}.v[{j}])'
                            for i, j in part)
            tops = '"=&v"(top1), "=&v"(top2)' if first else '"+v"(top1), "+v"(top2)'
            out.append(f"    asm({asm_text(pair_chunk_asm(cm, first))}")
            out.append(f'        : "+v"(acc1), "+v"(acc2), {tops}, "=&s"(s1_), "=&s"(s2_), "=&s"(s3_)')
            out.append(f'        : "v"(0u), {ins}')
            out.append('        : "vcc");')
        out.append("  }")
        out.append(f"  t1[{k}] = (uint32_t)acc1;")
        out.append(f"  t2[{k}] = (uint32_t)acc2;")
        out.append("  acc1 = (acc1 >> 32) | ((uint64_t)top1 << 32);")
        out.append("  acc2 = (acc2 >> 32) | ((uint64_t)top2 << 32);")


def main():
    o = []
    o.append("// fe_cols.hpp -- GENERATED by tools/gen_fe_cols.py; do not edit.")
    o.append("//")
    o.append("// The 512-bit products of fe25519.hpp (fe_mul, fe_sq, fe_mul2, fe_sq2) with each")
    o.append("// product-scanning column one asm block whose carry reads sit >= 2 instructions after")
    o.append("// their writes (no s_nop padding but in columns of one or two MACs); see the generator's")
    o.append("// docstring for the instruction order.  Included by fe25519.hpp (PRAOS_MACG).")
    o.append("#pragma once")
    o.append("")
    # single product
    o.append("// t[0 .. 16) = a * b")
    o.append("FE_INLINE void fe_prod_g(uint32_t (&t)[16], const fe& a, const fe& b) {")
    o.append("  uint64_t acc = (uint64_t)a.v[0] * b.v[0];")
    o.append("  uint32_t top;")
    o.append("  t[0] = (uint32_t)acc;")
    o.append("  acc >>= 32;")
    emit_single("mul", mul_cols(), "a", "b", o)
    o.append("  acc += (uint64_t)a.v[7] * b.v[7];           // column 14: the product's top 64 bits, no carry")
    o.append("  t[14] = (uint32_t)acc;")
    o.append("  t[15] = (uint32_t)(acc >> 32);")
    o.append("}")
    o.append("")
    o.append("// t[0 .. 16) = sum over i < j of a_i a_j 2^(32(i+j))  (the cross products, not doubled)")
    o.append("FE_INLINE void fe_cross_g(uint32_t (&t)[16], const fe& a) {")
    o.append("  uint32_t top;")
    o.append("  t[0] = 0;")
    o.append("  uint64_t acc = (uint64_t)a.v[0] * a.v[1];      // column 1")
    o.append("  t[1] = (uint32_t)acc;")
    o.append("  acc = (acc >> 32) + (uint64_t)a.v[0] * a.v[2];  // column 2: < 2^32 + (2^32-1)^2, no carry")
    o.append("  t[2] = (uint32_t)acc;")
    o.append("  acc >>= 32;")
    emit_single("sq", sq_cols(), "a", "a", o)
    o.append("  t[14] = (uint32_t)acc;                         // column 14 has no cross product")
    o.append("  t[15] = (uint32_t)(acc >> 32);")
    o.append("}")
    o.append("")
    o.append("// t1 = a1 b1, t2 = a2 b2, MACs of the two products interleaved")
    o.append("FE_INLINE void fe_prod2_g(uint32_t (&t1)[16], uint32_t (&t2)[16], const fe& a1, const fe& b1,")
    o.append("                          const fe& a2, const fe& b2) {")
    o.append("  uint64_t acc1 = (uint64_t)a1.v[0] * b1.v[0], acc2 = (uint64_t)a2.v[0] * b2.v[0];")
    o.append("  uint32_t top1, top2;")
    o.append("  t1[0] = (uint32_t)acc1;")
    o.append("  t2[0] = (uint32_t)acc2;")
    o.append("  acc1 >>= 32;")
    o.append("  acc2 >>= 32;")
    emit_pair(mul_cols(), "a1", "b1", "a2", "b2", o)
    o.append("  acc1 += (uint64_t)a1.v[7] * b1.v[7];")
    o.append("  acc2 += (uint64_t)a2.v[7] * b2.v[7];")
    o.append("  t1[14] = (uint32_t)acc1;")
    o.append("  t2[14] = (uint32_t)acc2;")
    o.append("  t1[15] = (uint32_t)(acc1 >> 32);")
    o.append("  t2[15] = (uint32_t)(acc2 >> 32);")
    o.append("}")
    o.append("")
    o.append("// the cross products of a1 and of a2, interleaved")
    o.append("FE_INLINE void fe_cross2_g(uint32_t (&t1)[16], uint32_t (&t2)[16], const fe& a1, const fe& a2) {")
    o.append("  uint32_t top1, top2;")
    o.append("  t1[0] = 0;")
    o.append("  t2[0] = 0;")
    o.append("  uint64_t acc1 = (uint64_t)a1.v[0] * a1.v[1], acc2 = (uint64_t)a2.v[0] * a2.v[1];")
    o.append("  t1[1] = (uint32_t)acc1;")
    o.append("  t2[1] = (uint32_t)acc2;")
    o.append("  acc1 = (acc1 >> 32) + (uint64_t)a1.v[0] * a1.v[2];")
    o.append("  acc2 = (acc2 >> 32) + (uint64_t)a2.v[0] * a2.v[2];")
    o.append("  t1[2] = (uint32_t)acc1;")
    o.append("  t2[2] = (uint32_t)acc2;")
    o.append("  acc1 >>= 32;")
    o.append("  acc2 >>= 32;")
    emit_pair(sq_cols(), "a1", "a1", "a2", "a2", o)
    o.append("  t1[14] = (uint32_t)acc1;")
    o.append("  t2[14] = (uint32_t)acc2;")
    o.append("  t1[15] = (uint32_t)(acc1 >> 32);")
    o.append("  t2[15] = (uint32_t)(acc2 >> 32);")
    o.append("}")
    print("\n".join(o))


if __name__ == "__main__":
    main()
