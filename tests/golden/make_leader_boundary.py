#!/usr/bin/env python3
"""Leader-decision boundary vectors (checkLeaderNatValue, Praos.hs:549, cardano-ledger-core
taylorExpCmp in Fixed E34): for each (sigma, f) the exact leader value l* at which the
decision flips, found by bisection on the C oracle (oracle/praos.c orc_check_leader) and
re-derived by a pure-Python big-integer restatement, written with the pairs around it
(l*-2, l*-1 = leader; l*, l*+1 = not leader) and the Taylor iteration counts (the runs at
the boundary are the longest ones).  The same for the TPraos 512-bit form.

c_raw is activeSlotLog as praos_hip/fixed.py restates it (NonIntegral ln' in Fixed E34;
cardano-ledger-core is not vendored, so its last digits are unpinned): the vectors pin
the decision GIVEN c_raw -- which is what the ABI takes as input.

    python tests/golden/make_leader_boundary.py   # rewrites tests/golden/leader_boundary.json
"""
import json
import os
import sys
from fractions import Fraction

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "ouroboros-consensus_amd"))

R = 10 ** 34
C_RAW_NOTE = ("unpinned: c_raw = activeSlotLog f from praos_hip/fixed.py's restatement of cardano-ledger-core "
              "ln' (not vendored; constants recalled); the vectors pin the decision GIVEN c_raw, so a later "
              "correction of ln' changes c_raw and the boundaries without being a regression")


def leader_python(l, bound_bits, sigma_fp, c_raw):
    """checkLeaderNatValue restated on Python integers (floor = Haskell div)."""
    x = -((sigma_fp * c_raw) // R)
    q_num, q_den = (2 ** bound_bits) * R, (2 ** bound_bits - l)
    q = q_num // q_den                      # fromRational (certNatMax % (certNatMax - l))
    err, acc, n = x, R, 0
    while True:
        if n == 1000:
            return False, n
        k = n + 2
        errp = ((err * x) // R) // k
        accp = acc + err
        e = 3 * errp
        if q >= accp + e:
            return False, n + 1
        if q < accp - e:
            return True, n + 1
        err, acc, n = errp, accp, n + 1


def main():
    import oracle
    from praos_hip import fixed
    cases = [(Fraction(1, 3000), Fraction(1, 20)), (Fraction(1, 100), Fraction(1, 20)),
             (Fraction(17, 10007), Fraction(1, 20)), (Fraction(1, 2), Fraction(1, 20)),
             (Fraction(1), Fraction(1, 20)), (Fraction(3, 4), Fraction(1, 2)), (Fraction(1, 7), Fraction(9, 10)),
             (Fraction(1, 10 ** 9), Fraction(1, 20))]
    out = []
    for bits in (256, 512):
        check = oracle.check_leader if bits == 256 else oracle.check_leader512
        for sigma, f in cases:
            s_fp = fixed.from_rational(sigma)
            c_raw = fixed.active_slot_log(f)

            def lead(l):
                return check(l.to_bytes(bits // 8, "big"), s_fp, c_raw)[0]
            lo, hi = 0, 2 ** bits - 1          # lead(lo) and not lead(hi)
            assert lead(lo) and not lead(hi)
            while hi - lo > 1:
                mid = (lo + hi) // 2
                if lead(mid):
                    lo = mid
                else:
                    hi = mid
            vec = []
            for l in (hi - 2, hi - 1, hi, hi + 1):
                is_l, it = check(l.to_bytes(bits // 8, "big"), s_fp, c_raw)
                py_l, py_it = leader_python(l, bits, s_fp, c_raw)
                assert (is_l, it) == (py_l, py_it), (sigma, f, l)
                vec.append({"leader_value": hex(l), "is_leader": is_l, "iterations": it})
            assert [v["is_leader"] for v in vec] == [True, True, False, False]
            out.append({"bits": bits, "sigma": f"{sigma.numerator}/{sigma.denominator}",
                        "f": f"{f.numerator}/{f.denominator}", "sigma_fp": str(s_fp), "c_raw": str(c_raw),
                        "c_raw_parity": "unpinned",
                        "boundary": hex(hi), "vectors": vec})
    json.dump({"generator": "tests/golden/make_leader_boundary.py", "c_raw_parity": C_RAW_NOTE, "cases": out},
              open(os.path.join(HERE, "leader_boundary.json"), "w"), indent=1)
    print(len(out), "cases;", "max iterations", max(v["iterations"] for c in out for v in c["vectors"]))


if __name__ == "__main__":
    main()
