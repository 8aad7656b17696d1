"""GPU debug: leader check per item vs oracle, with Taylor iteration counts."""
import math, os, sys
from fractions import Fraction
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, p) for p in ("tests", "oracle", "ouroboros-consensus_amd")]
import numpy as np
import oracle
import praos_hip
from praos_hip import fixed
from helpers import rng, arr
c_raw = fixed.active_slot_log(Fraction(1, 20))
r = rng(14)
ls, xs, sfs = [], [], []
sigmas = [Fraction(1, 3000), Fraction(1, 100), Fraction(1, 2), Fraction(1), Fraction(0), Fraction(17, 10007)]
for i in range(400):
    s = sigmas[i % len(sigmas)] if i < 60 else Fraction(r.randrange(1, 10 ** 6), 10 ** 6 + r.randrange(10 ** 6))
    sf = fixed.from_rational(s)
    if i % 3 == 0:
        p = 1 - math.exp(float(s) * math.log(0.95))
        l = int(p * 2 ** 256) + r.randrange(-3, 4) * 2 ** 200
        l = min(max(l, 0), 2 ** 256 - 1)
    else:
        l = r.getrandbits(256) >> r.randrange(0, 32)
    R = 10 ** 34
    x = -((sf * c_raw) // R)
    ls.append(l.to_bytes(32, "big")); xs.append(x.to_bytes(16, "little")); sfs.append(sf)
ctx = praos_hip.Context(0)
res, it = ctx.debug_leader(arr(ls, 32), arr(xs, 16))
bad = 0
for i, (lb, sf) in enumerate(zip(ls, sfs)):
    w, wi = oracle.check_leader(lb, sf, c_raw)
    if bool(res[i]) != w or it[i] != wi:
        bad += 1
        if bad < 15:
            print("item", i, "gpu", res[i], it[i], "oracle", w, wi, "x", int.from_bytes(xs[i], "little"), "l", lb.hex())
print("mismatches", bad, "of", len(ls))
