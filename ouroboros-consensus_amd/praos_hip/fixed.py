"""Fixed E34 host helpers (cardano-ledger-core `FixedPoint` = Data.Fixed E34).

`fromRational q` floors q * 10^34 (Data.Fixed); `activeSlotLog f` is the raw
Fixed value of ln'(1 - f) computed by cardano-ledger-core `NonIntegral.ln'`
(a continued fraction evaluated in FixedPoint).  That library is not in
/root/reference, so `active_slot_log` here returns floor(10^34 * ln(1 - f))
from a 100-digit evaluation: PARITY UNPINNED in the last digits of c.  The
batch validator takes c_raw as an input (praos_params.c_raw), so a caller that
has the reference's own activeSlotLog value gets bit-exact leader decisions.
"""
from decimal import Decimal, getcontext
from fractions import Fraction

R = 10 ** 34


def from_rational(q) -> int:
    q = Fraction(q)
    return (q.numerator * R) // q.denominator


def active_slot_log(f) -> int:
    f = Fraction(f)
    if f == 1:
        return 0
    getcontext().prec = 100
    v = (Decimal(1) - Decimal(f.numerator) / Decimal(f.denominator)).ln() * Decimal(R)
    return int(v.to_integral_value(rounding="ROUND_FLOOR"))
