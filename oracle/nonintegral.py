"""ORACLE (test infrastructure only: imported by tests/, never by the product path).

cardano-ledger-core `Cardano.Ledger.NonIntegral.ln'` and `mkActiveSlotCoeff`'s
`unActiveSlotLog = floor (fpPrecision * ln' ((1 :: FixedPoint) - fromRational f))`,
restated over a Data.Fixed E34 model built on exact rationals (every operation
rounds its exact rational result down to the 10^-34 grid, as Data.Fixed's `*`, `/`
and `fromRational` do) -- deliberately a different construction from the raw-integer
one in praos_hip/fixed.py, which the tests compare it with.

The package is not in /root/reference ("[ext]"): the algorithm is the
published one (exp' by a Taylor series after scaling, findE / splitLn, ln(1+z) by its
continued fraction through the Wallis recurrences) with its constants as recalled
(maxN = 1000, eps = 10^-24): PARITY UNPINNED in the last ~10 digits of c_raw; the
leader decisions of the shipped chains are shown invariant over a band far wider
than that (tests/test_gpu_group.py::test_c5_full_epoch_single_and_group8).
"""
from fractions import Fraction
from math import floor

RES = 10 ** 34
MAX_N = 1000


class Fx:
    """Data.Fixed E34: the value is a multiple of 10^-34, kept as an exact Fraction."""
    __slots__ = ("q",)

    def __init__(self, q):
        q = Fraction(q)
        self.q = Fraction(floor(q * RES), RES)          # fromRational = floor to the grid

    def __add__(self, o): return Fx(self.q + o.q)       # exact on the grid
    def __sub__(self, o): return Fx(self.q - o.q)
    def __mul__(self, o): return Fx(self.q * o.q)       # MkFixed (div (a*b) res)
    def __truediv__(self, o): return Fx(self.q / o.q)   # MkFixed (div (a*res) b)
    def __lt__(self, o): return self.q < o.q
    def __le__(self, o): return self.q <= o.q
    def __eq__(self, o): return self.q == o.q
    def __abs__(self): return Fx(abs(self.q))
    def raw(self): return int(self.q * RES)


EPS = Fx(Fraction(1, 10 ** 24))
ONE, ZERO = Fx(1), Fx(0)


def ipow(x: Fx, n: int) -> Fx:
    def pos(x, n):
        if n == 0:
            return ONE
        d, m = divmod(n, 2)
        if m == 0:
            y = pos(x, d)
            return y * y
        return x * pos(x, n - 1)
    return ONE / pos(x, -n) if n < 0 else pos(x, n)


def taylor_exp(x: Fx) -> Fx:
    acc, last = ONE, ONE
    for k in range(1, MAX_N):
        nxt = (last * x) / Fx(k)
        if abs(nxt) < EPS:
            break
        acc, last = acc + nxt, nxt
    return acc


def exp_(x: Fx) -> Fx:
    if x < ZERO:
        return ONE / exp_(Fx(-x.q))
    n = -floor(-x.q)                       # ceiling
    if n == 0:
        return ONE
    return ipow(taylor_exp(x / Fx(n)), n)


def find_e(e: Fx, x: Fx) -> int:
    n = 0
    if ONE <= x:
        while ipow(e, n + 1) <= x:
            n += 1
    else:
        while x < ipow(e, n):
            n -= 1
    return n


def lncf(z: Fx) -> Fx:
    a2, b2, a1, b1 = ONE, ZERO, ZERO, ONE
    conv = ZERO
    for n in range(1, MAX_N + 1):
        an = z if n == 1 else Fx((n // 2) ** 2) * z
        bn = Fx(n)
        a, b = bn * a1 + an * a2, bn * b1 + an * b2
        conv = a / b
        if abs(conv - a1 / b1) < EPS:
            return conv
        a2, b2, a1, b1 = a1, b1, a, b
    return conv


def ln_(x: Fx) -> Fx:
    assert ZERO < x
    e = exp_(ONE)
    n = find_e(e, x)
    z = x / ipow(e, n) - ONE
    return Fx(n) if z == ZERO else Fx(n) + lncf(z)


def active_slot_log(f) -> int:
    """unActiveSlotLog (raw Fixed E34 integer) for active slot coefficient f."""
    f = Fraction(f)
    if f == 1:
        return 0
    return ln_(ONE - Fx(f)).raw()
