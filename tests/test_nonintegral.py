"""activeSlotLog = raw Fixed E34 value of cardano-ledger-core NonIntegral.ln' (1 - f)
(mkActiveSlotCoeff; consumed by checkLeaderNatValue, Praos.hs:549): the host restatement
praos_hip/fixed.py (raw integers) against the oracle's (oracle/nonintegral.py, exact
rationals floored to the 10^-34 grid), and both against the true ln to the continued
fraction's 10^-24 convergence bound.  cardano-ledger-core is not vendored, so the last
digits stay unpinned; test_gpu_group.py::test_c5_full_epoch_single_and_group8 pins the
decisions that depend on them."""
from fractions import Fraction

import pytest

FS = [Fraction(1, 20), Fraction(1, 10), Fraction(1, 2), Fraction(9, 10), Fraction(1, 1000), Fraction(99, 100),
      Fraction(3, 7), Fraction(1, 3), Fraction(1, 100000)]


@pytest.mark.parametrize("f", FS)
def test_ln_restatements_agree(f):
    import nonintegral
    from praos_hip import fixed
    a = fixed.active_slot_log(f)
    assert a == nonintegral.active_slot_log(f)
    assert a < 0
    assert abs(a - fixed.active_slot_log_decimal(f)) < 10 ** 11      # |error| < 1e-23


def test_ln_special_values():
    import nonintegral as N
    from praos_hip import fixed
    assert fixed.active_slot_log(1) == 0 and N.active_slot_log(1) == 0
    assert fixed.ln_fixed(fixed.R) == 0                              # ln' 1 = 0 (z = 0)
    e = fixed._exp(fixed.R)
    assert abs(e - 27182818284590452353602874713526624) < 10 ** 11
    for k in (-3, -1, 2, 5):                                         # ln' (e^k) ~ k
        assert abs(fixed.ln_fixed(fixed._ipow(e, k)) - k * fixed.R) < 10 ** 12
    with pytest.raises(ValueError):
        fixed.ln_fixed(0)
