"""GPU parity of the arithmetic layers (through the C ABI self-test entry points)
against Python big integers, hashlib and the C oracle.  Bit-exact."""
import hashlib

import numpy as np
import pytest

from helpers import L, P, arr, b2b, rbytes, rng

pytestmark = pytest.mark.gpu


def _edge_values():
    v = [0, 1, 2, 19, P - 1, P, P + 1, 2 * P - 1, 2 * P, 2 ** 255 - 1, 2 ** 255, 2 ** 256 - 1, 2 ** 256 - 38,
         2 ** 256 - 39, 38, 2 ** 32 - 1, 2 ** 224]
    return [x % 2 ** 256 for x in v]


def _fe_inputs(seed, n):
    r = rng(seed)
    xs = _edge_values() + [r.getrandbits(256) for _ in range(n)]
    ys = list(reversed(_edge_values())) + [r.getrandbits(256) for _ in range(n)]
    return xs, ys


def _to(xs):
    return arr([x.to_bytes(32, "little") for x in xs], 32)


def _from(a):
    return [int.from_bytes(bytes(row), "little") for row in a]


@pytest.mark.parametrize("op", ["mul", "sq", "add", "sub"])
def test_fe_ring_ops(ctx, op):
    xs, ys = _fe_inputs(1, 400)
    code = {"mul": 0, "sq": 1, "add": 2, "sub": 3}[op]
    out = _from(ctx.debug_fe(code, _to(xs), _to(ys)))
    for x, y, z in zip(xs, ys, out):
        want = {"mul": x * y, "sq": x * x, "add": x + y, "sub": x - y}[op] % P
        assert z < 2 ** 256 and z % P == want, (op, hex(x), hex(y))


def _rare_fold_pairs():
    """(op, x, y) pairs whose second 2^256 fold carries (add, mul) or borrows (sub) out of limb 0,
    the branch fe25519.hpp takes with probability < 2^-21 on random operands (PRAOS_RED_BRANCH)."""
    m = 2 ** 256
    pairs = [("add", m - 1, 2 ** 32 - 9), ("add", m - 1, m - 9), ("add", m - 1, m - 1),
             ("add", m - 38, m - 1), ("sub", 3, 2 ** 32), ("sub", 0, m - 5), ("sub", 37, m - 1),
             ("sub", 0, 1), ("sub", 0, m - 1)]
    # (2^256 - 1) b folds to 37 b - 38 (b < 2^256 / 37): limb 0 = 2^32 - 1 for b = 2^32 j + 1, and
    # 37 b - 38 >= 2^256 - 38 (the carry runs through every limb) for b = ceil(2^256 / 37)
    pairs += [("mul", m - 1, 2 ** 32 * j + 1) for j in (1, 2, 3, 2 ** 64, 2 ** 190)]
    pairs += [("mul", m - 1, -(-m // 37)), ("mul", -(-m // 37), m - 1)]
    return pairs


def test_fe_rare_fold_carry(ctx):
    code = {"mul": 0, "add": 2, "sub": 3}
    for op in code:
        pr = [(x, y) for o, x, y in _rare_fold_pairs() if o == op]
        xs, ys = [x for x, _ in pr], [y for _, y in pr]
        out = _from(ctx.debug_fe(code[op], _to(xs), _to(ys)))
        for x, y, z in zip(xs, ys, out):
            want = {"mul": x * y, "add": x + y, "sub": x - y}[op] % P
            assert z < 2 ** 256 and z % P == want, (op, hex(x), hex(y))


def test_fe_invert_pow_canon(ctx):
    xs, _ = _fe_inputs(2, 200)
    inv = _from(ctx.debug_fe(4, _to(xs)))
    pw = _from(ctx.debug_fe(5, _to(xs)))
    can = _from(ctx.debug_fe(6, _to(xs)))
    for x, a, b, c in zip(xs, inv, pw, can):
        assert a % P == pow(x % P, P - 2, P)
        assert b % P == pow(x % P, (P - 5) // 8, P)
        assert c == x % P


def test_fe_invert_gcd_vs_fermat(ctx):
    """The binary-GCD inversion (fe_inv_gcd.hpp, op 8) and Fermat's chain (op 7) give the same
    field element on edge, structured and random inputs, weakly reduced (< 2^256)."""
    xs, _ = _fe_inputs(5, 3000)
    xs += [2 ** k for k in range(256)] + [P - 2 ** k for k in range(255)] + [2 ** k - 1 for k in range(1, 257)]
    a, b = 1, 1
    while b < 2 ** 256:
        xs.append(b)
        a, b = b, a + b
    g = _from(ctx.debug_fe(8, _to(xs)))
    f = _from(ctx.debug_fe(7, _to(xs)))
    for x, u, v in zip(xs, g, f):
        assert u % P == v % P == pow(x % P, P - 2, P), hex(x)


def test_sha512_stream(ctx):
    r = rng(3)
    lens = list(range(0, 140)) + [300, 397, 461, 511, 512, 1000]
    msgs = [rbytes(r, n) for n in lens]
    pre = [rbytes(r, 64) for _ in lens]
    out = ctx.debug_sha512(arr(pre, 64), msgs)
    for p, m, o in zip(pre, msgs, out):
        assert bytes(o) == hashlib.sha512(p + m).digest(), len(m)


def test_blake2b_64(ctx):
    r = rng(4)
    ins = [rbytes(r, 64) for _ in range(300)]
    out = ctx.debug_blake2b(arr(ins, 64))
    for i, o in zip(ins, out):
        assert bytes(o) == b2b(i)


def test_sc_reduce(ctx):
    r = rng(5)
    xs = [0, 1, L - 1, L, L + 1, 2 * L, 2 ** 512 - 1, (2 ** 512 - 1) // L * L] + \
         [r.getrandbits(512) for _ in range(500)]
    out = ctx.debug_sc_reduce(arr([x.to_bytes(64, "little") for x in xs], 64))
    for x, o in zip(xs, out):
        assert int.from_bytes(bytes(o), "little") == x % L


def test_decode_reencode(ctx, oracle):
    r = rng(6)
    ins = [rbytes(r, 32) for _ in range(400)]
    # valid points, non-canonical y, small order, sign-bit games
    ins += [oracle.ed25519_pk(rbytes(r, 32)) for _ in range(50)]
    ins += [(P + k).to_bytes(32, "little") for k in range(0, 19)]
    ins += [bytes([1] + [0] * 30 + [0x80]), bytes(32), bytes([0] * 31 + [0x80])]
    out, ok = ctx.debug_decode(arr(ins, 32))
    for i, o, k in zip(ins, out, ok):
        want_ok, want = oracle.reencode(i)
        assert bool(k) == want_ok, i.hex()
        if want_ok:
            assert bytes(o) == want, i.hex()


def test_scalarmult_base(ctx, oracle):
    r = rng(7)
    ss = [0, 1, 2, 8, L - 1, L, 2 ** 255 - 1] + [r.getrandbits(255) for _ in range(300)]
    sb = [s.to_bytes(32, "little") for s in ss]
    out = ctx.debug_scalarmult_base(arr(sb, 32))
    for s, o in zip(sb, out):
        assert bytes(o) == oracle.scalarmult_base(s), s.hex()


def test_hash_to_curve(ctx, oracle):
    r = rng(8)
    pks = [oracle.vrf_pk(rbytes(r, 32)) for _ in range(100)]
    al = [rbytes(r, 32) for _ in pks]
    out = ctx.debug_hash_to_curve(arr(pks, 32), arr(al, 32))
    for pk, a, o in zip(pks, al, out):
        assert bytes(o) == oracle.vrf_hash_to_curve(pk, a)
