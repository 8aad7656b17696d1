"""CPU: the oracle pinned against the reference's golden KATs, the standards'
known-answer tests and independent restatements (hashlib, Python ints)."""
import hashlib
import json
import os
from fractions import Fraction

import pytest

from helpers import L, P, b2b, corrupt, rbytes, rng

HERE = os.path.dirname(os.path.abspath(__file__))
KATS = json.load(open(os.path.join(HERE, "golden", "reference_kats.json")))["kats"]
H = bytes.fromhex


def test_hashes_vs_hashlib(oracle):
    r = rng(1)
    for n in list(range(0, 260, 7)) + [1000]:
        m = rbytes(r, n)
        assert oracle.sha512(m) == hashlib.sha512(m).digest()
        assert oracle.blake2b(m, 32) == b2b(m)
        assert oracle.blake2b(m, 28) == b2b(m, 28)


def test_rfc8032_vectors(oracle):
    # RFC 8032 sec. 7.1 TEST 1-3
    vec = [("9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60",
            "d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a", "",
            "e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e065224901555fb8821590a33bacc61e39701cf9b46bd25bf5f0595bbe24655141438e7a100b"),
           ("4ccd089b28ff96da9db6c346ec114e0f5b8a319f35aba624da8cf6ed4fb8a6fb",
            "3d4017c3e843895a92b70aa74d1b7ebc9c982ccf2ec4968cc0cd55f12af4660c", "72",
            "92a009a9f0d4cab8720e820b5f642540a2b27b5416503f8fb3762223ebdb69da085ac1e43e15996e458f3613d0f11d8c387b2eaeb4302aeeb00d291612bb0c00"),
           ("c5aa8df43f9f837bedb7442f31dcb7b166d38535076f094b85ce3a2e0b4458f7",
            "fc51cd8e6218a1a38da47ed00230f0580816ed13ba3303ac5deb911548908025", "af82",
            "6291d657deec24024827e69c3abe01a30ce548a284743a445e3680d7db5ac3ac18ff9b538d16f290ae67f760984dc6594a7c15e9716ed28dc027beceea1ec40a")]
    for sk, pk, m, sig in vec:
        assert oracle.ed25519_pk(H(sk)) == H(pk)
        assert oracle.ed25519_sign(H(sk), H(m)) == H(sig)
        assert oracle.ed25519_verify(H(pk), H(m), H(sig))
        assert not oracle.ed25519_verify(H(pk), H(m) + b"x", H(sig))


@pytest.mark.parametrize("k", KATS, ids=[k["era"] for k in KATS])
def test_reference_golden_blocks(oracle, k):
    """Every golden block of the reference: OCert, Sum6KES and VRF outcomes."""
    msg = H(k["hot_vk"]) + k["n"].to_bytes(8, "big") + k["c0"].to_bytes(8, "big")
    assert oracle.ed25519_verify(H(k["cold_vk"]), msg, H(k["ocert_sig"]))
    kes = oracle.kes_verify(H(k["hot_vk"]), 0, H(k["body_cbor"]), H(k["kes_sig"]))
    if k["kind"] == "tpraos":
        assert kes == 0
        e = k["expect"]
        assert oracle.vrf_verify(H(k["vrf_vk"]), H(k["eta_proof"]), H(e["eta_alpha"])) == H(k["eta_out"])
        assert oracle.vrf_verify(H(k["vrf_vk"]), H(k["leader_proof"]), H(e["leader_alpha"])) == H(k["leader_out"])
    else:
        assert kes == 2                               # InvalidKesSignatureOCERT (leaf), Examples.hs:173-192
        assert oracle.kes_verify(H(k["hot_vk"]), 0, H(k["kes_recon_body"]), H(k["kes_sig"])) == 0
        assert oracle.vrf_verify(H(k["vrf_vk"]), H(k["vrf_proof"]), H(k["expect"]["vrf_alpha"])) == H(k["vrf_out"])
        assert oracle.vrf_proof_to_hash(H(k["vrf_proof"])) == H(k["vrf_out"])


def test_golden_header_bytes_roundtrip():
    """The fixture's header/body spans decode back to the recorded fields."""
    import sys
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import cbor_min
    for k in KATS:
        hdr = H(k["header_cbor"])
        it = cbor_min.decode(hdr)
        body, sig = it.value
        assert body.raw(hdr) == H(k["body_cbor"])
        assert sig.value == H(k["kes_sig"])
        assert body.value[1].value == k["slot"]


def test_small_order_blacklist(oracle):
    # every blacklisted encoding is a point of order dividing 8 (or y >= p alias)
    encs = [0, 1, P - 1,
            2707385501144840649318225287225658788936804267575313519463743609750303402022,
            55188659117513257062467267217118295137698188065244968500265048394206261417927]
    for y in encs:
        b = y.to_bytes(32, "little")
        assert oracle.has_small_order(b)
        assert oracle.has_small_order(b[:31] + bytes([b[31] | 0x80]))
        if oracle.decode_ok(b):
            assert oracle.lib().orc_point_order_divides(b, 8) == 1
    for y in (P, P + 1):
        assert oracle.has_small_order(y.to_bytes(32, "little"))
    r = rng(2)
    for _ in range(50):
        assert not oracle.has_small_order(oracle.ed25519_pk(rbytes(r, 32)))


def test_ed25519_libsodium_rules(oracle):
    r = rng(3)
    sk = rbytes(r, 32)
    pk = oracle.ed25519_pk(sk)
    m = b"ocert"
    s = oracle.ed25519_sign(sk, m)
    assert oracle.ed25519_verify(pk, m, s)
    S = int.from_bytes(s[32:], "little")
    assert not oracle.ed25519_verify(pk, m, s[:32] + (S + L).to_bytes(32, "little"))   # S >= L
    assert not oracle.ed25519_verify(pk, m, bytes(32) + s[32:])                       # small-order R
    assert not oracle.ed25519_verify((P - 1).to_bytes(32, "little"), m, s)           # small-order A
    assert not oracle.ed25519_verify(pk[:31] + bytes([pk[31] ^ 0x80]), m, s)         # -A
    for k in range(0, 64, 7):
        assert not oracle.ed25519_verify(pk, m, corrupt(s, k))


def test_kes_roundtrip_and_rejections(oracle):
    r = rng(4)
    seed = rbytes(r, 32)
    vk = oracle.kes_vk(seed)
    for t in (0, 1, 31, 32, 62, 63):
        m = rbytes(r, 397)
        sig = oracle.kes_sign(seed, t, m)
        assert oracle.kes_verify(vk, t, m, sig) == 0
        assert oracle.kes_verify(vk, t, corrupt(m, t), sig) == 2
        assert oracle.kes_verify(vk, t, m, corrupt(sig, 64 + 64 * (t % 6) + 5)) == 1
        assert oracle.kes_verify(corrupt(vk, 3), t, m, sig) == 1
    # Word-valued period beyond 2^6: always the vk1 branch at every level
    m = b"x"
    sig = oracle.kes_sign(seed, 63, m)
    assert oracle.kes_verify(vk, 63 + 64, m, sig) == 0


def test_vrf_roundtrip(oracle):
    r = rng(5)
    for _ in range(6):
        sk = rbytes(r, 32)
        pk = oracle.vrf_pk(sk)
        a = rbytes(r, 32)
        proof = oracle.vrf_prove(sk, a)
        beta = oracle.vrf_verify(pk, proof, a)
        assert beta is not None and beta == oracle.vrf_proof_to_hash(proof)
        assert oracle.vrf_verify(pk, proof, corrupt(a, 1)) is None
        assert oracle.vrf_verify(pk, corrupt(proof, 40), a) is None


def _leader_exact_fraction(l, sigma, f):
    """Real-number criterion the Taylor test approximates: l/2^256 < 1-(1-f)^sigma."""
    import math
    return l / 2 ** 256 < 1 - math.exp(float(sigma) * math.log(1 - float(f)))


def test_leader_oracle_vs_python(oracle):
    from test_gpu_verify import _leader_python
    from praos_hip import fixed
    r = rng(6)
    c_raw = fixed.active_slot_log(Fraction(1, 20))
    n_lead = 0
    for i in range(600):
        s = Fraction(r.randrange(1, 1000), 1000)
        sf = fixed.from_rational(s)
        l = r.getrandbits(256) >> r.randrange(0, 12)
        a, _ = oracle.check_leader(l.to_bytes(32, "big"), sf, c_raw)
        assert a == _leader_python(l, sf, c_raw)
        n_lead += a
        # away from the threshold the decision equals the real-number criterion
        p = 1 - (0.95 ** float(s))
        if abs(l / 2 ** 256 - p) > 1e-9:
            assert a == _leader_exact_fraction(l, s, Fraction(1, 20))
    assert 0 < n_lead < 600


def test_leader_f_one_and_zero_stake(oracle):
    from praos_hip import fixed
    c_raw = fixed.active_slot_log(Fraction(1, 20))
    assert oracle.check_leader(bytes([0xff] * 32), 0, 0, True)[0]
    assert not oracle.check_leader(bytes(32), 0, c_raw)[0]          # sigma = 0 never leads
    assert oracle.check_leader(bytes(32), fixed.from_rational(1), c_raw)[0]


def test_active_slot_log_value():
    from praos_hip import fixed
    import math
    c = fixed.active_slot_log(Fraction(1, 20))
    assert abs(c / 10 ** 34 - math.log(0.95)) < 1e-15 and c < 0
    assert fixed.from_rational(Fraction(1, 3)) == 10 ** 34 // 3


def test_leader_boundary_fixture():
    """The bisected boundary vectors reproduce on the C oracle and on the pure-Python
    restatement of checkLeaderNatValue (tests/golden/make_leader_boundary.py)."""
    import json
    import os
    import oracle
    from golden.make_leader_boundary import leader_python
    cases = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "leader_boundary.json")))["cases"]
    assert len(cases) == 16
    for c in cases:
        bits, s_fp, c_raw = c["bits"], int(c["sigma_fp"]), int(c["c_raw"])
        check = oracle.check_leader if bits == 256 else oracle.check_leader512
        for v in c["vectors"]:
            l = int(v["leader_value"], 16)
            assert check(l.to_bytes(bits // 8, "big"), s_fp, c_raw) == (v["is_leader"], v["iterations"])
            assert leader_python(l, bits, s_fp, c_raw) == (v["is_leader"], v["iterations"])
        assert int(c["boundary"], 16) == int(c["vectors"][2]["leader_value"], 16)


def test_elligator_single_exponentiation():
    """k_vrf's vrf_from_uniform (praos_core.hpp) takes libsodium's two exponentiations
    (chi of g(x1), then the square root of the chosen ratio) as ONE: case 1 <=> the
    case-1 ratio a1 is a square, and the case-2 root comes from the same candidate times
    2^((p+3)/8) r.  Checked here against the two-exponentiation restatement on random and
    edge inputs; libsodium's u + 1 = 0 corner (D = 0) is unreachable: both r^2 it needs
    are non-residues."""
    import random
    p, A = 2 ** 255 - 19, 486662
    d = (-121665 * pow(121666, p - 2, p)) % p
    I = pow(2, (p - 1) // 4, p)
    k = (p - 5) // 8

    def root(u, v):                                  # libsodium-style sqrt_ratio candidate
        v3 = v * v * v % p
        return u * v3 * pow(u * v3 * v3 * v % p, k, p) % p

    def fix(x, u, v):
        return x if (v * x * x - u) % p == 0 else x * I % p

    def even(x):
        return (p - x) % p if x & 1 else x

    def two_exp(r):
        w = (1 + 2 * r * r) % p
        e = (-A * w * (A * A - A * A * w + w * w)) % p
        if pow(e, (p - 1) // 2, p) != p - 1:
            N, D = (-(A + w)) % p, (w - A) % p
        else:
            N, D = (A - A * w - w) % p, (A - A * w + w) % p
        if D == 0:
            N, D = 0, 1
        U, V = (N * N - D * D) % p, (d * N * N + D * D) % p
        return N, D, even(fix(root(U, V), U, V))

    def one_exp(r):
        w = (1 + 2 * r * r) % p
        N1, D1 = (-(A + w)) % p, (w - A) % p
        U, V = (N1 * N1 - D1 * D1) % p, (d * N1 * N1 + D1 * D1) % p
        s = root(U, V)
        if (V * s * s - U) % p == 0 or (V * s * s + U) % p == 0:
            return N1, D1, even(fix(s, U, V))
        U2 = U * (w - 1) % p
        t = s * pow(2, k + 1, p) % p * r % p
        return (A - A * w - w) % p, (A - A * w + w) % p, even(fix(t, U2, V))

    rng = random.Random(0xE11)
    for r in [0, 1, 2, p - 1, (p - 1) // 2] + [rng.getrandbits(255) % p for _ in range(400)]:
        assert one_exp(r) == two_exp(r), r
    assert pow(2, k + 1, p) == (I + 1) % p                      # the constant FE_2_P38
    for r2 in ((A - 1) * pow(2, p - 2, p) % p, (A * pow(A - 1, p - 2, p) - 1) * pow(2, p - 2, p) % p):
        assert pow(r2, (p - 1) // 2, p) == p - 1                 # D1 = 0 / D2 = 0 unreachable
