"""ctypes front-end of the CPU oracle (oracle/*.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, always as the checker.  The product path
(ouroboros-consensus_amd, libpraos_hip.so) never imports this module.
"""
import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        c = ctypes
        L.orc_sha512.argtypes = [c.c_char_p, c.c_char_p, c.c_size_t]
        L.orc_blake2b.argtypes = [c.c_char_p, c.c_size_t, c.c_char_p, c.c_size_t]
        L.orc_ed25519_verify.argtypes = [c.c_char_p, c.c_char_p, c.c_size_t, c.c_char_p]
        L.orc_ed25519_pk_from_seed.argtypes = [c.c_char_p, c.c_char_p]
        L.orc_ed25519_sign.argtypes = [c.c_char_p, c.c_char_p, c.c_size_t, c.c_char_p]
        L.orc_vrf_verify.argtypes = [c.c_char_p, c.c_char_p, c.c_char_p, c.c_char_p, c.c_size_t]
        L.orc_vrf_proof_to_hash.argtypes = [c.c_char_p, c.c_char_p]
        L.orc_vrf_pk_from_seed.argtypes = [c.c_char_p, c.c_char_p]
        L.orc_vrf_prove.argtypes = [c.c_char_p, c.c_char_p, c.c_char_p, c.c_size_t]
        L.orc_kes_verify.argtypes = [c.c_char_p, c.c_uint32, c.c_char_p, c.c_size_t, c.c_char_p]
        L.orc_kes_vk_from_seed.argtypes = [c.c_char_p, c.c_char_p]
        L.orc_kes_sign.argtypes = [c.c_char_p, c.c_char_p, c.c_uint32, c.c_char_p, c.c_size_t]
        L.orc_check_leader.argtypes = [c.c_char_p, c.c_char_p, c.c_char_p, c.c_int, c.POINTER(c.c_int)]
        L.orc_has_small_order.argtypes = [c.c_char_p]
        L.orc_ge_decode_ok.argtypes = [c.c_char_p]
        L.orc_point_order_divides.argtypes = [c.c_char_p, c.c_int]
        L.orc_praos_header.argtypes = [c.c_void_p, c.c_void_p, c.c_void_p]
        L.orc_scalarmult_base.argtypes = [c.c_char_p, c.c_char_p]
        L.orc_tpraos_header.argtypes = [c.c_void_p, c.c_void_p, c.c_void_p]
        L.orc_tpraos_seed.argtypes = [c.c_char_p, c.c_uint64, c.c_char_p, c.c_int, c.c_uint64]
        L.orc_check_leader512.argtypes = [c.c_char_p, c.c_char_p, c.c_char_p, c.c_int, c.POINTER(c.c_int)]
        L.orc_ge_reencode.argtypes = [c.c_char_p, c.c_char_p]
        L.orc_vrf_hash_to_curve.argtypes = [c.c_char_p, c.c_char_p, c.c_char_p, c.c_size_t]
        _lib = L
    return _lib


def sha512(m: bytes) -> bytes:
    o = ctypes.create_string_buffer(64)
    lib().orc_sha512(o, m, len(m))
    return o.raw


def blake2b(m: bytes, n: int = 32) -> bytes:
    o = ctypes.create_string_buffer(n)
    lib().orc_blake2b(o, n, m, len(m))
    return o.raw


def ed25519_verify(pk: bytes, msg: bytes, sig: bytes) -> bool:
    return lib().orc_ed25519_verify(sig, msg, len(msg), pk) == 0


def ed25519_pk(seed: bytes) -> bytes:
    o = ctypes.create_string_buffer(32)
    lib().orc_ed25519_pk_from_seed(o, seed)
    return o.raw


def ed25519_sign(seed: bytes, msg: bytes) -> bytes:
    o = ctypes.create_string_buffer(64)
    lib().orc_ed25519_sign(o, msg, len(msg), seed)
    return o.raw


def vrf_verify(pk: bytes, proof: bytes, alpha: bytes):
    """Returns beta (64 B) if the draft-03 proof verifies, else None."""
    o = ctypes.create_string_buffer(64)
    return o.raw if lib().orc_vrf_verify(o, pk, proof, alpha, len(alpha)) == 0 else None


def vrf_proof_to_hash(proof: bytes):
    o = ctypes.create_string_buffer(64)
    return o.raw if lib().orc_vrf_proof_to_hash(o, proof) == 0 else None


def vrf_pk(seed: bytes) -> bytes:
    o = ctypes.create_string_buffer(32)
    lib().orc_vrf_pk_from_seed(o, seed)
    return o.raw


def vrf_prove(seed: bytes, alpha: bytes) -> bytes:
    o = ctypes.create_string_buffer(80)
    assert lib().orc_vrf_prove(o, seed, alpha, len(alpha)) == 0
    return o.raw


KES_SIG_BYTES = 448


def kes_verify(vk: bytes, t: int, msg: bytes, sig: bytes) -> int:
    """0 ok, 1 Merkle "Reject", 2 leaf Ed25519 failure."""
    return lib().orc_kes_verify(vk, t, msg, len(msg), sig)


def kes_vk(seed: bytes) -> bytes:
    o = ctypes.create_string_buffer(32)
    lib().orc_kes_vk_from_seed(o, seed)
    return o.raw


def kes_sign(seed: bytes, t: int, msg: bytes) -> bytes:
    o = ctypes.create_string_buffer(KES_SIG_BYTES)
    assert lib().orc_kes_sign(o, seed, t, msg, len(msg)) == 0
    return o.raw


def check_leader(leader_be: bytes, sigma_fp: int, c_raw: int, f_is_one: bool = False):
    """Returns (is_leader, taylor_iterations)."""
    it = ctypes.c_int(0)
    r = lib().orc_check_leader(leader_be, sigma_fp.to_bytes(16, "little"),
                               (c_raw & ((1 << 128) - 1)).to_bytes(16, "little"),
                               int(bool(f_is_one)), ctypes.byref(it))
    return bool(r), it.value


def has_small_order(s: bytes) -> bool:
    return bool(lib().orc_has_small_order(s))


def scalarmult_base(s: bytes) -> bytes:
    o = ctypes.create_string_buffer(32)
    lib().orc_scalarmult_base(o, s)
    return o.raw


def reencode(s: bytes):
    """(on_curve, canonical re-encoding) with libsodium ge25519_frombytes rules."""
    o = ctypes.create_string_buffer(32)
    ok = lib().orc_ge_reencode(o, s)
    return bool(ok), o.raw


def vrf_hash_to_curve(pk: bytes, alpha: bytes):
    o = ctypes.create_string_buffer(32)
    ok = lib().orc_vrf_hash_to_curve(o, pk, alpha, len(alpha))
    return o.raw if ok else None


def decode_ok(s: bytes) -> bool:
    return bool(lib().orc_ge_decode_ok(s))


# ---- per-header restatement (struct layouts mirror oracle.h) ----
class Pool(ctypes.Structure):
    _fields_ = [("hash28", ctypes.c_uint8 * 28), ("vrf_hash32", ctypes.c_uint8 * 32),
                ("sigma_fp", ctypes.c_uint8 * 16)]


class Header(ctypes.Structure):
    _fields_ = [("slot", ctypes.c_uint64), ("cold_vk", ctypes.c_uint8 * 32), ("vrf_vk", ctypes.c_uint8 * 32),
                ("vrf_out", ctypes.c_uint8 * 64), ("vrf_proof", ctypes.c_uint8 * 80),
                ("hot_vk", ctypes.c_uint8 * 32), ("ocert_n", ctypes.c_uint64), ("ocert_c0", ctypes.c_uint64),
                ("ocert_sig", ctypes.c_uint8 * 64), ("kes_sig", ctypes.c_uint8 * 448),
                ("body", ctypes.c_void_p), ("body_len", ctypes.c_size_t)]


class Epoch(ctypes.Structure):
    _fields_ = [("eta0", ctypes.c_uint8 * 32), ("eta0_neutral", ctypes.c_int),
                ("slots_per_kes_period", ctypes.c_uint64), ("max_kes_evo", ctypes.c_uint64),
                ("f_is_one", ctypes.c_int), ("c_raw", ctypes.c_uint8 * 16),
                ("pools", ctypes.c_void_p), ("npools", ctypes.c_uint32)]


class Result(ctypes.Structure):
    _fields_ = [("bits", ctypes.c_uint32), ("pool_idx", ctypes.c_int32), ("beta", ctypes.c_uint8 * 64),
                ("leader", ctypes.c_uint8 * 32), ("nonce", ctypes.c_uint8 * 32),
                ("issuer_hash", ctypes.c_uint8 * 28)]


def _fill(arr, b: bytes):
    ctypes.memmove(arr, b, len(b))


def make_epoch(eta0, slots_per_kes_period, max_kes_evo, c_raw, pools, f_is_one=False):
    """pools: list of (hash28, vrf_hash32, sigma_fp int), any order (sorted here)."""
    pools = sorted(pools, key=lambda p: p[0])
    parr = (Pool * max(1, len(pools)))()
    for i, (h, v, s) in enumerate(pools):
        _fill(parr[i].hash28, h)
        _fill(parr[i].vrf_hash32, v)
        _fill(parr[i].sigma_fp, s.to_bytes(16, "little"))
    ep = Epoch()
    if eta0 is None:
        ep.eta0_neutral = 1
    else:
        _fill(ep.eta0, eta0)
    ep.slots_per_kes_period = slots_per_kes_period
    ep.max_kes_evo = max_kes_evo
    ep.f_is_one = int(bool(f_is_one))
    _fill(ep.c_raw, (c_raw & ((1 << 128) - 1)).to_bytes(16, "little"))
    ep.pools = ctypes.cast(parr, ctypes.c_void_p)
    ep.npools = len(pools)
    ep._keep = (parr, pools)
    return ep


def praos_header(ep, h: dict) -> dict:
    """h: dict with slot, cold_vk, vrf_vk, vrf_out, vrf_proof, hot_vk, n, c0,
    ocert_sig, kes_sig, body.  Returns bits, pool_idx, beta, leader, nonce."""
    H = Header()
    H.slot = h["slot"]
    for k in ("cold_vk", "vrf_vk", "vrf_out", "vrf_proof", "hot_vk", "ocert_sig", "kes_sig"):
        _fill(getattr(H, k), h[k])
    H.ocert_n = h["n"]
    H.ocert_c0 = h["c0"]
    body = ctypes.create_string_buffer(h["body"], len(h["body"]))
    H.body = ctypes.cast(body, ctypes.c_void_p)
    H.body_len = len(h["body"])
    R = Result()
    lib().orc_praos_header(ctypes.byref(ep), ctypes.byref(H), ctypes.byref(R))
    return {"bits": R.bits, "pool_idx": R.pool_idx, "beta": bytes(R.beta),
            "leader": bytes(R.leader), "nonce": bytes(R.nonce), "issuer_hash": bytes(R.issuer_hash)}


class TPHeader(ctypes.Structure):
    _fields_ = [("h", Header), ("leader_out", ctypes.c_uint8 * 64), ("leader_proof", ctypes.c_uint8 * 80)]


class TPResult(ctypes.Structure):
    _fields_ = [("bits", ctypes.c_uint32), ("pool_idx", ctypes.c_int32), ("beta_eta", ctypes.c_uint8 * 64),
                ("beta_leader", ctypes.c_uint8 * 64), ("nonce", ctypes.c_uint8 * 32)]


def tpraos_seed(slot: int, eta0, k: int) -> bytes:
    o = ctypes.create_string_buffer(32)
    lib().orc_tpraos_seed(o, slot, eta0 if eta0 is not None else bytes(32), int(eta0 is None), k)
    return o.raw


def check_leader512(leader_be: bytes, sigma_fp: int, c_raw: int, f_is_one: bool = False):
    it = ctypes.c_int(0)
    r = lib().orc_check_leader512(leader_be, sigma_fp.to_bytes(16, "little"),
                                  (c_raw & ((1 << 128) - 1)).to_bytes(16, "little"), int(bool(f_is_one)),
                                  ctypes.byref(it))
    return bool(r), it.value


def tpraos_header(ep, h: dict) -> dict:
    """h: praos_header fields (vrf_out/vrf_proof = eta cert) + leader_out, leader_proof."""
    T = TPHeader()
    H = T.h
    H.slot = h["slot"]
    for k in ("cold_vk", "vrf_vk", "vrf_out", "vrf_proof", "hot_vk", "ocert_sig", "kes_sig"):
        _fill(getattr(H, k), h[k])
    H.ocert_n = h["n"]
    H.ocert_c0 = h["c0"]
    body = ctypes.create_string_buffer(h["body"], len(h["body"]))
    H.body = ctypes.cast(body, ctypes.c_void_p)
    H.body_len = len(h["body"])
    _fill(T.leader_out, h["leader_out"])
    _fill(T.leader_proof, h["leader_proof"])
    R = TPResult()
    lib().orc_tpraos_header(ctypes.byref(ep), ctypes.byref(T), ctypes.byref(R))
    return {"bits": R.bits, "pool_idx": R.pool_idx, "beta_eta": bytes(R.beta_eta),
            "beta_leader": bytes(R.beta_leader), "nonce": bytes(R.nonce)}


# ---- generator restatement (db-synthesizer first-leader-wins, Forging.hs:139-148) ----
def mk_input_vrf(slot: int, eta0) -> bytes:
    """mkInputVRF (Praos/VRF.hs:55-69): Blake2b-256(BE64 slot || eta0), eta0 omitted when Neutral."""
    return blake2b(slot.to_bytes(8, "big") + (bytes(eta0) if eta0 is not None else b""))


def synth_seed(master: bytes, tag: int, i: int) -> bytes:
    """Key seeds of the GPU generator's pool i: Blake2b-256(tag || master || BE32 i);
    tag 1 = cold key, 2 = VRF key, 3 = KES key (k_synth.hip derive_seed)."""
    return blake2b(bytes([tag]) + bytes(master) + i.to_bytes(4, "big"))


def is_leader_at(vrf_seed: bytes, slot: int, eta0, sigma_fp: int, c_raw: int, f_is_one=False, tpraos=False):
    """checkIsLeader (Praos.hs:375-397) of one pool: evalCertified on mkInputVRF, then
    meetsLeaderThreshold (:505-526) -- or the TPraos leader cert (mkSeed seedL, 2^512)."""
    if tpraos:
        beta = vrf_proof_to_hash(vrf_prove(vrf_seed, tpraos_seed(slot, eta0, 1)))
        return check_leader512(beta, sigma_fp, c_raw, f_is_one)[0]
    beta = vrf_proof_to_hash(vrf_prove(vrf_seed, mk_input_vrf(slot, eta0)))
    return check_leader(blake2b(b"L" + beta), sigma_fp, c_raw, f_is_one)[0]


def leader_schedule(master: bytes, sigmas, c_raw: int, eta0, slots, f_is_one=False, tpraos=False):
    """Forger of each slot: the first pool (index order = forger order) that leads, else -1."""
    seeds = [synth_seed(master, 2, p) for p in range(len(sigmas))]
    out = []
    for s in slots:
        lead = -1
        for p, sg in enumerate(sigmas):
            if is_leader_at(seeds[p], int(s), eta0, sg, c_raw, f_is_one, tpraos):
                lead = p
                break
        out.append(lead)
    return out
