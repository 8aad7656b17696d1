"""Algorithmic work model of the HIP kernels (int32 VALU lane-ops per item).

The roofline in bench.py prices each kernel by the field operations its
schedule performs (counted here by construction, mirroring the code in
ouroboros-consensus_amd/csrc/*.hpp) times the int32 instruction count of
each operation in the radix-2^32 implementation (fe25519.hpp):

    M   field multiply   64 v_mad_u64_u32 + 64 carry adds + 26 reduction  = 154
    S   field square     28 cross MACs x 2 + doubling + 8 diagonals + red. = 130
    A   add / sub / neg  8 + 8 carry-propagating adds + fold                =  17
    SHA-512 compression  80 rounds on 64-bit words in VGPR pairs            = 5000
    BLAKE2b compression  12 rounds                                          = 2700
    X   exponentiation   ((p-5)/8, (p-1)/2): 254 S + 11 M (+ canon)
    INV inversion        binary GCD (fe_inv_gcd.hpp): ~13.5 outer iterations x ~1,300 VALU
                         (30 steps x ~24 + the matrix applied to a, b, u, v) + the 2^(-30k) product

Everything else (digit extraction, table selection, sign handling, loads,
loop control) is overhead and not counted: `frac` therefore reports how much
of the integer-VALU issue rate goes into the counted arithmetic.

Run `python tools/workmodel.py` to print the per-item figures.
"""
M, S, A = 154, 130, 17
SHA, B2B = 5000, 2700
CANON = 30
X = 254 * S + 11 * M + CANON            # one exponentiation chain
INV = 27 * 1300 // 2 + M + CANON          # one inversion (binary GCD; Fermat's z^(p-2) was X)

# group operations (ge25519.hpp)
DBL = 4 * S + 6 * A                     # ge_p2_dbl -> p1p1
ADD = 4 * M + 6 * A + 2 * A             # ge_add (incl. Y+X, Y-X of p)
MADD = 3 * M + 6 * A + 2 * A            # ge_madd
TO_P2, TO_P3 = 3 * M, 4 * M
CNEG = A                                # negation of the selected entry
TABLE8 = 8 * (M + 2 * A) + (DBL + TO_P3) + 6 * (ADD + TO_P3)   # {1..8}P cached
DECODE = X + 2 * S + 10 * M + 3 * A + 3 * CANON                # ge_frombytes (sqrt ratio)
ENCODE = INV + 2 * M + CANON                                   # ge_tobytes (one inversion)
SC_REDUCE = 600


def straus(nwin, np_, nq, nfixed_adds):
    """Horner chain: (nwin-1) x 4 doublings, per-lane adds, fixed-base madds."""
    w = (nwin - 1) * (4 * DBL + 3 * TO_P2)          # dbl4 (last one left as p1p1)
    w += (np_ + nq) * (TO_P3 + ADD + CNEG)
    w += nfixed_adds * (TO_P3 + MADD + CNEG)
    w += (nwin - 1) * TO_P2
    return w


def ed25519_verify(sha_blocks):
    return (sha_blocks * SHA + SC_REDUCE + DECODE + TABLE8 + straus(64, 64, 0, 32)
            + TO_P2 + ENCODE + 200)


def vrf_verify():
    w = 2 * DECODE                                   # Y, Gamma
    w += SHA                                         # hash_to_curve digest
    w += 10 * M + 6 * S + 12 * A                     # Elligator2 numerators N1/D1, N2/D2, ratio
    w += DECODE                                      # ONE sqrt-ratio exponentiation (chi merged)
    w += 6 * M + 2 * S + 2 * A                       # case-2 candidate 2^((p+3)/8) r s and its check
    w += 3 * (DBL + TO_P3)                           # cofactor 8
    w += TABLE8 + straus(33, 33, 0, 32) + TO_P2      # U = [s]B - [c]Y (B, 2^128 B)
    w += 2 * TABLE8 + straus(64, 64, 33, 0) + TO_P2  # V = [s]H - [c]Gamma
    w += 3 * (DBL + TO_P3)                           # 8 Gamma
    w += INV + 10 * M + 4 * (2 * M + CANON)          # batched inversion + 4 encodings
    w += 3 * SHA + SC_REDUCE                         # c' (2 blocks), beta (1 block)
    return w


def straus_comb(npc, p_top):
    """4-window chain over cached key tables (16-bit chunks) + 16 radix-2^16 comb madds (scalarmult.hpp)."""
    w = 3 * (4 * DBL + 3 * TO_P2) + 3 * TO_P2
    w += (4 * npc + (1 if p_top else 0)) * (TO_P3 + ADD + CNEG)
    w += 16 * (TO_P3 + MADD + CNEG)                  # 16-bit fixed-base digits from the comb, after the chain
    return w


def key_precompute(nchunks):
    """k_key_precompute: decode, nchunks tables, 16 doublings between chunks."""
    return DECODE + nchunks * TABLE8 + (nchunks - 1) * 16 * (DBL + TO_P2)


W_OCERT = ed25519_verify(2)
W_KES = ed25519_verify(4) + 6 * B2B
W_VRF = vrf_verify() + 6 * B2B + 1000                # mkInputVRF, issuer/key hashes, L/N, search
W_LEADER = 3000
# key-cache path (k_keys.hip): per header on a cached key, and per cached key
W_OCERT_CK = W_OCERT - DECODE - TABLE8 - straus(64, 64, 0, 32) + straus_comb(16, False)
W_VRF_CK = W_VRF - DECODE - TABLE8 - straus(33, 33, 0, 32) + straus_comb(8, True)
W_KES_CK = W_KES - DECODE - TABLE8 - straus(64, 64, 0, 32) + straus_comb(16, False)
# two-stage VRF (praos_core.hpp vrf_v_core / vrf_fin_core, k_vrf.hip): what each kernel computes
ELLIGATOR = SHA + (10 * M + 6 * S + 12 * A) + DECODE + (6 * M + 2 * S + 2 * A) + 3 * (DBL + TO_P3)
W_VRF_V = (B2B                                        # alpha = mkInputVRF(slot, eta0)
           + CANON + ELLIGATOR                        # canonical Y (no decode), H = hash_to_curve
           + DECODE + 3 * (DBL + TO_P3)               # Gamma, 8 Gamma
           + 2 * TABLE8 + SC_REDUCE + straus(64, 64, 33, 0) + TO_P2)   # V = [s]H - [c]Gamma
_FIN = SC_REDUCE + TO_P2 + INV + 10 * M + 4 * (2 * M + CANON) + 3 * SHA + 5 * B2B + 1000
W_VRF_F_CK = _FIN + straus_comb(8, True)             # U from the cached key + comb; inversion, c', beta, L/N
W_VRF_F = _FIN + DECODE + TABLE8 + straus(33, 33, 0, 32)
# TPraos header (TPraos.hs:361-387, k_vrf_tp): two certificates (eta, L) per header, each a full
# uncached draft-03 verify with its mkSeed input (2 Blake2b), issuer + VRF-key hashes, the
# eta nonce hash; the leader test against 2^512
W_VRF_TP = 2 * (vrf_verify() + 2 * B2B) + 3 * B2B + 1000
W_LEADER_TP = 6000
W_TP_HEADER = W_OCERT + W_KES + W_VRF_TP + W_LEADER_TP
W_KEY_COLD = key_precompute(16)
W_KEY_KES = key_precompute(16)                       # leaf keys: same tables as cold keys
W_KEY_VRF = key_precompute(9) + CANON

if __name__ == "__main__":
    for k, v in (("ocert", W_OCERT), ("kes", W_KES), ("vrf", W_VRF), ("leader", W_LEADER),
                 ("ocert_ck", W_OCERT_CK), ("vrf_ck", W_VRF_CK), ("kes_ck", W_KES_CK), ("key_cold", W_KEY_COLD), ("key_vrf", W_KEY_VRF),
                 ("vrf_v", W_VRF_V), ("vrf_f_ck", W_VRF_F_CK), ("vrf_f", W_VRF_F), ("vrf_tp", W_VRF_TP),
                 ("tp_hdr", W_TP_HEADER)):
        print(f"W_{k:7s} {v:>10,d} int32 ops / item")
    print(f"W_header  {W_OCERT + W_KES + W_VRF + W_LEADER:>10,d}")
