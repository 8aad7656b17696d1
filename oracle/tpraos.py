"""Pure-Python restatement of the TPraos (Shelley..Alonzo) rules around the per-header
crypto: the decentralisation overlay schedule, the OVERLAY / OCERT predicate failures and
the chain-dependent state fold (TICKN + PRTCL = UPDN + OVERLAY + OCERT).

TEST INFRASTRUCTURE ONLY (see oracle.h): the checker of praos_set_overlay /
praos_overlay_classify / praos_verify_tpraos_headers (overlay bits) and
praos_tpraos_update_chain_dep_state; never part of the product.

The rules live in cardano-protocol-tpraos (>= 1.0.1 && < 1.1, ouroboros-consensus-
cardano.cabal:132; not vendored in the reference).  The reference's own call sites:
TPraos.checkIsLeader (ouroboros-consensus-protocol/.../Protocol/TPraos.hs:304-337, the
same lookupInOverlaySchedule firstSlot gkeys d asc slot the validator runs),
tickChainDepState / updateChainDepState (:361-387).  Restated from the published package:
  Rules/Overlay.hs  isOverlaySlot, classifyOverlaySlot, lookupInOverlaySchedule,
                    overlayTransition, praosVrfChecks, pbftVrfChecks, vrfChecks
  Rules/OCert.hs    ocertTransition, currentIssueNo
  Rules/Prtcl.hs    prtclTransition (UPDN then OVERLAY), Rules/Updn.hs, Rules/Tickn.hs
  API.hs            tickChainDepState, updateChainDepState (lab := prevHashToNonce)
Parity status: these rules are parity unpinned (no reference fixture exercises d > 0);
the restatement is exact rational arithmetic on the Haskell definitions.
"""
import hashlib
from fractions import Fraction
from math import ceil, floor

import chainstate as cs

# praos_hip.h bits (GPU) and TPraos predicate failures (PRAOS_TPF_*)
BIT_KES_BEFORE_START, BIT_KES_AFTER_END, BIT_OCERT_SIG, BIT_KES_MERKLE, BIT_KES_LEAF = 0x1, 0x2, 0x4, 0x8, 0x10
BIT_VRF_KEY_UNKNOWN, BIT_VRF_KEY_WRONG, BIT_TP_NONCE, BIT_TP_LEADER, BIT_LEADER = 0x100, 0x200, 0x400, 0x800, 0x1000
BIT_TP_OVERLAY, BIT_TP_NOT_ACTIVE, BIT_INPUT = 0x2000, 0x4000, 0x8000
BIT_TP_GEN_COLD, BIT_TP_GEN_VRF = 0x100, 0x200
OCERT_BITS = BIT_KES_BEFORE_START | BIT_KES_AFTER_END | BIT_OCERT_SIG | BIT_KES_MERKLE | BIT_KES_LEAF
(TPF_KES_BEFORE_START, TPF_KES_AFTER_END, TPF_OCERT_SIG, TPF_KES_SIG, TPF_COUNTER_MISSING, TPF_COUNTER_TOO_SMALL,
 TPF_COUNTER_OVER_INC) = 0x1, 0x2, 0x4, 0x8, 0x10, 0x20, 0x40
(TPF_VRF_KEY_UNKNOWN, TPF_VRF_KEY_WRONG, TPF_BAD_NONCE, TPF_BAD_LEADER, TPF_LEADER_TOO_BIG, TPF_NOT_ACTIVE,
 TPF_GEN_COLD, TPF_GEN_VRF) = 0x100, 0x200, 0x400, 0x800, 0x1000, 0x2000, 0x4000, 0x8000
V_OK, V_INPUT, V_TPRAOS = 0, 12, 19


def classify(slot, d: Fraction, f: Fraction, base_slot, length, ngen):
    """lookupInOverlaySchedule firstSlotNo gkeys d asc slot: -1 Nothing (not an overlay
    slot), -2 Just NonActiveSlot, k >= 0 Just (ActiveSlot (Set.elemAt k gkeys))."""
    if d == 0 or slot < base_slot:
        return -1
    first = base_slot + (slot - base_slot) // length * length       # epochInfoFirst (epochInfoEpoch slot)
    s = slot - first

    def step(x):                                                    # ceiling (x * d)
        return ceil(Fraction(x) * d)
    if not step(s) < step(s + 1):                                   # isOverlaySlot
        return -1
    position = step(s)
    asc_inv = floor(1 / f)
    if position % asc_inv != 0:                                     # isActive
        return -2
    return (position // asc_inv) % ngen                             # always < length gkeys


def overlay_bits(base_bits, cls, cold_vk, vrf_vk, gen_sorted):
    """GPU bit layout for a TPraos header given the d = 0 bits of the same header
    (oracle.tpraos_header: OCERT + praosVrfChecks pieces) and its overlay class;
    gen_sorted = [(genesis28, delegate28, vrf32)] in ascending genesis-hash order."""
    if cls == -1:
        return base_bits
    if cls == -2:                                                    # no VRF check at all
        return (base_bits & OCERT_BITS) | BIT_TP_NOT_ACTIVE
    _, dlg, vrfh = gen_sorted[cls]
    b = (base_bits & (OCERT_BITS | BIT_TP_NONCE | BIT_TP_LEADER)) | BIT_TP_OVERLAY
    if hashlib.blake2b(bytes(cold_vk), digest_size=28).digest() != bytes(dlg):
        b |= BIT_TP_GEN_COLD
    if hashlib.blake2b(bytes(vrf_vk), digest_size=32).digest() != bytes(vrfh):
        b |= BIT_TP_GEN_VRF
    return b


def failures(b, m, n):
    """PRTCL's predicate failures (ValidateAll): OVERLAY's Either-chains + every OCERT
    predicate.  m = currentIssueNo (None = Nothing)."""
    f = 0
    if b & BIT_TP_NOT_ACTIVE:
        f |= TPF_NOT_ACTIVE
    elif b & BIT_TP_OVERLAY:
        if b & BIT_TP_GEN_COLD:                                      # ?! (collected)
            f |= TPF_GEN_COLD
        if b & BIT_TP_GEN_VRF:                                       # pbftVrfChecks: first Left
            f |= TPF_GEN_VRF
        elif b & BIT_TP_NONCE:
            f |= TPF_BAD_NONCE
        elif b & BIT_TP_LEADER:
            f |= TPF_BAD_LEADER
    else:                                                            # praosVrfChecks: first Left
        for bit, fail in ((BIT_VRF_KEY_UNKNOWN, TPF_VRF_KEY_UNKNOWN), (BIT_VRF_KEY_WRONG, TPF_VRF_KEY_WRONG),
                          (BIT_TP_NONCE, TPF_BAD_NONCE), (BIT_TP_LEADER, TPF_BAD_LEADER),
                          (BIT_LEADER, TPF_LEADER_TOO_BIG)):
            if b & bit:
                f |= fail
                break
    if b & BIT_KES_BEFORE_START:
        f |= TPF_KES_BEFORE_START
    if b & BIT_KES_AFTER_END:
        f |= TPF_KES_AFTER_END
    if b & BIT_OCERT_SIG:
        f |= TPF_OCERT_SIG
    if b & (BIT_KES_MERKLE | BIT_KES_LEAF):
        f |= TPF_KES_SIG
    if m is None:
        f |= TPF_COUNTER_MISSING
    else:
        if not m <= n:
            f |= TPF_COUNTER_TOO_SMALL
        if not n <= m + 1:
            f |= TPF_COUNTER_OVER_INC
    return f


def fold(st, hk, slots, bits, ocert_n, nonces, prev_hash, known, eta0, base_slot, base_no, length, window,
         extra_entropy=None):
    """TPraos tickChainDepState + updateChainDepState over a batch.  st as in
    chainstate.fold (evolving/candidate = eta_v/eta_c, epoch_nonce/leb = TicknState
    eta_0/eta_h, lab = csLabNonce); known = pool hashes + genesis-delegate hashes
    (currentIssueNo's Just 0).  Returns (verdicts, failures, chain_stop, processed)."""
    def epoch(s):
        return base_no + (s - base_slot) // length
    w = cs._copy(st)
    frozen, stop = None, None
    out, fl = [], []
    i = 0
    for i in range(len(slots) + 1):
        if i == len(slots):
            break
        s = int(slots[i])
        e_new = epoch(s)
        e_old = 0 if w["last_slot"] is None else epoch(w["last_slot"])
        t_epoch, t_leb = w["epoch_nonce"], w["leb"]
        if e_new > e_old:                                            # TICKN
            t_epoch = cs.combine(cs.combine(w["candidate"], w["leb"]), extra_entropy)
            t_leb = w["lab"]
        if t_epoch != eta0:
            break
        b = int(bits[i])
        if b & BIT_INPUT:
            f, v = 0, V_INPUT
        else:
            m = w["counters"].get(hk[i], 0 if hk[i] in known else None)
            f = failures(b, m, int(ocert_n[i]))
            v = V_TPRAOS if f else V_OK
        out.append(v)
        fl.append(f)
        if v != V_OK:
            if stop is None:
                stop = i
                frozen = cs._copy(w)
            continue
        w["epoch_nonce"], w["leb"] = t_epoch, t_leb
        w["last_slot"] = s
        w["lab"] = prev_hash[i]                                      # prevHashToNonce
        w["evolving"] = cs.combine(w["evolving"], bytes(nonces[i]))  # UPDN
        if s + window < base_slot + (e_new - base_no + 1) * length:
            w["candidate"] = w["evolving"]
        w["counters"][hk[i]] = int(ocert_n[i])                       # OCERT: Map.insert hk n
    processed = i
    res = frozen if frozen is not None else w
    st.clear()
    st.update(res)
    return out, fl, min(len(slots) if stop is None else stop, processed), processed
