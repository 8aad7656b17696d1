"""Pure-Python restatement of the sequential part of Praos header validation.

TEST INFRASTRUCTURE ONLY (see oracle.h): used by tests/ as the checker of
praos_apply_batch / praos_update_chain_dep_state; never by the product.

Follows ouroboros-consensus-protocol/.../Protocol/Praos.hs:
  * first-error order of updateChainDepState (:441-459) over the per-check bits
    (validateKESSignature :558-606, validateVRFSignature :528-556);
  * OCert counter rule (:584-606; PoolDistr membership stands in for a missing counter);
  * tickChainDepState (:407-431) with isNewEpoch (Ledger/Util.hs:20-40);
  * reupdateChainDepState (:468-502): lab, evolving (⭒), candidate (stability window),
    counters.
Nonces are None (NeutralNonce) or 32 bytes; a ⭒ b = Blake2b-256(a || b).
"""
import hashlib

BIT_KES_BEFORE_START, BIT_KES_AFTER_END, BIT_OCERT_SIG = 0x1, 0x2, 0x4
BIT_KES_MERKLE, BIT_KES_LEAF = 0x8, 0x10
BIT_VRF_KEY_UNKNOWN, BIT_VRF_KEY_WRONG, BIT_VRF_PROOF, BIT_VRF_OUTPUT, BIT_LEADER = 0x100, 0x200, 0x400, 0x800, 0x1000
BIT_INPUT = 0x8000
(V_OK, V_KES_BEFORE_START, V_KES_AFTER_END, V_OCERT_SIG, V_KES_SIG, V_COUNTER_MISSING, V_COUNTER_TOO_SMALL,
 V_COUNTER_OVER_INC, V_VRF_KEY_UNKNOWN, V_VRF_KEY_WRONG, V_VRF_BAD_PROOF, V_LEADER_TOO_BIG, V_INPUT,
 V_ENV_BLOCK_NO, V_ENV_SLOT_NO, V_ENV_PREV_HASH, V_ENV_OBSOLETE_NODE, V_ENV_HEADER_SIZE,
 V_ENV_BLOCK_SIZE) = range(19)


def verdict(b, m, n):
    """m = counter (None when the issuer has neither a counter nor a PoolDistr entry)."""
    if b & BIT_INPUT:
        return V_INPUT
    if b & BIT_KES_BEFORE_START:
        return V_KES_BEFORE_START
    if b & BIT_KES_AFTER_END:
        return V_KES_AFTER_END
    if b & BIT_OCERT_SIG:
        return V_OCERT_SIG
    if b & (BIT_KES_MERKLE | BIT_KES_LEAF):
        return V_KES_SIG
    if m is None:
        return V_COUNTER_MISSING
    if not m <= n:
        return V_COUNTER_TOO_SMALL
    if not n <= m + 1:
        return V_COUNTER_OVER_INC
    if b & BIT_VRF_KEY_UNKNOWN:
        return V_VRF_KEY_UNKNOWN
    if b & BIT_VRF_KEY_WRONG:
        return V_VRF_KEY_WRONG
    if b & (BIT_VRF_PROOF | BIT_VRF_OUTPUT):
        return V_VRF_BAD_PROOF
    if b & BIT_LEADER:
        return V_LEADER_TOO_BIG
    return V_OK


def envelope_verdict(env, tip, i, slot, prev_hash):
    """validateEnvelope (HeaderValidation.hs:297-344) + Praos envelopeChecks
    (Shelley/Protocol/Praos.hs:66-80); tip = None (Origin) or (slot, block_no, hash)."""
    if env["block_no"][i] != (0 if tip is None else tip[1] + 1):
        return V_ENV_BLOCK_NO
    if not slot >= (0 if tip is None else tip[0] + 1):
        return V_ENV_SLOT_NO
    if not ((prev_hash is None) if tip is None else (prev_hash is not None and bytes(prev_hash) == tip[2])):
        return V_ENV_PREV_HASH
    if not env["lv_prot_major"] <= env["max_major_pv"]:
        return V_ENV_OBSOLETE_NODE
    if not env["header_size"][i] <= env["max_header_size"]:
        return V_ENV_HEADER_SIZE
    if not env["body_size"][i] <= env["max_body_size"]:
        return V_ENV_BLOCK_SIZE
    return V_OK


def combine(a, b):
    """Nonce semigroup (⭒)."""
    if a is None:
        return b
    if b is None:
        return a
    return hashlib.blake2b(a + b, digest_size=32).digest()


def apply_batch(hk, bits, ocert_n, known, counters):
    """Verdicts with counters only (praos_apply_batch)."""
    cm = dict(counters)
    out, stop = [], None
    for i in range(len(bits)):
        m = cm.get(hk[i], 0 if hk[i] in known else None)
        v = verdict(int(bits[i]), m, int(ocert_n[i]))
        out.append(v)
        if v == V_OK:
            cm[hk[i]] = int(ocert_n[i])
        elif stop is None:
            stop = i
    return out, (len(bits) if stop is None else stop), cm


def _copy(st):
    return {k: (dict(v) if isinstance(v, dict) else v) for k, v in st.items()}


def fold(st, hk, slots, bits, ocert_n, nonces, prev_hash, known, eta0, base_slot, base_no, length, window,
         env=None):
    """st: dict(last_slot (None = Origin), counters, evolving, candidate, epoch_nonce, lab, leb).
    Returns (verdicts, chain_stop, processed).  st is updated in place to the state the
    reference chain reaches: after the last valid header before the first invalid one
    (the reference stops the chain there).  Verdicts of later headers are would-be
    verdicts, judged against a working copy that skips the invalid headers.  env (optional):
    validateHeader's envelope checks first (envelope_verdict); env["tip"] is the chain tip,
    updated like st."""
    def epoch(s):
        return base_no + (s - base_slot) // length
    w = _copy(st)
    if env is not None:
        w["tip"] = env["tip"]
    frozen = None
    out, stop = [], None
    i = 0
    for i in range(len(slots) + 1):
        if i == len(slots):
            break
        s = int(slots[i])
        e_new = epoch(s)
        e_old = 0 if w["last_slot"] is None else epoch(w["last_slot"])
        t_epoch, t_leb = w["epoch_nonce"], w["leb"]
        if e_new > e_old:
            t_epoch, t_leb = combine(w["candidate"], w["leb"]), w["lab"]
        if t_epoch != eta0:
            break
        m = w["counters"].get(hk[i], 0 if hk[i] in known else None)
        v = verdict(int(bits[i]), m, int(ocert_n[i]))
        if env is not None and v != V_INPUT:
            ve = envelope_verdict(env, w["tip"], i, s, prev_hash[i])
            v = ve if ve != V_OK else v
        out.append(v)
        if v != V_OK:
            if stop is None:
                stop = i
                frozen = _copy(w)
            continue
        w["epoch_nonce"], w["leb"] = t_epoch, t_leb
        w["last_slot"] = s
        w["lab"] = prev_hash[i]
        w["evolving"] = combine(w["evolving"], bytes(nonces[i]))
        if s + window < base_slot + (e_new - base_no + 1) * length:
            w["candidate"] = w["evolving"]
        w["counters"][hk[i]] = int(ocert_n[i])
        if env is not None:
            w["tip"] = (s, int(env["block_no"][i]), bytes(env["header_hash"][i]))
    processed = i
    res = frozen if frozen is not None else w
    if env is not None:
        env["tip"] = res.pop("tip")
    st.clear()
    st.update(res)
    return out, min(len(slots) if stop is None else stop, processed), processed
