"""The FFI call sequence of the Haskell binding, replayed from C (integration/c/
ffi_harness.c against libpraos_hip.so; module integration/haskell/.../Praos/Batch.hs),
and the multi-threaded uses of the C ABI (one context per POSIX thread; a praos_group
of several members on one device).

The harness streams a multi-epoch ImmutableDB the way the binding does (cut at epoch
boundaries, praos_ticked_epoch_nonce -> praos_set_epoch -> praos_verify_header_bytes ->
praos_validate_headers) and must end in the PraosState (CBOR) and tip that both the
library's own driver (praos_replay_immutable) and the Python replay reach; on a copy
with a corrupted header all three stop at the same header with the same verdict."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from test_gpu_replay import ENV, EPOCH_LEN, _genesis_state, _locate, chain, tchain  # noqa: F401  (fixtures)

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "integration", "c", "ffi_harness")


def _epoch_file(path, chain, tpraos_extra=None):
    p = chain["params"]
    lv_major = ENV['lv_prot_major'] if tpraos_extra is None else 6
    lines = [f"eta0 {chain['cfg']['eta0'].hex()}",
             f"params {p.slots_per_kes_period} {p.max_kes_evo} {p.f_is_one} {p.vrf_check_output} {bytes(p.c_raw).hex()}",
             "epoch " + " ".join(str(x) for x in chain["epoch_info"]),
             f"env {ENV['max_major_pv']} {lv_major} {ENV['max_header_size']} {ENV['max_body_size']}"]
    if tpraos_extra is not None:
        lines.append(f"tpraos {tpraos_extra.hex()}")
    lines += [f"pool {h.hex()} {v.hex()} {int(s).to_bytes(16, 'little').hex()}" for h, v, s in chain["pools"]]
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def _run_harness(db, epoch_file, threads=4):
    assert os.path.exists(HARNESS), "build it: make -C integration/c (done by __graft_entry__.build())"
    r = subprocess.run([HARNESS, db, epoch_file, str(threads)], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr
    return {d["phase"]: d for d in (json.loads(x) for x in r.stdout.splitlines() if x.strip())}


def _python_replay(ctx, chain, db):
    from praos_hip import abi
    st, env = _genesis_state(chain["cfg"]["eta0"]), dict(ENV, tip=None)
    stats, _ = ctx.replay_immutable(db, chain["pools"], chain["params"], chain["epoch_info"], st, env)
    return stats, abi.state_encode(st).hex(), env["tip"]


def _agree(out, stats, cbor, tip):
    for phase in ("binding", "binding_group", "typed", "typed_group", "typed_stream", "replay", "replay_group"):
        if phase not in out:                 # (no typed phases for TPraos databases, no binding_group for Praos)
            continue
        o = out[phase]
        assert (o["validated"], o["stop_index"], o["stop_verdict"]) == \
            (stats["validated"], stats["stop_index"], stats["stop_verdict"]), phase
        assert o["state_cbor"] == cbor, phase
        assert (o["tip_slot"], o["tip_block_no"], bytes.fromhex(o["tip_hash"])) == tip, phase


def test_ffi_sequence_matches_replay(ctx, chain, tmp_path):  # noqa: F811
    ef = str(tmp_path / "epoch.txt")
    _epoch_file(ef, chain)
    out = _run_harness(chain["path"], ef)
    stats, cbor, tip = _python_replay(ctx, chain, chain["path"])
    n = len(chain["off"])
    assert stats["validated"] == n and out["binding"]["epochs"] == stats["epochs"] == 4
    assert out["typed"]["epochs"] == 4 and out["typed"]["stop_bits"] == 0
    # the group sequences (validateEpochHeaders on withPraosBatchDevices [0,0,0,0]; the replay dealt
    # over 4 members in 97-header batches) end in the same state
    assert {"typed_group", "replay_group"} <= set(out) and out["typed_group"]["stop_bits"] == 0
    # the streaming form (praosSubmitHeaderBytes: each epoch as 3 batches in flight, then the drain)
    assert out["typed_stream"]["epochs"] == 4 and out["typed_stream"]["stop_bits"] == 0
    _agree(out, stats, cbor, tip)
    t = out["threads"]
    assert t["threads_equal"] and t["group_equal"] and t["group_size"] == 4
    assert t["valid"] == t["headers"] == int((chain["slots"] < EPOCH_LEN).sum())


def test_ffi_sequence_stops_with_replay(ctx, chain, tmp_path):  # noqa: F811
    from praos_hip import abi
    k = int(np.nonzero(chain["slots"] >= EPOCH_LEN)[0][17])
    db = str(tmp_path / "bad")
    shutil.copytree(chain["path"], db)
    fname, pos = _locate(chain, k)
    raw = bytearray(open(os.path.join(db, fname), "rb").read())
    raw[pos + int(chain["len"][k]) - 200] ^= 0x01              # inside the KES signature
    open(os.path.join(db, fname), "wb").write(bytes(raw))
    ef = str(tmp_path / "epoch.txt")
    _epoch_file(ef, chain)
    out = _run_harness(db, ef, threads=2)
    stats, cbor, tip = _python_replay(ctx, chain, db)
    assert (stats["stop_index"], stats["stop_verdict"]) == (k, abi.V_KES_SIG)
    _agree(out, stats, cbor, tip)
    # the typed path (Batch/Validate.hs) gets the stopping header's bits: a KES failure in
    # the leaf signature, which Batch.Errors turns into InvalidKesSignatureOCERT
    assert out["typed"]["stop_bits"] & (abi.BIT_KES_MERKLE | abi.BIT_KES_LEAF)
    assert out["typed_group"]["stop_bits"] == out["typed"]["stop_bits"] == out["typed_stream"]["stop_bits"]


def test_ffi_tpraos_sequence_matches_replay(ctx, tchain, tmp_path):  # noqa: F811
    """The TPraos call sequence (praos_tpraos_ticked_epoch_nonce -> praos_set_epoch ->
    praos_verify_tpraos_header_bytes -> praos_tpraos_update_chain_dep_state, epoch by epoch)
    and praos_replay_immutable_tpraos, from C, over the TPraos database: both end in the
    Python TPraos replay's state and tip; with a damaged KES signature all three stop at
    the same header."""
    from praos_hip import abi
    from test_gpu_replay import TP_EXTRA
    ef = str(tmp_path / "epoch_tp.txt")
    _epoch_file(ef, tchain, tpraos_extra=TP_EXTRA)

    def py(db):
        st, env = _genesis_state(tchain["cfg"]["eta0"]), dict(ENV, tip=None, lv_prot_major=6)
        stats, _, _ = ctx.replay_immutable(db, tchain["pools"], tchain["params"], tchain["epoch_info"], st, env,
                                           tpraos=True, extra_entropy=TP_EXTRA)
        return stats, abi.state_encode(st).hex(), env["tip"]
    out = _run_harness(tchain["path"], ef)
    stats, cbor, tip = py(tchain["path"])
    assert stats["validated"] == len(tchain["off"]) and out["binding"]["epochs"] == stats["epochs"] == 3
    _agree(out, stats, cbor, tip)
    assert "threads" not in out
    k = int(np.nonzero(tchain["slots"] >= EPOCH_LEN)[0][11])
    db = str(tmp_path / "bad_tp")
    shutil.copytree(tchain["path"], db)
    fname, pos = _locate(tchain, k)
    raw = bytearray(open(os.path.join(db, fname), "rb").read())
    raw[pos + int(tchain["len"][k]) - 200] ^= 0x01
    open(os.path.join(db, fname), "wb").write(bytes(raw))
    out = _run_harness(db, ef, threads=2)
    stats, cbor, tip = py(db)
    assert (stats["stop_index"], stats["stop_verdict"]) == (k, abi.V_TPRAOS)
    _agree(out, stats, cbor, tip)
    assert {"binding_group", "replay_group"} <= set(out)
    assert out["tpraos_stop"]["failures"] == abi.TPF_KES_SIG
    assert out["tpraos_stop"]["errors"] == ["OverlayFailure (OcertFailure InvalidKesSignatureOCERT)"]


# PRAOS_TPF_* -> the SL.ChainTransitionError constructor, in ValidateAll's order (Batch/Errors.hs
# tpraosFailureTable; tests/test_abi.py holds it equal to the harness's table)
_TPF_ORDER = [("TPF_NOT_ACTIVE", "NotActiveSlotOVERLAY"), ("TPF_GEN_COLD", "WrongGenesisColdKeyOVERLAY"),
              ("TPF_VRF_KEY_UNKNOWN", "VRFKeyUnknown"), ("TPF_VRF_KEY_WRONG", "VRFKeyWrongVRFKey"),
              ("TPF_GEN_VRF", "WrongGenesisVRFKeyOVERLAY"), ("TPF_BAD_NONCE", "VRFKeyBadNonce"),
              ("TPF_BAD_LEADER", "VRFKeyBadLeaderValue"), ("TPF_LEADER_TOO_BIG", "VRFLeaderValueTooBig"),
              ("TPF_KES_BEFORE_START", "OcertFailure KESBeforeStartOCERT"),
              ("TPF_KES_AFTER_END", "OcertFailure KESAfterEndOCERT"),
              ("TPF_OCERT_SIG", "OcertFailure InvalidSignatureOCERT"),
              ("TPF_KES_SIG", "OcertFailure InvalidKesSignatureOCERT"),
              ("TPF_COUNTER_MISSING", "OcertFailure NoCounterForKeyHashOCERT"),
              ("TPF_COUNTER_TOO_SMALL", "OcertFailure CounterTooSmallOCERT"),
              ("TPF_COUNTER_OVER_INC", "OcertFailure CounterOverIncrementedOCERT")]


@pytest.mark.parametrize("field", ["eta_proof", "leader_proof", "vrf_vk", "cold_vk", "ocert_sig"])
def test_ffi_tpraos_stop_errors(ctx, tchain, tmp_path, field):  # noqa: F811
    """One stopping header per TPraos failure kind: a byte of the stored BHeader's field damaged
    on disk (every such change also breaks the KES signature over the body).  The harness's
    TPraos sequence stops where the library's replay and the oracle's fold stop, with the
    oracle's PRTCL failure set, and names the ChainTransitionError constructors in the order
    ValidateAll collects them -- the list Batch/Errors.hs tpraosChainTransitionError builds."""
    from praos_hip import abi
    from test_gpu_replay import TP_EXTRA, _tp_oracle_fold
    k = int(np.nonzero(tchain["slots"] >= EPOCH_LEN)[0][5])
    o, D = ctx.verify_tpraos_header_bytes(tchain["arena"], tchain["off"][k:k + 1], tchain["len"][k:k + 1],
                                          decoded=True)
    hdr = bytes(tchain["arena"][int(tchain["off"][k]):int(tchain["off"][k]) + int(tchain["len"][k])])
    value = {"eta_proof": D["vrf_proof"][0], "leader_proof": D["leader_proof"][0], "vrf_vk": D["vrf_vk"][0],
             "cold_vk": D["cold_vk"][0], "ocert_sig": D["ocert_sig"][0]}[field]
    at = hdr.index(bytes(value)) + 9
    db = str(tmp_path / f"tp_{field}")
    shutil.copytree(tchain["path"], db)
    fname, pos = _locate(tchain, k)
    raw = bytearray(open(os.path.join(db, fname), "rb").read())
    raw[pos + at] ^= 0x04
    open(os.path.join(db, fname), "wb").write(bytes(raw))
    ef = str(tmp_path / "epoch_tp.txt")
    _epoch_file(ef, tchain, tpraos_extra=TP_EXTRA)
    out = _run_harness(db, ef, threads=2)
    st, env = _genesis_state(tchain["cfg"]["eta0"]), dict(ENV, tip=None, lv_prot_major=6)
    stats, v, f = ctx.replay_immutable(db, tchain["pools"], tchain["params"], tchain["epoch_info"], st, env,
                                       verdicts_cap=len(tchain["off"]), tpraos=True, extra_entropy=TP_EXTRA)
    assert (stats["stop_index"], stats["stop_verdict"]) == (k, abi.V_TPRAOS)
    assert out["binding"]["stop_index"] == out["binding_group"]["stop_index"] == k
    fails = int(out["tpraos_stop"]["failures"])
    assert fails == int(f[k])
    # the oracle's fold (oracle/tpraos.py, crypto from the GPU) over the damaged headers: same set
    data = dict(tchain, path=db)
    raw_arena = bytearray(tchain["arena"])
    raw_arena[int(tchain["off"][k]) + at] ^= 0x04
    data["arena"] = np.frombuffer(bytes(raw_arena), np.uint8)
    _, ofails, _, _, ostop = _tp_oracle_fold(ctx, data, k + 1)
    assert ostop == k and ofails[k] == fails
    want = [f"OverlayFailure ({name})" for bit, name in _TPF_ORDER if fails & getattr(abi, bit)]
    assert out["tpraos_stop"]["errors"] == want and len(want) >= 2
    assert fails & abi.TPF_KES_SIG
