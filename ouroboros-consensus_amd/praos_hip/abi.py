"""ctypes binding of libpraos_hip.so (include/praos_hip.h).

This is plumbing for tests and bench.py; the product is the C ABI itself.  The
library is the gfx950 HIP build; there is deliberately no CPU fallback: every
call here goes to the GPU, and a missing library raises.
"""
import ctypes
import os

import numpy as np

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_PKG), "libpraos_hip.so")
# A/B experiments only: load an alternative in-tree build (same ABI)
LIB_PATH = os.environ.get("PRAOS_HIP_LIB", LIB_PATH)
HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(_PKG)), "include", "praos_hip.h")

u8p = ctypes.POINTER(ctypes.c_uint8)
u16p = ctypes.POINTER(ctypes.c_uint16)
u32p = ctypes.POINTER(ctypes.c_uint32)
u64p = ctypes.POINTER(ctypes.c_uint64)
i32p = ctypes.POINTER(ctypes.c_int32)

# bits (PRAOS_BIT_*)
BLK_DECODE = 0x01      # block-integrity result bits (praos_verify_block_integrity)
BLK_KES = 0x02
BLK_BODY_HASH = 0x04
BIT_KES_BEFORE_START = 0x0001
BIT_KES_AFTER_END = 0x0002
BIT_OCERT_SIG = 0x0004
BIT_KES_MERKLE = 0x0008
BIT_KES_LEAF = 0x0010
BIT_COUNTER_MISSING = 0x0020
BIT_COUNTER_TOO_SMALL = 0x0040
BIT_COUNTER_OVER_INC = 0x0080
BIT_VRF_KEY_UNKNOWN = 0x0100
BIT_VRF_KEY_WRONG = 0x0200
BIT_VRF_PROOF = 0x0400
BIT_VRF_OUTPUT = 0x0800
BIT_LEADER = 0x1000
BIT_INPUT = 0x8000
HOST_ONLY = -1
BIT_TP_VRF_NONCE = 0x0400
BIT_TP_VRF_LEADER = 0x0800
# praos_synth_params.corrupt_fields
CORRUPT_OCERT, CORRUPT_KES_SIG, CORRUPT_VRF_PROOF, CORRUPT_VRF_OUT, CORRUPT_BODY = 0x01, 0x02, 0x04, 0x08, 0x10

# verdicts (enum praos_verdict)
V_OK, V_KES_BEFORE_START, V_KES_AFTER_END, V_OCERT_SIG, V_KES_SIG, V_COUNTER_MISSING, \
    V_COUNTER_TOO_SMALL, V_COUNTER_OVER_INC, V_VRF_KEY_UNKNOWN, V_VRF_KEY_WRONG, V_VRF_BAD_PROOF, \
    V_LEADER_TOO_BIG, V_INPUT, V_ENV_BLOCK_NO, V_ENV_SLOT_NO, V_ENV_PREV_HASH, V_ENV_OBSOLETE_NODE, \
    V_ENV_HEADER_SIZE, V_ENV_BLOCK_SIZE = range(19)
V_TPRAOS = 19
# TPraos PRTCL predicate failures (PRAOS_TPF_*)
TPF_KES_BEFORE_START, TPF_KES_AFTER_END, TPF_OCERT_SIG, TPF_KES_SIG, TPF_COUNTER_MISSING, \
    TPF_COUNTER_TOO_SMALL, TPF_COUNTER_OVER_INC = 0x1, 0x2, 0x4, 0x8, 0x10, 0x20, 0x40
TPF_VRF_KEY_UNKNOWN, TPF_VRF_KEY_WRONG, TPF_BAD_NONCE, TPF_BAD_LEADER, TPF_LEADER_TOO_BIG, TPF_NOT_ACTIVE, \
    TPF_GEN_COLD, TPF_GEN_VRF = 0x100, 0x200, 0x400, 0x800, 0x1000, 0x2000, 0x4000, 0x8000


class Params(ctypes.Structure):
    _fields_ = [("slots_per_kes_period", ctypes.c_uint64), ("max_kes_evo", ctypes.c_uint64),
                ("f_is_one", ctypes.c_int32), ("vrf_check_output", ctypes.c_int32),
                ("c_raw", ctypes.c_uint8 * 16)]


class Pool(ctypes.Structure):
    _fields_ = [("hash28", ctypes.c_uint8 * 28), ("vrf_hash32", ctypes.c_uint8 * 32),
                ("sigma_fp", ctypes.c_uint8 * 16)]


class Headers(ctypes.Structure):
    _fields_ = [("n", ctypes.c_size_t), ("slot", u64p), ("cold_vk", u8p), ("vrf_vk", u8p), ("vrf_out", u8p),
                ("vrf_proof", u8p), ("hot_vk", u8p), ("ocert_n", u64p), ("ocert_c0", u64p), ("ocert_sig", u8p),
                ("kes_sig", u8p), ("body_off", u64p), ("body_len", u32p), ("body_bytes", u8p),
                ("body_bytes_len", ctypes.c_size_t)]


class Out(ctypes.Structure):
    _fields_ = [("bits", u16p), ("pool_idx", i32p), ("beta", u8p), ("leader", u8p), ("nonce", u8p)]


class TPHeaders(ctypes.Structure):
    _fields_ = [("h", Headers), ("leader_out", u8p), ("leader_proof", u8p)]


class TPOut(ctypes.Structure):
    _fields_ = [("bits", u16p), ("pool_idx", i32p), ("beta_eta", u8p), ("beta_leader", u8p), ("nonce", u8p)]


class GenDeleg(ctypes.Structure):
    _fields_ = [("genesis_hash28", ctypes.c_uint8 * 28), ("delegate_hash28", ctypes.c_uint8 * 28),
                ("vrf_hash32", ctypes.c_uint8 * 32)]


class Overlay(ctypes.Structure):
    _fields_ = [("d_num", ctypes.c_uint64), ("d_den", ctypes.c_uint64), ("asc_num", ctypes.c_uint64),
                ("asc_den", ctypes.c_uint64), ("epoch_base_slot", ctypes.c_uint64), ("epoch_length", ctypes.c_uint64),
                ("gen_delegs", ctypes.POINTER(GenDeleg)), ("n_gen_delegs", ctypes.c_uint32)]


class Nonce(ctypes.Structure):
    _fields_ = [("hash", ctypes.c_uint8 * 32), ("neutral", ctypes.c_int32)]


class ChainState(ctypes.Structure):
    _fields_ = [("last_slot_origin", ctypes.c_int32), ("last_slot", ctypes.c_uint64),
                ("counter_hash28", u8p), ("counter", u64p), ("m", ctypes.c_size_t), ("cap", ctypes.c_size_t),
                ("evolving", Nonce), ("candidate", Nonce), ("epoch_nonce", Nonce), ("lab", Nonce),
                ("last_epoch_block", Nonce)]


class EpochInfo(ctypes.Structure):
    _fields_ = [("epoch_base_slot", ctypes.c_uint64), ("epoch_base_no", ctypes.c_uint64),
                ("epoch_length", ctypes.c_uint64), ("stability_window", ctypes.c_uint64)]


class Envelope(ctypes.Structure):
    _fields_ = [("block_no", u64p), ("header_hash", u8p), ("header_size", u32p), ("body_size", u32p),
                ("tip_is_origin", ctypes.c_int32), ("tip_slot", ctypes.c_uint64), ("tip_block_no", ctypes.c_uint64),
                ("tip_hash", ctypes.c_uint8 * 32), ("max_major_pv", ctypes.c_uint64),
                ("lv_prot_major", ctypes.c_uint64), ("max_header_size", ctypes.c_uint64),
                ("max_body_size", ctypes.c_uint64)]


class ReplayStats(ctypes.Structure):
    _fields_ = [("skipped", ctypes.c_uint64), ("headers", ctypes.c_uint64), ("validated", ctypes.c_uint64), ("stop_index", ctypes.c_uint64),
                ("stop_verdict", ctypes.c_uint32), ("epochs", ctypes.c_uint32), ("batches", ctypes.c_uint32),
                ("chunks", ctypes.c_uint32), ("ms_io", ctypes.c_double), ("ms_device", ctypes.c_double),
                ("ms_fold", ctypes.c_double), ("ms_nonce", ctypes.c_double)]


class LedgerView(ctypes.Structure):
    _fields_ = [("first_epoch", ctypes.c_uint64), ("pools", ctypes.c_void_p), ("npools", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32), ("lv_prot_major", ctypes.c_uint64),
                ("max_header_size", ctypes.c_uint64), ("max_body_size", ctypes.c_uint64)]


class Counters(ctypes.Structure):
    _fields_ = [("hash28", u8p), ("counter", u64p), ("m", ctypes.c_size_t)]


class SynthParams(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint64), ("npools", ctypes.c_uint32), ("first_slot", ctypes.c_uint64),
                ("slot_stride", ctypes.c_uint64), ("body_len", ctypes.c_uint32),
                ("corrupt_per_10000", ctypes.c_uint32), ("nkes", ctypes.c_uint32), ("seed", ctypes.c_uint8 * 32),
                ("body_hash", u8p), ("sched_slot", u64p), ("sched_pool", u32p), ("block_no0", ctypes.c_uint64),
                ("link_prev", ctypes.c_int32), ("prev0", u8p), ("header_hash", u8p),
                ("corrupt_fields", ctypes.c_uint32)]


class HeaderBytes(ctypes.Structure):
    _fields_ = [("n", ctypes.c_size_t), ("bytes", u8p), ("bytes_len", ctypes.c_size_t), ("off", u64p),
                ("len", u32p)]


DECODED_FIELDS = (  # name, dtype, record shape (praos_decoded, include/praos_hip.h)
    ("status", np.uint16, ()), ("block_no", np.uint64, ()), ("slot", np.uint64, ()), ("prev_hash", np.uint8, (32,)),
    ("prev_is_genesis", np.uint8, ()), ("cold_vk", np.uint8, (32,)), ("vrf_vk", np.uint8, (32,)),
    ("vrf_out", np.uint8, (64,)), ("vrf_proof", np.uint8, (80,)), ("body_size", np.uint32, ()),
    ("body_hash", np.uint8, (32,)), ("hot_vk", np.uint8, (32,)), ("ocert_n", np.uint64, ()),
    ("ocert_c0", np.uint64, ()), ("ocert_sig", np.uint8, (64,)), ("prot_major", np.uint64, ()),
    ("prot_minor", np.uint64, ()), ("kes_sig", np.uint8, (448,)), ("signed_len", np.uint32, ()),
    ("signed_body", np.uint8, (448,)), ("header_hash", np.uint8, (32,)))
_CT = {np.uint8: u8p, np.uint16: u16p, np.uint32: u32p, np.uint64: u64p}


class Decoded(ctypes.Structure):
    _fields_ = [(name, _CT[dt]) for name, dt, _ in DECODED_FIELDS]


# decode status (PRAOS_DEC_*)
DEC_RANGE, DEC_SYNTAX, DEC_SIZE, DEC_UNSUPPORTED, DEC_TRAILING, DEC_NONCANONICAL, DEC_OVERFLOW = \
    0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40
DEC_FAILED = 0x5F
SIGNED_STRIDE = 448
TP_SIGNED_STRIDE = 640

# every entry point declared in include/praos_hip.h: name -> (restype, argtypes)
SIGNATURES = {
    "praos_abi_version": (ctypes.c_int, []),
    "praos_host_register": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]),
    "praos_host_unregister": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "praos_open": (ctypes.c_void_p, [ctypes.c_int]),
    "praos_close": (None, [ctypes.c_void_p]),
    "praos_last_error": (ctypes.c_char_p, [ctypes.c_void_p]),
    "praos_set_epoch": (ctypes.c_int, [ctypes.c_void_p, u8p, ctypes.POINTER(Pool), ctypes.c_uint32,
                                       ctypes.POINTER(Params)]),
    "praos_verify_headers": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Headers), ctypes.POINTER(Out)]),
    "praos_batch_upload": (ctypes.c_void_p, [ctypes.c_void_p, ctypes.POINTER(Headers)]),
    "praos_batch_run": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "praos_batch_sync": (ctypes.c_int, [ctypes.c_void_p]),
    "praos_batch_download": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(Out)]),
    "praos_batch_free": (None, [ctypes.c_void_p, ctypes.c_void_p]),
    "praos_batch_kernel_ms": (ctypes.c_float, [ctypes.c_void_p, ctypes.c_int]),
    "praos_set_option": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "praos_batch_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, u32p]),
    "praos_batch_dedup_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, u32p]),
    "praos_verify_ocert": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, u8p, u8p, u64p, u64p, u8p, u8p]),
    "praos_verify_kes": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, u8p, u32p, u8p, u64p, u32p, u8p,
                                        ctypes.c_size_t, u8p]),
    "praos_verify_vrf": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, u8p, u8p, u8p, u8p, u8p]),
    "praos_check_leader": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, u8p, u8p, ctypes.POINTER(Params), u8p]),
    "praos_apply_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Headers), ctypes.POINTER(Out),
                                         ctypes.POINTER(Counters), u8p, ctypes.POINTER(ctypes.c_size_t)]),
    "praos_update_chain_dep_state": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Headers), u8p, u8p,
                                                    ctypes.POINTER(Out), ctypes.POINTER(EpochInfo),
                                                    ctypes.POINTER(ChainState), u8p, ctypes.POINTER(ctypes.c_size_t),
                                                    ctypes.POINTER(ctypes.c_size_t)]),
    "praos_validate_headers": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Headers), u8p, u8p, ctypes.POINTER(Out),
                                              ctypes.POINTER(Envelope), ctypes.POINTER(EpochInfo),
                                              ctypes.POINTER(ChainState), u8p, ctypes.POINTER(ctypes.c_size_t),
                                              ctypes.POINTER(ctypes.c_size_t)]),
    "praos_state_encode": (ctypes.c_int, [ctypes.POINTER(ChainState), u8p, ctypes.c_size_t,
                                          ctypes.POINTER(ctypes.c_size_t)]),
    "praos_state_decode": (ctypes.c_int, [u8p, ctypes.c_size_t, ctypes.POINTER(ChainState)]),
    "praos_replay_immutable": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(Pool), ctypes.c_uint32,
                                              ctypes.POINTER(Params), ctypes.POINTER(EpochInfo),
                                              ctypes.POINTER(Envelope), ctypes.POINTER(ChainState), ctypes.c_size_t,
                                              u8p, ctypes.c_size_t, ctypes.POINTER(ReplayStats)]),
    "praos_replay_immutable_tpraos": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(Pool),
                                                     ctypes.c_uint32, ctypes.POINTER(Params),
                                                     ctypes.POINTER(EpochInfo), ctypes.POINTER(Nonce),
                                                     ctypes.POINTER(Envelope), ctypes.POINTER(ChainState),
                                                     ctypes.c_size_t, u8p, u16p, ctypes.c_size_t,
                                                     ctypes.POINTER(ReplayStats)]),
    "praos_replay_immutable_views": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(LedgerView),
                                                    ctypes.c_uint32, ctypes.POINTER(Params), ctypes.POINTER(EpochInfo),
                                                    ctypes.POINTER(Envelope), ctypes.POINTER(ChainState),
                                                    ctypes.c_size_t, u8p, ctypes.c_size_t,
                                                    ctypes.POINTER(ReplayStats)]),
    "praos_batch_upload_tpraos_bytes": (ctypes.c_void_p, [ctypes.c_void_p, ctypes.POINTER(HeaderBytes)]),
    "praos_batch_download_tpraos": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(TPOut)]),
    "praos_tpraos_validate_headers_nonces": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(TPHeaders), u8p, u8p,
                                                            ctypes.POINTER(TPOut), ctypes.POINTER(Envelope),
                                                            ctypes.POINTER(EpochInfo), ctypes.POINTER(Nonce),
                                                            ctypes.POINTER(ChainState), ctypes.POINTER(Nonce),
                                                            ctypes.c_uint32, u8p, u8p, u16p,
                                                            ctypes.POINTER(ctypes.c_size_t),
                                                            ctypes.POINTER(ctypes.c_size_t)]),
    "praos_ticked_epoch_nonce": (ctypes.c_int, [ctypes.POINTER(ChainState), ctypes.POINTER(EpochInfo), ctypes.c_uint64,
                                                ctypes.POINTER(Nonce)]),
    "praos_tpraos_ticked_epoch_nonce": (ctypes.c_int, [ctypes.POINTER(ChainState), ctypes.POINTER(EpochInfo),
                                                       ctypes.c_uint64, ctypes.POINTER(Nonce), ctypes.POINTER(Nonce)]),
    "praos_group_open": (ctypes.c_void_p, [i32p, ctypes.c_int]),
    "praos_group_close": (None, [ctypes.c_void_p]),
    "praos_group_size": (ctypes.c_int, [ctypes.c_void_p]),
    "praos_group_ctx": (ctypes.c_void_p, [ctypes.c_void_p, ctypes.c_int]),
    "praos_group_last_error": (ctypes.c_char_p, [ctypes.c_void_p]),
    "praos_group_set_option": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "praos_group_set_epoch": (ctypes.c_int, [ctypes.c_void_p, u8p, ctypes.POINTER(Pool), ctypes.c_uint32,
                                             ctypes.POINTER(Params)]),
    "praos_group_verify_headers": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Headers), ctypes.POINTER(Out)]),
    "praos_group_verify_header_bytes": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HeaderBytes),
                                                       ctypes.POINTER(Out), ctypes.POINTER(Decoded)]),
    "praos_group_verify_tpraos_headers": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(TPHeaders),
                                                         ctypes.POINTER(TPOut)]),
    "praos_group_verify_tpraos_header_bytes": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HeaderBytes),
                                                              ctypes.POINTER(TPOut), ctypes.POINTER(Decoded), u8p,
                                                              u8p]),
    "praos_group_set_overlay": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Overlay)]),
    "praos_group_host_register": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]),
    "praos_group_host_unregister": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "praos_group_replay_immutable": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(Pool),
                                                    ctypes.c_uint32, ctypes.POINTER(Params), ctypes.POINTER(EpochInfo),
                                                    ctypes.POINTER(Envelope), ctypes.POINTER(ChainState),
                                                    ctypes.c_size_t, u8p, ctypes.c_size_t,
                                                    ctypes.POINTER(ReplayStats)]),
    "praos_group_replay_immutable_tpraos": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(Pool),
                                                           ctypes.c_uint32, ctypes.POINTER(Params),
                                                           ctypes.POINTER(EpochInfo), ctypes.POINTER(Nonce),
                                                           ctypes.POINTER(Envelope), ctypes.POINTER(ChainState),
                                                           ctypes.c_size_t, u8p, u16p, ctypes.c_size_t,
                                                           ctypes.POINTER(ReplayStats)]),
    "praos_group_verify_block_integrity": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HeaderBytes),
                                                          ctypes.c_uint64, u8p, u8p]),
    "praos_group_replay_immutable_views": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p,
                                                          ctypes.POINTER(LedgerView), ctypes.c_uint32,
                                                          ctypes.POINTER(Params), ctypes.POINTER(EpochInfo),
                                                          ctypes.POINTER(Envelope), ctypes.POINTER(ChainState),
                                                          ctypes.c_size_t, u8p, ctypes.c_size_t,
                                                          ctypes.POINTER(ReplayStats)]),
    "praos_synthesize": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(SynthParams), ctypes.POINTER(Params), u8p,
                                        ctypes.POINTER(Pool), u64p, u8p, u8p, u8p, u8p, u8p, u64p, u64p, u8p, u8p,
                                        u64p, u32p, u8p, u8p]),
    "praos_leader_schedule": (ctypes.c_int, [ctypes.c_void_p, u8p, ctypes.c_uint32, u8p, ctypes.POINTER(Params), u8p,
                                             ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, i32p]),
    "praos_verify_tpraos_headers": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(TPHeaders),
                                                   ctypes.POINTER(TPOut)]),
    "praos_set_overlay": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Overlay)]),
    "praos_overlay_classify": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, u64p, i32p]),
    "praos_tpraos_update_chain_dep_state": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(TPHeaders), u8p, u8p,
                                                           ctypes.POINTER(TPOut), ctypes.POINTER(Envelope),
                                                           ctypes.POINTER(EpochInfo), ctypes.POINTER(Nonce),
                                                           ctypes.POINTER(ChainState), u8p, u16p,
                                                           ctypes.POINTER(ctypes.c_size_t),
                                                           ctypes.POINTER(ctypes.c_size_t)]),
    "praos_synthesize_tpraos": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(SynthParams), ctypes.POINTER(Params),
                                               u8p, ctypes.POINTER(Pool), u64p, u8p, u8p, u8p, u8p, u8p, u64p, u64p,
                                               u8p, u8p, u64p, u32p, u8p, u8p, u8p, u8p]),
    "praos_decode_headers": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HeaderBytes), ctypes.POINTER(Decoded)]),
    "praos_verify_header_bytes": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HeaderBytes), ctypes.POINTER(Out),
                                                 ctypes.POINTER(Decoded)]),
    "praos_verify_header_bytes_submit": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HeaderBytes),
                                                        ctypes.POINTER(Out), ctypes.POINTER(Decoded)]),
    "praos_verify_drain": (ctypes.c_int, [ctypes.c_void_p]),
    "praos_verify_tpraos_header_bytes": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HeaderBytes),
                                                        ctypes.POINTER(TPOut), ctypes.POINTER(Decoded), u8p, u8p]),
    "praos_batch_upload_bytes": (ctypes.c_void_p, [ctypes.c_void_p, ctypes.POINTER(HeaderBytes)]),
    "praos_batch_download_decoded": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(Decoded)]),
    "praos_batch_decode": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "praos_batch_set_nonces": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(Nonce), ctypes.c_uint32,
                                              u8p]),
    "praos_validate_headers_nonces": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Headers), u8p, u8p,
                                                     ctypes.POINTER(Out), ctypes.POINTER(Envelope),
                                                     ctypes.POINTER(EpochInfo), ctypes.POINTER(ChainState),
                                                     ctypes.POINTER(Nonce), ctypes.c_uint32, u8p, u8p,
                                                     ctypes.POINTER(ctypes.c_size_t),
                                                     ctypes.POINTER(ctypes.c_size_t)]),
    "praos_verify_block_integrity": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HeaderBytes), ctypes.c_uint64,
                                                    u8p, u8p]),
    "praos_block_batch_upload": (ctypes.c_void_p, [ctypes.c_void_p, ctypes.POINTER(HeaderBytes)]),
    "praos_block_batch_run": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]),
    "praos_block_batch_download": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, u8p, u8p]),
    "praos_debug_fe": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, u8p, u8p, u8p]),
    "praos_debug_sha512": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, u8p, u64p, u32p, u8p, ctypes.c_size_t,
                                          u8p]),
    "praos_debug_blake2b": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, u8p, u8p]),
    "praos_debug_sc_reduce": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, u8p, u8p]),
    "praos_debug_decode": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, u8p, u8p, u8p]),
    "praos_debug_scalarmult_base": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, u8p, u8p]),
    "praos_debug_leader": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, u8p, u8p, u8p, i32p]),
    "praos_debug_leader512": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, u8p, u8p, u8p, i32p]),
    "praos_debug_hash_to_curve": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, u8p, u8p, u8p]),
}

_lib = None


def load():
    """Load libpraos_hip.so (raises if it was not built: there is no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: build it with __graft_entry__.build() "
                               "(make -C ouroboros-consensus_amd/csrc)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def ptr(a, t=u8p):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(t)


OPT_CONCURRENT, OPT_KERNELS, OPT_KEYCACHE, OPT_DEDUP, OPT_PIPELINE, OPT_KES_PAIR, OPT_POOL_KEYS = 1, 2, 3, 4, 5, 6, 7
OPT_KES_NOCACHE = 8
# (praos_set_option, praos_hip.h)


class PraosError(RuntimeError):
    pass


class Context:
    """One praos_ctx (one GPU).  Mirrors the lifetime rules of the C ABI."""

    def __init__(self, device: int = 0):
        self.L = load()
        self.h = self.L.praos_open(device)
        if not self.h:
            raise PraosError(f"praos_open({device}) failed (no HIP device?)")
        self._keep = []

    def close(self):
        if self.h:
            self.L.praos_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def check(self, rc):
        if rc != 0:
            msg = self.L.praos_last_error(self.h)
            raise PraosError(f"praos rc={rc}: {msg.decode() if msg else ''}")

    # ---- epoch ----
    @staticmethod
    def pool_array(pools):
        """pools: list of (hash28: bytes, vrf_hash32: bytes, sigma_fp: int)."""
        if not pools:
            return (Pool * 1)()
        # one buffer of 76-byte records (the struct has no padding), copied in once
        data = b"".join(bytes(h)[:28].ljust(28, b"\0") + bytes(v)[:32].ljust(32, b"\0") + int(s).to_bytes(16, "little")
                        for h, v, s in pools)
        return (Pool * len(pools)).from_buffer_copy(data)

    def set_epoch(self, eta0, pools, params: Params):
        """pools: list of (hash28: bytes, vrf_hash32: bytes, sigma_fp: int)."""
        arr = self.pool_array(pools)
        e = None
        if eta0 is not None:
            eb = np.frombuffer(bytes(eta0), dtype=np.uint8).copy()
            self._keep.append(eb)
            e = ptr(eb)
        self.check(self.L.praos_set_epoch(self.h, e, arr, len(pools), ctypes.byref(params)))
        self._keep.append(arr)

    # ---- headers ----
    @staticmethod
    def headers_struct(H: dict):
        """H: dict of numpy arrays: slot u64[n], cold_vk u8[n,32], vrf_vk, vrf_out[n,64], vrf_proof[n,80],
        hot_vk, ocert_n u64, ocert_c0 u64, ocert_sig[n,64], kes_sig[n,448], body_off u64, body_len u32,
        body_bytes u8[]."""
        s = Headers()
        s.n = len(H["slot"])
        s.slot = ptr(H["slot"], u64p)
        for k in ("cold_vk", "vrf_vk", "vrf_out", "vrf_proof", "hot_vk", "ocert_sig", "kes_sig", "body_bytes"):
            setattr(s, k, ptr(H[k]))
        s.ocert_n = ptr(H["ocert_n"], u64p)
        s.ocert_c0 = ptr(H["ocert_c0"], u64p)
        s.body_off = ptr(H["body_off"], u64p)
        s.body_len = ptr(H["body_len"], u32p)
        s.body_bytes_len = len(H["body_bytes"])
        return s

    @staticmethod
    def alloc_out(n):
        return {"bits": np.zeros(n, np.uint16), "pool_idx": np.zeros(n, np.int32),
                "beta": np.zeros((n, 64), np.uint8), "leader": np.zeros((n, 32), np.uint8),
                "nonce": np.zeros((n, 32), np.uint8)}

    @staticmethod
    def out_struct(o):
        s = Out()
        s.bits = ptr(o["bits"], u16p)
        s.pool_idx = ptr(o["pool_idx"], i32p)
        s.beta = ptr(o["beta"])
        s.leader = ptr(o["leader"])
        s.nonce = ptr(o["nonce"])
        return s

    def verify_headers(self, H, out=None):
        """out: caller-owned output arrays (alloc_out) reused across calls, as a replay loop does."""
        n = len(H["slot"])
        o = self.alloc_out(n) if out is None else out
        hs = self.headers_struct(H)
        os_ = self.out_struct(o)
        self.check(self.L.praos_verify_headers(self.h, ctypes.byref(hs), ctypes.byref(os_)))
        return o

    @staticmethod
    def tp_headers_struct(H):
        th = TPHeaders()
        th.h = Context.headers_struct(H)
        th.leader_out = ptr(H["leader_out"])
        th.leader_proof = ptr(H["leader_proof"])
        return th

    @staticmethod
    def tp_out(n):
        """TPraos output arrays and their praos_tpraos_out struct."""
        o = {"bits": np.zeros(n, np.uint16), "pool_idx": np.zeros(n, np.int32),
             "beta_eta": np.zeros((n, 64), np.uint8), "beta_leader": np.zeros((n, 64), np.uint8),
             "nonce": np.zeros((n, 32), np.uint8)}
        to = TPOut()
        to.bits, to.pool_idx = ptr(o["bits"], u16p), ptr(o["pool_idx"], i32p)
        to.beta_eta, to.beta_leader, to.nonce = ptr(o["beta_eta"]), ptr(o["beta_leader"]), ptr(o["nonce"])
        return o, to

    def verify_tpraos_headers(self, H):
        """H as for verify_headers plus leader_out [n,64] / leader_proof [n,80] (the bheaderL cert)."""
        th = self.tp_headers_struct(H)
        o, to = self.tp_out(len(H["slot"]))
        self.check(self.L.praos_verify_tpraos_headers(self.h, ctypes.byref(th), ctypes.byref(to)))
        return o

    def set_overlay(self, d, f, epoch_base_slot, epoch_length, gen_delegs):
        """TPraos overlay schedule (praos_set_overlay): d, f Fractions; gen_delegs list of
        (genesis_hash28, delegate_hash28, vrf_hash32).  d = None clears everything."""
        if d is None:
            self.check(self.L.praos_set_overlay(self.h, None))
            return
        arr = (GenDeleg * max(1, len(gen_delegs)))()
        for k, (g, dl, v) in enumerate(gen_delegs):
            ctypes.memmove(arr[k].genesis_hash28, bytes(g), 28)
            ctypes.memmove(arr[k].delegate_hash28, bytes(dl), 28)
            ctypes.memmove(arr[k].vrf_hash32, bytes(v), 32)
        ov = Overlay(d.numerator, d.denominator, f.numerator, f.denominator, epoch_base_slot, epoch_length,
                     ctypes.cast(arr, ctypes.POINTER(GenDeleg)), len(gen_delegs))
        self._overlay_keep = arr
        self.check(self.L.praos_set_overlay(self.h, ctypes.byref(ov)))

    def overlay_classify(self, slots):
        s = np.ascontiguousarray(slots, dtype=np.uint64)
        out = np.zeros(len(s), np.int32)
        self.check(self.L.praos_overlay_classify(self.h, len(s), ptr(s, u64p), ptr(out, i32p)))
        return out

    def tpraos_update_chain_dep_state(self, H, crypto, prev_hash, state: dict, epoch_info, prev_is_genesis=None,
                                      extra_entropy=None):
        """praos_tpraos_update_chain_dep_state over TPraos outputs (verify_tpraos_headers);
        state as for update_chain_dep_state (updated in place).  Returns (verdict u8[n],
        failures u16[n], chain_stop, processed)."""
        n = len(H["slot"])
        th = TPHeaders()
        th.h = self.headers_struct(H)
        th.leader_out = ptr(H["leader_out"])
        th.leader_proof = ptr(H["leader_proof"])
        to = TPOut()
        to.bits = ptr(crypto["bits"], u16p)
        to.pool_idx = ptr(crypto["pool_idx"], i32p)
        to.nonce = ptr(crypto["nonce"])
        st, hk, cv = _state_struct(state, len(state.get("counters", {})) + n)
        ei = EpochInfo(*epoch_info)
        ph = np.ascontiguousarray(prev_hash, dtype=np.uint8)
        pg = None if prev_is_genesis is None else np.ascontiguousarray(prev_is_genesis, dtype=np.uint8)
        xe = None
        if extra_entropy is not None:
            xe = Nonce()
            ctypes.memmove(xe.hash, bytes(extra_entropy), 32)
        verdict = np.zeros(n, np.uint8)
        fails = np.zeros(n, np.uint16)
        stop, done = ctypes.c_size_t(0), ctypes.c_size_t(0)
        self.check(self.L.praos_tpraos_update_chain_dep_state(
            self.h, ctypes.byref(th), ptr(ph), ptr(pg) if pg is not None else None, ctypes.byref(to), None,
            ctypes.byref(ei), ctypes.byref(xe) if xe is not None else None, ctypes.byref(st), ptr(verdict),
            ptr(fails, u16p), ctypes.byref(stop), ctypes.byref(done)))
        new = _state_from_struct(st, hk, cv)
        state.clear()
        state.update(new)
        return verdict, fails, int(stop.value), int(done.value)

    def upload(self, H):
        hs = self.headers_struct(H)
        b = self.L.praos_batch_upload(self.h, ctypes.byref(hs))
        if not b:
            self.check(-3)
        return b

    def run(self, b):
        self.check(self.L.praos_batch_run(self.h, b))

    def sync(self):
        self.check(self.L.praos_batch_sync(self.h))

    def set_option(self, opt, value):
        self.check(self.L.praos_set_option(self.h, opt, value))

    def batch_stats(self, b):
        """Key-cache statistics of the last run: dict of cold/vrf/kes entries, hits, misses."""
        out = np.zeros(9, np.uint32)
        self.check(self.L.praos_batch_stats(self.h, b, ptr(out, u32p)))
        return {"cold_keys": int(out[0]), "cold_hits": int(out[1]), "cold_misses": int(out[2]),
                "vrf_keys": int(out[3]), "vrf_hits": int(out[4]), "vrf_misses": int(out[5]),
                "kes_keys": int(out[6]), "kes_hits": int(out[7]), "kes_misses": int(out[8])}

    def dedup_stats(self, b):
        """OCert dedup of the last run: distinct OCert tuples verified, headers."""
        out = np.zeros(2, np.uint32)
        self.check(self.L.praos_batch_dedup_stats(self.h, b, ptr(out, u32p)))
        return {"ocert_unique": int(out[0]), "headers": int(out[1])}

    def kernel_ms(self, which):
        return float(self.L.praos_batch_kernel_ms(self.h, which))

    def download(self, b, n, out=None):
        o = self.alloc_out(n) if out is None else out
        os_ = self.out_struct(o)
        self.check(self.L.praos_batch_download(self.h, b, ctypes.byref(os_)))
        return o

    def free(self, b):
        self.L.praos_batch_free(self.h, b)

    # ---- stored header bytes (GPU decode, k_decode.hip) ----
    @staticmethod
    def header_bytes_struct(arena, off, length):
        s = HeaderBytes()
        s.n = len(off)
        s.bytes = ptr(arena)
        s.bytes_len = len(arena)
        s.off = ptr(off, u64p)
        s.len = ptr(length, u32p)
        return s

    @staticmethod
    def alloc_decoded(n, stride=SIGNED_STRIDE):
        D = {name: np.zeros((n,) + (shp if name != "signed_body" else (stride,)), dt)
             for name, dt, shp in DECODED_FIELDS}
        d = Decoded()
        for name, dt, _ in DECODED_FIELDS:
            setattr(d, name, ptr(D[name], _CT[dt]))
        return D, d

    @staticmethod
    def _chunk(arena, off, length):
        return (np.ascontiguousarray(np.frombuffer(arena, np.uint8) if isinstance(arena, (bytes, bytearray))
                                     else arena, dtype=np.uint8),
                np.ascontiguousarray(off, dtype=np.uint64), np.ascontiguousarray(length, dtype=np.uint32))

    def decode_headers(self, arena, off, length):
        """Decode stored Praos headers arena[off[i]:off[i]+len[i]] on the GPU; returns a dict of arrays
        (DECODED_FIELDS)."""
        arena, off, length = self._chunk(arena, off, length)
        hb = self.header_bytes_struct(arena, off, length)
        D, d = self.alloc_decoded(len(off))
        self.check(self.L.praos_decode_headers(self.h, ctypes.byref(hb), ctypes.byref(d)))
        return D

    def verify_header_bytes(self, arena, off, length, decoded=False, out=None):
        """out: caller-owned output arrays (alloc_out) reused across calls."""
        arena, off, length = self._chunk(arena, off, length)
        n = len(off)
        hb = self.header_bytes_struct(arena, off, length)
        o = self.alloc_out(n) if out is None else out
        os_ = self.out_struct(o)
        D, d = self.alloc_decoded(n) if decoded else (None, None)
        self.check(self.L.praos_verify_header_bytes(self.h, ctypes.byref(hb), ctypes.byref(os_),
                                                    ctypes.byref(d) if d is not None else None))
        return (o, D) if decoded else o

    def submit_header_bytes(self, arena, off, length, out, decoded=None):
        """Streaming form of verify_header_bytes (praos_verify_header_bytes_submit): queued, returns
        at once; out (and decoded, an alloc_decoded pair) are written by the third submit after it
        or by drain().  The inputs and outputs stay referenced here until drained."""
        arena, off, length = self._chunk(arena, off, length)
        hb = self.header_bytes_struct(arena, off, length)
        os_ = self.out_struct(out)
        d = decoded[1] if decoded is not None else None
        self.check(self.L.praos_verify_header_bytes_submit(self.h, ctypes.byref(hb), ctypes.byref(os_),
                                                           ctypes.byref(d) if d is not None else None))
        self._inflight = (getattr(self, "_inflight", []) + [(arena, off, length, hb, os_, out, decoded)])[-4:]

    def drain(self):
        """Every submitted call's outputs written (praos_verify_drain)."""
        self.check(self.L.praos_verify_drain(self.h))
        self._inflight = []

    def verify_tpraos_header_bytes(self, arena, off, length, decoded=False):
        """Stored TPraos headers (BHeader = [BHBody, kesSig], Shelley..Alonzo) decoded and
        verified on the GPU (praos_verify_tpraos_header_bytes).  Returns the TPraos outputs
        (bits, pool_idx, beta_eta, beta_leader, nonce); with decoded=True also the decoded
        fields plus leader_out / leader_proof."""
        arena, off, length = self._chunk(arena, off, length)
        n = len(off)
        hb = self.header_bytes_struct(arena, off, length)
        o, to = self.tp_out(n)
        D, d = self.alloc_decoded(n, TP_SIGNED_STRIDE) if decoded else (None, None)
        lo = np.zeros((n, 64), np.uint8) if decoded else None
        lp = np.zeros((n, 80), np.uint8) if decoded else None
        self.check(self.L.praos_verify_tpraos_header_bytes(self.h, ctypes.byref(hb), ctypes.byref(to),
                                                           ctypes.byref(d) if d is not None else None,
                                                           ptr(lo) if decoded else None, ptr(lp) if decoded else None))
        if not decoded:
            return o
        D["leader_out"], D["leader_proof"] = lo, lp
        return o, D

    # ---- stored blocks: verifyBlockIntegrity (k_block.hip) ----
    def verify_block_integrity(self, arena, off, length, slots_per_kes_period):
        """Integrity.hs:14-20 over blocks arena[off[i]:off[i]+len[i]]; returns (result u8[n] of
        PRAOS_BLK_* bits, computed hashTxSeq u8[n,32])."""
        arena, off, length = self._chunk(arena, off, length)
        n = len(off)
        hb = self.header_bytes_struct(arena, off, length)
        res = np.zeros(n, np.uint8)
        bh = np.zeros((n, 32), np.uint8)
        self.check(self.L.praos_verify_block_integrity(self.h, ctypes.byref(hb), slots_per_kes_period, ptr(res),
                                                       ptr(bh)))
        return res, bh

    def upload_blocks(self, arena, off, length):
        arena, off, length = self._chunk(arena, off, length)
        hb = self.header_bytes_struct(arena, off, length)
        b = self.L.praos_block_batch_upload(self.h, ctypes.byref(hb))
        if not b:
            raise RuntimeError("praos_block_batch_upload: " + self.L.praos_last_error(self.h).decode())
        return b

    def run_blocks(self, b, slots_per_kes_period):
        self.check(self.L.praos_block_batch_run(self.h, b, slots_per_kes_period))

    def download_blocks(self, b, n):
        res = np.zeros(n, np.uint8)
        bh = np.zeros((n, 32), np.uint8)
        self.check(self.L.praos_block_batch_download(self.h, b, ptr(res), ptr(bh)))
        return res, bh

    def upload_bytes(self, arena, off, length):
        arena, off, length = self._chunk(arena, off, length)
        hb = self.header_bytes_struct(arena, off, length)
        b = self.L.praos_batch_upload_bytes(self.h, ctypes.byref(hb))
        if not b:
            self.check(-3)
        return b

    def host_register(self, arr):
        """Page-locks a numpy array's memory for this context (praos_host_register): uploads
        from it move by direct DMA.  Keep the array alive until host_unregister."""
        self.check(self.L.praos_host_register(self.h, arr.ctypes.data, arr.nbytes))

    def host_unregister(self, arr):
        self.check(self.L.praos_host_unregister(self.h, arr.ctypes.data))

    def upload_tpraos_bytes(self, arena, off, length):
        """Stored TPraos headers (BHeader) as a resident batch (praos_batch_upload_tpraos_bytes);
        every praos_batch_run decodes them on the device and runs the TPraos kernels."""
        arena, off, length = self._chunk(arena, off, length)
        hb = self.header_bytes_struct(arena, off, length)
        b = self.L.praos_batch_upload_tpraos_bytes(self.h, ctypes.byref(hb))
        if not b:
            self.check(-3)
        return b

    def download_tpraos(self, b, n):
        o = {"bits": np.zeros(n, np.uint16), "pool_idx": np.zeros(n, np.int32),
             "beta_eta": np.zeros((n, 64), np.uint8), "beta_leader": np.zeros((n, 64), np.uint8),
             "nonce": np.zeros((n, 32), np.uint8)}
        to = TPOut()
        to.bits, to.pool_idx = ptr(o["bits"], u16p), ptr(o["pool_idx"], i32p)
        to.beta_eta, to.beta_leader, to.nonce = ptr(o["beta_eta"]), ptr(o["beta_leader"]), ptr(o["nonce"])
        self.check(self.L.praos_batch_download_tpraos(self.h, b, ctypes.byref(to)))
        return o

    def batch_decode(self, b):
        self.check(self.L.praos_batch_decode(self.h, b))

    @staticmethod
    def nonce_array(etas):
        arr = (Nonce * max(1, len(etas)))()
        for k, e in enumerate(etas):
            arr[k].neutral = int(e is None)
            if e is not None:
                ctypes.memmove(arr[k].hash, bytes(e), 32)
        return arr

    def set_nonces(self, b, etas, eta_idx):
        """praos_batch_set_nonces: header i of batch b is verified under etas[eta_idx[i]]
        (None = NeutralNonce)."""
        idx = np.ascontiguousarray(eta_idx, dtype=np.uint8)
        self.check(self.L.praos_batch_set_nonces(self.h, b, self.nonce_array(etas), len(etas), ptr(idx)))

    def download_decoded(self, b, n):
        D, d = self.alloc_decoded(n)
        self.check(self.L.praos_batch_download_decoded(self.h, b, ctypes.byref(d)))
        return D

    def update_chain_dep_state(self, H, crypto, prev_hash, state: dict, epoch_info, prev_is_genesis=None,
                               envelope=None, etas=None, eta_idx=None):
        """state: dict(last_slot (None = Origin), counters {hash28: n}, evolving, candidate, epoch_nonce,
        lab, leb) with nonces None (Neutral) or 32 bytes; updated in place.  epoch_info: (base_slot,
        base_no, length, stability_window).  envelope (praos_validate_headers): dict(block_no u64[n],
        header_hash u8[n,32], header_size u32[n], body_size u32[n], tip (None = Origin, or (slot,
        block_no, hash32)), max_major_pv, lv_prot_major, max_header_size, max_body_size); its "tip" is
        updated in place.  etas / eta_idx: the per-header nonces the crypto ran under
        (praos_validate_headers_nonces).  Returns (verdict u8[n], chain_stop, processed)."""
        n = len(H["slot"])
        hs = self.headers_struct(H)
        os_ = self.out_struct(crypto)
        keys = list(state["counters"].keys())
        cap = len(keys) + n
        hk = np.zeros(28 * max(cap, 1), np.uint8)
        cv = np.zeros(max(cap, 1), np.uint64)
        for k, key in enumerate(keys):
            hk[28 * k:28 * k + 28] = np.frombuffer(key, np.uint8)
            cv[k] = state["counters"][key]
        st = ChainState()
        st.last_slot_origin = int(state["last_slot"] is None)
        st.last_slot = state["last_slot"] or 0
        st.counter_hash28, st.counter, st.m, st.cap = ptr(hk), ptr(cv, u64p), len(keys), cap

        def setn(dst, v):
            dst.neutral = int(v is None)
            if v is not None:
                ctypes.memmove(dst.hash, v, 32)

        def getn(src):
            return None if src.neutral else bytes(src.hash)
        for a, b in (("evolving", "evolving"), ("candidate", "candidate"), ("epoch_nonce", "epoch_nonce"),
                     ("lab", "lab"), ("last_epoch_block", "leb")):
            setn(getattr(st, a), state[b])
        ei = EpochInfo(*epoch_info)
        ph = np.ascontiguousarray(prev_hash, dtype=np.uint8)
        pg = None if prev_is_genesis is None else np.ascontiguousarray(prev_is_genesis, dtype=np.uint8)
        verdict = np.zeros(n, np.uint8)
        stop, done = ctypes.c_size_t(0), ctypes.c_size_t(0)
        E = None
        if envelope is not None:
            E = Envelope()
            arrs = {k: np.ascontiguousarray(envelope[k], dtype=dt) for k, dt in
                    (("block_no", np.uint64), ("header_hash", np.uint8), ("header_size", np.uint32),
                     ("body_size", np.uint32))}
            E.block_no, E.header_hash = ptr(arrs["block_no"], u64p), ptr(arrs["header_hash"])
            E.header_size, E.body_size = ptr(arrs["header_size"], u32p), ptr(arrs["body_size"], u32p)
            tip = envelope["tip"]
            E.tip_is_origin = int(tip is None)
            if tip is not None:
                E.tip_slot, E.tip_block_no = tip[0], tip[1]
                ctypes.memmove(E.tip_hash, bytes(tip[2]), 32)
            for k in ("max_major_pv", "lv_prot_major", "max_header_size", "max_body_size"):
                setattr(E, k, envelope[k])
        if etas is not None:
            idx = np.ascontiguousarray(eta_idx, dtype=np.uint8)
            self.check(self.L.praos_validate_headers_nonces(
                self.h, ctypes.byref(hs), ptr(ph), ptr(pg) if pg is not None else None, ctypes.byref(os_),
                ctypes.byref(E) if E is not None else None, ctypes.byref(ei), ctypes.byref(st),
                self.nonce_array(etas), len(etas), ptr(idx), ptr(verdict), ctypes.byref(stop), ctypes.byref(done)))
            if envelope is not None:
                envelope["tip"] = None if E.tip_is_origin else (int(E.tip_slot), int(E.tip_block_no),
                                                                bytes(E.tip_hash))
        elif envelope is None:
            self.check(self.L.praos_update_chain_dep_state(self.h, ctypes.byref(hs), ptr(ph),
                                                           ptr(pg) if pg is not None else None, ctypes.byref(os_),
                                                           ctypes.byref(ei), ctypes.byref(st), ptr(verdict),
                                                           ctypes.byref(stop), ctypes.byref(done)))
        else:
            E = Envelope()
            arrs = {k: np.ascontiguousarray(envelope[k], dtype=dt) for k, dt in
                    (("block_no", np.uint64), ("header_hash", np.uint8), ("header_size", np.uint32),
                     ("body_size", np.uint32))}
            E.block_no, E.header_hash = ptr(arrs["block_no"], u64p), ptr(arrs["header_hash"])
            E.header_size, E.body_size = ptr(arrs["header_size"], u32p), ptr(arrs["body_size"], u32p)
            tip = envelope["tip"]
            E.tip_is_origin = int(tip is None)
            if tip is not None:
                E.tip_slot, E.tip_block_no = tip[0], tip[1]
                ctypes.memmove(E.tip_hash, bytes(tip[2]), 32)
            for k in ("max_major_pv", "lv_prot_major", "max_header_size", "max_body_size"):
                setattr(E, k, envelope[k])
            self.check(self.L.praos_validate_headers(self.h, ctypes.byref(hs), ptr(ph),
                                                     ptr(pg) if pg is not None else None, ctypes.byref(os_),
                                                     ctypes.byref(E), ctypes.byref(ei), ctypes.byref(st),
                                                     ptr(verdict), ctypes.byref(stop), ctypes.byref(done)))
            envelope["tip"] = None if E.tip_is_origin else (int(E.tip_slot), int(E.tip_block_no), bytes(E.tip_hash))
        state["last_slot"] = None if st.last_slot_origin else int(st.last_slot)
        state["counters"] = {bytes(hk[28 * k:28 * k + 28]): int(cv[k]) for k in range(st.m)}
        for a, b in (("evolving", "evolving"), ("candidate", "candidate"), ("epoch_nonce", "epoch_nonce"),
                     ("lab", "lab"), ("last_epoch_block", "leb")):
            state[b] = getn(getattr(st, a))
        return verdict, stop.value, done.value

    def replay_immutable(self, path, pools, params: Params, epoch_info, state: dict, envelope: dict,
                         batch_max=1 << 16, verdicts_cap=0, counter_cap=1 << 16, tpraos=False, extra_entropy=None):
        """praos_replay_immutable over an ImmutableDB directory.  state (chain state dict, as
        update_chain_dep_state) and envelope (limits + "tip") are updated in place.
        Returns (stats dict, verdict u8[verdicts_cap]); tpraos=True (praos_replay_immutable_tpraos,
        extra_entropy None = NeutralNonce) returns (stats, verdict, failures u16[verdicts_cap])."""
        fn = self.L.praos_replay_immutable_tpraos if tpraos else self.L.praos_replay_immutable
        return _replay(fn, self.h, self.check, path, pools, params, epoch_info, state, envelope, batch_max,
                       verdicts_cap, counter_cap, tpraos, extra_entropy)

    def replay_immutable_views(self, path, views, params: Params, epoch_info, state: dict, envelope: dict,
                               batch_max=1 << 16, verdicts_cap=0, counter_cap=1 << 16):
        """praos_replay_immutable_views: views = [(first_epoch, pools, {lv_prot_major, max_header_size,
        max_body_size})] sorted by first_epoch, a ledger view per epoch range; otherwise as
        replay_immutable (envelope's limits are not read)."""
        return _replay_views(self.L.praos_replay_immutable_views, self.h, self.check, path, views, params, epoch_info,
                             state, envelope, batch_max, verdicts_cap, counter_cap)

    def apply_batch(self, H, crypto, counters=None):
        """counters: dict hash28 -> int.  Returns (verdict u8[n], chain_stop, counters_out)."""
        n = len(H["slot"])
        hs = self.headers_struct(H)
        os_ = self.out_struct(crypto)
        verdict = np.zeros(n, np.uint8)
        stop = ctypes.c_size_t(0)
        cs = None
        keys = list(counters.keys()) if counters else []
        hk = np.frombuffer(b"".join(keys), dtype=np.uint8).copy() if keys else np.zeros(28, np.uint8)
        cv = np.array([counters[k] for k in keys], dtype=np.uint64) if keys else np.zeros(1, np.uint64)
        if counters is not None:
            cs = Counters()
            cs.hash28 = ptr(hk)
            cs.counter = ptr(cv, u64p)
            cs.m = len(keys)
        self.check(self.L.praos_apply_batch(self.h, ctypes.byref(hs), ctypes.byref(os_),
                                            ctypes.byref(cs) if cs is not None else None, ptr(verdict),
                                            ctypes.byref(stop)))
        out_counters = {k: int(cv[i]) for i, k in enumerate(keys)}
        return verdict, stop.value, out_counters

    # ---- single primitives ----
    def verify_ocert(self, cold_vk, hot_vk, n_arr, c0_arr, sig):
        n = len(n_arr)
        ok = np.zeros(n, np.uint8)
        self.check(self.L.praos_verify_ocert(self.h, n, ptr(cold_vk), ptr(hot_vk), ptr(n_arr, u64p),
                                             ptr(c0_arr, u64p), ptr(sig), ptr(ok)))
        return ok

    def verify_kes(self, vk, period, sig, msgs):
        n = len(period)
        lens = np.array([len(m) for m in msgs], dtype=np.uint32)
        offs = np.zeros(n, np.uint64)
        if n > 1:
            offs[1:] = np.cumsum(lens[:-1].astype(np.uint64))
        blob = np.frombuffer(b"".join(msgs) + b"\0" * 8, dtype=np.uint8).copy()
        res = np.zeros(n, np.uint8)
        self.check(self.L.praos_verify_kes(self.h, n, ptr(vk), ptr(period, u32p), ptr(sig), ptr(offs, u64p),
                                           ptr(lens, u32p), ptr(blob), len(blob) - 8, ptr(res)))
        return res

    def verify_vrf(self, vk, proof, alpha):
        n = len(vk)
        ok = np.zeros(n, np.uint8)
        beta = np.zeros((n, 64), np.uint8)
        self.check(self.L.praos_verify_vrf(self.h, n, ptr(vk), ptr(proof), ptr(alpha), ptr(ok), ptr(beta)))
        return ok, beta

    def check_leader(self, leader_be, sigma_fp, params: Params):
        n = len(leader_be)
        res = np.zeros(n, np.uint8)
        self.check(self.L.praos_check_leader(self.h, n, ptr(leader_be), ptr(sigma_fp), ctypes.byref(params),
                                             ptr(res)))
        return res

    def leader_schedule(self, seed: bytes, sigma_fp, params: Params, eta0, first_slot, nslots, tpraos=False):
        """First-leader-wins forger per slot (praos_leader_schedule): int32[nslots], -1 = empty slot.
        sigma_fp: per-pool Fixed E34 stake (ints), in forger order."""
        npools = len(sigma_fp)
        sig = np.frombuffer(b"".join(int(x).to_bytes(16, "little") for x in sigma_fp), np.uint8).copy()
        sd = np.frombuffer(bytes(seed), np.uint8).copy()
        e = None if eta0 is None else np.frombuffer(bytes(eta0), np.uint8).copy()
        out = np.zeros(nslots, np.int32)
        self.check(self.L.praos_leader_schedule(self.h, ptr(sd), npools, ptr(sig), ctypes.byref(params), ptr(e),
                                                first_slot, nslots, int(bool(tpraos)), ptr(out, i32p)))
        return out

    def synthesize(self, n, npools, params: Params, eta0, seed: bytes, first_slot=0, slot_stride=20,
                   body_len=397, corrupt_per_10000=0, nkes=0, tpraos=False, body_hash=None, schedule=None,
                   block_no0=0, link=False, prev0=None, corrupt_fields=0):
        """schedule: (slots u64[n], pools u32[n]) from leader_schedule (a leader-valid chain), or None
        (evenly spaced slots, pools by hash: not leader-valid).  link=True chains the headers
        (prevHash = headerHash of the previous header; header 0: prev0, None = GenesisHash) and
        returns the header hashes in H["header_hash"]."""
        sp = SynthParams()
        if link:
            hh_out = np.zeros((n, 32), np.uint8)
            sp.link_prev, sp.header_hash = 1, ptr(hh_out)
            if prev0 is not None:
                p0 = np.frombuffer(bytes(prev0), np.uint8).copy()
                sp.prev0 = ptr(p0)
        if body_hash is not None:   # n*32 hbBodyHash values for the CBOR bodies (body_len=0)
            body_hash = np.ascontiguousarray(body_hash, dtype=np.uint8).reshape(n, 32)
            sp.body_hash = ptr(body_hash)
        if schedule is not None:
            ss = np.ascontiguousarray(schedule[0], dtype=np.uint64)
            sq = np.ascontiguousarray(schedule[1], dtype=np.uint32)
            assert len(ss) == n and len(sq) == n
            sp.sched_slot, sp.sched_pool, sp.block_no0 = ptr(ss, u64p), ptr(sq, u32p), block_no0
        sp.n = n
        sp.npools = npools
        sp.first_slot = first_slot
        sp.slot_stride = slot_stride
        sp.body_len = body_len
        sp.corrupt_per_10000 = corrupt_per_10000
        sp.corrupt_fields = corrupt_fields
        sp.nkes = nkes
        ctypes.memmove(sp.seed, seed, 32)
        bstride = (body_len + 7) & ~7 if body_len else (TP_SIGNED_STRIDE if tpraos else SIGNED_STRIDE)
        H = {"slot": np.zeros(n, np.uint64), "cold_vk": np.zeros((n, 32), np.uint8),
             "vrf_vk": np.zeros((n, 32), np.uint8), "vrf_out": np.zeros((n, 64), np.uint8),
             "vrf_proof": np.zeros((n, 80), np.uint8), "hot_vk": np.zeros((n, 32), np.uint8),
             "ocert_n": np.zeros(n, np.uint64), "ocert_c0": np.zeros(n, np.uint64),
             "ocert_sig": np.zeros((n, 64), np.uint8), "kes_sig": np.zeros((n, 448), np.uint8),
             "body_off": np.zeros(n, np.uint64), "body_len": np.zeros(n, np.uint32),
             "body_bytes": np.zeros(bstride * n + 8, np.uint8)}
        corrupted = np.zeros(n, np.uint8)
        pools = (Pool * npools)()
        e = None
        if eta0 is not None:
            eb = np.frombuffer(bytes(eta0), dtype=np.uint8).copy()
            e = ptr(eb)
        common = (self.h, ctypes.byref(sp), ctypes.byref(params), e, pools, ptr(H["slot"], u64p), ptr(H["cold_vk"]),
                  ptr(H["vrf_vk"]), ptr(H["vrf_out"]), ptr(H["vrf_proof"]), ptr(H["hot_vk"]),
                  ptr(H["ocert_n"], u64p), ptr(H["ocert_c0"], u64p), ptr(H["ocert_sig"]), ptr(H["kes_sig"]),
                  ptr(H["body_off"], u64p), ptr(H["body_len"], u32p), ptr(H["body_bytes"]))
        if tpraos:
            H["leader_out"] = np.zeros((n, 64), np.uint8)
            H["leader_proof"] = np.zeros((n, 80), np.uint8)
            self.check(self.L.praos_synthesize_tpraos(*common, ptr(H["leader_out"]), ptr(H["leader_proof"]),
                                                      ptr(corrupted)))
        else:
            self.check(self.L.praos_synthesize(*common, ptr(corrupted)))
        H["body_bytes"] = H["body_bytes"][:bstride * n]
        if link:
            H["header_hash"] = hh_out
        pool_list = [(bytes(p.hash28), bytes(p.vrf_hash32)) for p in pools]
        return H, pool_list, corrupted

    # ---- self tests ----
    def debug_fe(self, op, a, b=None):
        n = len(a)
        r = np.zeros((n, 32), np.uint8)
        self.check(self.L.praos_debug_fe(self.h, op, n, ptr(a), ptr(b if b is not None else a), ptr(r)))
        return r

    def debug_sha512(self, prefix, msgs):
        n = len(msgs)
        lens = np.array([len(m) for m in msgs], dtype=np.uint32)
        offs = np.zeros(n, np.uint64)
        if n > 1:
            offs[1:] = np.cumsum(lens[:-1].astype(np.uint64))
        blob = np.frombuffer(b"".join(msgs) + b"\0" * 8, dtype=np.uint8).copy()
        out = np.zeros((n, 64), np.uint8)
        self.check(self.L.praos_debug_sha512(self.h, n, ptr(prefix), ptr(offs, u64p), ptr(lens, u32p), ptr(blob),
                                             len(blob) - 8, ptr(out)))
        return out

    def debug_blake2b(self, in64):
        out = np.zeros((len(in64), 32), np.uint8)
        self.check(self.L.praos_debug_blake2b(self.h, len(in64), ptr(in64), ptr(out)))
        return out

    def debug_sc_reduce(self, in64):
        out = np.zeros((len(in64), 32), np.uint8)
        self.check(self.L.praos_debug_sc_reduce(self.h, len(in64), ptr(in64), ptr(out)))
        return out

    def debug_decode(self, in32):
        n = len(in32)
        out = np.zeros((n, 32), np.uint8)
        ok = np.zeros(n, np.uint8)
        self.check(self.L.praos_debug_decode(self.h, n, ptr(in32), ptr(out), ptr(ok)))
        return out, ok

    def debug_scalarmult_base(self, s):
        out = np.zeros((len(s), 32), np.uint8)
        self.check(self.L.praos_debug_scalarmult_base(self.h, len(s), ptr(s), ptr(out)))
        return out

    def debug_leader(self, leader_be, x_raw16):
        n = len(leader_be)
        res = np.zeros(n, np.uint8)
        it = np.zeros(n, np.int32)
        self.check(self.L.praos_debug_leader(self.h, n, ptr(leader_be), ptr(x_raw16), ptr(res), ptr(it, i32p)))
        return res, it

    def debug_leader512(self, leader_be64, x_raw16):
        n = len(leader_be64)
        res = np.zeros(n, np.uint8)
        it = np.zeros(n, np.int32)
        self.check(self.L.praos_debug_leader512(self.h, n, ptr(leader_be64), ptr(x_raw16), ptr(res), ptr(it, i32p)))
        return res, it

    def debug_hash_to_curve(self, pk, alpha):
        out = np.zeros((len(pk), 32), np.uint8)
        self.check(self.L.praos_debug_hash_to_curve(self.h, len(pk), ptr(pk), ptr(alpha), ptr(out)))
        return out


class Group:
    """praos_group: one context per listed device (repeats allowed), batches split into
    contiguous shards run concurrently, outputs gathered in place (include/praos_hip.h)."""

    def __init__(self, devices):
        self.L = load()
        arr = np.ascontiguousarray(devices, dtype=np.int32)
        self.g = self.L.praos_group_open(ptr(arr, i32p), len(arr))
        if not self.g:
            raise PraosError(f"praos_group_open({list(devices)}) failed")
        self.size = self.L.praos_group_size(self.g)

    def close(self):
        if self.g:
            self.L.praos_group_close(self.g)
            self.g = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def check(self, rc):
        if rc != 0:
            msg = self.L.praos_group_last_error(self.g)
            raise PraosError(f"praos group rc={rc}: {msg.decode() if msg else ''}")

    def member(self, k):
        """A Context view of member k (not owned: closing the group closes it)."""
        c = Context.__new__(Context)
        c.L, c.h, c._keep = self.L, self.L.praos_group_ctx(self.g, k), []
        return c

    def set_option(self, opt, value):
        self.check(self.L.praos_group_set_option(self.g, opt, value))

    def set_epoch(self, eta0, pools, params: Params):
        arr = Context.pool_array(pools)
        e = None
        if eta0 is not None:
            eb = np.frombuffer(bytes(eta0), dtype=np.uint8).copy()
            e = ptr(eb)
        self.check(self.L.praos_group_set_epoch(self.g, e, arr, len(pools), ctypes.byref(params)))

    def verify_headers(self, H):
        n = len(H["slot"])
        hs = Context.headers_struct(H)
        o = Context.alloc_out(n)
        os_ = Context.out_struct(o)
        self.check(self.L.praos_group_verify_headers(self.g, ctypes.byref(hs), ctypes.byref(os_)))
        return o

    def verify_header_bytes(self, arena, off, length, decoded=False):
        arena, off, length = Context._chunk(arena, off, length)
        n = len(off)
        hb = Context.header_bytes_struct(arena, off, length)
        o = Context.alloc_out(n)
        os_ = Context.out_struct(o)
        D, d = Context.alloc_decoded(n) if decoded else (None, None)
        self.check(self.L.praos_group_verify_header_bytes(self.g, ctypes.byref(hb), ctypes.byref(os_),
                                                          ctypes.byref(d) if decoded else None))
        return (o, D) if decoded else o

    def verify_tpraos_headers(self, H):
        th = Context.tp_headers_struct(H)
        o, to = Context.tp_out(len(H["slot"]))
        self.check(self.L.praos_group_verify_tpraos_headers(self.g, ctypes.byref(th), ctypes.byref(to)))
        return o

    def set_overlay(self, d, f, epoch_base_slot, epoch_length, gen_delegs):
        """praos_group_set_overlay (Context.set_overlay on every member)."""
        if d is None:
            self.check(self.L.praos_group_set_overlay(self.g, None))
            return
        arr = (GenDeleg * max(1, len(gen_delegs)))()
        for k, (g, dl, v) in enumerate(gen_delegs):
            ctypes.memmove(arr[k].genesis_hash28, bytes(g), 28)
            ctypes.memmove(arr[k].delegate_hash28, bytes(dl), 28)
            ctypes.memmove(arr[k].vrf_hash32, bytes(v), 32)
        ov = Overlay(d.numerator, d.denominator, f.numerator, f.denominator, epoch_base_slot, epoch_length,
                     ctypes.cast(arr, ctypes.POINTER(GenDeleg)), len(gen_delegs))
        self.check(self.L.praos_group_set_overlay(self.g, ctypes.byref(ov)))

    def host_register(self, a):
        """praos_group_host_register: page-lock a numpy array once for every member."""
        assert a.flags["C_CONTIGUOUS"] and a.nbytes > 0
        self.check(self.L.praos_group_host_register(self.g, a.ctypes.data, a.nbytes))

    def host_unregister(self, a):
        self.check(self.L.praos_group_host_unregister(self.g, a.ctypes.data))

    def replay_immutable(self, path, pools, params: Params, epoch_info, state: dict, envelope: dict,
                         batch_max=1 << 16, verdicts_cap=0, counter_cap=1 << 16, tpraos=False, extra_entropy=None):
        """praos_group_replay_immutable[_tpraos]: Context.replay_immutable over the group's members."""
        fn = self.L.praos_group_replay_immutable_tpraos if tpraos else self.L.praos_group_replay_immutable
        return _replay(fn, self.g, self.check, path, pools, params, epoch_info, state, envelope, batch_max,
                       verdicts_cap, counter_cap, tpraos, extra_entropy)

    def verify_block_integrity(self, arena, off, length, slots_per_kes_period):
        """praos_group_verify_block_integrity: Context.verify_block_integrity sharded over the members."""
        arena, off, length = Context._chunk(arena, off, length)
        n = len(off)
        hb = Context.header_bytes_struct(arena, off, length)
        res = np.zeros(n, np.uint8)
        bh = np.zeros((n, 32), np.uint8)
        self.check(self.L.praos_group_verify_block_integrity(self.g, ctypes.byref(hb), slots_per_kes_period,
                                                             ptr(res), ptr(bh)))
        return res, bh

    def replay_immutable_views(self, path, views, params: Params, epoch_info, state: dict, envelope: dict,
                               batch_max=1 << 16, verdicts_cap=0, counter_cap=1 << 16):
        """praos_group_replay_immutable_views: Context.replay_immutable_views over the group's members."""
        return _replay_views(self.L.praos_group_replay_immutable_views, self.g, self.check, path, views, params,
                             epoch_info, state, envelope, batch_max, verdicts_cap, counter_cap)

    def verify_tpraos_header_bytes(self, arena, off, length, decoded=False):
        arena, off, length = Context._chunk(arena, off, length)
        n = len(off)
        hb = Context.header_bytes_struct(arena, off, length)
        o, to = Context.tp_out(n)
        D, d = Context.alloc_decoded(n, TP_SIGNED_STRIDE) if decoded else (None, None)
        lo = np.zeros((n, 64), np.uint8) if decoded else None
        lp = np.zeros((n, 80), np.uint8) if decoded else None
        self.check(self.L.praos_group_verify_tpraos_header_bytes(self.g, ctypes.byref(hb), ctypes.byref(to),
                                                                 ctypes.byref(d) if decoded else None,
                                                                 ptr(lo) if decoded else None,
                                                                 ptr(lp) if decoded else None))
        if not decoded:
            return o
        D["leader_out"], D["leader_proof"] = lo, lp
        return o, D


def _replay(fn, handle, check, path, pools, params, epoch_info, state, envelope, batch_max, verdicts_cap, counter_cap,
            tpraos, extra_entropy):
    """praos_[group_]replay_immutable[_tpraos] (the same arguments after the context / group)."""
    arr = Context.pool_array(pools)
    st, hk, cv = _state_struct(state, counter_cap)
    E = Envelope()
    tip = envelope.get("tip")
    E.tip_is_origin = int(tip is None)
    if tip is not None:
        E.tip_slot, E.tip_block_no = tip[0], tip[1]
        ctypes.memmove(E.tip_hash, bytes(tip[2]), 32)
    for k in ("max_major_pv", "lv_prot_major", "max_header_size", "max_body_size"):
        setattr(E, k, envelope[k])
    ei = EpochInfo(*epoch_info)
    verdict = np.zeros(max(verdicts_cap, 1), np.uint8)
    fails = np.zeros(max(verdicts_cap, 1), np.uint16)
    S = ReplayStats()
    if tpraos:
        xe = None
        if extra_entropy is not None:
            xe = Nonce()
            ctypes.memmove(xe.hash, bytes(extra_entropy), 32)
        check(fn(handle, os.fsencode(str(path)), arr, len(pools), ctypes.byref(params), ctypes.byref(ei),
                 ctypes.byref(xe) if xe is not None else None, ctypes.byref(E), ctypes.byref(st), batch_max,
                 ptr(verdict), ptr(fails, u16p), verdicts_cap, ctypes.byref(S)))
    else:
        check(fn(handle, os.fsencode(str(path)), arr, len(pools), ctypes.byref(params), ctypes.byref(ei),
                 ctypes.byref(E), ctypes.byref(st), batch_max, ptr(verdict), verdicts_cap, ctypes.byref(S)))
    envelope["tip"] = None if E.tip_is_origin else (int(E.tip_slot), int(E.tip_block_no), bytes(E.tip_hash))
    state.update(_state_from_struct(st, hk, cv))
    stats = {name: getattr(S, name) for name, _ in ReplayStats._fields_}
    if tpraos:
        return stats, verdict[:verdicts_cap], fails[:verdicts_cap]
    return stats, verdict[:verdicts_cap]


def _replay_views(fn, handle, check, path, views, params, epoch_info, state, envelope, batch_max, verdicts_cap,
                  counter_cap):
    """praos_[group_]replay_immutable_views (the same arguments after the context / group)."""
    keep = [Context.pool_array(pools) for _, pools, _ in views]
    V = (LedgerView * max(1, len(views)))()
    for j, (first, pools, lim) in enumerate(views):
        V[j].first_epoch = first
        V[j].pools = ctypes.cast(keep[j], ctypes.c_void_p)
        V[j].npools = len(pools)
        V[j].lv_prot_major = lim["lv_prot_major"]
        V[j].max_header_size = lim["max_header_size"]
        V[j].max_body_size = lim["max_body_size"]
    st, hk, cv = _state_struct(state, counter_cap)
    E = Envelope()
    tip = envelope.get("tip")
    E.tip_is_origin = int(tip is None)
    if tip is not None:
        E.tip_slot, E.tip_block_no = tip[0], tip[1]
        ctypes.memmove(E.tip_hash, bytes(tip[2]), 32)
    E.max_major_pv = envelope["max_major_pv"]
    ei = EpochInfo(*epoch_info)
    verdict = np.zeros(max(verdicts_cap, 1), np.uint8)
    S = ReplayStats()
    check(fn(handle, os.fsencode(str(path)), V, len(views), ctypes.byref(params), ctypes.byref(ei), ctypes.byref(E),
             ctypes.byref(st), batch_max, ptr(verdict), verdicts_cap, ctypes.byref(S)))
    envelope["tip"] = None if E.tip_is_origin else (int(E.tip_slot), int(E.tip_block_no), bytes(E.tip_hash))
    state.update(_state_from_struct(st, hk, cv))
    stats = {name: getattr(S, name) for name, _ in ReplayStats._fields_}
    return stats, verdict[:verdicts_cap]


def _state_struct(state, cap):
    st = ChainState()
    counters = state.get("counters", {})
    keys = list(counters.keys())
    hk = np.zeros(28 * max(cap, 1), np.uint8)
    cv = np.zeros(max(cap, 1), np.uint64)
    if keys:
        hk[:28 * len(keys)] = np.frombuffer(b"".join(keys), np.uint8)
        cv[:len(keys)] = np.fromiter((counters[k] for k in keys), np.uint64, count=len(keys))
    st.last_slot_origin = int(state.get("last_slot") is None)
    st.last_slot = state.get("last_slot") or 0
    st.counter_hash28, st.counter, st.m, st.cap = ptr(hk), ptr(cv, u64p), len(keys), cap
    for a, b in (("evolving", "evolving"), ("candidate", "candidate"), ("epoch_nonce", "epoch_nonce"),
                 ("lab", "lab"), ("last_epoch_block", "leb")):
        v = state.get(b)
        getattr(st, a).neutral = int(v is None)
        if v is not None:
            ctypes.memmove(getattr(st, a).hash, v, 32)
    return st, hk, cv


def state_encode(state):
    """PraosState CBOR (praos_state_encode, Praos.hs:274-310) of a state dict (the form
    Context.update_chain_dep_state uses)."""
    L = load()
    st, hk, cv = _state_struct(state, len(state.get("counters", {})))
    n = ctypes.c_size_t(0)
    L.praos_state_encode(ctypes.byref(st), None, 0, ctypes.byref(n))
    out = np.zeros(max(n.value, 1), np.uint8)
    rc = L.praos_state_encode(ctypes.byref(st), ptr(out), n.value, ctypes.byref(n))
    if rc != 0:
        raise PraosError(f"praos_state_encode rc={rc}")
    return bytes(out[:n.value])


def _state_from_struct(st, hk, cv):
    hb = hk[:28 * st.m].tobytes()
    state = {"last_slot": None if st.last_slot_origin else int(st.last_slot),
             "counters": {hb[28 * k:28 * k + 28]: v for k, v in enumerate(cv[:st.m].tolist())}}
    for a, b in (("evolving", "evolving"), ("candidate", "candidate"), ("epoch_nonce", "epoch_nonce"),
                 ("lab", "lab"), ("last_epoch_block", "leb")):
        x = getattr(st, a)
        state[b] = None if x.neutral else bytes(x.hash)
    return state


def ticked_epoch_nonce(state, epoch_info, slot):
    """praos_ticked_epoch_nonce: the epoch nonce at `slot` (None = NeutralNonce)."""
    L = load()
    st, hk, cv = _state_struct(state, len(state.get("counters", {})))
    out = Nonce()
    rc = L.praos_ticked_epoch_nonce(ctypes.byref(st), ctypes.byref(EpochInfo(*epoch_info)), slot, ctypes.byref(out))
    if rc != 0:
        raise PraosError(f"praos_ticked_epoch_nonce rc={rc}")
    return None if out.neutral else bytes(out.hash)


def state_decode(data: bytes, cap=1 << 16):
    L = load()
    st, hk, cv = _state_struct({}, cap)
    buf = np.frombuffer(bytes(data), np.uint8).copy()
    rc = L.praos_state_decode(ptr(buf), len(buf), ctypes.byref(st))
    if rc != 0:
        raise PraosError(f"praos_state_decode rc={rc}")
    return _state_from_struct(st, hk, cv)


def params(slots_per_kes_period=129600, max_kes_evo=62, c_raw=0, f_is_one=False, vrf_check_output=True):
    p = Params()
    p.slots_per_kes_period = slots_per_kes_period
    p.max_kes_evo = max_kes_evo
    p.f_is_one = int(bool(f_is_one))
    p.vrf_check_output = int(bool(vrf_check_output))
    ctypes.memmove(p.c_raw, (int(c_raw) & ((1 << 128) - 1)).to_bytes(16, "little"), 16)
    return p
