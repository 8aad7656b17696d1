"""CPU: libpraos_hip.so loads without a GPU and exports every entry point that
include/praos_hip.h declares; the Python binding covers all of them; context
creation fails loudly (no silent CPU fallback) when no device is present."""
import ctypes
import os
import re

import pytest


def _declared():
    from praos_hip import abi
    src = open(abi.HEADER_PATH).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set(re.findall(r"\b(praos_[a-z0-9_]+)\s*\(", src))
    return names


def test_header_declares_expected_surface():
    names = _declared()
    for n in ("praos_open", "praos_set_epoch", "praos_verify_headers", "praos_verify_ocert", "praos_verify_kes",
              "praos_verify_vrf", "praos_check_leader", "praos_apply_batch", "praos_synthesize",
              "praos_batch_upload", "praos_batch_run"):
        assert n in names


def test_library_exports_every_declared_symbol():
    from praos_hip import abi
    lib = ctypes.CDLL(abi.LIB_PATH)
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_covers_header():
    from praos_hip import abi
    assert _declared() == set(abi.SIGNATURES)


def test_struct_sizes_match_c_layout():
    from praos_hip import abi
    assert ctypes.sizeof(abi.Params) == 40
    assert ctypes.sizeof(abi.Pool) == 76
    assert ctypes.sizeof(abi.Headers) == 15 * 8
    assert ctypes.sizeof(abi.HeaderBytes) == 5 * 8
    assert ctypes.sizeof(abi.Decoded) == 21 * 8


def test_abi_version():
    from praos_hip import abi
    assert abi.load().praos_abi_version() == 6


def test_no_silent_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from praos_hip import abi
    with pytest.raises(abi.PraosError):
        abi.Context(0)
