"""Host check of the binary-GCD field inversion (csrc/fe_inv_gcd.hpp).

The header is plain integer C++, so the exact text the kernels include is compiled here with
g++ (FEG_INLINE = static inline) and run over random and structured inputs; each result times
2^(-30 k) (k = the iterations run) must be y^-1 mod p (0 for y = 0), and the GCD must end within
its 17 x 30 steps (the kernels' Fermat fallback, taken when it does not, is then never needed).
The GPU-side form is compared with Fermat's chain in tests/test_gpu_primitives.py::test_fe_invert_gcd_vs_fermat.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

P = 2**255 - 19
HDR = os.path.join(os.path.dirname(__file__), "..", "ouroboros-consensus_amd", "csrc")

SHIM = r"""
#define FEG_INLINE static inline
#define FEG_ALL(x) (x)
#include "fe_inv_gcd.hpp"
extern "C" void feg_batch(long n, const uint32_t* in, uint32_t* out, uint8_t* ok, int32_t* iters) {
  for (long i = 0; i < n; i++) ok[i] = feg_core(out + 8 * i, in + 8 * i, iters + i) ? 1 : 0;
}
"""


@pytest.fixture(scope="module", params=["-DFEG_INNER32=0", "-DFEG_INNER32=1", "-DFEG_INNER_MASK=1"],
                ids=["inner64", "inner32", "inner_mask"])
def lib(tmp_path_factory, request):
    d = tmp_path_factory.mktemp("feg")
    src = d / "shim.cpp"
    src.write_text(SHIM)
    so = d / "libfeg.so"
    subprocess.run(["g++", "-O2", "-shared", "-fPIC", request.param, "-I", os.path.abspath(HDR),
                    str(src), "-o", str(so)],
                   check=True)
    L = ctypes.CDLL(str(so))
    L.feg_batch.argtypes = [ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    return L


def _to_words(vals):
    w = np.zeros((len(vals), 8), dtype=np.uint32)
    for i, v in enumerate(vals):
        for k in range(8):
            w[i, k] = (v >> (32 * k)) & 0xFFFFFFFF
    return w


def _from_words(w):
    return [sum(int(w[i, k]) << (32 * k) for k in range(8)) for i in range(w.shape[0])]


def _run(lib, vals):
    inp = _to_words(vals)
    out = np.zeros_like(inp)
    ok = np.zeros(len(vals), dtype=np.uint8)
    it = np.zeros(len(vals), dtype=np.int32)
    lib.feg_batch(len(vals), inp.ctypes.data, out.ctypes.data, ok.ctypes.data, it.ctypes.data)
    # each element leaves once its own a = 0 (the kernels: once every lane of the wave has, from
    # FEG_EXIT_FROM = 12 on); the result is y^-1 2^(30 k) for the k iterations run
    return [v * pow(2, -30 * int(k), P) % P for v, k in zip(_from_words(out), it)], ok, it


def _structured():
    v = [0, 1, 2, 3, 19, 38, P - 1, P - 2, P - 19, (P - 1) // 2, (P + 1) // 2, 2**254, 2**255 - 20,
         2**128, 2**128 - 1, 2**64 - 1, 2**62, 2**62 - 1, 2**61 + 1, 2**32 - 1, 2**31]
    v += [2**k for k in range(0, 255)] + [2**k - 1 for k in range(1, 255)] + [P - 2**k for k in range(0, 254)]
    v += [pow(3, k, P) for k in range(1, 200)] + [(2**k) * 3 % P for k in range(0, 250)]
    # consecutive Fibonacci numbers: the slowest inputs of Euclid-style GCDs
    a, b = 1, 1
    while b < P:
        v.append(b)
        a, b = b, a + b
    return [x % P for x in v]


def test_inverse_structured(lib):
    vals = _structured()
    out, ok, it = _run(lib, vals)
    assert ok.all(), [vals[i] for i in np.nonzero(ok == 0)[0][:5]]
    assert it.max() <= 17
    for y, v in zip(vals, out):
        assert v == pow(y, P - 2, P), hex(y)


def test_inverse_random(lib):
    rng = np.random.default_rng(20261019)
    n = 200_000
    raw = rng.integers(0, 2**32, size=(n, 8), dtype=np.uint64).astype(np.uint32)
    raw[:, 7] &= 0x7FFFFFFF
    vals = [x % P for x in _from_words(raw)]
    # small and sparse values too
    vals += [int(x) for x in rng.integers(1, 2**62, size=2000, dtype=np.uint64)]
    out, ok, it = _run(lib, vals)
    assert ok.all()
    # the margin the early exit relies on: random elements end within 14 of the 17 iterations
    assert it.max() <= 14 and (it <= 13).mean() > 0.99, np.bincount(it)
    for y, v in zip(vals[:20000], out[:20000]):
        assert v == pow(y, P - 2, P)
    # the rest by the cheaper y * y^-1 = 1 check
    for y, v in zip(vals[20000:], out[20000:]):
        assert (y * v) % P == 1
