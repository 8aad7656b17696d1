"""Shared test helpers: vector generation through the ORACLE (checker side)."""
import hashlib
import os
import random

import numpy as np

P = 2 ** 255 - 19
L = 2 ** 252 + 27742317777372353535851937790883648493


def b2b(m, n=32):
    return hashlib.blake2b(m, digest_size=n).digest()


def arr(list_of_bytes, width):
    return np.frombuffer(b"".join(list_of_bytes), dtype=np.uint8).reshape(-1, width).copy()


def rng(seed):
    return random.Random(seed)


def rbytes(r, n):
    return bytes(r.getrandbits(8) for _ in range(n))


def corrupt(b: bytes, k: int) -> bytes:
    """consensus-testlib Test/Util/Corruption.hs:29-35: increment byte k mod len."""
    b = bytearray(b)
    i = k % len(b)
    b[i] = (b[i] + 1) & 0xFF
    return bytes(b)
