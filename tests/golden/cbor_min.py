"""Minimal CBOR (RFC 8949) decoder that keeps byte spans.

Test infrastructure only: used by make_golden.py to pull the header fields and
the exact signed byte ranges out of the reference's golden block files
(/root/reference/ouroboros-consensus-cardano/golden/...).  Every decoded item is
returned as ``Item(value, start, end)`` so the caller can recover the raw
encoding of any sub-structure (e.g. the header body that the KES signature
covers, Header.hs:90-94).
"""
from dataclasses import dataclass
from typing import Any


@dataclass
class Item:
    value: Any
    start: int
    end: int
    tag: int | None = None

    def raw(self, buf: bytes) -> bytes:
        return buf[self.start:self.end]


def _arg(buf: bytes, pos: int, info: int):
    if info < 24:
        return info, pos
    if info == 24:
        return buf[pos], pos + 1
    if info == 25:
        return int.from_bytes(buf[pos:pos + 2], "big"), pos + 2
    if info == 26:
        return int.from_bytes(buf[pos:pos + 4], "big"), pos + 4
    if info == 27:
        return int.from_bytes(buf[pos:pos + 8], "big"), pos + 8
    if info == 31:
        return None, pos  # indefinite
    raise ValueError(f"bad additional info {info} at {pos}")


def decode(buf: bytes, pos: int = 0) -> Item:
    start = pos
    ib = buf[pos]
    pos += 1
    major, info = ib >> 5, ib & 31
    arg, pos = _arg(buf, pos, info)
    if major == 0:
        return Item(arg, start, pos)
    if major == 1:
        return Item(-1 - arg, start, pos)
    if major in (2, 3):
        if arg is None:  # indefinite string: concatenate chunks
            chunks = []
            while buf[pos] != 0xFF:
                it = decode(buf, pos)
                chunks.append(it.value)
                pos = it.end
            pos += 1
            v = b"".join(chunks) if major == 2 else "".join(chunks)
            return Item(v, start, pos)
        v = buf[pos:pos + arg]
        pos += arg
        return Item(bytes(v) if major == 2 else v.decode(), start, pos)
    if major == 4:
        items = []
        if arg is None:
            while buf[pos] != 0xFF:
                it = decode(buf, pos)
                items.append(it)
                pos = it.end
            pos += 1
        else:
            for _ in range(arg):
                it = decode(buf, pos)
                items.append(it)
                pos = it.end
        return Item(items, start, pos)
    if major == 5:
        kv = []
        n = arg
        while (n is None and buf[pos] != 0xFF) or (n is not None and len(kv) < n):
            k = decode(buf, pos)
            v = decode(buf, k.end)
            kv.append((k, v))
            pos = v.end
        if n is None:
            pos += 1
        return Item(kv, start, pos)
    if major == 6:
        inner = decode(buf, pos)
        return Item(inner.value, start, inner.end, tag=arg)
    if major == 7:
        if info == 20:
            return Item(False, start, pos)
        if info == 21:
            return Item(True, start, pos)
        if info == 22:
            return Item(None, start, pos)
        return Item(("simple", arg), start, pos)
    raise ValueError(major)
