"""Bencoding (BEP 3).  ``decode`` is lenient about dict key order (like
anacrolix) but exact about syntax; ``decode_with_spans`` also returns the raw
byte span of every top-level dict value, so the info-hash is the SHA-1 of the
info dict exactly as received (never re-encoded)."""

from __future__ import annotations

from typing import Any


class BencodeError(ValueError):
    pass


def encode(obj: Any) -> bytes:
    out: list[bytes] = []
    _enc(obj, out)
    return b"".join(out)


def _enc(o: Any, out: list[bytes]) -> None:
    if isinstance(o, bool):
        o = int(o)
    if isinstance(o, int):
        out.append(b"i%de" % o)
    elif isinstance(o, (bytes, bytearray, memoryview)):
        b = bytes(o)
        out.append(b"%d:" % len(b))
        out.append(b)
    elif isinstance(o, str):
        b = o.encode()
        out.append(b"%d:" % len(b))
        out.append(b)
    elif isinstance(o, (list, tuple)):
        out.append(b"l")
        for x in o:
            _enc(x, out)
        out.append(b"e")
    elif isinstance(o, dict):
        out.append(b"d")
        items = [((k.encode() if isinstance(k, str) else bytes(k)), v) for k, v in o.items()]
        for k, v in sorted(items, key=lambda kv: kv[0]):
            out.append(b"%d:" % len(k))
            out.append(k)
            _enc(v, out)
        out.append(b"e")
    else:
        raise BencodeError(f"cannot bencode {type(o).__name__}")


def _dec(b: bytes, i: int, depth: int = 0) -> tuple[Any, int]:
    if depth > 64:
        raise BencodeError("nesting too deep")
    if i >= len(b):
        raise BencodeError("unexpected end of data")
    c = b[i]
    if c == 0x69:  # i
        j = b.index(b"e", i)
        s = b[i + 1:j]
        if not s or s == b"-0" or (s[0:1] == b"0" and len(s) > 1) or (s[:2] == b"-0"):
            raise BencodeError(f"invalid integer {s!r}")
        try:
            return int(s), j + 1
        except ValueError as e:
            raise BencodeError(f"invalid integer {s!r}") from e
    if c == 0x6C:  # l
        i += 1
        lst = []
        while True:
            if i >= len(b):
                raise BencodeError("unterminated list")
            if b[i] == 0x65:
                return lst, i + 1
            v, i = _dec(b, i, depth + 1)
            lst.append(v)
    if c == 0x64:  # d
        i += 1
        d = {}
        while True:
            if i >= len(b):
                raise BencodeError("unterminated dict")
            if b[i] == 0x65:
                return d, i + 1
            k, i = _dec(b, i, depth + 1)
            if not isinstance(k, bytes):
                raise BencodeError("dict key must be a string")
            v, i = _dec(b, i, depth + 1)
            d[k] = v
    if 0x30 <= c <= 0x39:
        j = b.find(b":", i)
        if j < 0:
            raise BencodeError("bad string length")
        n = int(b[i:j])
        if b[i:i + 1] == b"0" and j - i > 1:
            raise BencodeError("leading zero in string length")
        if j + 1 + n > len(b):
            raise BencodeError("string exceeds data")
        return b[j + 1:j + 1 + n], j + 1 + n
    raise BencodeError(f"invalid token {chr(c)!r} at {i}")


def decode(b: bytes, allow_trailing: bool = False) -> Any:
    try:
        v, i = _dec(bytes(b), 0)
    except (IndexError, ValueError) as e:
        if isinstance(e, BencodeError):
            raise
        raise BencodeError(str(e)) from e
    if i != len(b) and not allow_trailing:
        raise BencodeError("trailing data after bencoded value")
    return v


def decode_prefix(b: bytes) -> tuple[Any, int]:
    """Decode one value at the start of ``b``; returns (value, bytes consumed)."""
    try:
        return _dec(bytes(b), 0)
    except (IndexError, ValueError) as e:
        if isinstance(e, BencodeError):
            raise
        raise BencodeError(str(e)) from e


def decode_with_spans(b: bytes) -> tuple[dict, dict[bytes, tuple[int, int]]]:
    """Decode a top-level dict and return the raw [start, end) span of each value."""
    b = bytes(b)
    if not b.startswith(b"d"):
        raise BencodeError("top-level value is not a dict")
    i = 1
    d: dict = {}
    spans: dict[bytes, tuple[int, int]] = {}
    while True:
        if i >= len(b):
            raise BencodeError("unterminated dict")
        if b[i] == 0x65:
            break
        k, i = _dec(b, i)
        if not isinstance(k, bytes):
            raise BencodeError("dict key must be a string")
        s = i
        v, i = _dec(b, i)
        d[k] = v
        spans[k] = (s, i)
    return d, spans
