"""Minimal protobuf (proto3) wire codec that preserves unknown fields.

Why hand-written: the upstream schema (tritonmedia.go v1.0.2, imported by the
reference as ``api`` at ``cmd/downloader/downloader.go:23``) is not available
offline and there is no ``protoc``.  A field-preserving codec lets the worker
decode only what it needs (``Media.id``, ``Media.sourceURI``) and re-emit the
``Media`` sub-message byte-for-byte into ``Convert`` — exactly what the Go
code achieves by copying ``job.Media`` (``downloader.go:138``) — even if our
field numbering for the *other* Media fields were off.
"""

from __future__ import annotations

from typing import Iterator

VARINT, I64, LEN, SGROUP, EGROUP, I32 = 0, 1, 2, 3, 4, 5


class DecodeError(ValueError):
    pass


def encode_varint(v: int) -> bytes:
    if v < 0:
        v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def decode_varint(buf: bytes | memoryview, pos: int) -> tuple[int, int]:
    result = 0
    shift = 0
    n = len(buf)
    while True:
        if pos >= n:
            raise DecodeError("truncated varint")
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            if shift >= 64 and result >> 64:
                raise DecodeError("varint overflow")
            return result, pos
        shift += 7
        if shift > 63 + 7:
            raise DecodeError("varint too long")


def iter_fields(buf: bytes) -> Iterator[tuple[int, int, object, bytes]]:
    """Yield (field_number, wire_type, value, raw_bytes_of_whole_field)."""
    mv = memoryview(buf)
    pos = 0
    n = len(buf)
    while pos < n:
        start = pos
        key, pos = decode_varint(mv, pos)
        fn, wt = key >> 3, key & 7
        if fn == 0:
            raise DecodeError("field number 0")
        if wt == VARINT:
            val, pos = decode_varint(mv, pos)
        elif wt == I64:
            if pos + 8 > n:
                raise DecodeError("truncated fixed64")
            val = bytes(mv[pos:pos + 8])
            pos += 8
        elif wt == LEN:
            ln, pos = decode_varint(mv, pos)
            if pos + ln > n:
                raise DecodeError("truncated length-delimited field")
            val = bytes(mv[pos:pos + ln])
            pos += ln
        elif wt == I32:
            if pos + 4 > n:
                raise DecodeError("truncated fixed32")
            val = bytes(mv[pos:pos + 4])
            pos += 4
        elif wt == SGROUP:
            # skip a (deprecated) group by scanning to the matching end tag
            depth = 1
            while depth:
                k2, pos = decode_varint(mv, pos)
                w2 = k2 & 7
                if w2 == SGROUP:
                    depth += 1
                elif w2 == EGROUP:
                    depth -= 1
                elif w2 == VARINT:
                    _, pos = decode_varint(mv, pos)
                elif w2 == I64:
                    pos += 8
                elif w2 == I32:
                    pos += 4
                elif w2 == LEN:
                    ln, pos = decode_varint(mv, pos)
                    pos += ln
                else:
                    raise DecodeError("bad wire type in group")
                if pos > n:
                    raise DecodeError("truncated group")
            val = None
        else:
            raise DecodeError(f"invalid wire type {wt}")
        yield fn, wt, val, bytes(mv[start:pos])


def key(fn: int, wt: int) -> bytes:
    return encode_varint((fn << 3) | wt)


def enc_string(fn: int, s: str | bytes) -> bytes:
    b = s.encode() if isinstance(s, str) else s
    if not b:
        return b""  # proto3: default values are not emitted
    return key(fn, LEN) + encode_varint(len(b)) + b


def enc_bytes_always(fn: int, b: bytes) -> bytes:
    return key(fn, LEN) + encode_varint(len(b)) + b


def enc_varint_field(fn: int, v: int) -> bytes:
    if not v:
        return b""
    return key(fn, VARINT) + encode_varint(v)
