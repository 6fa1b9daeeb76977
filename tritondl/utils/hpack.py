"""HPACK, the header compression of HTTP/2 (RFC 7541), for the HTTP/2 client
(:mod:`tritondl.fetch.h2`) and the test origin that speaks it.

The decoder handles every representation a server may send: indexed
fields, literals with and without indexing (and never-indexed ones), table
size updates, and Huffman-coded strings.  The encoder writes what a client
needs: static-table references and literals without indexing, optionally
Huffman-coded, with optional incremental indexing (the test origin uses it
to exercise a client's dynamic table).

Go's ``net/http`` (``golang.org/x/net/http2/hpack``) did this for grab's
transport, which negotiated HTTP/2 with any https origin offering it
(``internal/downloader/http/http.go:18-22``).
"""

from __future__ import annotations

# RFC 7541 Appendix B: (code, bit length) of each symbol 0..255, then EOS (256)
HUFFMAN = (
    (0x1ff8, 13), (0x7fffd8, 23), (0xfffffe2, 28), (0xfffffe3, 28), (0xfffffe4, 28), (0xfffffe5, 28), (0xfffffe6, 28), (0xfffffe7, 28),
    (0xfffffe8, 28), (0xffffea, 24), (0x3ffffffc, 30), (0xfffffe9, 28), (0xfffffea, 28), (0x3ffffffd, 30), (0xfffffeb, 28), (0xfffffec, 28),
    (0xfffffed, 28), (0xfffffee, 28), (0xfffffef, 28), (0xffffff0, 28), (0xffffff1, 28), (0xffffff2, 28), (0x3ffffffe, 30), (0xffffff3, 28),
    (0xffffff4, 28), (0xffffff5, 28), (0xffffff6, 28), (0xffffff7, 28), (0xffffff8, 28), (0xffffff9, 28), (0xffffffa, 28), (0xffffffb, 28),
    (0x14, 6), (0x3f8, 10), (0x3f9, 10), (0xffa, 12), (0x1ff9, 13), (0x15, 6), (0xf8, 8), (0x7fa, 11),
    (0x3fa, 10), (0x3fb, 10), (0xf9, 8), (0x7fb, 11), (0xfa, 8), (0x16, 6), (0x17, 6), (0x18, 6),
    (0x0, 5), (0x1, 5), (0x2, 5), (0x19, 6), (0x1a, 6), (0x1b, 6), (0x1c, 6), (0x1d, 6),
    (0x1e, 6), (0x1f, 6), (0x5c, 7), (0xfb, 8), (0x7ffc, 15), (0x20, 6), (0xffb, 12), (0x3fc, 10),
    (0x1ffa, 13), (0x21, 6), (0x5d, 7), (0x5e, 7), (0x5f, 7), (0x60, 7), (0x61, 7), (0x62, 7),
    (0x63, 7), (0x64, 7), (0x65, 7), (0x66, 7), (0x67, 7), (0x68, 7), (0x69, 7), (0x6a, 7),
    (0x6b, 7), (0x6c, 7), (0x6d, 7), (0x6e, 7), (0x6f, 7), (0x70, 7), (0x71, 7), (0x72, 7),
    (0xfc, 8), (0x73, 7), (0xfd, 8), (0x1ffb, 13), (0x7fff0, 19), (0x1ffc, 13), (0x3ffc, 14), (0x22, 6),
    (0x7ffd, 15), (0x3, 5), (0x23, 6), (0x4, 5), (0x24, 6), (0x5, 5), (0x25, 6), (0x26, 6),
    (0x27, 6), (0x6, 5), (0x74, 7), (0x75, 7), (0x28, 6), (0x29, 6), (0x2a, 6), (0x7, 5),
    (0x2b, 6), (0x76, 7), (0x2c, 6), (0x8, 5), (0x9, 5), (0x2d, 6), (0x77, 7), (0x78, 7),
    (0x79, 7), (0x7a, 7), (0x7b, 7), (0x7ffe, 15), (0x7fc, 11), (0x3ffd, 14), (0x1ffd, 13), (0xffffffc, 28),
    (0xfffe6, 20), (0x3fffd2, 22), (0xfffe7, 20), (0xfffe8, 20), (0x3fffd3, 22), (0x3fffd4, 22), (0x3fffd5, 22), (0x7fffd9, 23),
    (0x3fffd6, 22), (0x7fffda, 23), (0x7fffdb, 23), (0x7fffdc, 23), (0x7fffdd, 23), (0x7fffde, 23), (0xffffeb, 24), (0x7fffdf, 23),
    (0xffffec, 24), (0xffffed, 24), (0x3fffd7, 22), (0x7fffe0, 23), (0xffffee, 24), (0x7fffe1, 23), (0x7fffe2, 23), (0x7fffe3, 23),
    (0x7fffe4, 23), (0x1fffdc, 21), (0x3fffd8, 22), (0x7fffe5, 23), (0x3fffd9, 22), (0x7fffe6, 23), (0x7fffe7, 23), (0xffffef, 24),
    (0x3fffda, 22), (0x1fffdd, 21), (0xfffe9, 20), (0x3fffdb, 22), (0x3fffdc, 22), (0x7fffe8, 23), (0x7fffe9, 23), (0x1fffde, 21),
    (0x7fffea, 23), (0x3fffdd, 22), (0x3fffde, 22), (0xfffff0, 24), (0x1fffdf, 21), (0x3fffdf, 22), (0x7fffeb, 23), (0x7fffec, 23),
    (0x1fffe0, 21), (0x1fffe1, 21), (0x3fffe0, 22), (0x1fffe2, 21), (0x7fffed, 23), (0x3fffe1, 22), (0x7fffee, 23), (0x7fffef, 23),
    (0xfffea, 20), (0x3fffe2, 22), (0x3fffe3, 22), (0x3fffe4, 22), (0x7ffff0, 23), (0x3fffe5, 22), (0x3fffe6, 22), (0x7ffff1, 23),
    (0x3ffffe0, 26), (0x3ffffe1, 26), (0xfffeb, 20), (0x7fff1, 19), (0x3fffe7, 22), (0x7ffff2, 23), (0x3fffe8, 22), (0x1ffffec, 25),
    (0x3ffffe2, 26), (0x3ffffe3, 26), (0x3ffffe4, 26), (0x7ffffde, 27), (0x7ffffdf, 27), (0x3ffffe5, 26), (0xfffff1, 24), (0x1ffffed, 25),
    (0x7fff2, 19), (0x1fffe3, 21), (0x3ffffe6, 26), (0x7ffffe0, 27), (0x7ffffe1, 27), (0x3ffffe7, 26), (0x7ffffe2, 27), (0xfffff2, 24),
    (0x1fffe4, 21), (0x1fffe5, 21), (0x3ffffe8, 26), (0x3ffffe9, 26), (0xffffffd, 28), (0x7ffffe3, 27), (0x7ffffe4, 27), (0x7ffffe5, 27),
    (0xfffec, 20), (0xfffff3, 24), (0xfffed, 20), (0x1fffe6, 21), (0x3fffe9, 22), (0x1fffe7, 21), (0x1fffe8, 21), (0x7ffff3, 23),
    (0x3fffea, 22), (0x3fffeb, 22), (0x1ffffee, 25), (0x1ffffef, 25), (0xfffff4, 24), (0xfffff5, 24), (0x3ffffea, 26), (0x7ffff4, 23),
    (0x3ffffeb, 26), (0x7ffffe6, 27), (0x3ffffec, 26), (0x3ffffed, 26), (0x7ffffe7, 27), (0x7ffffe8, 27), (0x7ffffe9, 27), (0x7ffffea, 27),
    (0x7ffffeb, 27), (0xffffffe, 28), (0x7ffffec, 27), (0x7ffffed, 27), (0x7ffffee, 27), (0x7ffffef, 27), (0x7fffff0, 27), (0x3ffffee, 26),
    (0x3fffffff, 30),
)

# RFC 7541 Appendix A: the static table, index 1..61
STATIC = (
    (b":authority", b""), (b":method", b"GET"), (b":method", b"POST"), (b":path", b"/"),
    (b":path", b"/index.html"), (b":scheme", b"http"), (b":scheme", b"https"), (b":status", b"200"),
    (b":status", b"204"), (b":status", b"206"), (b":status", b"304"), (b":status", b"400"),
    (b":status", b"404"), (b":status", b"500"), (b"accept-charset", b""),
    (b"accept-encoding", b"gzip, deflate"), (b"accept-language", b""), (b"accept-ranges", b""),
    (b"accept", b""), (b"access-control-allow-origin", b""), (b"age", b""), (b"allow", b""),
    (b"authorization", b""), (b"cache-control", b""), (b"content-disposition", b""),
    (b"content-encoding", b""), (b"content-language", b""), (b"content-length", b""),
    (b"content-location", b""), (b"content-range", b""), (b"content-type", b""), (b"cookie", b""),
    (b"date", b""), (b"etag", b""), (b"expect", b""), (b"expires", b""), (b"from", b""), (b"host", b""),
    (b"if-match", b""), (b"if-modified-since", b""), (b"if-none-match", b""), (b"if-range", b""),
    (b"if-unmodified-since", b""), (b"last-modified", b""), (b"link", b""), (b"location", b""),
    (b"max-forwards", b""), (b"proxy-authenticate", b""), (b"proxy-authorization", b""), (b"range", b""),
    (b"referer", b""), (b"refresh", b""), (b"retry-after", b""), (b"server", b""), (b"set-cookie", b""),
    (b"strict-transport-security", b""), (b"transfer-encoding", b""), (b"user-agent", b""), (b"vary", b""),
    (b"via", b""), (b"www-authenticate", b""),
)
_STATIC_FULL = {nv: i + 1 for i, nv in enumerate(STATIC)}
_STATIC_NAME: dict[bytes, int] = {}
for _i, (_n, _v) in enumerate(STATIC):
    _STATIC_NAME.setdefault(_n, _i + 1)

# decoding trie: per bit length, code -> symbol
_DECODE: dict[tuple[int, int], int] = {(n, c): s for s, (c, n) in enumerate(HUFFMAN)}
_MIN_BITS = min(n for _c, n in HUFFMAN)


class HPACKError(Exception):
    """A header block that does not decode (a COMPRESSION_ERROR in HTTP/2)."""


def encode_int(value: int, prefix_bits: int, first: int = 0) -> bytes:
    """RFC 7541 5.1: ``value`` with an N-bit prefix; ``first`` holds the
    representation's flag bits above the prefix."""
    cap = (1 << prefix_bits) - 1
    if value < cap:
        return bytes([first | value])
    out = bytearray([first | cap])
    value -= cap
    while value >= 128:
        out.append((value & 0x7F) | 0x80)
        value >>= 7
    out.append(value)
    return bytes(out)


def decode_int(buf: bytes, pos: int, prefix_bits: int) -> tuple[int, int]:
    cap = (1 << prefix_bits) - 1
    if pos >= len(buf):
        raise HPACKError("truncated integer")
    v = buf[pos] & cap
    pos += 1
    if v < cap:
        return v, pos
    shift = 0
    while True:
        if pos >= len(buf):
            raise HPACKError("truncated integer")
        b = buf[pos]
        pos += 1
        v += (b & 0x7F) << shift
        shift += 7
        if not b & 0x80:
            return v, pos
        if shift > 56:
            raise HPACKError("integer too large")


def huffman_encode(data: bytes) -> bytes:
    acc = nbits = 0
    out = bytearray()
    for b in data:
        code, n = HUFFMAN[b]
        acc = (acc << n) | code
        nbits += n
        while nbits >= 8:
            nbits -= 8
            out.append((acc >> nbits) & 0xFF)
        acc &= (1 << nbits) - 1
    if nbits:
        out.append(((acc << (8 - nbits)) | ((1 << (8 - nbits)) - 1)) & 0xFF)   # EOS-prefix padding
    return bytes(out)


def huffman_decode(data: bytes) -> bytes:
    out = bytearray()
    code = n = 0
    for byte in data:
        for k in range(7, -1, -1):
            code = (code << 1) | ((byte >> k) & 1)
            n += 1
            if n >= _MIN_BITS:
                s = _DECODE.get((n, code))
                if s is not None:
                    if s == 256:
                        raise HPACKError("EOS in a Huffman string")
                    out.append(s)
                    code = n = 0
                elif n > 30:
                    raise HPACKError("bad Huffman code")
    # RFC 7541 5.2: padding is at most 7 bits, all ones (a prefix of EOS)
    if n > 7 or code != (1 << n) - 1:
        raise HPACKError("bad Huffman padding")
    return bytes(out)


def encode_str(s: bytes, huffman: bool) -> bytes:
    if huffman:
        h = huffman_encode(s)
        if len(h) < len(s):
            return encode_int(len(h), 7, 0x80) + h
    return encode_int(len(s), 7) + s


def _entry_size(name: bytes, value: bytes) -> int:
    return len(name) + len(value) + 32


class Table:
    """The dynamic table (RFC 7541 2.3.2, 4): newest first; evicted from the
    end when its size passes ``max_size``."""

    def __init__(self, max_size: int = 4096) -> None:
        self.max_size = max_size
        self.entries: list[tuple[bytes, bytes]] = []
        self.size = 0

    def add(self, name: bytes, value: bytes) -> None:
        self.entries.insert(0, (name, value))
        self.size += _entry_size(name, value)
        self._evict()

    def resize(self, n: int) -> None:
        self.max_size = n
        self._evict()

    def _evict(self) -> None:
        while self.size > self.max_size and self.entries:
            n, v = self.entries.pop()
            self.size -= _entry_size(n, v)

    def get(self, index: int) -> tuple[bytes, bytes]:
        if 1 <= index <= len(STATIC):
            return STATIC[index - 1]
        k = index - len(STATIC) - 1
        if 0 <= k < len(self.entries):
            return self.entries[k]
        raise HPACKError(f"header index {index} out of range")


class Decoder:
    def __init__(self, max_table_size: int = 4096) -> None:
        self.table = Table(max_table_size)
        self.limit = max_table_size           # what SETTINGS_HEADER_TABLE_SIZE allows

    def _str(self, buf: bytes, pos: int) -> tuple[bytes, int]:
        if pos >= len(buf):
            raise HPACKError("truncated string")
        huff = buf[pos] & 0x80
        n, pos = decode_int(buf, pos, 7)
        if pos + n > len(buf):
            raise HPACKError("truncated string")
        raw = buf[pos:pos + n]
        return (huffman_decode(raw) if huff else bytes(raw)), pos + n

    def decode(self, block: bytes) -> list[tuple[bytes, bytes]]:
        out = []
        pos = 0
        while pos < len(block):
            b = block[pos]
            if b & 0x80:                                   # indexed field
                i, pos = decode_int(block, pos, 7)
                if i == 0:
                    raise HPACKError("index 0")
                out.append(self.table.get(i))
            elif b & 0x40:                                 # literal, incremental indexing
                i, pos = decode_int(block, pos, 6)
                name = self.table.get(i)[0] if i else None
                if name is None:
                    name, pos = self._str(block, pos)
                value, pos = self._str(block, pos)
                self.table.add(name, value)
                out.append((name, value))
            elif b & 0x20:                                 # dynamic table size update
                n, pos = decode_int(block, pos, 5)
                if n > self.limit:
                    raise HPACKError(f"table size {n} above the {self.limit} allowed")
                self.table.resize(n)
            else:                                          # literal without indexing / never indexed
                i, pos = decode_int(block, pos, 4)
                name = self.table.get(i)[0] if i else None
                if name is None:
                    name, pos = self._str(block, pos)
                value, pos = self._str(block, pos)
                out.append((name, value))
        return out


class Encoder:
    """``index=False``: static references and literals without indexing (no
    state: what a client needs).  ``index=True`` also adds every literal to
    the dynamic table, as most servers do."""

    def __init__(self, huffman: bool = True, index: bool = False, max_table_size: int = 4096) -> None:
        self.huffman = huffman
        self.index = index
        self.table = Table(max_table_size)

    def encode(self, headers: list[tuple[bytes, bytes]]) -> bytes:
        out = bytearray()
        for name, value in headers:
            name = name.lower()
            full = _STATIC_FULL.get((name, value))
            if full is not None:
                out += encode_int(full, 7, 0x80)
                continue
            if self.index:
                dyn = next((k for k, nv in enumerate(self.table.entries) if nv == (name, value)), None)
                if dyn is not None:
                    out += encode_int(len(STATIC) + 1 + dyn, 7, 0x80)
                    continue
            ni = _STATIC_NAME.get(name, 0)
            if self.index:
                out += encode_int(ni, 6, 0x40)
            else:
                out += encode_int(ni, 4, 0x00)
            if not ni:
                out += encode_str(name, self.huffman)
            out += encode_str(value, self.huffman)
            if self.index:
                self.table.add(name, value)
        return bytes(out)
