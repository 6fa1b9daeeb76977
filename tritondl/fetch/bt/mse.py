"""Message Stream Encryption / Protocol Encryption (MSE/PE) for BitTorrent.

anacrolix/torrent negotiates MSE "header obfuscation" with
peers, and many swarms refuse plaintext connections, so a drop-in replacement
must speak it.  Handshake (both directions, over any asyncio stream pair):

    A->B  Ya, PadA                                    (768-bit DH, G=2)
    B->A  Yb, PadB
    A->B  H('req1',S), H('req2',SKEY)^H('req3',S),
          RC4a(VC, crypto_provide, len(PadC), PadC, len(IA)), RC4a(IA)
    B->A  RC4b(VC, crypto_select, len(PadD), PadD), then the payload stream

S is the DH secret, SKEY the info-hash, VC eight zero bytes; RC4 keys are
SHA1('keyA'|'keyB', S, SKEY) with the first 1024 keystream bytes dropped.
After the handshake the stream is RC4 (crypto 0x02) or plaintext (0x01) as
selected.  RC4 runs natively (``_hash_host.Rc4``); DH uses Python's ``pow``.

Policies (``TorrentConfig.encryption``):
  ``disable``  plaintext only (MSE connections are refused)
  ``allow``    dial plaintext, accept both (default)
  ``prefer``   dial MSE offering RC4+plain, fall back to plaintext; accept both
  ``require``  RC4 only, both directions
"""

from __future__ import annotations

import asyncio
import hashlib
import os
import struct

from ...ops.hashing import _host

P = int(
    "FFFFFFFFFFFFFFFFC90FDAA22168C234C4C6628B80DC1CD129024E088A67CC74020BBEA63B139B22514A08798E3404DD"
    "EF9519B3CD3A431B302B0A6DF25F14374FE1356D6D51C245E485B576625E7EC6F44C42E9A63A36210000000000090563", 16)
G = 2
VC = b"\x00" * 8
CRYPTO_PLAIN, CRYPTO_RC4 = 0x01, 0x02
MAX_PAD = 512
POLICIES = ("disable", "allow", "prefer", "require")
PLAIN_PREFIX = b"\x13BitTorrent protocol"
OFFLOAD_BYTES = 64 * 1024


class MseError(ConnectionError):
    pass


def _h(*parts: bytes) -> bytes:
    return hashlib.sha1(b"".join(parts)).digest()


def _keypair() -> tuple[int, bytes]:
    x = int.from_bytes(os.urandom(20), "big")          # 160-bit private exponent (spec: >= 128 bits)
    return x, pow(G, x, P).to_bytes(96, "big")


def _secret(x: int, their_pub: bytes) -> bytes:
    y = int.from_bytes(their_pub, "big")
    if not 1 < y < P - 1:
        raise MseError("bad DH public key")
    return pow(y, x, P).to_bytes(96, "big")


def _rc4(tag: bytes, s: bytes, skey: bytes):
    return _host.Rc4(_h(tag, s, skey), 1024)


class MseReader:
    """StreamReader look-alike that decrypts (or just passes through) and
    first serves bytes already pulled in during the handshake."""

    def __init__(self, reader: asyncio.StreamReader, dec, prefix: bytes = b"") -> None:
        self._r = reader
        self._dec = dec
        self._buf = bytearray(prefix)

    async def read(self, n: int = -1) -> bytes:
        if self._buf:
            k = len(self._buf) if n < 0 else min(n, len(self._buf))
            out = bytes(self._buf[:k])
            del self._buf[:k]
            return out
        data = await self._r.read(n)
        if not data or self._dec is None:
            return data
        if len(data) >= OFFLOAD_BYTES:
            # RC4 is byte-serial (~300 MB/s/core); big segments decrypt on a
            # worker thread (GIL released) so several peers decrypt in parallel.
            # One reader per connection keeps the keystream order.
            return await asyncio.get_running_loop().run_in_executor(None, self._dec.crypt, data)
        return self._dec.crypt(data)

    async def readexactly(self, n: int) -> bytes:
        out = bytearray()
        while len(out) < n:
            chunk = await self.read(n - len(out))
            if not chunk:
                raise asyncio.IncompleteReadError(bytes(out), n)
            out += chunk
        return bytes(out)

    def at_eof(self) -> bool:
        return not self._buf and self._r.at_eof()


class MseWriter:
    """StreamWriter look-alike that encrypts what it writes."""

    def __init__(self, writer: asyncio.StreamWriter, enc) -> None:
        self._w = writer
        self._enc = enc
        self.transport = writer.transport

    def write(self, data) -> None:
        self._w.write(self._enc.crypt(data) if self._enc is not None else data)

    async def drain(self) -> None:
        await self._w.drain()

    def close(self) -> None:
        self._w.close()

    def is_closing(self) -> bool:
        return self._w.is_closing()

    async def wait_closed(self) -> None:
        await self._w.wait_closed()

    def get_extra_info(self, name, default=None):
        return self._w.get_extra_info(name, default)


class _Feed:
    """Raw (undecrypted) handshake bytes: what the sync scan over-read plus
    whatever the socket delivers next, handed out exactly.  Bytes are only
    decrypted once we know they belong to the encrypted part, so a
    plaintext-selecting peer's payload that shares a segment with the
    handshake is never garbled."""

    def __init__(self, reader: asyncio.StreamReader, raw: bytes = b"") -> None:
        self.r = reader
        self.buf = bytearray(raw)

    async def take(self, n: int) -> bytes:
        while len(self.buf) < n:
            more = await self.r.read(4096)
            if not more:
                raise MseError("connection closed during MSE handshake")
            self.buf += more
        out = bytes(self.buf[:n])
        del self.buf[:n]
        return out

    def rest(self) -> bytes:
        out = bytes(self.buf)
        self.buf.clear()
        return out


async def _scan(reader: asyncio.StreamReader, buf: bytearray, pattern: bytes, limit: int) -> bytes:
    """Read until ``pattern`` appears within ``limit`` (+pattern) bytes of the
    start of ``buf``; return the raw bytes that followed it."""
    while True:
        k = buf.find(pattern)
        if k >= 0:
            return bytes(buf[k + len(pattern):])
        if len(buf) >= limit + len(pattern):
            raise MseError("MSE sync pattern not found")
        chunk = await reader.read(limit + len(pattern) - len(buf))
        if not chunk:
            raise MseError("connection closed during MSE handshake")
        buf += chunk


async def initiate(reader: asyncio.StreamReader, writer: asyncio.StreamWriter, skey: bytes, ia: bytes,
                   provide: int = CRYPTO_RC4 | CRYPTO_PLAIN, timeout: float = 10.0
                   ) -> tuple[MseReader, MseWriter, int]:
    """Outgoing MSE handshake carrying ``ia`` (our BT handshake) as the
    initial payload.  Returns wrapped streams and the selected crypto."""
    async def run():
        x, ya = _keypair()
        writer.write(ya + os.urandom(int.from_bytes(os.urandom(2), "big") % (MAX_PAD + 1)))
        yb = await reader.readexactly(96)
        s = _secret(x, yb)
        enc, dec = _rc4(b"keyA", s, skey), _rc4(b"keyB", s, skey)
        req23 = bytes(a ^ b for a, b in zip(_h(b"req2", skey), _h(b"req3", s)))
        writer.write(_h(b"req1", s) + req23 +
                     enc.crypt(VC + struct.pack(">IH", provide, 0) + struct.pack(">H", len(ia))) + enc.crypt(ia))
        # B's reply starts with RC4b(VC) somewhere within PadB's 512 bytes
        feed = _Feed(reader, await _scan(reader, bytearray(), dec.crypt(VC), MAX_PAD))
        select, pad_len = struct.unpack(">IH", dec.crypt(await feed.take(6)))
        if pad_len > MAX_PAD:
            raise MseError("bad PadD length")
        dec.crypt(await feed.take(pad_len))
        if select not in (CRYPTO_PLAIN, CRYPTO_RC4) or not (select & provide):
            raise MseError(f"peer selected unsupported crypto {select:#x}")
        tail = feed.rest()
        if select == CRYPTO_PLAIN:
            return MseReader(reader, None, tail), MseWriter(writer, None), select
        return MseReader(reader, dec, dec.crypt(tail)), MseWriter(writer, enc), select
    try:
        return await asyncio.wait_for(run(), timeout)
    except (asyncio.IncompleteReadError, asyncio.TimeoutError) as e:
        raise MseError(f"MSE handshake failed: {type(e).__name__}") from e


async def respond(reader: asyncio.StreamReader, writer: asyncio.StreamWriter, first: bytes, skey: bytes,
                  allow_plain: bool = True, timeout: float = 10.0) -> tuple[MseReader, MseWriter, int]:
    """Incoming MSE handshake; ``first`` holds bytes already read (the start
    of Ya).  Returns wrapped streams whose reader yields the peer's IA (its
    BT handshake) first."""
    async def run():
        head = _Feed(reader, first)
        ya = await head.take(96)
        x, yb = _keypair()
        s = _secret(x, ya)
        writer.write(yb + os.urandom(int.from_bytes(os.urandom(2), "big") % (MAX_PAD + 1)))
        feed = _Feed(reader, await _scan(reader, bytearray(head.rest()), _h(b"req1", s), MAX_PAD))
        want = bytes(a ^ b for a, b in zip(_h(b"req2", skey), _h(b"req3", s)))
        if await feed.take(20) != want:
            raise MseError("MSE: unknown info-hash")
        dec, enc = _rc4(b"keyA", s, skey), _rc4(b"keyB", s, skey)
        hdr = dec.crypt(await feed.take(14))
        if hdr[:8] != VC:
            raise MseError("MSE: bad verification constant")
        provide, pad_len = struct.unpack(">IH", hdr[8:14])
        if pad_len > MAX_PAD:
            raise MseError("bad PadC length")
        dec.crypt(await feed.take(pad_len))
        (ia_len,) = struct.unpack(">H", dec.crypt(await feed.take(2)))
        ia = dec.crypt(await feed.take(ia_len))
        if provide & CRYPTO_RC4:
            select = CRYPTO_RC4
        elif provide & CRYPTO_PLAIN and allow_plain:
            select = CRYPTO_PLAIN
        else:
            raise MseError(f"no acceptable crypto offered ({provide:#x})")
        writer.write(enc.crypt(VC + struct.pack(">IH", select, 0)))
        tail = feed.rest()
        if select == CRYPTO_RC4:
            return MseReader(reader, dec, ia + dec.crypt(tail)), MseWriter(writer, enc), select
        return MseReader(reader, None, ia + tail), MseWriter(writer, None), select
    try:
        return await asyncio.wait_for(run(), timeout)
    except (asyncio.IncompleteReadError, asyncio.TimeoutError) as e:
        raise MseError(f"MSE handshake failed: {type(e).__name__}") from e
