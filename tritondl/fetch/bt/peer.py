"""BitTorrent peer wire protocol: handshake + messages (BEP 3), Fast
extension subset (BEP 6: have_all / have_none / reject), extension protocol
(BEP 10), ut_metadata (BEP 9) and ut_pex peer exchange (BEP 11).

Transport-agnostic: works over any asyncio (reader, writer) pair — TCP, or
the native uTP transport (:mod:`tritondl.fetch.bt.utp`).
"""

from __future__ import annotations

import asyncio
import struct
from dataclasses import dataclass, field

from . import bencode

PSTR = b"BitTorrent protocol"
HANDSHAKE_LEN = 49 + len(PSTR)

CHOKE, UNCHOKE, INTERESTED, NOT_INTERESTED, HAVE, BITFIELD, REQUEST, PIECE, CANCEL, PORT = range(10)
SUGGEST, HAVE_ALL, HAVE_NONE, REJECT, ALLOWED_FAST = 0x0D, 0x0E, 0x0F, 0x10, 0x11
EXTENDED = 20
HASH_REQUEST, HASHES, HASH_REJECT = 21, 22, 23        # BEP 52
EXT_HANDSHAKE = 0
UT_METADATA_ID = 3            # the id WE assign to ut_metadata in our extended handshake
UT_PEX_ID = 1                 # ... and to ut_pex
PEX_MAX_ADDED = 50            # BEP 11: at most 50 added / 50 dropped per message
META_REQUEST, META_DATA, META_REJECT = 0, 1, 2
MAX_MSG = 2 * 1024 * 1024 + 13


def reserved_bytes(dht: bool = True, fast: bool = True, extended: bool = True, v2: bool = True) -> bytes:
    r = bytearray(8)
    if v2:
        r[7] |= 0x10          # BEP 52: supports v2 hash requests / messages
    if extended:
        r[5] |= 0x10
    if fast:
        r[7] |= 0x04
    if dht:
        r[7] |= 0x01
    return bytes(r)


class PeerError(Exception):
    pass


@dataclass
class Handshake:
    reserved: bytes
    infohash: bytes
    peer_id: bytes

    @property
    def extended(self) -> bool:
        return bool(self.reserved[5] & 0x10)

    @property
    def fast(self) -> bool:
        return bool(self.reserved[7] & 0x04)

    @property
    def dht(self) -> bool:
        return bool(self.reserved[7] & 0x01)

    @property
    def v2(self) -> bool:
        return bool(self.reserved[7] & 0x10)


def encode_handshake(infohash: bytes, peer_id: bytes, reserved: bytes | None = None) -> bytes:
    return bytes([len(PSTR)]) + PSTR + (reserved or reserved_bytes()) + infohash + peer_id


def parse_handshake(b: bytes) -> Handshake:
    if len(b) != HANDSHAKE_LEN or b[0] != len(PSTR) or b[1:20] != PSTR:
        raise PeerError("bad protocol string in handshake")
    return Handshake(b[20:28], b[28:48], b[48:68])


async def read_handshake(reader) -> Handshake:
    return parse_handshake(await reader.readexactly(HANDSHAKE_LEN))


@dataclass
class ExtHandshake:
    m: dict[str, int] = field(default_factory=dict)
    metadata_size: int | None = None
    reqq: int | None = None
    v: str = ""
    port: int | None = None


class Wire:
    """Framed message reader/writer over one connection.

    Batched in both directions, because per-message awaits and per-message
    ``send`` syscalls dominated a Python peer at swarm rates: ``read_batch``
    parses every complete message already received (one wake-up → many 16 KiB
    blocks), and outgoing messages are coalesced into one buffer flushed once
    per event-loop iteration."""

    def __init__(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        self.reader = reader
        self.writer = writer
        self.closed = False
        self._rbuf = bytearray()
        self._out: list[bytes] = []
        self._flush_scheduled = False

    async def read(self) -> tuple[int, bytes] | None:
        """Next message as (id, payload); None for keep-alive."""
        while True:
            msgs = self._parse(1)
            if msgs:
                return msgs[0]
            await self._fill()

    async def read_batch(self, limit: int = 256) -> list[tuple[int, bytes] | None]:
        """At least one message; all complete ones already buffered (≤ limit)."""
        while True:
            msgs = self._parse(limit)
            if msgs:
                return msgs
            await self._fill()

    async def read_raw(self) -> bytes:
        """The next chunk of the byte stream, unparsed (the native link parses
        it): whatever the message parser had buffered first, else one read."""
        if self._rbuf:
            data = bytes(self._rbuf)
            self._rbuf.clear()
            return data
        data = await self.reader.read(1 << 18)
        if not data:
            raise asyncio.IncompleteReadError(b"", None)
        return data

    def take_over(self, link, on_data, on_bytes=None) -> tuple[LinkReader, bytes] | None:
        """Switch a connection's receive side to the native link.  Plain TCP
        gets zero-copy receive (:class:`LinkReader`: ``on_data(nbytes)`` after
        the kernel wrote into the link's buffer); a uTP stream hands the
        engine's bytes straight to ``on_bytes(data)`` (:class:`UtpLinkReader`).
        Returns (reader, bytes already buffered — the caller feeds these
        first), or None (MSE-encrypted, closing): those keep :meth:`read_raw`.
        Call only while no read is pending."""
        tr = self.writer.transport
        buf = getattr(self.reader, "_buffer", None)
        if type(self.reader) is not asyncio.StreamReader or buf is None or tr.is_closing() \
                or self.reader.at_eof() or self.reader.exception() is not None:
            return None
        stream = getattr(tr, "stream", None)
        if type(tr).__name__ == "_UtpTransport" and stream is not None and on_bytes is not None:
            leftover = bytes(self._rbuf) + bytes(buf)
            self._rbuf.clear()
            buf.clear()
            urx = UtpLinkReader(tr, link, on_bytes)
            tr.set_protocol(urx)                 # its pause/resume_writing reach the reader (serve budget)
            stream.sink, stream.sink_eof = urx.deliver, urx.eof
            return urx, leftover
        if type(tr).__name__ != "_SelectorSocketTransport":
            return None
        leftover = bytes(self._rbuf) + bytes(buf)
        self._rbuf.clear()
        buf.clear()
        rx = LinkReader(tr, link, on_data)
        tr.set_protocol(rx)
        if not tr.is_reading():
            # the StreamReader had paused the transport (its buffer was over the
            # limit); that buffer is now the caller's `leftover`: read on
            tr.resume_reading()
        return rx, leftover

    async def _fill(self) -> None:
        data = await self.reader.read(1 << 18)
        if not data:
            raise asyncio.IncompleteReadError(bytes(self._rbuf), None)
        self._rbuf += data

    def _parse(self, limit: int) -> list:
        out: list = []
        buf = self._rbuf
        pos = 0
        n_buf = len(buf)
        while len(out) < limit and n_buf - pos >= 4:
            (n,) = struct.unpack_from(">I", buf, pos)
            if n > MAX_MSG:
                raise PeerError(f"message too large ({n})")
            if n_buf - pos - 4 < n:
                break
            if n == 0:
                out.append(None)
            else:
                out.append((buf[pos + 4], bytes(buf[pos + 5:pos + 4 + n])))
            pos += 4 + n
        if pos:
            del buf[:pos]
        return out

    def _queue(self, data: bytes) -> None:
        if self.closed:
            return
        self._out.append(data)
        if not self._flush_scheduled:
            self._flush_scheduled = True
            asyncio.get_running_loop().call_soon(self.flush)

    def flush(self) -> None:
        self._flush_scheduled = False
        if self._out and not self.closed:
            data = b"".join(self._out)
            self._out.clear()
            try:
                self.writer.write(data)
            except (RuntimeError, ConnectionError):
                self.closed = True

    def send(self, mid: int, payload: bytes = b"") -> None:
        self._queue(struct.pack(">IB", len(payload) + 1, mid) + payload)

    def send_raw(self, data: bytes) -> None:
        self._queue(data)

    def keepalive(self) -> None:
        self._queue(b"\x00\x00\x00\x00")

    async def drain(self) -> None:
        self.flush()
        await self.writer.drain()

    # -- typed senders ------------------------------------------------------
    def have(self, i: int) -> None:
        self.send(HAVE, struct.pack(">I", i))

    def bitfield(self, bits: bytes) -> None:
        self.send(BITFIELD, bits)

    def request(self, i: int, off: int, n: int) -> None:
        self.send(REQUEST, struct.pack(">III", i, off, n))

    def cancel(self, i: int, off: int, n: int) -> None:
        self.send(CANCEL, struct.pack(">III", i, off, n))

    def reject(self, i: int, off: int, n: int) -> None:
        self.send(REJECT, struct.pack(">III", i, off, n))

    def piece(self, i: int, off: int, data: bytes) -> None:
        self._queue(struct.pack(">IBII", len(data) + 9, PIECE, i, off))
        self._queue(data)

    def hash_request(self, root: bytes, base: int, index: int, length: int, proofs: int) -> None:
        self.send(HASH_REQUEST, root + struct.pack(">IIII", base, index, length, proofs))

    def hashes(self, root: bytes, base: int, index: int, length: int, proofs: int, hashes: bytes) -> None:
        self.send(HASHES, root + struct.pack(">IIII", base, index, length, proofs) + hashes)

    def hash_reject(self, root: bytes, base: int, index: int, length: int, proofs: int) -> None:
        self.send(HASH_REJECT, root + struct.pack(">IIII", base, index, length, proofs))

    def extended(self, ext_id: int, payload: bytes) -> None:
        self.send(EXTENDED, bytes([ext_id]) + payload)

    def ext_handshake(self, metadata_size: int | None, port: int | None = None, reqq: int = 512,
                      pex: bool = True) -> None:
        m = {b"ut_metadata": UT_METADATA_ID}
        if pex:
            m[b"ut_pex"] = UT_PEX_ID
        d: dict = {b"m": m, b"v": b"tritondl/0.1", b"reqq": reqq}
        if metadata_size:
            d[b"metadata_size"] = metadata_size
        if port:
            d[b"p"] = port
        self.extended(EXT_HANDSHAKE, bencode.encode(d))

    def close(self) -> None:
        if not self.closed:
            self.flush()
            self.closed = True
            try:
                self.writer.close()
            except Exception:
                pass


class LinkReader(asyncio.BufferedProtocol):
    """Zero-copy receive for a native link (csrc/btwire): installed on a plain
    TCP transport in place of the StreamReader's protocol, so the socket reads
    straight into the link's buffer (``recv_into``) and ``on_data(nbytes)``
    parses it on the spot — no StreamReader buffer, no bytes objects, no task
    wake-up per read.  Control messages the callback hands to :meth:`push`
    queue up for the peer loop (:meth:`get`); write flow control and
    connection loss are forwarded to the old protocol so the StreamWriter
    keeps working."""

    def __init__(self, transport: asyncio.Transport, link, on_data) -> None:
        self._tr = transport
        self._old = transport.get_protocol()
        self._link = link
        self._on_data = on_data
        self._msgs: list[tuple[int, bytes]] = []
        self._waiter: asyncio.Future | None = None
        self._exc: BaseException | None = None
        self._eof = False
        self._paused = False      # control messages queued up: the peer loop is behind
        self._wpaused = False     # write buffer over the high-water mark
        self._reading = True
        self._kick_scheduled = False
        self._empty = 0           # what _on_data gets to parse what is already buffered

    # -- transport callbacks --------------------------------------------------
    def get_buffer(self, sizehint: int):
        return self._link.recv_buffer(1 << 20)

    def buffer_updated(self, nbytes) -> None:
        try:
            self._on_data(nbytes)
        except Exception as e:  # a protocol violation: end the peer loop with it
            self._fail(e)
            return
        if self._link.stalled and not self._kick_scheduled:
            # the link stopped at its serve budget: parse the rest once the
            # replies are on their way (now, or when the socket drains)
            self._kick_scheduled = True
            if not self._wpaused:
                asyncio.get_running_loop().call_soon(self._kick)

    def _kick(self) -> None:
        self._kick_scheduled = False
        if self._exc is None and not self._tr.is_closing():
            self.buffer_updated(self._empty)

    def eof_received(self) -> bool:
        self._eof = True
        self._wake()
        return False

    def connection_lost(self, exc) -> None:
        self._eof = True
        if exc is not None and self._exc is None:
            self._exc = exc
        self._wake()
        self._old.connection_lost(exc)

    def pause_writing(self) -> None:
        # the link answers REQUESTs as it parses them: while the socket's send
        # side is backed up, stop reading, so served blocks do not pile up
        self._wpaused = True
        self._update_reading()
        self._old.pause_writing()

    def resume_writing(self) -> None:
        self._wpaused = False
        self._update_reading()
        self._old.resume_writing()
        if self._kick_scheduled:
            asyncio.get_running_loop().call_soon(self._kick)

    def _update_reading(self) -> None:
        want = not (self._paused or self._wpaused or self._exc is not None)
        if want != self._reading and not self._tr.is_closing():
            self._reading = want
            (self._tr.resume_reading if want else self._tr.pause_reading)()

    # -- peer-loop side -------------------------------------------------------
    def push(self, mid: int, payload: bytes) -> None:
        self._msgs.append((mid, payload))
        if len(self._msgs) >= 1024 and not self._paused:   # the loop is behind: stop reading
            self._paused = True
            self._update_reading()
        self._wake()

    async def get(self) -> list[tuple[int, bytes]]:
        """Control messages received since the last call (at least one)."""
        while not self._msgs:
            if self._exc is not None:
                raise self._exc
            if self._eof:
                raise asyncio.IncompleteReadError(b"", None)
            self._waiter = asyncio.get_running_loop().create_future()
            try:
                await self._waiter
            finally:
                self._waiter = None
        msgs, self._msgs = self._msgs, []
        if self._paused:
            self._paused = False
            self._update_reading()
        return msgs

    def _fail(self, e: BaseException) -> None:
        if self._exc is None:
            self._exc = e
        self._wake()
        self._update_reading()

    def _wake(self) -> None:
        w = self._waiter
        if w is not None and not w.done():
            w.set_result(None)


class UtpLinkReader(LinkReader):
    """:class:`LinkReader` for a uTP stream: the uTP engine's delivered bytes
    come in through :meth:`deliver` (the stream's sink) instead of a socket
    read callback.  Pausing works as on TCP: while the send side is backed up
    (or the peer loop is behind) the transport stops handing over bytes, they
    stay in the engine and its advertised receive window closes — so a peer
    pipelining REQUESTs cannot make the served PIECE replies pile up."""

    def __init__(self, transport: asyncio.Transport, link, on_bytes) -> None:
        super().__init__(transport, link, on_bytes)
        self._empty = b""           # on_bytes(b"") parses what the link already holds

    def deliver(self, data: bytes) -> None:
        if self._exc is None:
            self.buffer_updated(data)          # on_bytes(data), errors end the loop

    def eof(self) -> None:
        self._eof = True
        self._wake()


def parse_ext_handshake(payload: bytes) -> ExtHandshake:
    try:
        d = bencode.decode(payload, allow_trailing=True)
    except bencode.BencodeError as e:
        raise PeerError(f"bad extended handshake: {e}") from e
    if not isinstance(d, dict):
        raise PeerError("extended handshake is not a dict")
    m = {}
    mm = d.get(b"m")
    for k, v in (mm.items() if isinstance(mm, dict) else ()):
        if isinstance(v, int):
            m[k.decode(errors="replace")] = v
    ms = d.get(b"metadata_size")
    return ExtHandshake(m, ms if isinstance(ms, int) and ms > 0 else None,
                        d.get(b"reqq") if isinstance(d.get(b"reqq"), int) else None,
                        (d.get(b"v") or b"").decode(errors="replace") if isinstance(d.get(b"v"), bytes) else "",
                        d.get(b"p") if isinstance(d.get(b"p"), int) else None)


def pex_msg(added: list[tuple[str, int]], dropped: list[tuple[str, int]],
            flags: dict[tuple[str, int], int] | None = None) -> bytes:
    """ut_pex payload: compact IPv4 (``added``/``dropped``) and IPv6
    (``added6``/``dropped6``) peer lists with one flag byte per added peer
    (0x02 seed, 0x04 supports uTP, 0x10 reachable/outgoing-connectable)."""
    import ipaddress
    d: dict = {}
    for key, peers in ((b"added", added), (b"dropped", dropped)):
        v4 = [a for a in peers if ":" not in a[0]]
        v6 = [a for a in peers if ":" in a[0]]
        d[key] = b"".join(ipaddress.IPv4Address(h).packed + struct.pack(">H", pt) for h, pt in v4)
        if v6:
            d[key + b"6"] = b"".join(ipaddress.IPv6Address(h).packed + struct.pack(">H", pt) for h, pt in v6)
        if key == b"added":
            fl = flags or {}
            d[b"added.f"] = bytes(fl.get(a, 0) for a in v4)
            if v6:
                d[b"added6.f"] = bytes(fl.get(a, 0) for a in v6)
    return bencode.encode(d)


def parse_pex(payload: bytes) -> tuple[list[tuple[str, int]], list[tuple[str, int]]]:
    """-> (added, dropped) from a ut_pex message (IPv4 and IPv6)."""
    import ipaddress
    try:
        d = bencode.decode(payload, allow_trailing=True)
    except bencode.BencodeError as e:
        raise PeerError(f"bad ut_pex message: {e}") from e
    if not isinstance(d, dict):
        raise PeerError("ut_pex message is not a dict")

    def compact(b, step):
        out = []
        if not isinstance(b, bytes):
            return out
        for k in range(0, len(b) - step + 1, step):
            (port,) = struct.unpack(">H", b[k + step - 2:k + step])
            if port:
                out.append((str(ipaddress.ip_address(b[k:k + step - 2])), port))
        return out
    added = compact(d.get(b"added"), 6) + compact(d.get(b"added6"), 18)
    dropped = compact(d.get(b"dropped"), 6) + compact(d.get(b"dropped6"), 18)
    return added, dropped


def parse_hash_msg(pl: bytes) -> tuple[bytes, int, int, int, int, bytes]:
    """(pieces root, base layer, index, length, proof layers, hashes) of a
    BEP 52 hash request / hashes / hash reject message."""
    if len(pl) < 48 or (len(pl) - 48) % 32:
        raise PeerError("bad v2 hash message")
    base, index, length, proofs = struct.unpack(">IIII", pl[32:48])
    return pl[:32], base, index, length, proofs, pl[48:]


def meta_msg(msg_type: int, piece: int, total_size: int | None = None, data: bytes = b"") -> bytes:
    d: dict = {b"msg_type": msg_type, b"piece": piece}
    if total_size is not None:
        d[b"total_size"] = total_size
    return bencode.encode(d) + data


def parse_meta_msg(payload: bytes) -> tuple[dict, bytes]:
    try:
        d, n = bencode.decode_prefix(payload)
    except bencode.BencodeError as e:
        raise PeerError(f"bad ut_metadata message: {e}") from e
    if not isinstance(d, dict):
        raise PeerError("bad ut_metadata message")
    return d, payload[n:]


def bits_to_set(bits: bytes, n: int) -> set[int]:
    """Pieces set in a BITFIELD; one shorter than ``n`` bits is a protocol
    violation (BEP 3: drop the connection), a PeerError."""
    if len(bits) < (n + 7) // 8:
        raise PeerError(f"bitfield of {len(bits)} bytes for {n} pieces")
    out = set()
    for i in range(n):
        if bits[i >> 3] & (0x80 >> (i & 7)):
            out.add(i)
    return out


def set_to_bits(have: set[int] | list[bool], n: int) -> bytes:
    b = bytearray((n + 7) // 8)
    it = have if isinstance(have, set) else {i for i, v in enumerate(have) if v}
    for i in it:
        b[i >> 3] |= 0x80 >> (i & 7)
    return bytes(b)
