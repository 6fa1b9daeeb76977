"""HTTP/2 client connections (RFC 9113) for the HTTP downloader.

grab's transport was Go's ``http.Transport`` (``internal/downloader/http/
http.go:18-22``), which offers ``h2`` in the TLS handshake (ALPN) and speaks
HTTP/2 to any https origin that accepts it, carrying every request to that
origin as a stream of one TCP connection.  :class:`H2Connection` does the
same for :class:`~tritondl.fetch.http.HTTPDownloader` (``http2=True``): a job's
probe and its Range segments become concurrent streams of one connection
per origin.  An origin that answers ALPN with ``http/1.1`` (or nothing) is
remembered and served by the HTTP/1.1 paths.

What is implemented is what a downloading client needs: the connection
preface and SETTINGS exchange, HEADERS + CONTINUATION with HPACK
(:mod:`tritondl.utils.hpack`), DATA with padding, receive flow control with
large windows (16 MiB per stream, 256 MiB per connection) replenished as the
body is consumed (back-pressure reaches the server), RST_STREAM, PING,
GOAWAY (streams above the last processed id fail retryably), and
SETTINGS_MAX_CONCURRENT_STREAMS.  Server push is disabled.

Two transports carry the frames:

* **native** (:meth:`H2Connection.open_native`, the downloader's default when
  the relay extension is built): the relay's OpenSSL session, owned by one
  ``_relay.H2Session`` pump thread (``csrc/relay/h2.h``).  DATA payloads go
  from the decrypted records straight into the download's file at the
  stream's offset and onto its ``Flow`` (:meth:`H2Stream.sink`), and the
  window credit is returned there.  The other frames reach this module as
  events on an eventfd the event loop watches; this module's frames go back
  through the pump in order.
* **asyncio** (:meth:`H2Connection.open`): asyncio's TLS, every frame parsed
  here and bodies read with :meth:`H2Stream.read`.
"""

from __future__ import annotations

import asyncio
import collections
import ssl
import struct
import time

from multidict import CIMultiDict

from ..utils import dial
from ..utils.hpack import Decoder, Encoder, HPACKError

PREFACE = b"PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n"
DATA, HEADERS, PRIORITY, RST_STREAM, SETTINGS, PUSH_PROMISE, PING, GOAWAY, WINDOW_UPDATE, CONTINUATION = range(10)
END_STREAM = ACK = 0x1
END_HEADERS = 0x4
PADDED = 0x8
PRIORITY_FLAG = 0x20
S_HEADER_TABLE_SIZE, S_ENABLE_PUSH, S_MAX_CONCURRENT_STREAMS, S_INITIAL_WINDOW_SIZE, S_MAX_FRAME_SIZE, \
    S_MAX_HEADER_LIST_SIZE = range(1, 7)
NO_ERROR, PROTOCOL_ERROR, INTERNAL_ERROR, FLOW_CONTROL_ERROR, SETTINGS_TIMEOUT, STREAM_CLOSED, FRAME_SIZE_ERROR, \
    REFUSED_STREAM, CANCEL, COMPRESSION_ERROR = range(10)

STREAM_WINDOW = 16 << 20          # what the server may send on one stream before we consume it
CONN_WINDOW = 256 << 20           # ... on the whole connection
MAX_FRAME = 1 << 20               # largest frame we accept (the server may use 16 KiB..this)

# native pump events beyond frame types (csrc/relay/h2.h)
SINK_DONE, SINK_ERROR, CONN_ERROR = 0x100, 0x101, 0x102


def frame(ftype: int, flags: int, stream: int, payload: bytes = b"") -> bytes:
    n = len(payload)
    return struct.pack(">BHBBI", n >> 16, n & 0xFFFF, ftype, flags, stream & 0x7FFFFFFF) + payload


def _preface() -> bytes:
    return (PREFACE + frame(SETTINGS, 0, 0, struct.pack(">HIHIHIHI", S_ENABLE_PUSH, 0, S_INITIAL_WINDOW_SIZE,
                                                        STREAM_WINDOW, S_MAX_FRAME_SIZE, MAX_FRAME,
                                                        S_HEADER_TABLE_SIZE, 4096))
            + frame(WINDOW_UPDATE, 0, 0, struct.pack(">I", CONN_WINDOW - 65535)))


_FIXED_LEN = {PRIORITY: 5, RST_STREAM: 4, PING: 8, WINDOW_UPDATE: 4}   # RFC 9113 6.3-6.9


class H2Error(ConnectionError):
    """The connection failed (a protocol error, GOAWAY for this stream, EOF).
    ``written``: body bytes a native file sink had written before it."""
    written = 0


class StreamReset(H2Error):
    def __init__(self, stream: int, code: int) -> None:
        super().__init__(f"stream {stream} reset by the server (error code {code})")
        self.code = code


class H2Stream:
    """One request's response: ``status`` / ``headers`` once :meth:`response`
    returns, then the body through :meth:`read` or (native) :meth:`sink`."""

    def __init__(self, conn: "H2Connection", sid: int) -> None:
        self.conn, self.id = conn, sid
        self.status = 0
        self.headers: CIMultiDict = CIMultiDict()
        self._head = asyncio.get_running_loop().create_future()
        self._chunks: collections.deque = collections.deque()
        self._event = asyncio.Event()
        self.eof = False
        self.error: BaseException | None = None
        self._unacked = 0                  # bytes consumed and not yet returned as window credit
        self.window = STREAM_WINDOW        # bytes the server may still send on this stream
        self.buffered = 0                  # body bytes received and not yet read
        self.body_read = 0
        self.limit: int | None = None      # body bytes the reader will take in all (see want())
        self._sink: asyncio.Future | None = None
        self._events = False               # native: body delivered as events (read())

    async def response(self) -> "H2Stream":
        await self._head
        return self

    def _fail(self, e: BaseException) -> None:
        if self.error is None and not self.eof:
            self.error = e
        if not self._head.done():
            self._head.set_exception(e)
        if self._sink is not None and not self._sink.done():
            self._sink.set_exception(e)
        self._event.set()
        if self.conn._native is not None:
            self.conn._native.drop(self.id)

    async def read(self, n: int = -1) -> bytes:
        """Up to ``n`` body bytes (all that is buffered for ``n < 0``); b"" at
        the end of the body."""
        if self.conn._native is not None and not self._events and not self.eof and self.error is None:
            self._events = True
            self.conn._native.sink_events(self.id)
        while not self._chunks:
            if self.error is not None:
                raise self.error
            if self.eof:
                return b""
            self._event.clear()
            await self._event.wait()
        c = self._chunks.popleft()
        if 0 <= n < len(c):
            self._chunks.appendleft(c[n:])
            c = c[:n]
        self.buffered -= len(c)
        self.body_read += len(c)
        self.conn._consumed(self, len(c))
        return c

    async def sink(self, fd: int, offset: int, limit: int, flow, seg: int = 0, done0: int = 0,
                   idle_timeout: float = 120.0) -> tuple[int, bool]:
        """Native connections: the pump writes the body into ``fd`` at
        ``offset`` (at most ``limit`` bytes, < 0 = to the end), publishing
        ``done0 + written`` on ``flow`` segment ``seg``.  Returns (bytes
        written, END_STREAM seen); False means the limit was reached with
        more body to come (cancel the stream).  A stream that writes nothing
        for ``idle_timeout`` seconds fails retryably; every failure's
        :class:`H2Error` carries ``written``."""
        native = self.conn._native
        if native is None:
            raise RuntimeError("sink() needs a native HTTP/2 connection")
        if self.error is not None:
            raise self.error
        if self.eof:
            return 0, True                          # the response had no body
        loop = asyncio.get_running_loop()
        self._sink = loop.create_future()
        self.conn._sinks[self.id] = self            # the pump's answer is routed here
        native.sink_file(self.id, fd, offset, limit, flow, seg, done0)
        last = -1
        try:
            while True:
                try:
                    return await asyncio.wait_for(asyncio.shield(self._sink), idle_timeout)
                except asyncio.TimeoutError:
                    if self._sink.done():
                        return self._sink.result()
                    n = native.written(self.id)
                    if n == last:
                        e = H2Error(f"HTTP/2 stream {self.id}: no body bytes for {idle_timeout:g} s")
                        e.written = n
                        self.cancel()
                        raise e from None
                    last = n
        except asyncio.CancelledError:
            # the download is being torn down: the pump must stop writing into fd before the
            # caller closes it (drop() returns only once no write is in flight)
            self.cancel()
            raise

    def _sink_done(self, written: int, eof: bool) -> None:
        self.eof = eof
        if self._sink is not None and not self._sink.done():
            self._sink.set_result((written, eof))

    def _sink_failed(self, why: str, written: int) -> None:
        e = H2Error(f"HTTP/2 stream {self.id}: {why}")
        e.written = written
        if self._sink is not None and not self._sink.done():
            self._sink.set_exception(e)

    def want(self, n: int) -> None:
        """The reader takes only ``n`` more body bytes (then cancels): window
        credit stops there, so the server overshoots by no more than what
        was already granted.  A probe stream opened at ``bytes=0-`` that
        becomes segment 0 uses this to keep the next segments' bytes from
        being sent twice."""
        self.limit = self.body_read + n

    def at_eof(self) -> bool:
        return self.eof and not self._chunks

    def cancel(self) -> None:
        """Stop the response (RST_STREAM CANCEL) unless it has ended."""
        if not self.eof and self.error is None:
            self.error = H2Error("cancelled")
            self.conn._reset(self.id, CANCEL)
        self.conn.streams.pop(self.id, None)
        self.conn._slots.set()


class H2Connection:
    def __init__(self, reader: asyncio.StreamReader | None, writer, authority: str, native=None) -> None:
        self.r, self.w = reader, writer
        self.authority = authority
        self.streams: dict[int, H2Stream] = {}
        self.next_id = 1
        self.peer = {S_MAX_CONCURRENT_STREAMS: 1 << 31, S_MAX_FRAME_SIZE: 16384, S_HEADER_TABLE_SIZE: 4096}
        self.encoder = Encoder(huffman=True, index=False)
        self.decoder = Decoder(4096)
        self.closed: BaseException | None = None
        self.goaway_last: int | None = None
        self._conn_unacked = 0
        self._slots = asyncio.Event()
        self._slots.set()
        self._reader: asyncio.Task | None = None
        self.streams_opened = 0
        self._hblock: bytearray | None = None      # header block being assembled (HEADERS + CONTINUATION)
        self._hstream = self._hflags = 0
        self._native = native                      # _relay.H2Session (native transport)
        self._raw = None                           # its rawhttp.RawConn (owns the socket)
        self._sinks: dict[int, H2Stream] = {}      # native: streams whose body a pump sink takes
        self.last_active = time.monotonic()        # last request or frame (idle-connection reaping)
        self.pending = 0                           # requests a caller has picked this connection for

    @classmethod
    async def open(cls, host: str, port: int, ctx: ssl.SSLContext, *, timeout: float = 30.0) -> "H2Connection | None":
        """asyncio transport: dial (fast fallback, keep-alive) and handshake
        offering ``h2``; None when the server picks HTTP/1.1 (or no protocol)."""
        ctx.set_alpn_protocols(["h2", "http/1.1"])
        r, w = await asyncio.wait_for(dial.open_connection(host, port, timeout=timeout, ssl=ctx), timeout)
        sslobj = w.get_extra_info("ssl_object")
        if sslobj is None or sslobj.selected_alpn_protocol() != "h2":
            w.close()
            return None
        c = cls(r, w, host if port == 443 else f"{host}:{port}")
        w.write(_preface())
        await w.drain()
        c._reader = asyncio.ensure_future(c._read_loop())
        return c

    @classmethod
    async def open_native(cls, host: str, port: int, tls_ctx, *, timeout: float = 30.0) -> "H2Connection | None":
        """Native transport: dial, TLS handshake in the relay (``tls_ctx``: a
        ``_relay.TlsContext``) offering ``h2``, then hand the session to a
        ``_relay.H2Session`` pump; None when the server picks HTTP/1.1."""
        from ..utils import rawhttp
        relay = rawhttp.relay_module()
        s = await rawhttp._dial(host, port, timeout)
        try:
            t = relay.TlsConn(tls_ctx, s.fileno(), host, f"{host}:{port}")
            t.set_alpn(["h2", "http/1.1"])
            raw = rawhttp.RawConn(s, t)
            await raw.handshake(timeout)
        except BaseException:
            s.close()
            raise
        if t.alpn != "h2":
            raw.close()
            return None
        sess = relay.H2Session(t, STREAM_WINDOW, CONN_WINDOW, MAX_FRAME)
        c = cls(None, None, host if port == 443 else f"{host}:{port}", native=sess)
        c._raw = raw
        sess.send(_preface())
        sess.start()
        asyncio.get_running_loop().add_reader(sess.fileno(), c._on_native_events)
        return c

    @property
    def native(self) -> bool:
        return self._native is not None

    @property
    def alive(self) -> bool:
        return self.closed is None and self.goaway_last is None

    def idle_for(self, now: float) -> float:
        """Seconds without a stream open (0 while one is)."""
        return 0.0 if self.streams or self._sinks or self.pending else now - self.last_active

    @property
    def load(self) -> int:
        """Open streams plus the requests about to open one."""
        return len(self.streams) + self.pending

    def _write(self, data: bytes) -> None:
        if self._native is not None:
            self._native.send(data)
        else:
            self.w.write(data)

    # ------------------------------------------------------------ requests
    async def request(self, headers: list[tuple[bytes, bytes]]) -> H2Stream:
        """Send a GET (``headers`` include the pseudo-headers) as a new stream."""
        while len(self.streams) >= self.peer[S_MAX_CONCURRENT_STREAMS]:
            if not self.alive:
                break
            self._slots.clear()
            await self._slots.wait()
        if not self.alive:
            raise H2Error(f"connection to {self.authority} is closing: {self.closed or 'GOAWAY'}")
        sid = self.next_id
        self.next_id += 2
        self.last_active = time.monotonic()
        st = H2Stream(self, sid)
        self.streams[sid] = st
        self.streams_opened += 1
        block = self.encoder.encode(headers)
        mx = self.peer[S_MAX_FRAME_SIZE]
        first, rest = block[:mx], block[mx:]
        out = [frame(HEADERS, END_STREAM | (0 if rest else END_HEADERS), sid, first)]
        while rest:
            part, rest = rest[:mx], rest[mx:]
            out.append(frame(CONTINUATION, 0 if rest else END_HEADERS, sid, part))
        if self._native is not None:
            self._native.open_stream(sid)
            self._sinks[sid] = st
            self._native.send(b"".join(out))
        else:
            self.w.write(b"".join(out))      # one write: no other frame can land between them
            await self.w.drain()
        return st

    def _reset(self, sid: int, code: int) -> None:
        if self._native is not None:
            self._native.drop(sid)
            self._sinks.pop(sid, None)
        if self.closed is None:
            self._write(frame(RST_STREAM, 0, sid, struct.pack(">I", code)))
        self._slots.set()

    def _consumed(self, st: H2Stream | None, n: int) -> None:
        """Return window credit once a quarter of a window has been read (or
        the stream's window runs low), never past a stream's ``limit``.  The
        native pump returns its own credit."""
        if self._native is not None:
            return
        self._conn_unacked += n
        out = []
        if st is not None:
            st._unacked += n
        if st is not None and st._unacked and not st.eof:
            inc = st._unacked
            if st.limit is not None:
                need = st.limit - st.body_read - st.buffered
                inc = min(inc, max(0, need - st.window))
            if inc and (inc >= STREAM_WINDOW // 4 or st.window < STREAM_WINDOW // 4):
                out.append(frame(WINDOW_UPDATE, 0, st.id, struct.pack(">I", inc)))
                st._unacked -= inc
                st.window += inc
        if self._conn_unacked >= CONN_WINDOW // 4:
            out.append(frame(WINDOW_UPDATE, 0, 0, struct.pack(">I", self._conn_unacked)))
            self._conn_unacked = 0
        if out and self.closed is None:
            self.w.write(b"".join(out))

    async def close(self) -> None:
        if self.closed is None:
            self.closed = H2Error("closed by client")
            try:
                self._write(frame(GOAWAY, 0, 0, struct.pack(">II", 0, NO_ERROR)))
                if self.w is not None:
                    self.w.close()
            except (ConnectionError, RuntimeError):
                pass
        if self._reader is not None:
            self._reader.cancel()
        for st in list(self.streams.values()):
            st._fail(self.closed)
        if self._native is not None:
            await asyncio.get_running_loop().run_in_executor(None, self._native.close)
            self._stop_native()

    def _stop_native(self) -> None:
        """The pump has stopped (or is stopping): unwatch it, close the socket."""
        try:
            asyncio.get_running_loop().remove_reader(self._native.fileno())
        except (RuntimeError, ValueError):
            pass
        if self._raw is not None:
            self._raw.close()
            self._raw = None

    def _fail_conn(self, err: BaseException) -> None:
        if self.closed is None:
            self.closed = err
        for st in list(self.streams.values()) + list(self._sinks.values()):
            st._fail(err)
        self.streams.clear()
        self._sinks.clear()
        self._slots.set()

    # ------------------------------------------------------------ frames in
    async def _read_loop(self) -> None:
        try:
            while True:
                head = await self.r.readexactly(9)
                ln = (head[0] << 16) | (head[1] << 8) | head[2]
                ftype, flags = head[3], head[4]
                sid = struct.unpack(">I", head[5:9])[0] & 0x7FFFFFFF
                if ln > MAX_FRAME:
                    raise H2Error(f"frame of {ln} bytes above the {MAX_FRAME} we allow")
                payload = await self.r.readexactly(ln) if ln else b""
                self._on_frame(ftype, flags, sid, payload)
        except asyncio.CancelledError:
            return
        except Exception as e:  # noqa: BLE001 - whatever the server sent, every stream fails instead of hanging
            self._fail_conn(self._conn_error(e))
            try:
                self.w.close()
            except RuntimeError:
                pass

    def _conn_error(self, e: BaseException) -> H2Error:
        if isinstance(e, H2Error):
            return e
        if isinstance(e, HPACKError):
            return H2Error(f"HTTP/2 header block from {self.authority} does not decode: {e}")
        return H2Error(f"HTTP/2 connection to {self.authority}: {e!r}")

    def _on_native_events(self) -> None:
        """The pump's eventfd is readable: handle its frames and sink results."""
        native = self._native
        try:
            events = native.take_events()
        except RuntimeError as e:
            events = [(CONN_ERROR, 0, 0, str(e).encode(), 0)]
        for ftype, flags, sid, payload, n in events:
            if ftype < 256:
                try:
                    self._on_frame(ftype, flags, sid, payload)
                except Exception as e:  # noqa: BLE001 - a protocol error ends the connection
                    self._fail_conn(self._conn_error(e))
                    native.close()
                    self._stop_native()
                    return
            elif ftype == SINK_DONE:
                self.last_active = time.monotonic()
                st = self._sinks.pop(sid, None)
                if st is not None:
                    self.streams.pop(sid, None)
                    self._slots.set()
                    st._sink_done(n, bool(flags & 1))
            elif ftype == SINK_ERROR:
                st = self._sinks.pop(sid, None)
                if st is not None:
                    st._sink_failed(payload.decode("utf-8", "replace"), n)
            elif ftype == CONN_ERROR:
                self._fail_conn(H2Error(f"HTTP/2 connection to {self.authority}: "
                                        f"{payload.decode('utf-8', 'replace')}"))
                self._stop_native()
                return

    def _on_frame(self, ftype: int, flags: int, sid: int, payload: bytes) -> None:
        """One frame from the server (any transport); H2Error on a protocol error."""
        self.last_active = time.monotonic()
        ln = len(payload)
        want = _FIXED_LEN.get(ftype)
        if want is not None and ln != want or ftype == GOAWAY and ln < 8 or ftype == SETTINGS and ln % 6:
            raise H2Error(f"frame type {ftype} with a {ln}-byte payload (FRAME_SIZE_ERROR)")
        if self._hblock is not None and (ftype != CONTINUATION or sid != self._hstream):
            raise H2Error("header block interrupted by another frame")
        if ftype == DATA:
            self._on_data(sid, flags, payload)
        elif ftype in (HEADERS, CONTINUATION):
            if ftype == HEADERS:
                self._hblock = bytearray(self._strip(flags, payload, ftype))
                self._hstream, self._hflags = sid, flags
            else:
                if self._hblock is None:
                    raise H2Error("CONTINUATION without HEADERS")
                self._hblock += payload
            if flags & END_HEADERS:
                block, self._hblock = bytes(self._hblock), None
                self._on_headers(self._hstream, self._hflags, block)
        elif ftype == RST_STREAM:
            st = self.streams.pop(sid, None)
            self._sinks.pop(sid, None)
            if st is not None:
                st._fail(StreamReset(sid, struct.unpack(">I", payload)[0]))
            self._slots.set()
        elif ftype == SETTINGS:
            if not flags & ACK:
                for k in range(0, ln, 6):
                    key, val = struct.unpack(">HI", payload[k:k + 6])
                    self.peer[key] = val
                self._write(frame(SETTINGS, ACK, 0))
                self._slots.set()
        elif ftype == PING:
            if not flags & ACK:
                self._write(frame(PING, ACK, 0, payload))
        elif ftype == GOAWAY:
            last, code = struct.unpack(">II", payload[:8])
            self.goaway_last = last & 0x7FFFFFFF
            for k, st in list(self.streams.items()):
                if k > self.goaway_last:
                    self.streams.pop(k, None)
                    self._sinks.pop(k, None)
                    st._fail(H2Error(f"GOAWAY (code {code}): stream {k} was not processed; retry it"))
            self._slots.set()
        elif ftype == PUSH_PROMISE:
            raise H2Error("PUSH_PROMISE with push disabled")
        # WINDOW_UPDATE (we send no DATA), PRIORITY and unknown types are ignored

    @staticmethod
    def _strip(flags: int, payload: bytes, ftype: int) -> bytes:
        pad = 0
        if flags & PADDED:
            if not payload:
                raise H2Error("padded frame without a pad length")
            pad = payload[0]
            payload = payload[1:]
        if ftype == HEADERS and flags & PRIORITY_FLAG:
            payload = payload[5:]
        if pad:
            if pad > len(payload):
                raise H2Error("padding longer than the frame")
            payload = payload[:-pad]
        return payload

    def _on_data(self, sid: int, flags: int, payload: bytes) -> None:
        st = self.streams.get(sid)
        if st is None and self._native is not None:
            st = self._sinks.get(sid)               # ended by trailers, body still being delivered
        if self._native is not None:
            # events-mode body from the pump: padding stripped, flow control done there
            body = payload
        else:
            body = self._strip(flags, payload, DATA)
        if st is None:
            # a stream we reset or finished: its bytes still count against the connection window
            self._consumed(None, len(payload))
            return
        if not st._head.done():                     # RFC 9113 8.1: a response starts with HEADERS
            self._stream_error(st, H2Error(f"DATA before the response head on stream {sid}"))
            self._consumed(None, len(payload))
            return
        if self._native is None:
            st.window -= len(payload)
            if len(payload) > len(body):                # padding is flow-controlled too
                st._unacked += len(payload) - len(body)
                self._conn_unacked += len(payload) - len(body)
        if body:
            st._chunks.append(body)
            st.buffered += len(body)
        if flags & END_STREAM:
            st.eof = True
            self.streams.pop(sid, None)
            self._sinks.pop(sid, None)
            self._slots.set()
        st._event.set()

    def _stream_error(self, st: H2Stream, e: H2Error) -> None:
        """Fail one stream (RST_STREAM PROTOCOL_ERROR); the connection lives on."""
        self.streams.pop(st.id, None)
        self._sinks.pop(st.id, None)
        st._fail(e)
        self._reset(st.id, PROTOCOL_ERROR)

    def _on_headers(self, sid: int, flags: int, block: bytes) -> None:
        fields = self.decoder.decode(block)        # always: the HPACK state must follow every block
        st = self.streams.get(sid)
        if st is None:
            return
        head_now = False
        if not st._head.done():
            status = next((v for n, v in fields if n == b":status"), None)
            if status is None:
                raise H2Error(f"response on stream {sid} without :status")
            try:
                code = int(status)
            except ValueError:
                raise H2Error(f"response on stream {sid} with :status {status!r}") from None
            if 100 <= code < 200:
                if flags & END_STREAM:
                    self._stream_error(st, H2Error(f"stream {sid} ended after an informational {code}"))
                return                                  # informational: the real head follows
            st.status = code
            st.headers = CIMultiDict((n.decode("latin-1"), v.decode("latin-1")) for n, v in fields
                                     if not n.startswith(b":"))
            st._head.set_result(st)
            head_now = True
        if flags & END_STREAM:                          # (trailers are read and dropped)
            if self._native is not None and st._head.done() and st.status and not head_now:
                # trailers: the pump has ended (or will end) the stream's sink itself
                self.streams.pop(sid, None)
                self._slots.set()
                return
            st.eof = True
            self.streams.pop(sid, None)
            self._slots.set()
            st._event.set()
            if self._native is not None and head_now:
                self._sinks.pop(sid, None)              # a bodiless response: nothing to sink
                self._native.drop(sid)


__all__ = ["H2Connection", "H2Stream", "H2Error", "StreamReset", "frame"]
