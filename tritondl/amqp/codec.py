"""AMQP 0-9-1 wire codec: frames, method arguments, field tables, content
headers.  Written from the AMQP 0-9-1 specification (RabbitMQ field-table
type set); no client library is available offline.

The reference uses streadway/amqp for this (``internal/rabbitmq/client.go``,
SURVEY.md Appendix C).  Methods actually exercised there: Dial handshake,
Channel/Qos, ExchangeDeclare, QueueDeclare, QueueBind, Consume, Publish,
Ack, Nack (``client.go:224,248,309,333,347,351,366-368``,
``delivery.go:56,61,78``); we implement the full basic/queue/exchange/
channel/connection/confirm subset so that the fake broker and the client
share one codec.
"""

from __future__ import annotations

import struct
from dataclasses import dataclass, field
from datetime import datetime, timezone
from decimal import Decimal
from typing import Any

PROTOCOL_HEADER = b"AMQP\x00\x00\x09\x01"
FRAME_METHOD, FRAME_HEADER, FRAME_BODY, FRAME_HEARTBEAT = 1, 2, 3, 8
FRAME_END = 0xCE
FRAME_MIN_SIZE = 4096
DEFAULT_FRAME_MAX = 131072

# reply codes
REPLY_SUCCESS = 200
CONTENT_TOO_LARGE = 311
NO_ROUTE = 312
NO_CONSUMERS = 313
CONNECTION_FORCED = 320
INVALID_PATH = 402
ACCESS_REFUSED = 403
NOT_FOUND = 404
RESOURCE_LOCKED = 405
PRECONDITION_FAILED = 406
FRAME_ERROR = 501
SYNTAX_ERROR = 502
COMMAND_INVALID = 503
CHANNEL_ERROR = 504
UNEXPECTED_FRAME = 505
RESOURCE_ERROR = 506
NOT_ALLOWED = 530
NOT_IMPLEMENTED = 540
INTERNAL_ERROR = 541


class AMQPError(Exception):
    pass


class FrameError(AMQPError):
    pass


# ----------------------------------------------------------------- methods
# (class_id, method_id) -> (name, [(arg, type), ...], has_content, is_sync_request_expecting)
_o, _s, _l, _ll, _ss, _ls, _b, _t = "octet", "short", "long", "longlong", "shortstr", "longstr", "bit", "table"

METHODS: dict[tuple[int, int], tuple[str, list[tuple[str, str]]]] = {
    (10, 10): ("connection.start", [("version_major", _o), ("version_minor", _o), ("server_properties", _t),
                                    ("mechanisms", _ls), ("locales", _ls)]),
    (10, 11): ("connection.start_ok", [("client_properties", _t), ("mechanism", _ss), ("response", _ls),
                                       ("locale", _ss)]),
    (10, 20): ("connection.secure", [("challenge", _ls)]),
    (10, 21): ("connection.secure_ok", [("response", _ls)]),
    (10, 30): ("connection.tune", [("channel_max", _s), ("frame_max", _l), ("heartbeat", _s)]),
    (10, 31): ("connection.tune_ok", [("channel_max", _s), ("frame_max", _l), ("heartbeat", _s)]),
    (10, 40): ("connection.open", [("virtual_host", _ss), ("capabilities", _ss), ("insist", _b)]),
    (10, 41): ("connection.open_ok", [("known_hosts", _ss)]),
    (10, 50): ("connection.close", [("reply_code", _s), ("reply_text", _ss), ("class_id", _s), ("method_id", _s)]),
    (10, 51): ("connection.close_ok", []),
    (10, 60): ("connection.blocked", [("reason", _ss)]),
    (10, 61): ("connection.unblocked", []),
    (20, 10): ("channel.open", [("out_of_band", _ss)]),
    (20, 11): ("channel.open_ok", [("channel_id", _ls)]),
    (20, 20): ("channel.flow", [("active", _b)]),
    (20, 21): ("channel.flow_ok", [("active", _b)]),
    (20, 40): ("channel.close", [("reply_code", _s), ("reply_text", _ss), ("class_id", _s), ("method_id", _s)]),
    (20, 41): ("channel.close_ok", []),
    (40, 10): ("exchange.declare", [("ticket", _s), ("exchange", _ss), ("type", _ss), ("passive", _b),
                                    ("durable", _b), ("auto_delete", _b), ("internal", _b), ("nowait", _b),
                                    ("arguments", _t)]),
    (40, 11): ("exchange.declare_ok", []),
    (40, 20): ("exchange.delete", [("ticket", _s), ("exchange", _ss), ("if_unused", _b), ("nowait", _b)]),
    (40, 21): ("exchange.delete_ok", []),
    (40, 30): ("exchange.bind", [("ticket", _s), ("destination", _ss), ("source", _ss), ("routing_key", _ss),
                                 ("nowait", _b), ("arguments", _t)]),
    (40, 31): ("exchange.bind_ok", []),
    (40, 40): ("exchange.unbind", [("ticket", _s), ("destination", _ss), ("source", _ss), ("routing_key", _ss),
                                   ("nowait", _b), ("arguments", _t)]),
    (40, 51): ("exchange.unbind_ok", []),
    (50, 10): ("queue.declare", [("ticket", _s), ("queue", _ss), ("passive", _b), ("durable", _b),
                                 ("exclusive", _b), ("auto_delete", _b), ("nowait", _b), ("arguments", _t)]),
    (50, 11): ("queue.declare_ok", [("queue", _ss), ("message_count", _l), ("consumer_count", _l)]),
    (50, 20): ("queue.bind", [("ticket", _s), ("queue", _ss), ("exchange", _ss), ("routing_key", _ss),
                              ("nowait", _b), ("arguments", _t)]),
    (50, 21): ("queue.bind_ok", []),
    (50, 30): ("queue.purge", [("ticket", _s), ("queue", _ss), ("nowait", _b)]),
    (50, 31): ("queue.purge_ok", [("message_count", _l)]),
    (50, 40): ("queue.delete", [("ticket", _s), ("queue", _ss), ("if_unused", _b), ("if_empty", _b),
                                ("nowait", _b)]),
    (50, 41): ("queue.delete_ok", [("message_count", _l)]),
    (50, 50): ("queue.unbind", [("ticket", _s), ("queue", _ss), ("exchange", _ss), ("routing_key", _ss),
                                ("arguments", _t)]),
    (50, 51): ("queue.unbind_ok", []),
    (60, 10): ("basic.qos", [("prefetch_size", _l), ("prefetch_count", _s), ("global_", _b)]),
    (60, 11): ("basic.qos_ok", []),
    (60, 20): ("basic.consume", [("ticket", _s), ("queue", _ss), ("consumer_tag", _ss), ("no_local", _b),
                                 ("no_ack", _b), ("exclusive", _b), ("nowait", _b), ("arguments", _t)]),
    (60, 21): ("basic.consume_ok", [("consumer_tag", _ss)]),
    (60, 30): ("basic.cancel", [("consumer_tag", _ss), ("nowait", _b)]),
    (60, 31): ("basic.cancel_ok", [("consumer_tag", _ss)]),
    (60, 40): ("basic.publish", [("ticket", _s), ("exchange", _ss), ("routing_key", _ss), ("mandatory", _b),
                                 ("immediate", _b)]),
    (60, 50): ("basic.return", [("reply_code", _s), ("reply_text", _ss), ("exchange", _ss), ("routing_key", _ss)]),
    (60, 60): ("basic.deliver", [("consumer_tag", _ss), ("delivery_tag", _ll), ("redelivered", _b),
                                 ("exchange", _ss), ("routing_key", _ss)]),
    (60, 70): ("basic.get", [("ticket", _s), ("queue", _ss), ("no_ack", _b)]),
    (60, 71): ("basic.get_ok", [("delivery_tag", _ll), ("redelivered", _b), ("exchange", _ss),
                                ("routing_key", _ss), ("message_count", _l)]),
    (60, 72): ("basic.get_empty", [("cluster_id", _ss)]),
    (60, 80): ("basic.ack", [("delivery_tag", _ll), ("multiple", _b)]),
    (60, 90): ("basic.reject", [("delivery_tag", _ll), ("requeue", _b)]),
    (60, 100): ("basic.recover_async", [("requeue", _b)]),
    (60, 110): ("basic.recover", [("requeue", _b)]),
    (60, 111): ("basic.recover_ok", []),
    (60, 120): ("basic.nack", [("delivery_tag", _ll), ("multiple", _b), ("requeue", _b)]),
    (85, 10): ("confirm.select", [("nowait", _b)]),
    (85, 11): ("confirm.select_ok", []),
}
BY_NAME = {v[0]: k for k, v in METHODS.items()}
CONTENT_METHODS = {"basic.publish", "basic.return", "basic.deliver", "basic.get_ok"}


@dataclass
class Method:
    name: str
    args: dict[str, Any] = field(default_factory=dict)

    @property
    def ids(self) -> tuple[int, int]:
        return BY_NAME[self.name]

    def __getattr__(self, item: str) -> Any:
        try:
            return self.__dict__["args"][item]
        except KeyError:
            raise AttributeError(item) from None


def _default(t: str) -> Any:
    return {"bit": False, "table": {}, "shortstr": "", "longstr": b""}.get(t, 0)


# ------------------------------------------------------------ field tables


def _enc_shortstr(s: str | bytes) -> bytes:
    b = s.encode() if isinstance(s, str) else s
    if len(b) > 255:
        raise AMQPError("shortstr too long")
    return bytes([len(b)]) + b


def _enc_longstr(s: str | bytes) -> bytes:
    b = s.encode() if isinstance(s, str) else bytes(s)
    return struct.pack(">I", len(b)) + b


def _enc_value(v: Any) -> bytes:
    if isinstance(v, bool):
        return b"t" + (b"\x01" if v else b"\x00")
    if isinstance(v, int):
        if -(2**31) <= v < 2**31:
            return b"I" + struct.pack(">i", v)
        return b"l" + struct.pack(">q", v)
    if isinstance(v, float):
        return b"d" + struct.pack(">d", v)
    if isinstance(v, Decimal):
        sign, digits, exp = v.as_tuple()
        places = max(0, -int(exp))
        unscaled = int(v.scaleb(places))
        return b"D" + struct.pack(">Bi", places, unscaled)
    if isinstance(v, str):
        return b"S" + _enc_longstr(v)
    if isinstance(v, (bytes, bytearray)):
        return b"x" + _enc_longstr(bytes(v))
    if isinstance(v, datetime):
        return b"T" + struct.pack(">Q", int(v.timestamp()))
    if isinstance(v, dict):
        return b"F" + encode_table(v)
    if isinstance(v, (list, tuple)):
        inner = b"".join(_enc_value(x) for x in v)
        return b"A" + struct.pack(">I", len(inner)) + inner
    if v is None:
        return b"V"
    raise AMQPError(f"unsupported table value type {type(v)}")


def encode_table(t: dict | None) -> bytes:
    if not t:
        return b"\x00\x00\x00\x00"
    body = b"".join(_enc_shortstr(k) + _enc_value(v) for k, v in t.items())
    return struct.pack(">I", len(body)) + body


class _Reader:
    __slots__ = ("buf", "pos", "bitbuf", "bitpos")

    def __init__(self, buf: bytes, pos: int = 0) -> None:
        self.buf = buf
        self.pos = pos
        self.bitbuf = 0
        self.bitpos = 8

    def take(self, n: int) -> bytes:
        if self.pos + n > len(self.buf):
            raise FrameError("truncated payload")
        b = self.buf[self.pos:self.pos + n]
        self.pos += n
        return b

    def unpack(self, fmt: str):
        sz = struct.calcsize(fmt)
        return struct.unpack(fmt, self.take(sz))

    def octet(self) -> int:
        self.bitpos = 8
        return self.take(1)[0]

    def short(self) -> int:
        self.bitpos = 8
        return self.unpack(">H")[0]

    def long(self) -> int:
        self.bitpos = 8
        return self.unpack(">I")[0]

    def longlong(self) -> int:
        self.bitpos = 8
        return self.unpack(">Q")[0]

    def shortstr(self) -> str:
        self.bitpos = 8
        n = self.take(1)[0]
        return self.take(n).decode("utf-8", "surrogateescape")

    def longstr(self) -> bytes:
        self.bitpos = 8
        n = self.unpack(">I")[0]
        return bytes(self.take(n))

    def bit(self) -> bool:
        if self.bitpos >= 8:
            self.bitbuf = self.take(1)[0]
            self.bitpos = 0
        v = bool(self.bitbuf & (1 << self.bitpos))
        self.bitpos += 1
        return v

    def table(self) -> dict:
        self.bitpos = 8
        n = self.unpack(">I")[0]
        end = self.pos + n
        if end > len(self.buf):
            raise FrameError("truncated table")
        out = {}
        while self.pos < end:
            k = self.shortstr()
            out[k] = self.value()
        if self.pos != end:
            raise FrameError("table length mismatch")
        return out

    def value(self) -> Any:
        t = self.take(1)
        if t == b"t":
            return self.take(1)[0] != 0
        if t == b"b":
            return self.unpack(">b")[0]
        if t == b"B":
            return self.unpack(">B")[0]
        if t == b"s":
            return self.unpack(">h")[0]
        if t == b"u":
            return self.unpack(">H")[0]
        if t == b"I":
            return self.unpack(">i")[0]
        if t == b"i":
            return self.unpack(">I")[0]
        if t in (b"l", b"L"):
            return self.unpack(">q")[0]
        if t == b"f":
            return self.unpack(">f")[0]
        if t == b"d":
            return self.unpack(">d")[0]
        if t == b"D":
            places, val = self.unpack(">Bi")
            return Decimal(val).scaleb(-places)
        if t == b"S":
            raw = self.longstr()
            try:
                return raw.decode("utf-8")
            except UnicodeDecodeError:
                return raw
        if t == b"x":
            return self.longstr()
        if t == b"A":
            n = self.unpack(">I")[0]
            end = self.pos + n
            arr = []
            while self.pos < end:
                arr.append(self.value())
            return arr
        if t == b"T":
            return datetime.fromtimestamp(self.unpack(">Q")[0], tz=timezone.utc)
        if t == b"F":
            return self.table()
        if t == b"V":
            return None
        raise FrameError(f"unknown field type {t!r}")


def decode_table(buf: bytes) -> dict:
    return _Reader(buf).table()


# ---------------------------------------------------------------- methods


_S_HH = struct.Struct(">HH")
_S_ACK = struct.Struct(">HHQB")          # basic.ack / basic.nack: ids, delivery-tag, bits
_S_Q = struct.Struct(">Q")
_S_HHH = struct.Struct(">HHH")


def _ss_fast(s: str | bytes) -> bytes:
    b = s.encode() if isinstance(s, str) else s
    if len(b) > 255:
        raise AMQPError("shortstr too long")
    return bytes((len(b),)) + b


# Hand-packed encoders for the per-message methods (the table-driven path
# below costs ~10 Python operations per field): same bytes, pinned against
# the generic encoder in tests/test_amqp.py.
_FAST_ENC = {
    "basic.ack": lambda a: _S_ACK.pack(60, 80, a.get("delivery_tag", 0), 1 if a.get("multiple") else 0),
    "basic.nack": lambda a: _S_ACK.pack(60, 120, a.get("delivery_tag", 0),
                                        (1 if a.get("multiple") else 0) | (2 if a.get("requeue") else 0)),
    "basic.deliver": lambda a: (_S_HH.pack(60, 60) + _ss_fast(a.get("consumer_tag", "")) +
                                _S_Q.pack(a.get("delivery_tag", 0)) + (b"\x01" if a.get("redelivered") else b"\x00") +
                                _ss_fast(a.get("exchange", "")) + _ss_fast(a.get("routing_key", ""))),
    "basic.publish": lambda a: (_S_HHH.pack(60, 40, a.get("ticket", 0)) + _ss_fast(a.get("exchange", "")) +
                                _ss_fast(a.get("routing_key", "")) +
                                bytes(((1 if a.get("mandatory") else 0) | (2 if a.get("immediate") else 0),))),
}


def _fast_decode(cid: int, mid: int, payload: bytes) -> Method | None:
    """Hot methods without the table-driven reader; None: use the generic path."""
    if cid != 60:
        return None
    try:
        if mid == 80 and len(payload) == 13:
            tag, bits = struct.unpack_from(">QB", payload, 4)
            return Method("basic.ack", {"delivery_tag": tag, "multiple": bool(bits & 1)})
        if mid == 120 and len(payload) == 13:
            tag, bits = struct.unpack_from(">QB", payload, 4)
            return Method("basic.nack", {"delivery_tag": tag, "multiple": bool(bits & 1), "requeue": bool(bits & 2)})
        if mid == 60:
            pos = 4
            n = payload[pos]
            ctag = payload[pos + 1:pos + 1 + n].decode("utf-8", "surrogateescape")
            pos += 1 + n
            (tag,) = struct.unpack_from(">Q", payload, pos)
            red = bool(payload[pos + 8] & 1)
            pos += 9
            n = payload[pos]
            ex = payload[pos + 1:pos + 1 + n].decode("utf-8", "surrogateescape")
            pos += 1 + n
            n = payload[pos]
            rk = payload[pos + 1:pos + 1 + n]
            if pos + 1 + n != len(payload):
                return None
            return Method("basic.deliver", {"consumer_tag": ctag, "delivery_tag": tag, "redelivered": red,
                                            "exchange": ex, "routing_key": rk.decode("utf-8", "surrogateescape")})
        if mid == 40:
            (ticket,) = struct.unpack_from(">H", payload, 4)
            pos = 6
            n = payload[pos]
            ex = payload[pos + 1:pos + 1 + n].decode("utf-8", "surrogateescape")
            pos += 1 + n
            n = payload[pos]
            rk = payload[pos + 1:pos + 1 + n].decode("utf-8", "surrogateescape")
            pos += 1 + n
            if pos + 1 != len(payload):
                return None
            bits = payload[pos]
            return Method("basic.publish", {"ticket": ticket, "exchange": ex, "routing_key": rk,
                                            "mandatory": bool(bits & 1), "immediate": bool(bits & 2)})
    except (IndexError, struct.error):
        return None                     # malformed: the generic path raises the proper FrameError
    return None


def encode_method(m: Method) -> bytes:
    f = _FAST_ENC.get(m.name)
    if f is not None:
        return f(m.args)
    cid, mid = BY_NAME[m.name]
    out = bytearray(struct.pack(">HH", cid, mid))
    bits: list[bool] = []

    def flush_bits() -> None:
        if bits:
            v = 0
            for i, b in enumerate(bits):
                if b:
                    v |= 1 << i
            out.append(v)
            bits.clear()

    for name, t in METHODS[(cid, mid)][1]:
        v = m.args.get(name, _default(t))
        if t == "bit":
            if len(bits) == 8:
                flush_bits()
            bits.append(bool(v))
            continue
        flush_bits()
        if t == "octet":
            out += struct.pack(">B", v)
        elif t == "short":
            out += struct.pack(">H", v)
        elif t == "long":
            out += struct.pack(">I", v)
        elif t == "longlong":
            out += struct.pack(">Q", v)
        elif t == "shortstr":
            out += _enc_shortstr(v)
        elif t == "longstr":
            out += _enc_longstr(v)
        elif t == "table":
            out += encode_table(v)
    flush_bits()
    return bytes(out)


def decode_method(payload: bytes) -> Method:
    if len(payload) >= 4:
        cid, mid = _S_HH.unpack_from(payload)
        m = _fast_decode(cid, mid, payload)
        if m is not None:
            return m
    r = _Reader(payload)
    cid, mid = r.unpack(">HH")
    spec = METHODS.get((cid, mid))
    if spec is None:
        raise FrameError(f"unknown method {cid}.{mid}")
    name, args = spec
    vals = {}
    for a, t in args:
        vals[a] = getattr(r, t)()
    return Method(name, vals)


# ---------------------------------------------------------- content header

PROPS = [("content_type", _ss), ("content_encoding", _ss), ("headers", _t), ("delivery_mode", _o),
         ("priority", _o), ("correlation_id", _ss), ("reply_to", _ss), ("expiration", _ss),
         ("message_id", _ss), ("timestamp", _ll), ("type", _ss), ("user_id", _ss), ("app_id", _ss),
         ("cluster_id", _ss)]


@dataclass
class Properties:
    content_type: str | None = None
    content_encoding: str | None = None
    headers: dict | None = None
    delivery_mode: int | None = None
    priority: int | None = None
    correlation_id: str | None = None
    reply_to: str | None = None
    expiration: str | None = None
    message_id: str | None = None
    timestamp: int | None = None
    type: str | None = None
    user_id: str | None = None
    app_id: str | None = None
    cluster_id: str | None = None


PERSISTENT = 2
TRANSIENT = 1


def encode_header(class_id: int, body_size: int, props: Properties) -> bytes:
    flags = 0
    out = bytearray()
    for i, (name, t) in enumerate(PROPS):
        v = getattr(props, name)
        if v is None:
            continue
        flags |= 1 << (15 - i)
        if t == "shortstr":
            out += _enc_shortstr(v)
        elif t == "table":
            out += encode_table(v)
        elif t == "octet":
            out += struct.pack(">B", v)
        elif t == "longlong":
            out += struct.pack(">Q", v)
    return struct.pack(">HHQH", class_id, 0, body_size, flags) + bytes(out)


def decode_header(payload: bytes) -> tuple[int, int, Properties]:
    r = _Reader(payload)
    class_id, _weight, body_size, flags = r.unpack(">HHQH")
    if flags & 1:
        raise FrameError("property flag continuation not supported")
    p = Properties()
    for i, (name, t) in enumerate(PROPS):
        if flags & (1 << (15 - i)):
            setattr(p, name, getattr(r, t)())
    return class_id, body_size, p


# ------------------------------------------------------------------ frames


_S_FRAME = struct.Struct(">BHI")


def frame(ftype: int, channel: int, payload: bytes) -> bytes:
    return b"".join((_S_FRAME.pack(ftype, channel, len(payload)), payload, b"\xce"))


def method_frame(channel: int, m: Method) -> bytes:
    return frame(FRAME_METHOD, channel, encode_method(m))


HEARTBEAT_FRAME = frame(FRAME_HEARTBEAT, 0, b"")


def content_frames(channel: int, m: Method, body: bytes, props: Properties, frame_max: int) -> list[bytes]:
    """Method + header + body frames for a content-bearing method."""
    out = [method_frame(channel, m), frame(FRAME_HEADER, channel, encode_header(60, len(body), props))]
    chunk = max(1, frame_max - 8)
    mv = memoryview(body)
    for i in range(0, len(body), chunk):
        out.append(frame(FRAME_BODY, channel, bytes(mv[i:i + chunk])))
    return out


class FrameParser:
    """Incremental frame splitter: ``feed`` raw socket bytes, get every complete
    frame at once.  One ``read`` of up to 64 KiB usually holds several frames
    (a delivery is method + header + body frames), so this replaces two
    awaited ``readexactly`` calls per frame with one read per batch."""

    def __init__(self, frame_max: int = 0) -> None:
        self.frame_max = frame_max
        self._buf = bytearray()

    def feed(self, data: bytes) -> list[tuple[int, int, bytes]]:
        buf = self._buf
        buf += data
        out: list[tuple[int, int, bytes]] = []
        pos, n = 0, len(buf)
        while n - pos >= 8:
            ftype, ch, size = struct.unpack_from(">BHI", buf, pos)
            if self.frame_max and size > self.frame_max:
                raise FrameError(f"frame size {size} exceeds frame_max {self.frame_max}")
            end = pos + 8 + size
            if end > n:
                break
            if buf[end - 1] != FRAME_END:
                raise FrameError("missing frame-end octet")
            out.append((ftype, ch, bytes(buf[pos + 7:end - 1])))
            pos = end
        if pos:
            del buf[:pos]
        return out
