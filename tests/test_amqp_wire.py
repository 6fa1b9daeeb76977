"""AMQP 0-9-1 wire parity pinned to byte-exact fixtures derived by hand from
the specification (amqp0-9-1.xml / the 0-9-1 PDF, §4.2 frames, §4.2.5 field
tables) and the RabbitMQ errata (field-table type tags: 'I' signed 32-bit,
'l' signed 64-bit, 's' signed 16-bit, 'x' byte array, 'F' table, 't'
boolean).

The reference's broker traffic (streadway/amqp):
``internal/rabbitmq/client.go:224`` (publish), ``:333`` (exchange.declare),
``:347`` (queue.declare), ``:351`` (queue.bind), ``:368`` (basic.qos global),
``delivery.go:32-44`` (X-Retries int32 header), ``:56`` (ack), ``:61`` (nack),
``:74-79`` (republish with headers).

None of these tests involve the fake broker: the expected bytes are literal
hex, and the handshake test drives the real client against a scripted peer
that writes literal server frames and records the client's bytes."""

import asyncio
import struct

from tritondl.amqp import codec
from tritondl.amqp.codec import Method, Properties

H = bytes.fromhex


def frame(ftype: int, ch: int, payload: bytes) -> bytes:
    # §4.2.3: type(1) channel(2) size(4) payload frame-end(0xCE)
    return bytes([ftype]) + ch.to_bytes(2, "big") + len(payload).to_bytes(4, "big") + payload + b"\xce"


# --------------------------------------------------------------- literal fixtures

def test_protocol_header():
    assert codec.PROTOCOL_HEADER == H("414d515000000901")           # "AMQP" 0 0 9 1


def test_heartbeat_frame():
    assert codec.HEARTBEAT_FRAME == H("08 0000 00000000 ce")


def test_tune_ok_and_open():
    tune_ok = H("000a 001f" "07ff" "00020000" "001e")               # channel_max 2047, frame_max 131072, hb 30
    assert codec.encode_method(Method("connection.tune_ok", {"channel_max": 2047, "frame_max": 131072,
                                                              "heartbeat": 30})) == tune_ok
    opn = H("000a 0028" "01 2f" "00" "00")                          # vhost "/", capabilities "", insist=0
    assert codec.encode_method(Method("connection.open", {"virtual_host": "/"})) == opn
    assert codec.method_frame(0, Method("connection.open", {"virtual_host": "/"})) == \
        H("01 0000 00000008") + opn + b"\xce"


def test_start_ok_plain_with_capabilities_table():
    payload = (H("000a 000b")
               + H("0000003c")                                       # table length 60
               + b"\x07product" + b"S" + H("00000008") + b"tritondl"  # 21 bytes
               + b"\x0ccapabilities" + b"F" + H("00000015")            # nested table, 21 bytes
               + b"\x12publisher_confirms" + b"t" + H("01")
               + b"\x05PLAIN"
               + H("0000000c") + b"\x00guest\x00guest"
               + b"\x05en_US")
    m = Method("connection.start_ok", {"client_properties": {"product": "tritondl",
                                                             "capabilities": {"publisher_confirms": True}},
                                       "mechanism": "PLAIN", "response": b"\x00guest\x00guest",
                                       "locale": "en_US"})
    assert codec.encode_method(m) == payload
    d = codec.decode_method(payload)
    assert d.client_properties == {"product": "tritondl", "capabilities": {"publisher_confirms": True}}


def test_topology_methods_reference_flags():
    # exchange.declare(topic, "direct", durable=true, autoDelete=false, internal=false, noWait=false) client.go:333
    ex = H("0028 000a" "0000") + b"\x0bv1.download" + b"\x06direct" + H("02") + H("00000000")
    assert codec.encode_method(Method("exchange.declare", {"exchange": "v1.download", "type": "direct",
                                                           "durable": True})) == ex
    # queue.declare(name, durable=true, autoDelete=false, exclusive=false, noWait=false) client.go:347
    qd = H("0032 000a" "0000") + b"\x0dv1.download-0" + H("02") + H("00000000")
    assert codec.encode_method(Method("queue.declare", {"queue": "v1.download-0", "durable": True})) == qd
    # queue.bind(name, rk=name, exchange=topic) client.go:351
    qb = H("0032 0014" "0000") + b"\x0dv1.download-0" + b"\x0bv1.download" + b"\x0dv1.download-0" + H("00") + \
        H("00000000")
    assert codec.encode_method(Method("queue.bind", {"queue": "v1.download-0", "exchange": "v1.download",
                                                     "routing_key": "v1.download-0"})) == qb
    # basic.qos(prefetch=1, size=0, global=true) client.go:368
    assert codec.encode_method(Method("basic.qos", {"prefetch_count": 1, "global_": True})) == \
        H("003c 000a" "00000000" "0001" "01")
    # basic.consume(queue, "", autoAck=false, exclusive=false, noLocal=false, noWait=false) client.go:248
    assert codec.encode_method(Method("basic.consume", {"queue": "v1.download-1"})) == \
        H("003c 0014" "0000") + b"\x0dv1.download-1" + b"\x00" + H("00") + H("00000000")
    # queue.declare with a TTL + DLX argument table (the delayed-retry queues)
    args = {"x-message-ttl": 10000, "x-dead-letter-exchange": "v1.download"}
    tbl = (b"\x0dx-message-ttl" + b"I" + H("00002710")
           + b"\x16x-dead-letter-exchange" + b"S" + H("0000000b") + b"v1.download")
    qa = H("0032 000a" "0000") + b"\x19v1.download-0.retry.10000" + H("02") + len(tbl).to_bytes(4, "big") + tbl
    assert codec.encode_method(Method("queue.declare", {"queue": "v1.download-0.retry.10000", "durable": True,
                                                        "arguments": args})) == qa
    # confirm.select(noWait=false)
    assert codec.encode_method(Method("confirm.select")) == H("0055 000a 00")


def test_publish_persistent_with_x_retries_and_body_split():
    body = bytes(range(256)) * 40                                    # 10,240 bytes
    props = Properties(content_type="application/octet-stream", delivery_mode=2, headers={"X-Retries": 3})
    frames = codec.content_frames(5, Method("basic.publish", {"exchange": "v1.download",
                                                              "routing_key": "v1.download-0"}),
                                  body, props, 4096)
    pub = H("003c 0028" "0000") + b"\x0bv1.download" + b"\x0dv1.download-0" + H("00")
    assert frames[0] == frame(1, 5, pub)
    # content header §4.2.6: class 60, weight 0, body size, flags (content-type bit 15,
    # headers bit 13, delivery-mode bit 12 -> 0xB000), then the properties in order
    hdr = (H("003c" "0000") + (10240).to_bytes(8, "big") + H("b000")
           + b"\x18application/octet-stream"
           + H("0000000f") + b"\x09X-Retries" + b"I" + H("00000003")  # X-Retries int32 (delivery.go:32-44)
           + H("02"))                                                  # persistent
    assert frames[1] == frame(2, 5, hdr)
    # body frames: at most frame_max - 8 payload bytes each (§4.2.3)
    assert [len(f) - 8 for f in frames[2:]] == [4088, 4088, 2064]
    assert b"".join(f[7:-1] for f in frames[2:]) == body
    assert all(f[:3] == H("03 0005") and f[-1] == 0xCE for f in frames[2:])
    cid, size, p = codec.decode_header(hdr)
    assert (cid, size, p.headers, p.delivery_mode) == (60, 10240, {"X-Retries": 3}, 2)


def test_deliver_ack_nack_fixtures():
    deliver = H("003c 003c") + b"\x04ctag" + H("0000000000000007") + H("01") + b"\x0bv1.download" + \
        b"\x0dv1.download-1"
    m = codec.decode_method(deliver)
    assert m.name == "basic.deliver" and m.consumer_tag == "ctag" and m.delivery_tag == 7 and m.redelivered
    assert m.exchange == "v1.download" and m.routing_key == "v1.download-1"
    # Ack(multiple=false) delivery.go:56
    assert codec.encode_method(Method("basic.ack", {"delivery_tag": 7})) == H("003c 0050" "0000000000000007" "00")
    # Nack(multiple=false, requeue=false) delivery.go:61 — bit 0 multiple, bit 1 requeue
    assert codec.encode_method(Method("basic.nack", {"delivery_tag": 7, "requeue": False})) == \
        H("003c 0078" "0000000000000007" "00")
    assert codec.encode_method(Method("basic.nack", {"delivery_tag": 7, "multiple": True, "requeue": True})) == \
        H("003c 0078" "0000000000000007" "03")
    # publisher-confirm ack from the server
    assert codec.decode_method(H("003c 0050" "0000000000000003" "01")).args == {"delivery_tag": 3, "multiple": True}


def test_rabbitmq_errata_field_types():
    # a table as RabbitMQ writes it: 's' int16, 'l' int64, 'x' bytes, 'A' array, 'V' void, 'T' timestamp
    tbl = (b"\x01a" + b"s" + H("fffe")
           + b"\x01b" + b"l" + H("0000000100000000")
           + b"\x01c" + b"x" + H("00000002") + b"\x00\xff"
           + b"\x01d" + b"A" + H("0000000a") + b"I" + H("00000001") + b"t" + H("00") + b"V" + b"t" + H("01")
           + b"\x01e" + b"T" + H("000000005e0be100"))
    got = codec.decode_table(len(tbl).to_bytes(4, "big") + tbl)
    assert got["a"] == -2 and got["b"] == 1 << 32 and got["c"] == b"\x00\xff"
    assert got["d"] == [1, False, None, True]
    assert int(got["e"].timestamp()) == 1577836800
    # int32 header values stay 'I' (X-Retries), larger ones go 'l'
    assert codec.encode_table({"n": 2**31 - 1}) == H("00000007") + b"\x01n" + b"I" + H("7fffffff")
    assert codec.encode_table({"n": 2**31}) == H("0000000b") + b"\x01n" + b"l" + H("0000000080000000")


# --------------------------------------------------------------- scripted peer

def test_client_handshake_and_first_frames_against_scripted_peer():
    """The real client against a peer that writes literal server frames; the
    bytes the client sends are compared with hand-built expectations."""
    from tritondl.amqp.connection import Connection

    def tbl(d: dict) -> bytes:
        # spec encoder for the few value kinds the client sends (independent of codec.py)
        out = b""
        for k, v in d.items():
            out += bytes([len(k)]) + k.encode()
            if isinstance(v, bool):
                out += b"t" + (b"\x01" if v else b"\x00")
            elif isinstance(v, str):
                out += b"S" + len(v).to_bytes(4, "big") + v.encode()
            else:
                inner = tbl(v)
                out += b"F" + inner
        return len(out).to_bytes(4, "big") + out

    got = bytearray()

    async def main():
        start = (H("000a 000a") + H("00 09")                              # version 0-9
                 + H("00000000")                                          # server_properties {}
                 + H("00000005") + b"PLAIN" + H("00000005") + b"en_US")
        tune = H("000a 001e") + H("07ff") + H("00020000") + H("003c")
        open_ok = H("000a 0029") + b"\x00"
        chan_open_ok = H("0014 000b") + H("00000000")
        qos_ok = H("003c 000b")
        done = asyncio.Event()

        async def peer(reader, writer):
            got.extend(await reader.readexactly(8))
            writer.write(frame(1, 0, start))
            await writer.drain()
            while True:
                hdr = await reader.readexactly(7)
                size = struct.unpack(">I", hdr[3:])[0]
                body = await reader.readexactly(size + 1)
                got.extend(hdr + body)
                cm = body[:4]
                if cm == H("000a 000b"):
                    writer.write(frame(1, 0, tune))
                elif cm == H("000a 0028"):
                    writer.write(frame(1, 0, open_ok))
                elif cm == H("0014 000a"):
                    writer.write(frame(1, struct.unpack(">H", hdr[1:3])[0], chan_open_ok))
                elif cm == H("003c 000a"):
                    writer.write(frame(1, 1, qos_ok))
                    done.set()
                    return
                await writer.drain()

        srv = await asyncio.start_server(peer, "127.0.0.1", 0)
        port = srv.sockets[0].getsockname()[1]
        c = await Connection.open(f"amqp://guest:guest@127.0.0.1:{port}/", heartbeat=60)
        ch = await c.channel()
        await ch.basic_qos(1, 0, True)
        await asyncio.wait_for(done.wait(), 5)
        c._abort(ConnectionError("test over"))
        srv.close()

    asyncio.run(asyncio.wait_for(main(), 20))
    import os
    import socket
    props = {"product": "tritondl", "version": "0.1", "platform": "python-asyncio",
             "capabilities": {"publisher_confirms": True, "consumer_cancel_notify": True, "basic.nack": True,
                              "connection.blocked": True, "authentication_failure_close": True},
             "connection_name": f"tritondl@{socket.gethostname()} pid {os.getpid()}"}
    start_ok = H("000a 000b") + tbl(props) + b"\x05PLAIN" + H("0000000c") + b"\x00guest\x00guest" + b"\x05en_US"
    # tune-ok echoes the negotiated values: channel_max 2047, frame_max 131072, heartbeat min(60, 60)
    expect = (H("414d515000000901")
              + frame(1, 0, start_ok)
              + frame(1, 0, H("000a 001f" "07ff" "00020000" "003c"))
              + frame(1, 0, H("000a 0028" "01 2f" "00" "00"))
              + frame(1, 1, H("0014 000a" "00"))
              + frame(1, 1, H("003c 000a" "00000000" "0001" "01")))
    assert bytes(got) == expect, (bytes(got).hex(), expect.hex())
