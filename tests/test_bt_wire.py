"""BitTorrent wire formats pinned to the BEP texts, not to our own fakes.

Round-trip tests between our client and our own seeder/tracker/DHT fakes
would pass with a bug both share; these fixtures are byte strings and
offsets taken from the specifications themselves (the reference delegated
all of this to anacrolix/torrent, ``internal/downloader/torrent/
torrent.go:40-106``):

* BEP 3  — handshake layout, message framing, bitfield bit order, HTTP
  tracker query parameters;
* BEP 5  — the KRPC example messages quoted in the BEP, byte for byte, and
  our DHT server's answers to them;
* BEP 6/10/52 — reserved-bit positions;
* BEP 9  — ut_metadata request/data/reject examples;
* BEP 10 — extension handshake dictionary;
* BEP 11 — ut_pex compact lists;
* BEP 15 — UDP tracker connect/announce packet offsets (scripted peer);
* BEP 23 / BEP 32 — compact peer and node encodings (IPv4 and IPv6).
"""

import asyncio
import socket
import struct
from urllib.parse import unquote_to_bytes

import pytest

from tritondl.fetch.bt import bencode
from tritondl.fetch.bt import dht as D
from tritondl.fetch.bt import peer as pw
from tritondl.fetch.bt import tracker as T


def run(coro, timeout=30):
    return asyncio.run(asyncio.wait_for(coro, timeout))


# ----------------------------------------------------------------- BEP 5 KRPC
# the example encodings printed in BEP 5 ("DHT Queries" section)
PING_Q = b"d1:ad2:id20:abcdefghij0123456789e1:q4:ping1:t2:aa1:y1:qe"
PING_R = b"d1:rd2:id20:mnopqrstuvwxyz123456e1:t2:aa1:y1:re"
FIND_Q = b"d1:ad2:id20:abcdefghij01234567896:target20:mnopqrstuvwxyz123456e1:q9:find_node1:t2:aa1:y1:qe"
GETP_Q = b"d1:ad2:id20:abcdefghij01234567899:info_hash20:mnopqrstuvwxyz123456e1:q9:get_peers1:t2:aa1:y1:qe"
GETP_R = (b"d1:rd2:id20:abcdefghij01234567895:token8:aoeusnth6:valuesl6:axje.u6:idhtnmee"
          b"1:t2:aa1:y1:re")
ANN_Q = (b"d1:ad2:id20:abcdefghij012345678912:implied_porti1e9:info_hash20:mnopqrstuvwxyz123456"
         b"4:porti6881e5:token8:aoeusnthe1:q13:announce_peer1:t2:aa1:y1:qe")
ERR = b"d1:eli201e23:A Generic Error Ocurrede1:t2:aa1:y1:ee"


def test_bep5_example_messages_encode_byte_for_byte():
    assert bencode.encode({b"t": b"aa", b"y": b"q", b"q": b"ping",
                           b"a": {b"id": b"abcdefghij0123456789"}}) == PING_Q
    assert bencode.encode({b"t": b"aa", b"y": b"r", b"r": {b"id": b"mnopqrstuvwxyz123456"}}) == PING_R
    assert bencode.encode({b"t": b"aa", b"y": b"q", b"q": b"find_node",
                           b"a": {b"id": b"abcdefghij0123456789", b"target": b"mnopqrstuvwxyz123456"}}) == FIND_Q
    assert bencode.encode({b"t": b"aa", b"y": b"q", b"q": b"get_peers",
                           b"a": {b"id": b"abcdefghij0123456789", b"info_hash": b"mnopqrstuvwxyz123456"}}) == GETP_Q
    assert bencode.encode({b"t": b"aa", b"y": b"r", b"r": {b"id": b"abcdefghij0123456789", b"token": b"aoeusnth",
                                                         b"values": [b"axje.u", b"idhtnm"]}}) == GETP_R
    assert bencode.encode({b"t": b"aa", b"y": b"q", b"q": b"announce_peer",
                           b"a": {b"id": b"abcdefghij0123456789", b"implied_port": 1,
                                  b"info_hash": b"mnopqrstuvwxyz123456", b"port": 6881,
                                  b"token": b"aoeusnth"}}) == ANN_Q
    assert bencode.encode({b"t": b"aa", b"y": b"e", b"e": [201, b"A Generic Error Ocurred"]}) == ERR
    for m in (PING_Q, PING_R, FIND_Q, GETP_Q, GETP_R, ANN_Q, ERR):
        assert bencode.encode(bencode.decode(m)) == m
    # the example "values" are 6-byte compact peers (BEP 5 "Contact Encoding")
    assert D.parse_values([b"axje.u"]) == [(socket.inet_ntoa(b"axje"), struct.unpack(">H", b".u")[0])]


class _Capture:
    def __init__(self):
        self.sent = []

    def sendto(self, data, addr):
        self.sent.append((data, addr))

    def close(self):
        pass


def test_dht_server_answers_the_bep5_example_queries():
    """Feed the BEP's example queries to our node's server side; every reply
    must echo ``t``, carry ``y=r`` and the fields the BEP requires."""
    async def main():
        node = D.DHTNode(node_id=b"N" * 20, host=None)
        cap = _Capture()
        node._transports[socket.AF_INET] = cap
        src = ("10.1.2.3", 4000)
        node._on_datagram(PING_Q, src, socket.AF_INET)
        r = bencode.decode(cap.sent[-1][0])
        assert r == {b"t": b"aa", b"y": b"r", b"r": {b"id": b"N" * 20}} and cap.sent[-1][1] == src
        # the querier is now in our table (BEP 5: learn from queries)
        assert b"abcdefghij0123456789" in node.table
        node._on_datagram(FIND_Q, src, socket.AF_INET)
        r = bencode.decode(cap.sent[-1][0])[b"r"]
        assert len(r[b"nodes"]) % 26 == 0 and D.parse_nodes(r[b"nodes"]) == [(b"abcdefghij0123456789", src)]
        node._on_datagram(GETP_Q, src, socket.AF_INET)
        r = bencode.decode(cap.sent[-1][0])[b"r"]
        assert isinstance(r[b"token"], bytes) and b"values" not in r and b"nodes" in r
        tok = r[b"token"]
        # the example announce carries the example token: rejected (203) — ours differs
        node._on_datagram(ANN_Q, src, socket.AF_INET)
        e = bencode.decode(cap.sent[-1][0])
        assert e[b"y"] == b"e" and e[b"e"][0] == 203 and e[b"t"] == b"aa"
        # with our token and implied_port=1 the SOURCE port is stored, not "port"
        node._on_datagram(ANN_Q.replace(b"8:aoeusnth", b"8:" + tok), src, socket.AF_INET)
        assert bencode.decode(cap.sent[-1][0])[b"y"] == b"r"
        assert (src[0], src[1]) in node.peers[b"mnopqrstuvwxyz123456"]
        node._on_datagram(GETP_Q, ("10.9.9.9", 5000), socket.AF_INET)
        r = bencode.decode(cap.sent[-1][0])[b"r"]
        assert D.parse_values(r[b"values"]) == [src]
        # unknown method -> error 204
        node._on_datagram(b"d1:ad2:id20:abcdefghij0123456789e1:q4:blah1:t2:ab1:y1:qe", src, socket.AF_INET)
        e = bencode.decode(cap.sent[-1][0])
        assert e[b"e"][0] == 204 and e[b"t"] == b"ab"
    run(main())


def test_bep32_compact_node6_and_peer6_layout():
    nid = bytes(range(20))
    b = D.compact_node(nid, ("2001:db8::1", 6881))
    assert len(b) == 38 and b[:20] == nid and b[20:36] == socket.inet_pton(socket.AF_INET6, "2001:db8::1")
    assert b[36:] == b"\x1a\xe1"
    assert D.parse_nodes6(b) == [(nid, ("2001:db8::1", 6881))]
    assert D.compact_addr(("2001:db8::1", 6881)) == b[20:]
    assert D.parse_values([b[20:], b"\x7f\x00\x00\x01\x1a\xe1"]) == [("2001:db8::1", 6881), ("127.0.0.1", 6881)]


# ----------------------------------------------------------------- BEP 3 / 6 / 10 / 52
def test_bep3_handshake_layout_and_reserved_bits():
    ih, pid = bytes(range(20)), b"-TD0100-" + bytes(12)
    h = pw.encode_handshake(ih, pid)
    assert len(h) == 68 and h[0] == 19 and h[1:20] == b"BitTorrent protocol"
    assert h[28:48] == ih and h[48:68] == pid
    r = h[20:28]
    assert r[5] & 0x10                        # BEP 10 extension protocol: reserved byte 5, bit 0x10
    assert r[7] & 0x04                        # BEP 6 fast extension: byte 7, 0x04
    assert r[7] & 0x01                        # BEP 5 DHT (PORT message): byte 7, 0x01
    assert r[7] & 0x10                        # BEP 52 v2 upgrade: byte 7, 0x10
    assert pw.reserved_bytes(False, False, False, False) == bytes(8)
    hs = pw.parse_handshake(h)
    assert hs.extended and hs.fast and hs.dht and hs.v2 and hs.infohash == ih


class _Sink:
    def __init__(self):
        self.data = bytearray()

    def write(self, b):
        self.data += b

    def close(self):
        pass


def test_bep3_message_framing():
    run(_framing())


async def _framing():
    w = pw.Wire(asyncio.StreamReader(), _Sink())
    w.keepalive()
    w.have(0x01020304)
    w.request(1, 0x4000, 0x4000)
    w.cancel(1, 0x4000, 0x4000)
    w.piece(2, 0, b"xyz")
    w.bitfield(pw.set_to_bits({0, 9}, 10))
    w.flush()
    out = bytes(w.writer.data)
    want = (b"\x00\x00\x00\x00"
            + b"\x00\x00\x00\x05\x04\x01\x02\x03\x04"
            + b"\x00\x00\x00\x0d\x06" + struct.pack(">III", 1, 0x4000, 0x4000)
            + b"\x00\x00\x00\x0d\x08" + struct.pack(">III", 1, 0x4000, 0x4000)
            + b"\x00\x00\x00\x0c\x07" + struct.pack(">II", 2, 0) + b"xyz"
            + b"\x00\x00\x00\x03\x05\x80\x40")          # high bit of byte 0 = piece 0; piece 9 = 0x40 of byte 1
    assert out == want
    assert pw.bits_to_set(b"\x80\x40", 10) == {0, 9}


def test_bep9_ut_metadata_examples():
    # the three example messages of BEP 9 (the data message is followed by the raw piece)
    assert pw.meta_msg(pw.META_REQUEST, 0) == b"d8:msg_typei0e5:piecei0ee"
    assert pw.meta_msg(pw.META_DATA, 0, 34256, b"xxxx") == b"d8:msg_typei1e5:piecei0e10:total_sizei34256eexxxx"
    assert pw.meta_msg(pw.META_REJECT, 0) == b"d8:msg_typei2e5:piecei0ee"
    d, rest = pw.parse_meta_msg(b"d8:msg_typei1e5:piecei0e10:total_sizei34256eexxxx")
    assert d == {b"msg_type": 1, b"piece": 0, b"total_size": 34256} and rest == b"xxxx"


def test_bep10_extension_handshake():
    # BEP 10's example dictionary (UTF-8 "µ", lengths in bytes)
    ex = b"d1:md11:LT_metadatai1e7:\xc2\xb5T_PEXi2ee1:pi6881e1:v13:\xc2\xb5Torrent 1.2e"
    h = pw.parse_ext_handshake(ex)
    assert h.m == {"LT_metadata": 1, "µT_PEX": 2} and h.port == 6881 and h.v == "µTorrent 1.2"
    run(_ext_hs())


async def _ext_hs():
    w = pw.Wire(asyncio.StreamReader(), _Sink())
    w.ext_handshake(31235, port=6881, reqq=250)
    w.flush()
    out = bytes(w.writer.data)
    (ln, mid, ext) = struct.unpack(">IBB", out[:6])
    assert mid == 20 and ext == 0 and ln == len(out) - 4       # extended message id 20, handshake sub-id 0
    d = bencode.decode(out[6:])
    assert d[b"m"] == {b"ut_metadata": pw.UT_METADATA_ID, b"ut_pex": pw.UT_PEX_ID}
    assert d[b"metadata_size"] == 31235 and d[b"p"] == 6881 and d[b"reqq"] == 250
    assert bencode.encode(d) == out[6:]                        # keys sorted, canonical


def test_bep11_pex_compact_lists():
    msg = pw.pex_msg([("10.0.0.1", 6881), ("2001:db8::2", 51413)], [("10.0.0.9", 1)],
                     {("10.0.0.1", 6881): 0x12})
    d = bencode.decode(msg)
    assert d[b"added"] == b"\x0a\x00\x00\x01\x1a\xe1" and d[b"added.f"] == b"\x12"
    assert d[b"added6"] == socket.inet_pton(socket.AF_INET6, "2001:db8::2") + struct.pack(">H", 51413)
    assert d[b"dropped"] == b"\x0a\x00\x00\x09\x00\x01"
    assert pw.parse_pex(msg) == ([("10.0.0.1", 6881), ("2001:db8::2", 51413)], [("10.0.0.9", 1)])


def test_bep23_compact_peers():
    assert T.compact_peers([("1.2.3.4", 0x1ae1), ("::1", 9)]) == b"\x01\x02\x03\x04\x1a\xe1"
    assert T.parse_compact(b"\x01\x02\x03\x04\x1a\xe1") == [("1.2.3.4", 6881)]
    v6 = socket.inet_pton(socket.AF_INET6, "2001:db8::7") + b"\x00\x50"
    assert T.parse_compact(v6, v6=True) == [("2001:db8::7", 80)]


# ----------------------------------------------------------------- trackers
def test_bep15_udp_tracker_packets_against_a_scripted_peer():
    """Connect: 64-bit magic 0x41727101980, action 0, transaction id (16 B).
    Announce: 98 B — connection id, action 1, tid, info_hash, peer_id,
    downloaded, left, uploaded, event, IP 0, key, num_want, port."""
    seen = {}

    class Peer(asyncio.DatagramProtocol):
        def connection_made(self, tr):
            self.tr = tr

        def datagram_received(self, data, addr):
            if "connect" not in seen:
                seen["connect"] = data
                assert len(data) == 16
                magic, action, tid = struct.unpack(">QII", data)
                assert magic == 0x41727101980 and action == 0
                self.tr.sendto(struct.pack(">IIQ", 0, tid, 0xC0FFEE), addr)
            else:
                seen["announce"] = data
                assert len(data) == 98
                cid, action, tid = struct.unpack(">QII", data[:16])
                assert cid == 0xC0FFEE and action == 1
                self.tr.sendto(struct.pack(">IIIII", 1, tid, 1800, 3, 7) + b"\x0a\x00\x00\x05\x1a\xe1", addr)

    async def main():
        loop = asyncio.get_running_loop()
        tr, _ = await loop.create_datagram_endpoint(Peer, local_addr=("127.0.0.1", 0))
        port = tr.get_extra_info("sockname")[1]
        a = T.Announce(b"I" * 20, b"P" * 20, 6881, uploaded=5, downloaded=6, left=7, event="started", numwant=50)
        res = await T.udp_announce(f"udp://127.0.0.1:{port}/announce", a, timeout=1.0)
        tr.close()
        assert res.interval == 1800 and res.leechers == 3 and res.seeders == 7
        assert res.peers == [("10.0.0.5", 6881)]
        p = seen["announce"]
        assert p[16:36] == b"I" * 20 and p[36:56] == b"P" * 20
        assert struct.unpack(">QQQ", p[56:80]) == (6, 7, 5)          # downloaded, left, uploaded
        assert struct.unpack(">I", p[80:84])[0] == 2                 # event: started = 2
        assert p[84:88] == bytes(4)                                  # IP address: default (0)
        assert struct.unpack(">i", p[92:96])[0] == 50 and struct.unpack(">H", p[96:98])[0] == 6881
    run(main())


def test_bep3_http_tracker_query_against_a_scripted_peer():
    """GET <announce>?info_hash=<20 raw bytes, %-escaped>&peer_id=...&port&
    uploaded&downloaded&left&compact=1&event=started; reply is a bencoded
    dict with ``interval`` and compact ``peers`` (BEP 23)."""
    got = {}

    async def handle(r, w):
        line = (await r.readline()).decode()
        while (await r.readline()) not in (b"\r\n", b""):
            pass
        got["line"] = line
        body = bencode.encode({b"interval": 900, b"complete": 2, b"incomplete": 1,
                               b"peers": b"\x0a\x00\x00\x06\x1a\xe2"})
        w.write(b"HTTP/1.1 200 OK\r\nContent-Length: %d\r\nConnection: close\r\n\r\n" % len(body) + body)
        await w.drain()
        w.close()

    async def main():
        srv = await asyncio.start_server(handle, "127.0.0.1", 0)
        port = srv.sockets[0].getsockname()[1]
        ih = bytes([0, 1, 2, 0x7F, 0x80, 0xFF]) + b"abcdefghijklmn"
        a = T.Announce(ih, b"-TD0100-123456789012", 51413, uploaded=0, downloaded=10, left=99, event="started")
        res = await T.http_announce(f"http://127.0.0.1:{port}/announce", a)
        srv.close()
        assert res.interval == 900 and res.peers == [("10.0.0.6", 6882)] and res.seeders == 2
        method, target, _v = got["line"].split(" ")
        assert method == "GET" and target.startswith("/announce?")
        q = dict(kv.split("=", 1) for kv in target.split("?", 1)[1].split("&"))
        assert unquote_to_bytes(q["info_hash"]) == ih and unquote_to_bytes(q["peer_id"]) == a.peer_id
        assert (q["port"], q["uploaded"], q["downloaded"], q["left"], q["compact"], q["event"]) == \
            ("51413", "0", "10", "99", "1", "started")
    run(main())


def test_bep40_canonical_peer_priority_examples():
    """BEP 40's worked examples, CRC-32C's check value, and symmetry."""
    from tritondl.fetch.bt.bep40 import crc32c, priority
    assert crc32c(b"123456789") == 0xE3069283
    assert priority(("123.213.32.10", 0), ("98.76.54.32", 0)) == 0xEC2D7224
    assert priority(("123.213.32.10", 0), ("123.213.32.234", 0)) == 0x99568189
    a, b = ("10.0.0.1", 6881), ("10.0.0.1", 51413)          # same IP: ports decide
    assert priority(a, b) == priority(b, a) == crc32c(bytes.fromhex("1ae1c8d5"))
    assert priority(("2001:db8::1", 1), ("2001:db8:1::2", 2)) == priority(("2001:db8:1::2", 2), ("2001:db8::1", 1))


def test_topup_dials_highest_bep40_priority_first(tmp_path):
    from tritondl.fetch.bt.bep40 import priority
    from tritondl.fetch.bt.torrent import Torrent, TorrentConfig
    t = Torrent(b"\x01" * 20, str(tmp_path), TorrentConfig(announce_host="123.213.32.10"))
    t.port = 6881
    t.known = {("98.76.54.32", 1), ("123.213.32.234", 2), ("8.8.8.8", 3), ("1.2.3.4", 4)}
    best = t._best_candidates(2)
    ranked = sorted(t.known, key=lambda a: priority(("123.213.32.10", 6881), a), reverse=True)
    assert best == ranked[:2]


def test_unsolicited_or_out_of_range_metadata_pieces_are_not_kept(tmp_path):
    """A peer sending ut_metadata data for pieces outside the announced
    metadata size (or before any size is known, or bigger than a block)
    cannot grow the session's memory; a request for a negative piece is
    rejected instead of served from the end of the info dict."""
    import asyncio
    from tritondl.fetch.bt.metainfo import BLOCK
    from tritondl.fetch.bt.torrent import Torrent, TorrentConfig, _Peer

    class W:
        def __init__(self):
            self.sent = []

        def extended(self, eid, payload):
            self.sent.append((eid, payload))

    t = Torrent(b"\x01" * 20, str(tmp_path), TorrentConfig())
    p = _Peer(W(), ("1.2.3.4", 5), None, 0)
    p.ext = pw.ExtHandshake({"ut_metadata": 3}, None, None, "", None)

    def data(piece, body=b"x"):
        return bytes([pw.UT_METADATA_ID]) + pw.meta_msg(pw.META_DATA, piece, 40_000, body)

    async def main():
        await t._on_extended(p, data(0))                       # no size announced yet
        assert t._meta == {}
        t._meta_size = 40_000                                  # 3 pieces
        for piece in (-1, 3, 1 << 40):
            await t._on_extended(p, data(piece))
        await t._on_extended(p, data(1, b"y" * (BLOCK + 1)))
        assert t._meta == {}
        await t._on_extended(p, data(1))
        assert list(t._meta) == [1]
        t.info = type("I", (), {"raw": b"z" * 100})()
        await t._on_extended(p, bytes([pw.UT_METADATA_ID]) + pw.meta_msg(pw.META_REQUEST, -1))
        d, body = pw.parse_meta_msg(p.wire.sent[-1][1])
        assert d[b"msg_type"] == pw.META_REJECT and body == b""
    asyncio.run(main())


def test_peer_messages_of_any_shape_end_only_that_peer(tmp_path):
    """Every message id with any payload (short fixed fields, a bitfield
    too short for the torrent, out-of-range indices) is handled or ends the
    peer with PeerError / struct.error (caught per peer by the session);
    nothing else escapes into the session."""
    import asyncio
    import struct
    from hypothesis import HealthCheck, given, settings
    from hypothesis import strategies as st
    from tritondl_testkit.fakes.swarm import make_payload, torrent_for
    from tritondl.fetch.bt.torrent import Torrent, TorrentConfig, _Peer

    make_payload(str(tmp_path / "src"), {"a.mkv": 100_000})
    info = torrent_for(str(tmp_path / "src" / "a.mkv"), 16384)

    class AnyWire:
        def __getattr__(self, _k):
            return lambda *a, **kw: None

    @settings(max_examples=300, deadline=None, suppress_health_check=list(HealthCheck))
    @given(st.lists(st.tuples(st.integers(0, 25), st.binary(max_size=40)), max_size=20))
    def check(msgs):
        async def main():
            t = Torrent(info.infohash, str(tmp_path / "dst"), TorrentConfig(native_wire=False), info=info)
            hs = pw.Handshake(bytes([0, 0, 0, 0, 0, 0x10, 0, 0x04]), info.infohash, b"x" * 20)
            p = _Peer(AnyWire(), ("1.2.3.4", 5), hs, info.num_pieces)
            for mid, pl in msgs:
                try:
                    await t._dispatch(p, mid, pl)
                except (pw.PeerError, struct.error):
                    pass
        asyncio.run(main())
    check()
    with pytest.raises(pw.PeerError):
        pw.bits_to_set(b"", 7)
