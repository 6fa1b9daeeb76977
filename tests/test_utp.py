"""Native uTP (BEP 29): engine-level transfers over a simulated lossy FIFO
link, the asyncio socket wrapper on localhost, and a BitTorrent download
forced over uTP."""

import asyncio
import os
import random

import pytest

from tritondl import _utp
from tritondl_testkit.fakes.swarm import magnet_for, make_payload, torrent_for
from tritondl.fetch.bt.client import TorrentDownloader
from tritondl.fetch.bt.torrent import Torrent, TorrentConfig
from tritondl.fetch.bt.utp import UtpSocket


def _simulate(loss: float, n: int, seed: int = 1, reorder: bool = False):
    rnd = random.Random(seed)
    a, b = _utp.Engine(seed), _utp.Engine(seed + 1)
    now = 0
    ca = a.connect("B", now)
    data = rnd.randbytes(n)
    sent, got, cb = 0, bytearray(), None
    wire, last = [], {}
    for _ in range(400_000):
        now += 1000
        if sent < n:
            sent += a.write(ca, data[sent:sent + 65536])
        elif sent == n:
            a.close(ca, now)
            sent += 1
        for eng, name in ((a, "A"), (b, "B")):
            for addr, pkt in eng.outgoing():
                if rnd.random() < loss:
                    continue
                t = now + 5000 + rnd.randint(0, 3000 if reorder else 500)
                if not reorder:
                    t = max(t, last.get(name, 0))
                    last[name] = t
                wire.append((t, addr, pkt, name))
        wire.sort(key=lambda x: x[0])
        while wire and wire[0][0] <= now:
            _, dst, pkt, src = wire.pop(0)
            (b if dst == "B" else a).incoming(pkt, src, now)
        for c in b.accepted():
            cb = c
        if cb is not None:
            got += b.read(cb)
            if b.eof(cb):
                break
        a.tick(now)
        b.tick(now)
    return bytes(got) == data, (cb is not None and b.eof(cb)), a.stats(ca)


@pytest.mark.parametrize("loss,reorder", [(0.0, False), (0.03, False), (0.05, True)])
def test_engine_reliable_in_order_delivery(loss, reorder):
    ok, eof, st = _simulate(loss, 300_000, reorder=reorder)
    assert ok and eof, st
    if loss:
        assert st["retransmits"] > 0


def test_engine_rejects_garbage_and_resets_unknown():
    e = _utp.Engine(3)
    assert e.incoming(b"\x00" * 5, "X:1", 0) == -1
    # DATA for an unknown connection -> we answer with a RESET
    pkt = bytes([0x01, 0, 0x12, 0x34]) + b"\x00" * 16
    assert e.incoming(pkt, "X:1", 0) == -1
    out = e.outgoing()
    assert out and out[0][1][0] >> 4 == 3


def test_asyncio_socket_pair_transfer():
    async def main():
        srv = await UtpSocket().start("127.0.0.1", 0)
        cli = await UtpSocket().start("127.0.0.1", 0)
        data = os.urandom(3_000_000)

        async def echo_len():
            r, w, _ = await srv.accept()
            got = await r.readexactly(len(data))
            w.write(len(got).to_bytes(8, "big") + got[-16:])
            await w.drain()
            return got

        t = asyncio.ensure_future(echo_len())
        r, w = await cli.connect("127.0.0.1", srv.port)
        w.write(data)
        await w.drain()
        resp = await asyncio.wait_for(r.readexactly(24), 30)
        assert int.from_bytes(resp[:8], "big") == len(data) and resp[8:] == data[-16:]
        assert await t == data
        w.close()
        cli.close()
        srv.close()
    asyncio.run(asyncio.wait_for(main(), 60))


def test_utp_connect_timeout():
    async def main():
        cli = await UtpSocket().start("127.0.0.1", 0)
        with pytest.raises(ConnectionError):
            await cli.connect("127.0.0.1", 9, timeout=0.3)   # nothing listens there
        cli.close()
    asyncio.run(main())


def test_listen_moves_to_a_port_free_for_tcp_and_udp(tmp_path):
    """A listen port free on TCP but taken on UDP (a DHT node, another
    worker's uTP) moves the torrent to another port pair instead of running
    without uTP, as anacrolix's listenAll retries; a fixed port without the
    fallback keeps TCP and reports uTP off."""
    import socket

    async def main():
        src = tmp_path / "src"
        make_payload(str(src), {"film.mkv": 100_000})
        info = torrent_for(str(src / "film.mkv"), 65536)
        # a UDP port we hold whose TCP twin is free right now (tests running in parallel
        # take ephemeral TCP ports too: pick again if the twin is busy)
        for _ in range(20):
            udp = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
            udp.bind(("127.0.0.1", 0))
            taken = udp.getsockname()[1]
            probe = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            try:
                probe.bind(("127.0.0.1", taken))
                break
            except OSError:
                udp.close()
            finally:
                probe.close()
        try:
            t = Torrent(info.infohash, str(src), TorrentConfig(listen_host="127.0.0.1", seed=True,
                                                               verify_device="cpu", utp=True,
                                                               listen_port=taken), info=info)
            await t.start()
            assert t.utp is not None and t.port != taken and t.utp.port == t.port
            await t.close()
            fixed = Torrent(info.infohash, str(src), TorrentConfig(listen_host="127.0.0.1", seed=True,
                                                                   verify_device="cpu", utp=True, listen_port=taken,
                                                                   listen_port_fallback=False), info=info)
            await fixed.start()
            assert fixed.port == taken and fixed.utp is None
            await fixed.close()
        finally:
            udp.close()
    asyncio.run(asyncio.wait_for(main(), 30))


def test_bittorrent_over_utp_only(tmp_path, monkeypatch):
    async def main():
        src = tmp_path / "src"
        make_payload(str(src), {"film.mkv": 1_500_000})
        info = torrent_for(str(src / "film.mkv"), 65536)
        cfg = TorrentConfig(listen_host="127.0.0.1", seed=True, verify_device="cpu", utp=True)
        st = Torrent(info.infohash, str(src), cfg, info=info)
        await st.start()
        await st.download_all()

        async def no_tcp(self, addr):
            raise OSError("tcp disabled for this test")
        monkeypatch.setattr(Torrent, "_dial_tcp", no_tcp)
        from tritondl.fetch.bt import peer as pw
        delivered = []
        orig = pw.UtpLinkReader.deliver

        def spy(self, data):
            delivered.append(len(data))
            return orig(self, data)
        monkeypatch.setattr(pw.UtpLinkReader, "deliver", spy)   # the native link is fed straight from the engine
        dst = tmp_path / "job"
        os.makedirs(dst)
        dl = TorrentDownloader(TorrentConfig(listen_host="127.0.0.1", utp=True, verify_device="cpu"),
                               progress_interval=0.05, use_dht=False)
        await dl.download(str(dst), lambda u, p: None, magnet_for(info, peers=[("127.0.0.1", st.port)]))
        assert (dst / "film.mkv").read_bytes() == (src / "film.mkv").read_bytes()
        assert sum(delivered) > 1_000_000
        await st.close()
    asyncio.run(asyncio.wait_for(main(), 60))


def test_receive_batch_coalesces_acks():
    """Inside begin_batch/end_batch a burst of DATA yields one cumulative ACK."""
    a, b = _utp.Engine(11), _utp.Engine(12)
    cid = a.connect("B:1", 0)
    for k, pkt in a.outgoing():
        b.incoming(pkt, "A:1", 1)
    (sid,) = b.accepted()
    for k, pkt in b.outgoing():
        a.incoming(pkt, "B:1", 2)
    a.outgoing()
    assert a.write(cid, b"x" * (_utp.MSS * 6)) == _utp.MSS * 6
    a.tick(3)
    burst = [p for _k, p in a.outgoing()]
    assert len(burst) >= 4
    b.begin_batch()
    for p in burst:
        b.incoming(p, "A:1", 4)
    assert b.outgoing() == []            # nothing sent mid-batch
    assert b.end_batch(5) == [sid]
    acks = b.outgoing()
    assert len(acks) == 1 and acks[0][1][0] >> 4 == 2     # one ST_STATE
    assert b.read(sid) == b"x" * (_utp.MSS * len(burst))


from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402


def _pkt(typ, conn_id, seq, ack, ext_chain=b"", first_ext=0, payload=b"", ts=0, ts_diff=0, wnd=1 << 20):
    import struct
    return struct.pack(">BBHIIIHH", (typ << 4) | 1, first_ext, conn_id, ts, ts_diff, wnd, seq, ack) + \
        ext_chain + payload


_packets = st.lists(st.tuples(
    st.integers(0, 6),                                   # type (5, 6 invalid)
    st.sampled_from([0x1000, 0x1001, 0x0fff, 7]),        # conn ids around the live connection
    st.integers(0, 0xFFFF), st.integers(0, 0xFFFF),      # seq, ack
    st.integers(0, 3),                                   # first extension (1 = selective ack)
    st.binary(max_size=40),                              # extension chain bytes (often malformed)
    st.binary(max_size=1500),                            # payload
    st.integers(0, 2**32 - 1), st.integers(0, 2**32 - 1), st.integers(0, 2**32 - 1)),
    max_size=40)


@settings(max_examples=300, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(_packets, st.binary(max_size=64))
def test_engine_survives_any_packet_sequence(pkts, junk):
    """Remote peers control every byte of a uTP datagram: header fields,
    the extension chain (lengths past the end, unknown types, odd SACK
    bitmasks), sequence/ack numbers anywhere in the 16-bit space.  The
    native engine must keep memory-safe (the sanitizer builds run the same
    code) and keep answering; a live connection survives or is reset."""
    e = _utp.Engine(11)
    now = 1_000_000
    e.incoming(_pkt(4, 0x0fff, 100, 0), "P:1", now)          # inbound SYN: conn 0x1000 live
    assert e.accepted()
    for typ, cid, seq, ack, ext, chain, payload, ts, tsd, wnd in pkts:
        now += 997
        r = e.incoming(_pkt(typ, cid, seq, ack, chain, ext, payload, ts, tsd, wnd), "P:1", now)
        assert isinstance(r, int)
        e.tick(now)
        e.outgoing()
    e.incoming(junk, "P:1", now)
    for cid in list(e.accepted()) + [1]:
        e.read(cid)
        e.state(cid)
    e.tick(now + 10_000_000)
    e.outgoing()


def test_out_of_order_buffer_stays_within_the_receive_window():
    """A peer may send up to 1024 packets ahead of the next expected one;
    with 60 KiB datagrams that parked 60 MiB per connection.  What the
    engine holds out of order is capped at the advertised window, and the
    stream still completes in order once the gap is filled."""
    e = _utp.Engine(5)
    now = 1_000_000
    e.incoming(_pkt(4, 0x0fff, 99, 0), "P:1", now)         # SYN seq 99: next DATA expected is 100
    (cid,) = e.accepted()
    big = 60 * 1024
    for k in range(1, 200):                                # seq 101..299, all ahead of 100
        e.incoming(_pkt(0, 0x1000, 100 + k, 0, payload=bytes([k % 256]) * big), "P:1", now)
    assert e.stats(cid)["ooo_bytes"] <= 1 << 20
    small = [bytes([k]) * 1000 for k in range(1, 11)]
    e2 = _utp.Engine(6)
    e2.incoming(_pkt(4, 0x0fff, 99, 0), "P:1", now)
    (c2,) = e2.accepted()
    for k in range(10, 0, -1):                            # 110..101 arrive first, in reverse
        e2.incoming(_pkt(0, 0x1000, 100 + k, 0, payload=small[k - 1]), "P:1", now)
    e2.incoming(_pkt(0, 0x1000, 100, 0, payload=b"head"), "P:1", now)
    assert e2.read(c2) == b"head" + b"".join(small) and e2.stats(c2)["ooo_bytes"] == 0
