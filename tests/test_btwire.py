"""Native peer-wire data plane (csrc/btwire): block assembly into the shared
piece store, request pipelining, choke/reject handling, end-game cancels."""

import struct

import pytest

from tritondl import _btwire as W

B = W.BLOCK


def msgs(out: bytes):
    """Split a peer-wire byte stream into (id, payload) messages."""
    res, pos = [], 0
    while pos < len(out):
        (n,) = struct.unpack(">I", out[pos:pos + 4])
        res.append((out[pos + 4], out[pos + 5:pos + 4 + n]))
        pos += 4 + n
    return res


def piece_msg(i, off, data):
    return struct.pack(">IBII", 9 + len(data), 7, i, off) + data


def test_requests_pipeline_and_completion():
    store = W.PieceStore(3, 4 * B, 10 * B + 100)          # pieces of 4, 4, 2(+100 B) blocks
    assert [store.blocks(i) for i in range(3)] == [4, 4, 3] and store.piece_size(2) == 2 * B + 100
    link = W.Link(store, pipeline=5)
    link.assign(0)
    link.assign(2)
    assert link.pump() == b""                              # choked: nothing requested yet
    ev, out = link.feed(b"\x00\x00\x00\x01\x01")         # UNCHOKE
    assert list(ev) == [("unchoke",)]
    reqs = [struct.unpack(">III", p) for mid, p in msgs(out) if mid == 6]
    assert reqs == [(0, 0, B), (0, B, B), (0, 2 * B, B), (0, 3 * B, B), (2, 0, B)]
    assert link.need_work() and link.outstanding == 5      # only 2 unrequested blocks queued behind the pipeline
    data0 = bytes(range(256)) * (4 * B // 256)
    stream = b"".join(piece_msg(0, k * B, data0[k * B:(k + 1) * B]) for k in range(4))
    ev, out = link.feed(stream[:1000])                    # partial message: buffered
    assert list(ev) == [] and link.buffered == 1000
    ev, out = link.feed(stream[1000:])
    assert list(ev) == [("piece", 0)]
    assert bytes(store.take(0)) == data0 and not store.active(0)
    # the freed pipeline slots went to the rest of piece 2 (the tail block is short)
    reqs = [struct.unpack(">III", p) for mid, p in msgs(out) if mid == 6]
    assert reqs == [(2, B, B), (2, 2 * B, 100)]
    assert link.downloaded == 4 * B


def test_choke_lapses_and_reject_rerequests():
    store = W.PieceStore(1, 4 * B, 4 * B)
    link = W.Link(store, pipeline=4, fast=False)
    link.assign(0)
    link.peer_choking = False
    assert len(msgs(link.pump())) == 4
    ev, out = link.feed(b"\x00\x00\x00\x01\x00")         # CHOKE drops every pending request
    assert list(ev) == [("choke",)] and link.outstanding == 0 and out == b""
    ev, out = link.feed(b"\x00\x00\x00\x01\x01")
    assert len([m for m in msgs(out) if m[0] == 6]) == 4     # all asked for again after UNCHOKE
    fast = W.Link(W.PieceStore(1, 2 * B, 2 * B), pipeline=4, fast=True)
    fast.assign(0)
    fast.peer_choking = False
    fast.pump()
    ev, out = fast.feed(b"\x00\x00\x00\x01\x00")          # BEP 6: choke does not drop requests
    assert fast.outstanding == 2
    fast.peer_choking = False
    rej = struct.pack(">IBIII", 13, 16, 0, B, B)             # ... an explicit REJECT does
    ev, out = fast.feed(rej)
    assert [struct.unpack(">III", p) for m, p in msgs(out) if m == 6] == [(0, B, B)]


def test_endgame_two_links_share_the_store_and_cancel():
    store = W.PieceStore(1, 2 * B, 2 * B)
    a, b = W.Link(store, 8), W.Link(store, 8)
    for l in (a, b):
        l.assign(0)
        l.peer_choking = False
        assert len(msgs(l.pump())) == 2                    # both ask for both blocks (end game)
    ev, _ = a.feed(piece_msg(0, 0, b"x" * B))
    assert list(ev) == []
    ev, _ = b.feed(piece_msg(0, B, b"y" * B))
    assert list(ev) == [("piece", 0)]                      # completed by the second link's block
    a.piece_done(0)
    cancels = [struct.unpack(">III", p) for m, p in msgs(a.pump()) if m == 8]
    assert sorted(cancels) == [(0, B, B)]                 # a still had block 1 outstanding
    assert bytes(store.take(0)) == b"x" * B + b"y" * B
    ev, _ = a.feed(piece_msg(0, 0, b"z" * B))             # late duplicate: ignored
    assert list(ev) == []


def test_unrequested_blocks_are_dropped_not_stored():
    """A peer pushing blocks nobody asked it for cannot write into pieces other
    links are filling; blocks of requests withdrawn lately (lapsed, or
    cancelled because another link finished the piece) are still taken."""
    store = W.PieceStore(2, 2 * B, 4 * B)
    honest, pusher = W.Link(store, 2), W.Link(store, 2)
    honest.assign(0)
    honest.peer_choking = False
    assert len(msgs(honest.pump())) == 2                   # honest asked for piece 0's two blocks
    ev, _ = pusher.feed(piece_msg(0, 0, b"E" * B) + piece_msg(0, B, b"E" * B))
    assert list(ev) == [] and pusher.wasted == 2 * B and store.received(0) == 0
    ev, _ = honest.feed(piece_msg(0, 0, b"g" * B) + piece_msg(0, B, b"g" * B))
    assert list(ev) == [("piece", 0)] and bytes(store.take(0)) == b"g" * 2 * B
    late = W.Link(store, 4, False)
    late.assign(1)
    late.peer_choking = False
    late.pump()
    late.feed(b"\x00\x00\x00\x01\x00")                     # CHOKE: both requests lapse
    ev, _ = late.feed(piece_msg(1, 0, b"a" * B))           # ... but a block already in flight is kept
    assert late.wasted == 0 and store.received(1) == 1
    ev, _ = late.feed(piece_msg(1, 0, b"a" * B))           # the same block again: not asked any more
    assert late.wasted == B


def test_forwarded_messages_and_protocol_errors():
    store = W.PieceStore(2, B, 2 * B)
    link = W.Link(store, 4)
    have = struct.pack(">IBI", 5, 4, 1)
    ev, _ = link.feed(b"\x00\x00\x00\x00" + have)         # keep-alive + HAVE 1
    assert list(ev) == [("msg", 4, b"\x00\x00\x00\x01")]
    store.begin(0)
    ev, _ = link.feed(piece_msg(0, 3, b"q" * B))           # misaligned block
    assert ev[-1][0] == "bad"
    link2 = W.Link(store, 4)
    ev, _ = link2.feed(struct.pack(">I", 64 << 20))        # absurd length
    assert ev[-1] == ("bad", "message too large")
    link3 = W.Link(store, 4)
    ev, _ = link3.feed(piece_msg(9, 0, b"q" * 10))
    assert ev[-1][0] == "bad"
    with pytest.raises(IndexError):
        link3.assign(7)
    assert store.partial_bytes == 0


def test_take_is_zero_copy_and_recycles_buffers():
    store = W.PieceStore(4, 2 * B, 8 * B)
    for i in range(2):
        store.begin(i)
        store.put(i, 0, bytes([i + 1]) * B)
        store.put(i, B, bytes([i + 1]) * B)
    p0 = store.take(0)
    mv = memoryview(p0)
    assert mv.readonly and len(mv) == 2 * B and len(p0) == 2 * B
    assert mv[:4].tobytes() == b"\x01" * 4 and p0.tobytes() == b"\x01" * (2 * B)
    assert store.pooled == 0
    del p0
    assert store.pooled == 0            # the memoryview still holds it
    mv.release()
    del mv
    assert store.pooled == 1
    store.begin(2)                      # reuses the recycled buffer
    assert store.pooled == 0
    store.reset(2)
    assert store.pooled == 1


def test_zero_copy_receive_buffer_keeps_partial_messages():
    """recv_buffer/feed_n (the BufferedProtocol path): bytes written into the
    view are parsed in place; a message split across reads is completed by
    the next one even after the buffer compacts."""
    store = W.PieceStore(1, 4 * B, 4 * B)
    link = W.Link(store, pipeline=8)
    link.assign(0)
    link.peer_choking = False
    link.pump()
    data = bytes(range(256)) * (4 * B // 256)
    stream = b"\x00\x00\x00\x00" + b"".join(piece_msg(0, k * B, data[k * B:(k + 1) * B]) for k in range(4)) \
        + struct.pack(">IBI", 5, 4, 0)                    # keepalive, 4 blocks, HAVE 0
    events, pos = [], 0
    for cut in (3, 20000, 7, 30000, len(stream)):
        chunk = stream[pos:min(cut + pos, len(stream))]
        view = link.recv_buffer(1 << 16)
        assert len(view) >= len(chunk) and not view.readonly
        view[:len(chunk)] = chunk
        ev, _out = link.feed_n(len(chunk))
        events += list(ev)
        pos += len(chunk)
        if pos == len(stream):
            break
    assert events == [("piece", 0), ("msg", 4, b"\x00\x00\x00\x00")]
    assert bytes(store.take(0)) == data and link.buffered == 0
    with pytest.raises(IndexError):
        link.feed_n(1 << 30)


def test_download_uses_zero_copy_receive(tmp_path):
    """A plain-TCP leecher switches its peer connections to LinkReader."""
    import asyncio

    from tritondl_testkit.fakes.swarm import Seeder, magnet_for, make_payload, torrent_for
    from tritondl.fetch.bt.client import TorrentDownloader
    from tritondl.fetch.bt.torrent import TorrentConfig

    async def main():
        src = tmp_path / "src"
        make_payload(str(src / "P"), {"a.bin": 3_000_000})
        info = torrent_for(str(src / "P"), 65536)
        seed = await Seeder(info, str(src)).start()
        d = TorrentDownloader(TorrentConfig(listen_host="127.0.0.1"), use_dht=False)
        t, _ = await d.open(str(tmp_path / "dst"), magnet_for(info) + f"&x.pe=127.0.0.1:{seed.torrent.port}")
        await asyncio.wait_for(t.got_info.wait(), 20)
        await t.download_all()
        await asyncio.wait_for(t.complete.wait(), 30)
        assert any(p.rx is not None for p in t.peers.values())
        await t.close()
        await seed.stop()
    asyncio.run(main())


def test_link_serves_requests_from_source(tmp_path):
    """REQUESTs are answered natively from the files (padding reads as zeros,
    reads cross file boundaries); what cannot be served is REJECTed on a fast
    connection; the source keeps its own fd dups and stops on close()."""
    import os
    a, b = os.urandom(3 * B + 100), os.urandom(2 * B)
    pa, pb = tmp_path / "a", tmp_path / "b"
    pa.write_bytes(a)
    pb.write_bytes(b)
    pad = 500                                      # BEP 47 padding between the files
    stream = a + bytes(pad) + b
    plen = 2 * B
    n = (len(stream) + plen - 1) // plen
    src = W.Source(n, plen, len(stream))
    fa, fb = os.open(pa, os.O_RDONLY), os.open(pb, os.O_RDONLY)
    src.add_file(fa, 0, len(a))
    src.add_file(-1, len(a), pad)
    src.add_file(fb, len(a) + pad, len(b))
    os.close(fa)                                   # the source holds dups
    os.close(fb)
    src.set_have_bits(bytes([1] * (n - 1) + [0]))
    link = W.Link(W.PieceStore(n, plen, len(stream)), pipeline=4, fast=True)
    link.set_source(src)

    def req(i, off, ln):
        return struct.pack(">IBIII", 13, 6, i, off, ln)
    ev, out = link.feed(req(1, B, B) + req(1, 0, 100) + req(n - 1, 0, 10) + req(0, 0, 200 * 1024) +
                        struct.pack(">IBIII", 13, 8, 1, B, B))             # + a CANCEL: absorbed
    assert list(ev) == []
    got = msgs(out)
    assert got[0] == (7, struct.pack(">II", 1, B) + stream[plen + B:plen + 2 * B])   # crosses a -> padding
    assert got[1] == (7, struct.pack(">II", 1, 0) + stream[plen:plen + 100])
    assert got[2] == (16, struct.pack(">III", n - 1, 0, 10))                  # not ours yet
    assert got[3] == (16, struct.pack(">III", 0, 0, 200 * 1024))              # oversized
    assert link.uploaded == B + 100
    src.set_have(n - 1)
    ev, out = link.feed(req(n - 1, 0, 10))
    last = (n - 1) * plen
    assert msgs(out) == [(7, struct.pack(">II", n - 1, 0) + stream[last:last + 10])]
    link.serving = False                           # choked: refuse
    assert msgs(link.feed(req(0, 0, 10))[1])[0][0] == 16
    link.serving = True
    src.close()
    assert msgs(link.feed(req(0, 0, 10))[1])[0][0] == 16 and not src.has(0)
    plain = W.Link(W.PieceStore(n, plen, len(stream)), pipeline=4, fast=False)
    ev, out = plain.feed(req(0, 0, 10))            # no source: Python sees the REQUEST
    assert list(ev) == [("msg", 6, struct.pack(">III", 0, 0, 10))] and out == b""


def test_malformed_block_from_a_scripted_peer_drops_it(tmp_path):
    """End to end on the zero-copy path: a scripted seed answers the first
    REQUEST properly, then sends a PIECE of the wrong length; the native
    link flags it, the Torrent drops that connection (the peer sees EOF)
    and keeps the good block."""
    import asyncio

    from tritondl_testkit.fakes.swarm import make_payload, torrent_for
    from tritondl.fetch.bt import peer as pw
    from tritondl.fetch.bt.torrent import Torrent, TorrentConfig

    async def main():
        src = tmp_path / "src"
        make_payload(str(src / "P"), {"a.bin": 4 * B})
        info = torrent_for(str(src / "P"), 2 * B)
        payload = (src / "P" / "a.bin").read_bytes()
        seen: dict = {"eof": asyncio.Event(), "requests": []}

        async def scripted(r: asyncio.StreamReader, w: asyncio.StreamWriter) -> None:
            await pw.read_handshake(r)
            w.write(pw.encode_handshake(info.infohash, b"-SCRIPT-" + bytes(12)))
            w.write(struct.pack(">IB", 1, pw.HAVE_ALL) + struct.pack(">IB", 1, pw.UNCHOKE))
            try:
                while True:
                    (n,) = struct.unpack(">I", await r.readexactly(4))
                    body = await r.readexactly(n) if n else b""
                    if body[:1] != bytes([pw.REQUEST]):
                        continue
                    i, off, ln = struct.unpack(">III", body[1:13])
                    seen["requests"].append((i, off, ln))
                    data = payload[i * 2 * B + off:i * 2 * B + off + ln]
                    if len(seen["requests"]) == 2:
                        data = data[:-1]                    # short block: a protocol violation
                    w.write(struct.pack(">IBII", 9 + len(data), pw.PIECE, i, off) + data)
                    await w.drain()
            except (asyncio.IncompleteReadError, ConnectionError):
                seen["eof"].set()

        srv = await asyncio.start_server(scripted, "127.0.0.1", 0)
        port = srv.sockets[0].getsockname()[1]
        cfg = TorrentConfig(listen_host="127.0.0.1", verify_device="cpu", utp=False, encryption="disable")
        t = Torrent(info.infohash, str(tmp_path / "dst"), cfg, info=info)
        await t.start()
        await t.download_all()
        t.add_peer_addr(("127.0.0.1", port))
        await asyncio.wait_for(seen["eof"].wait(), 10)
        assert len(seen["requests"]) >= 2
        assert t.store is not None and t.store.partial_bytes >= B     # the good block stayed
        assert ("127.0.0.1", port) not in t.peers
        await t.close()
        srv.close()
    asyncio.run(main())


def test_take_over_resumes_a_transport_the_stream_reader_paused():
    """A StreamReader pauses its transport when its buffer passes the limit;
    switching to LinkReader must hand over those bytes AND resume reading,
    or the connection would stall forever."""
    import asyncio

    from tritondl.fetch.bt import peer as pw

    async def main():
        got = bytearray()
        done = asyncio.Event()

        async def serve(r, w):
            w.write(b"\x00\x00\x00\x00" * 100_000)              # 400 KB of keep-alives
            await w.drain()
            w.write(struct.pack(">IB", 5, 4) + struct.pack(">I", 7))   # then a HAVE
            await w.drain()
            await done.wait()
            w.close()

        srv = await asyncio.start_server(serve, "127.0.0.1", 0)
        r, w = await asyncio.open_connection("127.0.0.1", srv.sockets[0].getsockname()[1], limit=1 << 16)
        for _ in range(250):                                     # buffer fills past 2*limit: paused
            if not w.transport.is_reading():
                break
            await asyncio.sleep(0.02)
        assert not w.transport.is_reading()
        wire = pw.Wire(r, w)
        link = W.Link(W.PieceStore(1, B, B), 4, False)
        msgs = []

        def on_data(n):
            ev, _out = link.feed_n(n)
            for e in ev:
                if e[0] == "msg":
                    msgs.append(e)
            if msgs:
                done.set()
        rx, leftover = wire.take_over(link, on_data)
        assert leftover and w.transport.is_reading()
        ev, _out = link.feed(leftover)
        msgs += [e for e in ev if e[0] == "msg"]
        await asyncio.wait_for(done.wait(), 5)
        assert msgs == [("msg", 4, struct.pack(">I", 7))]
        w.close()
        srv.close()
    asyncio.run(main())


@pytest.mark.parametrize("native", [True, False])
@pytest.mark.parametrize("fast", [True, False])
def test_download_completes_against_chaotic_scripted_peers(tmp_path, fast, native):
    """Native links under churn: scripted seeds that randomly choke/unchoke
    (dropping queued requests), REJECT (fast), ignore requests, and hang up
    mid-stream.  The leecher must still finish with byte-exact data."""
    import asyncio
    import random

    from tritondl_testkit.fakes.swarm import make_payload, torrent_for
    from tritondl.fetch.bt import peer as pw
    from tritondl.fetch.bt.torrent import Torrent, TorrentConfig

    async def main():
        src = tmp_path / "src"
        make_payload(str(src / "P"), {"a.bin": 3_000_000 + 123})
        info = torrent_for(str(src / "P"), 32 * 1024)
        payload = (src / "P" / "a.bin").read_bytes()
        rng = random.Random(1234 + fast)
        reserved = bytearray(8)
        if fast:
            reserved[7] |= 0x04

        async def chaotic(r: asyncio.StreamReader, w: asyncio.StreamWriter) -> None:
            try:
                await pw.read_handshake(r)
                w.write(pw.encode_handshake(info.infohash, b"-CHAOS-" + bytes(13), bytes(reserved)))
                w.write(struct.pack(">IB", 1, pw.HAVE_ALL) if fast else
                        struct.pack(">IB", 1 + len(pw.set_to_bits([True] * info.num_pieces, info.num_pieces)),
                                    pw.BITFIELD) + pw.set_to_bits([True] * info.num_pieces, info.num_pieces))
                choked = True
                budget = rng.randint(20, 200)              # blocks before hanging up
                while budget > 0:
                    if choked and rng.random() < 0.5:
                        w.write(struct.pack(">IB", 1, pw.UNCHOKE))
                        choked = False
                    (n,) = struct.unpack(">I", await asyncio.wait_for(r.readexactly(4), 5))
                    body = await r.readexactly(n) if n else b""
                    if body[:1] != bytes([pw.REQUEST]):
                        continue
                    i, off, ln = struct.unpack(">III", body[1:13])
                    x = rng.random()
                    if choked or x < 0.05:
                        if fast:
                            w.write(struct.pack(">IBIII", 13, pw.REJECT, i, off, ln))
                        continue                             # non-fast: silently dropped
                    if x < 0.08:
                        w.write(struct.pack(">IB", 1, pw.CHOKE))
                        choked = True
                        continue
                    if x < 0.10:
                        continue                             # ignored: the timeout path re-asks
                    data = payload[i * info.piece_length + off:i * info.piece_length + off + ln]
                    w.write(struct.pack(">IBII", 9 + len(data), pw.PIECE, i, off) + data)
                    budget -= 1
                    await w.drain()
            except (asyncio.IncompleteReadError, ConnectionError, asyncio.TimeoutError):
                pass
            finally:
                w.close()

        servers = [await asyncio.start_server(chaotic, "127.0.0.1", 0) for _ in range(3)]
        addrs = [("127.0.0.1", s.sockets[0].getsockname()[1]) for s in servers]
        cfg = TorrentConfig(listen_host="127.0.0.1", verify_device="cpu", utp=False, request_timeout=1.0,
                            pipeline=16, native_wire=native)
        t = Torrent(info.infohash, str(tmp_path / "dst"), cfg, info=info, peers=addrs)
        await t.start()
        await t.download_all()

        async def redial():                                  # scripted seeds hang up: keep dialing them
            while not t.complete.is_set():
                for a in addrs:
                    t.banned.discard(a)
                    t.add_peer_addr(a)
                await asyncio.sleep(0.1)
        dialer = asyncio.ensure_future(redial())
        try:
            await asyncio.wait_for(t.complete.wait(), 60)
        finally:
            dialer.cancel()
        assert t.store is None or t.store.partial_bytes == 0
        mine = ~int.from_bytes(t.have, "little")
        for q in t.peers.values():                       # O(1) interest counters == the bitmap truth
            assert q.wants == (int.from_bytes(q.have, "little") & mine).bit_count() == 0
        with open(tmp_path / "dst" / "P" / "a.bin", "rb") as f:
            assert f.read() == payload
        await t.close()
        for s in servers:
            s.close()
    asyncio.run(main())


def test_native_serving_backpressure_bounds_the_write_buffer(tmp_path):
    """A peer that pipelines thousands of REQUESTs but does not read: the
    seeder's link answers as it parses, the transport signals pause_writing
    and LinkReader stops reading, so the seeder's write buffer stays bounded;
    once the peer reads, every request is answered with the right bytes."""
    import asyncio

    from tritondl_testkit.fakes.swarm import make_payload, torrent_for
    from tritondl.fetch.bt import peer as pw
    from tritondl.fetch.bt.torrent import Torrent, TorrentConfig

    async def main():
        src = tmp_path / "src"
        make_payload(str(src / "P"), {"a.bin": 8 << 20})
        info = torrent_for(str(src / "P"), 1 << 20)
        payload = (src / "P" / "a.bin").read_bytes()
        seed = Torrent(info.infohash, str(src), TorrentConfig(listen_host="127.0.0.1", seed=True, verify_device="cpu",
                                                              utp=False, encryption="disable"), info=info)
        await seed.start()
        await seed.download_all()
        r, w = await asyncio.open_connection("127.0.0.1", seed.port)
        w.transport.set_write_buffer_limits(1 << 20)
        sock = w.get_extra_info("socket")
        import socket as _s
        sock.setsockopt(_s.SOL_SOCKET, _s.SO_RCVBUF, 64 << 10)   # keep the kernel's share small
        w.write(pw.encode_handshake(info.infohash, b"-BPTEST-" + bytes(12)))
        await pw.read_handshake(r)
        reqs = [(i, off) for _rep in range(4) for i in range(8) for off in range(0, 1 << 20, B)]
        w.write(b"".join(struct.pack(">IBIII", 13, pw.REQUEST, i, off, B) for i, off in reqs))
        await w.drain()
        await asyncio.sleep(0.5)                                # seeder answers until its socket backs up
        for _ in range(250):
            peers = list(seed.peers.values())
            if peers and peers[0].rx is not None:
                break
            await asyncio.sleep(0.02)
        (peer,) = list(seed.peers.values())
        assert peer.rx is not None
        buffered = peer.wire.writer.transport.get_write_buffer_size()
        assert buffered < (24 << 20), buffered                  # 32 MiB were requested
        got = 0
        while got < len(reqs):                                   # now read everything back
            (n,) = struct.unpack(">I", await asyncio.wait_for(r.readexactly(4), 10))
            body = await r.readexactly(n)
            if body[:1] != bytes([pw.PIECE]):
                continue
            i, off = struct.unpack(">II", body[1:9])
            assert body[9:] == payload[i * (1 << 20) + off:i * (1 << 20) + off + B]
            got += 1
        w.close()
        await seed.close()
    asyncio.run(asyncio.wait_for(main(), 60))


def test_native_serving_backpressure_over_utp(tmp_path):
    """The same over uTP: the seeder's uTP reader stops taking bytes while its
    send side is backed up (they stay in the engine, whose advertised window
    closes), so the served replies stay bounded; the leecher's own reader is
    flow-controlled the same way (pause_reading on the uTP transport)."""
    import asyncio

    from tritondl_testkit.fakes.swarm import make_payload, torrent_for
    from tritondl.fetch.bt import peer as pw
    from tritondl.fetch.bt.torrent import Torrent, TorrentConfig
    from tritondl.fetch.bt.utp import UtpSocket

    async def main():
        src = tmp_path / "src"
        make_payload(str(src / "P"), {"a.bin": 8 << 20})
        info = torrent_for(str(src / "P"), 1 << 20)
        payload = (src / "P" / "a.bin").read_bytes()
        seed = Torrent(info.infohash, str(src), TorrentConfig(listen_host="127.0.0.1", seed=True, verify_device="cpu",
                                                              utp=True, encryption="disable"), info=info)
        await seed.start()
        await seed.download_all()
        cli = await UtpSocket().start("127.0.0.1", 0)
        r, w = await cli.connect("127.0.0.1", seed.port)
        w.write(pw.encode_handshake(info.infohash, b"-BPTEST-" + bytes(12)))
        await pw.read_handshake(r)
        w.transport.pause_reading()                            # the leecher stops reading: its window closes
        reqs = [(i, off) for _rep in range(4) for i in range(8) for off in range(0, 1 << 20, B)]
        for _ in range(250):
            peers = list(seed.peers.values())
            if peers and peers[0].rx is not None:
                break
            await asyncio.sleep(0.02)
        (peer,) = list(seed.peers.values())
        assert peer.rx is not None
        # the REQUESTs trickle in (keep-alives in between): every delivery is a new
        # chance to serve, so only a paused reader keeps the replies bounded
        for k in range(0, len(reqs), 64):
            w.write(b"".join(struct.pack(">IBIII", 13, pw.REQUEST, i, off, B) for i, off in reqs[k:k + 64]))
            w.write(b"\x00\x00\x00\x00")
            await asyncio.sleep(0.01)
        await asyncio.sleep(0.5)
        buffered = peer.wire.writer.transport.get_write_buffer_size()
        assert buffered < (16 << 20), buffered                  # 32 MiB were requested
        assert peer.link.uploaded < (24 << 20)                  # the rest waits, unparsed, in the engine
        assert len(r._buffer) < (2 << 20)                       # the paused leecher holds ~ one window
        w.transport.resume_reading()
        got = 0
        while got < len(reqs):                                   # now read everything back
            (n,) = struct.unpack(">I", await asyncio.wait_for(r.readexactly(4), 20))
            body = await asyncio.wait_for(r.readexactly(n), 20)
            if body[:1] != bytes([pw.PIECE]):
                continue
            i, off = struct.unpack(">II", body[1:9])
            assert body[9:] == payload[i * (1 << 20) + off:i * (1 << 20) + off + B]
            got += 1
        w.close()
        cli.close()
        await seed.close()
    asyncio.run(asyncio.wait_for(main(), 90))


def test_link_serve_budget_stalls_and_resumes(tmp_path):
    """One feed answers at most ~2 MiB of PIECEs; the rest of the REQUESTs
    stay buffered (stalled) until feed(b"") is called again."""
    import os
    data = os.urandom(4 << 20)
    (tmp_path / "f").write_bytes(data)
    src = W.Source(4, 1 << 20, len(data))
    fd = os.open(tmp_path / "f", os.O_RDONLY)
    src.add_file(fd, 0, len(data))
    os.close(fd)
    src.set_have_bits(b"\x01" * 4)
    link = W.Link(W.PieceStore(4, 1 << 20, len(data)), pipeline=4, fast=True)
    link.set_source(src)
    reqs = [(i, off) for i in range(4) for off in range(0, 1 << 20, B)]
    _ev, out = link.feed(b"".join(struct.pack(">IBIII", 13, 6, i, off, B) for i, off in reqs))
    served = msgs(out)
    assert link.stalled and (2 << 20) <= len(out) < (2 << 20) + B + 64
    rounds = 1
    while link.stalled:
        _ev, out = link.feed(b"")
        served += msgs(out)
        rounds += 1
    assert rounds == 2 and len(served) == len(reqs) and link.buffered == 0
    for (mid, pl), (i, off) in zip(served, reqs):
        assert mid == 7 and pl[:8] == struct.pack(">II", i, off)
        assert pl[8:] == data[i * (1 << 20) + off:i * (1 << 20) + off + B]


def test_seeding_falls_back_to_python_when_the_native_source_fails(tmp_path, monkeypatch):
    """If the serving Source cannot be built (e.g. no descriptors left for the
    fd dups), the Torrent keeps its native links but answers REQUESTs in
    Python; a download from it still completes."""
    import asyncio
    import types

    from tritondl_testkit.fakes.swarm import Seeder, magnet_for, make_payload, torrent_for
    from tritondl.fetch.bt import torrent as tmod
    from tritondl.fetch.bt.client import TorrentDownloader
    from tritondl.fetch.bt.torrent import TorrentConfig

    class NoFds:
        def __init__(self, *a):
            pass

        def add_file(self, *a):
            raise RuntimeError("dup failed")

        def close(self):
            pass
    shim = types.SimpleNamespace(PieceStore=W.PieceStore, Link=W.Link, Source=NoFds)

    async def main():
        src = tmp_path / "src"
        make_payload(str(src / "P"), {"a.bin": 2_000_000})
        info = torrent_for(str(src / "P"), 65536)
        monkeypatch.setattr(tmod, "_W", shim)
        seed = await Seeder(info, str(src)).start()
        assert seed.torrent.source is None and seed.torrent.store is not None
        d = TorrentDownloader(TorrentConfig(listen_host="127.0.0.1"), use_dht=False)
        t, _ = await d.open(str(tmp_path / "dst"), magnet_for(info) + f"&x.pe=127.0.0.1:{seed.torrent.port}")
        await asyncio.wait_for(t.got_info.wait(), 20)
        await t.download_all()
        await asyncio.wait_for(t.complete.wait(), 30)
        assert (tmp_path / "dst" / "P" / "a.bin").read_bytes() == (src / "P" / "a.bin").read_bytes()
        await t.close()
        await seed.stop()
    asyncio.run(main())
