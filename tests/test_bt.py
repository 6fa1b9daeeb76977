"""BitTorrent stack: bencode, metainfo/magnets, and full downloads against a
local swarm (HTTP tracker, UDP tracker, DHT, direct peers, .torrent over
HTTP, resume from partial data, corrupt seeder)."""

import asyncio
import hashlib
import os
import shutil
import time

import pytest

from tritondl_testkit.fakes.origin import Origin
from tritondl_testkit.fakes.swarm import (DHTNetwork, HTTPTracker, Seeder, UDPTracker, magnet_for, make_payload,
                                  torrent_file_bytes, torrent_for)
from tritondl.fetch.bt import bencode
from tritondl.fetch.bt.client import TorrentDownloader, TorrentError
from tritondl.fetch.bt.metainfo import Metainfo, MetainfoError, parse_magnet
from tritondl.fetch.bt.torrent import TorrentConfig
from tritondl.fetch.bt.tracker import Announce, parse_compact
from tritondl.select import dir_media


def run(coro, timeout=90):
    return asyncio.run(asyncio.wait_for(coro, timeout))


# ----------------------------------------------------------------- bencode


def test_bencode_roundtrip_and_errors():
    v = {b"a": [1, -2, b"xyz", {b"n": 0}], b"b": b""}
    assert bencode.decode(bencode.encode(v)) == v
    assert bencode.encode({"b": 1, "a": 2}) == b"d1:ai2e1:bi1ee"
    for bad in [b"i01e", b"i-0e", b"3:ab", b"l", b"d1:ai1e", b"x", b"i1ei2e", b"02:ab"]:
        with pytest.raises(bencode.BencodeError):
            bencode.decode(bad)


def test_spans_give_raw_info():
    info = b"d4:name1:x12:piece lengthi16384e6:pieces0:6:lengthi0ee"
    d, spans = bencode.decode_with_spans(b"d8:announce3:url4:info" + info + b"e")
    s, e = spans[b"info"]
    assert (b"d8:announce3:url4:info" + info + b"e")[s:e] == info


# ----------------------------------------------------------------- metainfo


def test_metainfo_single_and_multi(tmp_path):
    make_payload(str(tmp_path / "show"), {"season 1/e1.mkv": 100_000, "season 1/e2.mkv": 50_001})
    info = torrent_for(str(tmp_path / "show"), 32768)
    assert info.multi and info.name == "show" and info.total_length == 150_001
    assert info.num_pieces == -(-150_001 // 32768)
    mi = Metainfo.parse(torrent_file_bytes(info, ["http://t/announce"]))
    assert mi.infohash == info.infohash and mi.announce == [["http://t/announce"]]
    paths = info.file_paths("/base")
    assert paths[0][0] == "/base/show/season 1/e1.mkv"
    single = torrent_for(str(tmp_path / "show" / "season 1" / "e2.mkv"), 16384)
    assert not single.multi and single.file_paths("/b") == [("/b/e2.mkv", 50_001)]


def test_metainfo_rejects_traversal():
    bad = bencode.encode({b"name": b"x", b"piece length": 16384, b"pieces": b"",
                          b"files": [{b"length": 0, b"path": [b"..", b"etc"]}]})
    with pytest.raises(MetainfoError):
        from tritondl.fetch.bt.metainfo import Info
        Info.parse(bad)


def test_magnet_parse():
    ih = hashlib.sha1(b"x").digest()
    m = parse_magnet(f"magnet:?xt=urn:btih:{ih.hex()}&dn=My%20Show&tr=http%3A%2F%2Ft%2Fa&x.pe=1.2.3.4:5")
    assert m.infohash == ih and m.display_name == "My Show" and m.trackers == ["http://t/a"]
    assert m.peers == [("1.2.3.4", 5)]
    import base64
    m2 = parse_magnet("magnet:?xt=urn:btih:" + base64.b32encode(ih).decode())
    assert m2.infohash == ih
    assert parse_magnet(m.uri()).infohash == ih
    with pytest.raises(MetainfoError):
        parse_magnet("magnet:?dn=x")


def test_compact_peers():
    assert parse_compact(bytes([127, 0, 0, 1, 0x1A, 0xE1])) == [("127.0.0.1", 6881)]


def test_http_tracker_reply_is_size_capped():
    """A tracker that streams an endless or huge reply is cut off at
    MAX_REPLY instead of being buffered whole."""
    from tritondl.fetch.bt import tracker as T

    async def main():
        o = await Origin().start()
        url = o.add("/announce", b"d8:intervali60e5:peers" + b"6000000:" + bytes(6_000_000) + b"e")
        a = Announce(hashlib.sha1(b"cap").digest(), b"-A-" + bytes(17), 51413)
        with pytest.raises(T.TrackerError, match="larger than"):
            await T.http_announce(url, a)
        small = o.add("/small", bencode.encode({b"interval": 60, b"peers": bytes([10, 0, 0, 1, 0x1A, 0xE1])}))
        assert (await T.http_announce(small, a)).peers == [("10.0.0.1", 6881)]
        await o.stop()
    run(main())


def test_udp_tracker_over_ipv6_returns_ipv6_peers():
    """BEP 15: over IPv6 the announce reply carries 18-byte peers; read as
    6-byte IPv4 entries they would be three garbage addresses each."""
    from tritondl.fetch.bt.tracker import udp_announce

    async def main():
        tr = await UDPTracker().start("::1")
        assert tr.url.startswith("udp://[::1]:")
        ih = hashlib.sha1(b"v6").digest()
        a1 = Announce(ih, b"-A-" + bytes(17), 51413, 0, 0, 100, "started")
        a2 = Announce(ih, b"-B-" + bytes(17), 6881, 0, 0, 100, "started")
        assert (await udp_announce(tr.url, a1)).peers == []
        r = await udp_announce(tr.url, a2)
        assert r.peers == [("::1", 51413)]
        tr.stop()
    run(main())


# ----------------------------------------------------------------- swarm


def _dl(**kw):
    cfg = TorrentConfig(listen_host="127.0.0.1", tracker_min_interval=0.5, dht_interval=0.5,
                        verify_device="cpu", request_timeout=3)
    return TorrentDownloader(cfg, progress_interval=0.05, use_dht=kw.pop("use_dht", False), **kw)


class Sink:
    def __init__(self):
        self.p = []

    def __call__(self, url, p):
        self.p.append(p)


def _check_tree(src_root, dst_root):
    for root, _d, files in os.walk(src_root):
        for f in files:
            a = os.path.join(root, f)
            b = os.path.join(dst_root, os.path.relpath(a, os.path.dirname(src_root)))
            assert open(a, "rb").read() == open(b, "rb").read(), b


def test_magnet_via_http_tracker_multi_file(tmp_path):
    async def main():
        src = tmp_path / "src" / "My.Show"
        make_payload(str(src), {"season 1/e1.mkv": 700_000, "season 1/e2.mkv": 333_333, "notes.txt": 1000})
        info = torrent_for(str(src), 65536)
        tr = await HTTPTracker().start()
        seeds = [await Seeder(info, str(tmp_path / "src"), trackers=[tr.url]).start() for _ in range(2)]
        await asyncio.sleep(0.2)
        dst = tmp_path / "job"
        os.makedirs(dst)
        sink = Sink()
        await _dl().download(str(dst), sink, magnet_for(info, [tr.url]))
        _check_tree(str(src), str(dst))
        assert sink.p[-1] == 100
        files = dir_media(str(dst))   # sole top-level dir "My.Show" -> season dirs
        assert [os.path.basename(f) for f in files] == ["e1.mkv", "e2.mkv"]
        for s in seeds:
            await s.stop()
        await tr.stop()
    run(main())


def test_magnet_via_udp_tracker_single_file(tmp_path):
    async def main():
        src = tmp_path / "src"
        make_payload(str(src), {"movie.mkv": 1_234_567})
        info = torrent_for(str(src / "movie.mkv"), 32768)
        ut = await UDPTracker().start()
        s = await Seeder(info, str(src), trackers=[ut.url]).start()
        await asyncio.sleep(0.2)
        dst = tmp_path / "job"
        os.makedirs(dst)
        await _dl().download(str(dst), Sink(), magnet_for(info, [ut.url]))
        assert (dst / "movie.mkv").read_bytes() == (src / "movie.mkv").read_bytes()
        await s.stop()
        ut.stop()
    run(main())


def test_magnet_via_dht_only(tmp_path):
    async def main():
        src = tmp_path / "src"
        make_payload(str(src), {"movie.mp4": 600_000})
        info = torrent_for(str(src / "movie.mp4"), 16384)
        net = await DHTNetwork(5).start()
        s = await Seeder(info, str(src), dht_bootstrap=net.bootstrap).start()
        await s.dht.announce_peer(info.infohash, s.torrent.port)
        dst = tmp_path / "job"
        os.makedirs(dst)
        await _dl(use_dht=True, dht_bootstrap=net.bootstrap).download(str(dst), Sink(), magnet_for(info))
        assert (dst / "movie.mp4").read_bytes() == (src / "movie.mp4").read_bytes()
        await s.stop()
        net.stop()
    run(main())


def test_torrent_file_over_http_and_resume(tmp_path):
    async def main():
        src = tmp_path / "src"
        make_payload(str(src), {"film.webm": 2_000_000})
        info = torrent_for(str(src / "film.webm"), 65536)
        s = await Seeder(info, str(src)).start()
        o = await Origin().start()
        tor = torrent_file_bytes(info)
        url = o.add("/x/film.torrent", tor)
        dst = tmp_path / "job"
        os.makedirs(dst)
        # partial pre-existing data: first half correct, second half garbage
        data = (src / "film.webm").read_bytes()
        (dst / "film.webm").write_bytes(data[:1_000_000] + os.urandom(1_000_000))
        d = _dl(extra_trackers=[])
        t, dht = await d.open(str(dst), url)
        t.add_peer_addr(s.addr)
        await t.download_all()
        pre = t.nhave
        assert 0 < pre < info.num_pieces       # resume kept the verified half
        await asyncio.wait_for(t.complete.wait(), 30)
        await t.close()
        assert (dst / "film.webm").read_bytes() == data
        await s.stop()
        await o.stop()
    run(main())


def test_corrupt_seeder_is_banned_and_good_one_used(tmp_path):
    async def main():
        src = tmp_path / "src"
        make_payload(str(src), {"a.mkv": 500_000})
        info = torrent_for(str(src / "a.mkv"), 32768)
        bad = await Seeder(info, str(src), corrupt=True).start()
        good = await Seeder(info, str(src)).start()
        dst = tmp_path / "job"
        os.makedirs(dst)
        await _dl().download(str(dst), Sink(), magnet_for(info, peers=[bad.addr, good.addr]))
        assert (dst / "a.mkv").read_bytes() == (src / "a.mkv").read_bytes()
        await bad.stop()
        await good.stop()
    run(main())


def test_metadata_timeout_and_unsupported_scheme(tmp_path):
    async def main():
        d = _dl(metadata_timeout=0.3)
        with pytest.raises(TorrentError, match="failed to get metadata"):
            await d.download(str(tmp_path), Sink(), "magnet:?xt=urn:btih:" + "ab" * 20)
        with pytest.raises(TorrentError, match="unsupported scheme 'ftp'"):
            await d.download(str(tmp_path), Sink(), "ftp://x/a.torrent")
    run(main())


def test_announce_dataclass():
    a = Announce(b"\x01" * 20, b"-TD0100-" + b"x" * 12, 6881)
    assert a.event == "started"


def test_only_corrupt_seeder_never_completes_and_gets_banned(tmp_path):
    async def main():
        src = tmp_path / "src"
        make_payload(str(src), {"a.mkv": 200_000})
        info = torrent_for(str(src / "a.mkv"), 32768)
        bad = await Seeder(info, str(src), corrupt=True).start()
        dst = tmp_path / "job"
        os.makedirs(dst)
        d = _dl()
        t, _ = await d.open(str(dst), magnet_for(info, peers=[bad.addr]))
        await asyncio.wait_for(t.got_info.wait(), 10)
        await t.download_all()
        for _ in range(100):
            if bad.addr in t.banned:
                break
            await asyncio.sleep(0.05)
        assert bad.addr in t.banned and t.nhave == 0
        await t.close()
        await bad.stop()
    run(main())


# ----------------------------------------------------------------- PEX / web seeds


def test_pex_message_roundtrip():
    from tritondl.fetch.bt import peer as pw
    msg = pw.pex_msg([("10.0.0.1", 6881), ("::1", 7000)], [("10.0.0.2", 1)], {("10.0.0.1", 6881): 0x12})
    d = bencode.decode(msg)
    assert d[b"added.f"] == b"\x12" and len(d[b"added"]) == 6 and len(d[b"added6"]) == 18
    added, dropped = pw.parse_pex(msg)
    assert added == [("10.0.0.1", 6881), ("::1", 7000)] and dropped == [("10.0.0.2", 1)]


def test_pex_introduces_second_seeder(tmp_path):
    """The leecher only knows seeder A; A (connected to B) gossips B via
    ut_pex and the leecher dials B."""
    async def main():
        src = tmp_path / "src"
        make_payload(str(src), {"m.mkv": 400_000})
        info = torrent_for(str(src / "m.mkv"), 16384)
        b = await Seeder(info, str(src)).start()
        a = await Seeder(info, str(src)).start()
        a.torrent.add_peer_addr(b.addr)
        for _ in range(100):
            if b.addr in a.torrent.peers:
                break
            await asyncio.sleep(0.02)
        dst = tmp_path / "job"
        os.makedirs(dst)
        d = _dl()
        d.cfg.pex_interval = 0.1
        t, _ = await d.open(str(dst), magnet_for(info, peers=[a.addr]))
        for _ in range(200):
            a.torrent.pex_round()
            if b.addr in t.peers:
                break
            await asyncio.sleep(0.05)
        assert b.addr in t.peers and t.pex_learned >= 1
        await t.close()
        await a.stop()
        await b.stop()
    run(main())


def test_private_torrent_disables_pex(tmp_path):
    from tritondl.fetch.bt.metainfo import make_info
    async def main():
        src = tmp_path / "src"
        make_payload(str(src), {"p.mkv": 50_000})
        info = make_info(str(src / "p.mkv"), 16384, private=True)
        s = await Seeder(info, str(src)).start()
        assert s.torrent.private
        from tritondl.fetch.bt import peer as pw
        # a ut_pex message to a private torrent is ignored
        s.torrent.cfg.pex = True
        class P:  # minimal stand-in peer
            ext = None
        await s.torrent._on_extended(P(), bytes([pw.UT_PEX_ID]) + pw.pex_msg([("10.9.9.9", 5)], []))
        assert ("10.9.9.9", 5) not in s.torrent.known
        await s.stop()
    run(main())


def test_webseed_only_multi_file_torrent_file(tmp_path):
    """No peers at all: a .torrent with url-list downloads entirely from the
    HTTP web seed (BEP 19 multi-file layout, pieces straddling files)."""
    async def main():
        src = tmp_path / "src" / "Show"
        make_payload(str(src), {"a b.mkv": 300_001, "sub/c.srt": 70_000, "d.txt": 5})
        info = torrent_for(str(src), 32768)
        o = await Origin().start()
        for rel in ("a b.mkv", "sub/c.srt", "d.txt"):
            from urllib.parse import quote
            o.add("/seed/Show/" + quote(rel), (src / rel).read_bytes())
        url = o.add("/t/show.torrent", torrent_file_bytes(info, url_list=[f"http://127.0.0.1:{o.port}/seed/"]))
        dst = tmp_path / "job"
        os.makedirs(dst)
        d = _dl()
        t, _ = await d.open(str(dst), url)
        await t.download_all()
        await asyncio.wait_for(t.complete.wait(), 30)
        ws = t.webseed_clients[0]
        assert ws.pieces_ok == info.num_pieces
        await t.close()
        _check_tree(str(src), str(dst))
        await o.stop()
    run(main())


def test_webseed_ignoring_range_is_streamed_not_buffered_and_dropped_when_far(tmp_path, monkeypatch):
    """A web seed that answers Range requests with 200 and the whole file:
    each span is read by streaming past the prefix, holding only the span;
    once a span would stream past IGNORED_RANGE_MAX_SKIP the seed is
    dropped rather than re-reading a large file per piece."""
    from tritondl.fetch.bt import webseed as W

    async def main(limit):
        monkeypatch.setattr(W, "IGNORED_RANGE_MAX_SKIP", limit)
        src = tmp_path / "src"
        make_payload(str(src), {"film.mkv": 200_000})
        info = torrent_for(str(src / "film.mkv"), 16384)
        o = await Origin().start()
        o.ranges = False
        o.add("/seed/film.mkv", (src / "film.mkv").read_bytes())
        url = o.add("/t.torrent", torrent_file_bytes(info, url_list=[f"http://127.0.0.1:{o.port}/seed/film.mkv"]))
        dst = tmp_path / f"job{limit}"
        os.makedirs(dst)
        t, _ = await _dl().open(str(dst), url)
        await t.download_all()
        ws = t.webseed_clients[0]
        if limit >= 200_000:
            await asyncio.wait_for(t.complete.wait(), 30)
            assert ws.pieces_ok == info.num_pieces and not ws.dead
            assert (dst / "film.mkv").read_bytes() == (src / "film.mkv").read_bytes()
        else:
            for _ in range(200):
                if ws.dead:
                    break
                await asyncio.sleep(0.05)
            assert ws.dead and ws.pieces_ok <= limit // 16384 + 1
        await t.close()
        await o.stop()
    run(main(1 << 20))
    run(main(40_000))


def test_webseed_via_magnet_ws_single_file_and_bad_seed_dropped(tmp_path):
    async def main():
        src = tmp_path / "src"
        make_payload(str(src), {"film.mkv": 200_000})
        info = torrent_for(str(src / "film.mkv"), 16384)
        seeder = await Seeder(info, str(src)).start()   # metadata source (ut_metadata)
        o = await Origin().start()
        o.add("/good/film.mkv", (src / "film.mkv").read_bytes())
        o.add("/bad/film.mkv", os.urandom(200_000))
        dst = tmp_path / "job"
        os.makedirs(dst)
        good = f"http://127.0.0.1:{o.port}/good/film.mkv"
        bad = f"http://127.0.0.1:{o.port}/bad/film.mkv"
        m = magnet_for(info, peers=[seeder.addr], web_seeds=[bad, good])
        assert parse_magnet(m).web_seeds == [bad, good]
        await seeder.stop()                   # after metadata, only the web seeds remain
        d = _dl()
        t, _ = await d.open(str(dst), m)
        seeder2 = await Seeder(info, str(src)).start()
        t.add_peer_addr(seeder2.addr)
        await asyncio.wait_for(t.got_info.wait(), 10)
        await seeder2.stop()
        await t.download_all()
        await asyncio.wait_for(t.complete.wait(), 30)
        wbad, wgood = t.webseed_clients
        assert wbad.dead and wbad.pieces_ok == 0 and wgood.pieces_ok > 0
        await t.close()
        assert (dst / "film.mkv").read_bytes() == (src / "film.mkv").read_bytes()
        await seeder.stop()
        await o.stop()
    run(main())


def test_bep47_padding_files_swarm_resume_and_webseed(tmp_path):
    """Piece-aligned multi-file torrent with BEP 47 padding entries: pad
    files are never created, verification (host + resume) treats them as
    zeros, and both peers and a web seed deliver the real files."""
    from tritondl.fetch.bt.metainfo import make_info
    from tritondl.ops import hashing

    async def main():
        src = tmp_path / "src" / "Pack"
        make_payload(str(src), {"a.mkv": 100_000, "b.mkv": 70_001, "c.txt": 33})
        info = make_info(str(src), 32768, pad=True)
        pads = [f for f in info.files if f.pad]
        assert pads and all(f.offset % 32768 == 0 for f in info.files if not f.pad)
        # native verifiers read "" spans as zeros
        ok = hashing.verify_pieces(info.file_paths(str(tmp_path / "src")), 32768, info.pieces, device="cpu")
        assert all(ok)
        s = await Seeder(info, str(tmp_path / "src")).start()
        dst = tmp_path / "job"
        os.makedirs(dst)
        await _dl().download(str(dst), Sink(), magnet_for(info, peers=[s.addr]))
        _check_tree(str(src), str(dst))
        assert not (dst / "Pack" / ".pad").exists()
        await s.stop()
        # web seed path over the same layout
        o = await Origin().start()
        for rel in ("a.mkv", "b.mkv", "c.txt"):
            o.add("/ws/Pack/" + rel, (src / rel).read_bytes())
        dst2 = tmp_path / "job2"
        os.makedirs(dst2)
        url = o.add("/t.torrent", torrent_file_bytes(info, url_list=[f"http://127.0.0.1:{o.port}/ws/"]))
        await _dl().download(str(dst2), Sink(), url)
        _check_tree(str(src), str(dst2))
        await o.stop()
    run(main())


def test_large_torrent_file_over_http_is_read_whole(tmp_path):
    """A .torrent bigger than one socket read (v2 piece layers, many files)
    must be read to EOF, not truncated at the first chunk."""
    async def main():
        o = await Origin().start()
        o.rate = 2_000_000          # trickle so the body arrives in many reads
        pad = bencode.encode({b"info": {b"name": b"x", b"piece length": 16384, b"pieces": b"",
                                        b"length": 0}, b"comment": b"z" * 300_000})
        url = o.add("/big.torrent", pad)
        d = _dl()
        data = await d._fetch_torrent_file(url)
        assert data == pad
        await o.stop()
    run(main())


def test_watch_files_fires_in_file_order_and_on_resume(tmp_path):
    """Per-file completion (streamed uploads): each watched file fires once
    when its last piece verifies (they are requested first, in layout
    order); unwatched ones never fire; on a redelivered job the resume check
    fires every whole file at once."""
    async def main():
        src = tmp_path / "src" / "Pack"
        make_payload(str(src), {"a.mkv": 3_000_000, "b.mkv": 3_000_000, "c.txt": 1_000_000, "d.mkv": 2_500_000})
        info = torrent_for(str(src), 16384)
        tr = await HTTPTracker().start()
        seed = await Seeder(info, str(tmp_path / "src"), trackers=[tr.url]).start()
        dst = tmp_path / "job"
        os.makedirs(dst)
        order = []
        offered = []

        def pick(paths):
            offered.extend(paths)
            return {p for p in paths if p.endswith(".mkv")}

        await _dl().download(str(dst), Sink(), magnet_for(info, [tr.url]), pick_files=pick, on_file=order.append)
        base = str(dst / "Pack")
        assert sorted(offered) == sorted(os.path.join(base, n) for n in ("a.mkv", "b.mkv", "c.txt", "d.mkv"))
        # layout order is the picker's priority, not a guarantee: the native wire keeps
        # hundreds of block requests in flight, so on a loaded box files can finish in
        # any order; every watched file fires exactly once, the unwatched one never
        want = [os.path.join(base, n) for n in ("a.mkv", "b.mkv", "d.mkv")]
        assert sorted(order) == sorted(want), order
        _check_tree(str(src), str(dst))
        # redelivery: everything is on disk; the resume verify fires each watched file
        again = []
        await _dl().download(str(dst), Sink(), magnet_for(info, [tr.url]), pick_files=pick, on_file=again.append)
        assert sorted(again) == sorted(order)
        await seed.stop()
        await tr.stop()
    run(main())


@pytest.mark.parametrize("device", ["cpu", pytest.param("gpu", marks=pytest.mark.gpu),
                                    pytest.param("hybrid", marks=pytest.mark.gpu)])
def test_redelivered_job_gpu_resume_refetches_only_the_corrupt_piece(tmp_path, device):
    """Production resume path on the MI355X: a redelivered magnet job whose
    files are already on disk (no completion DB) is batch re-verified by the
    HIP pipeline inside FileStorage.verify_existing (TorrentDownloader with
    verify_device=gpu|hybrid); one piece was corrupted on disk, and exactly
    that piece — nothing else — is fetched from the swarm again."""
    from tritondl.ops import hashing

    async def main():
        src = tmp_path / "src" / "Pack"
        make_payload(str(src), {"e1.mkv": 3_000_000, "e2.mkv": 2_500_000})
        piece = 65536
        info = torrent_for(str(src), piece)
        seed = await Seeder(info, str(tmp_path / "src")).start()
        dst = tmp_path / "job"
        shutil.copytree(src, dst / "Pack")               # the first delivery's data, no .torrent.db
        bad = (3_000_000 + 700_000) // piece
        with open(dst / "Pack" / "e2.mkv", "r+b") as f:
            f.seek(700_000)
            f.write(b"\xde\xad\xbe\xef")
        calls = []
        real = hashing.verify_pieces

        def spy(files, piece_len, expected, kind="sha1", device="cpu", threads=0):
            calls.append(device)
            return real(files, piece_len, expected, kind, device=device, threads=threads)
        hashing.verify_pieces = spy
        try:
            cfg = TorrentConfig(listen_host="127.0.0.1", verify_device=device, request_timeout=3)
            d = TorrentDownloader(cfg, progress_interval=0.05, use_dht=False)
            t, _dht = await d.open(str(dst), magnet_for(info) + f"&x.pe=127.0.0.1:{seed.torrent.port}")
            await asyncio.wait_for(t.got_info.wait(), 20)
            await t.download_all()
            assert calls == [device]
            assert t.nhave == info.num_pieces - 1 and not t.have[bad]
            await asyncio.wait_for(t.complete.wait(), 30)
            assert t.downloaded == info.piece_size(bad)      # one piece, fetched once
            await t.close()
        finally:
            hashing.verify_pieces = real
        _check_tree(str(src), str(dst))
        await seed.stop()
    run(main())


def test_torrent_disk_space_preflight(tmp_path, monkeypatch):
    """Once the info dict is known the torrent checks it fits (minus what is
    already on disk) before opening storage."""
    from tritondl.utils import disk

    async def main():
        src = tmp_path / "src"
        make_payload(str(src), {"big.mkv": 600_000})
        info = torrent_for(str(src / "big.mkv"), 32768)
        s = await Seeder(info, str(src)).start()
        dst = tmp_path / "job"
        os.makedirs(dst)
        monkeypatch.setattr(disk, "free_bytes", lambda p: 500_000)
        with pytest.raises(disk.DiskSpaceError, match="not enough disk space"):
            await _dl().download(str(dst), Sink(), magnet_for(info, peers=[s.addr]))
        assert not (dst / "big.mkv").exists()
        # most of it already on disk (a redelivered job): only the rest must fit
        (dst / "big.mkv").write_bytes((src / "big.mkv").read_bytes()[:300_000])
        await _dl().download(str(dst), Sink(), magnet_for(info, peers=[s.addr]))
        assert (dst / "big.mkv").read_bytes() == (src / "big.mkv").read_bytes()
        await s.stop()
    run(main())


def test_ipv6_peer_dials_dual_stack_listener(tmp_path):
    """The listen port is also bound on IPv6 (peers from the IPv6 DHT / PEX
    are announced with it); an IPv6 x.pe peer ([::1]:port, BEP 9) serves the
    whole download."""
    async def main():
        src = tmp_path / "src"
        make_payload(str(src), {"v6.mkv": 300_000})
        info = torrent_for(str(src / "v6.mkv"), 16384)
        s = await Seeder(info, str(src), listen_host6="::1").start()
        uri = magnet_for(info, peers=[("::1", s.torrent.port)])
        assert f"x.pe=[::1]:{s.torrent.port}" in uri
        assert parse_magnet(uri).peers == [("::1", s.torrent.port)]
        dst = tmp_path / "job"
        os.makedirs(dst)
        await _dl().download(str(dst), Sink(), uri)
        assert (dst / "v6.mkv").read_bytes() == (src / "v6.mkv").read_bytes()
        await s.stop()
    run(main())


def test_interest_counters_track_the_bitmaps(tmp_path):
    """p.wants (O(1) 'does p have a piece we lack') stays equal to the bitmap
    computation through HAVE/BITFIELD, our own completions and a resume jump."""
    import random
    from tritondl.fetch.bt import peer as pw
    from tritondl.fetch.bt.torrent import Torrent, _Peer

    class StubWire:
        closed = False

        def __getattr__(self, _name):
            return lambda *a, **k: None

    src = tmp_path / "src"
    make_payload(str(src), {"a.bin": 40 * 16384})
    info = torrent_for(str(src / "a.bin"), 16384)
    t = Torrent(info.infohash, str(tmp_path / "dst"), TorrentConfig(native_wire=False), info=info)
    t._downloading = True
    rng = random.Random(9)
    n = info.num_pieces
    peers = []
    for k in range(4):
        p = _Peer(StubWire(), ("10.0.0.%d" % k, 1), pw.Handshake(bytes(8), info.infohash, bytes(20)), n)
        t.peers[p.key] = p
        peers.append(p)

    def truth(p):
        return (int.from_bytes(p.have, "little") & ~int.from_bytes(t.have, "little")).bit_count()
    for step in range(300):
        r = rng.random()
        if r < 0.6:
            t._peer_has(rng.choice(peers), [rng.randrange(n) for _ in range(rng.randint(1, 5))])
        elif r < 0.95:
            i = rng.randrange(n)
            if not t.have[i]:
                t._record_piece(i)
        else:                                             # resume-style jump of our bitmap
            for i in rng.sample(range(n), 5):
                if not t.have[i]:
                    t.have[i] = 1
                    t.nhave += 1
            t._recount_wants()
        for p in peers:
            assert p.wants == truth(p), step


def test_storage_write_error_fails_the_job_instead_of_hanging(tmp_path, monkeypatch):
    """A piece that cannot be written (disk full) ends the download with
    TorrentError; the reference would block in WaitAll forever."""
    import errno

    from tritondl.fetch.bt.storage import FileStorage

    async def main():
        src = tmp_path / "src"
        make_payload(str(src), {"a.mkv": 1_000_000})
        info = torrent_for(str(src / "a.mkv"), 65536)
        seed = await Seeder(info, str(src)).start()
        real = FileStorage.write
        calls = {"n": 0}

        def flaky(self, piece, offset, data):
            calls["n"] += 1
            if calls["n"] > 3:
                raise OSError(errno.ENOSPC, "No space left on device")
            return real(self, piece, offset, data)
        monkeypatch.setattr(FileStorage, "write", flaky)
        dst = tmp_path / "job"
        os.makedirs(dst)
        with pytest.raises(TorrentError, match="storage failed"):
            await asyncio.wait_for(_dl().download(str(dst), lambda u, p: None, magnet_for(info, peers=[seed.addr])), 30)
        await seed.stop()
    run(main())


def test_completion_db_batches_marks_and_flushes_on_read_and_close(tmp_path):
    """Piece marks are committed in batches (one WAL transaction per batch,
    not per piece) but every read and close sees them all."""
    from tritondl.fetch.bt.storage import CompletionDB
    import sqlite3
    p = str(tmp_path / ".torrent.db")
    db = CompletionDB(p, batch=8, max_delay_s=3600)
    ih = b"\x11" * 20
    for i in range(5):
        db.set(ih, i, True)
    other = sqlite3.connect(p)
    assert other.execute("SELECT COUNT(*) FROM piece_completion").fetchone()[0] == 0   # still pending
    for i in range(5, 9):
        db.set(ih, i, True)                      # the 8th mark commits the batch
    assert other.execute("SELECT COUNT(*) FROM piece_completion").fetchone()[0] == 8
    db.set(ih, 3, False)
    db.set(ih, 20, True)
    assert db.get(ih) == set(range(9)) - {3} | {20}                  # a read flushes first
    db.set(ih, 21, True)
    db.close()                                                        # close flushes
    assert {r[0] for r in other.execute("SELECT idx FROM piece_completion WHERE complete=1")} == \
        set(range(9)) - {3} | {20, 21}
    other.close()


# ----------------------------------------------------------------- bad-piece blame
def test_bad_piece_blame_rules():
    """anacrolix's pieceHashed(correct=false): every contributor is charged;
    a sole contributor is banned on its first failure; with several, the
    unique least-trusted (net good - bad pieces) is banned.  A tie bans
    nobody: the piece is re-fetched from one contributor only, and once it
    verifies, a peer whose earlier block differs from the verified data is
    banned (smart ban)."""
    from tritondl.fetch.bt.torrent import BLOCK, Torrent

    async def main():
        t = Torrent(b"\x01" * 20, "/nonexistent", TorrentConfig(listen_host="127.0.0.1"))
        H, C = ("10.0.0.1", 1), ("10.0.0.2", 2)
        good = os.urandom(4 * BLOCK)
        bad = bytearray(good)
        bad[2 * BLOCK + 5] ^= 0xFF                        # C's block 2 is corrupt
        t._bad_piece(0, [H, H, C, H], bad)                # shared, both untried: a tie
        assert not t.banned and t.trust[H] == [0, 1] and t.trust[C] == [0, 1]
        assert t._isolate[0] == H                         # re-fetched from the one that sent most of it
        t._good_piece(0, [H, H, H, H], good)              # it verifies: C's block 2 differed
        assert t.banned == {C} and 0 not in t._isolate and 0 not in t._failed_blocks
        assert t.trust[H] == [1, 1]
        t2 = Torrent(b"\x02" * 20, "/nonexistent", TorrentConfig(listen_host="127.0.0.1"))
        t2._bad_piece(0, [C, C], bad)                     # a sole contributor: banned at once
        assert t2.banned == {C}
        t2._bad_piece(1, [None, None], bad)               # a web seed's piece: nobody to blame
        assert t2.banned == {C}
        t3 = Torrent(b"\x03" * 20, "/nonexistent", TorrentConfig(listen_host="127.0.0.1"))
        t3._good_piece(5, [H], good)
        t3._bad_piece(1, [C, H, C, H], bad)               # H has a good piece: C is least trusted
        assert t3.banned == {C}
    run(main())


def test_native_store_records_which_link_supplied_each_block():
    from tritondl import _btwire as W
    B = W.BLOCK
    store = W.PieceStore(1, 3 * B, 3 * B)
    a, b = W.Link(store, 8, False, 7), W.Link(store, 8, False, 9)
    assert (a.id, b.id) == (7, 9)
    for link in (a, b):
        link.assign(0)
        link.peer_choking = False
        link.pump()
    import struct

    def piece_msg(i, off, data):
        return struct.pack(">IBII", 9 + len(data), 7, i, off) + data
    a.feed(piece_msg(0, 0, b"x" * B))
    assert list(store.block_sources(0)) == [7, 0, 0]
    b.feed(piece_msg(0, B, b"y" * B))
    ev, _ = a.feed(piece_msg(0, 2 * B, b"z" * B))
    assert list(ev) == [("piece", 0)]
    assert list(store.block_sources(0)) == [7, 9, 7]
    store.take(0)
    assert list(store.block_sources(0)) == []


@pytest.mark.parametrize("native", [True, False], ids=["native-wire", "python-wire"])
def test_corrupter_sharing_pieces_with_an_honest_peer_is_banned_never_the_honest_one(tmp_path, native):
    """One honest and one corrupting seeder (every block it serves is
    flipped); blocks of the same piece come from both (the Python picker
    fills open pieces from every peer; native links share pieces in end
    game).  Over several swarms the corrupter is always banned, the honest
    peer never is, and the download completes from the honest peer's data."""
    from tritondl.fetch.bt.torrent import Torrent

    async def one(k: int, piece_len: int, pieces: int) -> tuple[int, int]:
        src = tmp_path / f"src{k}"
        make_payload(str(src), {"a.mkv": pieces * piece_len}, seed=k)
        info = torrent_for(str(src / "a.mkv"), piece_len)
        bad = await Seeder(info, str(src), corrupt=True).start()
        good = await Seeder(info, str(src)).start()
        cfg = TorrentConfig(listen_host="127.0.0.1", verify_device="cpu", request_timeout=3, utp=False,
                            pipeline=4, native_wire=native)
        t = Torrent(info.infohash, str(tmp_path / f"dst{k}"), cfg, info=info, peers=[bad.addr, good.addr])
        await t.start()
        await t.download_all()
        await asyncio.wait_for(t.complete.wait(), 60)
        assert (tmp_path / f"dst{k}" / "a.mkv").read_bytes() == (src / "a.mkv").read_bytes()
        for _ in range(100):
            if bad.addr in t.banned:
                break
            await asyncio.sleep(0.02)
        assert good.addr not in t.banned, t.trust
        banned = bad.addr in t.banned or bad.addr not in t.trust   # (never delivered: nothing to judge)
        shared = t.trust.get(good.addr, [0, 0])[1]             # failed pieces the honest peer shared in
        await t.close()
        await bad.stop()
        await good.stop()
        return int(banned), shared

    async def main():
        # 16-block pieces: the Python picker spreads each piece over both peers; a few
        # 2-piece swarms put the native links into end game on shared pieces
        res = [await one(k, 16 * 16384, 6) for k in range(3)]
        res += [await one(10 + k, 8 * 16384, 2) for k in range(3)]
        assert all(b for b, _s in res), res
        return res
    res = run(main(), timeout=240)
    print("(banned, shared failures) per swarm:", res)
    assert any(s for _b, s in res), res                        # pieces really were shared


@pytest.mark.parametrize("lie", ["data", "size"])
def test_metadata_from_a_lying_peer_does_not_stall_the_job(tmp_path, lie):
    """BEP 9 metadata comes from untrusted peers.  One that serves metadata
    not matching the info-hash (flipped bytes, or another announced size) is
    found out: a sole contributor is never asked again, several are asked one
    at a time, and the size is re-chosen from the other peers.  The job gets
    its metadata from the honest peer instead of failing every assembly until
    the metadata timeout."""
    async def main():
        src = tmp_path / "src"
        make_payload(str(src), {"big.mkv": 14 << 20})
        info = torrent_for(str(src / "big.mkv"), 16384)            # > 16 KiB of metadata: 2 pieces
        assert len(info.raw) > 16384
        liar = await Seeder(info, str(src), lie_metadata=lie).start()
        honest = await Seeder(info, str(src)).start()
        dst = tmp_path / "job"
        os.makedirs(dst)
        t0 = time.monotonic()
        await _dl().download(str(dst), Sink(), magnet_for(info, peers=[liar.addr, honest.addr]))
        assert (dst / "big.mkv").read_bytes() == (src / "big.mkv").read_bytes()
        assert time.monotonic() - t0 < 30
        await liar.stop()
        await honest.stop()
    run(main())
