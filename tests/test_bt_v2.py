"""BitTorrent v2 / hybrid (BEP 52): merkle trees, metainfo, btmh magnets,
native (host) and HIP (GPU) per-piece merkle verification, hash-request
proofs, and end-to-end swarm downloads of pure-v2 (.torrent and magnet —
piece layers fetched over the wire) and hybrid torrents."""

import asyncio
import hashlib
import os

import pytest

from tritondl_testkit.fakes.origin import Origin
from tritondl_testkit.fakes.swarm import Seeder, make_payload, torrent_file_bytes
from tritondl.fetch.bt import merkle
from tritondl.fetch.bt.client import TorrentDownloader
from tritondl.fetch.bt.metainfo import Metainfo, MetainfoError, make_info, parse_magnet
from tritondl.fetch.bt.torrent import TorrentConfig
from tritondl.ops import hashing

H = lambda b: hashlib.sha256(b).digest()  # noqa: E731


def run(coro, timeout=90):
    return asyncio.run(asyncio.wait_for(coro, timeout))


# ----------------------------------------------------------------- merkle


def test_merkle_known_shapes():
    a, b, c = b"a" * 16384, b"b" * 16384, b"c" * 100
    assert merkle.file_root_and_layer(a, 16384) == (H(a), [])
    assert merkle.file_root_and_layer(a + b, 32768)[0] == H(H(a) + H(b))
    # 3 leaves -> padded to 4 with zero leaves
    root3 = H(H(H(a) + H(b)) + H(H(c) + bytes(32)))
    assert merkle.file_root_and_layer(a + b + c, 65536)[0] == root3
    # piece layer at 16 KiB x 2 leaves per piece, 2 pieces (last padded)
    root, layer = merkle.file_root_and_layer(a + b + c, 32768)
    assert layer == [H(H(a) + H(b)), H(H(c) + bytes(32))] and root == root3
    assert merkle.layer_root(layer, 32768) == root


@pytest.mark.parametrize("n_pieces,length", [(3, 2), (5, 4), (9, 2), (9, 8), (1, 1)])
def test_hash_request_proofs_roundtrip(n_pieces, length):
    layer = [H(bytes([k])) for k in range(n_pieces)]
    root = merkle.layer_root(layer, 16384 * 4)
    level = merkle.piece_levels(16384 * 4)
    width = merkle.next_pow2(n_pieces)
    length = min(length, width)
    total_h = width.bit_length() - 1
    proofs = total_h - (length.bit_length() - 1)
    for index in range(0, width, length):
        ans = merkle.serve_hashes(layer, level, index, length, proofs)
        got = merkle.check_hashes(root, level, index, length, ans, n_pieces)
        assert got is not None and got[:max(0, min(length, n_pieces - index))] == layer[index:index + length]
        bad = bytearray(ans)
        bad[0] ^= 1
        assert merkle.check_hashes(root, level, index, length, bytes(bad), n_pieces) is None


# ----------------------------------------------------------------- metainfo


def _tree(tmp_path):
    src = tmp_path / "src" / "Show"
    make_payload(str(src), {"e1.mkv": 300_000, "sub/e2.mkv": 70_001, "tiny.txt": 10, "empty.nfo": 0})
    return src


def test_v2_and_hybrid_metainfo(tmp_path):
    src = _tree(tmp_path)
    v2 = make_info(str(src), 32768, version=2)
    assert v2.has_v2 and not v2.has_v1 and len(v2.infohash_v2) == 32 and v2.infohash == v2.infohash_v2[:20]
    files = {"/".join(f.path): f for f in v2.v2_files}
    assert files["empty.nfo"].root == b"" and files["e1.mkv"].num_pieces == 10
    assert files["e1.mkv"].root in v2.piece_layers and files["tiny.txt"].root not in v2.piece_layers
    # round trip through a .torrent with piece layers
    mi = Metainfo.parse(torrent_file_bytes(v2))
    assert mi.info.infohash == v2.infohash and mi.info.piece_layers == v2.piece_layers
    # every piece checks out against the data (v2 pieces are file-aligned)
    blob = b""
    for p, n in v2.file_paths(str(tmp_path / "src")):
        blob += bytes(n) if not p else open(p, "rb").read()
    for i in range(v2.num_pieces):
        d = blob[i * 32768:(i + 1) * 32768]
        assert v2.check_piece(i, d), i
        assert not v2.check_piece(i, b"x" + d[1:])
    hy = make_info(str(src), 32768, version=3)
    assert hy.has_v1 and hy.has_v2 and hy.infohash == hashlib.sha1(hy.raw).digest()
    assert hy.num_pieces == v2.num_pieces                      # same piece-aligned index space
    with pytest.raises(MetainfoError):
        make_info(str(src), 3 * 16384, version=2)              # v2 piece length must be 2^k x 16 KiB


def test_bad_piece_layer_rejected(tmp_path):
    src = _tree(tmp_path)
    v2 = make_info(str(src), 32768, version=2)
    raw = bytearray(torrent_file_bytes(v2))
    root = next(iter(v2.piece_layers))
    k = raw.find(v2.piece_layers[root])
    raw[k] ^= 0xFF
    with pytest.raises(MetainfoError):
        Metainfo.parse(bytes(raw))


def test_btmh_magnets():
    ih2 = H(b"info")
    m = parse_magnet(f"magnet:?xt=urn:btmh:1220{ih2.hex()}&dn=x")
    assert m.infohash == ih2[:20] and m.infohash_v2 == ih2 and not m.has_v1
    assert parse_magnet(m.uri()).infohash_v2 == ih2
    ih1 = hashlib.sha1(b"info").digest()
    h = parse_magnet(f"magnet:?xt=urn:btih:{ih1.hex()}&xt=urn:btmh:1220{ih2.hex()}")
    assert h.infohash == ih1 and h.infohash_v2 == ih2 and h.has_v1
    with pytest.raises(MetainfoError):
        parse_magnet("magnet:?xt=urn:btmh:1114" + "00" * 20)


# ----------------------------------------------------------------- native verification


def _v2_layout(tmp_path, piece_len=32768):
    src = _tree(tmp_path)
    info = make_info(str(src), piece_len, version=2)
    return info, info.file_paths(str(tmp_path / "src"))


def test_native_merkle_verify_host(tmp_path):
    info, layout = _v2_layout(tmp_path)
    exp, widths, reals, known = info.v2_expectations()
    ok = hashing.verify_pieces_v2(layout, info.piece_length, exp, widths, reals, known, device="cpu")
    assert ok == b"\x01" * info.num_pieces
    # corrupt one byte of e1.mkv's 4th piece -> exactly that piece fails
    p = next(path for path, _n in layout if path.endswith("e1.mkv"))
    with open(p, "r+b") as f:
        f.seek(3 * 32768 + 5)
        f.write(b"\x00" if f.read(1) != b"\x00" else b"\x01")
    ok = hashing.verify_pieces_v2(layout, info.piece_length, exp, widths, reals, known, device="cpu")
    first = next(f.first_piece for f in info.v2_files if f.path[-1] == "e1.mkv")
    assert [i for i, v in enumerate(ok) if not v] == [first + 3]
    # unknown expectations are reported as not verified
    ok = hashing.verify_pieces_v2(layout, info.piece_length, exp, widths, reals, [False] * len(widths))
    assert ok == bytes(info.num_pieces)


@pytest.mark.gpu
def test_native_merkle_verify_gpu_matches_host(tmp_path):
    info, layout = _v2_layout(tmp_path, piece_len=65536)
    exp, widths, reals, known = info.v2_expectations()
    host = hashing.verify_pieces_v2(layout, info.piece_length, exp, widths, reals, known, device="cpu")
    gpu = hashing.verify_pieces_v2(layout, info.piece_length, exp, widths, reals, known, device="gpu")
    assert gpu == host == b"\x01" * info.num_pieces


# ----------------------------------------------------------------- swarm


def _dl(**kw):
    cfg = TorrentConfig(listen_host="127.0.0.1", verify_device="cpu", request_timeout=3, **kw)
    return TorrentDownloader(cfg, progress_interval=0.05, use_dht=False, metadata_timeout=10)


def _check(src, dst):
    for root, _d, files in os.walk(src):
        for f in files:
            a = os.path.join(root, f)
            b = os.path.join(dst, os.path.relpath(a, os.path.dirname(src)))
            assert open(a, "rb").read() == open(b, "rb").read(), b


@pytest.mark.parametrize("version", [2, 3])
def test_swarm_download_via_torrent_file(tmp_path, version):
    async def main():
        src = _tree(tmp_path)
        info = make_info(str(src), 32768, version=version)
        seed = await Seeder(info, str(tmp_path / "src")).start()
        o = await Origin().start()
        url = o.add("/t.torrent", torrent_file_bytes(info))
        dst = tmp_path / "job"
        os.makedirs(dst)
        d = _dl()
        t, _ = await d.open(str(dst), url)
        t.add_peer_addr(seed.addr)
        await t.download_all()
        await asyncio.wait_for(t.complete.wait(), 30)
        await t.close()
        _check(str(src), str(dst))
        assert not (dst / "Show" / ".pad").exists()
        await seed.stop()
        await o.stop()
    run(main())


def test_pure_v2_magnet_fetches_piece_layers_over_the_wire(tmp_path):
    async def main():
        src = _tree(tmp_path)
        info = make_info(str(src), 16384, version=2)
        assert info.missing_layers() == [] and len(info.piece_layers) >= 1
        seed = await Seeder(info, str(tmp_path / "src")).start()
        from tritondl.fetch.bt.metainfo import Magnet
        m = Magnet(info.infohash, info.name, [], [seed.addr], [], info.infohash_v2, has_v1=False).uri()
        assert "btih" not in m
        dst = tmp_path / "job"
        os.makedirs(dst)
        t, _ = await _dl().open(str(dst), m)
        await asyncio.wait_for(t.got_info.wait(), 10)
        assert t.info.missing_layers()                 # the info dict does not carry piece layers
        await t.download_all()                          # fetches them via BEP 52 hash requests
        assert not t.info.missing_layers()
        await asyncio.wait_for(t.complete.wait(), 30)
        await t.close()
        _check(str(src), str(dst))
        await seed.stop()
    run(main())


def test_v2_resume_verifies_existing_data(tmp_path):
    async def main():
        src = _tree(tmp_path)
        info = make_info(str(src), 32768, version=2)
        seed = await Seeder(info, str(tmp_path / "src")).start()
        dst = tmp_path / "job"
        # pre-seed the job dir with a partial copy: e1.mkv half right, half garbage
        os.makedirs(dst / "Show")
        good = (src / "e1.mkv").read_bytes()
        (dst / "Show" / "e1.mkv").write_bytes(good[:150_000] + os.urandom(150_000))
        o = await Origin().start()
        url = o.add("/t.torrent", torrent_file_bytes(info))
        t, _ = await _dl().open(str(dst), url)
        t.add_peer_addr(seed.addr)
        await t.download_all()
        pre = t.nhave
        assert 0 < pre < info.num_pieces
        await asyncio.wait_for(t.complete.wait(), 30)
        await t.close()
        _check(str(src), str(dst))
        await seed.stop()
        await o.stop()
    run(main())


def test_gpu_leaf_path_logic_emulated_on_host(tmp_path, monkeypatch):
    """The GPU path hashes whole 16 KiB blocks of the padded stream and then
    re-hashes each file's short last leaf on the host; emulate the kernel
    with the host piece hasher to pin that logic without a device."""
    info, layout = _v2_layout(tmp_path, piece_len=65536)
    exp, widths, reals, known = info.v2_expectations()

    class FakeGpu:
        def digest_files(self, files, pl, kind, cpu_threads=0):
            blob = b"".join(bytes(n) if not p else open(p, "rb").read() for p, n in files)
            return hashing._host.piece_hashes(kind, blob, pl, 2), b"\x01" * (-(-len(blob) // pl))
    monkeypatch.setattr(hashing, "gpu_backend", lambda *a, **k: FakeGpu())
    monkeypatch.setattr(hashing, "_resolve", lambda d: d)
    ok = hashing.verify_pieces_v2(layout, info.piece_length, exp, widths, reals, known, device="gpu")
    assert ok == b"\x01" * info.num_pieces


def test_native_merkle_root_matches_the_spec():
    """hashing.merkle_root (C++, SHA-NI pairs) == merkle.piece_root (spec)
    for lengths around leaf boundaries and padded widths."""
    import os as _os
    from tritondl.fetch.bt import merkle as mk
    from tritondl.ops import hashing
    for n in (1, 100, 16384, 16385, 3 * 16384, 3 * 16384 + 7, 64 * 16384):
        data = _os.urandom(n)
        nl = (n + 16383) // 16384
        for width in {mk.next_pow2(nl), 2 * mk.next_pow2(nl), 64}:
            if width >= nl:
                assert hashing.merkle_root(data, width) == mk.piece_root(data, width)
    with pytest.raises(ValueError):
        hashing.merkle_root(b"x" * 40000, 2)          # 3 leaves do not fit 2


# ------------------------------------------------------ over-long file names

def test_overlong_components_are_cut_distinct_and_keep_their_extension(tmp_path):
    from tritondl.fetch.bt import bencode
    from tritondl.fetch.bt.metainfo import COMPONENT_MAX, Info
    long_a = "A" * 300 + ".part1.mkv"
    long_b = "A" * 300 + ".part2.mkv"
    cjk = "影" * 100 + ".mp4"                     # 100 chars, 304 UTF-8 bytes (fits NTFS, not ext4)
    latin1 = b"\xe9" * 260 + b".avi"                  # not UTF-8: kept as raw bytes
    raw = bencode.encode({b"name": "N" * 280, b"piece length": 16384, b"pieces": b"\0" * 20,
                          b"files": [{b"length": 1, b"path": [p.encode() if isinstance(p, str) else p]}
                                     for p in (long_a, long_b, cjk, latin1, "short.mkv")]})
    info = Info.parse(raw)
    names = [f.path[-1] for f in info.files]
    assert names[-1] == "short.mkv"
    assert len(set(names)) == 5
    for n, ext in zip(names, (".mkv", ".mkv", ".mp4", ".avi")):
        assert n.endswith(ext) and len(n.encode("utf-8", "surrogateescape")) <= COMPONENT_MAX
    assert names[2].startswith("影") and "�" not in names[2]
    assert len(info.name.encode()) <= COMPONENT_MAX
    assert Info.parse(raw).files[0].path == info.files[0].path          # deterministic
    for p, _n in info.file_paths(str(tmp_path)):
        os.makedirs(os.path.dirname(p), exist_ok=True)
        for suffix in ("", ".s3upload.tmp", ".part.meta.tmp"):
            open(p + suffix, "wb").close()


@pytest.mark.parametrize("version", [1, 3])
def test_swarm_download_of_names_too_long_for_the_work_dir(tmp_path, version):
    """250-byte names fit the seeder's disk but not next to the worker's
    sidecars: the job lands them cut, hybrid v1/v2 file lists still agree."""
    from tritondl.select import dir_media

    async def main():
        src = tmp_path / "src" / "Show"
        names = {("E" * 240 + f".{k}.mkv"): 40_000 + k for k in range(2)}
        make_payload(str(src), names)
        info = make_info(str(src), 32768, version=version)
        seed_root = tmp_path / "seed"
        by_size = {n: os.path.join(src, f) for f, n in names.items()}
        for p, n in info.file_paths(str(seed_root)):
            if p:
                os.makedirs(os.path.dirname(p), exist_ok=True)
                os.link(by_size[n], p)
        seed = await Seeder(info, str(seed_root)).start()
        o = await Origin().start()
        url = o.add("/t.torrent", torrent_file_bytes(info))
        dst = tmp_path / "job"
        os.makedirs(dst)
        t, _ = await _dl().open(str(dst), url)
        t.add_peer_addr(seed.addr)
        await t.download_all()
        await asyncio.wait_for(t.complete.wait(), 30)
        await t.close()
        got = dir_media(str(dst))
        assert len(got) == 2 and all(f.endswith(".mkv") for f in got)
        for p, n in info.file_paths(str(dst)):
            if p:
                assert open(p, "rb").read() == open(by_size[n], "rb").read()
        await seed.stop()
        await o.stop()
    run(main())
