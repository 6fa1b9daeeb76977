"""MSE/PE (BitTorrent protocol encryption): native RC4 vectors, the DH/RC4
handshake in both crypto modes, and policy interplay in real downloads."""

import asyncio
import os

import pytest

from tritondl_testkit.fakes.swarm import Seeder, magnet_for, make_payload, torrent_for
from tritondl.fetch.bt import mse
from tritondl.fetch.bt.client import TorrentDownloader
from tritondl.fetch.bt.torrent import TorrentConfig
from tritondl.ops.hashing import _host


def test_rc4_known_vectors():
    # RFC 6229 (key 0102030405, offset 0) and the classic "Key"/"Plaintext"
    assert _host.Rc4(bytes([1, 2, 3, 4, 5]), 0).crypt(bytes(16)).hex() == "b2396305f03dc027ccc3524a0a1118a8"
    assert _host.Rc4(b"Key", 0).crypt(b"Plaintext").hex() == "bbf316e8d940af0ad3"
    # RFC 6229 offset 1024 for the same key == drop=1024
    assert _host.Rc4(bytes([1, 2, 3, 4, 5]), 1024).crypt(bytes(16)).hex() == "30abbcc7c20b01609f23ee2d5f6bb7df"
    r1, r2 = _host.Rc4(b"k" * 20), _host.Rc4(b"k" * 20)
    data = os.urandom(100_000)
    assert r2.crypt(r1.crypt(data)) == data


async def _pair(provide, allow_plain=True):
    skey = os.urandom(20)
    got = {}
    done = asyncio.Event()

    async def on_conn(r, w):
        try:
            first = await r.readexactly(20)
            rr, ww, sel = await mse.respond(r, w, first, skey, allow_plain=allow_plain, timeout=2.0)
            got["ia"] = await rr.readexactly(5)
            got["sel"] = sel
            ww.write(b"pong" * 1000)
            got["more"] = await rr.readexactly(6)
            await ww.drain()
        except Exception as e:  # noqa: BLE001
            got["err"] = e
        finally:
            done.set()
    srv = await asyncio.start_server(on_conn, "127.0.0.1", 0)
    port = srv.sockets[0].getsockname()[1]
    r, w = await asyncio.open_connection("127.0.0.1", port)
    try:
        rr, ww, sel = await mse.initiate(r, w, skey, b"hello", provide, timeout=2.0)
        ww.write(b"world!")
        assert await rr.readexactly(4000) == b"pong" * 1000
        await asyncio.wait_for(done.wait(), 5)
        assert got == {"ia": b"hello", "sel": sel, "more": b"world!"}
        return sel
    finally:
        w.close()
        srv.close()


def test_handshake_rc4_and_plain_selection():
    assert asyncio.run(_pair(mse.CRYPTO_RC4 | mse.CRYPTO_PLAIN)) == mse.CRYPTO_RC4
    assert asyncio.run(_pair(mse.CRYPTO_PLAIN)) == mse.CRYPTO_PLAIN
    with pytest.raises(Exception):
        asyncio.run(_pair(mse.CRYPTO_PLAIN, allow_plain=False))


@pytest.mark.parametrize("leech,seed,ok", [("require", "allow", True), ("prefer", "disable", True),
                                            ("allow", "require", False), ("require", "require", True),
                                            ("prefer", "allow", True)])
def test_download_under_encryption_policies(tmp_path, leech, seed, ok):
    async def main():
        src = tmp_path / "src"
        make_payload(str(src), {"e.mkv": 300_000})
        info = torrent_for(str(src / "e.mkv"), 32768)
        s = await Seeder(info, str(src), encryption=seed).start()
        dst = tmp_path / "job"
        os.makedirs(dst)
        d = TorrentDownloader(TorrentConfig(listen_host="127.0.0.1", verify_device="cpu", encryption=leech,
                                            connect_timeout=2), progress_interval=0.05, use_dht=False,
                              metadata_timeout=3)
        try:
            await d.download(str(dst), lambda u, p: None, magnet_for(info, peers=[s.addr]))
            assert (dst / "e.mkv").read_bytes() == (src / "e.mkv").read_bytes()
            return True
        except Exception:  # noqa: BLE001
            return False
        finally:
            await s.stop()
    assert asyncio.run(asyncio.wait_for(main(), 60)) is ok
