"""Library-default parity: the values the reference inherited from its
libraries without naming them.

* anacrolix ``NewDefaultClientConfig`` (``internal/downloader/torrent/torrent.go:40``):
  ListenPort 42069, HeaderObfuscationPolicy{Preferred: true}, the
  ``dht.GlobalBootstrapAddrs`` routers, EstablishedConnsPerTorrent 50 and
  HalfOpenConnsPerTorrent 25;
* streadway ``amqp.Dial`` (``internal/rabbitmq/client.go:309``): 10 s heartbeat;
* grab (``internal/downloader/http/http.go:37-42``): ``Last-Modified`` becomes
  the local file's mtime (``IgnoreRemoteTime`` false).

Kept different on purpose, see docs/PARITY.md "Library defaults": the
User-Agent."""

import asyncio
import os
import socket

import pytest

from tritondl_testkit.fakes.origin import Origin
from tritondl.fetch.bt.client import TorrentDownloader
from tritondl.fetch.bt.torrent import Torrent, TorrentConfig
from tritondl.fetch.http import HTTPDownloader
from tritondl.parallel.topology import plan
from tritondl.utils.config import Config


def run(coro, timeout=30):
    return asyncio.run(asyncio.wait_for(coro, timeout))


def test_anacrolix_and_streadway_defaults():
    c = Config()
    assert c.heartbeat_s == 10
    assert c.bt_listen_port == 42069
    assert c.bt_encryption == "prefer"
    assert c.bt_bootstrap.split(",") == ["router.utorrent.com:6881", "router.bittorrent.com:6881",
                                         "dht.transmissionbt.com:6881", "dht.aelitis.com:6881",
                                         "router.silotis.us:6881", "dht.libtorrent.org:25401"]
    assert (c.bt_established_conns, c.bt_half_open_conns) == (50, 25)
    td = TorrentDownloader.from_config(c)
    assert (td.cfg.listen_port, td.cfg.encryption) == (42069, "prefer")
    assert (td.cfg.established_conns, td.cfg.half_open_conns) == (50, 25)
    assert len(td.dht_bootstrap) == 6 and td.dht_bootstrap[-1] == ("dht.libtorrent.org", 25401)
    e = Config.from_env({"TRITONDL_BT_ESTABLISHED_CONNS": "80", "TRITONDL_BT_HALF_OPEN_CONNS": "9",
                         "TRITONDL_HEARTBEAT": "30"})
    assert (e.bt_established_conns, e.bt_half_open_conns, e.heartbeat_s) == (80, 9, 30)
    # the node launcher leaves the port to the worker default unless given a base port
    assert "TRITONDL_BT_LISTEN_PORT" not in plan(2, gpus=0, cpus=4)[0].env()
    assert plan(2, gpus=0, cpus=4, base_port=7000)[1].env()["TRITONDL_BT_LISTEN_PORT"] == "7001"


def test_listen_port_busy_falls_back_to_ephemeral(tmp_path):
    async def main():
        hold = socket.socket()
        hold.bind(("127.0.0.1", 0))
        hold.listen()
        busy = hold.getsockname()[1]
        t = Torrent(b"\x01" * 20, str(tmp_path), TorrentConfig(listen_host="127.0.0.1", listen_port=busy))
        await t.start()
        assert t.port not in (0, busy)
        await t.close()
        strict = Torrent(b"\x02" * 20, str(tmp_path),
                         TorrentConfig(listen_host="127.0.0.1", listen_port=busy, listen_port_fallback=False))
        with pytest.raises(OSError):
            await strict.start()
        hold.close()
        free = Torrent(b"\x03" * 20, str(tmp_path), TorrentConfig(listen_host="127.0.0.1", listen_port=busy))
        await free.start()
        assert free.port == busy                       # the configured port when it is free
        await free.close()
    run(main())


def test_connection_caps():
    async def main():
        t = Torrent(b"\x04" * 20, "/tmp", TorrentConfig(established_conns=5, half_open_conns=2))
        t._connect = _never                             # count dials without touching the network
        assert t._dial_slots() == 2                     # half-open cap
        t.connecting.update({("10.0.0.1", 1), ("10.0.0.2", 1)})
        assert t._dial_slots() == 0
        t.connecting.clear()
        t.peers.update({(f"10.0.1.{i}", 1): object() for i in range(4)})
        assert t._dial_slots() == 1                     # established + half-open <= 5
        t.add_peer_addrs([("10.0.2.1", 1), ("10.0.2.2", 1), ("10.0.2.3", 1)])
        assert len(t.connecting) == 1 and len(t.known) == 3
        for task in list(t._tasks):
            task.cancel()
    run(main())


async def _never(_addr):
    await asyncio.sleep(3600)


def test_last_modified_becomes_mtime(tmp_path):
    async def main():
        o = await Origin().start()
        url = o.add("/f.mkv", b"y" * 5000)
        h = HTTPDownloader(progress_interval=0.05)
        await h.download(str(tmp_path), lambda u, v: None, url)
        st = os.stat(tmp_path / "f.mkv")
        assert st.st_mtime == 1704067200 and st.st_atime == 1704067200   # Mon, 01 Jan 2024 00:00:00 GMT
        await h.close()
        await o.stop()
    run(main())


def test_s3_hash_device_knob():
    import pytest as _p
    assert Config().s3_hash_device == "cpu"
    assert Config.from_env({"TRITONDL_S3_HASH_DEVICE": "gpu"}).s3_hash_device == "gpu"
    with _p.raises(ValueError):
        Config.from_env({"TRITONDL_S3_HASH_DEVICE": "tpu"})


def test_known_peers_are_bounded_at_the_high_water_mark():
    """anacrolix TorrentPeersHighWater (500): a flood of PEX / tracker
    addresses keeps the known set bounded; connected ones are never the ones
    replaced."""
    from tritondl.fetch.bt.torrent import Torrent, TorrentConfig
    t = Torrent(b"\x05" * 20, "/tmp", TorrentConfig(established_conns=0, half_open_conns=0))
    assert t.cfg.peers_high_water == 500
    t.peers[("10.0.0.1", 1)] = object()
    t.known.add(("10.0.0.1", 1))
    t.add_peer_addrs([(f"10.{k >> 16 & 255}.{k >> 8 & 255}.{k & 255}", 6881) for k in range(5000)])
    for k in range(2000):
        t.add_peer_addr((f"11.0.{k >> 8}.{k & 255}", 51413))
    assert len(t.known) == 500 and ("10.0.0.1", 1) in t.known
    t.peers.clear()
