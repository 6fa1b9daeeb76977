"""Go's default TCP keep-alive on every socket the worker dials (VERDICT r05
Missing #2).

Every reference connection came from a zero-value ``net.Dialer``: grab's
transport (``internal/downloader/http/http.go:18-22``), minio-go's
(``internal/uploader/uploader.go:43-51``, ``KeepAlive: 30s`` in its
transport) and ``amqp.Dial`` (``internal/rabbitmq/client.go:308-309``).
Go enables keep-alive there with 15 s idle and 15 s between probes.  These
tests read the options back (``getsockopt``) from the sockets a real job
dials: its HTTP GET, its S3 PUT and S3 control requests, the AMQP
connection, and a BitTorrent peer."""

import os
import socket

from tritondl.models import Media
from tritondl.utils import dial
from tritondl_testkit.fakes.swarm import Seeder, magnet_for, make_payload, torrent_for

from .test_bt import Sink, _dl
from .test_permissions import Env, run

WANT = {"keepalive": 1, "idle": 15, "interval": 15, "count": 9, "nodelay": 1}


def _opts(s: socket.socket) -> dict:
    return {"keepalive": s.getsockopt(socket.SOL_SOCKET, socket.SO_KEEPALIVE),
            "idle": s.getsockopt(socket.IPPROTO_TCP, socket.TCP_KEEPIDLE),
            "interval": s.getsockopt(socket.IPPROTO_TCP, socket.TCP_KEEPINTVL),
            "count": s.getsockopt(socket.IPPROTO_TCP, socket.TCP_KEEPCNT),
            "nodelay": 1 if s.getsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY) else 0}


def _record_dials(monkeypatch) -> dict:
    """Peer port -> options of each socket :func:`dial.connect_any` returned."""
    seen: dict[int, list[dict]] = {}
    orig = dial.connect_any

    async def rec(infos, timeout, delay=dial.FALLBACK_DELAY):
        s = await orig(infos, timeout, delay)
        seen.setdefault(s.getpeername()[1], []).append(_opts(s))
        return s
    monkeypatch.setattr(dial, "connect_any", rec)
    return seen


def test_keepalive_helper_sets_go_s_defaults():
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    try:
        dial.tcp_options(s)
        assert _opts(s) == WANT
    finally:
        s.close()
    s = dial.socket_factory((socket.AF_INET, socket.SOCK_STREAM, socket.IPPROTO_TCP, "", ("127.0.0.1", 1)))
    try:
        assert _opts(s) == WANT
    finally:
        s.close()


def test_a_job_s_get_put_amqp_and_s3_control_sockets_keep_alive(tmp_path, monkeypatch):
    import tritondl.s3.client as s3client
    seen = _record_dials(monkeypatch)
    made: list[socket.socket] = []
    orig_factory = s3client.socket_factory

    def factory(info):
        s = orig_factory(info)
        made.append(s)
        return s
    monkeypatch.setattr(s3client, "socket_factory", factory)

    async def main():
        e = await Env().up(tmp_path)
        url = e.origin.add("/ka.mkv", os.urandom(3 << 20))
        e.submit(Media(id="ka", source_uri=url))
        res = await e.wait_results(1)
        assert res[0].ok, res
        assert seen.get(e.broker.port) == [WANT]                     # the AMQP connection
        assert seen.get(e.origin.port) and all(o == WANT for o in seen[e.origin.port])   # GET streams
        assert seen.get(e.s3.port) and all(o == WANT for o in seen[e.s3.port])           # native PUT
        assert made and all(_opts(s) == WANT for s in made if s.fileno() >= 0)           # aiohttp control
        await e.down()
    run(main())


def test_bt_peer_sockets_keep_alive(tmp_path, monkeypatch):
    seen = _record_dials(monkeypatch)

    async def main():
        src = tmp_path / "src"
        make_payload(str(src), {"movie.mkv": 300_000})
        info = torrent_for(str(src / "movie.mkv"), 32768)
        seed = await Seeder(info, str(src)).start()
        dst = tmp_path / "job"
        os.makedirs(dst)
        await _dl().download(str(dst), Sink(), magnet_for(info, [], peers=[("127.0.0.1", seed.torrent.port)]))
        assert (dst / "movie.mkv").read_bytes() == (src / "movie.mkv").read_bytes()
        assert seen.get(seed.torrent.port) and all(o == WANT for o in seen[seed.torrent.port])
        await seed.stop()
    run(main())
