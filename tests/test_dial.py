"""RFC 6555 / 8305 fast fallback on every outbound dial (VERDICT r04 Missing #1).

Go's ``net.Dialer`` (behind grab ``http.go:18-22``, minio-go
``uploader.go:43-51`` and ``amqp.Dial`` ``client.go:308-309``) starts the
next address family 300 ms after the first.  Here a name resolves to a
black-holed address first (a listener whose accept queue is full: the
kernel drops the SYNs, so a connect hangs exactly like a filtered AAAA
route) and to the live 127.0.0.1 second; every dial must get through in
well under a second instead of waiting out its connect timeout."""

import asyncio
import os
import socket
import time

import pytest

from tritondl.amqp.connection import Connection
from tritondl.models import Media
from tritondl.s3.client import S3Client
from tritondl.s3.credentials import Static
from tritondl.utils import dial
from tritondl.utils import rawhttp

NAME = "dualstackhost"   # no dot: the fake S3 would read "dualstack.test" as a virtual-hosted bucket


class BlackHoles:
    """Listeners on 127.0.0.2:<port> with a full accept queue."""

    def __init__(self) -> None:
        self.socks: list[socket.socket] = []

    def add(self, port: int) -> None:
        ls = socket.socket()
        ls.bind(("127.0.0.2", port))
        ls.listen(0)
        self.socks.append(ls)
        for _ in range(4):                      # fill the backlog: later SYNs are dropped
            c = socket.socket()
            c.setblocking(False)
            try:
                c.connect(("127.0.0.2", port))
            except BlockingIOError:
                pass
            self.socks.append(c)
        time.sleep(0.05)

    def close(self) -> None:
        for s in self.socks:
            s.close()


@pytest.fixture
def dualstack(monkeypatch):
    real = socket.getaddrinfo

    def fake(host, port, *a, **kw):
        if host == NAME:
            p = int(port)
            return [(socket.AF_INET, socket.SOCK_STREAM, 6, "", ("127.0.0.2", p)),
                    (socket.AF_INET, socket.SOCK_STREAM, 6, "", ("127.0.0.1", p))]
        return real(host, port, *a, **kw)
    monkeypatch.setattr(socket, "getaddrinfo", fake)
    holes = BlackHoles()
    yield holes
    holes.close()


def test_black_hole_really_hangs(dualstack):
    """The fixture's first address is a black hole, not a refusal."""
    ls = socket.socket()
    ls.bind(("127.0.0.1", 0))
    ls.listen(8)
    port = ls.getsockname()[1]
    dualstack.add(port)
    c = socket.socket()
    c.settimeout(0.5)
    with pytest.raises(OSError):
        c.connect(("127.0.0.2", port))
    c.close()
    ls.close()


def test_interleave_alternates_families():
    A, B = socket.AF_INET6, socket.AF_INET
    infos = [(A, 1, 6, "", ("::1", 1)), (A, 1, 6, "", ("::2", 1)), (A, 1, 6, "", ("::3", 1)),
             (B, 1, 6, "", ("1.1.1.1", 1))]
    out = dial.interleave(infos)
    assert [i[4][0] for i in out] == ["::1", "1.1.1.1", "::2", "::3"]
    assert dial.interleave([]) == []


def test_connect_any_falls_back_after_the_stagger(dualstack):
    async def main():
        srv = await asyncio.start_server(lambda r, w: w.close(), "127.0.0.1", 0)
        port = srv.sockets[0].getsockname()[1]
        dualstack.add(port)
        t0 = time.monotonic()
        s = await dial.dial(NAME, port, timeout=30)
        dt = time.monotonic() - t0
        assert s.getpeername() == ("127.0.0.1", port)
        assert 0.25 <= dt < 0.9, dt                  # one 300 ms stagger, not the 30 s timeout
        s.close()
        # a refused first address moves on at once (no stagger)
        ls = socket.socket()
        ls.bind(("127.0.0.1", 0))
        dead = ls.getsockname()[1]
        ls.close()
        infos = [(socket.AF_INET, socket.SOCK_STREAM, 6, "", ("127.0.0.1", dead)),
                 (socket.AF_INET, socket.SOCK_STREAM, 6, "", ("127.0.0.1", port))]
        t0 = time.monotonic()
        s = await dial.connect_any(infos, 30)
        assert time.monotonic() - t0 < 0.2
        s.close()
        # every address black-holed: the overall timeout, not one per address
        infos = [(socket.AF_INET, socket.SOCK_STREAM, 6, "", ("127.0.0.2", port))] * 3
        t0 = time.monotonic()
        with pytest.raises(OSError):
            await dial.connect_any(infos, 0.8)
        assert time.monotonic() - t0 < 1.5
        srv.close()
        await srv.wait_closed()
    asyncio.run(asyncio.wait_for(main(), 30))


def test_http_job_s3_put_and_amqp_connect_each_fall_back_in_under_a_second(dualstack, tmp_path):
    """An HTTP job (native GET pump + streamed S3 PUT), a direct S3 PUT and an
    AMQP connect, all to names whose first address is black-holed."""
    from tritondl_testkit.fakes.broker import Broker
    from tritondl_testkit.fakes.origin import Origin
    from tritondl_testkit.fakes.s3 import FakeS3
    from tritondl.amqp.client import Client
    from tritondl.fetch.http import HTTPDownloader
    from tritondl.fetch.registry import Dispatcher
    from tritondl.s3.uploader import Uploader, object_key
    from tritondl.service import Service
    from tritondl.utils.config import Config
    from tritondl.amqp.codec import Properties
    from tritondl.models import Download

    async def main():
        broker = await Broker().start()
        origin = await Origin().start()
        s3 = await FakeS3(access_key="ak", secret_key="sk").start()
        for port in (broker.port, origin.port, s3.port):
            dualstack.add(port)
        assert rawhttp.relay_module() is not None       # the native data plane does the dialling

        t0 = time.monotonic()
        conn = await Connection.open(f"amqp://guest:guest@{NAME}:{broker.port}/", heartbeat=0)
        t_amqp = time.monotonic() - t0
        await conn.close()

        cli = S3Client(f"http://{NAME}:{s3.port}", Static("ak", "sk"))
        t0 = time.monotonic()
        await cli.make_bucket("b")
        await cli.put_object("b", "k", b"z" * 100_000)
        t_s3 = time.monotonic() - t0
        assert s3.object_bytes("b", "k") == b"z" * 100_000
        await cli.close()

        cfg = Config()
        cfg.download_dir = str(tmp_path / "downloading")
        cfg.retry_delay_s = 0
        cfg.progress_log_interval_s = 0
        cfg.heartbeat_s = 0
        amqp = Client(f"amqp://guest:guest@{NAME}:{broker.port}/", heartbeat=0)
        svc = Service(cfg, amqp=amqp,
                      dispatcher=Dispatcher(cfg.download_dir, [HTTPDownloader(progress_interval=0.05)], 0),
                      uploader=Uploader(cfg.bucket, S3Client(f"http://{NAME}:{s3.port}", Static("ak", "sk"))))
        await svc.start()
        data = os.urandom(300_000)
        origin.add("/d.mkv", data)
        t0 = time.monotonic()
        broker.inject("v1.download", "v1.download-0",
                      Download(created_at="t", media=Media(id="d1", source_uri=f"http://{NAME}:{origin.port}/d.mkv"))
                      .encode(), Properties(delivery_mode=2))
        while not svc.results:
            assert time.monotonic() - t0 < 10
            await asyncio.sleep(0.01)
        t_job = time.monotonic() - t0
        assert svc.results[0].ok, svc.results[0]
        assert s3.object_bytes("triton-staging", object_key("d1", "d.mkv")) == data
        await svc.shutdown(grace=5)
        await s3.stop()
        await origin.stop()
        await broker.stop()
        return t_amqp, t_s3, t_job

    t_amqp, t_s3, t_job = asyncio.run(asyncio.wait_for(main(), 60))
    assert t_amqp < 1.0 and t_s3 < 1.0 and t_job < 1.0, (t_amqp, t_s3, t_job)


def test_ip_literals_skip_the_resolver():
    assert dial.literal_infos("127.0.0.1", 80)[0][4] == ("127.0.0.1", 80)
    assert dial.literal_infos("[::1]", 443)[0][0] == socket.AF_INET6
    assert dial.literal_infos("example.com", 80) is None
