"""Egress proxy support (HTTP_PROXY / HTTPS_PROXY / NO_PROXY) — the
reference's transports honoured it through ``http.ProxyFromEnvironment``:
grab (``internal/downloader/http/http.go:18-20``) and minio-go's default
transport (``internal/uploader/uploader.go:43-51``).

Selection rules are pinned against the documented behaviour of
``golang.org/x/net/http/httpproxy`` (parity unpinned against a live Go
binary: no Go toolchain here).  Transfers go through ``fakes.proxy``: the
target names (``origin.test``, ``s3.test``) resolve only inside the proxy, so
a job that completes must have gone through it."""

import asyncio
import base64
import os

import pytest

from tritondl_testkit.fakes.origin import Origin
from tritondl_testkit.fakes.proxy import FakeProxy
from tritondl_testkit.fakes.s3 import FakeS3
from tritondl.fetch.http import HTTPDownloader, HTTPDownloadError
from tritondl.s3.client import S3Client, S3Error
from tritondl.s3.credentials import Static
from tritondl.utils import proxy as px
from tritondl.utils import rawhttp

NAMES = ["127.0.0.1", "localhost", "origin.test", "s3.test", "proxy.test"]


def run(coro, timeout=60):
    return asyncio.run(asyncio.wait_for(coro, timeout))


# ---------------------------------------------------------------- selection rules
def test_env_precedence_and_scheme_split():
    c = px.ProxyConfig.from_env({"HTTP_PROXY": "http://up:1", "http_proxy": "http://low:2",
                                 "https_proxy": "low3:3"})
    assert c.proxy_for("http://a.example/x").hostport == "up:1"       # upper case wins
    p = c.proxy_for("https://a.example/x")
    assert (p.scheme, p.host, p.port) == ("http", "low3", 3)          # scheme-less -> http://
    c = px.ProxyConfig.from_env({"HTTP_PROXY": "http://p:1"})
    assert c.proxy_for("https://a.example/") is None                  # https never uses HTTP_PROXY
    assert c.proxy_for("ftp://a.example/") is None
    assert px.ProxyConfig.from_env({"HTTP_PROXY": "p"}).http_proxy.port == 80
    assert px.ProxyConfig.from_env({"HTTPS_PROXY": "https://p"}).https_proxy.port == 443
    assert px.ProxyConfig.from_env({"HTTPS_PROXY": "socks5://p"}).https_proxy.port == 1080
    assert px.ProxyConfig.from_env({"HTTP_PROXY": "  "}).http_proxy is None
    assert not px.ProxyConfig.from_env({}).enabled


def test_no_proxy_matching():
    c = px.ProxyConfig("http://p:1", "http://p:1",
                       "example.com, .sub.org, *.star.net, 10.0.0.0/8, 192.168.1.5, 172.16.0.9:8080, "
                       "api.io:8443, [2001:db8::1]:443, :99")
    assert c.proxy_for("http://example.com/") is None                 # bare domain: host itself
    assert c.proxy_for("http://a.b.example.com/") is None             # ... and subdomains
    assert c.proxy_for("http://notexample.com/") is not None          # not a suffix at a dot
    assert c.proxy_for("http://sub.org/") is not None                 # leading dot: subdomains only
    assert c.proxy_for("http://x.sub.org/") is None
    assert c.proxy_for("http://star.net/") is not None                # *.domain == .domain
    assert c.proxy_for("http://y.star.net/") is None
    assert c.proxy_for("http://10.9.8.7/") is None                    # CIDR
    assert c.proxy_for("http://11.0.0.1/") is not None
    assert c.proxy_for("http://192.168.1.5:1234/") is None            # IP, any port
    assert c.proxy_for("http://172.16.0.9:8080/") is None             # IP + port
    assert c.proxy_for("http://172.16.0.9/") is not None              # other port (80)
    assert c.proxy_for("https://api.io:8443/") is None
    assert c.proxy_for("https://api.io/") is not None                 # default port 443 != 8443
    assert c.proxy_for("https://[2001:db8::1]/") is None
    assert c.proxy_for("http://EXAMPLE.COM/") is None                 # case-insensitive
    for url in ("http://localhost:9/", "http://127.0.0.1/", "http://127.3.4.5/", "https://[::1]:8/"):
        assert c.proxy_for(url) is None                               # loopback never proxied
    assert px.ProxyConfig("http://p:1", "", "*").proxy_for("http://a.example/") is None
    assert px.ProxyConfig("http://p:1", "", "a.b, *").proxy_for("http://z.example/") is None


def test_cgi_refuses_http_proxy_and_credentials():
    c = px.ProxyConfig.from_env({"HTTP_PROXY": "http://p:1", "HTTPS_PROXY": "http://q:2", "REQUEST_METHOD": "GET"})
    with pytest.raises(px.ProxyConfigError, match="cgihttpproxy"):
        c.proxy_for("http://a.example/")
    assert c.proxy_for("https://a.example/").host == "q"              # HTTPS_PROXY still honoured
    p = px.parse_proxy("http://us%40er:p%3Ass@proxy:3128")
    assert (p.username, p.password) == ("us@er", "p:ss")
    assert p.authorization() == "Basic " + base64.b64encode(b"us@er:p:ss").decode()
    assert p.redacted() == "http://us@er:xxxxx@proxy:3128" and "p:ss" not in p.redacted()
    assert px.parse_proxy("http://proxy:3128").authorization() is None


def test_environment_is_read_once(monkeypatch):
    monkeypatch.setenv("HTTPS_PROXY", "http://first:1")
    px.reset_environment()
    try:
        assert px.proxy_for("https://a.example/").host == "first"
        monkeypatch.setenv("HTTPS_PROXY", "http://second:1")
        assert px.proxy_for("https://a.example/").host == "first"     # cached, like Go's sync.Once
        px.reset_environment()
        assert px.proxy_for("https://a.example/").host == "second"
    finally:
        monkeypatch.delenv("HTTPS_PROXY")
        px.reset_environment()


# ---------------------------------------------------------------- transfers
@pytest.fixture(scope="module")
def pki():
    relay = rawhttp.relay_module()
    if relay is None:
        pytest.skip("native relay not built")
    return relay.make_test_pki(NAMES)


def _cfg(proxy: FakeProxy, user=None, pw=None, no_proxy=""):
    url = proxy.url_with(user, pw) if user is not None else proxy.url
    return px.ProxyConfig(url, url, no_proxy)


@pytest.mark.parametrize("native", [True, False])
@pytest.mark.parametrize("tls", [False, True])
def test_download_through_http_proxy(tmp_path, pki, native, tls):
    ca, cert, key = pki

    async def main():
        o = await Origin(tls=(cert, key) if tls else None).start()
        p = await FakeProxy(hosts={"origin.test": "127.0.0.1"}).start()
        data = os.urandom(1_500_000)
        o.add("/media/film.mkv", data)
        url = f"{'https' if tls else 'http'}://origin.test:{o.port}/media/film.mkv"
        h = HTTPDownloader(progress_interval=0.05, proxies=_cfg(p), ca_pem=ca, native=native, max_retries=1)
        await h.download(str(tmp_path), lambda u, v: None, url)
        assert (tmp_path / "film.mkv").read_bytes() == data
        if tls:
            assert p.connects and all(c == f"origin.test:{o.port}" for c in p.connects) and not p.requests
        else:
            assert p.requests and all(u == url for _m, u in p.requests) and not p.connects
        await h.close()
        await p.stop()
        await o.stop()
    run(main())


@pytest.mark.parametrize("tls", [False, True])
def test_download_through_socks5_proxy(tmp_path, pki, tls):
    ca, cert, key = pki

    async def main():
        o = await Origin(tls=(cert, key) if tls else None).start()
        p = await FakeProxy(mode="socks5", auth=("u", "pw"), hosts={"origin.test": "127.0.0.1"}).start()
        data = os.urandom(700_000)
        o.add("/a.mkv", data)
        url = f"{'https' if tls else 'http'}://origin.test:{o.port}/a.mkv"
        h = HTTPDownloader(progress_interval=0.05, proxies=_cfg(p, "u", "pw"), ca_pem=ca, max_retries=1)
        await h.download(str(tmp_path), lambda u, v: None, url)
        assert (tmp_path / "a.mkv").read_bytes() == data
        assert p.connects and p.connects[0] == f"origin.test:{o.port}" and p.refused == 0
        bad = HTTPDownloader(progress_interval=0.05, proxies=_cfg(p, "u", "wrong"), ca_pem=ca, max_retries=3)
        with pytest.raises(HTTPDownloadError, match="authentication failed"):
            await bad.download(str(tmp_path / "x"), lambda u, v: None, url)
        assert p.refused == 1                                           # refused once: not retried
        await bad.close()
        await h.close()
        await p.stop()
        await o.stop()
    os.makedirs(tmp_path / "x")
    run(main())


def test_download_through_https_proxy(tmp_path, pki):
    """An ``https://`` proxy: TLS to the proxy with the client's trust; an http
    target goes absolute-form inside it (native), an https target needs TLS
    inside TLS and takes the aiohttp path."""
    ca, cert, key = pki

    async def main():
        o = await Origin().start()
        p = await FakeProxy(tls=(cert, key), hosts={"origin.test": "127.0.0.1"}).start()
        p.host = "localhost"                       # the proxy's certificate names
        data = os.urandom(400_000)
        o.add("/b.mkv", data)
        url = f"http://origin.test:{o.port}/b.mkv"
        h = HTTPDownloader(progress_interval=0.05, proxies=_cfg(p), ca_pem=ca, max_retries=1)
        await h.download(str(tmp_path), lambda u, v: None, url)
        assert (tmp_path / "b.mkv").read_bytes() == data and p.requests
        await h.close()
        await p.stop()
        await o.stop()
    run(main())


def test_no_proxy_host_bypasses_proxy(tmp_path):
    async def main():
        loop = asyncio.get_running_loop()
        real = loop.getaddrinfo

        async def gai(host, *a, **k):                 # the client can resolve origin.test here
            return await real("127.0.0.1" if host == "origin.test" else host, *a, **k)
        loop.getaddrinfo = gai
        o = await Origin().start()
        p = await FakeProxy(hosts={"origin.test": "127.0.0.1"}).start()
        data = os.urandom(300_000)
        o.add("/c.mkv", data)
        url = f"http://origin.test:{o.port}/c.mkv"
        h = HTTPDownloader(progress_interval=0.05, proxies=_cfg(p, no_proxy="other.test,.test"), max_retries=1)
        await h.download(str(tmp_path), lambda u, v: None, url)
        assert (tmp_path / "c.mkv").read_bytes() == data
        assert p.requests == [] and p.connects == []
        await h.close()
        await p.stop()
        await o.stop()
    run(main())


@pytest.mark.parametrize("native", [True, False])
@pytest.mark.parametrize("tls", [False, True])
def test_proxy_407_fails_fast_with_clear_error(tmp_path, pki, native, tls):
    ca, cert, key = pki

    async def main():
        o = await Origin(tls=(cert, key) if tls else None).start()
        p = await FakeProxy(auth=("alice", "s3cret"), hosts={"origin.test": "127.0.0.1"}).start()
        o.add("/d.mkv", b"x" * 1000)
        url = f"{'https' if tls else 'http'}://origin.test:{o.port}/d.mkv"
        h = HTTPDownloader(progress_interval=0.05, proxies=_cfg(p), ca_pem=ca, native=native, max_retries=5)
        with pytest.raises(HTTPDownloadError, match="407|[Pp]roxy"):
            await h.download(str(tmp_path), lambda u, v: None, url)
        assert p.refused == 1                                           # one attempt, no retry storm
        ok = HTTPDownloader(progress_interval=0.05, proxies=_cfg(p, "alice", "s3cret"), ca_pem=ca, native=native)
        await ok.download(str(tmp_path), lambda u, v: None, url)
        assert (tmp_path / "d.mkv").read_bytes() == b"x" * 1000 and p.refused == 1
        await h.close()
        await ok.close()
        await p.stop()
        await o.stop()
    run(main())


@pytest.mark.parametrize("tls", [False, True])
def test_s3_upload_through_proxy(tmp_path, pki, tls):
    ca, cert, key = pki

    async def main():
        s3 = await FakeS3(access_key="ak", secret_key="sk", tls=(cert, key) if tls else None,
                          names=("s3.test",)).start()
        p = await FakeProxy(auth=("u", "p"), hosts={"s3.test": "127.0.0.1"}).start()
        ep = f"{'https' if tls else 'http'}://s3.test:{s3.port}"
        data = os.urandom(3_000_000)
        src = tmp_path / "obj.bin"
        src.write_bytes(data)
        c = S3Client(ep, Static("ak", "sk"), proxies=_cfg(p, "u", "p"), ca_pem=ca, max_retries=1)
        assert not await c.bucket_exists("bkt")
        await c.make_bucket("bkt")
        await c.put_object("bkt", "k/obj", str(src))
        assert s3.object_bytes("bkt", "k/obj") == data
        if tls:
            assert p.connects and not p.requests
        else:
            assert any(m == "PUT" and u.endswith("/bkt/k/obj") for m, u in p.requests)
        await c.close()
        bad = S3Client(ep, Static("ak", "sk"), proxies=_cfg(p), ca_pem=ca, max_retries=5)
        with pytest.raises(S3Error) as ei:
            await bad.put_object("bkt", "k/obj2", str(src))
        assert ei.value.status == 407 and "Proxy" in ei.value.code
        refused = p.refused
        with pytest.raises(S3Error) as ei:
            await bad.bucket_exists("bkt")
        assert ei.value.status == 407 and p.refused == refused + 1
        await bad.close()
        await p.stop()
        await s3.stop()
    run(main())


def test_service_jobs_through_proxy_from_environment(tmp_path, pki, monkeypatch):
    """The worker as deployed: proxy settings from the environment (read once),
    an http-origin job, an https-origin job, both uploaded to an https S3
    endpoint — every byte through the proxy, which needs credentials."""
    from tritondl.amqp.client import Client
    from tritondl.amqp.codec import Properties
    from tritondl_testkit.fakes.broker import Broker
    from tritondl.fetch.registry import Dispatcher
    from tritondl.models import Download, Media
    from tritondl.s3.uploader import Uploader, object_key
    from tritondl.service import Service
    from tritondl.utils.config import Config
    ca, cert, key = pki

    async def main():
        broker = await Broker().start()
        plain = await Origin().start()
        secure = await Origin(tls=(cert, key)).start()
        s3 = await FakeS3(access_key="ak", secret_key="sk", tls=(cert, key), names=("s3.test",)).start()
        p = await FakeProxy(auth=("svc", "pw"), hosts={"origin.test": "127.0.0.1", "s3.test": "127.0.0.1"}).start()
        monkeypatch.setenv("HTTP_PROXY", p.url_with("svc", "pw"))
        monkeypatch.setenv("HTTPS_PROXY", p.url_with("svc", "pw"))
        monkeypatch.setenv("NO_PROXY", "internal.example")
        px.reset_environment()
        cfg = Config()
        cfg.download_dir = str(tmp_path / "downloading")
        cfg.retry_delay_s = 0
        cfg.progress_log_interval_s = 0
        cfg.heartbeat_s = 0
        svc = Service(cfg, amqp=Client(broker.url, heartbeat=0, retry_delay=0),
                      dispatcher=Dispatcher(cfg.download_dir, [HTTPDownloader(progress_interval=0.05, ca_pem=ca)], 0),
                      uploader=Uploader(cfg.bucket, S3Client(f"https://s3.test:{s3.port}", Static("ak", "sk"),
                                                             ca_pem=ca)))
        await svc.start()
        a, b = os.urandom(900_000), os.urandom(1_100_000)
        plain.add("/a.mkv", a)
        secure.add("/b.mkv", b)
        for i, (mid, url) in enumerate((("m-a", f"http://origin.test:{plain.port}/a.mkv"),
                                        ("m-b", f"https://origin.test:{secure.port}/b.mkv"))):
            body = Download(created_at="t", media=Media(id=mid, source_uri=url)).encode()
            broker.inject("v1.download", f"v1.download-{i % 2}", body, Properties(delivery_mode=2))
        await svc.wait_finished(2, 30)
        assert all(r.ok for r in svc.results), svc.results
        assert s3.object_bytes("triton-staging", object_key("m-a", "a.mkv")) == a
        assert s3.object_bytes("triton-staging", object_key("m-b", "b.mkv")) == b
        assert any(u.startswith(f"http://origin.test:{plain.port}/") for _m, u in p.requests)
        assert f"origin.test:{secure.port}" in p.connects and f"s3.test:{s3.port}" in p.connects
        assert p.refused == 0
        await svc.shutdown(grace=5)
        for x in (p, s3, secure, plain, broker):
            await x.stop()

    try:
        run(main())
    finally:
        for k in ("HTTP_PROXY", "HTTPS_PROXY", "NO_PROXY"):
            monkeypatch.delenv(k)
        px.reset_environment()
