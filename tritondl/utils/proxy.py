"""Egress proxy selection with Go's ``http.ProxyFromEnvironment`` semantics.

Both of the reference's data paths honour ``HTTP_PROXY`` / ``HTTPS_PROXY`` /
``NO_PROXY``, through their libraries' defaults:

* grab's ``grab.NewClient()`` (``internal/downloader/http/http.go:18-20``)
  builds an ``http.Transport`` with ``Proxy: http.ProxyFromEnvironment``;
* minio-go v6's ``DefaultTransport``, behind ``minio.NewWithOptions``
  (``internal/uploader/uploader.go:43-51``), does the same.

The rules reproduced here are those of ``golang.org/x/net/http/httpproxy``
(what ``ProxyFromEnvironment`` calls):

* ``HTTP_PROXY`` (else ``http_proxy``) serves ``http://`` URLs, and
  ``HTTPS_PROXY`` (else ``https_proxy``) serves ``https://`` URLs.  An https
  request never falls back to ``HTTP_PROXY``.
* A proxy value without an ``http``/``https``/``socks5`` scheme is read as
  ``http://<value>``.  A value that still does not parse is ignored.
* ``NO_PROXY`` (else ``no_proxy``) is a comma list.  ``*`` disables proxying.
  Each entry is one of:
  * a CIDR (``10.0.0.0/8``);
  * an IP, optionally with a port;
  * a domain, optionally with a port.  ``example.com`` matches the host and
    every subdomain.  ``.example.com`` and ``*.example.com`` match subdomains
    only.
* ``localhost`` and loopback IPs are never proxied.
* In a CGI environment (``REQUEST_METHOD`` set) ``HTTP_PROXY`` is refused
  (httpoxy), with Go's error text.
* The environment is read once per process (Go caches it with a
  ``sync.Once``); :func:`reset_environment` re-reads it, for tests.

Credentials come from the proxy URL's userinfo (percent-decoded) and are sent
as ``Proxy-Authorization: Basic``: on every request through an ``http``
proxy, on the ``CONNECT`` of an https tunnel, and as the RFC 1929
username/password step of a ``socks5`` proxy.
"""

from __future__ import annotations

import base64
import ipaddress
import os
import re
from dataclasses import dataclass
from typing import Mapping
from urllib.parse import unquote, urlsplit

from .log import log

DEFAULT_PORTS = {"http": 80, "https": 443, "socks5": 1080}
_HOSTCHARS = re.compile(r"^[A-Za-z0-9._~%!$&'()*+,;=:-]+$")    # what Go's url.Parse accepts in a host


class ProxyConfigError(Exception):
    """The request must not be sent: Go's ``proxyForURL`` returned an error."""


@dataclass(frozen=True)
class ProxyURL:
    scheme: str                  # http | https | socks5
    host: str                    # hostname or IP, without brackets
    port: int
    username: str | None = None
    password: str | None = None

    @property
    def hostport(self) -> str:
        h = f"[{self.host}]" if ":" in self.host else self.host
        return f"{h}:{self.port}"

    def authorization(self) -> str | None:
        """``Proxy-Authorization`` value, or None without userinfo."""
        if self.username is None:
            return None
        raw = f"{self.username}:{self.password or ''}".encode()
        return "Basic " + base64.b64encode(raw).decode()

    def redacted(self) -> str:
        """The URL for logs and errors, password masked (Go ``url.Redacted``)."""
        auth = ""
        if self.username is not None:
            auth = self.username + (":xxxxx" if self.password is not None else "") + "@"
        return f"{self.scheme}://{auth}{self.hostport}"

    def url(self) -> str:
        """``scheme://host:port`` without credentials (aiohttp takes them apart)."""
        return f"{self.scheme}://{self.hostport}"

    @property
    def key(self) -> tuple:
        return (self.scheme, self.host, self.port, self.username, self.password)


def parse_proxy(value: str) -> ProxyURL | None:
    """httpproxy ``parseProxy``: "" → None; a value without a known scheme is
    retried as ``http://<value>``; None when neither parses."""
    value = (value or "").strip()
    if not value:
        return None
    for cand in (value, "http://" + value):
        try:
            u = urlsplit(cand)
            port = u.port
        except ValueError:
            continue
        if u.scheme not in DEFAULT_PORTS or not u.hostname or not _HOSTCHARS.match(u.hostname):
            continue
        user = unquote(u.username) if u.username is not None else None
        pw = unquote(u.password) if u.password is not None else None
        return ProxyURL(u.scheme, u.hostname, port or DEFAULT_PORTS[u.scheme], user, pw)
    return None


def _split_host_port(s: str) -> tuple[str, str] | None:
    """Go ``net.SplitHostPort``; None when ``s`` has no port part."""
    if s.startswith("["):
        end = s.find("]")
        if end < 0 or not s[end + 1:].startswith(":"):
            return None
        return s[1:end], s[end + 2:]
    if s.count(":") != 1:
        return None
    h, _, p = s.partition(":")
    return h, p


def _idna(host: str) -> str:
    try:
        return host.encode("idna").decode("ascii")
    except UnicodeError:
        return host


def _ip(s: str):
    try:
        return ipaddress.ip_address(s)
    except ValueError:
        return None


@dataclass(frozen=True)
class _DomainMatch:
    host: str          # always starts with "."
    port: str
    match_host: bool   # also the bare domain (entry had no leading dot)

    def match(self, host: str, port: str) -> bool:
        if host.endswith(self.host) or (self.match_host and host == self.host[1:]):
            return self.port == "" or self.port == port
        return False


class ProxyConfig:
    """Parsed proxy settings; :meth:`proxy_for` picks the proxy of one URL."""

    def __init__(self, http_proxy: str = "", https_proxy: str = "", no_proxy: str = "",
                 cgi: bool = False) -> None:
        self.http_proxy_raw, self.https_proxy_raw, self.no_proxy_raw = http_proxy, https_proxy, no_proxy
        self.cgi = cgi
        self.http_proxy = parse_proxy(http_proxy)
        self.https_proxy = parse_proxy(https_proxy)
        for name, raw, got in (("HTTP_PROXY", http_proxy, self.http_proxy),
                               ("HTTPS_PROXY", https_proxy, self.https_proxy)):
            if raw.strip() and got is None:
                log.with_fields(var=name).warn("ignoring unparseable proxy setting")
        self.all = False
        self._ips: list[tuple[object, str]] = []
        self._cidrs: list = []
        self._domains: list[_DomainMatch] = []
        self._parse_no_proxy(no_proxy)

    @classmethod
    def from_env(cls, env: Mapping[str, str] | None = None) -> "ProxyConfig":
        env = os.environ if env is None else env

        def any_of(*names: str) -> str:
            for n in names:
                v = env.get(n, "")
                if v:
                    return v
            return ""
        return cls(any_of("HTTP_PROXY", "http_proxy"), any_of("HTTPS_PROXY", "https_proxy"),
                   any_of("NO_PROXY", "no_proxy"), bool(env.get("REQUEST_METHOD", "")))

    @property
    def enabled(self) -> bool:
        return self.http_proxy is not None or self.https_proxy is not None

    def _parse_no_proxy(self, s: str) -> None:
        if s == "*":
            self.all = True
            return
        for p in s.split(","):
            p = p.strip().lower()
            if not p:
                continue
            if p == "*":
                self.all = True
                return
            if "/" in p:
                try:
                    self._cidrs.append(ipaddress.ip_network(p, strict=False))
                    continue
                except ValueError:
                    pass
            hp = _split_host_port(p)
            if hp is not None:
                phost, pport = hp
                if not phost:
                    continue          # no host part: malformed, ignored (as Go does)
            else:
                phost, pport = p, ""
            ip = _ip(phost)
            if ip is not None:
                self._ips.append((ip, pport))
                continue
            if phost.startswith("*."):
                phost = phost[1:]
            match_host = False
            if not phost.startswith("."):
                match_host = True
                phost = "." + phost
            self._domains.append(_DomainMatch(_idna(phost), pport, match_host))

    def use_proxy(self, host: str, port: str) -> bool:
        """httpproxy ``useProxy`` for one canonical ``host``/``port``."""
        if not host:
            return True
        if host == "localhost":
            return False
        ip = _ip(host)
        if ip is not None and ip.is_loopback:
            return False
        if self.all:
            return False
        h = host.strip().lower()
        if ip is not None:
            for mip, mport in self._ips:
                if mip == ip and (mport == "" or mport == port):
                    return False
            for net in self._cidrs:
                if ip.version == net.version and ip in net:
                    return False
        for d in self._domains:
            if d.match(h, port):
                return False
        return True

    def proxy_for(self, url: str) -> ProxyURL | None:
        """The proxy for ``url`` (None = dial directly).  Raises
        :class:`ProxyConfigError` where Go's ``proxyForURL`` errors."""
        if self.http_proxy is None and self.https_proxy is None:
            return None                 # the common case: no proxy at all, nothing to parse
        u = urlsplit(url)
        scheme = u.scheme.lower()
        if scheme == "https":
            proxy = self.https_proxy
        elif scheme == "http":
            proxy = self.http_proxy
            if proxy is not None and self.cgi:
                raise ProxyConfigError("refusing to use HTTP_PROXY value in CGI environment; "
                                       "see golang.org/s/cgihttpproxy")
        else:
            return None
        if proxy is None:
            return None
        host = (u.hostname or "").lower()
        try:
            port = u.port
        except ValueError:
            port = None
        port = port or DEFAULT_PORTS[scheme]
        if not self.use_proxy(_idna(host), str(port)):
            return None
        return proxy


def aiohttp_kwargs(p: ProxyURL | None, secure: bool) -> tuple[dict, dict]:
    """(request kwargs, extra request headers) that route one aiohttp request
    through ``p``.  Credentials go on the ``CONNECT`` for https targets and on
    the request itself for http ones: aiohttp copies ``proxy_headers`` only
    into the ``CONNECT``.  A socks5 proxy raises ``ValueError``, because
    aiohttp has no SOCKS support; the native data plane has it."""
    if p is None:
        return {}, {}
    if p.scheme == "socks5":
        raise ValueError(f"the socks5 proxy {p.redacted()} needs the native data plane")
    auth = p.authorization()
    if auth is None:
        return {"proxy": p.url()}, {}
    if secure:
        return {"proxy": p.url(), "proxy_headers": {"Proxy-Authorization": auth}}, {}
    return {"proxy": p.url()}, {"Proxy-Authorization": auth}


_env: ProxyConfig | None = None


def from_environment() -> ProxyConfig:
    """The process-wide settings, read from the environment once."""
    global _env
    if _env is None:
        _env = ProxyConfig.from_env()
    return _env


def reset_environment() -> None:
    """Forget the cached settings (tests that change the environment)."""
    global _env
    _env = None


def proxy_for(url: str) -> ProxyURL | None:
    return from_environment().proxy_for(url)


__all__ = ["ProxyConfig", "ProxyConfigError", "ProxyURL", "from_environment", "parse_proxy", "proxy_for",
           "reset_environment"]
