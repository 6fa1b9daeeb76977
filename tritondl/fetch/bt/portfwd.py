"""NAT port forwarding through a UPnP Internet Gateway Device.

anacrolix's default client config (``NoDefaultPortForwarding: false``,
behind ``torrent.NewDefaultClientConfig()`` in the reference's
``internal/downloader/torrent/torrent.go:40``) asks the LAN's UPnP gateway to
forward the client's listen port, TCP and UDP, so that peers outside the NAT
can dial in.  This is that capability:

* SSDP ``M-SEARCH`` for ``InternetGatewayDevice:1``/``:2`` on
  239.255.255.250:1900 (or a given address), first answer wins;
* the device description (``LOCATION``) is walked for a
  ``WANIPConnection:1|2`` or ``WANPPPConnection:1`` service and its
  ``controlURL``;
* SOAP ``AddPortMapping`` for each protocol (internal client = the local
  address that routes to the gateway), ``GetExternalIPAddress``, and
  ``DeletePortMapping`` when the torrent closes;
* the discovered gateway is cached per process (``cache_ttl``), so a worker
  that opens a fresh client per job does one discovery, not one per job;
  a failed discovery is cached too (datacentre hosts have no gateway) and
  costs one ``timeout`` in the background, never on the job path.
"""

from __future__ import annotations

import asyncio
import socket
import time
import xml.etree.ElementTree as ET
from dataclasses import dataclass
from urllib.parse import urljoin, urlparse

from ...utils.log import log

SSDP_ADDR = ("239.255.255.250", 1900)
IGD_TYPES = ("urn:schemas-upnp-org:device:InternetGatewayDevice:1",
             "urn:schemas-upnp-org:device:InternetGatewayDevice:2")
WAN_SERVICES = ("urn:schemas-upnp-org:service:WANIPConnection:2",
                "urn:schemas-upnp-org:service:WANIPConnection:1",
                "urn:schemas-upnp-org:service:WANPPPConnection:1")


class UPnPError(Exception):
    pass


@dataclass
class Gateway:
    location: str
    control_url: str
    service_type: str
    local_ip: str


def _msearch(st: str) -> bytes:
    return ("M-SEARCH * HTTP/1.1\r\n"
            f"HOST: {SSDP_ADDR[0]}:{SSDP_ADDR[1]}\r\n"
            'MAN: "ssdp:discover"\r\n'
            "MX: 2\r\n"
            f"ST: {st}\r\n\r\n").encode()


def _headers(data: bytes) -> dict[str, str]:
    out: dict[str, str] = {}
    for line in data.decode("latin-1").split("\r\n")[1:]:
        k, sep, v = line.partition(":")
        if sep:
            out[k.strip().lower()] = v.strip()
    return out


async def ssdp_search(addr: tuple[str, int] = SSDP_ADDR, timeout: float = 2.0) -> str | None:
    """LOCATION of the first IGD that answers an M-SEARCH, or None."""
    loop = asyncio.get_running_loop()
    got: asyncio.Future = loop.create_future()

    class P(asyncio.DatagramProtocol):
        def datagram_received(self, data, src):
            h = _headers(data)
            if h.get("location") and not got.done() and \
                    any(t in (h.get("st", "") + h.get("nt", "")) for t in IGD_TYPES):
                got.set_result(h["location"])

        def error_received(self, exc):
            pass

    tr, _ = await loop.create_datagram_endpoint(P, local_addr=("0.0.0.0", 0), family=socket.AF_INET)
    try:
        sock = tr.get_extra_info("socket")
        if sock is not None:
            sock.setsockopt(socket.IPPROTO_IP, socket.IP_MULTICAST_TTL, 2)
        for st in IGD_TYPES:
            tr.sendto(_msearch(st), addr)
        try:
            return await asyncio.wait_for(got, timeout)
        except asyncio.TimeoutError:
            return None
    finally:
        tr.close()


async def _http(method: str, url: str, body: bytes = b"", headers: dict | None = None,
                timeout: float = 5.0) -> tuple[int, bytes]:
    """Minimal HTTP/1.1 client (gateways speak plain HTTP on the LAN)."""
    u = urlparse(url)
    host, port = u.hostname or "", u.port or 80
    path = (u.path or "/") + (f"?{u.query}" if u.query else "")
    hdrs = {"Host": f"{host}:{port}", "Connection": "close", "Content-Length": str(len(body)), **(headers or {})}
    req = f"{method} {path} HTTP/1.1\r\n" + "".join(f"{k}: {v}\r\n" for k, v in hdrs.items()) + "\r\n"

    async def go() -> tuple[int, bytes]:
        r, w = await asyncio.open_connection(host, port)
        try:
            w.write(req.encode() + body)
            await w.drain()
            raw = await r.read(1 << 20)
            while True:
                more = await r.read(1 << 20)
                if not more:
                    break
                raw += more
        finally:
            w.close()
        head, _, rest = raw.partition(b"\r\n\r\n")
        status = int(head.split(b" ", 2)[1]) if head.startswith(b"HTTP/") else 0
        hl = _headers(head + b"\r\n")
        if "chunked" in hl.get("transfer-encoding", "").lower():
            out, pos = b"", 0
            while True:
                eol = rest.find(b"\r\n", pos)
                if eol < 0:
                    break
                n = int(rest[pos:eol].split(b";")[0] or b"0", 16)
                if n == 0:
                    break
                out += rest[eol + 2:eol + 2 + n]
                pos = eol + 2 + n + 2
            rest = out
        return status, rest
    return await asyncio.wait_for(go(), timeout)


def _local_ip_for(host: str) -> str:
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    try:
        s.connect((host, 9))                 # no packet is sent: just a route lookup
        return s.getsockname()[0]
    finally:
        s.close()


def _strip(tag: str) -> str:
    return tag.rsplit("}", 1)[-1]


async def describe(location: str) -> Gateway:
    status, body = await _http("GET", location)
    if status != 200:
        raise UPnPError(f"device description: HTTP {status}")
    root = ET.fromstring(body)
    base = location
    for el in root.iter():
        if _strip(el.tag) == "URLBase" and (el.text or "").strip():
            base = el.text.strip()
    found: dict[str, str] = {}
    for svc in root.iter():
        if _strip(svc.tag) != "service":
            continue
        fields = {_strip(c.tag): (c.text or "").strip() for c in svc}
        if fields.get("serviceType") in WAN_SERVICES and fields.get("controlURL"):
            found.setdefault(fields["serviceType"], fields["controlURL"])
    for st in WAN_SERVICES:
        if st in found:
            return Gateway(location, urljoin(base, found[st]), st,
                           _local_ip_for(urlparse(location).hostname or "127.0.0.1"))
    raise UPnPError("no WANIPConnection/WANPPPConnection service")


async def soap(gw: Gateway, action: str, args: dict[str, str | int]) -> dict[str, str]:
    inner = "".join(f"<{k}>{v}</{k}>" for k, v in args.items())
    body = ('<?xml version="1.0"?>'
            '<s:Envelope xmlns:s="http://schemas.xmlsoap.org/soap/envelope/" '
            's:encodingStyle="http://schemas.xmlsoap.org/soap/encoding/"><s:Body>'
            f'<u:{action} xmlns:u="{gw.service_type}">{inner}</u:{action}>'
            '</s:Body></s:Envelope>').encode()
    status, resp = await _http("POST", gw.control_url, body, {
        "Content-Type": 'text/xml; charset="utf-8"', "SOAPAction": f'"{gw.service_type}#{action}"'})
    try:
        root = ET.fromstring(resp) if resp else None
    except ET.ParseError:
        root = None
    if status != 200:
        code = desc = ""
        if root is not None:
            for el in root.iter():
                if _strip(el.tag) == "errorCode":
                    code = (el.text or "").strip()
                elif _strip(el.tag) == "errorDescription":
                    desc = (el.text or "").strip()
        raise UPnPError(f"{action}: HTTP {status} UPnPError {code} {desc}".strip())
    out: dict[str, str] = {}
    if root is not None:
        for el in root.iter():
            if _strip(el.tag).endswith("Response"):
                for c in el:
                    out[_strip(c.tag)] = (c.text or "").strip()
    return out


_cache: dict[tuple, tuple[float, Gateway | None]] = {}


async def discover(addr: tuple[str, int] = SSDP_ADDR, timeout: float = 2.0, cache_ttl: float = 600.0) -> Gateway | None:
    key = (addr,)
    hit = _cache.get(key)
    if hit is not None and time.monotonic() - hit[0] < cache_ttl:
        return hit[1]
    gw = None
    try:
        loc = await ssdp_search(addr, timeout)
        if loc:
            gw = await describe(loc)
    except (OSError, UPnPError, ET.ParseError, asyncio.TimeoutError, ValueError) as e:
        log.with_field("error", str(e)).debug("upnp discovery failed")
    _cache[key] = (time.monotonic(), gw)
    return gw


class PortForwarder:
    """Forward ``port`` (TCP and UDP) for the life of one torrent client."""

    def __init__(self, port: int, *, protocols: tuple[str, ...] = ("TCP", "UDP"), lease: int = 0,
                 description: str = "tritondl", ssdp_addr: tuple[str, int] = SSDP_ADDR,
                 timeout: float = 2.0) -> None:
        self.port = port
        self.protocols = protocols
        self.lease = lease
        self.description = description
        self.ssdp_addr = ssdp_addr
        self.timeout = timeout
        self.gateway: Gateway | None = None
        self.external_ip: str | None = None
        self.mapped: list[str] = []

    async def start(self) -> bool:
        self.gateway = await discover(self.ssdp_addr, self.timeout)
        if self.gateway is None:
            return False
        gw = self.gateway
        for proto in self.protocols:
            try:
                await soap(gw, "AddPortMapping", {
                    "NewRemoteHost": "", "NewExternalPort": self.port, "NewProtocol": proto,
                    "NewInternalPort": self.port, "NewInternalClient": gw.local_ip, "NewEnabled": 1,
                    "NewPortMappingDescription": f"{self.description} ({proto})",
                    "NewLeaseDuration": self.lease})
                self.mapped.append(proto)
            except (UPnPError, OSError, asyncio.TimeoutError) as e:
                log.with_fields(port=self.port, proto=proto, error=str(e)).warn("upnp port mapping failed")
        try:
            self.external_ip = (await soap(gw, "GetExternalIPAddress", {})).get("NewExternalIPAddress")
        except (UPnPError, OSError, asyncio.TimeoutError):
            pass
        if self.mapped:
            log.with_fields(port=self.port, protocols=self.mapped, external_ip=self.external_ip).info(
                "forwarded listen port via upnp")
        return bool(self.mapped)

    async def close(self) -> None:
        gw = self.gateway
        if gw is None:
            return
        for proto in self.mapped:
            try:
                await soap(gw, "DeletePortMapping", {"NewRemoteHost": "", "NewExternalPort": self.port,
                                                     "NewProtocol": proto})
            except (UPnPError, OSError, asyncio.TimeoutError) as e:
                log.with_fields(port=self.port, proto=proto, error=str(e)).debug("upnp unmap failed")
        self.mapped = []
