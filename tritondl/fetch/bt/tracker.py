"""Tracker clients: HTTP(S) announce (BEP 3, compact peers BEP 23, IPv6
``peers6`` BEP 7) and UDP trackers (BEP 15).  anacrolix announces to every
tracker of a magnet's ``tr=`` list / the torrent's announce-list; so do we.
"""

from __future__ import annotations

import asyncio
import ipaddress
import os
import random
import re
import socket
import struct
from dataclasses import dataclass
from urllib.parse import quote_from_bytes, urlparse

import aiohttp

from . import bencode


class TrackerError(Exception):
    pass


@dataclass
class Announce:
    infohash: bytes
    peer_id: bytes
    port: int
    uploaded: int = 0
    downloaded: int = 0
    left: int = 0
    event: str = "started"  # started|completed|stopped|""
    numwant: int = 200


@dataclass
class AnnounceResult:
    interval: int
    peers: list[tuple[str, int]]
    seeders: int | None = None
    leechers: int | None = None


MAX_REPLY = 4 << 20          # an HTTP announce reply (200 dict peers is ~20 KB): more is refused


def parse_compact(b: bytes, v6: bool = False) -> list[tuple[str, int]]:
    step = 18 if v6 else 6
    out = []
    for i in range(0, len(b) - step + 1, step):
        ip = str(ipaddress.ip_address(b[i:i + step - 2]))
        (port,) = struct.unpack(">H", b[i + step - 2:i + step])
        if port:
            out.append((ip, port))
    return out


def compact_peers(peers: list[tuple[str, int]], v6: bool = False) -> bytes:
    """Compact peer list: 6-byte IPv4 entries, or (``v6``) 18-byte IPv6 ones."""
    if v6:
        return b"".join(socket.inet_pton(socket.AF_INET6, h) + struct.pack(">H", p) for h, p in peers if ":" in h)
    return b"".join(socket.inet_aton(h) + struct.pack(">H", p) for h, p in peers if ":" not in h)


async def http_announce(url: str, a: Announce, session: aiohttp.ClientSession | None = None,
                        timeout: float = 15.0) -> AnnounceResult:
    q = (f"info_hash={quote_from_bytes(a.infohash, safe='')}&peer_id={quote_from_bytes(a.peer_id, safe='')}"
         f"&port={a.port}&uploaded={a.uploaded}&downloaded={a.downloaded}&left={a.left}&compact=1"
         f"&numwant={a.numwant}")
    if a.event:
        q += f"&event={a.event}"
    full = url + ("&" if "?" in url else "?") + q
    own = session is None
    s = session or aiohttp.ClientSession()
    try:
        from yarl import URL
        async with s.get(URL(full, encoded=True), timeout=aiohttp.ClientTimeout(total=timeout)) as r:
            if r.status != 200:
                raise TrackerError(f"tracker HTTP {r.status}")
            body = bytearray()
            while chunk := await r.content.read(64 << 10):
                body += chunk
                if len(body) > MAX_REPLY:
                    raise TrackerError(f"tracker reply larger than {MAX_REPLY} bytes")
    except (aiohttp.ClientError, asyncio.TimeoutError) as e:
        raise TrackerError(f"tracker request failed: {e}") from e
    finally:
        if own:
            await s.close()
    return parse_announce_response(bytes(body))


_HOSTNAME = re.compile(r"[A-Za-z0-9](?:[A-Za-z0-9-]{0,61}[A-Za-z0-9])?(?:\.[A-Za-z0-9](?:[A-Za-z0-9-]{0,61}[A-Za-z0-9])?)*\.?")


def _peer_host(h: str) -> bool:
    """BEP 3 dict peers: ``ip`` is an IP address or a DNS name."""
    try:
        ipaddress.ip_address(h)
        return True
    except ValueError:
        return len(h) <= 253 and _HOSTNAME.fullmatch(h) is not None


def parse_announce_response(body: bytes) -> AnnounceResult:
    """BEP 3 / BEP 23 / BEP 7 HTTP announce reply: compact or dict peers,
    ``peers6``; anything malformed is a TrackerError (never another type)."""
    try:
        d = bencode.decode(body)
    except bencode.BencodeError as e:
        raise TrackerError(f"bad tracker response: {e}") from e
    if not isinstance(d, dict):
        raise TrackerError("tracker response is not a dict")
    if b"failure reason" in d:
        why = d[b"failure reason"]
        raise TrackerError(why.decode(errors="replace") if isinstance(why, bytes) else repr(why))
    peers: list[tuple[str, int]] = []
    p = d.get(b"peers", b"")
    if isinstance(p, bytes):
        peers += parse_compact(p)
    elif isinstance(p, list):
        for e in p:
            try:
                ip, port = e[b"ip"].decode(), int(e[b"port"])
            except (KeyError, TypeError, ValueError, AttributeError, UnicodeDecodeError):
                continue
            if 0 < port < 65536 and _peer_host(ip):
                peers.append((ip, port))
    p6 = d.get(b"peers6", b"")
    if isinstance(p6, bytes):
        peers += parse_compact(p6, v6=True)
    iv = d.get(b"interval", 1800)

    def count(k: bytes) -> int | None:
        v = d.get(k)
        return v if isinstance(v, int) and v >= 0 else None
    return AnnounceResult(iv if isinstance(iv, int) and iv > 0 else 1800, peers, count(b"complete"),
                          count(b"incomplete"))


class _UDPProto(asyncio.DatagramProtocol):
    def __init__(self) -> None:
        self.q: asyncio.Queue = asyncio.Queue()

    def datagram_received(self, data: bytes, addr) -> None:
        self.q.put_nowait(data)

    def error_received(self, exc: Exception) -> None:
        self.q.put_nowait(exc)


UDP_PROTOCOL_ID = 0x41727101980
EVENTS = {"": 0, "completed": 1, "started": 2, "stopped": 3}


async def udp_announce(url: str, a: Announce, timeout: float = 5.0, retries: int = 2) -> AnnounceResult:
    u = urlparse(url)
    host, port = u.hostname, u.port
    if not host or not port:
        raise TrackerError(f"bad udp tracker url {url}")
    loop = asyncio.get_running_loop()
    tr, proto = await loop.create_datagram_endpoint(_UDPProto, remote_addr=(host, port))
    try:
        async def rpc(pkt: bytes, tid: int) -> bytes:
            for attempt in range(retries + 1):
                tr.sendto(pkt)
                try:
                    while True:
                        r = await asyncio.wait_for(proto.q.get(), timeout * (2 ** attempt))
                        if isinstance(r, Exception):
                            raise TrackerError(str(r))
                        if len(r) >= 8 and struct.unpack(">I", r[4:8])[0] == tid:
                            if struct.unpack(">I", r[:4])[0] == 3:
                                raise TrackerError(r[8:].decode(errors="replace"))
                            return r
                except asyncio.TimeoutError:
                    continue
            raise TrackerError("udp tracker timed out")

        tid = random.getrandbits(32)
        r = await rpc(struct.pack(">QII", UDP_PROTOCOL_ID, 0, tid), tid)
        if len(r) < 16:
            raise TrackerError("short connect response")
        (conn_id,) = struct.unpack(">Q", r[8:16])
        tid = random.getrandbits(32)
        key = random.getrandbits(32)
        pkt = struct.pack(">QII20s20sQQQIIIiH", conn_id, 1, tid, a.infohash, a.peer_id, a.downloaded, a.left,
                          a.uploaded, EVENTS.get(a.event, 0), 0, key, a.numwant, a.port)
        r = await rpc(pkt, tid)
        if len(r) < 20:
            raise TrackerError("short announce response")
        interval, leech, seed = struct.unpack(">III", r[8:20])
        # BEP 15: a tracker reached over IPv6 answers with 18-byte IPv6 peers
        sock = tr.get_extra_info("socket")
        v6 = sock is not None and sock.family == socket.AF_INET6
        return AnnounceResult(interval, parse_compact(r[20:], v6=v6), seed, leech)
    finally:
        tr.close()


async def announce(url: str, a: Announce, session: aiohttp.ClientSession | None = None) -> AnnounceResult:
    scheme = urlparse(url).scheme
    if scheme in ("http", "https"):
        return await http_announce(url, a, session)
    if scheme == "udp":
        return await udp_announce(url, a)
    raise TrackerError(f"unsupported tracker scheme {scheme!r}")


def new_peer_id() -> bytes:
    return b"-TD0100-" + os.urandom(12)
