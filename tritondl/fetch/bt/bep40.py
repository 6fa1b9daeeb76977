"""BEP 40 canonical peer priority.

anacrolix/torrent (the reference's BitTorrent library, reached from
``internal/downloader/torrent/torrent.go:40-48``) dials the candidate peers
with the highest BEP 40 priority first.  Both ends of a pair compute the
same number, so a swarm forms the same preferred connections from either
side.  The priority is CRC-32C of the two masked addresses, sorted; it is
computed over the ports when the IPs are equal.
"""

from __future__ import annotations

import ipaddress
import struct


def _crc32c_table() -> list[int]:
    poly = 0x82F63B78                      # Castagnoli, reflected
    table = []
    for n in range(256):
        c = n
        for _ in range(8):
            c = (c >> 1) ^ poly if c & 1 else c >> 1
        table.append(c)
    return table


_T = _crc32c_table()


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c = _T[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def _mask(a: bytes, b: bytes) -> tuple[bytes, bytes]:
    """Mask both addresses per BEP 40: the more of the prefix they share,
    the more of the address enters the hash."""
    if len(a) == 4:
        if a[:2] != b[:2]:
            m = b"\xff\xff\x55\x55"
        elif a[:3] != b[:3]:
            m = b"\xff\xff\xff\x55"
        else:
            m = b"\xff\xff\xff\xff"
    else:
        if a[:6] != b[:6]:
            m = b"\xff" * 6 + b"\x55" * 10
        elif a[:7] != b[:7]:
            m = b"\xff" * 7 + b"\x55" * 9
        elif a[:8] != b[:8]:
            m = b"\xff" * 8 + b"\x55" * 8
        else:
            m = b"\xff" * 16
    return bytes(x & y for x, y in zip(a, m)), bytes(x & y for x, y in zip(b, m))


def priority(mine: tuple[str, int], peer: tuple[str, int]) -> int:
    """BEP 40 priority of the connection between ``mine`` and ``peer``
    (ip, port).  Mixed IPv4/IPv6 pairs compare the IPv4-mapped forms."""
    try:
        ia, ib = ipaddress.ip_address(mine[0]), ipaddress.ip_address(peer[0])
    except ValueError:
        return 0
    if ia.version != ib.version:
        ia = ia if ia.version == 6 else ipaddress.IPv6Address("::ffff:" + str(ia))
        ib = ib if ib.version == 6 else ipaddress.IPv6Address("::ffff:" + str(ib))
    a, b = ia.packed, ib.packed
    if a == b:
        pa, pb = sorted((mine[1] & 0xFFFF, peer[1] & 0xFFFF))
        return crc32c(struct.pack(">HH", pa, pb))
    ma, mb = _mask(a, b)
    lo, hi = sorted((ma, mb))
    return crc32c(lo + hi)
