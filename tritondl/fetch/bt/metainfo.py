"""Torrent metainfo (BEP 3), magnet links (BEP 9) and torrent creation.

``Info`` is the parsed info dictionary with the file layout used by the
storage (single-file: ``<name>``; multi-file: ``<name>/<path...>``, the
layout anacrolix ``storage.NewFile(baseDir)`` writes, reference
``internal/downloader/torrent/torrent.go:41``).
"""

from __future__ import annotations

import base64
import hashlib
import os
from dataclasses import dataclass, field
from urllib.parse import parse_qs, quote, unquote, urlparse

from . import bencode
from .bencode import BencodeError

BLOCK = 16 * 1024  # request/metadata block size


class MetainfoError(ValueError):
    pass


@dataclass
class FileEntry:
    path: list[str]      # path components below the torrent root
    length: int
    offset: int          # offset in the concatenated piece stream
    pad: bool = False    # BEP 47 padding file (attr "p"): zeros, never written to disk


def _safe_component(c: bytes | str) -> str:
    s = c.decode("utf-8", "surrogateescape") if isinstance(c, bytes) else c
    if s in ("", ".", "..") or "/" in s or "\x00" in s:
        raise MetainfoError(f"unsafe path component {s!r}")
    return s


@dataclass
class Info:
    name: str
    piece_length: int
    pieces: bytes                 # concatenated 20-byte SHA-1s
    files: list[FileEntry]
    multi: bool
    raw: bytes                    # exact bencoded info dict
    private: bool = False
    infohash: bytes = b""

    @property
    def total_length(self) -> int:
        return sum(f.length for f in self.files)

    @property
    def num_pieces(self) -> int:
        return len(self.pieces) // 20

    def piece_hash(self, i: int) -> bytes:
        return self.pieces[20 * i:20 * i + 20]

    def piece_size(self, i: int) -> int:
        if i == self.num_pieces - 1:
            rem = self.total_length - i * self.piece_length
            return rem
        return self.piece_length

    def file_paths(self, base_dir: str) -> list[tuple[str, int]]:
        """[(absolute path, length), ...] in stream order; a BEP 47 padding
        file's path is "" (zeros, never created — the native verifiers read
        an empty path as zero bytes)."""
        root = os.path.join(base_dir, self.name) if self.multi else base_dir
        if not self.multi:
            return [(os.path.join(base_dir, self.name), self.files[0].length)]
        return [("" if f.pad else os.path.join(root, *f.path), f.length) for f in self.files]

    @classmethod
    def parse(cls, raw: bytes) -> "Info":
        try:
            d = bencode.decode(raw)
        except BencodeError as e:
            raise MetainfoError(f"bad info dict: {e}") from e
        if not isinstance(d, dict):
            raise MetainfoError("info is not a dict")
        try:
            name = _safe_component(d[b"name"])
            plen = int(d[b"piece length"])
            pieces = bytes(d[b"pieces"])
        except (KeyError, TypeError, ValueError) as e:
            raise MetainfoError(f"info dict missing field: {e}") from e
        if plen <= 0 or len(pieces) % 20:
            raise MetainfoError("invalid piece length / pieces")
        files: list[FileEntry] = []
        off = 0
        if b"files" in d:
            multi = True
            for f in d[b"files"]:
                path = [_safe_component(c) for c in f[b"path"]]
                if not path:
                    raise MetainfoError("empty file path")
                ln = int(f[b"length"])
                if ln < 0:
                    raise MetainfoError("negative length")
                attr = f.get(b"attr", b"")
                files.append(FileEntry(path, ln, off, isinstance(attr, bytes) and b"p" in attr))
                off += ln
        else:
            multi = False
            ln = int(d[b"length"])
            files.append(FileEntry([name], ln, 0))
            off = ln
        npieces = len(pieces) // 20
        if npieces != (off + plen - 1) // plen:
            raise MetainfoError(f"piece count {npieces} does not match total length {off}")
        return cls(name, plen, pieces, files, multi, bytes(raw), bool(d.get(b"private", 0)),
                   hashlib.sha1(raw).digest())


@dataclass
class Metainfo:
    info: Info
    announce: list[list[str]] = field(default_factory=list)   # tiers
    nodes: list[tuple[str, int]] = field(default_factory=list)
    url_list: list[str] = field(default_factory=list)

    @property
    def infohash(self) -> bytes:
        return self.info.infohash

    @classmethod
    def parse(cls, data: bytes) -> "Metainfo":
        try:
            d, spans = bencode.decode_with_spans(data)
        except BencodeError as e:
            raise MetainfoError(f"bad torrent file: {e}") from e
        if b"info" not in spans:
            raise MetainfoError("torrent has no info dict")
        s, e = spans[b"info"]
        info = Info.parse(bytes(data[s:e]))
        tiers: list[list[str]] = []
        if b"announce-list" in d:
            for tier in d[b"announce-list"]:
                t = [u.decode(errors="replace") for u in tier if isinstance(u, bytes)]
                if t:
                    tiers.append(t)
        elif b"announce" in d:
            tiers.append([d[b"announce"].decode(errors="replace")])
        nodes = [(n[0].decode(), int(n[1])) for n in d.get(b"nodes", []) if isinstance(n, list) and len(n) == 2]
        ul = d.get(b"url-list", [])
        url_list = [ul.decode()] if isinstance(ul, bytes) else [u.decode() for u in ul if isinstance(u, bytes)]
        return cls(info, tiers, nodes, url_list)

    def encode(self) -> bytes:
        d: dict = {b"info": _Raw(self.info.raw)}
        if self.announce:
            d[b"announce"] = self.announce[0][0].encode()
            d[b"announce-list"] = [[u.encode() for u in t] for t in self.announce]
        if self.url_list:
            d[b"url-list"] = [u.encode() for u in self.url_list]
        return _encode_with_raw(d)


class _Raw:
    def __init__(self, b: bytes) -> None:
        self.b = b


def _encode_with_raw(d: dict) -> bytes:
    out = [b"d"]
    for k in sorted(d):
        out.append(b"%d:" % len(k) + k)
        v = d[k]
        out.append(v.b if isinstance(v, _Raw) else bencode.encode(v))
    out.append(b"e")
    return b"".join(out)


# ----------------------------------------------------------------- magnets


@dataclass
class Magnet:
    infohash: bytes
    display_name: str = ""
    trackers: list[str] = field(default_factory=list)
    peers: list[tuple[str, int]] = field(default_factory=list)
    web_seeds: list[str] = field(default_factory=list)

    @property
    def hex(self) -> str:
        return self.infohash.hex()

    def uri(self) -> str:
        parts = [f"xt=urn:btih:{self.hex}"]
        if self.display_name:
            parts.append("dn=" + quote(self.display_name))
        parts += ["tr=" + quote(t, safe="") for t in self.trackers]
        parts += [f"x.pe={h}:{p}" for h, p in self.peers]
        parts += ["ws=" + quote(w, safe="") for w in self.web_seeds]
        return "magnet:?" + "&".join(parts)


def parse_magnet(uri: str) -> Magnet:
    u = urlparse(uri)
    if u.scheme != "magnet":
        raise MetainfoError(f"unsupported scheme '{u.scheme}'")
    q = parse_qs(u.query, keep_blank_values=True)
    ih = None
    for xt in q.get("xt", []):
        if xt.lower().startswith("urn:btih:"):
            h = xt[9:]
            if len(h) == 40:
                ih = bytes.fromhex(h)
            elif len(h) == 32:
                ih = base64.b32decode(h.upper())
            else:
                raise MetainfoError(f"bad btih length {len(h)}")
    if ih is None:
        raise MetainfoError("magnet link has no urn:btih")
    peers = []
    for pe in q.get("x.pe", []):
        host, _, port = pe.rpartition(":")
        if host and port.isdigit():
            peers.append((host.strip("[]"), int(port)))
    return Magnet(ih, unquote(q.get("dn", [""])[0]), q.get("tr", []), peers, q.get("ws", []))


# ----------------------------------------------------------------- create


def make_info(base: str, piece_length: int = 256 * 1024, name: str | None = None,
              private: bool = False, pad: bool = False) -> Info:
    """Build an info dict for a file or directory (used by the test swarm).
    ``pad``: align every file to a piece boundary with BEP 47 padding files."""
    from ...ops import hashing
    if os.path.isdir(base):
        entries = []
        for root, _dirs, fnames in os.walk(base):
            for fn in fnames:
                full = os.path.join(root, fn)
                rel = os.path.relpath(full, base).split(os.sep)
                entries.append((rel, full))
        entries.sort()
        files, layout = [], []
        for k, (rel, f) in enumerate(entries):
            n = os.path.getsize(f)
            files.append({b"length": n, b"path": [c.encode() for c in rel]})
            layout.append((f, n))
            if pad and k < len(entries) - 1 and n % piece_length:
                gap = piece_length - n % piece_length
                files.append({b"attr": b"p", b"length": gap, b"path": [b".pad", str(gap).encode()]})
                layout.append(("", gap))
        d = {b"name": (name or os.path.basename(base.rstrip("/"))).encode(), b"piece length": piece_length,
             b"files": files}
    else:
        layout = [(base, os.path.getsize(base))]
        d = {b"name": (name or os.path.basename(base)).encode(), b"piece length": piece_length,
             b"length": os.path.getsize(base)}
    total = sum(n for _p, n in layout)
    blob = bytearray()
    for p, n in layout:
        if not p:
            blob += bytes(n)
            continue
        with open(p, "rb") as f:
            blob += f.read()
    d[b"pieces"] = hashing.piece_hashes(bytes(blob), piece_length, "sha1") if total else b""
    if private:
        d[b"private"] = 1
    return Info.parse(bencode.encode(d))
