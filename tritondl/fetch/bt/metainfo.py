"""Torrent metainfo (BEP 3; v2 and hybrid torrents, BEP 52), magnet links
(BEP 9, ``btih`` and ``btmh``) and torrent creation.

v2 torrents describe files in a ``file tree`` with per-file merkle roots
(:mod:`.merkle`); their piece index space is the files laid end to end, each
starting on a piece boundary.  A pure v2 torrent is mapped onto the same
``files`` layout the v1 code uses by inserting virtual BEP 47 padding
entries, so storage, the piece picker and the wire protocol are shared; only
piece verification differs (:meth:`Info.check_piece`).

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

from . import bencode, merkle
from .bencode import BencodeError

try:  # native piece roots (SHA-NI pairs, GIL released); merkle.piece_root is the executable spec
    from ...ops.hashing import merkle_root as _merkle_root
except ImportError:  # pragma: no cover - host extension not built
    _merkle_root = merkle.piece_root

BLOCK = 16 * 1024  # request/metadata block size


class MetainfoError(ValueError):
    pass


def _bint(v) -> int:
    """A bencoded integer field (not a string of digits, not a list)."""
    if isinstance(v, bool) or not isinstance(v, int):
        raise TypeError(f"expected an integer, got {type(v).__name__}")
    return v


def _bbytes(v) -> bytes:
    if not isinstance(v, (bytes, bytearray)):
        raise TypeError(f"expected a byte string, got {type(v).__name__}")
    return bytes(v)


@dataclass
class FileEntry:
    path: list[str]      # path components below the torrent root
    length: int
    offset: int          # offset in the concatenated piece stream
    pad: bool = False    # BEP 47 padding file (attr "p"): zeros, never written to disk


# longest component the work dir can hold next to its ``.s3upload.tmp`` /
# ``.part.meta.tmp`` sidecars (Linux NAME_MAX is 255 bytes)
COMPONENT_MAX = 255 - len(".part.meta.tmp")


def _safe_component(c: bytes | str) -> str:
    """A path component of the info dict as it goes on disk.  ``..``, ``/``
    and NUL are refused.  A component too long for the file system (names
    from Windows may be 255 UTF-16 units, up to 765 UTF-8 bytes) is cut in
    its stem on a character boundary, with ``~`` and 8 hex digits of its
    SHA-1 so that names sharing a long prefix stay distinct, keeping the
    extension the media filter selects on.  anacrolix opens the full name and
    fails the download with ENAMETOOLONG."""
    if not isinstance(c, (bytes, str)):
        raise MetainfoError(f"path component is not a string: {type(c).__name__}")
    s = c.decode("utf-8", "surrogateescape") if isinstance(c, bytes) else c
    if s in ("", ".", "..") or "/" in s or "\x00" in s:
        raise MetainfoError(f"unsafe path component {s!r}")
    raw = s.encode("utf-8", "surrogateescape")
    if len(raw) <= COMPONENT_MAX:
        return s
    stem, dot, ext = s.rpartition(".")
    if not (dot and stem and len(ext.encode("utf-8", "surrogateescape")) < 32):
        stem, dot, ext = s, "", ""
    tag = "~" + hashlib.sha1(raw).hexdigest()[:8]
    room = COMPONENT_MAX - len(tag) - len((dot + ext).encode("utf-8", "surrogateescape"))
    kept, n = [], 0
    for ch in stem:
        n += len(ch.encode("utf-8", "surrogateescape"))
        if n > room:
            break
        kept.append(ch)
    return "".join(kept) + tag + dot + ext


@dataclass
class V2File:
    path: list[str]
    length: int
    root: bytes          # 32-byte pieces root (b"" for empty files)
    first_piece: int     # index of its first piece in the (piece-aligned) piece space
    num_pieces: int


@dataclass
class Info:
    name: str
    piece_length: int
    pieces: bytes                 # concatenated 20-byte SHA-1s (b"" for pure v2)
    files: list[FileEntry]
    multi: bool
    raw: bytes                    # exact bencoded info dict
    private: bool = False
    infohash: bytes = b""         # the 20-byte wire info-hash (v1 SHA-1, or truncated v2 SHA-256)
    v2_files: list[V2File] = field(default_factory=list)
    infohash_v2: bytes = b""      # full SHA-256 of the info dict (v2 / hybrid)
    piece_layers: dict = field(default_factory=dict)   # pieces root -> concatenated piece-layer hashes

    @property
    def has_v1(self) -> bool:
        return bool(self.pieces) or (not self.v2_files and self.total_length == 0)

    @property
    def has_v2(self) -> bool:
        return bool(self.v2_files)

    @property
    def total_length(self) -> int:
        return sum(f.length for f in self.files)

    @property
    def num_pieces(self) -> int:
        if self.pieces or not self.v2_files:
            return len(self.pieces) // 20
        return sum(f.num_pieces for f in self.v2_files)

    def piece_hash(self, i: int) -> bytes:
        return self.pieces[20 * i:20 * i + 20]

    def piece_size(self, i: int) -> int:
        if i == self.num_pieces - 1:
            rem = self.total_length - i * self.piece_length
            return rem
        return self.piece_length

    # -- v2 piece verification ------------------------------------------------
    def v2_piece(self, i: int) -> tuple[bytes | None, int, int]:
        """(expected hash or None if the piece layer is not known yet, tree
        width in leaves, real data bytes) of piece ``i`` of a v2 torrent."""
        lo, hi = 0, len(self.v2_files)
        while hi - lo > 1:                      # last file whose first piece <= i
            mid = (lo + hi) // 2
            if self.v2_files[mid].first_piece <= i:
                lo = mid
            else:
                hi = mid
        f = self.v2_files[lo]
        while f.num_pieces == 0 or i >= f.first_piece + f.num_pieces:
            lo += 1
            f = self.v2_files[lo]
        k = i - f.first_piece
        real = min(self.piece_length, f.length - k * self.piece_length)
        if f.num_pieces == 1:
            return f.root, merkle.next_pow2(-(-f.length // merkle.LEAF)), real
        layer = self.piece_layers.get(f.root)
        exp = layer[32 * k:32 * k + 32] if layer else None
        return exp, self.piece_length // merkle.LEAF, real

    def v2_expectations(self) -> tuple[bytes, list[int], list[int], list[int]]:
        """Batch form for the native verifiers: expected hashes (32 B each,
        zeros where unknown), tree widths, real lengths and a known-mask."""
        exp, widths, reals, known = bytearray(), [], [], []
        for i in range(self.num_pieces):
            e, w, r = self.v2_piece(i)
            exp += e if e is not None else bytes(32)
            widths.append(w)
            reals.append(r)
            known.append(e is not None)
        return bytes(exp), widths, reals, known

    def missing_layers(self) -> list[V2File]:
        return [f for f in self.v2_files if f.num_pieces > 1 and f.root not in self.piece_layers]

    def set_piece_layer(self, root: bytes, layer: bytes) -> bool:
        """Accept a piece layer only if it reduces to the file's root."""
        f = next((x for x in self.v2_files if x.root == root), None)
        if f is None or len(layer) != 32 * f.num_pieces:
            return False
        nodes = [layer[k:k + 32] for k in range(0, len(layer), 32)]
        if merkle.layer_root(nodes, self.piece_length) != root:
            return False
        self.piece_layers[root] = bytes(layer)
        return True

    def check_piece(self, i: int, data) -> bool | None:
        """Verify piece ``i``: SHA-1 for v1/hybrid, merkle for pure v2 (None
        when the v2 piece layer is not known yet)."""
        if self.pieces:
            return hashlib.sha1(data).digest() == self.piece_hash(i)
        exp, width, real = self.v2_piece(i)
        if exp is None:
            return None
        return _merkle_root(memoryview(data)[:real], width) == exp

    def matches(self, infohash: bytes) -> bool:
        return infohash in (self.infohash, self.infohash_v2, self.infohash_v2[:20]) and len(infohash) in (20, 32)

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
        """Parse a bencoded info dict (remote input: any malformation is a
        :class:`MetainfoError`, never another exception)."""
        try:
            d = bencode.decode(raw)
        except BencodeError as e:
            raise MetainfoError(f"bad info dict: {e}") from e
        if not isinstance(d, dict):
            raise MetainfoError("info is not a dict")
        if d.get(b"meta version") == 2 and b"pieces" not in d:
            return cls._parse_v2_only(d, raw)
        try:
            name = _safe_component(d[b"name"])
            plen = _bint(d[b"piece length"])
            pieces = _bbytes(d[b"pieces"])
        except (KeyError, TypeError, ValueError) as e:
            raise MetainfoError(f"info dict missing field: {e}") from e
        if plen <= 0 or len(pieces) % 20:
            raise MetainfoError("invalid piece length / pieces")
        v2_files: list[V2File] = []
        if d.get(b"meta version") == 2:
            v2_files = _parse_file_tree(d.get(b"file tree"), plen)
        files: list[FileEntry] = []
        off = 0
        try:
            if b"files" in d:
                multi = True
                for f in d[b"files"]:
                    path = [_safe_component(c) for c in f[b"path"]]
                    if not path:
                        raise MetainfoError("empty file path")
                    ln = _bint(f[b"length"])
                    if ln < 0:
                        raise MetainfoError("negative length")
                    attr = f.get(b"attr", b"")
                    files.append(FileEntry(path, ln, off, isinstance(attr, bytes) and b"p" in attr))
                    off += ln
            else:
                multi = False
                ln = _bint(d[b"length"])
                if ln < 0:
                    raise MetainfoError("negative length")
                files.append(FileEntry([name], ln, 0))
                off = ln
        except (KeyError, TypeError, ValueError, AttributeError) as e:   # remote input of any shape
            raise MetainfoError(f"bad file list: {type(e).__name__}: {e}") from e
        npieces = len(pieces) // 20
        if npieces != (off + plen - 1) // plen:
            raise MetainfoError(f"piece count {npieces} does not match total length {off}")
        info = cls(name, plen, pieces, files, multi, bytes(raw), bool(d.get(b"private", 0)),
                   hashlib.sha1(raw).digest())
        if v2_files:                                 # hybrid: v1 pieces drive verification
            real = [f for f in files if not f.pad]
            if [(f.path, f.length) for f in real] != [(v.path if multi else [name], v.length) for v in v2_files]:
                raise MetainfoError("hybrid torrent: v1 and v2 file lists differ")
            info.v2_files = v2_files
            info.infohash_v2 = hashlib.sha256(raw).digest()
        return info

    @classmethod
    def _parse_v2_only(cls, d: dict, raw: bytes) -> "Info":
        try:
            name = _safe_component(d[b"name"])
            plen = int(d[b"piece length"])
        except (KeyError, TypeError, ValueError) as e:
            raise MetainfoError(f"info dict missing field: {e}") from e
        v2 = _parse_file_tree(d.get(b"file tree"), plen)
        # single file: the tree is exactly {name: {"": ...}}
        multi = not (len(v2) == 1 and v2[0].path == [name])
        files: list[FileEntry] = []
        off = 0
        for k, v in enumerate(v2):
            files.append(FileEntry(v.path if multi else [name], v.length, off))
            off += v.length
            gap = (-v.length) % plen
            if gap and k < len(v2) - 1:              # virtual BEP 47 padding: next file on a piece boundary
                files.append(FileEntry([".pad", str(gap)], gap, off, True))
                off += gap
        h2 = hashlib.sha256(raw).digest()
        return cls(name, plen, b"", files, multi, bytes(raw), bool(d.get(b"private", 0)), h2[:20],
                   v2_files=v2, infohash_v2=h2)


def _parse_file_tree(tree, plen: int) -> list[V2File]:
    if not isinstance(tree, dict) or not tree:
        raise MetainfoError("v2 info has no file tree")
    try:
        merkle.piece_levels(plen)
    except ValueError as e:
        raise MetainfoError(str(e)) from e
    out: list[V2File] = []
    piece = 0

    def walk(node: dict, path: list[str], depth: int) -> None:
        nonlocal piece
        if depth > 64:
            raise MetainfoError("file tree too deep")
        for k in sorted(node):
            v = node[k]
            if not isinstance(v, dict):
                raise MetainfoError("bad file tree node")
            comp = _safe_component(k)
            if b"" in v and isinstance(v[b""], dict):
                leaf = v[b""]
                ln = leaf.get(b"length")
                if not isinstance(ln, int) or ln < 0:
                    raise MetainfoError("bad file length in file tree")
                root = leaf.get(b"pieces root", b"")
                if ln > 0 and (not isinstance(root, bytes) or len(root) != 32):
                    raise MetainfoError("file without a 32-byte pieces root")
                n = -(-ln // plen)
                out.append(V2File(path + [comp], ln, root if ln else b"", piece, n))
                piece += n
            else:
                walk(v, path + [comp], depth + 1)
    walk(tree, [], 0)
    return out


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
        layers = d.get(b"piece layers", {})
        if info.has_v2 and isinstance(layers, dict):
            for root, layer in layers.items():
                if isinstance(root, bytes) and isinstance(layer, bytes) and not info.set_piece_layer(root, layer):
                    raise MetainfoError("piece layer does not match its pieces root")
        return cls(info, tiers, nodes, url_list)

    def encode(self) -> bytes:
        d: dict = {b"info": _Raw(self.info.raw)}
        if self.announce:
            d[b"announce"] = self.announce[0][0].encode()
            d[b"announce-list"] = [[u.encode() for u in t] for t in self.announce]
        if self.url_list:
            d[b"url-list"] = [u.encode() for u in self.url_list]
        if self.info.piece_layers:
            d[b"piece layers"] = dict(self.info.piece_layers)
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
    infohash: bytes                  # 20-byte wire info-hash (btih, or truncated btmh)
    display_name: str = ""
    trackers: list[str] = field(default_factory=list)
    peers: list[tuple[str, int]] = field(default_factory=list)
    web_seeds: list[str] = field(default_factory=list)
    infohash_v2: bytes = b""         # full SHA-256 from ``xt=urn:btmh:1220...``
    has_v1: bool = True

    @property
    def hex(self) -> str:
        return self.infohash.hex()

    def uri(self) -> str:
        parts = [f"xt=urn:btih:{self.hex}"] if self.has_v1 else []
        if self.infohash_v2:
            parts.append(f"xt=urn:btmh:1220{self.infohash_v2.hex()}")
        if self.display_name:
            parts.append("dn=" + quote(self.display_name))
        parts += ["tr=" + quote(t, safe="") for t in self.trackers]
        parts += [f"x.pe=[{h}]:{p}" if ":" in h else f"x.pe={h}:{p}" for h, p in self.peers]
        parts += ["ws=" + quote(w, safe="") for w in self.web_seeds]
        return "magnet:?" + "&".join(parts)


def parse_magnet(uri: str) -> Magnet:
    u = urlparse(uri)
    if u.scheme != "magnet":
        raise MetainfoError(f"unsupported scheme '{u.scheme}'")
    q = parse_qs(u.query, keep_blank_values=True)
    ih = None
    ih2 = b""
    for xt in q.get("xt", []):
        if xt.lower().startswith("urn:btmh:"):
            mh = xt[9:]
            if not mh.lower().startswith("1220") or len(mh) != 68:
                raise MetainfoError("btmh must be a SHA-256 multihash (1220 + 64 hex)")
            ih2 = bytes.fromhex(mh[4:])
        elif xt.lower().startswith("urn:btih:"):
            h = xt[9:]
            if len(h) == 40:
                ih = bytes.fromhex(h)
            elif len(h) == 32:
                ih = base64.b32decode(h.upper())
            else:
                raise MetainfoError(f"bad btih length {len(h)}")
    has_v1 = ih is not None
    if ih is None and ih2:
        ih = ih2[:20]                # v2-only swarm: peers use the truncated SHA-256
    if ih is None:
        raise MetainfoError("magnet link has no urn:btih or urn:btmh")
    peers = []
    for pe in q.get("x.pe", []):
        host, _, port = pe.rpartition(":")
        if host and port.isascii() and port.isdigit() and 0 < int(port) < 65536:
            peers.append((host.strip("[]"), int(port)))
    return Magnet(ih, unquote(q.get("dn", [""])[0]), q.get("tr", []), peers, q.get("ws", []), ih2, has_v1)


# ----------------------------------------------------------------- create


def make_info(base: str, piece_length: int = 256 * 1024, name: str | None = None,
              private: bool = False, pad: bool = False, version: int = 1) -> Info:
    """Build an info dict for a file or directory (used by the test swarm).
    ``pad``: align every file to a piece boundary with BEP 47 padding files.
    ``version``: 1 (BEP 3), 2 (pure BEP 52) or 3 (hybrid v1+v2; implies
    ``pad``).  For v2/hybrid the returned Info carries its piece layers."""
    from ...ops import hashing
    if version not in (1, 2, 3):
        raise ValueError("version must be 1, 2 or 3 (hybrid)")
    if version != 1:
        try:
            merkle.piece_levels(piece_length)
        except ValueError as e:
            raise MetainfoError(str(e)) from e
        pad = True
    tname = name or os.path.basename(base.rstrip("/"))
    if os.path.isdir(base):
        entries = []
        for root, _dirs, fnames in os.walk(base):
            for fn in fnames:
                full = os.path.join(root, fn)
                rel = os.path.relpath(full, base).split(os.sep)
                entries.append((rel, full))
        entries.sort()
        multi = True
    else:
        entries = [([tname], base)]
        multi = False
    d: dict = {b"name": tname.encode(), b"piece length": piece_length}
    layers: dict[bytes, bytes] = {}
    if version != 1:
        tree: dict = {}
        for rel, f in entries:
            data = open(f, "rb").read()
            leaf: dict = {b"length": len(data)}
            if data:
                root, layer = merkle.file_root_and_layer(data, piece_length)
                leaf[b"pieces root"] = root
                if layer:
                    layers[root] = b"".join(layer)
            node = tree
            for c in rel[:-1]:
                node = node.setdefault(c.encode(), {})
            node[rel[-1].encode()] = {b"": leaf}
        d[b"file tree"] = tree
        d[b"meta version"] = 2
    if version != 2:
        files, layout = [], []
        for k, (rel, f) in enumerate(entries):
            n = os.path.getsize(f)
            files.append({b"length": n, b"path": [c.encode() for c in rel]})
            layout.append((f, n))
            if pad and k < len(entries) - 1 and n % piece_length:
                gap = piece_length - n % piece_length
                files.append({b"attr": b"p", b"length": gap, b"path": [b".pad", str(gap).encode()]})
                layout.append(("", gap))
        if multi:
            d[b"files"] = files
        else:
            d[b"length"] = layout[0][1]
        total = sum(n for _p, n in layout)
        blob = bytearray()
        for p, n in layout:
            if not p:
                blob += bytes(n)
                continue
            with open(p, "rb") as fh:
                blob += fh.read()
        d[b"pieces"] = hashing.piece_hashes(bytes(blob), piece_length, "sha1") if total else b""
    if private:
        d[b"private"] = 1
    info = Info.parse(bencode.encode(d))
    for root, layer in layers.items():
        if not info.set_piece_layer(root, layer):
            raise MetainfoError("internal: piece layer does not reduce to its root")
    return info
