"""BitTorrent v2 (BEP 52) merkle trees — reference implementation.

Every file is hashed on its own: SHA-256 of each 16 KiB block is a leaf; the
leaf row is padded with all-zero 32-byte hashes up to a power of two and
reduced pairwise with SHA-256 to the file's ``pieces root``.  For files longer
than one piece, the nodes whose subtrees cover exactly ``piece length`` bytes
form the *piece layer* (shipped in the torrent's ``piece layers``); a piece is
verified against its piece-layer node.  A file of at most one piece is
verified against its root, whose tree is only ``next_pow2(blocks)`` leaves
wide.

This module is the executable spec the native paths are tested against:
``_hash_host.merkle_verify`` (threaded C++) and the HIP leaf kernel
(``GpuHasher.digest_files`` at 16 KiB) + host reduction.
"""

from __future__ import annotations

import hashlib

LEAF = 16 * 1024
ZERO = bytes(32)
_pad_cache: list[bytes] = [ZERO]


def pad_hash(level: int) -> bytes:
    """Root of an all-padding subtree ``level`` layers above the leaves."""
    while len(_pad_cache) <= level:
        h = _pad_cache[-1]
        _pad_cache.append(hashlib.sha256(h + h).digest())
    return _pad_cache[level]


def next_pow2(n: int) -> int:
    return 1 if n <= 1 else 1 << (n - 1).bit_length()


def leaf_hashes(data: bytes | memoryview) -> list[bytes]:
    mv = memoryview(data)
    return [hashlib.sha256(mv[k:k + LEAF]).digest() for k in range(0, len(mv), LEAF)]


def reduce(nodes: list[bytes], width: int, level: int = 0) -> bytes:
    """Root of ``nodes`` (at ``level``) padded to ``width`` entries with the
    all-padding hash of that level."""
    if width & (width - 1):
        raise ValueError("width must be a power of two")
    if len(nodes) > width:
        raise ValueError("more nodes than the tree is wide")
    row = list(nodes) + [pad_hash(level)] * (width - len(nodes))
    while len(row) > 1:
        row = [hashlib.sha256(row[k] + row[k + 1]).digest() for k in range(0, len(row), 2)]
        level += 1
    return row[0]


def piece_levels(piece_length: int) -> int:
    n = piece_length // LEAF
    if piece_length % LEAF or n & (n - 1):
        raise ValueError("v2 piece length must be a power of two >= 16 KiB")
    return n.bit_length() - 1


def file_root_and_layer(data: bytes, piece_length: int) -> tuple[bytes, list[bytes]]:
    """(pieces root, piece layer) of one file; the layer is empty for files
    of at most one piece (BEP 52 omits them from ``piece layers``)."""
    if not data:
        raise ValueError("empty files have no pieces root")
    leaves = leaf_hashes(data)
    per = piece_length // LEAF
    if len(data) <= piece_length:
        return reduce(leaves, next_pow2(len(leaves))), []
    layer = [reduce(leaves[k:k + per], per) for k in range(0, len(leaves), per)]
    lv = piece_levels(piece_length)
    return reduce(layer, next_pow2(len(layer)), lv), layer


def piece_root(data: bytes, width: int) -> bytes:
    """Merkle root over one piece's data with a ``width``-leaf tree."""
    return reduce(leaf_hashes(data), width)


def layer_root(layer: list[bytes], piece_length: int) -> bytes:
    """Root implied by a piece layer (to check ``piece layers`` entries)."""
    return reduce(layer, next_pow2(len(layer)), piece_levels(piece_length))


# -- BEP 52 hash requests: a slice of one layer plus its uncle-hash proof ------


def layer_rows(layer: list[bytes], level: int) -> list[list[bytes]]:
    """Every row of the tree from ``layer`` (at ``level``) up to the root,
    padded to a power of two with the all-padding hash of each level."""
    width = next_pow2(len(layer))
    rows = [list(layer) + [pad_hash(level)] * (width - len(layer))]
    while len(rows[-1]) > 1:
        r = rows[-1]
        rows.append([hashlib.sha256(r[k] + r[k + 1]).digest() for k in range(0, len(r), 2)])
    return rows


def serve_hashes(layer: list[bytes], level: int, index: int, length: int, proofs: int) -> bytes | None:
    """Answer a hash request against a full piece layer: ``length`` hashes
    from ``index`` (padded), then ``proofs`` uncle hashes bottom-up starting
    at the layer above the requested slice.  None if the request is invalid."""
    rows = layer_rows(layer, level)
    if length < 1 or length & (length - 1) or index % length or index + length > len(rows[0]):
        return None
    out = b"".join(rows[0][index:index + length])
    h = length.bit_length() - 1          # rows[h] holds the slice's subtree root
    node = index >> h
    for k in range(proofs):
        row = h + k
        if row >= len(rows) - 1:
            break
        out += rows[row][node ^ 1]
        node >>= 1
    return out


def check_hashes(root: bytes, level: int, index: int, length: int, hashes: bytes, n_layer: int) -> list[bytes] | None:
    """Verify a hashes response: the ``length`` layer hashes plus uncle
    proofs must reduce to ``root``.  ``n_layer`` is the file's number of
    pieces (the layer's unpadded length).  Returns the layer slice or None."""
    if length < 1 or length & (length - 1) or index % length or len(hashes) < 32 * length or len(hashes) % 32:
        return None
    nodes = [hashes[32 * k:32 * k + 32] for k in range(length)]
    uncles = [hashes[32 * k:32 * k + 32] for k in range(length, len(hashes) // 32)]
    total_h = next_pow2(n_layer).bit_length() - 1
    h = length.bit_length() - 1
    if h > total_h or len(uncles) != total_h - h:
        return None
    row = nodes
    while len(row) > 1:
        row = [hashlib.sha256(row[k] + row[k + 1]).digest() for k in range(0, len(row), 2)]
    node, pos = row[0], index >> h
    for u in uncles:
        node = hashlib.sha256(node + u).digest() if pos % 2 == 0 else hashlib.sha256(u + node).digest()
        pos >>= 1
    return nodes if node == root else None
