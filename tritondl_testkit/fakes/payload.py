"""Synthetic job payloads that differ per job, and their content fingerprint.

The bench's origin used to serve one deterministic payload for every job, so
a worker that uploaded stale bytes (say a recycled spare file from the job
before, ``utils/spares.py``) could not be told from a correct one.  Here a
job's file name carries a *variant* (``movie-<i>-v<k>.mkv``): the origin
serves the base pseudo-random payload with every 4 KiB page stamped with
``k`` and the page index, and the S3 fake knows the variant's fingerprint
from the object key, so a PUT whose bytes are not the origin's fails.

Fingerprint (:func:`leaf_digest`): SHA-256 over the concatenated SHA-256s
of the payload's 64 KiB leaves — the aws-chunked client signs exactly those
leaves, so the S3 side gets the received leaf hashes free from its chunk
signature check (``csrc/relay/relay_core.h``, ``VerifyResult.leaf_hashes``).
"""

from __future__ import annotations

import functools
import hashlib
import re

import numpy as np

LEAF = 64 * 1024
_VARIANT = re.compile(r"-v(\d+)\.[^./]*$")


@functools.lru_cache(maxsize=4)
def synthetic_bytes(size: int, seed: int = 1234) -> bytes:
    return np.random.default_rng(seed).integers(0, 256, size, dtype=np.uint8).tobytes()


def variant_bytes(size: int, variant: int | None) -> bytes:
    """The base payload with each whole 4 KiB page's first 16 bytes replaced
    by (variant, page index, a variant-keyed constant): every page of two
    variants differs."""
    base = synthetic_bytes(size)
    if variant is None:
        return base
    a = np.frombuffer(base, dtype=np.uint8).copy()
    pages = size // 4096
    if pages:
        v = a[: pages * 4096].view("<u8").reshape(pages, 512)
        v[:, 0] = (np.uint64(variant) << np.uint64(40)) | np.arange(pages, dtype=np.uint64)
        v[:, 1] = np.uint64((0x9E3779B97F4A7C15 * (variant + 1)) & 0xFFFFFFFFFFFFFFFF)
    tail = size - pages * 4096
    if tail:
        a[pages * 4096:] ^= np.uint8((variant * 37 + 11) & 0xFF)
    return a.tobytes()


def variant_of(name: str) -> int | None:
    """``movie-12-v7.mkv`` -> 7; None for names without a variant."""
    m = _VARIANT.search(name)
    return int(m.group(1)) if m else None


def leaf_hashes(data) -> bytes:
    """SHA-256 of each 64 KiB leaf, concatenated (native multi-buffer kernel)."""
    from tritondl.ops import hashing
    return hashing.piece_hashes(data, LEAF, kind="sha256") if len(data) else b""


def leaf_digest(data) -> bytes:
    return hashlib.sha256(leaf_hashes(data)).digest()


class Expectations:
    """Expected fingerprints of the variants of one payload size (computed on
    first use, or all up front with :meth:`precompute`)."""

    def __init__(self, size: int, variants: int) -> None:
        self.size = size
        self.variants = variants
        self._digest: dict[int, bytes] = {}

    def precompute(self) -> None:
        for k in range(self.variants):
            self.get(k)

    def get(self, variant: int) -> bytes:
        d = self._digest.get(variant)
        if d is None:
            d = self._digest[variant] = leaf_digest(variant_bytes(self.size, variant))
        return d

    def expected_for_key(self, key: str, size: int) -> bytes | None:
        """For an object key ``<media id>/original/<base64(file name)>``
        (``uploader.go:86-89``) or a plain file name."""
        import base64
        import binascii
        # the std alphabet can put "/" inside the encoded name
        last = key.split("/original/", 1)[1] if "/original/" in key else key.rsplit("/", 1)[-1]
        try:
            name = base64.b64decode(last, validate=True).decode()
        except (binascii.Error, UnicodeDecodeError, ValueError):
            name = last
        return self.expected(name, size)

    def expected(self, name: str, size: int) -> bytes | None:
        """The fingerprint a PUT of file ``name`` with ``size`` bytes must have
        (None: not a synthetic variant of this size — nothing to check)."""
        k = variant_of(name)
        if k is None or size != self.size:
            return None
        return self.get(k)
