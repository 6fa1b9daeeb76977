"""AWS Signature Version 4 for S3 — written from the SigV4 specification.

The reference delegates this to minio-go v6 (``internal/uploader/uploader.go:43-51,89``;
SURVEY.md Appendix C).  Payload modes supported, selected like minio-go:

* ``UNSIGNED-PAYLOAD``                      – over TLS
* ``STREAMING-AWS4-HMAC-SHA256-PAYLOAD``    – over plain HTTP (aws-chunked,
  64 KiB chunks, each chunk signed; single read pass over the file)
* hex SHA-256 of the payload                – small bodies / explicit choice

HMAC/SHA-256 of chunk chains run in the native C++ module (OpenSSL SHA-NI).
"""

from __future__ import annotations

import datetime as _dt
import functools
import hashlib
import hmac
import os
import re
from dataclasses import dataclass
from urllib.parse import quote

from ..ops import hashing

ALGO = "AWS4-HMAC-SHA256"
UNSIGNED_PAYLOAD = "UNSIGNED-PAYLOAD"
STREAMING_PAYLOAD = "STREAMING-AWS4-HMAC-SHA256-PAYLOAD"
EMPTY_SHA256 = hashlib.sha256(b"").hexdigest()
# aws-chunked payload chunk: minio-go's 64 KiB (TRITONDL_S3_CHUNK_KB: 8 KiB and up, any size S3 accepts)
STREAM_CHUNK = max(8, int(os.environ.get("TRITONDL_S3_CHUNK_KB", "64"))) * 1024
SIGN_THREADS = 4


_PLAIN = re.compile(r"[A-Za-z0-9\-_.~]*")
_PLAIN_PATH = re.compile(r"[A-Za-z0-9\-_.~/]*")


def uri_encode(s: str, encode_slash: bool = True) -> str:
    """AWS UriEncode: unreserved = A-Za-z0-9-._~ ; uppercase hex escapes.
    Strings with nothing to escape (most object keys) skip ``quote``."""
    if (_PLAIN if encode_slash else _PLAIN_PATH).fullmatch(s):
        return s
    return quote(s, safe="-_.~" if encode_slash else "-_.~/")


def canonical_query(params: dict | list | None) -> str:
    if not params:
        return ""
    items = params.items() if isinstance(params, dict) else params
    enc = sorted((uri_encode(str(k)), uri_encode("" if v is None else str(v))) for k, v in items)
    return "&".join(f"{k}={v}" for k, v in enc)


def _trim(v: str) -> str:
    return " ".join(str(v).strip().split())


@functools.lru_cache(maxsize=16)
def signing_key(secret: str, date: str, region: str, service: str = "s3") -> bytes:
    """The derived key changes once a day per credential and region (four
    HMACs per request otherwise), so it is cached."""
    k = hmac.new(("AWS4" + secret).encode(), date.encode(), hashlib.sha256).digest()
    k = hmac.new(k, region.encode(), hashlib.sha256).digest()
    k = hmac.new(k, service.encode(), hashlib.sha256).digest()
    return hmac.new(k, b"aws4_request", hashlib.sha256).digest()


@dataclass
class Signed:
    authorization: str
    signature: str
    signed_headers: str
    canonical_request: str
    string_to_sign: str
    scope: str
    amzdate: str
    key: bytes


def amz_dates(now: _dt.datetime | None = None) -> tuple[str, str]:
    now = now or _dt.datetime.now(_dt.timezone.utc)
    amzdate = now.strftime("%Y%m%dT%H%M%SZ")
    return amzdate, amzdate[:8]


def sign(method: str, path: str, query: dict | list | None, headers: dict[str, str], payload_hash: str,
         access_key: str, secret_key: str, region: str, amzdate: str, service: str = "s3",
         path_is_encoded: bool = False) -> Signed:
    """Compute the SigV4 signature.  ``headers`` must already contain ``host``,
    ``x-amz-date`` and ``x-amz-content-sha256`` (all are signed)."""
    date = amzdate[:8]
    hdrs = {k.lower(): _trim(v) for k, v in headers.items()}
    names = sorted(hdrs)
    canon_headers = "".join(f"{n}:{hdrs[n]}\n" for n in names)
    signed_headers = ";".join(names)
    canon_uri = path if path_is_encoded else uri_encode(path or "/", encode_slash=False)
    creq = "\n".join([method.upper(), canon_uri, canonical_query(query), canon_headers, signed_headers,
                      payload_hash])
    scope = f"{date}/{region}/{service}/aws4_request"
    sts = "\n".join([ALGO, amzdate, scope, hashlib.sha256(creq.encode()).hexdigest()])
    key = signing_key(secret_key, date, region, service)
    sig = hmac.new(key, sts.encode(), hashlib.sha256).hexdigest()
    auth = f"{ALGO} Credential={access_key}/{scope}, SignedHeaders={signed_headers}, Signature={sig}"
    return Signed(auth, sig, signed_headers, creq, sts, scope, amzdate, key)


# ----------------------------------------------------------- aws-chunked


def chunked_length(decoded: int, chunk: int = STREAM_CHUNK) -> int:
    """Content-Length of an aws-chunked body carrying ``decoded`` bytes."""
    sig_part = len(";chunk-signature=") + 64 + 2  # + CRLF
    full, rem = divmod(decoded, chunk)
    n = full * (len(f"{chunk:x}") + sig_part + chunk + 2)
    if rem:
        n += len(f"{rem:x}") + sig_part + rem + 2
    n += 1 + sig_part + 2  # final "0;chunk-signature=...\r\n\r\n"
    return n


class ChunkSigner:
    """Incremental aws-chunked encoder: feed data blocks (any size), get
    encoded bytes; ``finish()`` emits the trailing zero-length chunk."""

    def __init__(self, key: bytes, amzdate: str, scope: str, seed_signature: str, chunk: int = STREAM_CHUNK,
                 threads: int = SIGN_THREADS):
        self.threads = threads
        self.key = key
        self.amzdate = amzdate
        self.scope = scope
        self.prev = seed_signature
        self.chunk = chunk
        self._buf = bytearray()

    def _encode(self, data, final: bool) -> bytes:
        out, self.prev = hashing.aws_chunk_encode(self.key, self.amzdate, self.scope, self.prev, data,
                                                  self.chunk, final, self.threads)
        return out

    def feed(self, data: bytes) -> bytes:
        """Encode every whole chunk available; keep the remainder buffered."""
        if self._buf:
            self._buf += data
            data = bytes(self._buf)
            self._buf.clear()
        n = len(data)
        full = n - n % self.chunk
        out = self._encode(memoryview(data)[:full], False) if full else b""
        if full < n:
            self._buf += memoryview(data)[full:]
        return out

    def finish(self) -> bytes:
        """Encode the buffered tail (one short chunk) plus the final empty chunk."""
        rest = bytes(self._buf)
        self._buf.clear()
        return self._encode(rest, True)
