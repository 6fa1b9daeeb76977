"""Async S3 client (aiohttp) with SigV4, bucket ensure, streaming PutObject
and parallel multipart upload.

Capability of the minio-go v6 calls the reference makes
(``internal/uploader/uploader.go:43-51,64-65,89``): ``NewWithOptions{Secure,
Creds, BucketLookupAuto}``, ``BucketExists``, ``MakeBucket``,
``PutObjectWithContext`` (single PUT below the multipart threshold, multipart
above it).  Memory stays O(part_size × parallel_parts) regardless of file
size; file reads and chunk signing run in worker threads
(the native hash module releases the GIL), so several uploads overlap.

minio-go library behaviours the reference relied on without naming them:

* no Region in ``NewWithOptions`` (``uploader.go:43-51``) means minio looks
  the bucket's region up (``GET /<bucket>?location``, cached per bucket) and
  signs with it; a reply of ``AuthorizationHeaderMalformed`` /
  ``InvalidRegion`` / a 301 naming ``x-amz-bucket-region`` re-signs with the
  region S3 names (:meth:`S3Client.bucket_region`);
* ``PutObject`` sizes parts so an object never needs more than 10,000 parts
  and refuses objects over 5 TiB (minio ``optimalPartInfo``; :func:`plan_parts`);
* an empty or malformed endpoint is an error when the client is built
  (minio ``NewWithOptions`` → ``log.Fatal`` in ``downloader.go:95-98``;
  :meth:`Endpoint.parse`);
* every request is retried on connection errors, on 429/500/502/503 (and
  504) and on minio's retryable S3 codes (``RequestTimeout``, ``SlowDown``,
  ``ExpiredToken``, ... :data:`RETRYABLE_CODES`), up to 10 attempts spaced
  1 s × 2^k up to 30 s (minio ``retry.go``; :meth:`S3Client.retry_delay`),
  so a throttling burst or a MinIO rolling restart of a minute or two does
  not fail the job.
"""

from __future__ import annotations

import asyncio
import calendar
import contextlib
import datetime as _dt
import email.utils
import hashlib
import json
import os
import random
import re
import time
import xml.etree.ElementTree as ET
from dataclasses import dataclass
from typing import AsyncIterator
from urllib.parse import urlparse

import aiohttp
from multidict import CIMultiDict
from yarl import URL

from ..ops import hashing
from ..utils import proxy as _proxy
from ..utils import rawhttp
from ..utils.dial import FALLBACK_DELAY, socket_factory
from ..utils.log import log
from . import sigv4
from .credentials import Chain, Provider, Value, default_chain

S3_NS = "{http://s3.amazonaws.com/doc/2006-03-01/}"
_DNS_BUCKET = re.compile(r"^[a-z0-9][a-z0-9.-]{1,61}[a-z0-9]$")
_HOST = re.compile(r"^(?:[A-Za-z0-9](?:[A-Za-z0-9-]{0,61}[A-Za-z0-9])?)(?:\.[A-Za-z0-9](?:[A-Za-z0-9-]{0,61}[A-Za-z0-9])?)*$")

# S3 limits (minio-go constants.go): parts per upload, object / part / single-PUT sizes
MAX_PARTS = 10000
MIN_PART_SIZE = 5 << 20
MAX_PART_SIZE = 5 << 30
MAX_SINGLE_PUT = 5 << 30
MAX_OBJECT_SIZE = 5 << 40
DEFAULT_REGION = "us-east-1"
_REGION_CODES = ("AuthorizationHeaderMalformed", "InvalidRegion", "PermanentRedirect", "IllegalLocationConstraintException")


# minio-go v6's retry classifier (retry.go: retryableS3Codes, retryableHTTPStatusCodes),
# which every reference S3 call went through (internal/uploader/uploader.go:43-51,64-65,89);
# 504 is retried as well (a gateway in front of the store timing out).
RETRYABLE_CODES = frozenset({"RequestError", "RequestTimeout", "Throttling", "ThrottlingException",
                             "RequestLimitExceeded", "RequestThrottled", "InternalError", "ExpiredToken",
                             "ExpiredTokenException", "SlowDown"})
RETRYABLE_STATUS = frozenset({429, 500, 502, 503, 504})


def is_retryable(err: "S3Error") -> bool:
    """Worth another attempt: a retryable status or S3 error code.  Any other
    4xx, and 501 NotImplemented, fail at once."""
    return err.status in RETRYABLE_STATUS or err.code in RETRYABLE_CODES


class S3Error(Exception):
    def __init__(self, status: int, code: str = "", message: str = "", resource: str = "",
                 region: str = "") -> None:
        super().__init__(f"S3 {status} {code}: {message} ({resource})")
        self.status, self.code, self.message, self.resource = status, code, message, resource
        self.region = region          # the bucket's region when S3 names it (XML <Region> / x-amz-bucket-region)
        self.server_time: float | None = None   # RequestTimeTooSkewed: S3's clock (epoch s)


def _xml(body: bytes, what: str) -> ET.Element:
    """The root of a 2xx reply's XML body; a body that is not XML is an
    S3Error (MalformedXML), like any other failed request."""
    try:
        return ET.fromstring(body)
    except ET.ParseError as e:
        raise S3Error(0, "MalformedXML", f"unparsable {what} reply: {e}") from e


def _server_time(xml_time: str, date_header: str) -> float | None:
    """S3's clock from a RequestTimeTooSkewed reply: ``<ServerTime>``
    (ISO 8601, AWS) or else the ``Date`` header (RFC 7231, minio and AWS)."""
    if xml_time:
        with contextlib.suppress(ValueError):
            return calendar.timegm(time.strptime(xml_time.split(".")[0].rstrip("Z"), "%Y-%m-%dT%H:%M:%S"))
    if date_header:
        with contextlib.suppress(TypeError, ValueError):
            return email.utils.parsedate_to_datetime(date_header).timestamp()
    return None


def _parse_error(status: int, body: bytes, resource: str, headers=None) -> S3Error:
    code = msg = region = stime = ""
    if body:
        try:
            root = ET.fromstring(body)
            code = (root.findtext("Code") or "")
            msg = (root.findtext("Message") or "")
            region = (root.findtext("Region") or "")
            stime = (root.findtext("ServerTime") or "")
        except ET.ParseError:
            msg = body[:200].decode(errors="replace")
    if headers is not None:
        region = region or headers.get("x-amz-bucket-region", "") or ""
    if not code:     # HEAD replies carry no body: name the error like minio does
        code = {301: "PermanentRedirect", 400: "BadRequest", 403: "AccessDenied", 404: "NoSuchBucket" if
                resource.count("/") <= 1 and "?" not in resource else "NoSuchKey"}.get(status, "")
    err = S3Error(status, code, msg, resource, region)
    if code == "RequestTimeTooSkewed" or status in (401, 403):
        # a HEAD's 403 has no body to name the skew: S3's Date header still tells its clock
        err.server_time = _server_time(stime, (headers.get("Date", "") or "") if headers is not None else "")
    return err


def multipart_etag(part_etags: list[str]) -> str:
    """The ETag S3 gives a multipart object: hex MD5 over the concatenated
    binary part MD5s, then ``-<parts>``.  "" when a part ETag is not a plain
    MD5 (SSE-KMS / SSE-C parts), where nothing can be predicted."""
    raw = []
    for e in part_etags:
        e = e.strip('"')
        if len(e) != 32:
            return ""
        try:
            raw.append(bytes.fromhex(e))
        except ValueError:
            return ""
    if not raw:
        return ""
    return hashlib.md5(b"".join(raw)).hexdigest() + f"-{len(raw)}"


def _proxy_auth_error(px, resource: str, status: int = 407, detail: str = "") -> S3Error:
    """A proxy that refuses this client: not retried (another try cannot pass)."""
    who = px.redacted() if px is not None else "the proxy"
    return S3Error(status, "ProxyAuthenticationRequired" if status == 407 else "ProxyRefused",
                   detail or f"{who} refused the request ({status})", resource)


def _save_json(path: str, obj: dict) -> None:
    tmp = path + ".tmp"
    with contextlib.suppress(OSError):
        with open(tmp, "w") as f:
            json.dump(obj, f)
        os.replace(tmp, path)


def plan_parts(size: int, part_size: int) -> tuple[int, int]:
    """(part size, part count) for a multipart upload of ``size`` bytes.

    minio-go ``optimalPartInfo``: the smallest multiple of the configured part
    size that keeps the upload within 10,000 parts; objects over 5 TiB are
    refused before any byte is sent."""
    if size > MAX_OBJECT_SIZE:
        raise S3Error(0, "EntityTooLarge", f"object of {size} bytes exceeds the 5 TiB S3 maximum")
    base = max(part_size, MIN_PART_SIZE)
    need = -(-size // MAX_PARTS)
    ps = base if need <= base else -(-need // base) * base
    ps = min(ps, MAX_PART_SIZE)
    return ps, max(1, -(-size // ps))


@dataclass
class Endpoint:
    host: str           # host[:port] as sent in the Host header
    secure: bool

    @classmethod
    def parse(cls, s3_endpoint: str) -> "Endpoint":
        """Reference parsing of ``S3_ENDPOINT`` (``uploader.go:25-40``): TLS iff
        scheme is https; keep hostname[:port].  An endpoint minio-go would
        refuse (empty, no host, bad host or port) raises ``ValueError``."""
        raw = s3_endpoint or ""
        if raw.strip() == "":
            raise ValueError("S3_ENDPOINT is empty: endpoint url cannot be empty")
        if "://" not in raw:
            raw = "http://" + raw  # bare host[:port] (Go would yield an empty host)
        u = urlparse(raw)
        if u.scheme not in ("http", "https"):
            raise ValueError(f"S3_ENDPOINT {s3_endpoint!r}: scheme must be http or https")
        host = u.hostname or ""
        try:
            port = u.port
        except ValueError as e:
            raise ValueError(f"S3_ENDPOINT {s3_endpoint!r}: invalid port") from e
        if not host:
            raise ValueError(f"S3_ENDPOINT {s3_endpoint!r}: no host")
        if ":" in host:                 # IPv6 literal
            try:
                import ipaddress
                ipaddress.IPv6Address(host)
            except ValueError as e:
                raise ValueError(f"S3_ENDPOINT {s3_endpoint!r}: invalid host") from e
            host = f"[{host}]"
        elif not _HOST.match(host):
            raise ValueError(f"S3_ENDPOINT {s3_endpoint!r}: {host!r} is not a valid domain name or ip address")
        if u.path not in ("", "/"):
            raise ValueError(f"S3_ENDPOINT {s3_endpoint!r}: endpoint url cannot have a path")
        if port:
            host = f"{host}:{port}"
        return cls(host, u.scheme == "https")

    @property
    def base(self) -> str:
        return ("https://" if self.secure else "http://") + self.host


class S3Client:
    def __init__(self, endpoint: Endpoint | str, creds: Provider | None = None, *, region: str = "",
                 lookup: str = "auto", payload_mode: str = "auto", part_size: int = 64 << 20,
                 multipart_threshold: int = 64 << 20, parallel_parts: int = 4, max_retries: int = 9,
                 retry_unit: float = 1.0, retry_cap: float = 30.0,
                 io_block: int = 4 << 20, session: aiohttp.ClientSession | None = None,
                 native: bool = True, sign_threads: int = 4, ca_pem: str = "", ca_file: str = "",
                 proxies: "_proxy.ProxyConfig | None" = None, hash_device: str = "cpu") -> None:
        self.ep = Endpoint.parse(endpoint) if isinstance(endpoint, str) else endpoint
        # "gpu": aws-chunked chunk SHA-256s on the HIP kernel (plain-http native PUTs);
        # fails loudly at the first PUT if the GPU module or a device is missing
        if hash_device not in ("cpu", "gpu"):
            raise ValueError(f"hash_device must be cpu|gpu, got {hash_device!r}")
        self.hash_device = hash_device
        self._gpu_api = None
        # egress proxy (minio-go's DefaultTransport: ProxyFromEnvironment); None = the environment
        self.proxies = proxies
        self.creds = creds or default_chain()
        self.region = region            # "" = discover each bucket's region (minio-go without Region)
        self._regions: dict[str, str] = {}
        self.clock_skew = 0.0               # seconds S3's clock is ahead of this host's (learned)
        self.lookup = lookup
        self.payload_mode = payload_mode
        self.part_size = max(part_size, 5 << 20)
        self.multipart_threshold = multipart_threshold
        self.parallel_parts = max(1, parallel_parts)
        # minio-go's budget (retry.go: MaxRetry 10 attempts, DefaultRetryUnit 1 s, DefaultRetryCap
        # 30 s): a request is tried up to max_retries + 1 times, waiting unit * 2^k (capped)
        # between tries, half of it jittered (minio-go jitters all of it: "equal" jitter keeps
        # the herd spread and guarantees the budget rides out an outage of about a minute)
        self.max_retries = max_retries
        self.retry_unit = retry_unit
        self.retry_cap = retry_cap
        self.io_block = max(io_block, sigv4.STREAM_CHUNK)
        self._session = session
        self._own_session = session is None
        # native data plane (csrc/relay): file/fd PUT bodies over plain http
        self.native = native
        self.sign_threads = sign_threads
        self._raw = rawhttp.Pool()
        # TLS trust for https endpoints: a private CA (PEM text / file), else the system store
        self.ca_pem, self.ca_file = ca_pem, ca_file or os.environ.get("TRITONDL_CA_FILE", "")
        self._ntls = None

    def _ssl(self):
        """Python ``ssl`` context for the aiohttp control requests (None = default)."""
        if not (self.ep.secure and (self.ca_pem or self.ca_file)):
            return None
        import ssl
        ctx = ssl.create_default_context(cafile=self.ca_file or None, cadata=self.ca_pem or None)
        return ctx

    def _tls_ctx(self, force: bool = False):
        """Native client TLS context for the relay pumps (None for plain http
        unless ``force``: an https proxy in front of a plain endpoint)."""
        if not (self.ep.secure or force):
            return None
        if self._ntls is None:
            relay = rawhttp.relay_module()
            if self.ca_pem and relay is not None:
                self._ntls = relay.TlsContext.client(ca_pem=self.ca_pem)
            else:
                self._ntls = rawhttp.client_tls_context(self.ca_file)
        return self._ntls

    async def _sess(self) -> aiohttp.ClientSession:
        if self._session is None or self._session.closed:
            ssl_ctx = self._ssl()
            self._session = aiohttp.ClientSession(
                timeout=aiohttp.ClientTimeout(total=None, sock_connect=30, sock_read=300),
                connector=aiohttp.TCPConnector(limit=64, ssl=ssl_ctx if ssl_ctx is not None else True,
                                             happy_eyeballs_delay=FALLBACK_DELAY, socket_factory=socket_factory),
                auto_decompress=False)
            self._own_session = True
        return self._session

    async def close(self) -> None:
        self._raw.close()
        if self._own_session and self._session is not None:
            await self._session.close()
            self._session = None

    # ------------------------------------------------------------ helpers
    def _virtual(self, bucket: str) -> bool:
        if self.lookup == "dns":
            return True
        if self.lookup == "path" or not bucket:
            return False
        host = self.ep.host.split(":")[0]
        # BucketLookupAuto: virtual-host style for AWS / Aliyun style endpoints only
        return (host.endswith("amazonaws.com") or host.endswith("aliyuncs.com")) and \
            bool(_DNS_BUCKET.match(bucket)) and "." not in bucket

    def _target(self, bucket: str, key: str = "", path_style: bool = False) -> tuple[str, str]:
        ekey = sigv4.uri_encode(key, encode_slash=False) if key else ""
        if not path_style and self._virtual(bucket):
            return f"{bucket}.{self.ep.host}", "/" + ekey
        path = "/" + bucket if bucket else "/"
        if key:
            path += "/" + ekey
        return self.ep.host, path

    def _payload_mode(self) -> str:
        if self.payload_mode != "auto":
            return self.payload_mode
        return "unsigned" if self.ep.secure else "streaming"

    def _creds(self) -> Value:
        return self.creds.retrieve()

    def _chunk_gpu(self):
        """The HIP chunk-hashing API for the send pump (``hash_device="gpu"``)."""
        if self.hash_device != "gpu":
            return None
        if self._gpu_api is None:
            try:
                mod = hashing.gpu_module()
                ok = mod.device_count() > 0
            except Exception:  # noqa: BLE001 - reported below
                ok = False
            if not ok:
                raise S3Error(0, "GPUUnavailable", "TRITONDL_S3_HASH_DEVICE=gpu but no HIP device / _gpu_hash module")
            self._gpu_api = mod.chunk_api(hashing.default_device())
        return self._gpu_api

    def _proxy(self, host: str) -> "_proxy.ProxyURL | None":
        """The egress proxy for requests to ``host`` (the endpoint, or a
        virtual-host bucket name under it), chosen as Go's
        ``ProxyFromEnvironment`` chooses it for minio-go's request URL."""
        url = f"{'https' if self.ep.secure else 'http'}://{host}/"
        try:
            return (self.proxies or _proxy.from_environment()).proxy_for(url)
        except _proxy.ProxyConfigError as e:
            raise S3Error(0, "ProxyConfig", str(e), host) from e

    def _aio_proxy(self, host: str, headers: dict) -> dict:
        """aiohttp request kwargs (``headers`` included) through the proxy of ``host``."""
        try:
            kw, extra = _proxy.aiohttp_kwargs(self._proxy(host), self.ep.secure)
        except ValueError as e:
            raise S3Error(0, "ProxyUnsupported", str(e), host) from e
        return {**kw, "headers": {**headers, **extra}}

    # ------------------------------------------------------------ regions
    async def bucket_region(self, bucket: str) -> str:
        """Signing region for ``bucket``: the configured one, else the cached
        ``GET ?location`` answer (minio-go ``getBucketLocation``)."""
        if self.region:
            return self.region
        if not bucket:
            return DEFAULT_REGION
        r = self._regions.get(bucket)
        if r is not None:
            return r
        try:
            _st, _h, body = await self._do("GET", bucket, query={"location": ""}, region=DEFAULT_REGION,
                                           path_style=True)
            loc = ""
            try:
                root = ET.fromstring(body)
                loc = (root.text or "").strip()
            except ET.ParseError:
                pass
            r = {"": DEFAULT_REGION, "EU": "eu-west-1"}.get(loc, loc)
        except S3Error as e:
            # minio: access-denied / wrong-region replies still name a usable region
            if e.code in _REGION_CODES + ("AccessDenied",):
                r = e.region or DEFAULT_REGION
            elif e.code == "NoSuchBucket":
                return DEFAULT_REGION       # not cached: the bucket may be created next
            else:
                raise
        self._regions[bucket] = r
        return r

    def forget_bucket(self, bucket: str) -> None:
        """Drop cached facts about ``bucket`` (deleted / recreated elsewhere)."""
        self._regions.pop(bucket, None)

    def _learn_region(self, bucket: str, err: S3Error, used: str) -> bool:
        """True when ``err`` says the request was signed for the wrong region and
        names the right one (cached; the caller re-signs without counting a try)."""
        if self.region or not bucket or not err.region or err.region == used:
            return False
        if err.code in _REGION_CODES or err.status in (301, 400):
            log.with_fields(bucket=bucket, region=err.region).info("bucket region discovered")
            self._regions[bucket] = err.region
            return True
        return False

    def retry_delay(self, attempt: int) -> float:
        """Wait after failed attempt number ``attempt`` (1-based)."""
        d = min(self.retry_cap, self.retry_unit * (2.0 ** min(attempt - 1, 30)))
        return d / 2 + random.uniform(0.0, d / 2)

    def _amzdate(self) -> str:
        """``x-amz-date`` on S3's clock: the host's plus the learned skew."""
        now = _dt.datetime.now(_dt.timezone.utc)
        if self.clock_skew:
            now += _dt.timedelta(seconds=self.clock_skew)
        return sigv4.amz_dates(now)[0]

    def _learn_skew(self, err: S3Error) -> bool:
        """True when S3 refused the request as signed too far from its clock
        and told its time: RequestTimeTooSkewed (> 15 min) with
        ``<ServerTime>``, or any 401/403 whose ``Date`` header is more than
        4 minutes off (a HEAD's 403 has no body; the AWS SDKs' clock-skew
        adjuster uses the same rule).  Later requests are dated on S3's clock
        and the caller re-signs without counting a try.  minio-go did not
        correct skew, so a worker on a drifted node failed every upload."""
        if err.server_time is None:
            return False
        skew = err.server_time - time.time()
        if err.code != "RequestTimeTooSkewed" and abs(skew) < 240.0:
            return False                    # a 403 from a server whose clock agrees: a real refusal
        if abs(skew - self.clock_skew) < 2.0:
            return False                    # already dated on S3's clock: something else is wrong
        log.with_fields(skew_s=round(skew, 1)).warn("host clock differs from S3's; signing on S3's clock")
        self.clock_skew = skew
        return True

    async def _do(self, method: str, bucket: str, key: str = "", query: dict | None = None,
                  headers: dict | None = None, body: bytes | None = None, *, body_factory=None,
                  payload_hash: str | None = None, expect: tuple[int, ...] = (200,),
                  retry: bool = True, region: str | None = None, path_style: bool = False) -> tuple[int, dict, bytes]:
        """One signed request, retried (:meth:`retry_delay`) on connection errors
        and on the statuses and S3 error codes minio-go retries (:func:`is_retryable`)."""
        attempt = 0
        region_hops = skew_hops = 0
        while True:
            attempt += 1
            host, path = self._target(bucket, key, path_style)
            sreg = region if region is not None else await self.bucket_region(bucket)
            amzdate = self._amzdate()
            hdrs = {"host": host, "x-amz-date": amzdate}
            hdrs.update({k.lower(): str(v) for k, v in (headers or {}).items()})
            cred = self._creds()
            data = body
            if body_factory is not None:
                data, phash, extra = await body_factory(cred, amzdate, host, path, query, hdrs)
                hdrs.update(extra)
            else:
                phash = payload_hash or (hashing.digest("sha256", body or b"").hex() if body is not None
                                         else sigv4.EMPTY_SHA256)
                if body is not None:
                    hdrs["content-length"] = str(len(body))
            hdrs["x-amz-content-sha256"] = phash
            if not cred.anonymous:
                if cred.session_token:
                    hdrs["x-amz-security-token"] = cred.session_token
                signed = sigv4.sign(method, path, query, hdrs, phash, cred.access_key_id, cred.secret_access_key,
                                    sreg, amzdate, path_is_encoded=True)
                if callable(getattr(data, "bind_seed", None)):
                    data.bind_seed(signed)
                hdrs["authorization"] = signed.authorization
            url = URL(f"{'https' if self.ep.secure else 'http'}://{host}{path}" +
                      (("?" + sigv4.canonical_query(query)) if query else ""), encoded=True)
            send_headers = {k: v for k, v in hdrs.items() if k != "host"}
            send_headers["Host"] = host
            try:
                sess = await self._sess()
                payload = data.stream() if hasattr(data, "stream") else data
                async with sess.request(method, url, data=payload, skip_auto_headers=("Content-Type",),
                                        allow_redirects=False, **self._aio_proxy(host, send_headers)) as r:
                    rbody = await r.read()
                    if r.status in expect:
                        return r.status, CIMultiDict(r.headers), rbody
                    if r.status == 407:
                        raise _proxy_auth_error(self._proxy(host), f"{method} {path}")
                    err = _parse_error(r.status, rbody, f"{method} {path}", r.headers)
                    if region is None and region_hops < 2 and self._learn_region(bucket, err, sreg):
                        region_hops += 1
                        attempt -= 1
                        continue
                    if skew_hops < 2 and self._learn_skew(err):
                        skew_hops += 1
                        attempt -= 1
                        continue
                    if not is_retryable(err) or not retry or attempt > self.max_retries:
                        raise err
            except aiohttp.ClientHttpProxyError as e:
                if e.status in (401, 403, 407):
                    raise _proxy_auth_error(self._proxy(host), f"{method} {path}", e.status) from e
                if not retry or attempt > self.max_retries:
                    raise S3Error(0, "ProxyError", str(e), f"{method} {path}") from e
                err = e  # type: ignore[assignment]
            except (aiohttp.ClientError, asyncio.TimeoutError, ConnectionError) as e:
                if not retry or attempt > self.max_retries:
                    raise S3Error(0, "ConnectionError", str(e), f"{method} {path}") from e
                err = e  # type: ignore[assignment]
            d = self.retry_delay(attempt)
            log.with_fields(error=str(err), attempt=attempt).warn("s3 request failed; retrying in %.2fs", d)
            await asyncio.sleep(d)

    # ------------------------------------------------------------ buckets
    async def bucket_exists(self, bucket: str) -> bool:
        try:
            await self._do("HEAD", bucket, expect=(200,))
            return True
        except S3Error as e:
            if e.status == 404 or e.code == "NoSuchBucket":
                return False
            raise

    async def make_bucket(self, bucket: str, location: str = "") -> None:
        """minio ``MakeBucket``: location "" → the client's region, else us-east-1;
        the request is signed for that location and the answer cached."""
        location = location or self.region or DEFAULT_REGION
        body = None
        if location != DEFAULT_REGION:
            body = (f'<CreateBucketConfiguration xmlns="http://s3.amazonaws.com/doc/2006-03-01/">'
                    f"<LocationConstraint>{location}</LocationConstraint></CreateBucketConfiguration>").encode()
        await self._do("PUT", bucket, body=body if body is not None else b"", expect=(200,), region=location)
        if not self.region:
            self._regions[bucket] = location

    # ------------------------------------------------------------ objects
    async def put_object(self, bucket: str, key: str, src: str | bytes | int, size: int | None = None,
                         content_type: str = "application/octet-stream", wait_bytes=None, flow=None,
                         resume_path: str | None = None) -> str:
        """Upload a file path or fd (streamed) or bytes; returns the ETag.

        ``resume_path``: a state file for multipart uploads — an interrupted
        upload is kept open (not aborted) and a later call with the same
        state continues it, re-sending only parts whose bytes S3 does not
        already hold (checked by MD5 against the local file).

        ``wait_bytes(n)`` (optional coroutine) is awaited before bytes < n are
        read — lets the upload follow a file that is still being downloaded.
        ``flow`` (a native ``_relay.Flow`` of that download) lets the native
        send pump follow it without coming back to Python."""
        if size is None:
            if isinstance(src, (bytes, bytearray)):
                size = len(src)
            elif isinstance(src, int):
                size = os.fstat(src).st_size
            else:
                size = os.path.getsize(src)
        if size > MAX_SINGLE_PUT or (size >= self.multipart_threshold and size > self.part_size):
            return await self._put_multipart(bucket, key, src, size, content_type, wait_bytes, flow, resume_path)
        return await self._put_range(bucket, key, src, 0, size, {"content-type": content_type},
                                     wait_bytes=wait_bytes, flow=flow)

    async def _put_range(self, bucket: str, key: str, src: str | bytes | int, offset: int, length: int,
                         headers: dict, query: dict | None = None, wait_bytes=None, flow=None) -> str:
        mode = self._payload_mode()
        relay = rawhttp.relay_module() if self.native else None
        if relay is not None and not rawhttp.native_proxy_ok(self._proxy(self._target(bucket, key)[0]),
                                                             self.ep.secure):
            relay = None                     # TLS inside an https proxy: aiohttp
        if relay is not None and mode in ("streaming", "unsigned") and \
                not isinstance(src, (bytes, bytearray, memoryview)) and (flow is not None or wait_bytes is None):
            return await self._put_native(relay, bucket, key, src, offset, length, headers, query, mode, flow)
        factory = _BodyFactory(self, src, offset, length, mode, wait_bytes)
        _st, rh, _b = await self._do("PUT", bucket, key, query=query, headers=headers, body_factory=factory)
        return rh.get("ETag", "").strip('"')

    async def list_parts(self, bucket: str, key: str, upload_id: str) -> dict[int, tuple[str, int]]:
        """ListParts (paged by ``part-number-marker``): {part number: (etag, size)}."""
        out: dict[int, tuple[str, int]] = {}
        marker = "0"
        while True:
            _st, _h, body = await self._do("GET", bucket, key, query={"uploadId": upload_id,
                                                                       "part-number-marker": marker})
            root = _xml(body, "ListParts")
            for part in root.iter():
                if part.tag.rsplit("}", 1)[-1] != "Part":
                    continue
                f = {c.tag.rsplit("}", 1)[-1]: (c.text or "") for c in part}
                out[int(f["PartNumber"])] = (f.get("ETag", "").strip('"'), int(f.get("Size", "0") or 0))
            trunc = (root.findtext(f"{S3_NS}IsTruncated") or root.findtext("IsTruncated") or "false")
            marker = root.findtext(f"{S3_NS}NextPartNumberMarker") or root.findtext("NextPartNumberMarker") or ""
            if trunc.lower() != "true" or not marker:
                return out

    async def _resume_parts(self, state_path: str, bucket: str, key: str, src, size: int, part_size: int,
                            nparts: int) -> tuple[str, dict[int, str]]:
        """(upload id, {part index: etag}) of an interrupted multipart upload of
        this object that can be continued: same bucket/key/size/part size,
        the upload still open on the server, and every reused part's ETag
        equal to the MD5 of the local bytes it claims to hold."""
        try:
            with open(state_path) as f:
                st = json.load(f)
        except (OSError, ValueError):
            return "", {}
        if not isinstance(st, dict) or \
                (st.get("bucket"), st.get("key"), st.get("size"), st.get("part_size")) != (bucket, key, size, part_size):
            return "", {}
        uid = st.get("upload_id")
        if not isinstance(uid, str) or not uid:
            return "", {}
        try:
            listed = await self.list_parts(bucket, key, uid)
        except (S3Error, ET.ParseError, KeyError, ValueError) as e:
            log.with_fields(key=key, error=str(e)).info("interrupted multipart upload is gone; starting over")
            return "", {}
        path = src if isinstance(src, str) else f"/proc/self/fd/{src}" if isinstance(src, int) else None
        want = {pn: tag for pn, (tag, sz) in listed.items()
                if 1 <= pn <= nparts and sz == min(part_size, size - (pn - 1) * part_size) and len(tag) == 32}
        if path is None or not want:
            return uid, {}

        def md5_of(pn: int) -> str:
            off = (pn - 1) * part_size
            return hashing.hash_file(path, ["md5"], off, min(part_size, size - off))["md5"].hex()
        loop = asyncio.get_running_loop()
        sums = await asyncio.gather(*(loop.run_in_executor(None, md5_of, pn) for pn in want))
        ok = {pn - 1: tag for (pn, tag), got in zip(want.items(), sums) if got == tag}
        log.with_fields(key=key, upload_id=uid, reused_parts=len(ok), of=nparts).info(
            "resuming interrupted multipart upload")
        return uid, ok

    async def _put_multipart(self, bucket: str, key: str, src: str | bytes | int, size: int, content_type: str,
                             wait_bytes=None, flow=None, resume_path: str | None = None) -> str:
        plan_parts(size, self.part_size)           # refuse > 5 TiB before initiating
        part_size, nparts = plan_parts(size, self.part_size)
        upload_id, reused = ("", {})
        if resume_path and not isinstance(src, (bytes, bytearray, memoryview)):
            upload_id, reused = await self._resume_parts(resume_path, bucket, key, src, size, part_size, nparts)
        if not upload_id:
            _st, _h, body = await self._do("POST", bucket, key, query={"uploads": ""},
                                           headers={"content-type": content_type}, body=b"")
            root = _xml(body, "InitiateMultipartUpload")
            upload_id = root.findtext(f"{S3_NS}UploadId") or root.findtext("UploadId") or ""
            if not upload_id:
                raise S3Error(0, "MalformedXML", "no UploadId in InitiateMultipartUpload response")
        if resume_path:
            _save_json(resume_path, {"bucket": bucket, "key": key, "size": size, "part_size": part_size,
                                     "upload_id": upload_id})
        etags: list[str] = [""] * nparts
        for i, tag in reused.items():
            etags[i] = tag
        todo = _PartQueue(nparts, part_size, size, flow, skip=reused)

        async def worker() -> None:
            while todo:
                i = todo.pick()
                off = i * part_size
                ln = min(part_size, size - off)
                etags[i] = await self._put_range(bucket, key, src, off, ln, {},
                                                 query={"partNumber": str(i + 1), "uploadId": upload_id},
                                                 wait_bytes=wait_bytes, flow=flow)
        workers = [asyncio.ensure_future(worker()) for _ in range(min(self.parallel_parts, nparts))]
        try:
            try:
                await asyncio.gather(*workers)
            except BaseException:
                # stop the siblings and wait for them (their native pumps hold fds)
                for w in workers:
                    w.cancel()
                await asyncio.gather(*workers, return_exceptions=True)
                raise
            xml = "".join(f"<Part><PartNumber>{i + 1}</PartNumber><ETag>\"{e}\"</ETag></Part>"
                          for i, e in enumerate(etags))
            cbody = f"<CompleteMultipartUpload>{xml}</CompleteMultipartUpload>".encode()
            etag = await self._complete(bucket, key, upload_id, cbody, etags)
            if resume_path:
                with contextlib.suppress(OSError):
                    os.remove(resume_path)
            return etag
        except BaseException as e:
            if resume_path and not isinstance(e, asyncio.CancelledError):
                # keep the upload: a retry of this job continues from the parts that landed
                # (stale uploads are the bucket lifecycle's AbortIncompleteMultipartUpload job)
                log.with_fields(key=key, upload_id=upload_id).warn("multipart upload interrupted; kept for resume")
                raise
            if resume_path:
                with contextlib.suppress(OSError):
                    os.remove(resume_path)
            try:
                await self._do("DELETE", bucket, key, query={"uploadId": upload_id}, expect=(204, 200),
                               retry=False)
            except Exception:
                pass
            raise

    # S3 sends CompleteMultipartUpload's status line before it stitches the
    # parts, so a failure while stitching comes back as 200 with an <Error>
    # body; the API reference asks clients to retry these.
    COMPLETE_RETRY_CODES = frozenset({"InternalError", "SlowDown", "ServiceUnavailable", "RequestTimeout"})

    async def _complete(self, bucket: str, key: str, upload_id: str, cbody: bytes, etags: list[str]) -> str:
        """CompleteMultipartUpload with both of its failure shapes handled.

        * 200 + ``<Error>``: a transient code (:attr:`COMPLETE_RETRY_CODES`)
          is retried in place; the upload is still open.  minio-go
          (``api-put-object-multipart.go`` ``completeMultipartUploadCore``)
          returned it as the job's error, so the whole job ran again.
        * A reply lost after S3 committed (reset, a proxy's 5xx): the retry
          that ``_do`` makes answers NoSuchUpload.  The object is then HEADed
          and accepted when its ETag is the multipart ETag of exactly these
          parts (MD5 over the part MD5s, ``-N``), else the error stands.
        """
        attempt = 0
        while True:
            attempt += 1
            try:
                _st, _h, rb = await self._do("POST", bucket, key, query={"uploadId": upload_id}, body=cbody)
            except S3Error as e:
                want = multipart_etag(etags)
                if e.code == "NoSuchUpload" and want:
                    got = await self._stat_etag(bucket, key)
                    if got == want:
                        log.with_fields(key=key, etag=got).info("complete reply lost; object already committed")
                        return got
                raise
            if b"<Error>" not in rb:
                r = _xml(rb, "CompleteMultipartUpload")
                return (r.findtext(f"{S3_NS}ETag") or r.findtext("ETag") or "").strip('"')
            err = _parse_error(200, rb, f"complete {key}")
            if (err.code not in self.COMPLETE_RETRY_CODES and err.code not in RETRYABLE_CODES) or \
                    attempt > self.max_retries:
                raise err
            d = self.retry_delay(attempt)
            log.with_fields(key=key, code=err.code, attempt=attempt).warn(
                "complete multipart answered 200 with an error; retrying in %.2fs", d)
            await asyncio.sleep(d)

    async def _stat_etag(self, bucket: str, key: str) -> str:
        try:
            h = await self.stat_object(bucket, key)
        except S3Error as e:
            if e.status == 404:
                return ""
            raise
        return (h.get("ETag") or "").strip('"')

    async def _put_native(self, relay, bucket: str, key: str, src: str | int, offset: int, length: int,
                          headers: dict, query: dict | None, mode: str, flow) -> str:
        """One PUT whose body never enters Python: the head is signed here,
        then ``_relay.send_body`` writes head + body (aws-chunked with chunk
        signatures hashed on a native pool, or sendfile for unsigned) from the
        file straight to the socket; the reply is parsed here.  Same retry
        policy as :meth:`_do`.  When the download it follows stalls for the
        flow's ``stall`` seconds the pump stops and this raises S3Error
        ``SourceStalled`` (the caller uploads after the download instead).

        The pump owns ``sock`` and ``fd`` while it runs: if this coroutine is
        cancelled the pump is stopped (socket shut down, native cancel token
        set) and awaited before either is closed, so a reused fd number can
        never receive its writes."""
        fd = os.dup(src) if isinstance(src, int) else os.open(src, os.O_RDONLY)
        attempt = 0
        region_hops = skew_hops = 0
        try:
            while True:
                attempt += 1
                cred = self._creds()
                m = "unsigned" if (cred.anonymous and mode == "streaming") else mode
                host, path = self._target(bucket, key)
                sreg = await self.bucket_region(bucket)
                amzdate = self._amzdate()
                hdrs = {"host": host, "x-amz-date": amzdate}
                hdrs.update({k.lower(): str(v) for k, v in (headers or {}).items()})
                if m == "streaming":
                    hdrs.update({"content-encoding": "aws-chunked", "x-amz-decoded-content-length": str(length),
                                 "content-length": str(sigv4.chunked_length(length))})
                    hdrs["x-amz-content-sha256"] = sigv4.STREAMING_PAYLOAD
                else:
                    hdrs["content-length"] = str(length)
                    hdrs["x-amz-content-sha256"] = sigv4.UNSIGNED_PAYLOAD
                signed = None
                if not cred.anonymous:
                    if cred.session_token:
                        hdrs["x-amz-security-token"] = cred.session_token
                    signed = sigv4.sign("PUT", path, query, hdrs, hdrs["x-amz-content-sha256"], cred.access_key_id,
                                        cred.secret_access_key, sreg, amzdate, path_is_encoded=True)
                    hdrs["authorization"] = signed.authorization
                target = path + (("?" + sigv4.canonical_query(query)) if query else "")
                px = self._proxy(host)
                if rawhttp.absolute_form(px) and not self.ep.secure:
                    target = f"http://{host}{target}"
                send = {"Host": host, **{k: v for k, v in hdrs.items() if k != "host"},
                        **rawhttp.proxy_auth_header(px)}
                head = rawhttp.request_head("PUT", target, send)
                chost, cport = rawhttp.split_host(host, 443 if self.ep.secure else 80)
                err: Exception | None = None
                conn = None
                try:
                    try:
                        conn, reused = await self._raw.connect(
                            chost, cport, tls=self._tls_ctx(), proxy=px,
                            proxy_tls=self._tls_ctx(True) if px is not None and px.scheme == "https" else None)
                    except rawhttp.ProxyRefused as e:
                        raise _proxy_auth_error(px, f"PUT {path}", e.status or 407, str(e)) from e
                    rawhttp.trace("put_pump_start")
                    sent, _last, perr = await rawhttp.run_pump(
                        conn, relay.send_body, head, fd, offset, length, flow,
                        1 if m == "streaming" else 0, signed.key if signed else b"", amzdate,
                        signed.scope if signed else "", signed.signature if signed else "", sigv4.STREAM_CHUNK,
                        self.sign_threads, 300.0, self._chunk_gpu() if m == "streaming" else None)
                    rawhttp.trace("put_sent")
                    if perr and "source stalled" in perr:
                        raise S3Error(0, "SourceStalled", f"no download progress for {flow.stall:g}s",
                                      f"PUT {path}")
                    if perr and ("source" in perr or perr == "cancelled"):
                        raise S3Error(0, "SourceFailed", perr, f"PUT {path}")
                    try:
                        resp = await rawhttp.read_head(conn, 1.0 if perr else 300.0)
                    except rawhttp.RawHTTPError:
                        if perr:
                            if reused and sent == 0:
                                attempt -= 1          # stale keep-alive socket: not a real attempt
                            raise rawhttp.RawHTTPError(perr)
                        raise
                    rawhttp.trace("put_pump_end")
                    body = await rawhttp.read_small_body(conn, resp, 60.0, method="PUT")
                    rawhttp.trace("put_response")
                    if resp.status == 200 and not perr:
                        if resp.keep_alive:
                            self._raw.release(chost, cport, conn)
                            conn = None
                        return resp.headers.get("ETag", "").strip('"')
                    if resp.status == 407 and px is not None:
                        raise _proxy_auth_error(px, f"PUT {path}")
                    err = _parse_error(resp.status, body, f"PUT {path}", resp.headers)
                    if region_hops < 2 and self._learn_region(bucket, err, sreg):
                        region_hops += 1
                        attempt -= 1
                        continue
                    if skew_hops < 2 and self._learn_skew(err):
                        skew_hops += 1
                        attempt -= 1
                        continue
                    if not is_retryable(err) or attempt > self.max_retries:
                        raise err
                except (rawhttp.RawHTTPError, OSError, asyncio.TimeoutError) as e:
                    if attempt > self.max_retries:
                        raise S3Error(0, "ConnectionError", str(e), f"PUT {path}") from e
                    err = e
                finally:
                    if conn is not None:
                        conn.close()
                if attempt <= 0:
                    continue
                d = self.retry_delay(attempt)
                log.with_fields(error=str(err), attempt=attempt).warn("s3 request failed; retrying in %.2fs", d)
                await asyncio.sleep(d)
        finally:
            os.close(fd)

    async def get_object(self, bucket: str, key: str) -> bytes:
        _st, _h, b = await self._do("GET", bucket, key)
        return b

    async def stat_object(self, bucket: str, key: str) -> dict:
        _st, h, _b = await self._do("HEAD", bucket, key)
        return h

    async def delete_object(self, bucket: str, key: str) -> None:
        await self._do("DELETE", bucket, key, expect=(204, 200))

    async def list_objects(self, bucket: str, prefix: str = "") -> list[str]:
        keys: list[str] = []
        token = None
        while True:
            q = {"list-type": "2", "prefix": prefix}
            if token:
                q["continuation-token"] = token
            _st, _h, b = await self._do("GET", bucket, query=q)
            root = _xml(b, "ListObjectsV2")
            for c in root.iter():
                if c.tag.endswith("Contents"):
                    k = c.find(f"{S3_NS}Key")
                    if k is None:
                        k = c.find("Key")
                    keys.append(k.text or "")
            trunc = (root.findtext(f"{S3_NS}IsTruncated") or root.findtext("IsTruncated") or "false")
            token = root.findtext(f"{S3_NS}NextContinuationToken") or root.findtext("NextContinuationToken")
            if trunc != "true" or not token:
                return keys


class _PartQueue:
    """Pending part numbers of one multipart upload, handed out in the order
    their bytes land on disk.

    Following a segmented download, a segment fills front to back, so within
    a segment the part that will be complete soonest is its first pending one;
    only those (one per unfinished segment, plus the start of every run of
    pending parts) are ranked with ``Flow.bytes_until_covered``.  Each pick
    costs O(runs + segments), not O(pending parts), so 10,000-part uploads stay
    cheap.  Without a flow (or once it finished) parts go in order."""

    def __init__(self, nparts: int, part_size: int, size: int, flow=None, skip=()) -> None:
        self.part_size, self.size, self.flow = part_size, size, flow
        skip = set(skip)
        self._todo = [p for p in range(nparts) if p not in skip]              # ascending
        pending = set(self._todo)
        self._runs = {p for p in self._todo if p - 1 not in pending}        # parts that start a run

    def __len__(self) -> int:
        return len(self._todo)

    def __bool__(self) -> bool:
        return bool(self._todo)

    def _take(self, part: int) -> int:
        import bisect
        self._todo.pop(bisect.bisect_left(self._todo, part))
        self._runs.discard(part)
        nxt = part + 1
        k = bisect.bisect_left(self._todo, nxt)
        if k < len(self._todo) and self._todo[k] == nxt:
            self._runs.add(nxt)
        return part

    def _candidates(self) -> set[int]:
        import bisect
        todo = self._todo
        cand = set(self._runs)
        starts = getattr(self.flow, "open_starts", None)
        if starts is not None:
            last = max(0, (self.size - 1) // self.part_size)
            for st in starts():
                k = bisect.bisect_left(todo, min(st // self.part_size, last))
                if k < len(todo):
                    cand.add(todo[k])
        return cand

    def pick(self) -> int:
        todo = self._todo
        flow = self.flow
        if flow is None or len(todo) == 1 or flow.finished:
            return self._take(todo[0])
        ps, size = self.part_size, self.size
        best = min(self._candidates(), key=lambda p: (flow.bytes_until_covered(p * ps, min(size, (p + 1) * ps)), p))
        return self._take(best)


class _StreamBody:
    """Payload for one PUT: plain bytes, or an aws-chunked stream signed
    incrementally once the seed signature is known."""

    def __init__(self, client: S3Client, src: str | bytes | int, offset: int, length: int, mode: str,
                 scope: str = "", amzdate: str = "", wait_bytes=None) -> None:
        self.wait_bytes = wait_bytes
        self.client = client
        self.src = src
        self.offset = offset
        self.length = length
        self.mode = mode
        self.scope = scope
        self.amzdate = amzdate
        self.signer: sigv4.ChunkSigner | None = None

    def bind_seed(self, signed: sigv4.Signed) -> None:
        if self.mode == "streaming":
            self.signer = sigv4.ChunkSigner(signed.key, signed.amzdate, signed.scope, signed.signature)

    def _read(self, fd: int | None, pos: int, n: int) -> bytes:
        if fd is None:
            return bytes(memoryview(self.src)[pos:pos + n])  # type: ignore[arg-type]
        data = os.pread(fd, n, pos)
        if len(data) != n:
            raise S3Error(0, "ShortRead", f"file shrank while uploading ({pos + len(data)} < {pos + n})")
        return data

    def _produce_block(self, fd: int | None, pos: int, n: int, last: bool) -> bytes:
        """Worker thread: read one block and (streaming mode) aws-chunk-encode it."""
        data = self._read(fd, pos, n)
        if self.signer is None:
            return data
        out = self.signer.feed(data)
        if last:
            out += self.signer.finish()
        return out

    async def stream(self) -> AsyncIterator[bytes]:
        """Body generator with a 2-deep read→sign pipeline running ahead of
        the socket writer (the native encoder releases the GIL)."""
        if self.mode == "streaming":
            assert self.signer is not None, "seed signature not bound"
        loop = asyncio.get_running_loop()
        blk = self.client.io_block
        if isinstance(self.src, (bytes, bytearray, memoryview)):
            fd = None
        elif isinstance(self.src, int):
            fd = os.dup(self.src)
        else:
            fd = os.open(self.src, os.O_RDONLY)
        q: asyncio.Queue = asyncio.Queue(maxsize=2)

        async def produce() -> None:
            try:
                pos, end = self.offset, self.offset + self.length
                if pos == end and self.signer is not None:
                    await q.put(self.signer.finish())
                while pos < end:
                    n = min(blk, end - pos)
                    if self.wait_bytes is not None:
                        await self.wait_bytes(pos + n)
                    out = await loop.run_in_executor(None, self._produce_block, fd, pos, n, pos + n >= end)
                    pos += n
                    if out:
                        await q.put(out)
                await q.put(None)
            except BaseException as e:  # noqa: BLE001 - forwarded to the consumer
                await q.put(e)

        task = asyncio.ensure_future(produce())
        try:
            while True:
                item = await q.get()
                if item is None:
                    return
                if isinstance(item, BaseException):
                    raise item
                yield item
        finally:
            task.cancel()
            if fd is not None:
                os.close(fd)


class _BodyFactory:
    """Builds the body + payload hash + extra headers for each (re)try."""

    def __init__(self, client: S3Client, src: str | bytes | int, offset: int, length: int, mode: str,
                 wait_bytes=None) -> None:
        self.client, self.src, self.offset, self.length, self.mode = client, src, offset, length, mode
        self.wait_bytes = wait_bytes

    async def __call__(self, cred: Value, amzdate: str, host: str, path: str, query, hdrs):
        mode = self.mode
        if cred.anonymous and mode == "streaming":
            mode = "unsigned"  # chunk signatures need credentials
        body = _StreamBody(self.client, self.src, self.offset, self.length, mode, wait_bytes=self.wait_bytes)
        if mode == "streaming":
            extra = {"content-encoding": "aws-chunked", "x-amz-decoded-content-length": str(self.length),
                     "content-length": str(sigv4.chunked_length(self.length))}
            return body, sigv4.STREAMING_PAYLOAD, extra
        extra = {"content-length": str(self.length)}
        if mode == "signed":
            loop = asyncio.get_running_loop()
            if self.wait_bytes is not None:
                await self.wait_bytes(self.offset + self.length)
            if isinstance(self.src, (bytes, bytearray)):
                h = hashing.digest("sha256", memoryview(self.src)[self.offset:self.offset + self.length]).hex()
            else:
                path = f"/proc/self/fd/{self.src}" if isinstance(self.src, int) else self.src
                d = await loop.run_in_executor(None, hashing.hash_file, path, ["sha256"], self.offset,
                                               self.length)
                h = d["sha256"].hex()
            return body, h, extra
        return body, sigv4.UNSIGNED_PAYLOAD, extra


__all__ = ["S3Client", "S3Error", "Endpoint", "Chain"]
