"""In-process S3 server (raw asyncio HTTP, ``rawserver``) that VERIFIES SigV4 — the MinIO/S3
stand-in for tests, smoke and bench (the reference had none).

Supports: HEAD/PUT bucket (path-style and virtual-host style), PUT object
(plain, UNSIGNED-PAYLOAD, signed SHA-256, and aws-chunked streaming with
per-chunk signature verification), multipart (initiate / upload part /
complete / abort), GET/HEAD/DELETE object, ListObjectsV2.

Storage modes: ``memory`` (default), ``disk`` (under ``root``) or
``discard`` (keep only size + ETag — for throughput benches).  With the
native relay built, aws-chunked and unsigned PUT bodies are received (and
every chunk signature verified) by ``_relay.recv_verify_chunked`` /
``_relay.recv_body`` outside the interpreter, as MinIO would on its own box.
Fault injection, with the codes AWS S3 uses: :meth:`fail_next` answers the
next N requests with a status and S3 error code (503 ``SlowDown``, 429,
500 ``InternalError``, 400 ``RequestTimeout``, 403 ``ExpiredToken``, ...),
:meth:`fail_for` every request during an outage window, :meth:`down_for`
refuses connections for a while (the listener is closed, as during a
restart), and ``idle_timeout`` answers 400 ``RequestTimeout`` and drops the
connection when a request body sends nothing for that long (AWS does after
~20 s).  Content check
(``expect``, a :class:`~tritondl_testkit.fakes.payload.Expectations`): a PUT of a
synthetic payload variant whose bytes are not the origin's is refused with
400 ``BadDigest`` — in discard mode too, from the leaf hashes the native
chunk verifier already computed (``counts["content_ok"]`` /
``["content_bad"]``).

AWS behaviours the client must cope with (minio-go does): every bucket lives
in a region (``create_bucket(name, region)``, or a ``LocationConstraint``);
a request signed for another region gets 400 ``AuthorizationHeaderMalformed``
naming the bucket's ``<Region>`` (and ``x-amz-bucket-region``), while
``GET ?location`` answers for any signing region.  Part numbers are limited to
1..10000 and every part but the last must be ≥ 5 MiB (``strict_parts``).
``tls=(cert_pem, key_pem)`` serves https.
"""

from __future__ import annotations

import asyncio
import hashlib
import hmac
import itertools
import os
import re
import time
from dataclasses import dataclass, field
from urllib.parse import parse_qsl, unquote

from tritondl.s3 import sigv4
from tritondl.utils import rawhttp
from . import rawserver as web

_CHUNK_HDR = re.compile(rb"([0-9a-fA-F]+);chunk-signature=([0-9a-f]{64})\r\n")
_AUTH_RE = re.compile(r"AWS4-HMAC-SHA256 Credential=([^/]+)/([^,]+), *SignedHeaders=([^,]+), *Signature=([0-9a-f]+)")


@dataclass
class Obj:
    size: int
    etag: str
    data: bytes | None = None
    path: str | None = None
    content_type: str = ""
    leaves: bytes | None = None        # 64 KiB leaf SHA-256s when a content check needs them


@dataclass
class Upload:
    bucket: str
    key: str
    parts: dict = field(default_factory=dict)  # n -> Obj


_IDLE_MSG = ("Your socket connection to the server was not read from or written to within the timeout "
             "period. Idle connections will be closed.")


def _xml_err(status: int, code: str, msg: str, region: str = "") -> web.Response:
    reg = f"<Region>{region}</Region>" if region else ""
    body = (f"<?xml version=\"1.0\" encoding=\"UTF-8\"?><Error><Code>{code}</Code><Message>{msg}</Message>"
            f"{reg}</Error>")
    return web.Response(status=status, body=body.encode(), content_type="application/xml")


class FakeS3:
    def __init__(self, host: str = "127.0.0.1", port: int = 0, *, access_key: str | None = None,
                 secret_key: str | None = None, region: str = "us-east-1", store: str = "memory",
                 root: str | None = None, tls: tuple[str, str] | None = None, strict_parts: bool = True,
                 names: tuple[str, ...] = (), expect=None) -> None:
        self.host, self.port = host, port
        self.expect = expect           # payload.Expectations: check PUT content against the origin's
        self.counts: dict[str, int] = {"content_ok": 0, "content_bad": 0}
        self.names = set(names)        # other names of the service endpoint (path-style, not a bucket)
        self.tls = tls
        self.strict_parts = strict_parts
        self.bucket_regions: dict[str, str] = {}
        self._outage_until = 0.0
        self.rate: float | None = None          # bytes/s of a shared ingest link (None: unlimited)
        self.stream_rate = web.fake_stream_rate()   # bytes/s of one PUT's stream (None: unlimited)
        self._link_free = 0.0
        self.access_key, self.secret_key = access_key, secret_key
        self.region = region
        self.store = store
        self.root = root
        self.buckets: dict[str, dict[str, Obj]] = {}
        self.uploads: dict[str, Upload] = {}
        self.list_parts_page = 1000
        self.fail_parts: set[int] = set()       # fault injection: these part numbers get HTTP 500
        self.fail_parts_once = False            # ... only the first time each is sent
        # CompleteMultipartUpload faults: the next N completes answer 200 with an
        # <Error> body (upload left open), or commit and then lose the reply (503)
        self.complete_error_200 = 0
        self.complete_error_code = "InternalError"
        self.complete_lose_reply = 0
        self.clock_offset = 0.0                 # seconds this server's clock is ahead of the host's
        self.skew_refusals = 0
        self._ids = itertools.count(1)
        self._fail = 0
        self._fail_status = 503
        self._fail_code = "ServiceUnavailable"
        self._fail_methods: tuple[str, ...] = ()
        self.failed = 0                          # requests answered with an injected failure
        # AWS: 400 RequestTimeout when a request body sends nothing for ~20 s (None: wait forever)
        self.idle_timeout: float | None = None
        self.idle_timeouts = 0
        self.requests: list[tuple[str, str]] = []
        self.bytes_received = 0
        # native aws-chunked verifier threads per PUT (stands in for a remote S3's capacity)
        self.verify_threads = int(os.environ.get("TRITONDL_FAKE_S3_VERIFY_THREADS", "4"))
        self._server: web.Server | None = None
        self.native = True

    # ------------------------------------------------------------ lifecycle
    async def start(self) -> "FakeS3":
        self._server = web.Server(self._handle, tls=self.tls)
        self.port = await self._server.start(self.host, self.port)
        return self

    async def stop(self) -> None:
        if self._server is not None:
            await self._server.stop()
            self._server = None

    @property
    def endpoint(self) -> str:
        return f"{'https' if self.tls else 'http'}://{self.host}:{self.port}"

    # the S3 error code AWS sends with each status (RequestTimeout, ExpiredToken: see fail_next)
    DEFAULT_CODES = {500: "InternalError", 502: "BadGateway", 503: "ServiceUnavailable", 504: "GatewayTimeout",
                     429: "SlowDown", 400: "RequestTimeout", 403: "ExpiredToken", 501: "NotImplemented"}

    def fail_next(self, n: int, status: int = 503, code: str | None = None, methods: tuple[str, ...] = ()) -> None:
        """The next ``n`` requests (of ``methods``, default any) get ``status``
        with S3 error ``code`` (default: the one AWS sends with that status)."""
        self._fail, self._fail_status = n, status
        self._fail_code = code or self.DEFAULT_CODES.get(status, "ServiceUnavailable")
        self._fail_methods = tuple(methods)

    def fail_for(self, seconds: float, status: int = 503, code: str | None = None) -> None:
        """Outage: every request gets ``status`` for the next ``seconds``."""
        self._outage_until, self._fail_status = time.monotonic() + seconds, status
        self._fail_code = code or self.DEFAULT_CODES.get(status, "ServiceUnavailable")
        self._fail_methods = ()

    async def down_for(self, seconds: float) -> None:
        """Outage: the server stops listening and drops its connections, then
        comes back on the same port after ``seconds`` (a MinIO restart)."""
        port = self.port
        await self.stop()

        async def back() -> None:
            await asyncio.sleep(seconds)
            self.port = port
            await self.start()
        self._restart = asyncio.ensure_future(back())

    def create_bucket(self, name: str, region: str | None = None) -> None:
        self.buckets.setdefault(name, {})
        self.bucket_regions[name] = region or self.region

    def delete_bucket(self, name: str) -> None:
        self.buckets.pop(name, None)
        self.bucket_regions.pop(name, None)

    def object_bytes(self, bucket: str, key: str) -> bytes:
        o = self.buckets[bucket][key]
        if o.data is not None:
            return o.data
        if o.path is not None:
            with open(o.path, "rb") as f:
                return f.read()
        raise KeyError("object content discarded")

    # ------------------------------------------------------------ routing
    def _split(self, request: web.Request) -> tuple[str, str]:
        raw = request.raw_path.split("?", 1)[0]
        host = request.headers.get("Host", "").split(":")[0]
        if host.count(".") and not re.match(r"^\d+\.\d+\.\d+\.\d+$", host) and host not in ("localhost",) \
                and not host.startswith(self.host) and host not in self.names:
            bucket = host.split(".", 1)[0]
            return bucket, unquote(raw[1:])
        parts = raw[1:].split("/", 1)
        bucket = unquote(parts[0]) if parts and parts[0] else ""
        key = unquote(parts[1]) if len(parts) > 1 else ""
        return bucket, key

    def _verify(self, request: web.Request) -> tuple[bytes, str, str, str] | web.Response | None:
        """Return (signing_key, seed_sig, amzdate, scope) for signed requests,
        None for allowed anonymous ones, or an error response."""
        auth = request.headers.get("Authorization")
        if auth is None:
            if self.access_key is None:
                return None
            return _xml_err(403, "AccessDenied", "Anonymous access denied")
        m = _AUTH_RE.match(auth)
        if not m:
            return _xml_err(400, "AuthorizationHeaderMalformed", "bad Authorization header")
        akid, scope_rest, signed_headers, sig = m.groups()
        if self.access_key is not None and akid != self.access_key:
            return _xml_err(403, "InvalidAccessKeyId", "unknown access key")
        secret = self.secret_key or ""
        date, region, service, _term = scope_rest.split("/")
        request.signed_region = region
        amzdate = request.headers.get("x-amz-date", "")
        hdrs = {}
        for h in signed_headers.split(";"):
            v = request.headers.get(h)
            if v is None:
                return _xml_err(400, "SignatureDoesNotMatch", f"signed header {h} missing")
            hdrs[h] = v
        query = parse_qsl(request.query_string, keep_blank_values=True)
        phash = request.headers.get("x-amz-content-sha256", "")
        raw_path = request.raw_path.split("?", 1)[0]
        s = sigv4.sign(request.method, raw_path, query, hdrs, phash, akid, secret, region, amzdate,
                       service=service, path_is_encoded=True)
        if not hmac.compare_digest(s.signature, sig):
            return _xml_err(403, "SignatureDoesNotMatch",
                            "The request signature we calculated does not match the signature you provided.")
        skewed = self._skewed(amzdate)
        if skewed is not None:
            return skewed
        return s.key, sig, amzdate, s.scope

    def _skewed(self, amzdate: str) -> web.Response | None:
        """S3 refuses a request signed more than 15 minutes from its clock
        (403 RequestTimeTooSkewed, naming both times); ``clock_offset``
        moves this server's clock."""
        import calendar
        try:
            t = calendar.timegm(time.strptime(amzdate, "%Y%m%dT%H%M%SZ"))
        except ValueError:
            return _xml_err(403, "AccessDenied", "bad x-amz-date")
        now = time.time() + self.clock_offset
        if abs(t - now) <= 900:
            return None
        self.skew_refusals += 1
        st = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(now))
        body = (f"<?xml version=\"1.0\" encoding=\"UTF-8\"?><Error><Code>RequestTimeTooSkewed</Code>"
                f"<Message>The difference between the request time and the current time is too large."
                f"</Message><RequestTime>{amzdate}</RequestTime><ServerTime>{st}</ServerTime>"
                f"<MaxAllowedSkewMilliseconds>900000</MaxAllowedSkewMilliseconds></Error>")
        return web.Response(status=403, body=body.encode(), content_type="application/xml",
                            headers={"Date": time.strftime("%a, %d %b %Y %H:%M:%S GMT", time.gmtime(now))})

    async def _read_body(self, request: web.Request, auth, keep: bool = True):
        """Verified request body.  ``keep=False`` (object data in discard
        mode): aws-chunked bodies are verified without materialising the
        decoded bytes and only their length is returned (as ``_Sized``).
        With ``rate`` set, the reply waits until a shared link of that many
        bytes/s would have carried the body (all requests queue on it)."""
        n = request.body_length or 0                 # remaining bytes: read it before the body is consumed
        t0 = time.monotonic()
        body = await self._read_body_raw(request, auth, keep)
        if self.stream_rate:                         # this stream cannot have carried it faster
            wait = t0 + n / self.stream_rate - time.monotonic()
            if wait > 0:
                await asyncio.sleep(wait)
        if self.rate:
            now = time.monotonic()
            self._link_free = max(now, self._link_free) + n / self.rate
            await asyncio.sleep(self._link_free - now)
        return body

    async def _read_body_raw(self, request: web.Request, auth, keep: bool = True):
        phash = request.headers.get("x-amz-content-sha256", sigv4.UNSIGNED_PAYLOAD)
        relay = rawhttp.relay_module() if self.native else None
        if phash == sigv4.STREAMING_PAYLOAD:
            if not isinstance(auth, tuple):
                raise _BadReq(400, "InvalidRequest", "streaming payload needs a signature")
            if relay is not None and request.body_length:
                return await self._read_chunked_native(relay, request, auth, keep)
            return await self._read_chunked(request, auth, keep)
        if relay is not None and not keep and phash in (sigv4.UNSIGNED_PAYLOAD, "") and request.body_length:
            n = request.body_length
            stream, pre = request.take_body()
            leaves = None
            if self.expect is None:
                got, _eof, err = await asyncio.get_running_loop().run_in_executor(
                    None, relay.recv_body, stream, -1, 0, n, pre, None, 0, 0, self.idle_timeout or 300.0)
            else:                       # content check: leaf hashes computed while the body lands
                got, err, leaves = await asyncio.get_running_loop().run_in_executor(
                    None, relay.recv_leaf_hashes, stream, n, pre, self.verify_threads, self.idle_timeout or 300.0)
            if err:
                request.transport.close()
                if "timeout" in err:
                    raise _BadReq(400, "RequestTimeout", _IDLE_MSG)
                raise _BadReq(400, "IncompleteBody", err)
            self.bytes_received += got
            return _Sized(got, leaves)
        data = await request.read()
        self.bytes_received += len(data)
        if phash not in (sigv4.UNSIGNED_PAYLOAD, "") and auth is not None:
            if hashlib.sha256(data).hexdigest() != phash:
                raise _BadReq(400, "XAmzContentSHA256Mismatch", "payload hash mismatch")
        return data

    async def _read_chunked_native(self, relay, request: web.Request, auth, keep: bool):
        """Native receive + per-chunk signature verification (GIL released)."""
        key, seed, amzdate, scope = auth
        decoded_len = int(request.headers.get("x-amz-decoded-content-length", "-1"))
        raw_len = request.body_length
        stream, pre = request.take_body()
        n, err, data, leaves = await asyncio.get_running_loop().run_in_executor(
            None, relay.recv_verify_chunked, stream, raw_len, pre, key, amzdate, scope, seed, keep,
            self.verify_threads, self.idle_timeout or 300.0)
        self.bytes_received += raw_len
        if err:
            if "closed" in err or "timeout" in err or "socket" in err or "recv" in err:
                request.transport.close()
            else:
                # the body was consumed up to the error: drop the connection after replying
                request.transport_close_after = True
            if "timeout" in err:
                raise _BadReq(400, "RequestTimeout", _IDLE_MSG)
            code = 403 if "signature" in err else 400
            raise _BadReq(code, "SignatureDoesNotMatch" if code == 403 else "IncompleteBody", err)
        if decoded_len >= 0 and decoded_len != n:
            raise _BadReq(400, "IncompleteBody", "decoded length mismatch")
        return data if keep else _Sized(n, leaves)

    async def _read_chunked(self, request: web.Request, auth, keep: bool = True):
        """Decode an aws-chunked body and verify EVERY chunk signature while it
        streams in.  Frame boundaries are tracked here; each ~1 MiB run of
        whole frames is verified + decoded by the native parser in a worker
        thread (payload SHA-256 map + signature-chain scan), seeded with the
        previous run's last *claimed* signature — so runs verify in parallel
        and a forged claim still fails its own run."""
        key, seed, amzdate, scope = auth
        decoded_len = int(request.headers.get("x-amz-decoded-content-length", "-1"))
        loop = asyncio.get_running_loop()
        from tritondl.ops import hashing
        buf = bytearray()
        pos = 0           # parse cursor in buf
        run_start = 0     # start of the current run of whole frames
        prev = seed
        last_sig = seed
        runs: list[asyncio.Future] = []
        finished = False
        decoded = [0]        # payload bytes dispatched (keep=False)
        frame_bytes = [0]    # payload bytes in the current run

        def dispatch(end: int, final: bool) -> None:
            nonlocal run_start, prev
            if end > run_start:
                with memoryview(buf) as mv:
                    chunk = bytes(mv[run_start:end])
                runs.append(loop.run_in_executor(None, hashing.aws_chunk_decode, key, amzdate, scope, prev, chunk,
                                                 2, keep, final))
                if not keep:
                    decoded[0] += frame_bytes[0]
                frame_bytes[0] = 0
                prev = last_sig
                run_start = end

        async for data in request.content.iter_chunked(1 << 20):
            self.bytes_received += len(data)
            buf += data
            while not finished:
                eol = buf.find(b"\r\n", pos, pos + 128)
                if eol < 0:
                    if len(buf) - pos > 128:
                        raise _BadReq(400, "IncompleteBody", "malformed aws-chunked framing")
                    break
                m = _CHUNK_HDR.match(buf, pos, eol + 2)
                if not m:
                    raise _BadReq(400, "IncompleteBody", "malformed aws-chunked framing")
                n = int(m.group(1), 16)
                if len(buf) < eol + 2 + n + 2:
                    break
                last_sig = m.group(2).decode()
                pos = eol + 2 + n + 2
                frame_bytes[0] += n
                if n == 0:
                    finished = True
                elif pos - run_start >= (1 << 20):
                    dispatch(pos, False)
            if run_start:               # drop dispatched bytes (keeps buf ~1 run long)
                del buf[:run_start]
                pos -= run_start
                run_start = 0
        if not finished:
            raise _BadReq(400, "IncompleteBody", "missing final chunk")
        if pos != len(buf):
            raise _BadReq(400, "IncompleteBody", "trailing bytes after final chunk")
        dispatch(pos, True)
        results = await asyncio.gather(*runs)
        for ok, _d, err in results:
            if not ok:
                code = 403 if "signature" in err else 400
                raise _BadReq(code, "SignatureDoesNotMatch" if code == 403 else "IncompleteBody", err)
        data = b"".join(d for _ok, d, _e in results) if keep else _Sized(decoded[0])
        if decoded_len >= 0 and decoded_len != len(data):
            raise _BadReq(400, "IncompleteBody", "decoded length mismatch")
        return data

    async def _leaves(self, data) -> bytes | None:
        """Leaf hashes of a received body (free from the native verifier,
        else computed off the loop); None if unknown."""
        if isinstance(data, _Sized):
            return data.leaves or None
        from .payload import leaf_hashes
        return await asyncio.get_running_loop().run_in_executor(None, leaf_hashes, bytes(data))

    def _content_check(self, key: str, size: int, leaves: bytes | None) -> None:
        if self.expect is None:
            return
        want = self.expect.expected_for_key(key, size)
        if want is None:
            return
        if leaves is None or hashlib.sha256(leaves).digest() != want:
            self.counts["content_bad"] += 1
            raise _BadReq(400, "BadDigest", f"content of {key} is not the origin's payload")
        self.counts["content_ok"] += 1

    def _save(self, data: bytes, content_type: str = "") -> Obj:
        if self.store == "discard":
            # throughput mode: bytes were already verified (payload hash / chunk
            # signatures); skip the serial MD5 and return a size-derived ETag
            return Obj(len(data), f"{len(data):032x}", content_type=content_type)
        etag = hashlib.md5(data).hexdigest()
        if self.store == "disk":
            assert self.root
            p = os.path.join(self.root, f"obj-{next(self._ids)}")
            with open(p, "wb") as f:
                f.write(data)
            return Obj(len(data), etag, path=p, content_type=content_type)
        return Obj(len(data), etag, data=data, content_type=content_type)

    async def _handle(self, request: web.Request) -> web.StreamResponse:
        self.requests.append((request.method, request.raw_path))
        request.idle_timeout = self.idle_timeout
        outage = time.monotonic() < self._outage_until
        if outage or (self._fail > 0 and (not self._fail_methods or request.method in self._fail_methods)):
            if not outage:
                self._fail -= 1
            self.failed += 1
            try:
                await request.read()
            except (asyncio.TimeoutError, ConnectionError):
                request.transport.close()
            return _xml_err(self._fail_status, self._fail_code, "injected failure")
        request.signed_region = None
        auth = self._verify(request)
        if isinstance(auth, web.Response):
            await request.read()
            return auth
        bucket, key = self._split(request)
        q = dict(parse_qsl(request.query_string, keep_blank_values=True))
        # region check (AWS): requests on a bucket must be signed for its region;
        # GET ?location answers whatever the signing region
        breg = self.bucket_regions.get(bucket, self.region) if bucket in self.buckets else None
        sreg = request.signed_region
        if breg is not None and sreg is not None and sreg != breg and not (request.method == "GET" and not key
                                                                           and "location" in q):
            await request.read()
            r = _xml_err(400, "AuthorizationHeaderMalformed",
                         f"the region '{sreg}' is wrong; expecting '{breg}'", region=breg)
            r.headers["x-amz-bucket-region"] = breg
            return r
        try:
            if not key:
                return await self._bucket_op(request, bucket, q, auth)
            return await self._object_op(request, bucket, key, q, auth)
        except asyncio.TimeoutError:
            self.idle_timeouts += 1
            request.transport_close_after = True
            return _xml_err(400, "RequestTimeout", _IDLE_MSG)
        except _BadReq as e:
            if e.code == "RequestTimeout":
                self.idle_timeouts += 1
            return _xml_err(e.status, e.code, e.msg)

    async def _bucket_op(self, request: web.Request, bucket: str, q: dict, auth) -> web.StreamResponse:
        m = request.method
        if m == "HEAD":
            return web.Response(status=200 if bucket in self.buckets else 404)
        if m == "PUT":
            body = await self._read_body(request, auth)
            if bucket in self.buckets:
                return _xml_err(409, "BucketAlreadyOwnedByYou", "bucket exists")
            mm = re.search(rb"<LocationConstraint>([^<]*)</LocationConstraint>", bytes(body or b""))
            loc = mm.group(1).decode() if mm else "us-east-1"
            sreg = getattr(request, "signed_region", None)
            if sreg is not None and sreg != loc:
                return _xml_err(400, "AuthorizationHeaderMalformed",
                                f"the region '{sreg}' is wrong; expecting '{loc}'", region=loc)
            self.create_bucket(bucket, loc)
            return web.Response(status=200, headers={"Location": "/" + bucket})
        if m == "GET" and bucket in self.buckets:
            if "location" in q:
                reg = self.bucket_regions.get(bucket, self.region)
                val = "" if reg == "us-east-1" else reg
                body = (f'<?xml version="1.0" encoding="UTF-8"?><LocationConstraint '
                        f'xmlns="http://s3.amazonaws.com/doc/2006-03-01/">{val}</LocationConstraint>')
                return web.Response(body=body.encode(), content_type="application/xml")
            prefix = q.get("prefix", "")
            keys = sorted(k for k in self.buckets[bucket] if k.startswith(prefix))
            items = "".join(f"<Contents><Key>{_xml_escape(k)}</Key><Size>{self.buckets[bucket][k].size}</Size>"
                            f"<ETag>\"{self.buckets[bucket][k].etag}\"</ETag></Contents>" for k in keys)
            body = (f"<ListBucketResult xmlns=\"http://s3.amazonaws.com/doc/2006-03-01/\"><Name>{bucket}</Name>"
                    f"<Prefix>{prefix}</Prefix><KeyCount>{len(keys)}</KeyCount><IsTruncated>false</IsTruncated>"
                    f"{items}</ListBucketResult>")
            return web.Response(body=body.encode(), content_type="application/xml")
        if bucket not in self.buckets:
            return _xml_err(404, "NoSuchBucket", "The specified bucket does not exist")
        return _xml_err(405, "MethodNotAllowed", m)

    async def _object_op(self, request: web.Request, bucket: str, key: str, q: dict, auth) -> web.StreamResponse:
        m = request.method
        if bucket not in self.buckets:
            await request.read()
            return _xml_err(404, "NoSuchBucket", "The specified bucket does not exist")
        objs = self.buckets[bucket]
        if m == "PUT" and "uploadId" in q:
            up = self.uploads.get(q["uploadId"])
            if up is None:
                await request.read()
                return _xml_err(404, "NoSuchUpload", "no such upload")
            pn = int(q.get("partNumber", "0") or 0)
            if pn in self.fail_parts:
                if self.fail_parts_once:
                    self.fail_parts.discard(pn)
                await request.read()
                return _xml_err(500, "InternalError", "injected part failure")
            if self.strict_parts and not 1 <= pn <= 10000:
                await request.read()
                return _xml_err(400, "InvalidArgument", "Part number must be an integer between 1 and 10000")
            data = await self._read_body(request, auth, keep=self.store != "discard")
            o = self._save(data)
            if self.expect is not None:
                o.leaves = await self._leaves(data)
            up.parts[int(q["partNumber"])] = o
            return web.Response(status=200, headers={"ETag": f"\"{o.etag}\""})
        if m == "PUT":
            data = await self._read_body(request, auth, keep=self.store != "discard")
            if self.expect is not None:
                self._content_check(key, len(data), await self._leaves(data))
            o = self._save(data, request.headers.get("Content-Type", ""))
            objs[key] = o
            return web.Response(status=200, headers={"ETag": f"\"{o.etag}\""})
        if m == "POST" and "uploads" in q:
            await self._read_body(request, auth)
            uid = f"upload-{next(self._ids)}"
            self.uploads[uid] = Upload(bucket, key)
            body = (f"<InitiateMultipartUploadResult xmlns=\"http://s3.amazonaws.com/doc/2006-03-01/\">"
                    f"<Bucket>{bucket}</Bucket><Key>{_xml_escape(key)}</Key><UploadId>{uid}</UploadId>"
                    f"</InitiateMultipartUploadResult>")
            return web.Response(body=body.encode(), content_type="application/xml")
        if m == "POST" and "uploadId" in q:
            body = await self._read_body(request, auth)
            if self.complete_error_200 > 0 and q["uploadId"] in self.uploads:
                self.complete_error_200 -= 1
                eb = (f"<Error><Code>{self.complete_error_code}</Code><Message>We encountered an internal "
                      f"error. Please try again.</Message><Resource>{_xml_escape(key)}</Resource></Error>")
                return web.Response(body=eb.encode(), content_type="application/xml")
            up = self.uploads.pop(q["uploadId"], None)
            if up is None:
                return _xml_err(404, "NoSuchUpload", "no such upload")
            nums = [int(x) for x in re.findall(rb"<PartNumber>(\d+)</PartNumber>", body)]
            tags = [x.decode().strip('"') for x in re.findall(rb"<ETag>([^<]*)</ETag>", body)]
            if nums != sorted(nums) or any(up.parts.get(n) is None or up.parts[n].etag != t
                                           for n, t in zip(nums, tags)):
                return _xml_err(400, "InvalidPart", "parts mismatch")
            if self.strict_parts and (len(nums) > 10000 or
                                      any(up.parts[n].size < (5 << 20) for n in nums[:-1])):
                return _xml_err(400, "EntityTooSmall", "Your proposed upload is smaller than the minimum "
                                "allowed object size.")
            if self.expect is not None:
                aligned = all(up.parts[n].size % (64 << 10) == 0 for n in nums[:-1])
                parts_leaves = [up.parts[n].leaves for n in nums]
                self._content_check(up.key, sum(up.parts[n].size for n in nums),
                                    b"".join(parts_leaves) if aligned and all(parts_leaves) else None)
            if self.store == "memory":
                data = b"".join(up.parts[n].data or b"" for n in nums)
                o = self._save(data)
            else:
                size = sum(up.parts[n].size for n in nums)
                o = Obj(size, "")
                if self.store == "disk":
                    assert self.root
                    p = os.path.join(self.root, f"obj-{next(self._ids)}")
                    with open(p, "wb") as f:
                        for n in nums:
                            with open(up.parts[n].path or "", "rb") as pf:
                                f.write(pf.read())
                    o.path = p
            md5s = b"".join(bytes.fromhex(up.parts[n].etag) for n in nums)
            o.etag = hashlib.md5(md5s).hexdigest() + f"-{len(nums)}"
            objs[up.key] = o
            if self.complete_lose_reply > 0:
                self.complete_lose_reply -= 1
                return _xml_err(503, "ServiceUnavailable", "reply lost after commit")
            rb = (f"<CompleteMultipartUploadResult xmlns=\"http://s3.amazonaws.com/doc/2006-03-01/\">"
                  f"<Bucket>{bucket}</Bucket><Key>{_xml_escape(up.key)}</Key><ETag>\"{o.etag}\"</ETag>"
                  f"</CompleteMultipartUploadResult>")
            return web.Response(body=rb.encode(), content_type="application/xml")
        if m == "DELETE" and "uploadId" in q:
            self.uploads.pop(q["uploadId"], None)
            return web.Response(status=204)
        if m == "GET" and "uploadId" in q:                   # ListParts, paged like S3 (max-parts, marker)
            up = self.uploads.get(q["uploadId"])
            if up is None or up.key != key:
                return _xml_err(404, "NoSuchUpload", "The specified upload does not exist.")
            marker = int(q.get("part-number-marker", "0") or 0)
            maxp = int(q.get("max-parts", str(self.list_parts_page)) or self.list_parts_page)
            nums = sorted(n for n in up.parts if n > marker)
            page, more = nums[:maxp], len(nums) > maxp
            xml = "".join(f"<Part><PartNumber>{n}</PartNumber><ETag>\"{up.parts[n].etag}\"</ETag>"
                          f"<Size>{up.parts[n].size}</Size></Part>" for n in page)
            body = (f"<ListPartsResult xmlns=\"http://s3.amazonaws.com/doc/2006-03-01/\"><Bucket>{bucket}</Bucket>"
                    f"<Key>{_xml_escape(key)}</Key><UploadId>{q['uploadId']}</UploadId>"
                    f"<PartNumberMarker>{marker}</PartNumberMarker>"
                    f"<NextPartNumberMarker>{page[-1] if page else marker}</NextPartNumberMarker>"
                    f"<MaxParts>{maxp}</MaxParts><IsTruncated>{'true' if more else 'false'}</IsTruncated>"
                    f"{xml}</ListPartsResult>")
            return web.Response(body=body.encode(), content_type="application/xml")
        if m in ("GET", "HEAD"):
            o = objs.get(key)
            if o is None:
                return _xml_err(404, "NoSuchKey", "The specified key does not exist.")
            hdrs = {"ETag": f"\"{o.etag}\"", "Content-Length": str(o.size)}
            if m == "HEAD":
                return web.Response(status=200, headers=hdrs)
            return web.Response(status=200, body=self.object_bytes(bucket, key), headers={"ETag": hdrs["ETag"]})
        if m == "DELETE":
            objs.pop(key, None)
            return web.Response(status=204)
        return _xml_err(405, "MethodNotAllowed", m)


class _Sized:
    """Length-only stand-in for a verified body we chose not to keep (with
    the 64 KiB leaf hashes of its content, when the verifier had them)."""

    __slots__ = ("n", "leaves")

    def __init__(self, n: int, leaves: bytes | None = None) -> None:
        self.n = n
        self.leaves = leaves

    def __len__(self) -> int:
        return self.n


class _BadReq(Exception):
    def __init__(self, status: int, code: str, msg: str) -> None:
        super().__init__(msg)
        self.status, self.code, self.msg = status, code, msg


def _xml_escape(s: str) -> str:
    return s.replace("&", "&amp;").replace("<", "&lt;").replace(">", "&gt;")


async def _main() -> None:  # pragma: no cover - manual use
    s = await FakeS3(port=9000).start()
    print("fake s3 on", s.endpoint, flush=True)
    await asyncio.Event().wait()
