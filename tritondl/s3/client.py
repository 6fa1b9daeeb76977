"""Async S3 client (aiohttp) with SigV4, bucket ensure, streaming PutObject
and parallel multipart upload.

Capability of the minio-go v6 calls the reference makes
(``internal/uploader/uploader.go:43-51,64-65,89``): ``NewWithOptions{Secure,
Creds, BucketLookupAuto}``, ``BucketExists``, ``MakeBucket``,
``PutObjectWithContext`` (single PUT below the multipart threshold, multipart
above it).  Memory stays O(part_size × parallel_parts) regardless of file
size; file reads and chunk signing run in worker threads
(the native hash module releases the GIL), so several uploads overlap.
"""

from __future__ import annotations

import asyncio
import os
import re
import xml.etree.ElementTree as ET
from dataclasses import dataclass
from typing import AsyncIterator
from urllib.parse import urlparse

import aiohttp
from multidict import CIMultiDict
from yarl import URL

from ..ops import hashing
from ..utils.backoff import ExponentialBackoff
from ..utils import rawhttp
from ..utils.log import log
from . import sigv4
from .credentials import Chain, Provider, Value, default_chain

S3_NS = "{http://s3.amazonaws.com/doc/2006-03-01/}"
_DNS_BUCKET = re.compile(r"^[a-z0-9][a-z0-9.-]{1,61}[a-z0-9]$")


class S3Error(Exception):
    def __init__(self, status: int, code: str = "", message: str = "", resource: str = "") -> None:
        super().__init__(f"S3 {status} {code}: {message} ({resource})")
        self.status, self.code, self.message, self.resource = status, code, message, resource


def _parse_error(status: int, body: bytes, resource: str) -> S3Error:
    code = msg = ""
    try:
        root = ET.fromstring(body)
        code = (root.findtext("Code") or "")
        msg = (root.findtext("Message") or "")
    except ET.ParseError:
        msg = body[:200].decode(errors="replace")
    return S3Error(status, code, msg, resource)


@dataclass
class Endpoint:
    host: str           # host[:port] as sent in the Host header
    secure: bool

    @classmethod
    def parse(cls, s3_endpoint: str) -> "Endpoint":
        """Reference parsing of ``S3_ENDPOINT`` (``uploader.go:25-40``): TLS iff
        scheme is https; keep hostname[:port]."""
        if s3_endpoint and "://" not in s3_endpoint:
            s3_endpoint = "http://" + s3_endpoint  # bare host[:port] (Go would yield an empty host)
        u = urlparse(s3_endpoint)
        host = u.hostname or ""
        if u.port:
            host = f"{host}:{u.port}"
        return cls(host, u.scheme == "https")

    @property
    def base(self) -> str:
        return ("https://" if self.secure else "http://") + self.host


class S3Client:
    def __init__(self, endpoint: Endpoint | str, creds: Provider | None = None, *, region: str = "us-east-1",
                 lookup: str = "auto", payload_mode: str = "auto", part_size: int = 64 << 20,
                 multipart_threshold: int = 64 << 20, parallel_parts: int = 4, max_retries: int = 5,
                 io_block: int = 4 << 20, session: aiohttp.ClientSession | None = None,
                 native: bool = True, sign_threads: int = 4) -> None:
        self.ep = Endpoint.parse(endpoint) if isinstance(endpoint, str) else endpoint
        self.creds = creds or default_chain()
        self.region = region
        self.lookup = lookup
        self.payload_mode = payload_mode
        self.part_size = max(part_size, 5 << 20)
        self.multipart_threshold = multipart_threshold
        self.parallel_parts = max(1, parallel_parts)
        self.max_retries = max_retries
        self.io_block = max(io_block, sigv4.STREAM_CHUNK)
        self._session = session
        self._own_session = session is None
        # native data plane (csrc/relay): file/fd PUT bodies over plain http
        self.native = native
        self.sign_threads = sign_threads
        self._raw = rawhttp.Pool()

    async def _sess(self) -> aiohttp.ClientSession:
        if self._session is None or self._session.closed:
            self._session = aiohttp.ClientSession(
                timeout=aiohttp.ClientTimeout(total=None, sock_connect=30, sock_read=300),
                connector=aiohttp.TCPConnector(limit=64), auto_decompress=False)
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

    def _target(self, bucket: str, key: str = "") -> tuple[str, str]:
        ekey = sigv4.uri_encode(key, encode_slash=False) if key else ""
        if self._virtual(bucket):
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

    async def _do(self, method: str, bucket: str, key: str = "", query: dict | None = None,
                  headers: dict | None = None, body: bytes | None = None, *, body_factory=None,
                  payload_hash: str | None = None, expect: tuple[int, ...] = (200,),
                  retry: bool = True) -> tuple[int, dict, bytes]:
        """One signed request with retries on connection errors / 5xx."""
        pol = ExponentialBackoff(initial=0.2, multiplier=2, max_interval=5, max_elapsed=None)
        attempt = 0
        while True:
            attempt += 1
            host, path = self._target(bucket, key)
            amzdate, _ = sigv4.amz_dates()
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
                                    self.region, amzdate, path_is_encoded=True)
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
                async with sess.request(method, url, headers=send_headers, data=payload,
                                        skip_auto_headers=("Content-Type",)) as r:
                    rbody = await r.read()
                    if r.status in expect:
                        return r.status, CIMultiDict(r.headers), rbody
                    err = _parse_error(r.status, rbody, f"{method} {path}")
                    if r.status < 500 or not retry or attempt > self.max_retries:
                        raise err
            except (aiohttp.ClientError, asyncio.TimeoutError, ConnectionError) as e:
                if not retry or attempt > self.max_retries:
                    raise S3Error(0, "ConnectionError", str(e), f"{method} {path}") from e
                err = e  # type: ignore[assignment]
            d = pol.next_delay() or 1.0
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
        body = None
        if location and location != "us-east-1":
            body = (f'<CreateBucketConfiguration xmlns="http://s3.amazonaws.com/doc/2006-03-01/">'
                    f"<LocationConstraint>{location}</LocationConstraint></CreateBucketConfiguration>").encode()
        await self._do("PUT", bucket, body=body if body is not None else b"", expect=(200,))

    # ------------------------------------------------------------ objects
    async def put_object(self, bucket: str, key: str, src: str | bytes | int, size: int | None = None,
                         content_type: str = "application/octet-stream", wait_bytes=None, flow=None) -> str:
        """Upload a file path or fd (streamed) or bytes; returns the ETag.

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
        if size >= self.multipart_threshold and size > self.part_size:
            return await self._put_multipart(bucket, key, src, size, content_type, wait_bytes, flow)
        return await self._put_range(bucket, key, src, 0, size, {"content-type": content_type},
                                     wait_bytes=wait_bytes, flow=flow)

    async def _put_range(self, bucket: str, key: str, src: str | bytes | int, offset: int, length: int,
                         headers: dict, query: dict | None = None, wait_bytes=None, flow=None) -> str:
        mode = self._payload_mode()
        relay = rawhttp.relay_module() if self.native else None
        if relay is not None and not self.ep.secure and mode in ("streaming", "unsigned") and \
                not isinstance(src, (bytes, bytearray, memoryview)) and (flow is not None or wait_bytes is None):
            return await self._put_native(relay, bucket, key, src, offset, length, headers, query, mode, flow)
        factory = _BodyFactory(self, src, offset, length, mode, wait_bytes)
        _st, rh, _b = await self._do("PUT", bucket, key, query=query, headers=headers, body_factory=factory)
        return rh.get("ETag", "").strip('"')

    async def _put_multipart(self, bucket: str, key: str, src: str | bytes | int, size: int, content_type: str,
                             wait_bytes=None, flow=None) -> str:
        _st, _h, body = await self._do("POST", bucket, key, query={"uploads": ""},
                                       headers={"content-type": content_type}, body=b"")
        root = ET.fromstring(body)
        upload_id = root.findtext(f"{S3_NS}UploadId") or root.findtext("UploadId") or ""
        if not upload_id:
            raise S3Error(0, "MalformedXML", "no UploadId in InitiateMultipartUpload response")
        nparts = (size + self.part_size - 1) // self.part_size
        etags: list[str] = [""] * nparts
        todo = list(range(nparts))

        def pick() -> int:
            # Following a download: take the part that will be on disk soonest (a segmented
            # download fills several regions at once; in part order the uploads would queue
            # behind the first segment).  Otherwise in order.
            if flow is None or len(todo) == 1:
                return todo.pop(0)
            best = min(range(len(todo)), key=lambda k: (flow.bytes_until_covered(
                todo[k] * self.part_size, min(size, (todo[k] + 1) * self.part_size)), todo[k]))
            return todo.pop(best)

        async def worker() -> None:
            while todo:
                i = pick()
                off = i * self.part_size
                ln = min(self.part_size, size - off)
                etags[i] = await self._put_range(bucket, key, src, off, ln, {},
                                                 query={"partNumber": str(i + 1), "uploadId": upload_id},
                                                 wait_bytes=wait_bytes, flow=flow)
        try:
            await asyncio.gather(*(worker() for _ in range(min(self.parallel_parts, nparts))))
            xml = "".join(f"<Part><PartNumber>{i + 1}</PartNumber><ETag>\"{e}\"</ETag></Part>"
                          for i, e in enumerate(etags))
            cbody = f"<CompleteMultipartUpload>{xml}</CompleteMultipartUpload>".encode()
            _st, _h, rb = await self._do("POST", bucket, key, query={"uploadId": upload_id}, body=cbody)
            if b"<Error>" in rb:
                raise _parse_error(200, rb, f"complete {key}")
            r = ET.fromstring(rb)
            return (r.findtext(f"{S3_NS}ETag") or r.findtext("ETag") or "").strip('"')
        except BaseException:
            try:
                await self._do("DELETE", bucket, key, query={"uploadId": upload_id}, expect=(204, 200),
                               retry=False)
            except Exception:
                pass
            raise

    async def _put_native(self, relay, bucket: str, key: str, src: str | int, offset: int, length: int,
                          headers: dict, query: dict | None, mode: str, flow) -> str:
        """One PUT whose body never enters Python: the head is signed here,
        then ``_relay.send_body`` writes head + body (aws-chunked with chunk
        signatures hashed on a native pool, or sendfile for unsigned) from the
        file straight to the socket; the reply is parsed here.  Same retry
        policy as :meth:`_do` (connection errors and 5xx)."""
        loop = asyncio.get_running_loop()
        pol = ExponentialBackoff(initial=0.2, multiplier=2, max_interval=5, max_elapsed=None)
        fd = os.dup(src) if isinstance(src, int) else os.open(src, os.O_RDONLY)
        attempt = 0
        try:
            while True:
                attempt += 1
                cred = self._creds()
                m = "unsigned" if (cred.anonymous and mode == "streaming") else mode
                host, path = self._target(bucket, key)
                amzdate, _ = sigv4.amz_dates()
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
                                        cred.secret_access_key, self.region, amzdate, path_is_encoded=True)
                    hdrs["authorization"] = signed.authorization
                target = path + (("?" + sigv4.canonical_query(query)) if query else "")
                send = {"Host": host, **{k: v for k, v in hdrs.items() if k != "host"}}
                head = rawhttp.request_head("PUT", target, send)
                chost, cport = rawhttp.split_host(host)
                err: Exception | None = None
                sock = None
                try:
                    sock, reused = await self._raw.connect(chost, cport)
                    rawhttp.trace("put_pump_start")
                    sent, _last, perr = await loop.run_in_executor(
                        None, relay.send_body, sock.fileno(), head, fd, offset, length, flow,
                        1 if m == "streaming" else 0, signed.key if signed else b"", amzdate,
                        signed.scope if signed else "", signed.signature if signed else "", sigv4.STREAM_CHUNK,
                        self.sign_threads, 300.0)
                    if perr and ("source" in perr or perr == "cancelled"):
                        raise S3Error(0, "SourceFailed", perr, f"PUT {path}")
                    try:
                        resp = await rawhttp.read_head(sock, 1.0 if perr else 300.0)
                    except rawhttp.RawHTTPError:
                        if perr:
                            if reused and sent == 0:
                                attempt -= 1          # stale keep-alive socket: not a real attempt
                            raise rawhttp.RawHTTPError(perr)
                        raise
                    rawhttp.trace("put_pump_end")
                    body = await rawhttp.read_small_body(sock, resp, 60.0, method="PUT")
                    rawhttp.trace("put_response")
                    if resp.status == 200 and not perr:
                        if resp.keep_alive:
                            self._raw.release(chost, cport, sock)
                            sock = None
                        return resp.headers.get("ETag", "").strip('"')
                    err = _parse_error(resp.status, body, f"PUT {path}")
                    if resp.status < 500 or attempt > self.max_retries:
                        raise err
                except (rawhttp.RawHTTPError, OSError, asyncio.TimeoutError) as e:
                    if attempt > self.max_retries:
                        raise S3Error(0, "ConnectionError", str(e), f"PUT {path}") from e
                    err = e
                finally:
                    if sock is not None:
                        sock.close()
                if attempt <= 0:
                    continue
                d = pol.next_delay() or 1.0
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
            root = ET.fromstring(b)
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
