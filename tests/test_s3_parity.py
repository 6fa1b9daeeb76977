"""minio-go library behaviours the reference relied on without naming them
(internal/uploader/uploader.go:43-51,64-70,89; cmd/downloader/downloader.go:95-98):
bucket-region discovery, 10,000-part sizing, fatal endpoint validation,
and healing when the bucket disappears."""

import asyncio
import os
import time

import pytest

from tritondl_testkit.fakes.s3 import FakeS3
from tritondl.s3.client import (MAX_OBJECT_SIZE, MAX_PARTS, Endpoint, S3Client, S3Error, _PartQueue,
                                plan_parts)
from tritondl.s3.credentials import Static
from tritondl.s3.uploader import Uploader, object_key


def run(coro, timeout=60):
    return asyncio.run(asyncio.wait_for(coro, timeout))


# --------------------------------------------------------------- endpoint

@pytest.mark.parametrize("bad", ["", "   ", "http://", "ftp://minio:9000", "http://exa mple:9000",
                                 "http://minio:99999", "http://minio:9000/some/path", "https://-bad-.host"])
def test_endpoint_rejects_what_minio_refuses(bad):
    with pytest.raises(ValueError):
        Endpoint.parse(bad)


@pytest.mark.parametrize("good,host,secure", [("http://minio:9000", "minio:9000", False),
                                              ("https://s3.eu-west-1.amazonaws.com", "s3.eu-west-1.amazonaws.com", True),
                                              ("127.0.0.1:9000", "127.0.0.1:9000", False),
                                              ("http://[::1]:9000", "[::1]:9000", False)])
def test_endpoint_accepts(good, host, secure):
    ep = Endpoint.parse(good)
    assert (ep.host, ep.secure) == (host, secure)


def test_uploader_from_env_fails_fast_on_empty_endpoint():
    with pytest.raises(ValueError, match="S3_ENDPOINT"):
        Uploader.from_env("triton-staging", "")


# --------------------------------------------------------------- part sizing

def test_plan_parts_minio_optimal_sizes():
    mib, gib, tib = 1 << 20, 1 << 30, 1 << 40
    assert plan_parts(100 * mib, 64 * mib) == (64 * mib, 2)
    ps, n = plan_parts(700 * gib, 64 * mib)          # 11,200 parts at 64 MiB: too many
    assert ps == 128 * mib and n == 5600 and n <= MAX_PARTS
    ps, n = plan_parts(5 * tib, 64 * mib)            # minio optimalPartInfo: 576 MiB, 9103 parts
    assert ps == 576 * mib and n == 9103
    assert (n - 1) * ps < 5 * tib <= n * ps
    with pytest.raises(S3Error, match="EntityTooLarge"):
        plan_parts(MAX_OBJECT_SIZE + 1, 64 * mib)
    # tiny configured part sizes are lifted to S3's 5 MiB minimum
    assert plan_parts(12 * mib, 1 * mib) == (5 * mib, 3)


class _FakeFlow:
    """Segments filling from their starts at different speeds (Flow stand-in)."""

    def __init__(self, size, nseg, done):
        self.size = size
        step = -(-size // nseg)
        self.segs = [[i * step, min(size, (i + 1) * step)] for i in range(nseg)]
        self.done = done
        self.finished = False
        self.calls = 0

    def open_starts(self):
        return [s for (s, e), d in zip(self.segs, self.done) if s + d < e]

    def bytes_until_covered(self, a, b):
        self.calls += 1
        worst = 0
        for (s, e), d in zip(self.segs, self.done):
            hi = min(b, e)
            if hi <= max(a, s):
                continue
            if hi > s + d:
                worst = max(worst, hi - (s + d))
        return worst


def test_part_queue_picks_arrival_order_and_scales():
    ps = 5 << 20
    nparts = MAX_PARTS
    size = nparts * ps
    flow = _FakeFlow(size, 4, [0, 3 * ps, 0, 7 * ps])
    q = _PartQueue(nparts, ps, size, flow)
    # parts already on disk first (lowest number on ties): segment 1's three,
    # then segment 3's seven; then the part nearest its frontier
    picked = [q.pick() for _ in range(11)]
    assert picked == [2500, 2501, 2502, 7500, 7501, 7502, 7503, 7504, 7505, 7506, 0]
    t0 = time.perf_counter()
    seen = set(picked)
    while q:
        seen.add(q.pick())
    assert seen == set(range(nparts))
    # bounded work per pick (candidates = run starts + segment heads), not O(pending)
    assert flow.calls < 20 * nparts, flow.calls
    assert time.perf_counter() - t0 < 5.0


# --------------------------------------------------------------- regions

def test_region_discovery_signs_with_bucket_region():
    """No S3_REGION: the client asks GET ?location once and signs every later
    request for eu-west-1 (a us-east-1 signature would be refused)."""
    async def main():
        s3 = await FakeS3(access_key="ak", secret_key="sk").start()
        s3.create_bucket("media-eu", "eu-west-1")
        c = S3Client(s3.endpoint, Static("ak", "sk"), region="")
        assert await c.bucket_region("media-eu") == "eu-west-1"
        up = Uploader("media-eu", c)
        data = os.urandom(300_000)
        p = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"eu-{os.getpid()}.mkv")
        with open(p, "wb") as f:
            f.write(data)
        res = await up.upload_files("m1", os.path.dirname(p), [p])
        assert s3.object_bytes("media-eu", res[0].key) == data
        assert sum(1 for m, path in s3.requests if "location" in path) == 1      # cached
        os.remove(p)
        await up.close()
        await s3.stop()
    run(main())


def test_wrong_region_reply_is_learned_and_retried():
    """A stale cached region (bucket moved) → AuthorizationHeaderMalformed
    naming the right one → re-signed without spending a retry."""
    async def main():
        s3 = await FakeS3(access_key="ak", secret_key="sk").start()
        s3.create_bucket("b", "ap-south-1")
        c = S3Client(s3.endpoint, Static("ak", "sk"), region="", max_retries=0)
        c._regions["b"] = "us-east-1"
        etag = await c.put_object("b", "k", b"x" * 1000)
        assert etag and c._regions["b"] == "ap-south-1"
        # the native (file) path learns too
        c._regions["b"] = "us-west-2"
        p = f"/tmp/regional-{os.getpid()}"
        with open(p, "wb") as f:
            f.write(os.urandom(200_000))
        await c.put_object("b", "k2", p)
        assert c._regions["b"] == "ap-south-1"
        os.remove(p)
        await c.close()
        await s3.stop()
    run(main())


def test_explicit_region_is_not_overridden():
    async def main():
        s3 = await FakeS3(access_key="ak", secret_key="sk").start()
        s3.create_bucket("b", "eu-west-1")
        c = S3Client(s3.endpoint, Static("ak", "sk"), region="us-east-1", max_retries=0)
        with pytest.raises(S3Error, match="AuthorizationHeaderMalformed"):
            await c.put_object("b", "k", b"abc")
        await c.close()
        await s3.stop()
    run(main())


def test_make_bucket_in_discovered_default_region():
    async def main():
        s3 = await FakeS3(access_key="ak", secret_key="sk").start()
        up = Uploader("fresh", S3Client(s3.endpoint, Static("ak", "sk")))
        await up.ensure_bucket()
        assert s3.bucket_regions["fresh"] == "us-east-1"
        await up.close()
        await s3.stop()
    run(main())


# --------------------------------------------------------------- bucket healing

def test_deleted_then_recreated_bucket_heals_without_restart(tmp_path):
    async def main():
        s3 = await FakeS3(access_key="ak", secret_key="sk").start()
        up = Uploader("triton-staging", S3Client(s3.endpoint, Static("ak", "sk"), region=""))
        f1 = tmp_path / "a.mkv"
        f1.write_bytes(os.urandom(100_000))
        await up.upload_files("m1", str(tmp_path), [str(f1)])
        # operator deletes the bucket (and it comes back elsewhere, or not at all)
        s3.delete_bucket("triton-staging")
        f2 = tmp_path / "b.mkv"
        f2.write_bytes(os.urandom(150_000))
        res = await up.upload_files("m2", str(tmp_path), [str(f2)])
        assert s3.object_bytes("triton-staging", res[0].key) == f2.read_bytes()
        assert up.heals == 1
        # recreated in another region while we hold a cached region
        s3.delete_bucket("triton-staging")
        s3.create_bucket("triton-staging", "eu-central-1")
        res = await up.upload_files("m3", str(tmp_path), [str(f1)])
        assert res[0].key == object_key("m3", "a.mkv")
        assert up.client._regions["triton-staging"] == "eu-central-1"
        await up.close()
        await s3.stop()
    run(main())


# --------------------------------------------------------------- part limits

def test_fake_s3_enforces_part_limits():
    async def main():
        s3 = await FakeS3(access_key="ak", secret_key="sk").start()
        s3.create_bucket("b")
        c = S3Client(s3.endpoint, Static("ak", "sk"), max_retries=0)
        st, _h, body = await c._do("POST", "b", "k", query={"uploads": ""}, body=b"")
        uid = body.split(b"<UploadId>")[1].split(b"</UploadId>")[0].decode()
        with pytest.raises(S3Error, match="InvalidArgument"):
            await c._put_range("b", "k", b"x" * 10, 0, 10, {}, query={"partNumber": "10001", "uploadId": uid})
        e1 = await c._put_range("b", "k", b"x" * 10, 0, 10, {}, query={"partNumber": "1", "uploadId": uid})
        e2 = await c._put_range("b", "k", b"y" * 10, 0, 10, {}, query={"partNumber": "2", "uploadId": uid})
        xml = (f"<CompleteMultipartUpload><Part><PartNumber>1</PartNumber><ETag>\"{e1}\"</ETag></Part>"
               f"<Part><PartNumber>2</PartNumber><ETag>\"{e2}\"</ETag></Part></CompleteMultipartUpload>")
        with pytest.raises(S3Error, match="EntityTooSmall"):
            await c._do("POST", "b", "k", query={"uploadId": uid}, body=xml.encode())
        await c.close()
        await s3.stop()
    run(main())


def test_multipart_upload_respects_limits_end_to_end(tmp_path):
    async def main():
        s3 = await FakeS3(access_key="ak", secret_key="sk").start()
        s3.create_bucket("b")
        c = S3Client(s3.endpoint, Static("ak", "sk"), part_size=5 << 20, multipart_threshold=5 << 20)
        data = os.urandom((12 << 20) + 12345)
        p = tmp_path / "big.bin"
        p.write_bytes(data)
        await c.put_object("b", "big", str(p))
        assert s3.object_bytes("b", "big") == data
        assert s3.buckets["b"]["big"].etag.endswith("-3")
        await c.close()
        await s3.stop()
    run(main())


# --------------------------------------------------------------- resumable multipart

def test_interrupted_multipart_upload_resumes_from_landed_parts(tmp_path):
    """Beyond minio-go (which starts a failed multipart upload over): with a
    state file the upload is kept open on failure, and the retry lists its
    parts (paged), re-sends only parts S3 does not hold — a part whose local
    bytes no longer match its ETag (MD5) is re-sent — and completes it."""
    async def main():
        s3 = await FakeS3(access_key="ak", secret_key="sk", store="memory").start()
        s3.create_bucket("b")
        s3.list_parts_page = 1                               # exercise ListParts paging
        c = S3Client(s3.endpoint, Static("ak", "sk"), part_size=5 << 20, multipart_threshold=5 << 20,
                     parallel_parts=1, max_retries=0)
        data = bytearray(os.urandom((17 << 20) + 999))       # 4 parts
        p = tmp_path / "show.mkv"
        p.write_bytes(data)
        state = str(p) + ".s3upload"
        s3.fail_parts = {3}
        with pytest.raises(S3Error):
            await c.put_object("b", "k", str(p), resume_path=state)
        assert os.path.exists(state) and len(s3.uploads) == 1          # kept open, not aborted
        up = next(iter(s3.uploads.values()))
        assert sorted(up.parts) == [1, 2]
        # the local bytes of part 2 changed since (re-downloaded file): it must go again
        data[(5 << 20) + 10] ^= 0xFF
        p.write_bytes(data)
        s3.fail_parts = set()
        n0 = len(s3.requests)
        await c.put_object("b", "k", str(p), resume_path=state)
        sent = [r[1] for r in s3.requests[n0:] if r[0] == "PUT"]
        assert sorted(int(x.split("partNumber=")[1].split("&")[0]) for x in sent) == [2, 3, 4]
        assert s3.object_bytes("b", "k") == bytes(data)
        assert not os.path.exists(state) and not s3.uploads
        # without a state file a failure aborts the upload (minio-go behaviour)
        s3.fail_parts = {2}
        with pytest.raises(S3Error):
            await c.put_object("b", "k2", str(p))
        assert not s3.uploads
        await c.close()
        await s3.stop()
    run(main())


def test_complete_multipart_200_error_and_lost_reply(tmp_path):
    """S3 quirks of CompleteMultipartUpload: a 200 whose body is <Error>
    (InternalError/SlowDown: retried in place, the parts are not re-sent; any
    other code fails the upload), and a reply lost after the commit (the
    retry answers NoSuchUpload; the object's multipart ETag proves it landed)."""
    from tritondl.s3.client import multipart_etag
    async def main():
        s3 = await FakeS3(access_key="ak", secret_key="sk", store="memory").start()
        s3.create_bucket("b")
        c = S3Client(s3.endpoint, Static("ak", "sk"), part_size=5 << 20, multipart_threshold=5 << 20)
        data = os.urandom((10 << 20) + 7)
        p = tmp_path / "f.bin"
        p.write_bytes(data)

        s3.complete_error_200 = 2
        n0 = len(s3.requests)
        etag = await c.put_object("b", "k1", str(p))
        assert s3.object_bytes("b", "k1") == data and s3.buckets["b"]["k1"].etag == etag
        reqs = s3.requests[n0:]
        assert sum(1 for m, u in reqs if m == "PUT") == 3                  # each part went once
        assert sum(1 for m, u in reqs if m == "POST" and "uploadId" in u) == 3
        assert not s3.uploads

        s3.complete_lose_reply = 1
        etag = await c.put_object("b", "k2", str(p))
        assert etag == s3.buckets["b"]["k2"].etag and etag.endswith("-3")
        assert s3.object_bytes("b", "k2") == data

        # a non-transient 200 error fails (and aborts) the upload
        s3.complete_error_200, s3.complete_error_code = 1, "InvalidPart"
        with pytest.raises(S3Error) as ei:
            await c.put_object("b", "k3", str(p))
        assert ei.value.code == "InvalidPart" and "k3" not in s3.buckets["b"] and not s3.uploads
        await c.close()
        await s3.stop()
    run(main())
    md5 = __import__("hashlib").md5
    a, b = md5(b"x").hexdigest(), md5(b"y").hexdigest()
    assert multipart_etag([f'"{a}"', b]) == md5(bytes.fromhex(a) + bytes.fromhex(b)).hexdigest() + "-2"
    assert multipart_etag(["not-an-md5"]) == "" and multipart_etag([]) == ""


@pytest.mark.parametrize("offset", [3600.0, -7200.0])
def test_clock_skew_is_learned_from_request_time_too_skewed(tmp_path, offset):
    """A node whose clock drifted past S3's 15-minute window gets 403
    RequestTimeTooSkewed naming S3's time; the client signs on S3's clock
    from then on (one refusal, not one per request) on the aiohttp path, the
    native PUT pump and multipart."""
    async def main():
        s3 = await FakeS3(access_key="ak", secret_key="sk", store="memory").start()
        s3.create_bucket("b")
        s3.clock_offset = offset
        c = S3Client(s3.endpoint, Static("ak", "sk"), region="us-east-1", max_retries=0,
                     part_size=5 << 20, multipart_threshold=5 << 20)
        # the uploader's first request is a HEAD bucket: its 403 has no body, S3's Date tells
        h = S3Client(s3.endpoint, Static("ak", "sk"), region="us-east-1", max_retries=0)
        assert await h.bucket_exists("b") and abs(h.clock_skew - offset) < 5 and s3.skew_refusals == 1
        await h.close()
        await c.put_object("b", "small", b"x" * 1000)
        assert abs(c.clock_skew - offset) < 5 and s3.skew_refusals == 2
        small = tmp_path / "s.bin"
        small.write_bytes(os.urandom(300_000))
        big = tmp_path / "b.bin"
        big.write_bytes(os.urandom((11 << 20) + 3))
        await c.put_object("b", "file", str(small))
        await c.put_object("b", "multi", str(big))
        assert s3.object_bytes("b", "multi") == big.read_bytes() and s3.skew_refusals == 2
        # a fresh client learns it on the native PUT path too
        c2 = S3Client(s3.endpoint, Static("ak", "sk"), region="us-east-1", max_retries=0)
        await c2.put_object("b", "file2", str(small))
        assert abs(c2.clock_skew - offset) < 5 and s3.object_bytes("b", "file2") == small.read_bytes()
        # the server's clock moves back: the skew is re-learned, never looped on
        s3.clock_offset = 0.0
        await c2.put_object("b", "file3", str(small))
        assert abs(c2.clock_skew) < 5
        await c.close()
        await c2.close()
        await s3.stop()
    run(main())


def test_server_time_parsing():
    from tritondl.s3.client import _parse_error
    body = (b"<Error><Code>RequestTimeTooSkewed</Code><Message>m</Message><RequestTime>20260101T000000Z"
            b"</RequestTime><ServerTime>2026-10-18T02:40:49.123Z</ServerTime></Error>")
    e = _parse_error(403, body, "PUT /b/k")
    assert e.server_time == 1792291249.0
    e = _parse_error(403, b"<Error><Code>RequestTimeTooSkewed</Code></Error>", "PUT /b/k",
                     {"Date": "Sun, 18 Oct 2026 02:40:49 GMT"})
    assert e.server_time == 1792291249.0
    assert _parse_error(404, b"<Error><Code>NoSuchKey</Code></Error>", "x").server_time is None
    # a genuine 403 from a server whose clock agrees is not taken for skew
    from tritondl.s3.client import S3Client
    c = S3Client("http://127.0.0.1:9", Static("ak", "sk"))
    now = __import__("email.utils").utils.formatdate(usegmt=True)
    assert not c._learn_skew(_parse_error(403, b"", "HEAD /b", {"Date": now})) and c.clock_skew == 0.0


def test_stale_resume_state_starts_over(tmp_path):
    """A state file whose upload the server no longer has (aborted by a
    lifecycle rule) or that describes another object is ignored."""
    import json
    async def main():
        s3 = await FakeS3(access_key="ak", secret_key="sk", store="memory").start()
        s3.create_bucket("b")
        c = S3Client(s3.endpoint, Static("ak", "sk"), part_size=5 << 20, multipart_threshold=5 << 20)
        data = os.urandom((11 << 20) + 1)
        p = tmp_path / "f.mkv"
        p.write_bytes(data)
        state = str(p) + ".s3upload"
        with open(state, "w") as f:
            json.dump({"bucket": "b", "key": "k", "size": len(data), "part_size": 5 << 20,
                       "upload_id": "upload-does-not-exist"}, f)
        await c.put_object("b", "k", str(p), resume_path=state)
        assert s3.object_bytes("b", "k") == data and not os.path.exists(state)
        with open(state, "w") as f:
            json.dump({"bucket": "other", "key": "k", "size": 1, "part_size": 5, "upload_id": "x"}, f)
        await c.put_object("b", "k", str(p), resume_path=state)
        assert s3.object_bytes("b", "k") == data
        # malformed state (another version, hand-edited, torn): ignored, never a crash
        same = {"bucket": "b", "key": "k", "size": len(data), "part_size": 5 << 20}
        for bad in ([same], {**same, "upload_id": 7}, {**same, "upload_id": ""}, {**same}, "[", "\x00"):
            with open(state, "w") as f:
                f.write(bad if isinstance(bad, str) else json.dumps(bad))
            await c.put_object("b", "k", str(p), resume_path=state)
            assert s3.object_bytes("b", "k") == data and not os.path.exists(state)
        await c.close()
        await s3.stop()
    run(main())


def test_unparsable_xml_replies_are_s3_errors(tmp_path):
    """A 2xx reply whose body is not XML (a proxy's HTML page, a truncated
    body) fails the request as an S3Error like any other failure, never an
    XML parser exception."""
    async def main():
        c = S3Client("http://127.0.0.1:9", Static("ak", "sk"), part_size=5 << 20, multipart_threshold=5 << 20)

        async def garbage(*_a, **_k):
            return 200, {}, b"<html>gateway"
        c._do = garbage
        p = tmp_path / "f.mkv"
        p.write_bytes(os.urandom((5 << 20) + 1))
        for call in (lambda: c.put_object("b", "k", str(p)), lambda: c.list_parts("b", "k", "u"),
                     lambda: c.list_objects("b")):
            with pytest.raises(S3Error) as ei:
                await call()
            assert ei.value.code == "MalformedXML"
        await c.close()
    run(main())
