"""S3 request resilience at minio-go's level (VERDICT r05 Missing #1, Weak
#2, #5).

Every reference S3 call went through minio-go v6
(``internal/uploader/uploader.go:43-51,64-65,89``), whose request loop
(``retry.go``) retries connection errors, the statuses 429/500/502/503 and
the S3 codes RequestTimeout, RequestError, Throttling(Exception),
RequestLimitExceeded, RequestThrottled, SlowDown, InternalError and
ExpiredToken(Exception), up to 10 times, 1 s × 2^k apart up to 30 s.  The fake
S3 now refuses what AWS refuses: real error codes, an idle request body
timed out with 400 RequestTimeout, outages that outlast a short budget."""

import asyncio
import os
import time

import pytest

from tritondl.models import Media
from tritondl.s3.client import RETRYABLE_CODES, S3Client, S3Error, is_retryable
from tritondl.s3.credentials import Static
from tritondl.s3.uploader import object_key
from tritondl_testkit.fakes.s3 import FakeS3

from .test_permissions import Env, run

# (status, code) pairs minio-go retries, as AWS / MinIO send them
RETRYABLE = [(400, "RequestTimeout"), (503, "SlowDown"), (429, "SlowDown"), (500, "InternalError"),
             (502, "BadGateway"), (503, "ServiceUnavailable"), (504, "GatewayTimeout"), (403, "ExpiredToken"),
             (400, "ExpiredTokenException"), (400, "Throttling"), (400, "ThrottlingException"),
             (503, "RequestLimitExceeded"), (503, "RequestThrottled"), (400, "RequestError")]


def test_classifier_matches_minio_go():
    for status, code in RETRYABLE:
        assert is_retryable(S3Error(status, code)), (status, code)
    for status, code in [(400, "InvalidArgument"), (403, "AccessDenied"), (404, "NoSuchKey"),
                         (501, "NotImplemented"), (400, "BadDigest"), (403, "SignatureDoesNotMatch"),
                         (0, "SourceStalled"), (0, "SourceFailed")]:
        assert not is_retryable(S3Error(status, code)), (status, code)
    assert {"RequestTimeout", "SlowDown", "ExpiredToken", "InternalError"} <= RETRYABLE_CODES


def test_default_budget_is_minio_go_s_and_rides_out_a_minute():
    c = S3Client("http://127.0.0.1:1", Static("a", "b"))
    assert c.max_retries + 1 == 10 and c.retry_unit == 1.0 and c.retry_cap == 30.0
    for _ in range(200):
        waits = [c.retry_delay(k) for k in range(1, 10)]
        assert all(min(30.0, 2.0 ** (k - 1)) / 2 <= w <= min(30.0, 2.0 ** (k - 1)) for k, w in zip(range(1, 10), waits))
        assert sum(waits) >= 75.5                    # half of every wait is fixed: never < ~75 s in total


@pytest.mark.parametrize("status,code", RETRYABLE)
def test_each_retryable_code_injected_three_times_is_ridden_out(status, code):
    async def main():
        s3 = await FakeS3(access_key="ak", secret_key="sk").start()
        c = S3Client(s3.endpoint, Static("ak", "sk"), retry_unit=0.01)
        s3.create_bucket("b")
        data = os.urandom(300_000)
        s3.fail_next(3, status, code)
        await c.put_object("b", "k", data)                       # aiohttp path
        assert s3.object_bytes("b", "k") == data and s3.failed == 3
        path = f"/tmp/tdl-s3r-{os.getpid()}-{status}-{code}"
        with open(path, "wb") as f:
            f.write(data)
        try:
            s3.fail_next(3, status, code, methods=("PUT",))
            await c.put_object("b", "k2", path)                  # native pump path
            assert s3.object_bytes("b", "k2") == data and s3.failed == 6
        finally:
            os.unlink(path)
        await c.close()
        await s3.stop()
    run(main())


def test_non_retryable_errors_fail_at_once():
    async def main():
        s3 = await FakeS3(access_key="ak", secret_key="sk").start()
        c = S3Client(s3.endpoint, Static("ak", "sk"), retry_unit=0.01)
        s3.create_bucket("b")
        for status, code in [(400, "InvalidArgument"), (501, "NotImplemented")]:
            s3.fail_next(3, status, code)
            n0 = len(s3.requests)
            with pytest.raises(S3Error) as e:
                await c.put_object("b", "k", b"x" * 1000)
            assert e.value.code == code and len(s3.requests) == n0 + 1
            s3.fail_next(0)
        await c.close()
        await s3.stop()
    run(main())


def test_budget_is_bounded():
    async def main():
        s3 = await FakeS3(access_key="ak", secret_key="sk").start()
        c = S3Client(s3.endpoint, Static("ak", "sk"), retry_unit=0.001, max_retries=4)
        s3.create_bucket("b")
        s3.fail_next(100, 503, "SlowDown")
        n0 = len(s3.requests)
        with pytest.raises(S3Error) as e:
            await c.put_object("b", "k", b"x")
        assert e.value.code == "SlowDown" and len(s3.requests) - n0 == 5
        await c.close()
        await s3.stop()
    run(main())


def test_multipart_complete_and_parts_retry_minio_codes(tmp_path):
    async def main():
        s3 = await FakeS3(access_key="ak", secret_key="sk").start()
        c = S3Client(s3.endpoint, Static("ak", "sk"), retry_unit=0.01, part_size=5 << 20, multipart_threshold=5 << 20,
                     parallel_parts=2)
        s3.create_bucket("b")
        data = os.urandom(12 << 20)
        p = tmp_path / "f.mkv"
        p.write_bytes(data)
        s3.fail_next(4, 429, "SlowDown", methods=("PUT",))
        await c.put_object("b", "big", str(p), resume_path=str(p) + ".s3upload")
        assert s3.object_bytes("b", "big") == data and s3.failed == 4
        s3.complete_error_200, s3.complete_error_code = 2, "SlowDown"
        await c.put_object("b", "big2", str(p))
        assert s3.object_bytes("b", "big2") == data
        await c.close()
        await s3.stop()
    run(main())


def test_fake_s3_times_out_an_idle_request_body():
    """The fake answers 400 RequestTimeout and drops the connection when a
    PUT body goes silent, as AWS does after ~20 s."""
    async def main():
        s3 = await FakeS3().start()
        s3.idle_timeout = 0.3
        s3.create_bucket("b")
        r, w = await asyncio.open_connection("127.0.0.1", s3.port)
        w.write(b"PUT /b/k HTTP/1.1\r\nHost: x\r\nContent-Length: 100\r\nx-amz-content-sha256: UNSIGNED-PAYLOAD\r\n\r\n"
                b"0123456789")
        await w.drain()
        t0 = time.monotonic()
        head = await asyncio.wait_for(r.read(4096), 5)
        assert time.monotonic() - t0 >= 0.25
        assert head.startswith(b"HTTP/1.1 400") and b"<Code>RequestTimeout</Code>" in head
        assert s3.idle_timeouts == 1
        w.close()
        await s3.stop()
    run(main())


def _no_broker_retry(e):
    assert e.svc.metrics.get("jobs_retried") in (0, None, 0.0), "the job went back through the broker"


def test_streamed_put_survives_an_origin_that_stalls_past_s3_s_idle_timeout(tmp_path):
    """The origin stalls 3 s mid-body; the fake S3 drops a request body idle
    for 1 s.  With the default stall limit (10 s) the PUT is timed out by S3
    (400 RequestTimeout, retried); the job still finishes on its first
    delivery."""
    async def main():
        e = await Env().up(tmp_path)
        e.svc.uploader.client.retry_unit = 0.3
        e.s3.idle_timeout = 1.0
        data = os.urandom(6 << 20)
        url = e.origin.add("/stall.mkv", data)
        e.origin.stall = (2 << 20, 3.0)
        e.submit(Media(id="st", source_uri=url))
        res = await e.wait_results(1, timeout=60)
        assert res[0].ok and res[0].stage == "done", res
        assert e.s3.object_bytes("triton-staging", object_key("st", "stall.mkv")) == data
        assert e.s3.idle_timeouts >= 1
        _no_broker_retry(e)
        assert len(e.converts()) == 1
        await e.down()
    run(main(), 90)


def test_streamed_put_falls_back_to_upload_after_download_on_a_stall(tmp_path):
    """With the stall limit below S3's idle timeout, the PUT is dropped by the
    worker itself and the file uploaded once the download is done: S3 never
    times a body out."""
    async def main():
        e = await Env().up(tmp_path, s3_stream_stall_s=0.4)
        e.s3.idle_timeout = 1.0
        data = os.urandom(6 << 20)
        url = e.origin.add("/stall2.mkv", data)
        e.origin.stall = (2 << 20, 2.0)
        e.submit(Media(id="st2", source_uri=url))
        res = await e.wait_results(1, timeout=60)
        assert res[0].ok and res[0].stage == "done", res
        assert e.s3.object_bytes("triton-staging", object_key("st2", "stall2.mkv")) == data
        assert e.svc.uploader.stalls == 1 and e.s3.idle_timeouts == 0
        _no_broker_retry(e)
        await e.down()
    run(main(), 90)


def test_streamed_multipart_put_keeps_its_landed_parts_on_a_stall(tmp_path):
    async def main():
        e = await Env().up(tmp_path, s3_stream_stall_s=0.4, http_segments=1)
        cl = e.svc.uploader.client
        cl.part_size, cl.multipart_threshold, cl.parallel_parts = 5 << 20, 5 << 20, 1
        data = os.urandom(16 << 20)
        url = e.origin.add("/mp.mkv", data)
        e.origin.stall = (11 << 20, 1.5)                # parts 1-2 land, part 3 stalls
        e.submit(Media(id="mp", source_uri=url))
        res = await e.wait_results(1, timeout=60)
        assert res[0].ok, res
        assert e.s3.object_bytes("triton-staging", object_key("mp", "mp.mkv")) == data
        assert e.svc.uploader.stalls == 1
        part_puts = [r for r in e.s3.requests if r[0] == "PUT" and "partNumber=1&" in r[1] + "&"]
        assert len(part_puts) == 1                      # part 1 was not sent again
        await e.down()
    run(main(), 90)


def test_each_retryable_code_during_a_job_passes_on_the_first_delivery(tmp_path):
    async def main():
        e = await Env().up(tmp_path)
        e.svc.uploader.client.retry_unit = 0.01
        data = os.urandom(1 << 20)
        for i, (status, code) in enumerate(RETRYABLE):
            url = e.origin.add(f"/c{i}.mkv", data)
            e.s3.fail_next(3, status, code, methods=("PUT",))
            e.submit(Media(id=f"c{i}", source_uri=url), i)
            res = await e.wait_results(i + 1, timeout=30)
            assert res[-1].ok, (status, code, res[-1])
        assert e.s3.failed == 3 * len(RETRYABLE)
        _no_broker_retry(e)
        assert len(e.converts()) == len(RETRYABLE)
        await e.down()
    run(main(), 120)


def test_a_20s_s3_outage_during_a_256mib_multipart_upload(tmp_path):
    """The default budget (10 attempts, 1 s unit, 30 s cap) rides out a 20 s
    outage in which S3 refuses connections, in the middle of a 256 MiB
    multipart upload: the job passes on its first delivery."""
    async def main():
        e = await Env().up(tmp_path)
        cl = e.svc.uploader.client
        assert (cl.max_retries, cl.retry_unit, cl.retry_cap) == (9, 1.0, 30.0)
        e.s3.store = "discard"
        data = os.urandom(1 << 20) * 256
        url = e.origin.add("/big.mkv", data)
        e.origin.rate = 64 << 20                         # ~4 s of download: the outage lands mid-upload
        e.submit(Media(id="big", source_uri=url))
        t0 = time.monotonic()
        while not any(r[0] == "PUT" and "partNumber" in r[1] for r in e.s3.requests):
            assert time.monotonic() - t0 < 30
            await asyncio.sleep(0.01)
        await e.s3.down_for(20.0)
        res = await e.wait_results(1, timeout=200)
        assert res[0].ok, res
        assert time.monotonic() - t0 >= 20
        o = e.s3.buckets["triton-staging"][object_key("big", "big.mkv")]
        assert o.size == len(data)
        _no_broker_retry(e)
        await e.down()
    run(main(), 240)
