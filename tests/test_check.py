"""python -m tritondl.check: preflight against the fakes."""

import asyncio
import json
import os
import subprocess
import sys

from tritondl import check
from tritondl_testkit.fakes.broker import Broker
from tritondl_testkit.fakes.s3 import FakeS3

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(monkeypatch, tmp_path, broker_url_hostport: str, s3: str):
    monkeypatch.setenv("RABBITMQ_ENDPOINT", broker_url_hostport)
    monkeypatch.setenv("RABBITMQ_USERNAME", "guest")
    monkeypatch.setenv("RABBITMQ_PASSWORD", "guest")
    monkeypatch.setenv("S3_ENDPOINT", s3)
    monkeypatch.setenv("S3_ACCESS_KEY", "ak")
    monkeypatch.setenv("S3_SECRET_KEY", "sk")
    monkeypatch.setenv("TRITONDL_DOWNLOAD_DIR", str(tmp_path / "dl"))
    monkeypatch.setenv("TRITONDL_GPU_VERIFY", "off")


def test_preflight_passes_and_reports_missing_topology(tmp_path, monkeypatch):
    async def main():
        b = await Broker(username="guest", password="guest").start()
        s3 = await FakeS3(access_key="ak", secret_key="sk").start()
        try:
            _env(monkeypatch, tmp_path, b.url.split("@", 1)[1].rstrip("/"), s3.endpoint)
            r = await check.run([])
            by = {(i["area"], i["status"]) for i in r.items}
            assert not r.failed, r.items
            assert ("broker", "ok") in by and ("s3", "ok") in by and ("download_dir", "ok") in by
            # nothing declared yet: the exchanges/queues are reported as missing, not created
            warns = [i["detail"] for i in r.items if i["area"] == "broker" and i["status"] == "warn"]
            assert any("v1.download does not exist" in w for w in warns)
            assert "v1.download" not in b.exchanges
            assert any("bucket triton-staging does not exist yet" in i["detail"] for i in r.items)
            # a wrong secret fails the S3 check; a dead broker fails the broker check
            monkeypatch.setenv("S3_SECRET_KEY", "nope")
            monkeypatch.setenv("RABBITMQ_ENDPOINT", "127.0.0.1:1")
            r2 = await check.run([], timeout=3)
            bad = {i["area"] for i in r2.items if i["status"] == "fail"}
            assert r2.failed and {"broker", "s3"} <= bad
        finally:
            await s3.stop()
            await b.stop()
    asyncio.run(asyncio.wait_for(main(), 60))


def test_preflight_cli_fails_on_an_unusable_endpoint(tmp_path):
    env = dict(os.environ, S3_ENDPOINT="ftp://", TRITONDL_DOWNLOAD_DIR=str(tmp_path / "dl"), PYTHONPATH=ROOT,
               TRITONDL_GPU_VERIFY="off")
    p = subprocess.run([sys.executable, "-m", "tritondl.check", "--json", "--no-broker"], capture_output=True,
                       text=True, timeout=120, env=env, cwd=ROOT)
    assert p.returncode == 1, p.stderr
    doc = json.loads(p.stdout)
    assert doc["ok"] is False
    assert any(i["area"] == "s3" and i["status"] == "fail" and "unusable" in i["detail"] for i in doc["checks"])
    assert any(i["area"] == "native" and i["status"] == "ok" for i in doc["checks"])


def test_preflight_warns_about_a_skewed_clock(tmp_path, monkeypatch):
    """S3's clock two hours ahead: the bucket check still passes (the client
    re-dates its requests) and the report says how far off the host is."""
    async def main():
        s3 = await FakeS3(access_key="ak", secret_key="sk").start()
        s3.create_bucket("triton-staging")
        s3.clock_offset = 7200.0
        try:
            _env(monkeypatch, tmp_path, "127.0.0.1:1", s3.endpoint)
            r = await check.run([], timeout=5, skip_broker=True)
            s3_items = [i for i in r.items if i["area"] == "s3"]
            assert any(i["status"] == "ok" and "exists" in i["detail"] for i in s3_items), s3_items
            skew = [i for i in s3_items if i["status"] == "warn" and "clock" in i["detail"]]
            assert skew and abs(skew[0]["skew_s"] - 7200) < 5
        finally:
            await s3.stop()
    asyncio.run(asyncio.wait_for(main(), 60))


def test_lease_probe_tells_whether_leases_will_work(tmp_path, monkeypatch):
    """--lease-probe declares and deletes one lease-shaped queue: OK for a
    user who may, a warning naming the permission for one who may not (the
    worker then holds deliveries unacked, as the reference did)."""
    async def main():
        b = await Broker(username="guest", password="guest").start()
        b.add_user("narrow", "pw", configure=r"^v1\.download(-\d+)?$", write=".*", read=r"^v1\.download-\d+$")
        try:
            _env(monkeypatch, tmp_path, b.url.split("@", 1)[1].rstrip("/"), "http://127.0.0.1:1")
            r = await check.run([], timeout=5, skip_s3=True, lease_probe=True)
            leases = [i for i in r.items if i["area"] == "leases"]
            assert leases and leases[0]["status"] == "ok", leases
            assert not [q for q in b.queues if ".lease." in q]          # nothing left behind
            monkeypatch.setenv("RABBITMQ_USERNAME", "narrow")
            monkeypatch.setenv("RABBITMQ_PASSWORD", "pw")
            r2 = await check.run([], timeout=5, skip_s3=True, lease_probe=True)
            leases = [i for i in r2.items if i["area"] == "leases"]
            assert leases and leases[0]["status"] == "warn" and "configure and read" in leases[0]["detail"]
            assert not r2.failed or {i["area"] for i in r2.items if i["status"] == "fail"} == set()
        finally:
            await b.stop()
    asyncio.run(asyncio.wait_for(main(), 60))


def test_cpu_check_reports_each_l3_domain_s_load(monkeypatch):
    """The preflight shows how busy other tenants keep each L3 domain, as
    placement sees it (TRITONDL_CPUS=auto and the pool take idle ones first)."""
    from tritondl.parallel import topology
    monkeypatch.setattr(topology, "l3_domains", lambda allowed=None: [[0, 1], [2, 3], [4, 5]])
    monkeypatch.setattr(topology, "domain_busy", lambda d, interval=0.2: [0.0, 0.25, 0.004])
    r = check.Report()
    check.check_cpus(r)
    (item,) = [i for i in r.items if i["area"] == "cpus"]
    assert "2 of 3 L3 domains idle now" in item["detail"]
    assert item["domain_busy"] == {"0": 0.0, "2": 0.25, "4": 0.004}
