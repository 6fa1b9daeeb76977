"""The GPU verification helper process (ops/gpu_helper.py): the worker
never brings up HIP itself; a helper does, and exits when idle.  These CPU
tests drive the protocol with the helper's host stand-in
(``TRITONDL_GPU_HELPER_FAKE=1``); the HIP helper is covered by the GPU
tests (tests/test_hashing.py)."""

import os
import time

import pytest

from tritondl.ops import gpu_helper, hashing


@pytest.fixture
def fake_helper(monkeypatch):
    monkeypatch.setenv("TRITONDL_GPU_HELPER_FAKE", "1")
    monkeypatch.setenv("TRITONDL_GPU_IDLE_S", "30")
    h = gpu_helper.GpuHelper()
    yield h
    h.close()


def _layout(tmp_path, sizes, piece_len):
    data = os.urandom(sum(sizes))
    files, off = [], 0
    for i, n in enumerate(sizes):
        p = tmp_path / f"f{i}"
        p.write_bytes(data[off:off + n])
        files.append((str(p), n))
        off += n
    exp = hashing.piece_hashes(data, piece_len, "sha1")
    return files, data, exp


def test_helper_verifies_and_reports(tmp_path, fake_helper):
    files, data, exp = _layout(tmp_path, [100_000, 5, 70_000], 16384)
    n = len(exp) // 20
    assert fake_helper.verify_files(files, 16384, exp) == b"\x01" * n
    pid = fake_helper.pid
    assert pid and pid != os.getpid() and fake_helper.spawned == 1
    with open(files[0][0], "r+b") as f:
        f.seek(40_000)
        f.write(b"\x00\xff")
    ok = fake_helper.verify_files(files, 16384, exp)
    assert [i for i, v in enumerate(ok) if not v] == [40_000 // 16384]
    assert fake_helper.hash_buffer("sha256", data, 65536) == hashing.piece_hashes(data, 65536, "sha256")
    d, complete = fake_helper.digest_files(files, 16384, "sha256")
    assert len(d) == 32 * len(complete) and fake_helper.pid == pid       # one process served everything


def test_helper_exits_idle_and_comes_back(tmp_path, fake_helper, monkeypatch):
    monkeypatch.setenv("TRITONDL_GPU_IDLE_S", "0.5")
    files, _data, exp = _layout(tmp_path, [50_000], 16384)
    assert fake_helper.verify_files(files, 16384, exp) == b"\x01" * 4
    assert fake_helper.wait_exit(10)                  # idle: gone, with everything it held
    assert fake_helper.pid is None
    assert fake_helper.verify_files(files, 16384, exp) == b"\x01" * 4
    assert fake_helper.spawned == 2


def test_helper_exiting_as_a_request_arrives_is_retried(tmp_path, fake_helper, monkeypatch):
    """The idle exit can race a request: a clean exit (rc 0) gets one respawn."""
    monkeypatch.setenv("TRITONDL_GPU_IDLE_S", "0.3")
    files, _data, exp = _layout(tmp_path, [20_000], 16384)
    for _ in range(6):
        assert fake_helper.verify_files(files, 16384, exp) == b"\x01\x01"
        time.sleep(0.3)


def test_helper_crash_fails_the_call_loudly(tmp_path, fake_helper):
    files, _data, exp = _layout(tmp_path, [20_000], 16384)
    assert fake_helper.ping()
    os.kill(fake_helper.pid, 9)
    time.sleep(0.1)
    # the next call starts a new helper (the old one is reaped, not waited on forever)
    assert fake_helper.verify_files(files, 16384, exp) == b"\x01\x01"
    with pytest.raises(gpu_helper.HelperError, match="unknown op"):
        fake_helper._call({"op": "nope"})
    assert fake_helper.ping()                          # a bad request does not kill it


def test_helper_that_cannot_start_says_why(monkeypatch):
    monkeypatch.delenv("TRITONDL_GPU_HELPER_FAKE", raising=False)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")      # no device in the helper
    h = gpu_helper.GpuHelper(start_timeout=60)
    with pytest.raises(gpu_helper.HelperError, match="failed to start"):
        h.ping()


def test_worker_side_never_loads_hip(monkeypatch):
    """gpu_available() in helper mode reads the KFD topology; it does not
    import the HIP extension into the worker."""
    import subprocess
    import sys
    code = ("import sys\n"
            "from tritondl.ops import hashing\n"
            "hashing.gpu_available(); hashing.choose_device(1000, 1 << 20, 1 << 30)\n"
            "print('LOADED', 'tritondl._gpu_hash' in sys.modules, 'torch' in sys.modules)\n")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, timeout=60,
                       cwd=gpu_helper.ROOT, env={k: v for k, v in os.environ.items() if k != "TRITONDL_GPU_HELPER"})
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    assert b"LOADED False False" in p.stdout


def test_auto_verify_falls_back_to_the_host_when_the_helper_cannot_start(tmp_path, monkeypatch):
    """A node whose KFD lists a GPU but whose HIP stack is broken: the first
    'auto' resume finds the helper dead on arrival, verifies on the host, and
    the GPU is not offered again in this process."""
    from tritondl_testkit.fakes.swarm import make_payload
    from tritondl.fetch.bt.metainfo import make_info
    from tritondl.fetch.bt.storage import FileStorage

    src = tmp_path / "src" / "T"
    make_payload(str(src), {"a.mkv": 300_000, "b.mkv": 120_000})
    info = make_info(str(src), 32768)
    monkeypatch.setattr(hashing, "_kfd_gpus", lambda: 1)
    monkeypatch.setattr(hashing, "_gpu_ext_present", lambda: True)
    monkeypatch.setattr(hashing, "choose_device", lambda *a, **k: "gpu")
    monkeypatch.setattr(hashing, "_helper", gpu_helper.GpuHelper(start_timeout=60))
    monkeypatch.setattr(hashing, "_gpu_disabled", None)
    monkeypatch.setattr(hashing, "_gpu_failures", 0)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")       # what the helper sees: no device
    st = FileStorage(str(tmp_path / "src"), info)
    have = st.verify_existing("auto")
    assert have == set(range(info.num_pieces))
    # a helper that cannot start sets the GPU aside at once ...
    assert hashing._gpu_disabled and not hashing.gpu_available()
    # ... for the cool-down only: then it is offered again
    monkeypatch.setattr(hashing, "_gpu_disabled_until", 0.0)
    assert hashing.gpu_available()
    assert hashing._gpu_disabled is None


def test_helper_stuck_in_a_call_is_killed_and_auto_verify_uses_the_host(tmp_path, monkeypatch):
    """A helper that never answers (a kernel that does not finish) is killed
    after the call timeout; the call fails with HelperError, which the 'auto'
    verify path answers by hashing on the host — the worker's executor
    thread and job slot are not held forever."""
    monkeypatch.setenv("TRITONDL_GPU_HELPER_FAKE", "1")
    monkeypatch.setenv("TRITONDL_GPU_HELPER_FAKE_STALL", "60")
    h = gpu_helper.GpuHelper(call_timeout=0.5)
    files, _data, exp = _layout(tmp_path, [20_000], 16384)
    try:
        assert h.ping()                                  # pings are answered at once
        pid = h.pid
        t0 = time.monotonic()
        with pytest.raises(gpu_helper.HelperError, match="no progress"):
            h.verify_files(files, 16384, exp)
        assert time.monotonic() - t0 < 10
        assert h.pid is None
        with pytest.raises(OSError):
            os.kill(pid, 0)                              # reaped, not left running
    finally:
        h.close()

    from tritondl_testkit.fakes.swarm import make_payload
    from tritondl.fetch.bt.metainfo import make_info
    from tritondl.fetch.bt.storage import FileStorage
    src = tmp_path / "src" / "T"
    make_payload(str(src), {"a.mkv": 200_000})
    info = make_info(str(src), 32768)
    monkeypatch.setattr(hashing, "_kfd_gpus", lambda: 1)
    monkeypatch.setattr(hashing, "_gpu_ext_present", lambda: True)
    monkeypatch.setattr(hashing, "choose_device", lambda *a, **k: "gpu")
    monkeypatch.setattr(hashing, "_helper", gpu_helper.GpuHelper(call_timeout=0.5))
    monkeypatch.setattr(hashing, "_gpu_disabled", None)
    monkeypatch.setattr(hashing, "_gpu_failures", 0)
    try:
        # one stuck call costs that batch the GPU, not the worker: still offered
        have = FileStorage(str(tmp_path / "src"), info).verify_existing("auto")
        assert have == set(range(info.num_pieces))
        assert hashing._gpu_disabled is None and hashing._gpu_failures == 1 and hashing.gpu_available()
        # repeated faults set it aside (for the cool-down)
        for _ in range(gpu_helper_max := hashing.GPU_MAX_FAILURES - 1):
            FileStorage(str(tmp_path / "src"), info).verify_existing("auto")
        assert gpu_helper_max >= 1
        assert hashing._gpu_disabled and "no progress" in hashing._gpu_disabled
        assert not hashing.gpu_available()
    finally:
        hashing._helper.close()


def test_slow_but_progressing_call_is_not_killed(tmp_path, monkeypatch):
    """a call that keeps reading (a cold HDD or NFS resume) runs
    past the no-progress limit: every heartbeat whose byte count grew
    extends it.  A successful call also resets the failure count."""
    monkeypatch.setenv("TRITONDL_GPU_HELPER_FAKE", "1")
    monkeypatch.setenv("TRITONDL_GPU_HELPER_FAKE_SLOW", "2.0")
    monkeypatch.setenv("TRITONDL_GPU_PROGRESS_S", "0.1")
    monkeypatch.setattr(hashing, "_gpu_failures", 2)
    h = gpu_helper.GpuHelper(call_timeout=0.6)
    files, _data, exp = _layout(tmp_path, [50_000], 16384)
    try:
        t0 = time.monotonic()
        assert h.verify_files(files, 16384, exp) == b"\x01" * 4
        assert time.monotonic() - t0 >= 2.0          # far past the 0.6 s no-progress limit
        assert h.spawned == 1
        assert hashing._gpu_failures == 0
    finally:
        h.close()


def test_reap_does_not_block_on_an_unkillable_helper(monkeypatch):
    """after SIGKILL the wait is bounded; a child stuck in the
    kernel (D state) is left to a daemon thread instead of blocking the call
    lock forever."""
    import subprocess

    class Stuck:
        stdin = None
        killed = 0

        def poll(self):
            return None

        def kill(self):
            self.killed += 1

        def wait(self, timeout=None):
            if timeout is None:
                return -9
            raise subprocess.TimeoutExpired("helper", timeout)
    p = Stuck()
    t0 = time.monotonic()
    assert gpu_helper.GpuHelper._reap(p, kill=True) is None
    assert time.monotonic() - t0 < 1 and p.killed >= 2
