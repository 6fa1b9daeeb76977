"""Relay pumps on the native task pool, reported through a CompletionPort
(eventfd) to the event loop instead of an executor thread
(csrc/relay/relay_core.h::CompletionPort, utils/rawhttp.py::run_pump)."""

import asyncio
import os
import socket

import pytest

from tritondl.utils import rawhttp

relay = rawhttp.relay_module()
pytestmark = pytest.mark.skipif(relay is None or not hasattr(relay, "CompletionPort"),
                                reason="native relay module not built")


def test_port_runs_recv_and_send_pumps(tmp_path):
    port = relay.CompletionPort()
    a, b = socket.socketpair()
    a.setblocking(False)
    b.setblocking(False)
    data = os.urandom(3 << 20)
    (tmp_path / "src").write_bytes(data)
    sfd = os.open(tmp_path / "src", os.O_RDONLY)
    dfd = os.open(tmp_path / "dst", os.O_RDWR | os.O_CREAT, 0o600)
    try:
        relay.start_recv_body(port, 7, b.fileno(), dfd, 0, len(data), b"", None)
        relay.start_send_body(port, 8, a.fileno(), b"", sfd, 0, len(data), None, 0)
        got = {}
        while len(got) < 2:
            assert port.wait(10_000), "no completion within 10 s"
            got.update(dict(port.reap()))
        assert got[7] == (len(data), False, "")
        assert got[8][0] == len(data) and got[8][2] == ""
        assert (tmp_path / "dst").read_bytes() == data
        assert port.inflight == 0
        assert port.reap() == []                      # drained: nothing twice
    finally:
        os.close(sfd)
        os.close(dfd)
        a.close()
        b.close()


def test_port_results_keep_the_chunked_form(tmp_path):
    port = relay.CompletionPort()
    a, b = socket.socketpair()
    b.setblocking(False)
    dfd = os.open(tmp_path / "dst", os.O_RDWR | os.O_CREAT, 0o600)
    try:
        relay.start_recv_body(port, 1, b.fileno(), dfd, 0, -1, b"5\r\nhello\r\n", None, chunked=True)
        a.sendall(b"6\r\n world\r\n0\r\n\r\n")
        assert port.wait(10_000)
        [(pid, res)] = port.reap()
        assert pid == 1 and res == (11, False, "", True)
        assert (tmp_path / "dst").read_bytes() == b"hello world"
    finally:
        os.close(dfd)
        a.close()
        b.close()


def test_run_pump_uses_the_port_and_cancel_waits_for_the_pump(tmp_path, monkeypatch):
    """A cancelled run_pump aborts the native pump and returns only once it
    finished, so the caller may close the fd right after."""
    monkeypatch.setenv("TRITONDL_RELAY_PORT", "1")

    async def main():
        a, b = socket.socketpair()
        b.setblocking(False)
        conn = rawhttp.RawConn(b)
        dfd = os.open(tmp_path / "dst", os.O_RDWR | os.O_CREAT, 0o600)
        try:
            a.sendall(b"x" * 1000)            # part of a 1 MiB body; the rest never comes
            t = asyncio.ensure_future(rawhttp.run_pump(conn, relay.recv_body, dfd, 0, 1 << 20, b"", None))
            for _ in range(200):
                await asyncio.sleep(0.005)
                if os.fstat(dfd).st_size >= 1000:
                    break
            assert asyncio.get_running_loop() in rawhttp._ports, "pump did not go through the port"
            assert rawhttp.active_pumps() == 1
            t.cancel()
            with pytest.raises(asyncio.CancelledError):
                await t
            assert rawhttp.active_pumps() == 0     # the pump had finished when the cancel surfaced
        finally:
            os.close(dfd)
            a.close()
            conn.close()
        assert (tmp_path / "dst").read_bytes() == b"x" * 1000

    asyncio.run(asyncio.wait_for(main(), 30))


def test_run_pump_executor_by_default(tmp_path, monkeypatch):
    monkeypatch.delenv("TRITONDL_RELAY_PORT", raising=False)

    async def main():
        a, b = socket.socketpair()
        b.setblocking(False)
        conn = rawhttp.RawConn(b)
        dfd = os.open(tmp_path / "dst", os.O_RDWR | os.O_CREAT, 0o600)
        try:
            a.sendall(b"y" * 5000)
            res = await rawhttp.run_pump(conn, relay.recv_body, dfd, 0, 5000, b"", None)
            assert res == (5000, False, "")
            assert asyncio.get_running_loop() not in rawhttp._ports
        finally:
            os.close(dfd)
            a.close()
            conn.close()

    asyncio.run(asyncio.wait_for(main(), 30))
