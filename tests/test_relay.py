"""Native data plane (csrc/relay): Flow semantics, receive/send pumps and the
server-side aws-chunked verifier, checked against the reference encoder in
``tritondl.ops.hashing`` (itself pinned to AWS's SigV4 streaming example in
test_s3.py)."""

import os
import socket
import threading
import time

import pytest

from tritondl.ops import hashing
from tritondl.s3 import sigv4
from tritondl.utils import rawhttp

relay = rawhttp.relay_module()
pytestmark = pytest.mark.skipif(relay is None, reason="_relay extension not built")

KEY = b"k" * 32
AMZ = "20260101T000000Z"
SCOPE = "20260101/us-east-1/s3/aws4_request"
SEED = "0" * 64


def _pair():
    a, b = socket.socketpair()
    a.setblocking(False)
    b.setblocking(False)
    return a, b


def _file(tmp_path, data: bytes) -> int:
    p = tmp_path / "src.bin"
    p.write_bytes(data)
    return os.open(p, os.O_RDONLY)


def _drain(sock, n: int) -> bytes:
    out = bytearray()
    sock.setblocking(True)
    while len(out) < n:
        d = sock.recv(min(1 << 20, n - len(out)))
        if not d:
            break
        out += d
    return bytes(out)


def test_flow_coverage_and_states():
    f = relay.Flow([(0, 100, 0), (100, 200, 0), (200, -1, 0)])
    assert f.watermark() == 0
    f.advance(1, 50)                               # [100, 150) on disk, prefix still empty
    assert f.wait_covered(100, 150, 0.0) == 0
    assert f.wait_covered(0, 10, 0.0) == 2         # timeout
    f.advance(0, 100)
    assert f.watermark() == 150 and f.wait_covered(0, 150, 0.0) == 0
    assert f.wait_covered(90, 160, 0.0) == 2
    f.advance(1, 100)
    f.advance(2, 10)
    assert f.watermark() == 210 and f.wait_covered(0, 210, 0.0) == 0
    f.advance(1, 20)                               # progress never goes backwards
    assert f.done(1) == 100
    f.finish(230)
    assert f.wait_covered(0, 230, 0.0) == 0 and f.wait_covered(0, 231, 0.0) == 3
    # multipart scheduling metric: bytes each overlapping segment still has to receive
    m = relay.Flow([(0, 400, 0), (400, 800, 0)])
    m.advance(0, 150)
    assert m.bytes_until_covered(0, 100) == 0 and m.bytes_until_covered(100, 200) == 50
    assert m.bytes_until_covered(400, 500) == 100 and m.bytes_until_covered(350, 450) == 250
    assert m.covered_bytes(100, 500) == 50
    # contiguous coverage from a point (what a streamed PUT may send now): stops at a gap
    m.advance(1, 30)                               # [0,150) and [400,430) on disk
    assert m.covered_prefix(0, 400) == 150 and m.covered_prefix(100, 120) == 20
    assert m.covered_prefix(150, 400) == 0 and m.covered_prefix(400, 800) == 30
    m.advance(0, 400)                              # the gap closes: [0, 430) contiguous
    assert m.covered_prefix(0, 800) == 430 and m.covered_prefix(390, 420) == 30
    m.finish(800)
    assert m.covered_prefix(0, 900) == 800 and m.covered_prefix(900, 950) == 0
    g = relay.Flow([(0, 10, 0)])
    threading.Timer(0.05, g.fail, args=("boom",)).start()
    assert g.wait_covered(0, 10, 5.0) == 1 and g.error == "boom"
    h = relay.Flow([(0, 10, 0)])
    h.cancel()
    assert h.cancelled and h.wait_covered(0, 1, 1.0) == 1


@pytest.mark.parametrize("size", [0, 1, 65536, 65537, 3 * 65536 + 123, 5 << 20])
def test_chunked_send_matches_reference_encoder(tmp_path, size):
    data = os.urandom(size)
    fd = _file(tmp_path, data)
    a, b = _pair()
    try:
        head = b"PUT /x HTTP/1.1\r\n\r\n"
        n = len(head) + sigv4.chunked_length(size)
        got = {}
        t = threading.Thread(target=lambda: got.setdefault("raw", _drain(b, n)))
        t.start()
        sent, last, err = relay.send_body(a.fileno(), head, fd, 0, size, None, 1, KEY, AMZ, SCOPE, SEED, 65536, 3)
        t.join()
        assert err == "" and sent == size
        ref, ref_last = hashing.aws_chunk_encode(KEY, AMZ, SCOPE, SEED, data, 65536, True, 1)
        assert got["raw"] == head + ref and last == ref_last
    finally:
        os.close(fd)
        a.close()
        b.close()


def test_plain_send_offset_range(tmp_path):
    data = os.urandom(1 << 20)
    fd = _file(tmp_path, data)
    a, b = _pair()
    try:
        got = {}
        t = threading.Thread(target=lambda: got.setdefault("raw", _drain(b, 3 + 500_000)))
        t.start()
        sent, _l, err = relay.send_body(a.fileno(), b"hd:", fd, 1234, 500_000, None, 0)
        t.join()
        assert err == "" and sent == 500_000 and got["raw"] == b"hd:" + data[1234:1234 + 500_000]
    finally:
        os.close(fd)
        a.close()
        b.close()


@pytest.mark.parametrize("size", [0, 70000, 9 << 20])
def test_send_then_verify_roundtrip(tmp_path, size):
    data = os.urandom(size)
    fd = _file(tmp_path, data)
    a, b = _pair()
    try:
        raw_len = sigv4.chunked_length(size)
        out = {}
        t = threading.Thread(target=lambda: out.setdefault(
            "r", relay.recv_verify_chunked(b.fileno(), raw_len, b"", KEY, AMZ, SCOPE, SEED, True, 3, 10.0)))
        t.start()
        _s, _l, err = relay.send_body(a.fileno(), b"", fd, 0, size, None, 1, KEY, AMZ, SCOPE, SEED, 65536, 2)
        t.join()
        n, verr, body, _leaf = out["r"]
        assert err == "" and verr == "" and n == size and body == data
    finally:
        os.close(fd)
        a.close()
        b.close()


def test_verifier_rejects_tampering_and_truncation():
    data = os.urandom(300_000)
    enc, _ = hashing.aws_chunk_encode(KEY, AMZ, SCOPE, SEED, data, 65536, True, 1)
    a, b = _pair()
    try:
        # whole body in the prefix: no socket reads needed
        assert relay.recv_verify_chunked(b.fileno(), len(enc), enc, KEY, AMZ, SCOPE, SEED)[1] == ""
        bad = bytearray(enc)
        bad[200_000] ^= 1                                         # payload bit flip
        assert "signature" in relay.recv_verify_chunked(b.fileno(), len(bad), bytes(bad), KEY, AMZ, SCOPE, SEED)[1]
        assert relay.recv_verify_chunked(b.fileno(), len(enc), enc, KEY, AMZ, SCOPE, "1" * 64)[1] != ""
        a.sendall(enc[:1000])
        a.close()                                                 # client goes away mid-body
        err = relay.recv_verify_chunked(b.fileno(), len(enc), b"", KEY, AMZ, SCOPE, SEED, False, 2, 5.0)[1]
        assert "closed" in err
    finally:
        b.close()


def test_recv_body_prefix_length_and_early_eof(tmp_path):
    p = tmp_path / "out.bin"
    fd = os.open(p, os.O_RDWR | os.O_CREAT, 0o644)
    a, b = _pair()
    try:
        flow = relay.Flow([(0, 1000, 0)])
        a.sendall(b"y" * 700)
        got, eof, err = relay.recv_body(b.fileno(), fd, 0, 1000, b"x" * 300, flow, 0, 0, 5.0)
        assert got == 1000 and err == "" and not eof and flow.done(0) == 1000
        assert p.read_bytes() == b"x" * 300 + b"y" * 700
        a.sendall(b"z" * 10)
        a.close()
        got, eof, err = relay.recv_body(b.fileno(), fd, 2000, 50, b"", None, 0, 0, 5.0)
        assert got == 10 and eof and err == "connection closed early"
    finally:
        os.close(fd)
        b.close()


def test_upload_follows_a_growing_download(tmp_path):
    """send_body blocks on the flow until each range is on disk."""
    size = 3 << 20
    data = os.urandom(size)
    p = tmp_path / "grow.bin"
    wfd = os.open(p, os.O_RDWR | os.O_CREAT, 0o644)
    os.ftruncate(wfd, size)
    rfd = os.open(p, os.O_RDONLY)
    flow = relay.Flow([(0, size, 0)])
    a, b = _pair()

    def writer():
        for off in range(0, size, 256 << 10):
            os.pwrite(wfd, data[off:off + (256 << 10)], off)
            flow.advance(0, min(size, off + (256 << 10)))
            time.sleep(0.005)
        flow.finish(size)

    try:
        raw_len = sigv4.chunked_length(size)
        out = {}
        t = threading.Thread(target=lambda: out.setdefault(
            "r", relay.recv_verify_chunked(b.fileno(), raw_len, b"", KEY, AMZ, SCOPE, SEED, True, 2, 10.0)))
        t.start()
        w = threading.Thread(target=writer)
        w.start()
        _s, _l, err = relay.send_body(a.fileno(), b"", rfd, 0, size, flow, 1, KEY, AMZ, SCOPE, SEED, 65536, 3, 10.0)
        w.join()
        t.join()
        assert err == "" and out["r"][1] == "" and out["r"][2] == data
        # a failed source aborts the upload with the source's error
        f2 = relay.Flow([(0, size, 0)])
        threading.Timer(0.05, f2.fail, args=("origin reset",)).start()
        _s, _l, err = relay.send_body(a.fileno(), b"", rfd, 0, size, f2, 1, KEY, AMZ, SCOPE, SEED, 65536, 2, 10.0)
        assert "origin reset" in err
    finally:
        os.close(wfd)
        os.close(rfd)
        a.close()
        b.close()
