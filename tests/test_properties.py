"""Property-based tests (hypothesis) for every hand-written codec: bencode,
AMQP field tables and frames, protobuf varints and the Download envelope,
peer-wire framing under arbitrary segmentation, MSE RC4 symmetry, and the
native aws-chunked encoder/decoder pair, the native HTTP chunked-transfer
decoder under any chunking and head/body split, the S3 multipart planner's
invariants, SigV4 UriEncode and canonical queries against the spec's byte
rule, the safety of server-supplied file names, and fuzzing of every parser of
remote BitTorrent input (info dicts, magnets, tracker replies, extension
messages, KRPC datagrams) and of HTTP response heads.  Decoders must
round-trip what the encoders produce and reject garbage only with their own
error types."""

import asyncio
import math
import os

import pytest
from hypothesis import HealthCheck, example, given, settings
from hypothesis import strategies as st

from tritondl.amqp import codec
from tritondl.fetch.bt import bencode
from tritondl.fetch.bt import peer as pw
from tritondl.models import messages, wire
from tritondl.ops import hashing

SETTINGS = settings(max_examples=int(__import__("os").environ.get("TRITONDL_HYPOTHESIS_EXAMPLES", "150")), deadline=None, suppress_health_check=[HealthCheck.too_slow])

# ----------------------------------------------------------------- bencode

bvals = st.recursive(
    st.integers(min_value=-(2**70), max_value=2**70) | st.binary(max_size=40),
    lambda kids: st.lists(kids, max_size=5) | st.dictionaries(st.binary(max_size=10), kids, max_size=5),
    max_leaves=25)


@SETTINGS
@given(bvals)
def test_bencode_roundtrip(v):
    assert bencode.decode(bencode.encode(v)) == v


@SETTINGS
@given(st.binary(max_size=64))
def test_bencode_garbage_only_raises_bencode_error(b):
    try:
        v = bencode.decode(b)
    except bencode.BencodeError:
        return
    assert bencode.encode(v) == b     # anything accepted is canonical


# ----------------------------------------------------------------- AMQP tables

keys = st.text(min_size=1, max_size=20).filter(lambda k: len(k.encode()) <= 255)
scalars = (st.booleans() | st.integers(min_value=-(2**63), max_value=2**63 - 1)
           | st.floats(allow_nan=False) | st.text(max_size=30) | st.none()
           | st.binary(max_size=30).filter(lambda b: _not_utf8(b)))


def _not_utf8(b: bytes) -> bool:
    try:
        b.decode("utf-8")
        return False
    except UnicodeDecodeError:
        return True


tables = st.recursive(scalars, lambda kids: st.lists(kids, max_size=4) | st.dictionaries(keys, kids, max_size=4),
                      max_leaves=20)


def _norm(v):
    if isinstance(v, tuple):
        return [_norm(x) for x in v]
    if isinstance(v, list):
        return [_norm(x) for x in v]
    if isinstance(v, dict):
        return {k: _norm(x) for k, x in v.items()}
    return v


@SETTINGS
@given(st.dictionaries(keys, tables, max_size=6))
def test_amqp_table_roundtrip(t):
    got = codec.decode_table(codec.encode_table(t))
    assert got == _norm(t) or _float_eq(got, _norm(t))


def _float_eq(a, b):
    if isinstance(a, float) and isinstance(b, float):
        return a == b or (math.isinf(a) and a == b)
    if isinstance(a, dict) and isinstance(b, dict):
        return a.keys() == b.keys() and all(_float_eq(a[k], b[k]) for k in a)
    if isinstance(a, list) and isinstance(b, list):
        return len(a) == len(b) and all(_float_eq(x, y) for x, y in zip(a, b))
    return a == b


@SETTINGS
@given(st.binary(max_size=80))
def test_amqp_table_garbage_raises_frame_error(b):
    try:
        codec.decode_table(b)
    except codec.AMQPError:
        pass


def _known_method_prefix():
    """A class/method id pair the codec knows, then arbitrary argument bytes."""
    ids = sorted(codec.METHODS)
    return st.builds(lambda k, tail: bytes(__import__("struct").pack(">HH", *ids[k % len(ids)])) + tail,
                     st.integers(min_value=0, max_value=10 ** 6), st.binary(max_size=120))


@SETTINGS
@given(st.one_of(st.binary(max_size=120), _known_method_prefix()))
def test_amqp_method_garbage_raises_only_amqp_errors(b):
    """A broker (or a man in the middle) sending a malformed method frame:
    the decoder returns a Method or raises AMQPError, nothing else
    (IndexError, struct.error, UnicodeDecodeError would kill the reader)."""
    try:
        codec.decode_method(b)
    except codec.AMQPError:
        pass


@SETTINGS
@given(st.binary(max_size=200))
def test_amqp_content_header_garbage_raises_only_amqp_errors(b):
    try:
        codec.decode_header(b)
    except codec.AMQPError:
        pass


@SETTINGS
@given(st.lists(st.binary(max_size=64), max_size=8))
def test_amqp_frame_parser_garbage_raises_only_amqp_errors(chunks):
    p = codec.FrameParser()
    p.frame_max = 4096
    try:
        for c in chunks:
            p.feed(c)
    except codec.AMQPError:
        pass


@SETTINGS
@given(st.binary(max_size=3000), st.integers(min_value=4096, max_value=8192),
       st.text(max_size=20), st.dictionaries(keys, st.integers(min_value=-5, max_value=5), max_size=3))
def test_amqp_content_frames_roundtrip(body, frame_max, ctype, headers):
    m = codec.Method("basic.publish", {"exchange": "x", "routing_key": "rk"})
    props = codec.Properties(content_type=ctype or None, headers=headers or None, delivery_mode=2)
    frames = codec.content_frames(1, m, body, props, frame_max)
    buf = b"".join(frames)
    pos, out = 0, []
    while pos < len(buf):
        ftype, ch, size = __import__("struct").unpack(">BHI", buf[pos:pos + 7])
        assert size + 8 <= frame_max and buf[pos + 7 + size] == 0xCE
        out.append((ftype, buf[pos + 7:pos + 7 + size]))
        pos += 8 + size
    assert out[0][0] == 1 and codec.decode_method(out[0][1]).name == "basic.publish"
    cls, size, p2 = codec.decode_header(out[1][1])
    assert size == len(body) and p2.content_type == (ctype or None) and (p2.headers or None) == (headers or None)
    assert b"".join(x[1] for x in out[2:]) == body


# ----------------------------------------------------------------- protobuf


@SETTINGS
@given(st.integers(min_value=0, max_value=2**64 - 1))
def test_varint_roundtrip(v):
    enc = wire.encode_varint(v)
    assert wire.decode_varint(enc, 0) == (v, len(enc))


@SETTINGS
@given(st.integers(min_value=-(2**63), max_value=-1))
def test_negative_varint_is_twos_complement(v):
    enc = wire.encode_varint(v)
    assert len(enc) == 10 and wire.decode_varint(enc, 0)[0] == v + 2**64


media = st.builds(messages.Media, id=st.text(max_size=20), name=st.text(max_size=20),
                  creator=st.integers(0, 3), creator_id=st.text(max_size=10), type=st.integers(0, 2),
                  source=st.integers(0, 4), source_uri=st.text(max_size=40), metadata=st.integers(0, 3),
                  metadata_id=st.text(max_size=10), status=st.integers(-(2**63), 2**63 - 1))


@SETTINGS
@given(st.text(max_size=30), media)
def test_download_envelope_roundtrip(created, m):
    d = messages.Download(created_at=created, media=m)
    back = messages.Download.decode(d.encode())
    assert back.created_at == created and back.media == m
    # Convert.from_download re-emits the media bytes verbatim
    c = messages.Convert.from_download(back, "t")
    assert messages.Convert.decode(c.encode()).media == m


@SETTINGS
@given(st.binary(max_size=60))
def test_envelope_garbage_raises_decode_error(b):
    try:
        messages.Download.decode(b)
    except wire.DecodeError:
        pass


# ----------------------------------------------------------------- peer wire


class _FakeReader:
    def __init__(self, chunks):
        self.chunks = list(chunks)

    async def read(self, n):
        return self.chunks.pop(0) if self.chunks else b""


msgs = st.lists(st.one_of(st.none(), st.tuples(st.integers(0, 20), st.binary(max_size=300))), max_size=30)


@SETTINGS
@given(msgs, st.lists(st.integers(1, 97), min_size=1, max_size=50))
def test_wire_parses_any_segmentation(ms, cuts):
    import struct
    stream = b"".join(b"\x00\x00\x00\x00" if m is None else struct.pack(">IB", len(m[1]) + 1, m[0]) + m[1]
                      for m in ms)
    chunks, pos, k = [], 0, 0
    while pos < len(stream):
        n = cuts[k % len(cuts)]
        chunks.append(stream[pos:pos + n])
        pos += n
        k += 1

    async def run():
        w = pw.Wire(_FakeReader(chunks), None)
        out = []
        while len(out) < len(ms):
            out += await w.read_batch()
        return out
    got = asyncio.run(run()) if ms else []
    assert got == [None if m is None else (m[0], m[1]) for m in ms]


# ----------------------------------------------------------------- crypto / S3 framing


@SETTINGS
@given(st.binary(min_size=1, max_size=64), st.binary(max_size=5000), st.integers(1, 4999))
def test_rc4_split_stream_symmetry(key, data, cut):
    a, b = hashing._host.Rc4(key), hashing._host.Rc4(key)
    ct = a.crypt(data[:cut]) + a.crypt(data[cut:])
    assert b.crypt(ct) == data


KEY = bytes(range(32))
SCOPE = "20130524/us-east-1/s3/aws4_request"
DATE = "20130524T000000Z"
SEED = "4f232c4386841ef735655705268965c44a0e4690baa4adea153f7db9fa80a0a9"


@SETTINGS
@given(st.binary(max_size=20000), st.sampled_from([8192, 16384, 65536]), st.sampled_from([1, 3]))
def test_aws_chunked_encode_decode_roundtrip(data, chunk, threads):
    enc, last = hashing.aws_chunk_encode(KEY, DATE, SCOPE, SEED, data, chunk, final=True, threads=threads)
    ok, dec, err = hashing.aws_chunk_decode(KEY, DATE, SCOPE, SEED, enc, threads=threads)
    assert ok and dec == data and err == ""
    sigs = hashing.chunk_signatures(KEY, DATE, SCOPE, SEED, data, chunk, include_final=True, threads=threads)
    assert sigs[-1] == last
    if enc:
        bad = bytearray(enc)
        bad[-40] ^= 1                         # flip a bit inside the final signature / frame
        ok2, _d, _e = hashing.aws_chunk_decode(KEY, DATE, SCOPE, SEED, bytes(bad))
        assert not ok2


@pytest.mark.parametrize("n", [0, 1, 63, 64, 65])
def test_aws_chunked_boundaries(n):
    data = bytes(range(256)) * 1 + b"z" * n
    enc, _ = hashing.aws_chunk_encode(KEY, DATE, SCOPE, SEED, data, 8192, final=True)
    assert hashing.aws_chunk_decode(KEY, DATE, SCOPE, SEED, enc)[1] == data


# ------------------------------------------------------------ S3 multipart plan

@SETTINGS
@given(st.integers(min_value=0, max_value=5 << 40), st.integers(min_value=1, max_value=6 << 30))
def test_multipart_plan_invariants(size, part_size):
    """minio-go optimalPartInfo's contract for any object up to 5 TiB: parts of
    5 MiB..5 GiB, at most 10,000 of them, covering the object with no empty
    last part, the part size a multiple of the configured one unless capped."""
    from tritondl.s3.client import MAX_PART_SIZE, MAX_PARTS, MIN_PART_SIZE, plan_parts
    ps, n = plan_parts(size, part_size)
    assert MIN_PART_SIZE <= ps <= MAX_PART_SIZE
    assert 1 <= n <= MAX_PARTS and ps * n >= size
    assert size == 0 or (n - 1) * ps < size
    base = max(part_size, MIN_PART_SIZE)
    assert ps == MAX_PART_SIZE or ps % base == 0


@SETTINGS
@given(st.integers(min_value=(5 << 40) + 1, max_value=1 << 50))
def test_multipart_plan_refuses_objects_over_5_tib(size):
    from tritondl.s3.client import S3Error, plan_parts
    with pytest.raises(S3Error):
        plan_parts(size, 16 << 20)


# ------------------------------------------------- HTTP chunked transfer decoding

@SETTINGS
@given(st.binary(max_size=3000), st.lists(st.integers(1, 700), min_size=1, max_size=12),
       st.booleans(), st.booleans(), st.integers(0, 4000))
def test_native_chunked_decoder_roundtrip(payload, sizes, ext, trailer, cut):
    """Any chunking of any payload (chunk extensions, trailer fields, and the
    head/body boundary anywhere: ``prefix`` = bytes that arrived with the head)
    decodes to exactly the payload, and the connection stays reusable."""
    import os
    import socket
    import tempfile

    from tritondl.utils import rawhttp
    relay = rawhttp.relay_module()
    if relay is None:
        pytest.skip("native relay not built")
    body, pos, k = bytearray(), 0, 0
    while pos < len(payload):
        n = min(sizes[k % len(sizes)], len(payload) - pos)
        body += f"{n:x}{';a=b' if ext else ''}\r\n".encode() + payload[pos:pos + n] + b"\r\n"
        pos += n
        k += 1
    body += b"0\r\n" + (b"X-Sum: 1\r\n" if trailer else b"") + b"\r\n"
    cut = min(cut, len(body))
    with tempfile.TemporaryDirectory() as d:
        fd = os.open(os.path.join(d, "out"), os.O_RDWR | os.O_CREAT, 0o644)
        a, b = socket.socketpair()
        try:
            a.sendall(bytes(body[cut:]))
            got, _eof, err, reusable = relay.recv_body(b.fileno(), fd, 0, -1, bytes(body[:cut]), None,
                                                       chunked=True)
            assert err == "" and got == len(payload) and reusable
            assert os.pread(fd, len(payload) + 1, 0) == payload
        finally:
            a.close()
            b.close()
            os.close(fd)


# ------------------------------------------------- server-supplied file names

def _usable_name(n: str, d: str) -> None:
    from tritondl.fetch.http import _NAME_MAX
    assert n not in (".", "..") and "/" not in n and "\\" not in n
    assert not any(ord(c) < 32 or c == "\x7f" for c in n)
    assert len(n.encode()) <= _NAME_MAX          # encodes: no lone surrogates
    # the download's own files land inside the job dir, whatever the server said
    for suffix in ("", ".part", ".part.meta.tmp"):
        with open(os.path.join(d, n + suffix), "wb"):
            pass
    assert sorted(os.listdir(d)) == sorted(n + s for s in ("", ".part", ".part.meta.tmp"))
    for f in os.listdir(d):
        os.unlink(os.path.join(d, f))


names = st.text(max_size=300) | st.text(st.sampled_from("ab./\\\x00\n é"), max_size=12)


@SETTINGS
@given(names)
def test_server_file_names_are_one_creatable_component(s):
    """Any Content-Disposition (plain, quoted, RFC 5987) or URL path yields ""
    or one component the job dir can hold with its sidecars."""
    import tempfile
    from urllib.parse import quote
    from tritondl.fetch.http import filename_from_disposition, filename_from_url
    got = [filename_from_disposition(cd) for cd in
           (s, f'attachment; filename="{s}"', f"attachment; filename*=UTF-8''{quote(s, safe='')}")]
    got.append(filename_from_url("http://h/dir/" + quote(s, safe="/")))
    with tempfile.TemporaryDirectory() as d:
        for n in got:
            if n:
                _usable_name(n, d)


@SETTINGS
@given(st.text(st.characters(blacklist_categories=("Cs", "Cc"), blacklist_characters="/\\\"'%;"),
               min_size=1, max_size=400),
       st.sampled_from(["mkv", "mp4", "avi", "en.srt"]))
def test_long_names_keep_their_extension_and_short_ones_are_untouched(stem, ext):
    from urllib.parse import quote
    from tritondl.fetch.http import _NAME_MAX, filename_from_url
    name = f"{stem}.{ext}"
    n = filename_from_url("http://h/" + quote(name))
    if len(name.encode()) <= _NAME_MAX:
        assert n == name
    else:
        last = ext.rpartition(".")[2]
        assert n.endswith("." + last) and len(n.encode()) <= _NAME_MAX
        assert name.startswith(n[:-len(last) - 1])


# ------------------------------------------------------------ SigV4 UriEncode

_UNRESERVED = set(b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_.~")


def _uri_encode_model(s: str, encode_slash: bool) -> str:
    """The AWS SigV4 UriEncode rule, byte by byte over UTF-8."""
    keep = _UNRESERVED if encode_slash else _UNRESERVED | {ord("/")}
    return "".join(chr(b) if b in keep else f"%{b:02X}" for b in s.encode())


@SETTINGS
@given(st.text(st.characters(blacklist_categories=("Cs",)), max_size=60) |
       st.text(st.sampled_from("aZ09-_.~/ +=%&?é€😀"), max_size=20), st.booleans())
def test_sigv4_uri_encode_matches_the_spec_rule(s, encode_slash):
    from tritondl.s3 import sigv4
    assert sigv4.uri_encode(s, encode_slash) == _uri_encode_model(s, encode_slash)


@SETTINGS
@given(st.lists(st.tuples(st.text(max_size=8, alphabet=st.characters(blacklist_categories=("Cs",))),
                          st.text(max_size=8, alphabet=st.characters(blacklist_categories=("Cs",)))),
                max_size=6))
def test_sigv4_canonical_query_sorts_encoded_pairs(pairs):
    from tritondl.s3 import sigv4
    want = "&".join(f"{k}={v}" for k, v in sorted((_uri_encode_model(k, True), _uri_encode_model(v, True))
                                                  for k, v in pairs))
    assert sigv4.canonical_query(pairs) == want


# ------------------------------------------- untrusted BitTorrent inputs (fuzz)
# Peers, trackers and .torrent files are remote input: their parsers may only
# raise their own error types, whatever shape the (valid) bencoding has.

_bleaf = st.integers(-5, 70000) | st.binary(max_size=40) | st.sampled_from([b"..", b"x/y", b"", b"\x00", b"a.mkv"])
_bkeys = st.sampled_from([b"", b"length", b"path", b"pieces root", b"attr", b"ip", b"port", b"m", b"ut_metadata",
                          b"msg_type", b"piece", b"added", b"added6", b"dropped", b"name", b"files"])
_bany = st.recursive(_bleaf, lambda k: st.lists(k, max_size=4) | st.dictionaries(_bkeys, k, max_size=4),
                     max_leaves=14)


@SETTINGS
@given(st.dictionaries(st.sampled_from([b"name", b"piece length", b"pieces", b"files", b"length",
                                        b"meta version", b"file tree", b"private"]), _bany, max_size=8))
def test_info_dict_of_any_shape_raises_only_metainfo_error(d):
    from tritondl.fetch.bt.metainfo import Info, MetainfoError
    try:
        info = Info.parse(bencode.encode(d))
    except MetainfoError:
        return
    for f in info.files:                       # whatever was accepted is safe to put on disk
        assert all(c not in ("", ".", "..") and "/" not in c for c in f.path)


@SETTINGS
@given(st.dictionaries(st.sampled_from([b"info", b"announce", b"announce-list", b"url-list", b"piece layers"]),
                       _bany, max_size=5), st.text(max_size=80))
@example({}, "xt=urn:btih:" + "ab" * 20 + "&x.pe=1.2.3.4:²")      # a Unicode digit in a peer port
def test_torrent_file_and_magnet_raise_only_metainfo_error(d, q):
    from tritondl.fetch.bt.metainfo import Metainfo, MetainfoError, parse_magnet
    for f in (lambda: Metainfo.parse(bencode.encode(d)), lambda: parse_magnet("magnet:?" + q)):
        try:
            f()
        except MetainfoError:
            pass


@SETTINGS
@given(_bany | st.dictionaries(st.sampled_from([b"failure reason", b"interval", b"peers", b"peers6",
                                                b"complete", b"incomplete"]), _bany, max_size=6),
       st.binary(max_size=30))
def test_tracker_reply_of_any_shape_raises_only_tracker_error(d, junk):
    from tritondl.fetch.bt.tracker import TrackerError, parse_announce_response
    for body in (bencode.encode(d), junk):
        try:
            r = parse_announce_response(body)
        except TrackerError:
            continue
        assert r.interval > 0 and all(0 < port < 65536 for _ip, port in r.peers)


@SETTINGS
@given(_bany, st.binary(max_size=30))
def test_extension_messages_of_any_shape_raise_only_peer_error(d, tail):
    for parse in (pw.parse_ext_handshake, pw.parse_pex, pw.parse_meta_msg):
        for body in (bencode.encode(d) + tail, tail):
            try:
                parse(body)
            except pw.PeerError:
                pass


@SETTINGS
@given(st.dictionaries(st.sampled_from([b"t", b"y", b"q", b"a", b"r", b"e"]),
                       _bany | st.sampled_from([b"q", b"r", b"e", b"ping", b"find_node", b"get_peers",
                                                b"announce_peer", b"aa"]), max_size=6) |
       _bany, st.binary(max_size=30))
@example({b"t": [1], b"y": b"r", b"r": {}}, b"")        # an unhashable transaction id
def test_dht_datagram_of_any_shape_is_absorbed(msg, junk):
    """Any KRPC datagram — query, reply or error, of any shape, from the
    node a transaction waits on or another — is answered, resolves that
    transaction or is dropped; nothing escapes into the event loop."""
    from tritondl.fetch.bt import dht as D

    async def main():
        n = D.DHTNode()
        f = asyncio.get_running_loop().create_future()
        n._pending[b"aa"] = (("1.2.3.4", 5), f)
        for data in (bencode.encode(msg), junk):
            for addr in (("1.2.3.4", 5), ("5.6.7.8", 9)):
                n._on_datagram(data, addr, 2)
        if f.done() and not f.cancelled():
            f.exception()
    asyncio.run(main())


# ------------------------------------------------- HTTP response heads (fuzz)

_head_line = st.sampled_from(["Content-Length: 10", "Content-Length: -1", "Content-Length: 1e3",
                              "Content-Length: 5, 5", "Content-Length: 5, 6", "Content-Length: ²",
                              "Transfer-Encoding: chunked", "Connection: close", "Connection: keep-alive",
                              "X: y", ": novalue", "bare"]) | st.text(max_size=30)


@SETTINGS
@given(st.sampled_from(["HTTP/1.1 200 OK", "HTTP/1.0 206 Partial", "HTTP/1.1 ²00 OK", "HTTP/1.1 20 OK",
                        "ICY 200 OK", "HTTP/1.1 999"]) | st.text(max_size=20),
       st.lists(_head_line, max_size=6))
def test_response_head_of_any_shape(status, lines):
    """Any response head parses to a status of three ASCII digits and a
    Content-Length that is absent or a non-negative integer — or raises
    RawHTTPError; never another exception (the relay sizes files by it)."""
    from tritondl.utils.rawhttp import RawHTTPError, parse_head
    raw = "\r\n".join([status] + lines).encode("latin-1", "replace")
    try:
        h = parse_head(raw)
    except RawHTTPError:
        return
    assert 0 <= h.status <= 999
    cl = h.content_length
    assert cl is None or cl >= 0
    assert not (h.keep_alive and h.chunked and "Content-Length" in h.headers)


def test_tracker_dict_peers_take_ips_and_dns_names():
    from tritondl.fetch.bt.tracker import parse_announce_response
    body = bencode.encode({b"interval": 60, b"peers": [
        {b"ip": b"10.0.0.1", b"port": 6881}, {b"ip": b"seed.example.org", b"port": 51413},
        {b"ip": b"::1", b"port": 1}, {b"ip": b"bad host", b"port": 2}, {b"ip": b"10.0.0.2", b"port": 0},
        {b"ip": 7, b"port": 3}, {b"port": 4}]})
    r = parse_announce_response(body)
    assert r.peers == [("10.0.0.1", 6881), ("seed.example.org", 51413), ("::1", 1)] and r.interval == 60


@SETTINGS
@given(st.binary(max_size=24) | st.sampled_from([b"-5", b"+5", b"0x5", b" 5", b"", b"5;ext=1", b"fffffffffffffffff",
                                                 b"A", b"10 "]))
def test_chunk_size_line_is_hex_or_an_error(line):
    """A chunk-size line is parsed as RFC 9112 hex (with optional
    extensions and trailing blanks) or refused; never a negative size."""
    from tritondl.utils.rawhttp import RawHTTPError, _chunk_size
    try:
        n = _chunk_size(line)
    except RawHTTPError:
        return
    assert n >= 0
    digits = line.split(b";", 1)[0].rstrip(b" \t")
    assert int(digits, 16) == n and not digits.startswith((b"-", b"+", b"0x", b"0X"))
