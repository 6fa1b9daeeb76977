"""Wire-schema tests: round trips, unknown-field preservation and wire
compatibility with the official protobuf runtime (dynamic descriptors)."""

import pytest

from tritondl.models import Convert, DecodeError, Download, Media
from tritondl.models import wire
from tritondl.utils.gocompat import go_time_string


def test_media_roundtrip():
    m = Media(id="abc", name="n", creator=1, creator_id="cid", type=1, source=1,
              source_uri="magnet:?xt=urn:btih:00", metadata=2, metadata_id="tt1", status=3)
    assert Media.decode(m.encode()) == m


def test_download_to_convert_preserves_media_bytes():
    # unknown field 15 inside media and 9 at top level must survive
    media = Media(id="x", source_uri="http://h/f.mkv").encode() + wire.enc_string(15, "future")
    d = wire.enc_string(1, "then") + wire.enc_bytes_always(2, media) + wire.enc_varint_field(9, 7)
    job = Download.decode(d)
    assert job.media.id == "x" and job.media.source_uri == "http://h/f.mkv"
    assert job.unknown == wire.enc_varint_field(9, 7)
    c = Convert.from_download(job, "now")
    out = Convert.decode(c.encode())
    assert out.media_raw == media
    assert out.created_at == "now"


@pytest.mark.parametrize("bad", [b"\x0a\x05ab", b"\xff", b"\x0b", b"\x00\x01"])
def test_decode_errors(bad):
    with pytest.raises(DecodeError):
        Download.decode(bad)


def test_varint_edges():
    for v in [0, 1, 127, 128, 300, 2**32, 2**63 - 1, 2**64 - 1]:
        assert wire.decode_varint(wire.encode_varint(v), 0)[0] == v
    assert wire.decode_varint(wire.encode_varint(-1), 0)[0] == 2**64 - 1


def _dynamic_classes():
    from google.protobuf import descriptor_pb2, descriptor_pool
    from google.protobuf import message_factory
    fdp = descriptor_pb2.FileDescriptorProto(name="api_test.proto", package="api", syntax="proto3")
    media = fdp.message_type.add(name="Media")
    T = descriptor_pb2.FieldDescriptorProto
    for num, name, typ in [(1, "id", T.TYPE_STRING), (2, "name", T.TYPE_STRING), (3, "creator", T.TYPE_INT32),
                           (4, "creatorId", T.TYPE_STRING), (5, "type", T.TYPE_INT32), (6, "source", T.TYPE_INT32),
                           (7, "sourceURI", T.TYPE_STRING), (8, "metadata", T.TYPE_INT32),
                           (9, "metadataId", T.TYPE_STRING), (10, "status", T.TYPE_INT32)]:
        media.field.add(name=name, number=num, type=typ, label=T.LABEL_OPTIONAL)
    for mname in ("Download", "Convert"):
        msg = fdp.message_type.add(name=mname)
        msg.field.add(name="createdAt", number=1, type=T.TYPE_STRING, label=T.LABEL_OPTIONAL)
        msg.field.add(name="media", number=2, type=T.TYPE_MESSAGE, type_name=".api.Media", label=T.LABEL_OPTIONAL)
    pool = descriptor_pool.DescriptorPool()
    fd = pool.Add(fdp)
    get = message_factory.GetMessageClass
    return get(pool.FindMessageTypeByName("api.Media")), get(pool.FindMessageTypeByName("api.Download"))


def test_wire_compat_with_protobuf_runtime():
    pytest.importorskip("google.protobuf")
    PMedia, PDownload = _dynamic_classes()
    pd = PDownload(createdAt="2020", media=PMedia(id="id1", sourceURI="https://x/y.mkv", type=1, status=2))
    ours = Download.decode(pd.SerializeToString())
    assert ours.media.id == "id1" and ours.media.source_uri == "https://x/y.mkv"
    assert ours.media.type == 1 and ours.media.status == 2
    back = PDownload()
    back.ParseFromString(ours.encode())
    assert back == pd
    # our encoder == protobuf's canonical encoding
    assert Media(id="id1", source_uri="https://x/y.mkv", type=1, status=2).encode() == \
        pd.media.SerializeToString()


def test_go_time_string_format():
    s = go_time_string(now_ns=1_600_000_000_123_450_000, mono_ns=1_500_000_000)
    date, clock, zone, abbr, mono = s.split(" ")
    assert clock.endswith(".12345") and len(date) == 10
    assert zone[0] in "+-" and len(zone) == 5
    assert mono == "m=+1.500000000"
    assert go_time_string(now_ns=1_600_000_000_000_000_000, mono_ns=0).split(" ")[1].count(".") == 0


def test_field_numbers_operator_override():
    """TRITONDL_MEDIA_FIELDS / TRITONDL_ENVELOPE_FIELDS remap the reconstructed
    field numbers (parity unpinned): a message written with another numbering
    decodes once the operator supplies it; media bytes still pass verbatim."""
    import pytest

    from tritondl.models import messages
    # the producer's schema: source_uri=3, creator=7 (swapped), createdAt=4, media=5
    media = (wire.enc_string(1, "m1") + wire.enc_string(3, "http://h/a.mkv") + wire.enc_varint_field(7, 1))
    body = wire.enc_string(4, "t0") + wire.enc_bytes_always(5, media)
    try:
        d = Download.decode(body)
        assert d.media is None and d.created_at == ""          # default numbering cannot read it
        messages.configure_fields("source_uri=3,creator=7", "created_at=4,media=5")
        d = Download.decode(body)
        assert (d.created_at, d.media.id, d.media.source_uri, d.media.creator) == ("t0", "m1", "http://h/a.mkv", 1)
        c = Convert.from_download(d, "now").encode()
        assert wire.enc_bytes_always(5, media) in c and c.startswith(wire.enc_string(4, "now"))
        assert Media.decode(Media(id="x", source_uri="u", creator=1).encode()).source_uri == "u"
        for bad in ("nope=3", "id=0", "id=19000", "id=x", "id=2"):   # unknown, invalid, reserved, duplicate
            with pytest.raises(ValueError):
                messages.configure_fields(bad)
        with pytest.raises(ValueError):
            messages.configure_fields("", "media=1")
    finally:
        messages.configure_fields()
    assert messages._MEDIA_STR[7] == "source_uri" and messages._ENV_FIELDS == {"created_at": 1, "media": 2}
