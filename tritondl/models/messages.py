"""Wire schema: ``api.Media``, ``api.Download``, ``api.Convert`` (reference C10).

Used fields (reference): ``Download.Media.Id``, ``Download.Media.SourceURI``
(``cmd/downloader/downloader.go:116``), ``Convert.CreatedAt = time.Now().String()``
and ``Convert.Media = job.Media`` (``:136-139``); gogo ``proto.Marshal`` /
``Unmarshal`` (``:106,141``).

Parity unpinned: the field numbers below are a reconstruction of
tritonmedia.go v1.0.2 ``api.proto`` (the schema is not vendored and not
available offline, ``go.sum:272-273``).  Two safeguards: every message keeps
its unknown fields and the raw bytes of ``media``, so ``Convert.media`` is
re-emitted exactly as received; and the numbers are operator-overridable
without a rebuild (``TRITONDL_MEDIA_FIELDS="id=1,source_uri=7"``,
``TRITONDL_ENVELOPE_FIELDS="created_at=1,media=2"``; see
:func:`configure_fields`).
"""

from __future__ import annotations

from dataclasses import dataclass
from enum import IntEnum

import os

from . import wire

# ----------------------------------------------------------------- enums


class CreatorType(IntEnum):
    TRELLO = 0
    API = 1


class MediaType(IntEnum):
    MOVIE = 0
    TV = 1


class SourceType(IntEnum):
    HTTP = 0
    TORRENT = 1
    FILE = 2


class MetadataType(IntEnum):
    TVDB = 0
    IMDB = 1
    MAL = 2


class MediaStatus(IntEnum):
    QUEUED = 0
    DOWNLOADING = 1
    CONVERTING = 2
    UPLOADING = 3
    DEPLOYED = 4


# ----------------------------------------------------------------- Media

_MEDIA_STR = {1: "id", 2: "name", 4: "creator_id", 7: "source_uri", 9: "metadata_id"}
_MEDIA_INT = {3: "creator", 5: "type", 6: "source", 8: "metadata", 10: "status"}
_ENV_FIELDS = {"created_at": 1, "media": 2}         # api.Download / api.Convert
_DEFAULT_MEDIA = ({**_MEDIA_STR}, {**_MEDIA_INT})


def _parse_spec(spec: str, names: set[str], what: str) -> dict[str, int]:
    out: dict[str, int] = {}
    for item in filter(None, (x.strip() for x in spec.split(","))):
        name, sep, num = item.partition("=")
        name = name.strip()
        if not sep or name not in names:
            raise ValueError(f"{what}: unknown field {name!r} (known: {', '.join(sorted(names))})")
        try:
            n = int(num)
        except ValueError:
            raise ValueError(f"{what}: field number for {name!r} is not an integer: {num!r}") from None
        if not 1 <= n < (1 << 29) or 19000 <= n <= 19999:
            raise ValueError(f"{what}: {n} is not a valid protobuf field number")
        out[name] = n
    return out


def configure_fields(media: str = "", envelope: str = "") -> None:
    """Override protobuf field numbers (``"name=N,..."``) for ``api.Media``
    and the ``api.Download``/``api.Convert`` envelope; names not listed keep
    their reconstructed number.  Numbers must stay unique per message.  Called
    at import with ``TRITONDL_MEDIA_FIELDS`` / ``TRITONDL_ENVELOPE_FIELDS``;
    ``configure_fields()`` restores the defaults."""
    dstr, dint = _DEFAULT_MEDIA
    by_name = {v: k for k, v in {**dstr, **dint}.items()}
    by_name.update(_parse_spec(media, set(by_name), "TRITONDL_MEDIA_FIELDS"))
    if len(set(by_name.values())) != len(by_name):
        raise ValueError(f"TRITONDL_MEDIA_FIELDS: duplicate field numbers in {by_name}")
    env = {"created_at": 1, "media": 2}
    env.update(_parse_spec(envelope, set(env), "TRITONDL_ENVELOPE_FIELDS"))
    if env["created_at"] == env["media"]:
        raise ValueError("TRITONDL_ENVELOPE_FIELDS: created_at and media share a number")
    _MEDIA_STR.clear()
    _MEDIA_STR.update({by_name[name]: name for name in dstr.values()})
    _MEDIA_INT.clear()
    _MEDIA_INT.update({by_name[name]: name for name in dint.values()})
    _ENV_FIELDS.update(env)


@dataclass
class Media:
    id: str = ""
    name: str = ""
    creator: int = 0
    creator_id: str = ""
    type: int = 0
    source: int = 0
    source_uri: str = ""
    metadata: int = 0
    metadata_id: str = ""
    status: int = 0
    unknown: bytes = b""

    @classmethod
    def decode(cls, buf: bytes) -> "Media":
        m = cls()
        unk = bytearray()
        for fn, wt, val, raw in wire.iter_fields(buf):
            if fn in _MEDIA_STR and wt == wire.LEN:
                try:
                    setattr(m, _MEDIA_STR[fn], val.decode("utf-8"))  # type: ignore[union-attr]
                except UnicodeDecodeError as e:
                    raise wire.DecodeError(f"invalid utf-8 in field {fn}") from e
            elif fn in _MEDIA_INT and wt == wire.VARINT:
                v = int(val)  # type: ignore[arg-type]
                if v >= 1 << 63:
                    v -= 1 << 64
                setattr(m, _MEDIA_INT[fn], v)
            else:
                unk += raw
        m.unknown = bytes(unk)
        return m

    def encode(self) -> bytes:
        out = bytearray()
        for fn in sorted((*_MEDIA_STR, *_MEDIA_INT)):
            if fn in _MEDIA_STR:
                out += wire.enc_string(fn, getattr(self, _MEDIA_STR[fn]))
            else:
                out += wire.enc_varint_field(fn, int(getattr(self, _MEDIA_INT[fn])))
        out += self.unknown
        return bytes(out)

    def to_dict(self) -> dict:
        return {"id": self.id, "name": self.name, "creator": self.creator, "creatorId": self.creator_id,
                "type": self.type, "source": self.source, "sourceURI": self.source_uri,
                "metadata": self.metadata, "metadataId": self.metadata_id, "status": self.status}


# ----------------------------------------------------- Download / Convert


@dataclass
class _Envelope:
    """``{ string createdAt = 1; Media media = 2; }``"""

    created_at: str = ""
    media: Media | None = None
    media_raw: bytes | None = None     # exact bytes of the media sub-message as received
    unknown: bytes = b""

    @classmethod
    def decode(cls, buf: bytes):
        m = cls()
        unk = bytearray()
        f_created, f_media = _ENV_FIELDS["created_at"], _ENV_FIELDS["media"]
        for fn, wt, val, raw in wire.iter_fields(buf):
            if fn == f_created and wt == wire.LEN:
                try:
                    m.created_at = val.decode("utf-8")  # type: ignore[union-attr]
                except UnicodeDecodeError as e:
                    raise wire.DecodeError("invalid utf-8 in createdAt") from e
            elif fn == f_media and wt == wire.LEN:
                # proto3 merge semantics for repeated occurrences: concatenate
                m.media_raw = (m.media_raw or b"") + val  # type: ignore[operator]
                m.media = Media.decode(m.media_raw)
            else:
                unk += raw
        m.unknown = bytes(unk)
        return m

    def encode(self) -> bytes:
        f_created, f_media = _ENV_FIELDS["created_at"], _ENV_FIELDS["media"]
        out = bytearray(wire.enc_string(f_created, self.created_at))
        if self.media_raw is not None:
            out += wire.enc_bytes_always(f_media, self.media_raw)
        elif self.media is not None:
            out += wire.enc_bytes_always(f_media, self.media.encode())
        out += self.unknown
        return bytes(out)

    def to_dict(self) -> dict:
        return {"createdAt": self.created_at, "media": self.media.to_dict() if self.media else None}


class Download(_Envelope):
    pass


class Convert(_Envelope):
    @classmethod
    def from_download(cls, job: Download, created_at: str) -> "Convert":
        """``api.Convert{CreatedAt: time.Now().String(), Media: job.Media}``."""
        c = cls()
        c.created_at = created_at
        c.media = job.media
        c.media_raw = job.media_raw
        return c


configure_fields(os.environ.get("TRITONDL_MEDIA_FIELDS", ""), os.environ.get("TRITONDL_ENVELOPE_FIELDS", ""))
