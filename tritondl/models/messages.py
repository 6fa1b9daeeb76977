"""Wire schema: ``api.Media``, ``api.Download``, ``api.Convert`` (reference C10).

Used fields (reference): ``Download.Media.Id``, ``Download.Media.SourceURI``
(``cmd/downloader/downloader.go:116``), ``Convert.CreatedAt = time.Now().String()``
and ``Convert.Media = job.Media`` (``:136-139``); gogo ``proto.Marshal`` /
``Unmarshal`` (``:106,141``).

TODO verify against tritonmedia.go v1.0.2 api.proto — the field numbers
below are our best reconstruction (not available offline).  Robustness by
construction: every message keeps its unknown fields and the raw bytes of
``media`` so that ``Convert.media`` is re-emitted exactly as received.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from enum import IntEnum

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
        for fn in range(1, 11):
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
        for fn, wt, val, raw in wire.iter_fields(buf):
            if fn == 1 and wt == wire.LEN:
                try:
                    m.created_at = val.decode("utf-8")  # type: ignore[union-attr]
                except UnicodeDecodeError as e:
                    raise wire.DecodeError("invalid utf-8 in createdAt") from e
            elif fn == 2 and wt == wire.LEN:
                # proto3 merge semantics for repeated occurrences: concatenate
                m.media_raw = (m.media_raw or b"") + val  # type: ignore[operator]
                m.media = Media.decode(m.media_raw)
            else:
                unk += raw
        m.unknown = bytes(unk)
        return m

    def encode(self) -> bytes:
        out = bytearray(wire.enc_string(1, self.created_at))
        if self.media_raw is not None:
            out += wire.enc_bytes_always(2, self.media_raw)
        elif self.media is not None:
            out += wire.enc_bytes_always(2, self.media.encode())
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
