"""Message models: the protobuf wire schema shared with the other tritonmedia
services (``api.Media`` / ``api.Download`` / ``api.Convert``)."""

from .messages import (Convert, CreatorType, Download, Media, MediaStatus, MediaType, MetadataType,
                       SourceType)
from .wire import DecodeError

__all__ = ["Media", "Download", "Convert", "DecodeError", "CreatorType", "MediaType", "SourceType",
           "MetadataType", "MediaStatus"]
