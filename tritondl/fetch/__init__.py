"""Fetch layer: download dispatcher (C5) and the protocol plug-ins —
HTTP(S) (C6) and BitTorrent (C7)."""

from .http import HTTPDownloader, HTTPDownloadError
from .registry import ClientImpl, ClientRegister, Dispatcher, ProgressSink, ProgressTracker, ProgressUpdate, \
    UnsupportedError

__all__ = ["Dispatcher", "ClientImpl", "ClientRegister", "ProgressUpdate", "ProgressSink", "ProgressTracker",
           "UnsupportedError", "HTTPDownloader", "HTTPDownloadError"]
