"""S3 object storage: SigV4 signer, credential chain, async client
(streaming + multipart) and the media uploader (reference C9/C9a)."""

from .client import Endpoint, S3Client, S3Error
from .credentials import Chain, EnvAWS, EnvGeneric, EnvMinio, Static, Value, default_chain
from .uploader import UploadError, Uploader, UploadResult, object_key

__all__ = ["S3Client", "S3Error", "Endpoint", "Chain", "EnvGeneric", "EnvAWS", "EnvMinio", "Static", "Value",
           "default_chain", "Uploader", "UploadResult", "UploadError", "object_key"]
