"""Media uploader — reference component C9 (``internal/uploader/uploader.go``).

* ``Uploader.from_env(bucket)`` parses ``S3_ENDPOINT`` (TLS iff https,
  host[:port]) and uses the credential chain ``[EnvGeneric, EnvAWS,
  EnvMinio]`` with auto bucket lookup (``uploader.go:24-59``).
* ``upload_files(media_id, base_dir, files)`` ensures the bucket exists
  (creating it in region ``""`` if missing, ``:64-70``) and streams every file
  to ``<mediaId>/original/<base64.StdEncoding(basename)>`` (``:72-94``) —
  the std alphabet may contain ``/`` which creates extra key "directories";
  kept for compatibility with the downstream converter.

Deviations (defect B8): any per-file failure fails the job (the reference
logged and skipped, and always returned nil), file handles are always
closed, and uploads of a job's files run concurrently (bounded).

The reference re-checked the bucket on every ``UploadFiles`` (one HEAD per
job).  Here the check is cached, and a ``NoSuchBucket`` reply (bucket
deleted or recreated — possibly in another region) drops the cache, re-runs
the ensure step and retries the upload once, so the worker heals without a
restart.  ``from_env`` refuses an unusable ``S3_ENDPOINT`` (``ValueError``),
as ``minio.NewWithOptions`` did (fatal in ``downloader.go:95-98``).
"""

from __future__ import annotations

import asyncio
import base64
import os
from dataclasses import dataclass

from ..utils.gocompat import go_base, go_join
from ..utils.log import log
from .client import Endpoint, S3Client, S3Error
from .credentials import default_chain


def object_key(media_id: str, file_name: str) -> str:
    """``filepath.Join(mediaId, "original/", base64.StdEncoding(basename))``."""
    enc = base64.b64encode(go_base(file_name).encode("utf-8", "surrogateescape")).decode()
    return go_join(media_id, "original/", enc)


@dataclass
class UploadResult:
    key: str
    size: int
    etag: str


class UploadError(Exception):
    pass


# next to each local file: the state of its interrupted multipart upload (resume on redelivery)
RESUME_SUFFIX = ".s3upload"


class Uploader:
    def __init__(self, bucket: str, client: S3Client, *, file_concurrency: int = 2) -> None:
        self.heals = 0
        self.stalls = 0                      # streamed uploads that fell back to upload-after-download
        self.bucket = bucket
        self.client = client
        self.file_concurrency = max(1, file_concurrency)
        self._bucket_ok = False

    @classmethod
    def from_env(cls, bucket: str, s3_endpoint: str | None = None, *, region: str = "",
                 part_size: int = 16 << 20, multipart_threshold: int = 64 << 20, parallel_parts: int = 4,
                 env=None, sign_threads: int = 4, ca_file: str = "", hash_device: str = "cpu",
                 max_retries: int = 9, retry_unit: float = 1.0, retry_cap: float = 30.0) -> "Uploader":
        ep = s3_endpoint if s3_endpoint is not None else os.environ.get("S3_ENDPOINT", "")
        Endpoint.parse(ep)                       # ValueError on an endpoint minio-go would refuse
        client = S3Client(ep, default_chain(env), region=region, part_size=part_size,
                          multipart_threshold=multipart_threshold, parallel_parts=parallel_parts,
                          sign_threads=sign_threads, ca_file=ca_file, hash_device=hash_device,
                          max_retries=max_retries, retry_unit=retry_unit, retry_cap=retry_cap)
        return cls(bucket, client)

    async def ensure_bucket(self) -> None:
        if self._bucket_ok:
            return
        try:
            exists = await self.client.bucket_exists(self.bucket)
        except S3Error as e:
            log.warn("failed to check bucket: %s", e)
            return
        if not exists:
            try:
                await self.client.make_bucket(self.bucket, "")
                log.info("created bucket")
            except S3Error as e:
                if e.code not in ("BucketAlreadyOwnedByYou", "BucketAlreadyExists"):
                    log.warn("failed to create bucket: %s", e)
                    return
        self._bucket_ok = True

    async def _healing(self, put):
        """Run ``put()``; on NoSuchBucket re-ensure the bucket and retry once."""
        try:
            return await put()
        except S3Error as e:
            if e.code != "NoSuchBucket":
                raise
            log.with_field("bucket", self.bucket).warn("bucket vanished; re-creating it and retrying the upload")
            self._bucket_ok = False
            self.client.forget_bucket(self.bucket)
            self.heals += 1
            await self.ensure_bucket()
            return await put()

    async def upload_files(self, media_id: str, base_dir: str, files: list[str]) -> list[UploadResult]:
        await self.ensure_bucket()
        sem = asyncio.Semaphore(self.file_concurrency)

        async def one(path: str) -> UploadResult:
            async with sem:
                try:
                    size = os.stat(path).st_size
                except OSError as e:
                    raise UploadError(f"failed to stat file {path}: {e}") from e
                key = object_key(media_id, path)
                log.info("starting upload of file '%s'", go_base(key))
                try:
                    etag = await self._healing(lambda: self.client.put_object(
                        self.bucket, key, path, size, resume_path=path + RESUME_SUFFIX))
                except (S3Error, OSError) as e:
                    raise UploadError(f"failed to upload file {path}: {e}") from e
                log.info("finished upload")
                return UploadResult(key, size, etag)

        return list(await asyncio.gather(*(one(f) for f in files)))

    async def upload_stream(self, media_id: str, name: str, src: int | str, size: int, wait_bytes=None,
                            flow=None, resume_path: str | None = None) -> UploadResult:
        """Upload one file that may still be growing (``wait_bytes`` gates reads;
        ``flow`` is the download's native progress, followed without Python).

        If the download stalls under the upload (no progress for the flow's
        ``stall`` seconds), the PUT is dropped before the store's own request
        timeout fails it (S3: 400 ``RequestTimeout`` after ~20 s of silence),
        and the file is uploaded once the download has finished.  A multipart
        upload keeps the parts that landed (``resume_path``) and sends only
        the rest.  The reference always uploaded after the download
        (``uploader.go:89`` after ``downloader.go:116-130``)."""
        await self.ensure_bucket()
        key = object_key(media_id, name)
        log.info("starting upload of file '%s'", go_base(key))
        try:
            try:
                etag = await self._healing(lambda: self.client.put_object(self.bucket, key, src, size,
                                                                          wait_bytes=wait_bytes, flow=flow,
                                                                          resume_path=resume_path))
            except S3Error as e:
                if e.code != "SourceStalled" or wait_bytes is None:
                    raise
                self.stalls += 1
                log.with_fields(key=go_base(key), error=e.message).warn(
                    "download stalled under a streamed upload; uploading once the download is done")
                await wait_bytes(size)
                etag = await self._healing(lambda: self.client.put_object(self.bucket, key, src, size,
                                                                          resume_path=resume_path))
        except (S3Error, OSError) as e:
            raise UploadError(f"failed to upload file {name}: {e}") from e
        log.info("finished upload")
        return UploadResult(key, size, etag)

    async def close(self) -> None:
        await self.client.close()
