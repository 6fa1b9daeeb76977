"""tritondl — MI355X-host-native media ingest worker.

Same capabilities as tritonmedia/downloader-go (reference: /root/reference):
consume protobuf ``Download`` jobs from RabbitMQ topic ``v1.download``, fetch
the source (HTTP(S) with resume, or BitTorrent magnet / .torrent), select the
media files, stream them to S3 bucket ``triton-staging`` and publish a
``Convert`` message on ``v1.convert``; the job is acked only after success.

Layout (mirrors SURVEY.md §7.1):

* ``tritondl.models``   – wire schema (protobuf Media/Download/Convert, C10)
* ``tritondl.amqp``     – AMQP 0-9-1 client: codec, connection, topology,
                          consumer fan-in, publisher, reconnect (C2-C4)
* ``tritondl.fetch``    – download dispatcher + HTTP + BitTorrent (C5-C7)
* ``tritondl.select``   – media-file selector ``process.Dir`` (C8)
* ``tritondl.s3``       – S3 SigV4 uploader + credential chain (C9, C9a)
* ``tritondl.ops``      – native hot paths: C++ SHA-1/SHA-256/MD5 and the
                          HIP (gfx950) batched piece-hash kernels
* ``tritondl.parallel`` – job-level data parallelism: worker pool /
                          competing consumers, rank wiring
* ``tritondl.utils``    – config, logging, backoff, profiler, metrics
* ``tritondl.service``  – the job orchestrator (C1), ``python -m tritondl``

The test harness (fake broker / S3 / origin / swarm, bench and soak
drivers) lives in the separate ``tritondl_testkit`` package, which is not
shipped in the wheel or the worker image.
"""

__version__ = "0.1.0"
