"""tritondl_testkit — the test and benchmark harness for :mod:`tritondl`.

Kept out of the product package so it ships in neither the wheel
(``pyproject.toml`` packages ``tritondl`` only) nor the worker image
(``docker/Dockerfile`` copies ``tritondl/`` only):

* ``tritondl_testkit.fakes``          – in-process AMQP broker, S3, HTTP origin,
                                         BitTorrent swarm, proxy, UPnP IGD
* ``tritondl_testkit.bench_job``      – the single-job stack ``bench.py`` times
* ``tritondl_testkit.bench_producer`` – the shared-broker job producer
* ``tritondl_testkit.soak``           – the long-running memory soak
"""
