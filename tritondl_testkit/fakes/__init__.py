"""In-process fakes (AMQP broker, S3, HTTP origin, BitTorrent swarm) for tests, smoke and bench."""
