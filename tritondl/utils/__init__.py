"""Cross-cutting utilities: config, logging, backoff, Go-compatible helpers."""
