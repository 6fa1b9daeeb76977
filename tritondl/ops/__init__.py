"""Native hot paths.

* :mod:`tritondl.ops.hashing` — host C++ hashing (OpenSSL EVP, threaded piece
  verification, aws-chunked signature chains) and the HIP gfx950 batched
  SHA-1 / SHA-256 piece kernels with a pinned, double-buffered file pipeline.
"""

from .hashing import (Hasher, digest, gpu_available, hash_file, piece_hashes, verify_pieces)

__all__ = ["Hasher", "digest", "hash_file", "piece_hashes", "verify_pieces", "gpu_available"]
