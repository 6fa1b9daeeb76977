// C ABI between the HIP module (_gpu_hash, hipcc) and the relay's S3 send
// pump (_relay, g++): the relay never links HIP; it receives this table as a
// PyCapsule from _gpu_hash.chunk_api() and calls through it.
#pragma once

#include <cstddef>

#define TDL_GPU_CHUNK_API_NAME "tritondl._gpu_hash.chunk_api"

struct TdlGpuChunkApi {
  int version;  // 1
  // SHA-256 of the ceil(len / chunk) consecutive `chunk`-byte messages at
  // host address `src` (the last one may be shorter); 32-byte digests to
  // `out`.  Blocking (the caller's thread sleeps on a blocking-sync event, it
  // does not spin); thread-safe, one HIP stream per calling thread.
  // Returns 0, or -1 with the reason in err.
  int (*sha256_chunks)(const void* src, size_t len, size_t chunk, unsigned char* out, char* err, size_t errlen);
};
