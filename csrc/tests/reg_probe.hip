// reg_probe: can the DMA engine read a torrent file straight from the page
// cache?  The GPU resume path copies page cache -> pinned staging with host
// reader threads (8 of the 16 CPUs) before each H2D copy; registering the
// file's read-only mapping with hipHostRegister would let the copy engine
// read it directly and leave every CPU to hash.  This measures, per GiB:
//   register      hipHostRegister of a MAP_SHARED PROT_READ file mapping
//   h2d           hipMemcpyAsync from that registered mapping to HBM
//   unregister    hipHostUnregister
// next to h2d from an ordinary pinned buffer (the staging ring's hop).
//
// Build: hipcc --offload-arch=gfx950 -O2 -o /tmp/reg_probe csrc/tests/reg_probe.hip
// Run:   /tmp/reg_probe [--dir /tmp] [--mb 1024] [--reps 3]
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::printf("{\"error\": \"%s\", \"call\": \"%s\"}\n", hipGetErrorString(e_), #x); \
      return false;                                                                   \
    }                                                                                 \
  } while (0)

bool run_mapping(const char* label, const std::string& path, size_t len, unsigned flags, bool populate,
                 void* dev, hipStream_t st) {
  const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) {
    perror("open");
    return false;
  }
  void* m = ::mmap(nullptr, len, PROT_READ, MAP_SHARED | (populate ? MAP_POPULATE : 0), fd, 0);
  ::close(fd);
  if (m == MAP_FAILED) {
    perror("mmap");
    return false;
  }
  double t = now_ms();
  hipError_t e = hipHostRegister(m, len, flags);
  const double reg = now_ms() - t;
  if (e != hipSuccess) {
    std::printf("{\"probe\": \"%s\", \"register\": \"failed: %s\", \"ms\": %.3f}\n", label, hipGetErrorString(e), reg);
    (void)hipGetLastError();
    ::munmap(m, len);
    return true;
  }
  void* devp = nullptr;
  (void)hipHostGetDevicePointer(&devp, m, 0);
  t = now_ms();
  CHECK(hipMemcpyAsync(dev, m, len, hipMemcpyHostToDevice, st));
  CHECK(hipStreamSynchronize(st));
  const double h2d = now_ms() - t;
  t = now_ms();
  CHECK(hipMemcpyAsync(dev, m, len, hipMemcpyHostToDevice, st));
  CHECK(hipStreamSynchronize(st));
  const double h2d2 = now_ms() - t;
  t = now_ms();
  CHECK(hipHostUnregister(m));
  const double unreg = now_ms() - t;
  ::munmap(m, len);
  std::printf("{\"probe\": \"%s\", \"register_ms\": %.3f, \"h2d_ms\": %.3f, \"h2d_again_ms\": %.3f, "
              "\"h2d_GBps\": %.1f, \"unregister_ms\": %.3f, \"dev_ptr\": %s}\n",
              label, reg, h2d, h2d2, len / h2d2 / 1e6, unreg, devp ? "true" : "false");
  return true;
}

}  // namespace

int main(int argc, char** argv) {
  std::string dir = "/tmp";
  size_t mb = 1024;
  int reps = 3;
  for (int i = 1; i + 1 < argc; i += 2) {
    if (!std::strcmp(argv[i], "--dir")) dir = argv[i + 1];
    if (!std::strcmp(argv[i], "--mb")) mb = std::strtoul(argv[i + 1], nullptr, 10);
    if (!std::strcmp(argv[i], "--reps")) reps = std::atoi(argv[i + 1]);
  }
  const size_t len = mb << 20;
  const std::string path = dir + "/reg_probe." + std::to_string(getpid());
  {
    std::vector<char> buf(8u << 20);
    for (size_t i = 0; i < buf.size(); ++i) buf[i] = static_cast<char>(i * 2654435761u >> 13);
    const int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0600);
    for (size_t o = 0; o < len; o += buf.size())
      if (::pwrite(fd, buf.data(), buf.size(), static_cast<off_t>(o)) != static_cast<ssize_t>(buf.size())) {
        perror("pwrite");
        return 1;
      }
    ::close(fd);
  }
  void* dev = nullptr;
  hipStream_t st;
  if (hipMalloc(&dev, len) != hipSuccess || hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
    std::printf("{\"error\": \"device setup\"}\n");
    ::unlink(path.c_str());
    return 1;
  }
  std::printf("{\"mb\": %zu, \"dir\": \"%s\"}\n", mb, dir.c_str());
  // baseline: the staging ring's hop (pinned -> HBM)
  void* pinned = nullptr;
  if (hipHostMalloc(&pinned, len, hipHostMallocDefault) == hipSuccess) {
    std::memset(pinned, 1, len);
    for (int r = 0; r < reps; ++r) {
      const double t = now_ms();
      (void)hipMemcpyAsync(dev, pinned, len, hipMemcpyHostToDevice, st);
      (void)hipStreamSynchronize(st);
      const double ms = now_ms() - t;
      std::printf("{\"probe\": \"pinned_h2d\", \"ms\": %.3f, \"GBps\": %.1f}\n", ms, len / ms / 1e6);
    }
    (void)hipHostFree(pinned);
  }
  bool ok = true;
  for (int r = 0; r < reps && ok; ++r) {
    ok = run_mapping("file_ro", path, len, hipHostRegisterReadOnly, false, dev, st) &&
         run_mapping("file_ro_populate", path, len, hipHostRegisterReadOnly, true, dev, st) &&
         run_mapping("file_default", path, len, hipHostRegisterDefault, false, dev, st) &&
         run_mapping("file_ro_mapped", path, len, hipHostRegisterReadOnly | hipHostRegisterMapped, true, dev, st);
  }
  (void)hipStreamDestroy(st);
  (void)hipFree(dev);
  ::unlink(path.c_str());
  return ok ? 0 : 1;
}
