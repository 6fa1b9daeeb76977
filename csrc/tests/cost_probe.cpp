// cost_probe: thread-CPU cost of each primitive of one headline job's data
// path (10 MiB body), measured in isolation, so the worker's per-class CPU in
// a profile (tdl-sha256, tritondl-io) can be split into floor costs:
//
//   sha_hot          SHA-256 of 64 KiB chunks in SHA-NI pairs, cache-warm buffer
//   pwrite_new       the download's writes: 256 KiB pwrites into a new sized file
//   sha_map[_seq]    chunk hashes from a fresh read-only mapping of that file
//                    (what send_chunked_zc does), with / without MADV_SEQUENTIAL
//   sha_map_pop      the same with MAP_POPULATE (page tables set up in one call)
//   sha_pread        pread each pair into an L2-sized scratch, hash there
//   recv_pwrite      loopback TCP receive (4 MiB buffer, fill loop) + pwrite
//   recv_small       the same with a 256 KiB receive buffer
//   sendfile         the sender side: sendfile 64 KiB frames (MSG_MORE heads)
//   unlink           removing the job file
//   pwrite_reuse     the download's writes into a recycled file (the previous
//                    job's, renamed into place and resized): cached pages are
//                    overwritten, none allocated, none freed by an unlink
//
// Build + run: python tools/cost_probe.py [--dir DIR] [--reps N]
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/mman.h>
#include <sys/sendfile.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <thread>
#include <vector>

#include "../hash/hash_core.h"
#include "../relay/relay_core.h"
#include "../hash/sha1_mb.h"
#include "../hash/sha256_mb.h"

namespace {

constexpr size_t kLen = 10u << 20;
constexpr size_t kChunk = 64u << 10;

double thread_ms() {
  timespec t;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &t);
  return t.tv_sec * 1e3 + t.tv_nsec / 1e6;
}
double wall_ms() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e3 + t.tv_nsec / 1e6;
}

struct Stat {
  std::vector<double> cpu, wall;
  void add(double c, double w) {
    cpu.push_back(c);
    wall.push_back(w);
  }
  static double med(std::vector<double> v) {
    if (v.empty()) return 0;
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  }
};

void hash_pairs(const char* p, size_t len) {
  unsigned char d[2][32];
  const size_t n = (len + kChunk - 1) / kChunk;
  for (size_t i = 0; i < n; i += 2) {
    const size_t m0 = std::min(kChunk, len - i * kChunk);
    if (i + 1 < n) {
      const size_t m1 = std::min(kChunk, len - (i + 1) * kChunk);
      tritondl_hash::sha256_pair(p + i * kChunk, m0, p + (i + 1) * kChunk, m1, d[0], d[1]);
    } else {
      tritondl_hash::sha256_raw(p + i * kChunk, m0, d[0]);
    }
  }
}

std::string g_dir = "/tmp";
int g_seq = 0;

std::string fresh_path() { return g_dir + "/cost_probe." + std::to_string(getpid()) + "." + std::to_string(g_seq++); }

// a new file of kLen written the way recv_body writes it
int write_file(const std::string& path, const std::vector<char>& src) {
  const int fd = ::open(path.c_str(), O_RDWR | O_CREAT | O_TRUNC | O_CLOEXEC, 0600);
  if (fd < 0) {
    perror("open");
    std::exit(1);
  }
  if (::ftruncate(fd, kLen) != 0) perror("ftruncate");
  for (size_t o = 0; o < kLen; o += 256u << 10) {
    const size_t m = std::min<size_t>(256u << 10, kLen - o);
    if (::pwrite(fd, src.data() + (o % (1u << 20)), m, static_cast<off_t>(o)) != static_cast<ssize_t>(m))
      perror("pwrite");
  }
  return fd;
}

void report(const char* name, const Stat& s) {
  std::printf("{\"probe\": \"%s\", \"cpu_ms\": %.3f, \"wall_ms\": %.3f, \"reps\": %zu}\n", name, Stat::med(s.cpu),
              Stat::med(s.wall), s.cpu.size());
  std::fflush(stdout);
}

void hash_x16(const char* p, size_t len) {
  unsigned char d[16 * 32];
  const size_t n = len / kChunk;
  size_t i = 0;
  for (; i + 16 <= n; i += 16) {
    const void* m[16];
    for (int j = 0; j < 16; ++j) m[j] = p + (i + j) * kChunk;
    tritondl_hash::sha16::sha256_x16(m, kChunk, d);
  }
  if (i < n) hash_pairs(p + i * kChunk, len - i * kChunk);
}

void probe_sha_hot(int reps) {
  std::vector<char> b(kLen, 'x');
  Stat s, s16;
  hash_pairs(b.data(), kLen);
  for (int r = 0; r < reps; ++r) {
    const double c = thread_ms(), w = wall_ms();
    hash_pairs(b.data(), kLen);
    s.add(thread_ms() - c, wall_ms() - w);
  }
  report("sha_hot", s);
  if (!tritondl_hash::sha16::cpu_has_avx512()) return;
  hash_x16(b.data(), kLen);
  for (int r = 0; r < reps; ++r) {
    const double c = thread_ms(), w = wall_ms();
    hash_x16(b.data(), kLen);
    s16.add(thread_ms() - c, wall_ms() - w);
  }
  report("sha_hot_x16", s16);
  // SHA-1 of 1 MiB pieces (BitTorrent v1), 16 at a time vs SHA-NI pairs
  Stat p2, p16;
  for (int r = 0; r < reps; ++r) {
    const void* m[16];
    size_t l[16];
    for (int j = 0; j < 10; ++j) {
      m[j] = b.data() + (size_t(j) << 20);
      l[j] = 1u << 20;
    }
    unsigned char d[16 * 20];
    double c = thread_ms(), w = wall_ms();
    for (int j = 0; j < 10; j += 2) tritondl_hash::sha2x::sha1_x2(m[j], l[j], m[j + 1], l[j + 1], d, d + 20);
    p2.add(thread_ms() - c, wall_ms() - w);
    const void* m16[16];
    for (int j = 0; j < 16; ++j) m16[j] = b.data() + (size_t(j % 10) << 20);
    c = thread_ms();
    w = wall_ms();
    tritondl_hash::sha16::sha1_x16(m16, 1u << 20, d);
    p16.add((thread_ms() - c) * 10 / 16, (wall_ms() - w) * 10 / 16);  // per 10 MiB
  }
  report("sha1_pieces_pairs", p2);
  report("sha1_pieces_x16", p16);
}

void probe_file(int reps) {
  std::vector<char> src(1u << 20);
  for (size_t i = 0; i < src.size(); ++i) src[i] = static_cast<char>(i * 131u);
  Stat pw, map_seq, map_plain, map_pop, pr, ul;
  for (int r = 0; r < reps; ++r) {
    for (int v = 0; v < 4; ++v) {
      const std::string path = fresh_path();
      double c = thread_ms(), w = wall_ms();
      const int fd = write_file(path, src);
      pw.add(thread_ms() - c, wall_ms() - w);
      c = thread_ms();
      w = wall_ms();
      if (v < 3) {
        const int flags = MAP_SHARED | (v == 2 ? MAP_POPULATE : 0);
        void* m = ::mmap(nullptr, kLen, PROT_READ, flags, fd, 0);
        if (m == MAP_FAILED) {
          perror("mmap");
          std::exit(1);
        }
        if (v == 0) ::madvise(m, kLen, MADV_SEQUENTIAL);
        hash_pairs(static_cast<const char*>(m), kLen);
        ::munmap(m, kLen);
        (v == 0 ? map_seq : v == 1 ? map_plain : map_pop).add(thread_ms() - c, wall_ms() - w);
      } else {
        std::vector<char> scratch(2 * kChunk);
        unsigned char d[2][32];
        for (size_t o = 0; o < kLen; o += 2 * kChunk) {
          tritondl_hash::pread_full(fd, scratch.data(), 2 * kChunk, static_cast<off_t>(o));
          tritondl_hash::sha256_pair(scratch.data(), kChunk, scratch.data() + kChunk, kChunk, d[0], d[1]);
        }
        pr.add(thread_ms() - c, wall_ms() - w);
      }
      ::close(fd);
      c = thread_ms();
      w = wall_ms();
      ::unlink(path.c_str());
      ul.add(thread_ms() - c, wall_ms() - w);
    }
  }
  report("pwrite_new", pw);
  report("sha_map_seq", map_seq);
  report("sha_map", map_plain);
  report("sha_map_pop", map_pop);
  report("sha_pread", pr);
  report("unlink", ul);
}

void sock_pair(int* a, int* b) {
  const int l = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  socklen_t sl = sizeof sa;
  if (::bind(l, reinterpret_cast<sockaddr*>(&sa), sizeof sa) || ::listen(l, 1) ||
      ::getsockname(l, reinterpret_cast<sockaddr*>(&sa), &sl)) {
    perror("listen");
    std::exit(1);
  }
  *a = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (::connect(*a, reinterpret_cast<sockaddr*>(&sa), sizeof sa)) {
    perror("connect");
    std::exit(1);
  }
  *b = ::accept4(l, nullptr, nullptr, SOCK_CLOEXEC);
  ::close(l);
  const int one = 1;
  ::setsockopt(*a, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  ::setsockopt(*b, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
}

// sender: 64 KiB frames, a ~90-byte head with MSG_MORE then sendfile (the
// zero-copy PUT); receiver: recv with a fill loop into buf_size, then pwrite
void probe_sock(int reps, size_t buf_size, const char* rname, bool report_send) {
  std::vector<char> src(1u << 20, 'y');
  const std::string spath = fresh_path();
  const int sfd = write_file(spath, src);
  Stat rs, ss;
  for (int r = 0; r < reps; ++r) {
    int a, b;
    sock_pair(&a, &b);
    const std::string dpath = fresh_path();
    const int dfd = ::open(dpath.c_str(), O_RDWR | O_CREAT | O_TRUNC | O_CLOEXEC, 0600);
    if (::ftruncate(dfd, kLen) != 0) perror("ftruncate");
    double scpu = 0, swall = 0;
    std::thread sender([&] {
      const double c = thread_ms(), w = wall_ms();
      char head[96];
      std::memset(head, 'h', sizeof head);
      for (size_t o = 0; o < kLen; o += kChunk) {
        ::send(a, head, sizeof head, MSG_MORE);
        off_t so = static_cast<off_t>(o);
        size_t left = kChunk;
        while (left) {
          const ssize_t n = ::sendfile(a, sfd, &so, left);
          if (n <= 0) {
            perror("sendfile");
            return;
          }
          left -= static_cast<size_t>(n);
        }
      }
      scpu = thread_ms() - c;
      swall = wall_ms() - w;
    });
    const double c = thread_ms(), w = wall_ms();
    std::vector<char> buf(buf_size);
    const size_t total = kLen + (kLen / kChunk) * 96;
    size_t got = 0, written = 0;
    if (buf_size == 0) {  // splice: socket -> pipe (page refs) -> file (one copy)
      int p[2];
      if (::pipe2(p, O_CLOEXEC) != 0) perror("pipe2");
      ::fcntl(p[1], F_SETPIPE_SZ, 1 << 20);
      while (got < total) {
        const ssize_t n = ::splice(b, nullptr, p[1], nullptr, std::min<size_t>(1u << 20, total - got), SPLICE_F_MOVE);
        if (n <= 0) {
          perror("splice in");
          break;
        }
        size_t left = static_cast<size_t>(n);
        while (left) {
          loff_t o = static_cast<loff_t>(got);
          const ssize_t m = ::splice(p[0], nullptr, dfd, &o, left, SPLICE_F_MOVE);
          if (m <= 0) {
            perror("splice out");
            break;
          }
          left -= static_cast<size_t>(m);
          got += static_cast<size_t>(m);
        }
      }
      ::close(p[0]);
      ::close(p[1]);
    }
    while (got < total) {
      const ssize_t n = ::recv(b, buf.data(), std::min(buf.size(), total - got), 0);
      if (n <= 0) {
        perror("recv");
        break;
      }
      size_t have = static_cast<size_t>(n);
      while (have < buf.size() && have < (256u << 10) && got + have < total) {
        const ssize_t m = ::recv(b, buf.data() + have, std::min(buf.size() - have, total - got - have), MSG_DONTWAIT);
        if (m <= 0) break;
        have += static_cast<size_t>(m);
      }
      const size_t wn = std::min(have, kLen - std::min(kLen, written));
      if (wn && ::pwrite(dfd, buf.data(), wn, static_cast<off_t>(written)) != static_cast<ssize_t>(wn))
        perror("pwrite");
      written += wn;
      got += have;
    }
    rs.add(thread_ms() - c, wall_ms() - w);
    sender.join();
    ss.add(scpu, swall);
    ::close(a);
    ::close(b);
    ::close(dfd);
    ::unlink(dpath.c_str());
  }
  ::close(sfd);
  ::unlink(spath.c_str());
  report(rname, rs);
  if (report_send) report("sendfile", ss);
}

// TLS 1.3 over loopback TCP (AES-128-GCM, the worker's default): thread CPU
// of the receiving pump (recv_body: SSL_read + pwrite) and of the sending
// pump (send_body unsigned: pread + SSL_write) for 10 MiB, next to the AES
// floor (openssl speed on the box: ~6.9 GB/s per core)
void probe_tls(int reps) {
  using namespace tritondl_relay;
  std::vector<char> src(1u << 20, 'z');
  const std::string spath = fresh_path();
  const int sfd = write_file(spath, src);
  TestPki pki = make_test_pki({"127.0.0.1"}, 1);
  auto sctx = TlsContext::server(pki.cert_pem, pki.key_pem);
  auto cctx = TlsContext::client(pki.ca_pem, "", true);
  Stat rs, ss;
  for (int r = 0; r < reps; ++r) {
    int a, b;
    sock_pair(&a, &b);
    ::fcntl(a, F_SETFL, O_NONBLOCK);
    ::fcntl(b, F_SETFL, O_NONBLOCK);
    TlsStream srv(sctx, a, "", ""), cli(cctx, b, "127.0.0.1", "probe");
    std::string serr;
    std::thread hs([&] { serr = srv.handshake(10.0); });
    const std::string cerr = cli.handshake(10.0);
    hs.join();
    if (!cerr.empty() || !serr.empty()) {
      std::fprintf(stderr, "tls handshake: %s %s\n", cerr.c_str(), serr.c_str());
      std::exit(1);
    }
    const std::string dpath = fresh_path();
    const int dfd = ::open(dpath.c_str(), O_RDWR | O_CREAT | O_TRUNC | O_CLOEXEC, 0600);
    if (::ftruncate(dfd, kLen) != 0) perror("ftruncate");
    double scpu = 0, swall = 0;
    std::thread sender([&] {
      const double c = thread_ms(), w = wall_ms();
      SendResult sr = send_body(srv, "", sfd, 0, kLen, nullptr, 0, "", "", "", "", 65536, 1, 10.0);
      if (!sr.err.empty()) std::fprintf(stderr, "tls send: %s\n", sr.err.c_str());
      scpu = thread_ms() - c;
      swall = wall_ms() - w;
    });
    const double c = thread_ms(), w = wall_ms();
    RecvResult rr = recv_body(cli, dfd, 0, static_cast<int64_t>(kLen), "", 0, nullptr, 0, 0, 10.0);
    rs.add(thread_ms() - c, wall_ms() - w);
    sender.join();
    ss.add(scpu, swall);
    if (!rr.err.empty() || rr.received != kLen) std::fprintf(stderr, "tls recv: %s\n", rr.err.c_str());
    ::close(dfd);
    ::unlink(dpath.c_str());
    ::close(a);
    ::close(b);
  }
  ::close(sfd);
  ::unlink(spath.c_str());
  report("tls_recv_pwrite", rs);
  report("tls_pread_send", ss);
}

}  // namespace

// what the service's spare-file recycling does per job: rename the finished
// file into the next job's place, size it, overwrite it
void probe_reuse(int reps) {
  std::vector<char> src(1u << 20);
  for (size_t i = 0; i < src.size(); ++i) src[i] = static_cast<char>(i * 7u);
  Stat pw;
  std::string cur = fresh_path();
  ::close(write_file(cur, src));
  for (int r = 0; r < 4 * reps; ++r) {
    const std::string next = fresh_path();
    const double c = thread_ms(), w = wall_ms();
    if (::rename(cur.c_str(), next.c_str()) != 0) perror("rename");
    const int fd = ::open(next.c_str(), O_WRONLY | O_CLOEXEC);
    if (fd < 0 || ::ftruncate(fd, kLen) != 0) perror("reuse open");
    for (size_t o = 0; o < kLen; o += 256u << 10) {
      const size_t m = std::min<size_t>(256u << 10, kLen - o);
      if (::pwrite(fd, src.data() + (o % (1u << 20)), m, static_cast<off_t>(o)) != static_cast<ssize_t>(m))
        perror("pwrite");
    }
    pw.add(thread_ms() - c, wall_ms() - w);
    ::close(fd);
    cur = next;
  }
  ::unlink(cur.c_str());
  report("pwrite_reuse", pw);
}

int main(int argc, char** argv) {
  int reps = 30;
  for (int i = 1; i + 1 < argc; i += 2) {
    if (!std::strcmp(argv[i], "--dir")) g_dir = argv[i + 1];
    if (!std::strcmp(argv[i], "--reps")) reps = std::atoi(argv[i + 1]);
  }
  std::printf("{\"sha_ni\": %s, \"dir\": \"%s\", \"len\": %zu}\n", tritondl_hash::sha2x::cpu_has_sha_ni() ? "true" : "false",
              g_dir.c_str(), kLen);
  probe_sha_hot(reps);
  probe_file(reps);
  probe_reuse(reps);
  probe_sock(reps, 4u << 20, "recv_pwrite", true);
  probe_sock(reps, 256u << 10, "recv_small", false);
  probe_sock(reps, 0, "splice_file", false);
  probe_tls(reps);
  return 0;
}
