// Native self-test for the host C++ cores, built by tools/native_selftest.py
// with -fsanitize=address,undefined (and a -fsanitize=thread variant for the
// threaded piece verifier).  Host code only: the GPU kernels are verified by
// the gpu-marked pytest suite against hashlib.
#include <cassert>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include <fcntl.h>
#include <sys/socket.h>
#include <unistd.h>

#include <thread>

#include "../hash/hash_core.h"
#include "../relay/h2.h"
#include "../relay/relay_core.h"
#include "../utp/utp_engine.h"
#include "../btwire/btwire_core.h"

using namespace tritondl_hash;

static int failures = 0;
#define CHECK(cond)                                                        \
  do {                                                                     \
    if (!(cond)) {                                                         \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                          \
    }                                                                      \
  } while (0)

static void test_vectors() {
  CHECK(hex(one_shot(EVP_sha1(), "abc", 3)) == "a9993e364706816aba3e25717850c26c9cd0d89d");
  CHECK(hex(one_shot(EVP_sha256(), "abc", 3)) ==
        "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad");
  CHECK(hex(one_shot(EVP_md5(), "abc", 3)) == "900150983cd24fb0d6963f7d28e17f72");
}

static std::string signing_key(const std::string& secret, const std::string& date) {
  std::string k = hmac256("AWS4" + secret, date);
  k = hmac256(k, "us-east-1");
  k = hmac256(k, "s3");
  return hmac256(k, "aws4_request");
}

// Two-stream SHA-NI SHA-256 and SHA-1 (sha_ni.h) against OpenSSL: random lengths
// around the block and padding boundaries, equal and unequal pairs.
static void test_sha256_pair() {
  std::mt19937 rng(11);
  std::string a(200000, '\0'), b(200000, '\0');
  for (auto& c : a) c = char(rng());
  for (auto& c : b) c = char(rng());
  for (int it = 0; it < 400; ++it) {
    const size_t na = it < 200 ? size_t(it) : rng() % a.size();
    const size_t nb = rng() % 3 ? na : rng() % b.size();
    unsigned char oa[32], ob[32], r1[32];
    sha256_pair(a.data(), na, b.data(), nb, oa, ob);
    sha256_raw(a.data(), na, r1);
    CHECK(std::string(reinterpret_cast<char*>(oa), 32) == one_shot(sha256_md(), a.data(), na));
    CHECK(std::string(reinterpret_cast<char*>(ob), 32) == one_shot(sha256_md(), b.data(), nb));
    CHECK(std::memcmp(oa, r1, 32) == 0);
    unsigned char s1a[20], s1b[20], s1[20];
    md_pair(sha1_md(), a.data(), na, b.data(), nb, s1a, s1b);
    md_raw(sha1_md(), a.data(), na, s1);
    CHECK(std::string(reinterpret_cast<char*>(s1a), 20) == one_shot(sha1_md(), a.data(), na));
    CHECK(std::string(reinterpret_cast<char*>(s1b), 20) == one_shot(sha1_md(), b.data(), nb));
    CHECK(std::memcmp(s1a, s1, 20) == 0);
  }
}

// 16-lane AVX-512 SHA-256 / SHA-1 (sha256_mb.h, sha1_mb.h) and the batch dispatchers against
// OpenSSL: every length class of the padding (0, < 56, 56..63, whole
// blocks, 64 KiB chunks), equal-length runs of 16 and mixed batches that
// fall back to pairs part-way.
static void test_sha256_batch() {
  std::mt19937 rng(29);
  std::string buf(40 * 70000, '\0');
  for (auto& c : buf) c = char(rng());
  for (int it = 0; it < 60; ++it) {
    const size_t n = it < 20 ? 16 : 1 + rng() % 40;
    const size_t base = it < 12 ? size_t(it * 7) : it < 20 ? size_t(65536) : 1 + rng() % 70000;
    std::vector<const void*> p(n);
    std::vector<size_t> len(n);
    for (size_t i = 0; i < n; ++i) {
      p[i] = buf.data() + (rng() % 64) + i * 70000;
      len[i] = (it % 3 == 2 && i == n / 2) ? base / 2 : base;  // one odd length breaks a run
    }
    std::vector<unsigned char> out(32 * n), out1(20 * n);
    sha256_batch(p.data(), len.data(), n, out.data());
    md_batch(sha1_md(), p.data(), len.data(), n, out1.data());  // 16-lane SHA-1 (sha1_mb.h)
    for (size_t i = 0; i < n; ++i) {
      CHECK(std::string(reinterpret_cast<char*>(&out[32 * i]), 32) == one_shot(sha256_md(), p[i], len[i]));
      CHECK(std::string(reinterpret_cast<char*>(&out1[20 * i]), 20) == one_shot(sha1_md(), p[i], len[i]));
    }
  }
}

static void test_aws_chunked() {
  // AWS S3 SigV4 streaming example: 66560 bytes of 'a', 64 KiB chunks
  const std::string key = signing_key("wJalrXUtnFEMI/K7MDENG/bPxRfiCYEXAMPLEKEY", "20130524");
  const std::string data(66560, 'a');
  const std::string scope = "20130524/us-east-1/s3/aws4_request";
  const std::string seed = "4f232c4386841ef735655705268965c44a0e4690baa4adea153f7db9fa80a0a9";
  auto sigs = chunk_signatures(key, "20130524T000000Z", scope, seed, data.data(), data.size(), 65536, true);
  CHECK(sigs.size() == 3);
  CHECK(sigs[0] == "ad80c730a21e5b8d04586a2213dd63b9a0e99e0e2307b0ade35a65485a288648");
  CHECK(sigs[2] == "b6c6ea8a5354eaf15b3cb7646744f4275b71ea724fed81ceb9323e279d449df9");
  std::string out(aws_chunk_encoded_size(data.size(), 65536, true), '\0');
  std::string last = aws_chunk_encode(key, "20130524T000000Z", scope, seed, data.data(), data.size(), 65536, true,
                                      &out[0]);
  CHECK(out.size() == 66824);
  CHECK(last == sigs[2]);
  CHECK(out.compare(out.size() - 4, 4, "\r\n\r\n") == 0);
}

static void test_pieces_and_verify() {
  std::mt19937 rng(7);
  std::string blob(4 << 20, '\0');
  for (auto& ch : blob) ch = static_cast<char>(rng());
  const size_t pl = 32768;
  std::string ph = piece_hashes(EVP_sha1(), blob.data(), blob.size(), pl, 4);
  CHECK(ph.size() == (blob.size() / pl) * 20);
  for (size_t i = 0; i < blob.size() / pl; ++i)
    CHECK(ph.compare(i * 20, 20, one_shot(EVP_sha1(), blob.data() + i * pl, pl)) == 0);
  // two files forming the torrent stream
  char tmpl[] = "/tmp/tdl_selftestXXXXXX";
  const char* dir = mkdtemp(tmpl);
  CHECK(dir != nullptr);
  if (!dir) return;
  std::string a = std::string(dir) + "/a", b = std::string(dir) + "/b";
  const size_t cut = 300001;
  FILE* fa = std::fopen(a.c_str(), "wb");
  std::fwrite(blob.data(), 1, cut, fa);
  std::fclose(fa);
  FILE* fb = std::fopen(b.c_str(), "wb");
  std::fwrite(blob.data() + cut, 1, blob.size() - cut, fb);
  std::fclose(fb);
  std::vector<std::pair<std::string, long long>> files = {{a, (long long)cut}, {b, (long long)(blob.size() - cut)}};
  std::string ok = verify_pieces(files, pl, ph, 8, EVP_sha1());
  CHECK(ok == std::string(ok.size(), '\1'));
  // sha1_md(): 16-piece groups streamed through the AVX-512 kernel (pieces of
  // 32 KiB, so one stage per piece; and 128 KiB pieces, two stages each)
  CHECK(verify_pieces(files, pl, ph, 8, sha1_md()) == std::string(ok.size(), '\1'));
  const std::string ph128 = piece_hashes(sha1_md(), blob.data(), blob.size(), 131072, 4);
  CHECK(ph128.size() == 32 * 20);
  {
    std::vector<std::pair<std::string, long long>> one = {{a, (long long)cut}, {b, (long long)(blob.size() - cut)}};
    CHECK(verify_pieces(one, 131072, ph128, 4, sha1_md()) == std::string(32, '\1'));
  }
  // corrupt one byte inside piece 20
  FILE* fc = std::fopen(b.c_str(), "r+b");
  std::fseek(fc, 20 * pl - cut + 5, SEEK_SET);
  std::fputc('X', fc);
  std::fclose(fc);
  ok = verify_pieces(files, pl, ph, 8, EVP_sha1());
  int bad = 0;
  for (char ch : ok) bad += ch == 0;
  CHECK(bad == 1 && ok[20] == 0);
  const std::string ok16 = verify_pieces(files, pl, ph, 8, sha1_md());
  CHECK(ok16 == ok);
  std::remove(a.c_str());
  ok = verify_pieces(files, pl, ph, 8, EVP_sha1());  // missing file -> its pieces fail, no crash
  CHECK(ok[0] == 0);
  CHECK(verify_pieces(files, pl, ph, 8, sha1_md()) == ok);
  std::remove(b.c_str());
  rmdir(dir);
}

static void test_utp(double loss, size_t n, unsigned seed) {
  using tritondl_utp::Engine;
  std::mt19937_64 rng(seed);
  std::uniform_real_distribution<double> u(0, 1);
  Engine A(seed), B(seed + 1);
  int64_t now = 0;
  int ca = A.connect("B", now);
  std::string data(n, '\0');
  for (auto& ch : data) ch = static_cast<char>(rng());
  size_t sent = 0;
  bool closed = false;
  std::string got;
  int cb = -1;
  struct Pkt { int64_t at; std::string dst, src, bytes; };
  std::vector<Pkt> wire;
  int64_t last_a = 0, last_b = 0;
  for (int step = 0; step < 300000; ++step) {
    now += 1000;
    if (sent < n) sent += A.write(ca, data.substr(sent, 65536));
    else if (!closed) { A.close(ca, now); closed = true; }
    for (Engine* e : {&A, &B}) {
      const std::string src = e == &A ? "A" : "B";
      for (auto& o : e->outgoing()) {
        if (u(rng) < loss) continue;
        int64_t& last = e == &A ? last_a : last_b;
        int64_t at = std::max<int64_t>(now + 5000 + static_cast<int64_t>(u(rng) * 500), last);
        last = at;
        wire.push_back({at, o.first, src, o.second});
      }
    }
    std::stable_sort(wire.begin(), wire.end(), [](const Pkt& x, const Pkt& y) { return x.at < y.at; });
    size_t k = 0;
    for (; k < wire.size() && wire[k].at <= now; ++k) (wire[k].dst == "B" ? B : A).incoming(wire[k].bytes, wire[k].src, now);
    wire.erase(wire.begin(), wire.begin() + static_cast<long>(k));
    for (int c : B.accepted()) cb = c;
    if (cb >= 0) {
      got += B.read(cb);
      if (B.eof(cb)) break;
    }
    A.tick(now);
    B.tick(now);
  }
  CHECK(got == data);
  CHECK(cb >= 0 && B.eof(cb));
}

// Datagrams from a hostile peer into an engine with one live inbound
// connection: random types, connection ids around the live one, sequence and
// ack numbers near and far from the window, well-formed and truncated
// extension chains, SACK bitmasks, payloads.  Under ASan/UBSan this is the
// memory-safety check of the header parser and the ack / SACK / reorder paths
// (tests/test_utp.py drives the same through the Python binding).
static void test_utp_fuzz(unsigned seed, int rounds) {
  using tritondl_utp::Engine;
  std::mt19937_64 rng(seed);
  auto put16 = [](std::string& s, size_t at, uint32_t v) {
    s[at] = static_cast<char>(v >> 8);
    s[at + 1] = static_cast<char>(v);
  };
  auto put32 = [](std::string& s, size_t at, uint32_t v) {
    for (int k = 0; k < 4; ++k) s[at + k] = static_cast<char>(v >> (24 - 8 * k));
  };
  for (int r = 0; r < rounds; ++r) {
    Engine e(seed + static_cast<unsigned>(r));
    int64_t now = 1000000;
    auto pkt = [&](unsigned type, uint16_t cid, uint16_t seq, uint16_t ack, uint8_t ext) {
      std::string s(20, '\0');
      s[0] = static_cast<char>((type << 4) | 1);
      s[1] = static_cast<char>(ext);
      put16(s, 2, cid);
      put32(s, 4, static_cast<uint32_t>(rng()));
      put32(s, 8, rng() % 2 ? 0u : static_cast<uint32_t>(rng()));
      put32(s, 12, static_cast<uint32_t>(rng()));
      put16(s, 16, seq);
      put16(s, 18, ack);
      return s;
    };
    e.incoming(pkt(4, 0x0fff, 100, 0, 0), "P:1", now);  // inbound SYN: connection 0x1000 is live
    CHECK(!e.accepted().empty());
    static const uint16_t ids[] = {0x1000, 0x1001, 0x0fff, 7};
    for (int i = 0; i < 80; ++i) {
      now += 997;
      const unsigned type = static_cast<unsigned>(rng() % 7);
      const uint16_t cid = ids[rng() % 4];
      const uint16_t seq = static_cast<uint16_t>(rng() % 2 ? 100 + rng() % 40 : rng());
      const uint16_t ack = static_cast<uint16_t>(rng());
      std::string ext_chain;
      uint8_t first = 0;
      switch (rng() % 4) {
        case 0: break;
        case 1: {  // one SACK extension, bitmask of 4..12 bytes
          first = 1;
          const size_t len = 4 + (rng() % 3) * 4;
          ext_chain = std::string{static_cast<char>(0), static_cast<char>(len)};
          for (size_t k = 0; k < len; ++k) ext_chain += static_cast<char>(rng());
          break;
        }
        case 2: {  // truncated / self-describing garbage chain
          first = static_cast<uint8_t>(rng() % 4);
          ext_chain.resize(rng() % 12);
          for (auto& ch : ext_chain) ch = static_cast<char>(rng());
          break;
        }
        default:  // unknown extension with a length past the end
          first = 2;
          ext_chain = std::string{static_cast<char>(0), static_cast<char>(200)} + "xy";
      }
      std::string payload(rng() % 1400, '\0');
      for (auto& ch : payload) ch = static_cast<char>(rng());
      e.incoming(pkt(type, cid, seq, ack, first) + ext_chain + payload, "P:1", now);
      e.tick(now);
      e.outgoing();
    }
    for (int c : e.accepted()) {
      e.read(c);
      e.state(c);
    }
    e.read(1);
    e.state(1);
    e.tick(now + 10000000);
    e.outgoing();
  }
}

static void test_merkle() {
  // one file of 3 leaves + 100 bytes in a 64 KiB piece: root over 4 leaves, 4th = zero hash
  std::mt19937 rng(11);
  std::string data(3 * kMerkleLeaf + 100, '\0');
  for (auto& ch : data) ch = static_cast<char>(rng());
  auto H = [](const std::string& x) { return one_shot(EVP_sha256(), x.data(), x.size()); };
  std::string l0 = H(data.substr(0, kMerkleLeaf)), l1 = H(data.substr(kMerkleLeaf, kMerkleLeaf)),
              l2 = H(data.substr(2 * kMerkleLeaf, kMerkleLeaf)), l3 = H(data.substr(3 * kMerkleLeaf));
  std::string root = H(H(l0 + l1) + H(l2 + l3));  // 4 real leaves
  std::string leaves = l0 + l1 + l2 + l3;
  std::string ok = merkle_check(leaves, std::string(4, '\1'), 65536, root, {4}, {(long long)data.size()},
                                std::string(1, '\1'), 2);
  CHECK(ok == std::string(1, '\1'));
  // width 8 pads with four zero leaves
  std::string z(32, '\0');
  std::string root8 = H(root + H(H(z + z) + H(z + z)));
  ok = merkle_check(leaves, std::string(4, '\1'), 131072, root8, {8}, {(long long)data.size()}, std::string(1, '\1'), 1);
  CHECK(ok == std::string(1, '\1'));
  // from a file, and an unreadable leaf fails
  char tmpl[] = "/tmp/tdl_merkleXXXXXX";
  const char* dir = mkdtemp(tmpl);
  CHECK(dir != nullptr);
  if (!dir) return;
  std::string f = std::string(dir) + "/f";
  FILE* fp = std::fopen(f.c_str(), "wb");
  std::fwrite(data.data(), 1, data.size(), fp);
  std::fclose(fp);
  ok = merkle_verify({{f, (long long)data.size()}}, 65536, root, {4}, {(long long)data.size()}, std::string(1, '\1'), 2);
  CHECK(ok == std::string(1, '\1'));
  ok = merkle_check(leaves, std::string("\1\0\1\1", 4), 65536, root, {4}, {(long long)data.size()},
                    std::string(1, '\1'), 1);
  CHECK(ok == std::string(1, '\0'));
  std::remove(f.c_str());
  rmdir(dir);
}

// Relay pumps over a socketpair: the chunked sender follows a Flow advanced by
// a writer thread while the streamed verifier checks every signature — the
// three-party hand-off (writer / hasher pool / sender, receiver / hasher
// pool / checker) is what TSan is here for.
static void test_relay(size_t size) {
  using namespace tritondl_relay;
  std::mt19937 rng(11);
  std::string data(size, '\0');
  for (auto& c : data) c = static_cast<char>(rng());
  char path[] = "/tmp/tdl_relayXXXXXX";
  const int wfd = ::mkstemp(path);
  CHECK(wfd >= 0);
  CHECK(::ftruncate(wfd, static_cast<off_t>(size)) == 0);
  const int rfd = ::open(path, O_RDONLY);
  int sv[2];
  CHECK(::socketpair(AF_UNIX, SOCK_STREAM, 0, sv) == 0);
  ::fcntl(sv[0], F_SETFL, O_NONBLOCK);
  ::fcntl(sv[1], F_SETFL, O_NONBLOCK);
  const std::string key(32, 'k'), amz = "20260101T000000Z", scope = "20260101/us-east-1/s3/aws4_request",
                    seed(64, '0');
  Flow flow({{0, static_cast<int64_t>(size), 0}});
  std::thread writer([&] {
    for (size_t off = 0; off < size; off += 100000) {
      const size_t n = std::min<size_t>(100000, size - off);
      std::string e;
      CHECK(pwrite_full(wfd, data.data() + off, n, off, &e));
      flow.advance(0, off + n);
    }
    flow.finish(size);
  });
  VerifyResult vr;
  const uint64_t raw_len = chunked_length(size, 65536);
  PlainStream s0(sv[0]), s1(sv[1]);
  std::thread receiver([&] { vr = recv_verify_chunked(s1, raw_len, "", 0, key, amz, scope, seed, true, 3, 10.0); });
  SendResult sr = send_body(s0, "", rfd, 0, size, &flow, 1, key, amz, scope, seed, 65536, 3, 10.0);
  writer.join();
  receiver.join();
  CHECK(sr.err.empty());
  CHECK(vr.err.empty());
  CHECK(vr.data == data);
  // receive pump into a file, plain sender with sendfile
  char opath[] = "/tmp/tdl_relayoutXXXXXX";
  const int ofd = ::mkstemp(opath);
  Flow f2({{0, static_cast<int64_t>(size), 0}});
  RecvResult rr;
  std::thread rcv([&] { rr = recv_body(s1, ofd, 0, static_cast<int64_t>(size), "", 0, &f2, 0, 0, 10.0); });
  SendResult ps = send_body(s0, "", rfd, 0, size, nullptr, 0, "", "", "", "", 65536, 1, 10.0);
  rcv.join();
  CHECK(ps.err.empty() && rr.err.empty() && rr.received == size && f2.watermark() == size);
  std::string back(size, '\0');
  CHECK(pread_full(ofd, &back[0], size, 0) == size && back == data);
  // the same without splice: recv + pwrite
  if (size >= 2) {
    CHECK(::ftruncate(ofd, 0) == 0);
    Flow f3({{0, static_cast<int64_t>(size), 0}});
    std::thread rcv2([&] { rr = recv_body(s1, ofd, 0, static_cast<int64_t>(size), "xy", 2, &f3, 0, 0, 10.0,
                                          4u << 20, false); });
    ps = send_body(s0, "", rfd, 2, size - 2, nullptr, 0, "", "", "", "", 65536, 1, 10.0);
    rcv2.join();
    CHECK(ps.err.empty() && rr.err.empty() && rr.received == size && f3.watermark() == size);
    back.assign(size, '\0');
    CHECK(pread_full(ofd, &back[0], size, 0) == size && back.substr(2) == data.substr(2) && back.substr(0, 2) == "xy");
  }
  ::close(sv[0]);
  ::close(sv[1]);
  ::close(wfd);
  ::close(rfd);
  ::close(ofd);
  ::unlink(path);
  ::unlink(opath);
}

// The streamed S3 verifier with its whole body already in hand (the prefix):
// every frame is published at once, so the hashers start far behind and
// claim 16 frames at a time (the AVX-512 path); a flipped payload byte in
// one frame must still fail the signature chain.
// HTTP/2 session pump (relay/h2.h) over a socket pair: a server thread sends
// two streams' DATA (padded and not, frames split anywhere), stream 3 with a
// sink limit below its body; the sinks must hold exactly the bodies, the
// credit frames must never grant stream 3 past its limit, and drop/close race
// cleanly with the pump (TSan build).
static std::string h2_frame(uint8_t type, uint8_t flags, uint32_t sid, const std::string& p) {
  std::string f;
  const uint32_t n = static_cast<uint32_t>(p.size());
  const char h[9] = {char(n >> 16), char(n >> 8), char(n), char(type), char(flags),
                     char((sid >> 24) & 0x7f), char(sid >> 16), char(sid >> 8), char(sid)};
  f.append(h, 9);
  f += p;
  return f;
}

static void test_h2(unsigned seed) {
  using namespace tritondl_relay;
  std::mt19937 rng(seed);
  int sv[2];
  CHECK(::socketpair(AF_UNIX, SOCK_STREAM, 0, sv) == 0);
  ::fcntl(sv[0], F_SETFL, O_NONBLOCK);
  const size_t n1 = (3u << 20) + 123, n3 = (2u << 20) + 45, limit3 = (1u << 20) + 7;
  std::string b1(n1, '\0'), b3(n3, '\0');
  for (auto& c : b1) c = static_cast<char>(rng());
  for (auto& c : b3) c = static_cast<char>(rng());
  std::string wire;
  wire += h2_frame(1, 0x4, 1, "h1");  // HEADERS: forwarded to the caller as an event
  wire += h2_frame(1, 0x4, 3, "h3");
  size_t o1 = 0, o3 = 0, pad3 = 0;
  while (o1 < n1 || o3 < n3) {
    const bool one = o3 >= n3 || (o1 < n1 && (rng() & 1));
    std::string& b = one ? b1 : b3;
    size_t& o = one ? o1 : o3;
    const size_t take = std::min<size_t>(b.size() - o, 1 + rng() % 60000);
    const bool last = o + take == b.size();
    if (rng() % 3 == 0) {
      const uint8_t pad = static_cast<uint8_t>(rng() % 40);
      if (!one) pad3 += 1 + pad;
      wire += h2_frame(0, 0x8 | (last ? 1 : 0), one ? 1 : 3, std::string(1, char(pad)) + b.substr(o, take) +
                                                          std::string(pad, '\0'));
    } else {
      wire += h2_frame(0, last ? 1 : 0, one ? 1 : 3, b.substr(o, take));
    }
    o += take;
  }
  char path[] = "/tmp/tdl_h2XXXXXX";
  const int fd = ::mkstemp(path);
  CHECK(fd >= 0);
  auto flow = std::make_shared<Flow>(std::vector<Flow::Seg>{{0, int64_t(n1), 0}, {uint64_t(n1), int64_t(n1 + limit3), 0}});
  auto sess = std::make_shared<H2Session>(std::make_shared<PlainStream>(sv[0]), 1u << 20, 64u << 20, 1u << 20);
  sess->open_stream(1);
  sess->open_stream(3);
  sess->open_stream(5);  // never answered: dropped while the pump runs
  sess->start();
  sess->sink_file(1, fd, 0, -1, flow, 0, 0);
  std::atomic<uint64_t> granted3{0};
  std::thread server([&, sseed = rng()] {
    std::mt19937 srng(sseed);
    size_t off = 0;
    std::string back;
    while (off < wire.size()) {
      const size_t m = std::min<size_t>(wire.size() - off, 1 + srng() % 200000);
      CHECK(::send(sv[1], wire.data() + off, m, MSG_NOSIGNAL) == ssize_t(m));
      off += m;
      char buf[4096];
      for (ssize_t r; (r = ::recv(sv[1], buf, sizeof buf, MSG_DONTWAIT)) > 0;) back.append(buf, size_t(r));
    }
    ::usleep(200000);
    char buf[4096];
    for (ssize_t r; (r = ::recv(sv[1], buf, sizeof buf, MSG_DONTWAIT)) > 0;) back.append(buf, size_t(r));
    for (size_t p = 0; p + 9 <= back.size();) {  // the credit the client returned
      const unsigned char* h = reinterpret_cast<const unsigned char*>(back.data() + p);
      const uint32_t len = (uint32_t(h[0]) << 16) | (uint32_t(h[1]) << 8) | h[2];
      const uint32_t sid = ((uint32_t(h[5]) << 24) | (uint32_t(h[6]) << 16) | (uint32_t(h[7]) << 8) | h[8]) & 0x7fffffffu;
      if (h[3] == 8 && sid == 3 && len == 4)
        granted3 += (uint32_t(h[9]) << 24 | uint32_t(h[10]) << 16 | uint32_t(h[11]) << 8 | h[12]) & 0x7fffffffu;
      p += 9 + len;
    }
  });
  ::usleep(1000 * (rng() % 20));
  sess->sink_file(3, fd, n1, int64_t(limit3), flow, 1, 0);
  sess->drop(5);
  int done = 0, headers = 0;
  uint64_t w1 = 0, w3 = 0;
  for (int spin = 0; done < 2 && spin < 20000; ++spin) {
    for (H2Event& e : sess->take_events()) {
      if (e.type == 1) ++headers;
      if (e.type == H2Session::kSinkDone) {
        ++done;
        (e.sid == 1 ? w1 : w3) = e.n;
        CHECK(e.sid == 1 ? e.flags == 1 : true);
      }
      CHECK(e.type != H2Session::kSinkError && e.type != H2Session::kConnError);
    }
    ::usleep(500);
  }
  server.join();
  CHECK(done == 2 && headers == 2 && w1 == n1 && w3 == limit3);
  // stream 3 was granted credit only up to its limit (initial window 1 MiB; padding costs window too)
  CHECK(granted3.load() + (1u << 20) <= limit3 + pad3);
  std::string back(n1 + limit3, '\0');
  CHECK(pread_full(fd, &back[0], back.size(), 0) == back.size());
  CHECK(back.substr(0, n1) == b1 && back.substr(n1) == b3.substr(0, limit3));
  CHECK(flow->done(0) == n1 && flow->done(1) == limit3);
  sess->close();
  bool conn_end = false;
  for (H2Event& e : sess->take_events()) conn_end = conn_end || e.type == H2Session::kConnError;
  CHECK(conn_end);
  ::close(sv[0]);
  ::close(sv[1]);
  ::close(fd);
  ::unlink(path);
}

static void test_verify_backlog() {
  using namespace tritondl_relay;
  const size_t size = (3u << 20) + 77;
  std::mt19937 rng(31);
  std::string data(size, '\0');
  for (auto& c : data) c = static_cast<char>(rng());
  const std::string key(32, 'k'), amz = "20260101T000000Z", scope = "20260101/us-east-1/s3/aws4_request",
                    seed(64, '0');
  std::string raw(tritondl_hash::aws_chunk_encoded_size(size, 65536, true), '\0');
  tritondl_hash::aws_chunk_encode(key, amz, scope, seed, data.data(), size, 65536, true, &raw[0], 2);
  int sv[2];
  CHECK(::socketpair(AF_UNIX, SOCK_STREAM, 0, sv) == 0);
  ::fcntl(sv[1], F_SETFL, O_NONBLOCK);
  PlainStream s1(sv[1]);
  VerifyResult vr = recv_verify_chunked(s1, raw.size(), raw.data(), raw.size(), key, amz, scope, seed, true, 2, 10.0);
  CHECK(vr.err.empty() && vr.data == data);
  std::string bad = raw;
  bad[20 * (65536 + 87) + 1000] ^= 1;  // inside frame 20's payload
  vr = recv_verify_chunked(s1, bad.size(), bad.data(), bad.size(), key, amz, scope, seed, false, 2, 10.0);
  CHECK(vr.err == "chunk signature mismatch");
  ::close(sv[0]);
  ::close(sv[1]);
}

// Pumps started on the task pool and reaped from a CompletionPort (the
// worker's path): a receive pump and an aws-chunked send following a Flow
// that a writer thread advances, with the verifier on a plain thread.
static void test_port(size_t size) {
  using namespace tritondl_relay;
  std::mt19937 rng(23);
  std::string data(size, '\0');
  for (auto& c : data) c = static_cast<char>(rng());
  char path[] = "/tmp/tdl_portXXXXXX";
  const int wfd = ::mkstemp(path);
  CHECK(wfd >= 0);
  CHECK(::ftruncate(wfd, static_cast<off_t>(size)) == 0);
  int a[2], b[2];
  CHECK(::socketpair(AF_UNIX, SOCK_STREAM, 0, a) == 0 && ::socketpair(AF_UNIX, SOCK_STREAM, 0, b) == 0);
  for (int fd : {a[0], a[1], b[0], b[1]}) ::fcntl(fd, F_SETFL, O_NONBLOCK);
  auto port = std::make_shared<CompletionPort>();
  auto flow = std::make_shared<Flow>(std::vector<Flow::Seg>{{0, static_cast<int64_t>(size), 0}});
  auto in = std::make_shared<PlainStream>(a[1]);
  auto out = std::make_shared<PlainStream>(b[0]);
  const std::string key(32, 'k'), amz = "20260101T000000Z", scope = "20260101/us-east-1/s3/aws4_request",
                    seed(64, '0');
  // origin -> a[0]; the receive pump lands a[1] in the file and advances the flow
  start_pump(port, 1, 1, false, [=](CompletionPort::Done& d) {
    d.rr = recv_body(*in, wfd, 0, static_cast<int64_t>(size), "", 0, flow.get(), 0, 0, 10.0, 1u << 20, false);
  }, "tdl-recv");
  start_pump(port, 2, 2, false, [=](CompletionPort::Done& d) {
    d.sr = send_body(*out, "", wfd, 0, size, flow.get(), 1, key, amz, scope, seed, 65536, 3, 10.0);
  }, "tdl-send");
  VerifyResult vr;
  PlainStream sink(b[1]);
  std::thread verifier([&] {
    vr = recv_verify_chunked(sink, chunked_length(size, 65536), "", 0, key, amz, scope, seed, true, 2, 10.0);
  });
  std::string e;
  PlainStream src(a[0]);
  CHECK(send_all(src, data.data(), data.size(), 10.0, nullptr, &e));
  std::vector<CompletionPort::Done> done;
  while (done.size() < 2) {
    CHECK(port->wait(10000));
    for (auto& d : port->reap()) done.push_back(std::move(d));
  }
  verifier.join();
  CHECK(port->inflight() == 0);
  for (const auto& d : done) {
    if (d.id == 1) CHECK(d.kind == 1 && d.rr.err.empty() && d.rr.received == size);
    if (d.id == 2) CHECK(d.kind == 2 && d.sr.err.empty() && d.sr.sent == size);
  }
  CHECK(vr.err.empty() && vr.data == data);
  for (int fd : {a[0], a[1], b[0], b[1], wfd}) ::close(fd);
  ::unlink(path);
}

// The same pumps over TLS (OpenSSL streams, batched ciphertext flushes): a
// handshake on two threads, then aws-chunked send/verify and plain
// send/receive following a Flow, plus an abort of a pump waiting for bytes.
static void test_tls_relay(size_t size) {
  using namespace tritondl_relay;
  std::mt19937 rng(5);
  std::string data(size, '\0');
  for (auto& c : data) c = static_cast<char>(rng());
  char path[] = "/tmp/tdl_tlsXXXXXX";
  const int wfd = ::mkstemp(path);
  CHECK(wfd >= 0);
  std::string e;
  CHECK(pwrite_full(wfd, data.data(), size, 0, &e));
  const int rfd = ::open(path, O_RDONLY);
  int sv[2];
  CHECK(::socketpair(AF_UNIX, SOCK_STREAM, 0, sv) == 0);
  ::fcntl(sv[0], F_SETFL, O_NONBLOCK);
  ::fcntl(sv[1], F_SETFL, O_NONBLOCK);
  TestPki pki = make_test_pki({"127.0.0.1", "localhost"}, 1);
  auto sctx = TlsContext::server(pki.cert_pem, pki.key_pem);
  auto cctx = TlsContext::client(pki.ca_pem, "", true);
  TlsStream cli(cctx, sv[0], "127.0.0.1", "selftest"), srv(sctx, sv[1], "", "");
  std::string serr;
  std::thread hs([&] { serr = srv.handshake(10.0); });
  const std::string cerr = cli.handshake(10.0);
  hs.join();
  CHECK(cerr.empty() && serr.empty());
  const std::string key(32, 'k'), amz = "20260101T000000Z", scope = "20260101/us-east-1/s3/aws4_request",
                    seed(64, '0');
  Flow flow({{0, static_cast<int64_t>(size), 0}});
  std::thread adv([&] {
    for (size_t off = 0; off < size; off += 300000) flow.advance(0, std::min(size, off + 300000));
    flow.finish(size);
  });
  VerifyResult vr;
  std::thread rcv([&] { vr = recv_verify_chunked(srv, chunked_length(size, 65536), "", 0, key, amz, scope, seed,
                                                 true, 2, 10.0); });
  SendResult sr = send_body(cli, "", rfd, 0, size, &flow, 1, key, amz, scope, seed, 65536, 2, 10.0);
  adv.join();
  rcv.join();
  CHECK(sr.err.empty() && vr.err.empty() && vr.data == data);
  char opath[] = "/tmp/tdl_tlsoutXXXXXX";
  const int ofd = ::mkstemp(opath);
  RecvResult rr;
  std::thread r2([&] { rr = recv_body(srv, ofd, 0, static_cast<int64_t>(size), "", 0, nullptr, 0, 0, 10.0); });
  SendResult ps = send_body(cli, "", rfd, 0, size, nullptr, 0, "", "", "", "", 65536, 1, 10.0);
  r2.join();
  CHECK(ps.err.empty() && rr.err.empty() && rr.received == size);
  std::string back(size, '\0');
  CHECK(pread_full(ofd, &back[0], size, 0) == size && back == data);
  // abort: a receive waiting for bytes that never come
  RecvResult ra;
  std::thread r3([&] { ra = recv_body(srv, -1, 0, 1 << 20, "", 0, nullptr, 0, 0, 10.0); });
  std::this_thread::sleep_for(std::chrono::milliseconds(30));
  srv.abort();
  r3.join();
  CHECK(ra.err == "cancelled");
  ::close(sv[0]);
  ::close(sv[1]);
  ::close(wfd);
  ::close(rfd);
  ::close(ofd);
  ::unlink(path);
  ::unlink(opath);
}

// BitTorrent peer wire (csrc/btwire): a seeded swarm stream cut at random
// points must assemble byte-exact pieces; mutated and random streams (it
// parses untrusted peer input) must end in a kBad event or be absorbed,
// never touch memory outside the buffers.
static std::string bt_msg(uint8_t id, const std::string& payload) {
  std::string m;
  const uint32_t n = uint32_t(payload.size() + 1);
  m.push_back(char(n >> 24));
  m.push_back(char(n >> 16));
  m.push_back(char(n >> 8));
  m.push_back(char(n));
  m.push_back(char(id));
  return m + payload;
}
static std::string be32s(uint32_t v) {
  return std::string{char(v >> 24), char(v >> 16), char(v >> 8), char(v)};
}

// chunked transfer decoding: random chunk sizes / extensions / trailers, fed
// in random cuts (the decoder works in place, so this is where a bounds slip
// would show under ASan)
static void test_chunked(unsigned seed, int rounds) {
  using tritondl_relay::ChunkedDecoder;
  std::mt19937 rng(seed);
  for (int round = 0; round < rounds; ++round) {
    std::string data(rng() % 200000, '\0');
    for (auto& c : data) c = char(rng());
    std::string enc;
    char hx[32];
    for (size_t pos = 0; pos < data.size();) {
      const size_t n = std::min<size_t>(data.size() - pos, 1 + rng() % 70000);
      snprintf(hx, sizeof hx, rng() % 2 ? "%zx" : "%zX", n);
      enc += hx;
      if (rng() % 4 == 0) enc += ";ext=\"v\"";
      enc += "\r\n" + data.substr(pos, n) + "\r\n";
      pos += n;
    }
    enc += "0\r\n";
    if (rng() % 2) enc += "X-T: 1\r\nY: 2\r\n";
    enc += "\r\n";
    const size_t extra = rng() % 3 == 0 ? 5 : 0;
    enc += std::string(extra, 'z');
    ChunkedDecoder dec;
    std::string out, err;
    size_t pos = 0;
    while (pos < enc.size() && !dec.done()) {
      const size_t cut = std::min<size_t>(enc.size() - pos, 1 + rng() % 9000);
      std::vector<char> buf(enc.begin() + long(pos), enc.begin() + long(pos + cut));
      size_t data_n = 0;
      const size_t used = dec.decode(buf.data(), cut, &data_n, &err);
      CHECK(err.empty());
      out.append(buf.data(), data_n);
      pos += used;
      if (!dec.done()) CHECK(used == cut);
    }
    CHECK(dec.done() && out == data && enc.size() - pos == extra);
  }
  ChunkedDecoder bad;
  std::string err;
  size_t dn = 0;
  char junk[] = "12\r\nabc";
  bad.decode(junk, 2, &dn, &err);
  CHECK(err.empty());
  char junk2[] = "g";
  ChunkedDecoder bad2;
  bad2.decode(junk2, 1, &dn, &err);
  CHECK(!err.empty());
}

static void test_btwire(unsigned seed, int rounds) {
  using namespace tritondl_btwire;
  std::mt19937 rng(seed);
  const uint32_t plen = 3 * kBlock, npieces = 5;
  const uint64_t total = uint64_t(npieces - 1) * plen + kBlock + 100;
  std::string content(total, 0);
  for (auto& c : content) c = char(rng());
  // well-formed stream, random cuts, interleaved control messages
  {
    auto store = std::make_shared<PieceStore>(npieces, plen, total);
    Link link(store, 16, true);
    for (uint32_t i = 0; i < npieces; ++i) link.assign(i);
    // a well-behaved peer: it answers exactly the REQUESTs the link sends
    // (unrequested blocks are dropped by design), with HAVEs and keep-alives
    // mixed in, and the stream arrives in random cuts through both receive paths
    std::string stream = bt_msg(kUnchoke, "");
    std::vector<Event> ev;
    std::string out;
    auto answer = [&](const std::string& o) {
      size_t p = 0;
      while (p + 4 <= o.size()) {
        const uint32_t ml = be32(reinterpret_cast<const uint8_t*>(o.data() + p));
        if (ml == 13 && uint8_t(o[p + 4]) == kRequest) {
          const uint8_t* q = reinterpret_cast<const uint8_t*>(o.data() + p + 5);
          const uint32_t i = be32(q), off = be32(q + 4), n = be32(q + 8);
          stream += bt_msg(kPiece, be32s(i) + be32s(off) + content.substr(i * plen + off, n));
          if (rng() % 3 == 0) stream += bt_msg(4, be32s(i));  // HAVE
          if (rng() % 5 == 0) stream += std::string(4, '\0');  // keep-alive
        }
        p += 4 + ml;
      }
    };
    while (!stream.empty()) {
      const size_t cut = std::min<size_t>(stream.size(), 1 + rng() % 40000);
      if (rng() % 2) {
        auto span = link.recv_buffer(cut);
        CHECK(span.second >= cut);
        std::memcpy(span.first, stream.data(), cut);
        link.feed_n(cut, &ev, &out);
      } else {
        link.feed(reinterpret_cast<const uint8_t*>(stream.data()), cut, &ev, &out);
      }
      stream.erase(0, cut);
      answer(out);
      out.clear();
    }
    uint32_t done = 0;
    for (const Event& e : ev) {
      CHECK(e.kind != Event::kBad);
      if (e.kind == Event::kPieceDone) {
        auto piece = store->take(e.piece);
        CHECK(std::memcmp(piece->data().data(), content.data() + e.piece * plen, piece->data().size()) == 0);
        ++done;
      }
    }
    CHECK(done == npieces && link.buffered() == 0);
  }
  // a source over the same content (serving REQUESTs), file + padding + file
  char path[] = "/tmp/tritondl_btwire_XXXXXX";
  const int sfd = ::mkstemp(path);
  CHECK(sfd >= 0);
  const uint64_t split = total / 2;
  CHECK(::pwrite(sfd, content.data(), split, 0) == ssize_t(split));
  auto src = std::make_shared<Source>(npieces, plen, total);
  src->add_file(sfd, 0, split - 1000);
  src->add_file(-1, split - 1000, 1000);
  src->add_file(sfd, split, 0);
  ::close(sfd);
  ::unlink(path);
  for (uint32_t i = 0; i < npieces; i += 2) src->set_have(i);
  {
    std::string out;
    std::vector<Event> ev;
    Link link(std::make_shared<PieceStore>(npieces, plen, total), 8, true);
    link.set_source(src);
    const std::string req = bt_msg(kRequest, be32s(0) + be32s(kBlock) + be32s(kBlock));
    link.feed(reinterpret_cast<const uint8_t*>(req.data()), req.size(), &ev, &out);
    CHECK(ev.empty() && out.size() == 13 + kBlock && out[4] == char(kPiece));
    CHECK(std::memcmp(out.data() + 13, content.data() + kBlock, kBlock) == 0);
  }
  // mutated / random streams
  for (int r = 0; r < rounds; ++r) {
    auto store = std::make_shared<PieceStore>(npieces, plen, total);
    Link link(store, 1 + int(rng() % 64), rng() % 2);
    if (rng() % 2) link.set_source(src);
    for (uint32_t i = 0; i < npieces; ++i)
      if (rng() % 2) link.assign(i);
    std::string stream;
    for (int k = 0; k < 30; ++k) {
      const uint32_t i = rng() % (npieces + 2), off = (rng() % 5) * kBlock + (rng() % 7 == 0 ? 1 : 0);
      switch (rng() % 6) {
        case 0: stream += bt_msg(kPiece, be32s(i) + be32s(off) + std::string(rng() % 3 ? kBlock : rng() % 20000, 'x')); break;
        case 1: stream += bt_msg(uint8_t(rng()), std::string(rng() % 64, char(rng()))); break;
        case 2: stream += bt_msg(kReject, be32s(i) + be32s(off) + be32s(kBlock)); break;
        case 3:
          if (rng() % 2) {
            stream += bt_msg(uint8_t(rng() % 2), "");  // (un)choke
          } else {
            const uint32_t len = rng() % 3 ? kBlock : uint32_t(rng());
            stream += bt_msg(kRequest, be32s(i) + be32s(uint32_t(rng() % (plen + 10))) + be32s(len));
          }
          break;
        case 4: {
          std::string junk(rng() % 300, 0);
          for (auto& c : junk) c = char(rng());
          stream += junk;
          break;
        }
        default: stream += bt_msg(kPiece, std::string(rng() % 8, 'p')); break;  // short
      }
    }
    for (int f = 0; f < 20 && !stream.empty(); ++f) stream[rng() % stream.size()] = char(rng());  // bit rot
    std::vector<Event> ev;
    std::string out;
    size_t pos = 0;
    bool bad = false;
    while (pos < stream.size() && !bad) {
      const size_t cut = std::min<size_t>(stream.size() - pos, 1 + rng() % 5000);
      link.feed(reinterpret_cast<const uint8_t*>(stream.data() + pos), cut, &ev, &out);
      for (const Event& e : ev) {
        if (e.kind == Event::kBad) bad = true;
        if (e.kind == Event::kPieceDone) store->take(e.piece);
      }
      ev.clear();
      pos += cut;
      if (rng() % 4 == 0) link.piece_done(rng() % npieces);
      if (rng() % 4 == 0) link.lapse_all();
      out = link.pump();
    }
    CHECK(store->partial_bytes() <= total);
  }
}

int main(int argc, char** argv) {
  bool quick = argc > 1 && std::string(argv[1]) == "--quick";
  test_vectors();
  test_sha256_pair();
  test_sha256_batch();
  test_aws_chunked();
  test_pieces_and_verify();
  test_merkle();
  test_relay(quick ? (3u << 20) + 777 : (8u << 20) + 777);
  test_relay(0);
  test_port(quick ? (2u << 20) + 99 : (6u << 20) + 99);
  test_verify_backlog();
  test_tls_relay(quick ? (1u << 20) + 333 : (6u << 20) + 333);
  test_utp(0.0, quick ? 100000 : 400000, 1);
  test_utp(0.03, quick ? 60000 : 200000, 2);
  test_utp_fuzz(5, quick ? 200 : 2000);
  test_btwire(7, quick ? 300 : 3000);
  test_chunked(3, quick ? 40 : 300);
  for (unsigned seed = 1; seed <= (quick ? 3u : 10u); ++seed) test_h2(seed);
  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::puts("native selftest OK");
  return 0;
}
