// Throughput of the sans-IO uTP engine alone (no sockets): engine A streams
// to engine B through an in-memory lossless link, both in this thread.
// Build: g++ -O3 -std=c++17 -I csrc/utp csrc/bench/utp_engine_bench.cpp -o /tmp/utp_bench
#include <chrono>
#include <cstdio>
#include <string>

#include "utp_engine.h"

int main(int argc, char** argv) {
  using tritondl_utp::Engine;
  const size_t total = (argc > 1 ? std::stoul(argv[1]) : 512) << 20;
  Engine A(1), B(2);
  int64_t now = 1;
  int ca = A.connect("B:1", now);
  std::string chunk(1 << 20, 'x');
  size_t sent = 0, got = 0;
  int cb = -1;
  auto t0 = std::chrono::steady_clock::now();
  while (got < total) {
    now += 50;
    while (sent < total) {
      size_t n = A.write(ca, chunk.substr(0, std::min(chunk.size(), total - sent)));
      if (!n) break;
      sent += n;
    }
    A.tick(now);
    B.begin_batch();
    for (auto& d : A.take_datagrams()) B.incoming(d.pkt->data(), d.pkt->size(), "A:1", now);
    B.end_batch(now);
    for (int c : B.accepted()) cb = c;
    if (cb >= 0) got += B.read(cb).size();
    A.begin_batch();
    for (auto& d : B.take_datagrams()) A.incoming(d.pkt->data(), d.pkt->size(), "B:1", now);
    A.end_batch(now);
  }
  double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::printf("{\"bench\": \"utp_engine\", \"MB\": %zu, \"seconds\": %.3f, \"MBps\": %.1f}\n", total >> 20, dt,
              total / dt / 1e6);
  return 0;
}
