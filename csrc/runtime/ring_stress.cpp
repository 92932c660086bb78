// Host-only stress test of the batch ring's scheduling core (ring_core.h) for the
// sanitizer builds (tests/test_ring_sanitizers_cpu.py): -fsanitize=thread finds data races
// on the slot states / payloads, -fsanitize=address,undefined finds lifetime and UB bugs.
// Payloads are plain heap buffers (the real ring uses pinned hipHostMalloc memory).
//
//   phase 1: native producer threads (run_producers, bounded source) + one consumer that
//            must see batches 0, 1, 2, ... in order with the payload its producer wrote;
//   phase 2: external producers (acquire_empty / commit from their own threads, batch
//            indices claimed from a shared counter, out of order) + the same consumer check;
//   phase 3: stop() while producers and a consumer are blocked.
#include "ring_core.h"

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>

using mpa_runtime::RingCore;

static int fail(const char* what, long a, long b) {
  std::fprintf(stderr, "ring_stress: %s (%ld vs %ld)\n", what, a, b);
  return 1;
}

int main(int argc, char** argv) {
  const int depth = 6, threads = 4, payload = 4096;
  const long nbatch = argc > 1 ? std::atol(argv[1]) : 2000;
  std::vector<std::unique_ptr<long[]>> buf(depth);
  for (auto& b : buf) b.reset(new long[payload]);

  {  // phase 1: native producers
    RingCore ring(depth, 0, 1);
    ring.run_producers(threads, [&](int id, int64_t bidx) {
      for (int i = 0; i < payload; ++i) buf[id][i] = bidx * 31 + i;
      return (int)(bidx % 7) + 1;
    }, nbatch);
    for (long k = 0; k < nbatch; ++k) {
      const int id = ring.acquire();
      if (id < 0) return fail("phase1 stopped early", k, -1);
      if (ring.batch_index(id) != k) return fail("phase1 order", ring.batch_index(id), k);
      if (ring.count(id) != (int)(k % 7) + 1) return fail("phase1 count", ring.count(id), k);
      for (int i = 0; i < payload; i += 97)
        if (buf[id][i] != k * 31 + i) return fail("phase1 payload", buf[id][i], k * 31 + i);
      ring.release(id);
    }
    int64_t st[3];
    ring.stats(st, true);  // every acquire counted; waits / blocked time consistent
    if (st[0] != nbatch || st[1] < 0 || st[1] > nbatch || (st[1] == 0) != (st[2] == 0))
      return fail("phase1 stats", st[0], st[1]);
    ring.stats(st, false);
    if (st[0] != 0) return fail("phase1 stats reset", st[0], 0);
    ring.stop();
  }
  {  // phase 2: external producers claiming indices out of order
    RingCore ring(depth, 0, 1);
    std::atomic<long> next{0};
    std::vector<std::thread> ext;
    for (int t = 0; t < threads; ++t)
      ext.emplace_back([&] {
        while (true) {
          const int id = ring.acquire_empty();
          if (id < 0) return;
          const long b = next.fetch_add(1);
          if (b >= nbatch) {  // nothing left: give the slot back to the free list
            ring.commit(id, -2, 0);
            return;
          }
          for (int i = 0; i < payload; ++i) buf[id][i] = b * 17 - i;
          ring.commit(id, b, 1);
        }
      });
    for (long k = 0; k < nbatch; ++k) {
      const int id = ring.acquire();
      if (id < 0) return fail("phase2 stopped early", k, -1);
      if (ring.batch_index(id) != k) return fail("phase2 order", ring.batch_index(id), k);
      for (int i = 0; i < payload; i += 89)
        if (buf[id][i] != k * 17 - i) return fail("phase2 payload", buf[id][i], k * 17 - i);
      ring.release(id);
    }
    ring.stop();
    for (auto& t : ext) t.join();
  }
  {  // phase 3: stop() wakes blocked producers and consumers
    RingCore ring(2, 0, 1);
    std::atomic<int> woke{0};
    std::thread consumer([&] { if (ring.acquire() < 0) ++woke; });
    const int a = ring.acquire_empty(), b = ring.acquire_empty();
    std::thread producer([&] { if (ring.acquire_empty() < 0) ++woke; });
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    ring.stop();
    consumer.join();
    producer.join();
    if (woke.load() != 2 || a < 0 || b < 0) return fail("phase3 wake", woke.load(), 2);
  }
  std::printf("ring_stress ok: %ld batches x 2 phases, stop wakes waiters\n", nbatch);
  return 0;
}
