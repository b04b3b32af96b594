// memcpy bandwidth into hipHostMalloc'd (pinned) vs malloc'd memory, 1..16
// threads: what bounds the queued host path's staging copy.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double bench(void* dst, const void* src, size_t bytes, int threads, int reps) {
  auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < reps; ++r) {
    std::vector<std::thread> ts;
    const size_t per = (bytes / threads + 63) & ~size_t(63);
    for (int t = 0; t < threads; ++t)
      ts.emplace_back([=] {
        const size_t off = per * t;
        if (off < bytes) std::memcpy((char*)dst + off, (const char*)src + off, std::min(per, bytes - off));
      });
    for (auto& t : ts) t.join();
  }
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return bytes * (double)reps / s / 1e9;
}

int main() {
  const size_t bytes = 8 * 640 * 480 * 3;
  void* src = aligned_alloc(4096, bytes);
  memset(src, 1, bytes);
  void* plain = aligned_alloc(4096, bytes);
  memset(plain, 0, bytes);
  void *pin = nullptr, *pinc = nullptr, *pinwc = nullptr;
  (void)hipHostMalloc(&pin, bytes, hipHostMallocDefault);
  (void)hipHostMalloc(&pinc, bytes, hipHostMallocNonCoherent);
  (void)hipHostMalloc(&pinwc, bytes, hipHostMallocWriteCombined);
  memset(pin, 0, bytes); memset(pinc, 0, bytes); memset(pinwc, 0, bytes);
  for (int th : {1, 2, 4, 8, 16}) {
    printf("threads %2d  malloc %6.1f  pinned(default) %6.1f  pinned(noncoherent) %6.1f  pinned(wc) %6.1f GB/s\n", th,
           bench(plain, src, bytes, th, 50), bench(pin, src, bytes, th, 50), bench(pinc, src, bytes, th, 50),
           bench(pinwc, src, bytes, th, 50));
  }
  return 0;
}
