// What the queued host path's completion step costs on the box's host:
//  1. memcpy bandwidth OUT of pinned memory (hipHostMalloc default / portable)
//     just filled by a D2H, into pageable memory the caller reuses;
//  2. the wake-up latency of hipEventSynchronize for a blocking-sync event vs
//     a spinning one, and of a hipEventQuery poll loop, after a kernel that
//     runs a fixed wall-clock time;
//  3. the whole completion of one 640x480 batch (1.18 MB of masks): D2H into
//     pinned, event, wait, copy to pageable.
// Build: hipcc --offload-arch=gfx950 -O2 -o completion_lat completion_lat.cpp
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

using clk = std::chrono::steady_clock;
static double us_since(clk::time_point t0) { return std::chrono::duration<double, std::micro>(clk::now() - t0).count(); }

// spins for `ticks` of the 100 MHz constant clock, then exits
__global__ void spin(unsigned long long ticks, int* out) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
  if (threadIdx.x == 0 && out) out[0] = 1;
}

int main() {
  const size_t mbytes = 8ull * 144 * 256 * 4;  // one batch of masks
  void* dev = nullptr;
  CK(hipMalloc(&dev, mbytes));
  CK(hipMemset(dev, 1, mbytes));
  void* pin = nullptr;
  CK(hipHostMalloc(&pin, mbytes, hipHostMallocDefault));
  void* pinp = nullptr;
  CK(hipHostMalloc(&pinp, mbytes, hipHostMallocPortable));
  std::vector<char> page(mbytes, 0);
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));

  // 1. copy out of pinned after a D2H
  for (void* src : {pin, pinp}) {
    double tot = 0;
    const int reps = 50;
    for (int r = 0; r < reps; ++r) {
      CK(hipMemcpyAsync(src, dev, mbytes, hipMemcpyDeviceToHost, st));
      CK(hipStreamSynchronize(st));
      auto t0 = clk::now();
      std::memcpy(page.data(), src, mbytes);
      tot += us_since(t0);
    }
    printf("memcpy %zu B pinned(%s) -> pageable: %.1f us (%.1f GB/s)\n", mbytes, src == pin ? "default" : "portable",
           tot / reps, mbytes / (tot / reps * 1e-6) / 1e9);
  }
  {
    double tot = 0;
    std::vector<char> a(mbytes, 1);
    for (int r = 0; r < 50; ++r) {
      auto t0 = clk::now();
      std::memcpy(page.data(), a.data(), mbytes);
      tot += us_since(t0);
    }
    printf("memcpy pageable -> pageable: %.1f us\n", tot / 50);
  }

  // 2. wake-up latency after a 300 us kernel
  const unsigned long long ticks = 30000;  // 300 us at 100 MHz
  hipEvent_t eb, es;
  CK(hipEventCreateWithFlags(&eb, hipEventBlockingSync | hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&es, hipEventDisableTiming));
  spin<<<1, 64, 0, st>>>(ticks, nullptr);
  CK(hipStreamSynchronize(st));
  for (int mode = 0; mode < 4; ++mode) {
    double tot = 0;
    const int reps = 30;
    for (int r = 0; r < reps; ++r) {
      auto t0 = clk::now();
      spin<<<1, 64, 0, st>>>(ticks, nullptr);
      hipEvent_t e = mode == 0 ? eb : es;
      CK(hipEventRecord(e, st));
      if (mode <= 1) {
        CK(hipEventSynchronize(e));
      } else if (mode == 2) {
        while (hipEventQuery(e) == hipErrorNotReady) std::this_thread::yield();
      } else {
        while (hipEventQuery(e) == hipErrorNotReady) std::this_thread::sleep_for(std::chrono::microseconds(20));
      }
      tot += us_since(t0);
    }
    static const char* nm[] = {"blocking-sync event", "spin event", "query+yield", "query+sleep20us"};
    printf("%-20s: kernel 300 us -> host sees it after %.1f us (excess %.1f)\n", nm[mode], tot / reps, tot / reps - 300);
  }

  // 3. whole completion of one batch, blocking vs spin wait
  for (int mode = 0; mode < 2; ++mode) {
    double tot = 0;
    const int reps = 50;
    for (int r = 0; r < reps; ++r) {
      auto t0 = clk::now();
      CK(hipMemcpyAsync(pin, dev, mbytes, hipMemcpyDeviceToHost, st));
      hipEvent_t e = mode == 0 ? eb : es;
      CK(hipEventRecord(e, st));
      CK(hipEventSynchronize(e));
      std::memcpy(page.data(), pin, mbytes);
      tot += us_since(t0);
    }
    printf("D2H 1.18 MB + wait (%s) + copy out: %.1f us\n", mode == 0 ? "blocking" : "spin", tot / reps);
  }
  CK(hipStreamSynchronize(st));
  return 0;
}
