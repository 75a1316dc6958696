// ubench_h2d.cpp — host->device copy rate from pinned memory, the ceiling of the host mirror's
// staged batches (rpt_host.cpp): one hipMemcpyAsync of the whole buffer vs the same bytes split over
// 2 / 4 streams, and pieces of 4 / 32 MiB back to back on one stream. Prints one JSON line per case.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      return 1;                                                                \
    }                                                                          \
  } while (0)

int main() {
  const size_t bytes = 256ull << 20;
  void *h = nullptr, *d = nullptr;
  CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
  CK(hipMalloc(&d, bytes));
  std::memset(h, 1, bytes);
  std::vector<hipStream_t> ss(4);
  for (auto& s : ss) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  using clk = std::chrono::steady_clock;
  auto run = [&](const char* name, int streams, size_t piece, bool d2h) -> int {
    for (int rep = 0; rep < 4; rep++) {
      CK(hipDeviceSynchronize());
      auto t0 = clk::now();
      size_t k = 0;
      for (size_t off = 0; off < bytes; off += piece, k++) {
        const size_t n = off + piece <= bytes ? piece : bytes - off;
        hipStream_t s = ss[k % streams];
        if (d2h) CK(hipMemcpyAsync(static_cast<char*>(h) + off, static_cast<char*>(d) + off, n, hipMemcpyDeviceToHost, s));
        else CK(hipMemcpyAsync(static_cast<char*>(d) + off, static_cast<char*>(h) + off, n, hipMemcpyHostToDevice, s));
      }
      CK(hipDeviceSynchronize());
      const double sec = std::chrono::duration<double>(clk::now() - t0).count();
      if (rep == 3)
        printf("{\"case\": \"%s\", \"dir\": \"%s\", \"streams\": %d, \"piece_MiB\": %zu, \"GBps\": %.1f}\n", name,
               d2h ? "d2h" : "h2d", streams, piece >> 20, bytes / sec / 1e9);
    }
    return 0;
  };
  for (int d2h = 0; d2h < 2; d2h++) {
    if (run("whole", 1, bytes, d2h)) return 1;
    if (run("split", 2, bytes / 2, d2h)) return 1;
    if (run("split", 4, bytes / 4, d2h)) return 1;
    if (run("pieces", 1, 32ull << 20, d2h)) return 1;
    if (run("pieces", 1, 4ull << 20, d2h)) return 1;
    if (run("pieces", 2, 4ull << 20, d2h)) return 1;
  }
  return 0;
}
