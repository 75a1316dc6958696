// ubench_pinned_read.cpp — host CPU read / write rate of host memory by allocation kind (the host-resident
// path's split of a stage's selection vector reads pinned memory the device just wrote): malloc'd pageable
// memory, hipHostMalloc default / coherent / non-coherent / write-combined, and malloc'd memory registered
// with hipHostRegister; each after a device-to-host copy into it. One thread, 64 MiB, median of 5.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main() {
  const size_t bytes = 64 << 20, n = bytes / 4;
  void* dev = nullptr;
  if (hipMalloc(&dev, bytes) != hipSuccess) return 2;
  (void)hipMemset(dev, 1, bytes);
  std::vector<uint32_t> sink(n);
  struct Kind { const char* name; unsigned flags; int mode; };  // mode 0: hipHostMalloc, 1: malloc, 2: malloc + register
  const Kind kinds[] = {{"malloc", 0, 1}, {"hipHostMalloc_default", hipHostMallocDefault, 0},
                        {"hipHostMalloc_coherent", hipHostMallocCoherent, 0},
                        {"hipHostMalloc_noncoherent", hipHostMallocNonCoherent, 0},
                        {"hipHostMalloc_writecombined", hipHostMallocWriteCombined, 0},
                        {"malloc_hipHostRegister", 0, 2}};
  for (const Kind& k : kinds) {
    void* h = nullptr;
    if (k.mode == 0) {
      if (hipHostMalloc(&h, bytes, k.flags) != hipSuccess) { printf("{\"kind\": \"%s\", \"error\": \"alloc\"}\n", k.name); continue; }
    } else {
      h = aligned_alloc(4096, bytes);
      std::memset(h, 0, bytes);
      if (k.mode == 2 && hipHostRegister(h, bytes, hipHostRegisterDefault) != hipSuccess) { printf("{\"kind\": \"%s\", \"error\": \"register\"}\n", k.name); continue; }
    }
    std::vector<double> rd, wr, d2h;
    for (int it = 0; it < 5; it++) {
      double t0 = now();
      (void)hipMemcpy(h, dev, bytes, hipMemcpyDeviceToHost);
      d2h.push_back(bytes / (now() - t0) / 1e9);
      t0 = now();
      const uint32_t* p = static_cast<const uint32_t*>(h);
      uint64_t acc = 0;
      for (size_t i = 0; i < n; i++) { sink[i] = p[i] - 7; acc += sink[i] & 1; }  // the split's read pattern
      rd.push_back(bytes / (now() - t0) / 1e9);
      if (acc == 12345) printf(" ");
      t0 = now();
      std::memcpy(h, sink.data(), bytes);  // the flatten's write pattern
      wr.push_back(bytes / (now() - t0) / 1e9);
    }
    std::sort(rd.begin(), rd.end()); std::sort(wr.begin(), wr.end()); std::sort(d2h.begin(), d2h.end());
    printf("{\"kind\": \"%s\", \"cpu_read_GBps\": %.2f, \"cpu_write_GBps\": %.2f, \"d2h_GBps\": %.2f}\n", k.name, rd[2], wr[2], d2h[2]);
    if (k.mode == 0) (void)hipHostFree(h);
    else { if (k.mode == 2) (void)hipHostUnregister(h); free(h); }
  }
  return 0;
}
