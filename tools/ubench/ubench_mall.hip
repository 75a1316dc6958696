// Infinity-Cache (MALL, 256 MiB L3) micro-benchmark for the partitioned probe's intermediates.
//
// Question: can the probe's per-key intermediates (4-B records + 2-B row map,
// written by the partition and re-read by the slice probe / unpermute) live in the Infinity Cache
// instead of HBM, if the probe runs over row chunks that reuse one workspace small enough to stay
// resident?
//
// Three measurements, GB/s of bytes moved (device time, hipEvents, median of reps):
//   read   S      : a buffer of S bytes re-read in full, 16 B per lane (L3-resident below ~256 MiB?)
//   wr+rd  S      : the same buffer rewritten then re-read (the intermediate's life cycle)
//   pipe   R      : the probe's traffic shape over N = 2^30 keys in chunks of R rows:
//                   kernel A reads R keys (8 B, streamed once from a 8 GiB column) and writes 6 B per
//                   row into the workspace (4-B "record" + 2-B "row map"); kernel B reads the 6 B and
//                   writes 1 bit per row. Workspace = one chunk (reused) or two (ping-pong).
//                   R = N is the unchunked design (intermediates through HBM).
// Key loads: plain or non-temporal; workspace stores: plain or non-temporal.
//   ./ubench_mall
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

using u4 = __attribute__((ext_vector_type(4))) unsigned;
using u2 = __attribute__((ext_vector_type(2))) unsigned;

__global__ __launch_bounds__(256) void k_read(const u4* __restrict__ p, uint64_t n, unsigned* sink) {
  unsigned acc = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride * 4) {
    u4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) v[u] = (i + u * stride < n) ? p[i + u * stride] : u4{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < 4; u++) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_write(u4* __restrict__ p, uint64_t n, unsigned salt) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    p[i] = u4{(unsigned)i ^ salt, salt, (unsigned)(i >> 32), salt + 1};
}

// kernel A: 4 keys per lane (32 B: two 16-B loads), 16 B of records + 8 B of row map per lane.
template <bool NT_LOAD, bool NT_STORE>
__global__ __launch_bounds__(256) void k_part(const u4* __restrict__ keys, u4* __restrict__ rec,
                                              u2* __restrict__ rmap, uint64_t lanes) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < lanes; i += stride) {
    u4 a, b;
    if (NT_LOAD) {
      a = __builtin_nontemporal_load(&keys[2 * i]);
      b = __builtin_nontemporal_load(&keys[2 * i + 1]);
    } else {
      a = keys[2 * i];
      b = keys[2 * i + 1];
    }
    const u4 r = {a.x ^ a.y, a.z ^ a.w, b.x ^ b.y, b.z ^ b.w};
    const u2 m = {a.x * 3u, b.y * 5u};
    if (NT_STORE) {
      __builtin_nontemporal_store(r, &rec[i]);
      __builtin_nontemporal_store(m, &rmap[i]);
    } else {
      rec[i] = r;
      rmap[i] = m;
    }
  }
}

// kernel B: reads the lane's 24 B, writes 4 bits per lane (one byte per 2 lanes, via a wave ballot).
__global__ __launch_bounds__(256) void k_probe(const u4* __restrict__ rec, const u2* __restrict__ rmap,
                                               uint64_t* __restrict__ bits, uint64_t lanes) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x; i0 < lanes; i0 += stride) {
    const uint64_t i = i0 + threadIdx.x;
    bool pass = false;
    if (i < lanes) {
      const u4 r = rec[i];
      const u2 m = rmap[i];
      pass = ((r.x ^ r.y ^ r.z ^ r.w ^ m.x ^ m.y) & 7u) == 0;
    }
    const uint64_t bal = __ballot(pass);
    if ((threadIdx.x & 63) == 0 && i < lanes) bits[i / 64] = bal;
  }
}

static float median(std::vector<float> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int grid = cus * 8;  // 8 x 256-thread workgroups per CU (32 waves)
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  unsigned* sink;
  CK(hipMalloc(&sink, 64));

  // ---- read / write+read of a buffer of S bytes -------------------------------------------------
  const uint64_t big = 4ull << 30;
  u4* buf;
  CK(hipMalloc(&buf, big));
  CK(hipMemset(buf, 1, big));
  u4* flush;
  const uint64_t flush_bytes = 1ull << 30;
  CK(hipMalloc(&flush, flush_bytes));
  printf("# %s, %d CUs\n", prop.name, cus);
  for (uint64_t mib : {16, 32, 64, 96, 128, 160, 192, 224, 256, 320, 512, 1024, 4096}) {
    const uint64_t S = mib << 20, n = S / 16;
    std::vector<float> tr, twr;
    for (int rep = 0; rep < 12; rep++) {
      k_read<<<grid, 256>>>(buf, n, sink);  // warm
      CK(hipEventRecord(e0));
      k_read<<<grid, 256>>>(buf, n, sink);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      tr.push_back(ms);
      CK(hipEventRecord(e0));
      k_write<<<grid, 256>>>(buf, n, rep);
      k_read<<<grid, 256>>>(buf, n, sink);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      twr.push_back(ms);
    }
    printf("buffer %5llu MiB  read %7.0f GB/s   write+read %7.0f GB/s\n", (unsigned long long)mib,
           S / (median(tr) * 1e-3) / 1e9, 2.0 * S / (median(twr) * 1e-3) / 1e9);
  }
  CK(hipFree(flush));
  CK(hipFree(buf));

  // ---- chunked pipeline over 2^30 keys -----------------------------------------------------------
  const uint64_t N = 1ull << 30;  // keys
  u4* keys;
  CK(hipMalloc(&keys, N * 8));
  CK(hipMemset(keys, 3, N * 8));
  const uint64_t max_ws_rows = N;
  u4* rec;
  u2* rmap;
  uint64_t* bits;
  CK(hipMalloc(&rec, max_ws_rows * 4));
  CK(hipMalloc(&rmap, max_ws_rows * 2));
  CK(hipMalloc(&bits, N / 8));
  printf("# pipeline: 2^30 keys, A = read 8 B/key + write 6 B/key, B = read 6 B/key + write 1 bit/key\n");
  for (int mode = 0; mode < 4; mode++) {
    const bool ntl = mode & 1, nts = mode & 2;
    for (int lg : {20, 21, 22, 23, 24, 25, 26, 30}) {
      for (int bufs : {1, 2}) {
        if (lg == 30 && bufs == 2) continue;
        const uint64_t R = 1ull << lg, chunks = N / R, lanes = R / 4;
        std::vector<float> t;
        for (int rep = 0; rep < 5; rep++) {
          CK(hipEventRecord(e0));
          for (uint64_t c = 0; c < chunks; c++) {
            const uint64_t w = (bufs == 2 ? (c & 1) : 0) * lanes;
            const u4* kc = keys + c * R / 2;
            auto launch_a = [&](auto kern) { kern<<<std::min<uint64_t>(grid, (lanes + 255) / 256), 256>>>(kc, rec + w, rmap + w, lanes); };
            if (ntl && nts) launch_a(k_part<true, true>);
            else if (ntl) launch_a(k_part<true, false>);
            else if (nts) launch_a(k_part<false, true>);
            else launch_a(k_part<false, false>);
            k_probe<<<std::min<uint64_t>(grid, (lanes + 255) / 256), 256>>>(rec + w, rmap + w, bits + c * R / 64, lanes);
          }
          CK(hipEventRecord(e1));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          if (rep) t.push_back(ms);
        }
        const float ms = median(t);
        printf("pipe keys %s ws-stores %s  chunk 2^%d rows x %d buf (%6.1f MiB ws)  %7.3f ms per 2^30 keys  "
               "%6.0f GB/s of 20.1 B/key\n",
               ntl ? "nt   " : "plain", nts ? "nt   " : "plain", lg, bufs, bufs * R * 6.0 / (1 << 20), ms,
               N * 20.125 / (ms * 1e-3) / 1e9);
        fflush(stdout);
      }
    }
  }
  CK(hipFree(keys));
  CK(hipFree(rec));
  CK(hipFree(rmap));
  CK(hipFree(bits));
  return 0;
}
