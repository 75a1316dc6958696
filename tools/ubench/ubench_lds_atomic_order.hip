// Does a wave's LDS atomicAdd with return hand out ranks in lane order when several lanes hit the
// same counter? (Deterministic ranks would let a kernel re-derive a scatter order instead of storing it.)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void ranks(const unsigned* ids, unsigned* out, int per_thread) {
  __shared__ unsigned cnt[16][128];
  const unsigned wave = threadIdx.x >> 6;
  for (unsigned i = threadIdx.x; i < 16 * 128; i += blockDim.x) (&cnt[0][0])[i] = 0;
  __syncthreads();
  const size_t base = (size_t)blockIdx.x * blockDim.x * per_thread;
  for (int j = 0; j < per_thread; j++) {
    const size_t i = base + (size_t)j * blockDim.x + threadIdx.x;
    out[i] = atomicAdd(&cnt[wave][ids[i] & 127], 1u);
  }
}

int main() {
  const int blocks = 4096, threads = 1024, per = 16;
  const size_t n = (size_t)blocks * threads * per;
  std::vector<unsigned> h(n), a(n), b(n);
  srand(1);
  for (auto& x : h) x = rand() & 127;
  unsigned *d_ids, *d_out;
  hipMalloc(&d_ids, n * 4);
  hipMalloc(&d_out, n * 4);
  hipMemcpy(d_ids, h.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(ranks, dim3(blocks), dim3(threads), 0, 0, d_ids, d_out, per);
  hipMemcpy(a.data(), d_out, n * 4, hipMemcpyDeviceToHost);
  hipLaunchKernelGGL(ranks, dim3(blocks), dim3(threads), 0, 0, d_ids, d_out, per);
  hipMemcpy(b.data(), d_out, n * 4, hipMemcpyDeviceToHost);
  size_t diff = 0, not_lane_order = 0;
  // expected if lane order within each wave instruction: rank = (count in earlier instructions of the
  // wave) + (number of lower lanes in this instruction with the same id)
  for (int blk = 0; blk < blocks; blk++) {
    for (int w = 0; w < threads / 64; w++) {
      unsigned c[128] = {0};
      for (int j = 0; j < per; j++) {
        const size_t i0 = (size_t)blk * threads * per + (size_t)j * threads + w * 64;
        for (int l = 0; l < 64; l++) {
          const unsigned id = h[i0 + l];
          if (a[i0 + l] != c[id]) not_lane_order++;
          c[id]++;
        }
      }
    }
  }
  for (size_t i = 0; i < n; i++) diff += a[i] != b[i];
  printf("n=%zu run-to-run differences=%zu not-lane-order=%zu\n", n, diff, not_lane_order);
  return 0;
}
