// Ring-exchange micro-benchmark: the go/no-go gate for an on-chip C2 probe.
//
// The design under test: half the CUs are "partitioners" (producers), half hold one 128 KiB filter
// slice each in LDS ("slice holders", consumers). A partitioner streams its share of the 8-B keys from
// HBM, hashes them, sorts each 8192-row tile by destination slice in LDS and sends each slice its
// 4-B records through a single-producer / single-consumer ring in global memory (L2 / Infinity-Cache
// resident: 64 MiB); the slice holder probes the records against its LDS slice and returns one pass
// bit per record through a return ring; the partitioner restores row order from the permutation it
// kept in LDS / registers, so no row map ever reaches memory. Per key: 8 B read from HBM, 4 B out and
// 4 B in over the fabric, 2 bits back.
//
// Transport (MI355X_MICROARCH.md, inter-workgroup visibility, hand-off row 1): payload written by one
// wave with 8-B agent-scope (sc1) stores, s_waitcnt vmcnt(0), then one lane stores the slot header
// {seq, count} (sc1); the consumer wave polls the header with sc1 loads and reads the payload with sc1
// loads. Credits: a producer reuses slot k of a ring only after the consumer returned the message that
// last used it. Every wait is bounded and raises a global abort flag that every loop checks, and a
// co-residency barrier at launch aborts if the 2 x 128 workgroups are not all resident.
//
//   ./ubench_ring [log2_keys=30] [reps=3]
// Prints the exchange time per 1e9 keys, the key-read-only time, and checks the survivor count
// against the host's.
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

constexpr int kP = 128, kC = 128;        // partitioners, slice holders
constexpr int kR = 4;                    // slots per ring
constexpr int kS = 256;                  // records per slot
constexpr int kThreads = 512;            // 8 waves per workgroup
constexpr int kWaves = kThreads / 64;
constexpr int kRowsPerThread = 16;
constexpr int kTile = kThreads * kRowsPerThread;  // 8192 rows
constexpr int kDestPerWave = kC / kWaves;        // 16
constexpr int kSrcPerWave = kP / kWaves;         // 16
constexpr uint32_t kFinal = 0xFFFFFFFFu;
constexpr uint32_t kSpinLimit = 1u << 22;
constexpr int kSliceWords = 16384;       // 128 KiB slice

constexpr int kLineWords = 16;           // one 128-B line per slot header / return (no two slots share a line)
struct Shared {
  uint32_t* ring;      // [P][C][R][S] records
  uint64_t* hdr;       // [P][C][R] line: word 0 = seq << 32 | count
  uint64_t* rbits;     // [P][C][R] line: words 0..3 = pass bits
  uint64_t* rhdr;      // [P][C][R] line: word 0 = returned seq
  uint32_t* abort_flag;
  uint32_t* arrived;
  unsigned long long* survivors;
};

__device__ __forceinline__ uint64_t mix64(uint64_t x) {  // splitmix64 finalizer as the key hash
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ULL;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebULL;
  return x ^ (x >> 31);
}
__host__ __device__ __forceinline__ uint64_t slice_pattern(uint32_t i) {
  uint64_t x = 0x9e3779b97f4a7c15ULL * (i + 1);
  x ^= x >> 29;
  x *= 0xbf58476d1ce4e5b9ULL;
  return x ^ (x >> 32);
}
// pass bit of a record against slice word w: ~50 % of (pattern) bits set -> 2 bits tested ~25 % pass
__host__ __device__ __forceinline__ bool probe_bits(uint64_t w, uint32_t rec) {
  const uint32_t a = rec & 63, b = (rec >> 6) & 63;
  return ((w >> a) & 1) && ((w >> b) & 1);
}

__device__ __forceinline__ uint64_t ld_sc1(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool aborted(const Shared& sh) {
  return __hip_atomic_load(sh.abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}
__device__ __forceinline__ void raise_abort(const Shared& sh) {
  __hip_atomic_store(sh.abort_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Poll *p until pred(value) (one lane); bounded; returns false on abort / time-out.
template <typename Pred>
__device__ __forceinline__ bool wait_for(const Shared& sh, const uint64_t* p, Pred pred, uint64_t& v) {
  for (uint32_t i = 0; i < kSpinLimit; i++) {
    v = ld_sc1(p);
    if (pred(v)) return true;
    if ((i & 63) == 63 && aborted(sh)) return false;
    __builtin_amdgcn_s_sleep(1);
  }
  raise_abort(sh);
  return false;
}

// Lanes with `need` poll their own *p until pred(value): one round trip for up to 64 flags; bounded.
// Returns a wave-uniform false on abort / time-out.
template <typename Pred>
__device__ __forceinline__ bool wait_lanes(const Shared& sh, bool need, const uint64_t* p, Pred pred) {
  bool pending = need;
  for (uint32_t i = 0; i < kSpinLimit; i++) {
    if (pending && pred(ld_sc1(p))) pending = false;
    if (__ballot(pending) == 0) return true;
    if ((i & 63) == 63 && aborted(sh)) return false;
    __builtin_amdgcn_s_sleep(1);
  }
  raise_abort(sh);
  return false;
}

__device__ __forceinline__ size_t slot_index(int p, int c, int k) { return (static_cast<size_t>(p) * kC + c) * kR + k; }

// ---- partitioner -------------------------------------------------------------------------------------
// mode 1 (transport only): no key reads, no sort, no reassembly: every tile sends 64 records to each of the
// 128 holders (8192 per tile, as the even split of a real tile) and only waits for slot credits.
__device__ void producer(const Shared& sh, const uint64_t* __restrict__ keys, uint64_t n, int p, uint8_t* lds, int mode) {
  uint32_t* s_rec = reinterpret_cast<uint32_t*>(lds);                     // [2][kTile] sorted records
  uint8_t* s_pass = reinterpret_cast<uint8_t*>(s_rec + 2 * kTile);        // [2][kTile] pass flags (sorted order)
  uint32_t* s_cnt = reinterpret_cast<uint32_t*>(s_pass + 2 * kTile);      // [2][kC]
  uint32_t* s_start = s_cnt + 2 * kC;                                     // [2][kC]
  uint32_t* s_seq0 = s_start + 2 * kC;                                    // [2][kC] first seq of the tile's messages
  uint32_t* s_next = s_seq0 + 2 * kC;                                     // [kC] next seq per destination
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < kC; i += kThreads) s_next[i] = 1;
  const uint64_t per = (n + kP - 1) / kP;
  const uint64_t lo = std::min<uint64_t>(n, per * p), hi = std::min<uint64_t>(n, lo + per);
  const uint64_t ntiles = (hi - lo + kTile - 1) / kTile;
  __shared__ int s_ok;  // workgroup-uniform "no wait failed": every barrier below is reached by all waves
  if (threadIdx.x == 0) s_ok = 1;
  uint32_t rk[kRowsPerThread], rk_prev[kRowsPerThread];  // rank | dest << 16 of this thread's rows (this / previous tile)
  unsigned long long surv = 0;
  bool ok = true;
  for (uint64_t t = 0; t <= ntiles && ok; t++) {
    const int b = static_cast<int>(t & 1), pb = b ^ 1;
#pragma unroll
    for (int j = 0; j < kRowsPerThread; j++) rk_prev[j] = rk[j];
    if (t < ntiles && mode == 1) {
      for (int i = threadIdx.x; i < kC; i += kThreads) {
        s_cnt[b * kC + i] = kTile / kC;
        s_start[b * kC + i] = i * (kTile / kC);
      }
      for (int i = threadIdx.x; i < kTile; i += kThreads) s_rec[b * kTile + i] = static_cast<uint32_t>(i * 2654435761u);
      __syncthreads();
    } else if (t < ntiles) {
      // 1. keys -> records, ranked by destination
      for (int i = threadIdx.x; i < kC; i += kThreads) s_cnt[b * kC + i] = 0;
      __syncthreads();
      const uint64_t base = lo + t * kTile;
      uint32_t rec[kRowsPerThread];
#pragma unroll
      for (int j = 0; j < kRowsPerThread / 2; j++) {
        const uint64_t r = base + (static_cast<uint64_t>(j) * kThreads + threadIdx.x) * 2;
        uint64_t k0 = 0, k1 = 0;
        if (r + 1 < hi) {
          const auto v = *reinterpret_cast<const __attribute__((ext_vector_type(2))) uint64_t*>(keys + r);
          k0 = v.x;
          k1 = v.y;
        } else if (r < hi) {
          k0 = keys[r];
        }
        const uint64_t h0 = mix64(k0), h1 = mix64(k1);
        rec[2 * j] = static_cast<uint32_t>(h0);
        rec[2 * j + 1] = static_cast<uint32_t>(h1);
        rk[2 * j] = r < hi ? ((static_cast<uint32_t>(h0 >> 32) & (kC - 1)) << 16) : 0xFFFFFFFFu;
        rk[2 * j + 1] = r + 1 < hi ? ((static_cast<uint32_t>(h1 >> 32) & (kC - 1)) << 16) : 0xFFFFFFFFu;
      }
#pragma unroll
      for (int j = 0; j < kRowsPerThread; j++)
        if (rk[j] != 0xFFFFFFFFu) rk[j] |= atomicAdd(&s_cnt[b * kC + (rk[j] >> 16)], 1u);
      __syncthreads();
      if (wave == 0) {  // exclusive scan of the 128 counts: 2 per lane
        const uint32_t c0 = s_cnt[b * kC + 2 * lane], c1 = s_cnt[b * kC + 2 * lane + 1];
        uint32_t incl = c0 + c1;
        for (int d = 1; d < 64; d <<= 1) {
          const uint32_t o = __shfl_up(incl, d, 64);
          if (lane >= d) incl += o;
        }
        s_start[b * kC + 2 * lane] = incl - c0 - c1;
        s_start[b * kC + 2 * lane + 1] = incl - c1;
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < kRowsPerThread; j++)
        if (rk[j] != 0xFFFFFFFFu) s_rec[b * kTile + s_start[b * kC + (rk[j] >> 16)] + (rk[j] & 0xFFFF)] = rec[j];
      __syncthreads();
    }
    if (t < ntiles) {
      // 2. send: wave w owns destinations [16w, 16w + 16), lane i < 16 keeps destination 16w + i's
      //    books; the m-th messages of all 16 go out together: one credit round trip, one vmcnt wait
      {
        const int myd = wave * kDestPerWave + (lane & (kDestPerWave - 1));
        const bool own = lane < kDestPerWave;
        const uint32_t cnt = own ? s_cnt[b * kC + myd] : 0, seq0 = own ? s_next[myd] : 0;
        const uint32_t nmsg = own ? (cnt == 0 ? 1 : (cnt + kS - 1) / kS) : 0;
        if (own) s_seq0[b * kC + myd] = seq0;
        uint32_t max_m = nmsg;
        for (int o = 32; o >= 1; o >>= 1) max_m = max(max_m, static_cast<uint32_t>(__shfl_xor(max_m, o, 64)));
        for (uint32_t m = 0; m < max_m; m++) {
          const bool has = m < nmsg;
          const uint32_t seq = seq0 + m;
          const size_t si = slot_index(p, myd, static_cast<int>(seq % kR));
          if (!wait_lanes(sh, has && seq > kR, sh.rhdr + si * kLineWords, [&](uint64_t x) { return x >= seq - kR; })) {
            ok = false;
            if (lane == 0) atomicAnd(&s_ok, 0);
            break;
          }
          for (int dd = 0; dd < kDestPerWave; dd++) {
            if (!__shfl(has ? 1 : 0, dd, 64)) continue;  // uniform
            const uint32_t cd = __shfl(cnt, dd, 64), mc = min(static_cast<uint32_t>(kS), cd - min(cd, m * kS));
            const int d = wave * kDestPerWave + dd;
            const size_t sd = slot_index(p, d, static_cast<int>(__shfl(seq, dd, 64) % kR));
            uint64_t* dst = reinterpret_cast<uint64_t*>(sh.ring + sd * kS);
            const uint32_t* src = s_rec + b * kTile + s_start[b * kC + d] + m * kS;
            for (uint32_t i = 2 * lane; i < mc; i += 128) {
              const uint64_t v = static_cast<uint64_t>(src[i]) | (i + 1 < mc ? static_cast<uint64_t>(src[i + 1]) << 32 : 0);
              st_sc1(dst + i / 2, v);
            }
          }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          if (has) st_sc1(sh.hdr + si * kLineWords, (static_cast<uint64_t>(seq) << 32) | min(static_cast<uint32_t>(kS), cnt - min(cnt, m * kS)));
        }
        if (own) s_next[myd] = seq0 + nmsg;
      }
    }
    __syncthreads();
    if (threadIdx.x == 0 && aborted(sh)) s_ok = 0;
    __syncthreads();
    ok = s_ok != 0;
    if (t == 0 || !ok || mode == 1) continue;
    // 3. returns of the previous tile (again the m-th messages of a wave's 16 destinations together): pass
    //    bits into sorted order, then rows through their ranks
    {
      const int myd = wave * kDestPerWave + (lane & (kDestPerWave - 1));
      const bool own = lane < kDestPerWave;
      const uint32_t cnt = own ? s_cnt[pb * kC + myd] : 0, seq0 = own ? s_seq0[pb * kC + myd] : 0;
      const uint32_t nmsg = own ? (cnt == 0 ? 1 : (cnt + kS - 1) / kS) : 0;
      uint32_t max_m = nmsg;
      for (int o = 32; o >= 1; o >>= 1) max_m = max(max_m, static_cast<uint32_t>(__shfl_xor(max_m, o, 64)));
      for (uint32_t m = 0; m < max_m && ok; m++) {
        const bool has = m < nmsg;
        const uint32_t seq = seq0 + m;
        const size_t si = slot_index(p, myd, static_cast<int>(seq % kR));
        if (!wait_lanes(sh, has, sh.rhdr + si * kLineWords, [&](uint64_t x) { return x >= seq; })) {
          ok = false;
          if (lane == 0) atomicAnd(&s_ok, 0);
          break;
        }
        // lane 4 dd + q loads word q of destination dd's bits: one load for the wave's 16 messages
        const int ld = lane >> 2;
        const bool hl = __shfl(has ? 1 : 0, ld, 64) != 0;
        const size_t sl = static_cast<size_t>(__shfl(static_cast<unsigned long long>(si), ld, 64));
        const uint64_t w = hl ? ld_sc1(sh.rbits + sl * kLineWords + (lane & 3)) : 0;
        for (int dd = 0; dd < kDestPerWave; dd++) {
          if (!__shfl(has ? 1 : 0, dd, 64)) continue;  // uniform
          const uint32_t cd = __shfl(cnt, dd, 64), mc = min(static_cast<uint32_t>(kS), cd - min(cd, m * kS));
          const uint32_t st = s_start[pb * kC + wave * kDestPerWave + dd];
          // word 2q + e holds records q * 128 + 2l + e at bit l (the consumer's ballots, see there)
          // (the shuffle runs with every lane active: ds_bpermute from an inactive lane returns 0)
          for (uint32_t i0 = 0; i0 < mc; i0 += 64) {  // uniform
            const uint32_t i = i0 + lane;
            const uint64_t wi = __shfl(w, dd * 4 + static_cast<int>(2 * ((i & 255) / 128) + (i & 1)), 64);
            if (i < mc) s_pass[pb * kTile + st + m * kS + i] = static_cast<uint8_t>((wi >> ((i & 127) >> 1)) & 1);
          }
        }
      }
    }
    __syncthreads();
    ok = s_ok != 0;
#pragma unroll
    for (int j = 0; j < kRowsPerThread; j++)
      if (rk_prev[j] != 0xFFFFFFFFu) surv += s_pass[pb * kTile + s_start[pb * kC + (rk_prev[j] >> 16)] + (rk_prev[j] & 0xFFFF)];
  }
  // finals: one per destination
  for (int dd = 0; dd < kDestPerWave; dd++) {
    const int d = wave * kDestPerWave + dd;
    const uint32_t seq = s_next[d];
    const size_t si = slot_index(p, d, static_cast<int>(seq % kR));
    if (lane == 0 && ok) {
      uint64_t v = 0;
      if (seq > kR) ok = wait_for(sh, sh.rhdr + si * kLineWords, [&](uint64_t x) { return x >= seq - kR; }, v);
      if (ok) st_sc1(sh.hdr + si * kLineWords, (static_cast<uint64_t>(seq) << 32) | kFinal);
    }
  }
  for (int o = 32; o >= 1; o >>= 1) surv += __shfl_xor(surv, o, 64);
  if (lane == 0) atomicAdd(sh.survivors, surv);
}

// ---- slice holder --------------------------------------------------------------------------------------
__device__ void consumer(const Shared& sh, int c, uint8_t* lds) {
  uint64_t* s_slice = reinterpret_cast<uint64_t*>(lds);
  for (int i = threadIdx.x; i < kSliceWords; i += kThreads) s_slice[i] = slice_pattern(static_cast<uint32_t>(c * kSliceWords + i));
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // lane i < 16 tracks producer p = 16 * wave + i
  const int myp = wave * kSrcPerWave + (lane & (kSrcPerWave - 1));
  uint32_t expect = 1;
  bool fin = lane >= kSrcPerWave;
  uint32_t idle = 0;
  while (true) {
    const bool all_fin = __builtin_amdgcn_readfirstlane(__all(fin) ? 1 : 0) != 0;
    if (all_fin) break;
    uint64_t h = 0;
    const size_t si = slot_index(myp, c, static_cast<int>(expect % kR));
    if (!fin) h = ld_sc1(sh.hdr + si * kLineWords);
    const bool ready = !fin && static_cast<uint32_t>(h >> 32) == expect;
    uint64_t mask = __ballot(ready);
    if (mask == 0) {
      if (++idle > kSpinLimit) {
        raise_abort(sh);
        break;
      }
      if ((idle & 63) == 63 && aborted(sh)) break;
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    idle = 0;
    // every ready message of this wave's 16 producers, then all their returns with one vmcnt wait:
    // lane 4 i + q holds word q of producer slot i's pass bits
    const uint32_t cnt_l = static_cast<uint32_t>(h);
    uint64_t mine = 0;
    for (uint64_t mm = mask; mm; mm &= mm - 1) {
      const int src = __builtin_ctzll(mm);
      const uint32_t cnt = __shfl(cnt_l, src, 64);
      if (cnt == kFinal) continue;  // uniform
      const size_t ss = static_cast<size_t>(__shfl(static_cast<unsigned long long>(si), src, 64));
      const uint64_t* rp = reinterpret_cast<const uint64_t*>(sh.ring + ss * kS);
      uint64_t bits[kS / 64];
#pragma unroll
      for (int q = 0; q < kS / 128; q++) {  // 128 records per 8-B load
        const uint32_t i = q * 128 + 2 * lane;
        const uint64_t v = i < cnt ? ld_sc1(rp + i / 2) : 0;
        const uint32_t r0 = static_cast<uint32_t>(v), r1 = static_cast<uint32_t>(v >> 32);
        const bool p0 = i < cnt && probe_bits(s_slice[(r0 >> 12) & (kSliceWords - 1)], r0);
        const bool p1 = i + 1 < cnt && probe_bits(s_slice[(r1 >> 12) & (kSliceWords - 1)], r1);
        // word 2q: records q * 128 + 2l (bit l), word 2q + 1: records q * 128 + 2l + 1
        bits[2 * q] = __ballot(p0);
        bits[2 * q + 1] = __ballot(p1);
      }
#pragma unroll
      for (int q = 0; q < kS / 64; q++) mine = lane == src * 4 + q ? bits[q] : mine;
    }
    const int lsrc = lane >> 2;
    const uint32_t lcnt = __shfl(cnt_l, lsrc, 64);
    const bool lready = ((mask >> lsrc) & 1) && lcnt != kFinal;
    const size_t lss = static_cast<size_t>(__shfl(static_cast<unsigned long long>(si), lsrc, 64));
    if (lready) st_sc1(sh.rbits + lss * kLineWords + (lane & 3), mine);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (ready) {
      if (cnt_l == kFinal) fin = true;
      else st_sc1(sh.rhdr + si * kLineWords, expect);
      expect++;
    }
  }
}

__global__ __launch_bounds__(kThreads) void ring_kernel(Shared sh, const uint64_t* keys, uint64_t n, int mode) {
  extern __shared__ uint8_t lds[];
  // co-residency: every workgroup must be running before anyone waits on anyone
  if (threadIdx.x == 0) {
    atomicAdd(sh.arrived, 1u);
    uint32_t i = 0;
    while (__hip_atomic_load(sh.arrived, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gridDim.x && i < kSpinLimit) {
      __builtin_amdgcn_s_sleep(4);
      i++;
    }
    if (i >= kSpinLimit) raise_abort(sh);
  }
  __syncthreads();
  if (aborted(sh)) return;
  // blocks b, b + 8, ... share an XCD (round-robin dealing): each XCD gets 16 partitioners and 16 holders
  const int b = blockIdx.x, k = b / 8;
  const int idx = (k >> 1) * 8 + (b % 8);
  if (k & 1) consumer(sh, idx, lds);
  else producer(sh, keys, n, idx, lds, mode);
}

__global__ void key_read_kernel(const uint64_t* __restrict__ keys, uint64_t n, unsigned long long* out) {
  uint64_t acc = 0;
  for (uint64_t i = (static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x) * 2; i + 1 < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x * 2) {
    const auto v = *reinterpret_cast<const __attribute__((ext_vector_type(2))) uint64_t*>(keys + i);
    acc += (mix64(v.x) >> 63) + (mix64(v.y) >> 63);
  }
  if (acc == 0xFFFFFFFF) atomicAdd(out, acc);
}

__global__ void fill_keys(uint64_t* k, uint64_t n, uint64_t seed) {
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    k[i] = mix64(i ^ seed);
}

static uint64_t host_mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ULL;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebULL;
  return x ^ (x >> 31);
}

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 30;
  const int reps = argc > 2 ? atoi(argv[2]) : 3;
  const uint64_t n = 1ULL << lg;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  if (prop.multiProcessorCount < kP + kC) {
    printf("needs %d CUs, device has %d\n", kP + kC, prop.multiProcessorCount);
    return 1;
  }
  uint64_t* keys;
  CK(hipMalloc(&keys, n * 8));
  hipLaunchKernelGGL(fill_keys, dim3(4096), dim3(256), 0, 0, keys, n, 12345ULL);
  Shared sh{};
  const size_t slots = static_cast<size_t>(kP) * kC * kR;
  CK(hipMalloc(&sh.ring, slots * kS * 4));
  CK(hipMalloc(&sh.hdr, slots * kLineWords * 8));
  CK(hipMalloc(&sh.rbits, slots * kLineWords * 8));
  CK(hipMalloc(&sh.rhdr, slots * kLineWords * 8));
  uint32_t* small;
  CK(hipMalloc(&small, 256));
  sh.abort_flag = small;
  sh.arrived = small + 1;
  sh.survivors = reinterpret_cast<unsigned long long*>(small + 2);
  const size_t prod_lds = 2 * kTile * 4 + 2 * kTile + 7 * kC * 4;
  const size_t lds = std::max<size_t>(prod_lds, kSliceWords * 8);
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&ring_kernel), hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
  // host survivors: the same hash, destination and pass rule
  unsigned long long want = 0;
  {
    std::vector<uint64_t> hk(n);
    CK(hipMemcpy(hk.data(), keys, n * 8, hipMemcpyDeviceToHost));
    for (uint64_t i = 0; i < n; i++) {
      const uint64_t h = host_mix64(hk[i]);
      const uint32_t rec = static_cast<uint32_t>(h), c = static_cast<uint32_t>(h >> 32) & (kC - 1);
      want += probe_bits(slice_pattern(c * kSliceWords + ((rec >> 12) & (kSliceWords - 1))), rec);
    }
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  unsigned long long* sink;
  CK(hipMalloc(&sink, 8));
  float best_ring = 1e30f, best_read = 1e30f;
  for (int r = 0; r < reps; r++) {
    CK(hipMemset(sh.hdr, 0, slots * kLineWords * 8));
    CK(hipMemset(sh.rhdr, 0, slots * kLineWords * 8));
    CK(hipMemset(small, 0, 256));
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(ring_kernel, dim3(kP + kC), dim3(kThreads), lds, 0, sh, keys, n, 0);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    CK(hipGetLastError());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    uint32_t hs[4];
    CK(hipMemcpy(hs, small, 16, hipMemcpyDeviceToHost));
    const unsigned long long got = (static_cast<unsigned long long>(hs[3]) << 32) | hs[2];
    printf("ring rep %d: %.3f ms for 2^%d keys (%.3f ms per 1e9), abort %u, survivors %llu (host %llu)%s\n", r, ms, lg,
           ms * 1e9 / n, hs[0], got, want, (hs[0] || got != want) ? "  MISMATCH" : "");
    if (hs[0] || got != want) return 2;
    best_ring = std::min(best_ring, ms);
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(key_read_kernel, dim3(4096), dim3(256), 0, 0, keys, n, sink);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    best_read = std::min(best_read, ms);
  }
  float best_tx = 1e30f;
  for (int r = 0; r < reps; r++) {  // transport only: the ring path's own ceiling
    CK(hipMemset(sh.hdr, 0, slots * kLineWords * 8));
    CK(hipMemset(sh.rhdr, 0, slots * kLineWords * 8));
    CK(hipMemset(small, 0, 256));
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(ring_kernel, dim3(kP + kC), dim3(kThreads), lds, 0, sh, keys, n, 1);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    CK(hipGetLastError());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    uint32_t hs[1];
    CK(hipMemcpy(hs, small, 4, hipMemcpyDeviceToHost));
    printf("transport only rep %d: %.3f ms for 2^%d records (%.3f ms per 1e9), abort %u\n", r, ms, lg, ms * 1e9 / n, hs[0]);
    if (hs[0]) return 2;
    best_tx = std::min(best_tx, ms);
  }
  printf("best: transport only %.3f ms per 1e9 records\n", best_tx * 1e9 / n);
  printf("best: ring %.3f ms per 1e9 keys; key read alone (all CUs) %.3f ms per 1e9 keys (%.0f GB/s)\n",
         best_ring * 1e9 / n, best_read * 1e9 / n, n * 8 / (best_read * 1e6));
  return 0;
}
