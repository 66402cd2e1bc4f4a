// rk_sort.hip -- device-wide exclusive scan of u32 (gfx950).
//
// Used by the radix sort (digit offsets, rk_radix.hip) and for the new-group
// ranks (gid = exclusive scan of "opens a group" flags in processing order,
// the creation order of commonFunctions.cpp:72-74).
//
// Scan: 256-thread blocks, 4096 u32 per tile (4 rows of 1024; each row one
// coalesced uint4 per lane), wave inclusive scan in DPP (row_shr 1/2/4/8 then
// row_bcast 15/31 -- GFX9 DPP, 6 VALU ops for 64 lanes), wave totals through
// LDS, tiles chained by a recursive reduce-then-scan.
#include <atomic>
#include <cstdlib>

#include "rk_internal.h"

namespace rk {
namespace {

constexpr int SCAN_THREADS = 256;
constexpr int SCAN_ROW = SCAN_THREADS * 4;  // 1024
constexpr int SCAN_TILE = SCAN_ROW * 4;     // 4096

__device__ __forceinline__ uint4 load4(const uint32_t *in, size_t base, size_t n) {
  if (base + 3 < n) return *reinterpret_cast<const uint4 *>(in + base);
  uint4 v = {0, 0, 0, 0};
  if (base + 0 < n) v.x = in[base + 0];
  if (base + 1 < n) v.y = in[base + 1];
  if (base + 2 < n) v.z = in[base + 2];
  return v;
}

__device__ __forceinline__ void store4(uint32_t *out, size_t base, size_t n, uint4 v) {
  if (base + 3 < n) {
    *reinterpret_cast<uint4 *>(out + base) = v;
    return;
  }
  if (base + 0 < n) out[base + 0] = v.x;
  if (base + 1 < n) out[base + 1] = v.y;
  if (base + 2 < n) out[base + 2] = v.z;
}

// exclusive block scan of one value per thread; returns the block total in *tot
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *tot) {
  __shared__ uint32_t wsum[SCAN_THREADS / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t inc = wave_incl_scan(v);
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t pre = 0, all = 0;
#pragma unroll
  for (int k = 0; k < SCAN_THREADS / 64; ++k) {
    uint32_t s = wsum[k];
    pre += k < w ? s : 0u;
    all += s;
  }
  __syncthreads();
  *tot = all;
  return pre + inc - v;
}

// the scanned words: an array, or the root flags (par[k] == k, k < m) of a
// parent array -- the new-group ranks straight from the parents, no flag array
struct WordsIn {
  const uint32_t *in;
  __device__ __forceinline__ uint4 load(size_t base, size_t n) const { return load4(in, base, n); }
};
struct RootsIn {
  const uint32_t *par;
  size_t m;
  __device__ __forceinline__ uint4 load(size_t base, size_t) const {
    if (base + 3 < m) {
      const uint4 p = *reinterpret_cast<const uint4 *>(par + base);
      return make_uint4(p.x == base, p.y == base + 1, p.z == base + 2, p.w == base + 3);
    }
    uint4 v = {0, 0, 0, 0};
    if (base + 0 < m) v.x = par[base + 0] == base + 0;
    if (base + 1 < m) v.y = par[base + 1] == base + 1;
    if (base + 2 < m) v.z = par[base + 2] == base + 2;
    return v;
  }
};

template <class In>
__global__ void __launch_bounds__(SCAN_THREADS) k_reduce_tiles(const In in, size_t n,
                                                               uint32_t *sums) {
  __shared__ uint32_t red[SCAN_THREADS / 64];
  const size_t tile = (size_t)blockIdx.x * SCAN_TILE;
  uint32_t s = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    uint4 v = in.load(tile + (size_t)r * SCAN_ROW + threadIdx.x * 4, n);
    s += v.x + v.y + v.z + v.w;
  }
  s = wave_incl_scan(s);
  if ((threadIdx.x & 63) == 63) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int k = 0; k < SCAN_THREADS / 64; ++k) t += red[k];
    sums[blockIdx.x] = t;
  }
}

// exclusive scan of each tile, plus prefix[blockIdx] when given; in may == out
template <class In>
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_tiles(const In in, uint32_t *out,
                                                             size_t n, const uint32_t *prefix,
                                                             uint32_t *total, uint32_t *clear0) {
  const size_t tile = (size_t)blockIdx.x * SCAN_TILE;
  uint32_t carry = prefix ? prefix[blockIdx.x] : 0u;
  uint4 v[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = in.load(tile + (size_t)r * SCAN_ROW + threadIdx.x * 4, n);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    uint32_t t = v[r].x + v[r].y + v[r].z + v[r].w, tot;
    uint32_t e = block_excl_scan(t, &tot) + carry;
    uint4 o;
    o.x = e;
    o.y = o.x + v[r].x;
    o.z = o.y + v[r].y;
    o.w = o.z + v[r].z;
    const size_t base = tile + (size_t)r * SCAN_ROW + threadIdx.x * 4;
    store4(out, base, n, o);
    if (total && base <= n - 1 && n - 1 < base + 4) {  // out[n - 1] also into *total
      const uint32_t j = (uint32_t)(n - 1 - base);
      *total = j == 0 ? o.x : j == 1 ? o.y : j == 2 ? o.z : o.w;
    }
    carry += tot;
  }
  // the input's first word cleared once read (block 0 alone reads it): a
  // count array reused as a list, its count word zero without a launch
  if (clear0 && blockIdx.x == 0 && threadIdx.x == 0) *clear0 = 0u;
}

// Single pass (one launch instead of three, the input read once): tile b
// (= blockIdx.x) scans its 4096 words, publishes its aggregate, finds its
// prefix by a decoupled look-back over the tiles before it and publishes its
// inclusive prefix.  A status word is epoch << 33 | inclusive << 32 | value:
// a word of another epoch (an earlier scan, or never written) is unpublished,
// so the words need no clear launch.  Tiles are block ids: a workgroup
// dispatcher starts its blocks in order and a tile waits only on lower ones,
// so the lowest unfinished tile can always finish (no ticket counter to
// clear either).  Wave 0 walks back 64 tiles per round trip.
__device__ __forceinline__ unsigned long long st_load(const unsigned long long *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_store(unsigned long long *p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class In>
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_1pass(const In in, uint32_t *out, size_t n,
                                                             unsigned long long *status,
                                                             uint32_t epoch, uint32_t *total,
                                                             uint32_t *clear0) {
  __shared__ uint32_t s_pre;
  const uint32_t b = blockIdx.x, lane = threadIdx.x & 63;
  const size_t tile = (size_t)b * SCAN_TILE;
  uint4 v[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = in.load(tile + (size_t)r * SCAN_ROW + threadIdx.x * 4, n);
  uint32_t e[4], agg = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    uint32_t tot;
    e[r] = block_excl_scan(v[r].x + v[r].y + v[r].z + v[r].w, &tot) + agg;
    agg += tot;
  }
  const unsigned long long tag = (unsigned long long)epoch << 33;
  if (threadIdx.x < 64) {
    uint32_t pre = 0;
    if (b > 0) {
      if (threadIdx.x == 0) st_store(&status[b], tag | agg);  // the aggregate first
      uint32_t j = b;  // tiles [0, j) not yet accounted for
      for (;;) {
        const bool in_range = lane < j;
        const unsigned long long w = in_range ? st_load(&status[j - 1 - lane]) : 0ull;
        const bool pub = in_range && (w >> 33) == epoch;
        const bool inc = pub && ((w >> 32) & 1ull);
        const uint64_t stop = __builtin_amdgcn_ballot_w64(!pub || inc);  // (lane j: tile 0 passed)
        const uint64_t incm = __builtin_amdgcn_ballot_w64(inc);
        const uint32_t f = stop ? (uint32_t)__builtin_ctzll(stop) : 64u;
        const bool done = f < 64 && (((incm >> f) & 1ull) || f >= j);  // (uniform)
        // the published words before the first stop (and that stop when inclusive)
        const bool take = lane < f || (lane == f && inc);
        uint32_t x = take ? (uint32_t)w : 0u;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
        pre += x;
        if (done) break;  // (f >= j: walked past tile 0 -- tile 0 publishes INC alone)
        j = f < j ? j - f : 0u;
        if (f < 64) __builtin_amdgcn_s_sleep(1);  // an unpublished tile: poll it again
      }
      if (threadIdx.x == 0) st_store(&status[b], tag | 1ull << 32 | (unsigned long long)(pre + agg));
    } else if (threadIdx.x == 0) {
      st_store(&status[0], tag | 1ull << 32 | agg);
    }
    if (threadIdx.x == 0) s_pre = pre;
  }
  __syncthreads();
  const uint32_t pre = s_pre;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    uint4 o;
    o.x = e[r] + pre;
    o.y = o.x + v[r].x;
    o.z = o.y + v[r].y;
    o.w = o.z + v[r].z;
    const size_t base = tile + (size_t)r * SCAN_ROW + threadIdx.x * 4;
    store4(out, base, n, o);
    if (total && base <= n - 1 && n - 1 < base + 4) {
      const uint32_t j = (uint32_t)(n - 1 - base);
      *total = j == 0 ? o.x : j == 1 ? o.y : j == 2 ? o.z : o.w;
    }
  }
  if (clear0 && b == 0 && threadIdx.x == 0) *clear0 = 0u;
}

}  // namespace

size_t scan_blocks(size_t n) {
  size_t total = 0;
  const size_t tiles = (n + SCAN_TILE - 1) / SCAN_TILE;
  while (n > (size_t)SCAN_TILE) {
    n = (n + SCAN_TILE - 1) / SCAN_TILE;
    total += (n + 4) & ~(size_t)3;  // keeps every level 16-B aligned
  }
  // the single pass' status words: 8 B a tile, 8-B aligned
  const size_t onepass = 2 * tiles + 2;
  return (total > onepass ? total : onepass) + 1;
}

// RK_SCAN_1PASS=0: the three-launch reduce-then-scan for every scan
static bool scan_1pass() {
  static const bool on = [] {
    const char *e = getenv("RK_SCAN_1PASS");
    return !(e && e[0] == '0');
  }();
  return on;
}
// one epoch a single-pass scan (bit 30 set: never a zeroed word's)
static uint32_t scan_epoch() {
  static std::atomic<uint32_t> next{0};
  return (next.fetch_add(1, std::memory_order_relaxed) & 0x3FFFFFFFu) | 0x40000000u;
}

template <class In>
static void scan_any(const In in, uint32_t *out, size_t n, ScanScratch ss, hipStream_t st,
                     uint32_t *total = nullptr, uint32_t *clear0 = nullptr) {
  if (n == 0) return;
  if (n <= (size_t)SCAN_TILE) {
    k_scan_tiles<<<1, SCAN_THREADS, 0, st>>>(in, out, n, nullptr, total, clear0);
    return;
  }
  const size_t tiles = (n + SCAN_TILE - 1) / SCAN_TILE;
  // (up to 256 tiles: over cfg3's 50M root flags, 12K tiles, the look-back
  // chain cost more than the second read pass: group_roots 0.555 -> 0.575 ms)
  if (scan_1pass() && tiles <= 256 && 2 * tiles + 2 <= ss.cap) {
    uintptr_t a = (uintptr_t)ss.block_sums;
    a = (a + 7) & ~(uintptr_t)7;
    k_scan_1pass<<<(unsigned)tiles, SCAN_THREADS, 0, st>>>(in, out, n, (unsigned long long *)a,
                                                           scan_epoch(), total, clear0);
    return;
  }
  size_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
  uint32_t *sums = ss.block_sums;
  const size_t stride = (nb + 4) & ~(size_t)3;  // uint4 loads need 16-B alignment
  ScanScratch rest{ss.block_sums + stride, ss.cap - stride};
  k_reduce_tiles<<<(unsigned)nb, SCAN_THREADS, 0, st>>>(in, n, sums);
  scan_any(WordsIn{sums}, sums, nb, rest, st);
  k_scan_tiles<<<(unsigned)nb, SCAN_THREADS, 0, st>>>(in, out, n, sums, total, clear0);
}

void exclusive_scan_u32(const uint32_t *in, uint32_t *out, size_t n, ScanScratch ss,
                        hipStream_t st) {
  scan_any(WordsIn{in}, out, n, ss, st);
}
void exclusive_scan_u32_clear0(uint32_t *in, uint32_t *out, size_t n, ScanScratch ss,
                               hipStream_t st) {
  scan_any(WordsIn{in}, out, n, ss, st, nullptr, in);
}

void exclusive_scan_roots(const uint32_t *par, uint32_t m, uint32_t *out, ScanScratch ss,
                          hipStream_t st, uint32_t *total) {
  scan_any(RootsIn{par, m}, out, (size_t)m + 1, ss, st, total);
}

}  // namespace rk
