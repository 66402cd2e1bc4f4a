// rk_radix.hip -- stable LSD radix sort of (u32 key, u32 value) pairs (gfx950).
//
// Every bucketed structure of the reference becomes a sorted array here: the
// xStart/10 processing buckets (FragmentsDatabase.cpp:84-97, stable in file
// order), the 100-bp occupancy buckets (SequenceOcupationList.cpp:5-7,17,95,
// entries in insertion order) and the group member lists (commonFunctions.cpp:
// 58,66,73, members in insertion order).  All three need a STABLE sort by a
// small integer key, which is what LSD radix gives without atomics.
//
// One pass per 8-bit digit, three kernels:
//   k_digit_hist   256-bin histogram of each 4096-key tile in LDS (LDS atomics),
//                  written tile-major: counts[tile * 256 + digit] (one 1-KB row)
//   column scan    offset of (tile, digit) = all keys of smaller digits + the
//                  same digit in earlier tiles, in place, three small kernels
//   k_digit_scatter  re-reads the tile in index order, ranks every key among
//                  equal digits (8 wave ballots -> peer mask -> popcount against
//                  a wave-private counter), places it at its tile-local sorted
//                  slot in LDS, then writes the tile out slot by slot
//                  (coalesced per digit segment).
// Tiles: 256 threads x 16 keys; wave w owns keys [1024w, 1024w+1024) of the
// tile, read 64 at a time -- coalesced, and rank order == index order; tiles
// are mapped to blocks XCD by XCD (xcd_tile).
#include "rk_internal.h"

#include <cstdlib>

namespace rk {
namespace {

// digit widths 8..10 bits (RADIX = 1 << DB bins); tiles of T threads x ITEMS keys
template <int T, int ITEMS, int DB>
__global__ void __launch_bounds__(T) k_digit_hist(const uint32_t *__restrict__ key, uint32_t n,
                                                  int shift, uint32_t tiles,
                                                  uint32_t *__restrict__ counts) {
  constexpr int TILE = T * ITEMS, RADIX = 1 << DB;
  __shared__ uint32_t hist[RADIX];
  for (int d = threadIdx.x; d < RADIX; d += T) hist[d] = 0;
  __syncthreads();
  const uint32_t base = blockIdx.x * (uint32_t)TILE;
  uint32_t kk[ITEMS];
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const uint32_t i = base + r * T + threadIdx.x;
    kk[r] = i < n ? __builtin_nontemporal_load(key + i) : 0u;
  }
#pragma unroll
  for (int r = 0; r < ITEMS; ++r)
    if (base + r * T + threadIdx.x < n) atomicAdd(&hist[(kk[r] >> shift) & (RADIX - 1)], 1u);
  __syncthreads();
  for (int d = threadIdx.x; d < RADIX; d += T)
    counts[(size_t)blockIdx.x * RADIX + d] = hist[d];
}

// Column scan of the [tiles][RADIX] digit counts: thread d of block b sums
// digit d over the rows [b*ROWS, (b+1)*ROWS) (each row read coalesced)...
constexpr uint32_t ROWS = 16;
template <int DB>
__global__ void __launch_bounds__(1 << DB) k_col_partial(const uint32_t *__restrict__ counts,
                                                         uint32_t tiles,
                                                         uint32_t *__restrict__ part) {
  constexpr int RADIX = 1 << DB;
  const uint32_t t0 = blockIdx.x * ROWS, t1 = min(t0 + ROWS, tiles);
  uint32_t s = 0;
  for (uint32_t t = t0; t < t1; ++t) s += counts[(size_t)t * RADIX + threadIdx.x];
  part[blockIdx.x * RADIX + threadIdx.x] = s;
}
// ...block d scans digit d's partial sums over the row blocks (exclusive) and
// stores the digit total...
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *tot) {
  __shared__ uint32_t wsum[NT / 64];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t inc = v;
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t o = __shfl_up(inc, off);
    if ((int)lane >= off) inc += o;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t pre = 0, all = 0;
  for (uint32_t k = 0; k < NT / 64; ++k) {
    pre += k < w ? wsum[k] : 0u;
    all += wsum[k];
  }
  __syncthreads();
  *tot = all;
  return pre + inc - v;
}
template <int DB>
__global__ void __launch_bounds__(256) k_col_digit(uint32_t *__restrict__ part, uint32_t nb,
                                                   uint32_t *__restrict__ dtot) {
  constexpr int RADIX = 1 << DB;
  const uint32_t d = blockIdx.x;
  uint32_t carry = 0;
  for (uint32_t b0 = 0; b0 < nb; b0 += 256) {
    const uint32_t b = b0 + threadIdx.x;
    const uint32_t v = b < nb ? part[(size_t)b * RADIX + d] : 0u;
    uint32_t tot;
    const uint32_t e = block_excl_scan<256>(v, &tot);
    if (b < nb) part[(size_t)b * RADIX + d] = carry + e;
    carry += tot;
  }
  if (threadIdx.x == 0) dtot[d] = carry;
}
// ...and every block rewrites its rows with running offsets (in place).
// (the digit base -- keys of all smaller digits -- is re-derived per block
// from the digit totals)
template <int DB>
__global__ void __launch_bounds__(1 << DB) k_col_final(uint32_t *__restrict__ counts,
                                                       uint32_t tiles,
                                                       const uint32_t *__restrict__ part,
                                                       const uint32_t *__restrict__ dtot) {
  constexpr int RADIX = 1 << DB;
  const uint32_t t0 = blockIdx.x * ROWS, t1 = min(t0 + ROWS, tiles);
  uint32_t all;
  const uint32_t base = block_excl_scan<RADIX>(dtot[threadIdx.x], &all);
  uint32_t run = base + part[blockIdx.x * RADIX + threadIdx.x];
  for (uint32_t t = t0; t < t1; ++t) {
    const uint32_t c = counts[(size_t)t * RADIX + threadIdx.x];
    counts[(size_t)t * RADIX + threadIdx.x] = run;
    run += c;
  }
}

// Workgroups are dispatched round-robin over the 8 XCDs: block b takes the
// (b/8)-th tile of a contiguous 1/8 of the tiles, so neighbouring tiles (whose
// same-digit segments abut in the output) are written through one XCD's L2.
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t tiles) {
  const uint32_t x = b & 7u, j = b >> 3, per = tiles >> 3, rem = tiles & 7u;
  return x * per + (x < rem ? x : rem) + j;
}

// Stable scatter of one tile through LDS.  Each wavefront ranks its own
// contiguous slice of the tile (ITEMS rounds of 64 keys) against a
// wave-private digit counter in LDS -- no workgroup barrier inside the rounds;
// DB ballots give each key's peers (same digit) in the round, so
// rank = counter[d] + #peers in lower lanes.  One barrier then turns the
// waves' digit counts into tile-local offsets; every key is placed at its
// tile-local sorted slot in LDS and the tile is written out slot by slot
// (consecutive lanes -> consecutive addresses of one digit segment).
// Tile order = (wave, round, lane) = index order, hence stable.  Every load of
// the tile is issued before the first ballot (2*ITEMS loads in flight/lane).
template <int T, int ITEMS, int DB>
__global__ void __launch_bounds__(T) k_digit_scatter(const uint32_t *__restrict__ key_in,
                                                     const uint32_t *__restrict__ val_in,
                                                     uint32_t n, int shift, uint32_t tiles,
                                                     const uint32_t *__restrict__ offs,
                                                     uint32_t *__restrict__ key_out,
                                                     uint32_t *__restrict__ val_out) {
  constexpr int RADIX = 1 << DB, NW = T / 64, TILE = T * ITEMS, DPT = RADIX / T;
  static_assert(RADIX % T == 0, "whole digits per thread in the tile scan");
  __shared__ uint32_t sk[TILE];
  __shared__ uint32_t sv[TILE];
  __shared__ uint32_t wcnt[NW][RADIX];  // per-wave digit counters, then per-wave starts
  __shared__ uint32_t lbase[RADIX];     // tile-local start of digit d
  __shared__ uint32_t wsum[NW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
  const uint32_t tile = xcd_tile(blockIdx.x, tiles);
  const uint32_t tile0 = tile * (uint32_t)TILE;
  const uint32_t cnt = n - tile0 < (uint32_t)TILE ? n - tile0 : (uint32_t)TILE;
  for (uint32_t j = threadIdx.x; j < NW * RADIX; j += T) (&wcnt[0][0])[j] = 0;
  __syncthreads();

  uint32_t kk[ITEMS], vv[ITEMS], rk[ITEMS];
  const uint32_t wbase = (uint32_t)w * (TILE / NW) + lane;
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const uint32_t i = wbase + r * 64;
    kk[r] = i < cnt ? __builtin_nontemporal_load(key_in + tile0 + i) : 0u;
  }
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const uint32_t i = wbase + r * 64;
    vv[r] = val_in ? (i < cnt ? __builtin_nontemporal_load(val_in + tile0 + i) : 0u) : tile0 + i;
  }
  uint32_t *mycnt = wcnt[w];
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const uint32_t i = wbase + r * 64;
    const bool live = i < cnt;
    const uint32_t d = (kk[r] >> shift) & (RADIX - 1);
    uint64_t peer = __ballot(live);
#pragma unroll
    for (int b = 0; b < DB; ++b) {
      const bool bit = (d >> b) & 1u;
      const uint64_t bb = __ballot(bit);
      peer &= bit ? bb : ~bb;
    }
    const uint32_t below = __popcll(peer & lt);
    const uint32_t before = live ? mycnt[d] : 0u;  // all reads precede the leaders' writes
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    if (live && below == 0) mycnt[d] = before + __popcll(peer);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    rk[r] = live ? before + below : 0xFFFFFFFFu;
  }
  __syncthreads();
  // thread t owns digits [t*DPT, (t+1)*DPT): tile totals -> exclusive scan
  // (lbase); wave starts inside each digit
  uint32_t run[DPT], tsum = 0;
#pragma unroll
  for (int j = 0; j < DPT; ++j) {
    const uint32_t d = threadIdx.x * DPT + j;
    uint32_t r0 = 0;
#pragma unroll
    for (int k2 = 0; k2 < NW; ++k2) {
      const uint32_t c = wcnt[k2][d];
      wcnt[k2][d] = r0;
      r0 += c;
    }
    run[j] = r0;
    tsum += r0;
  }
  uint32_t inc = tsum;
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t o = __shfl_up(inc, off);
    if (lane >= off) inc += o;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  {
    uint32_t pre = 0;
    for (int k2 = 0; k2 < w; ++k2) pre += wsum[k2];
    uint32_t at = pre + inc - tsum;
#pragma unroll
    for (int j = 0; j < DPT; ++j) {
      lbase[threadIdx.x * DPT + j] = at;
      at += run[j];
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    if (rk[r] == 0xFFFFFFFFu) continue;
    const uint32_t d = (kk[r] >> shift) & (RADIX - 1);
    const uint32_t pos = lbase[d] + mycnt[d] + rk[r];
    sk[pos] = kk[r];
    sv[pos] = vv[r];
  }
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < cnt; j += T) {
    const uint32_t k = sk[j];
    const uint32_t d = (k >> shift) & (RADIX - 1);
    const uint32_t gpos = offs[(size_t)tile * RADIX + d] + (j - lbase[d]);
    key_out[gpos] = k;
    val_out[gpos] = sv[j];
  }
}

// Tile shape: 256 threads x 16 keys.  Measured on MI355X at 50M keys (scatter,
// per pass, 8-bit digits): 256x16 0.181 ms, 512x16 0.184, 256x32 0.229,
// 1024x16 0.252, 1024x8 0.282 -- four 37-KB blocks per CU beat fewer, larger
// tiles.
constexpr int RT = 256, RITEMS = 16;
constexpr uint32_t RTILE = RT * RITEMS;
constexpr int MAX_DB = 10;  // the column kernels use one thread per digit (<= 1024)

template <int T, int I, int DB>
void launch_pass(const uint32_t *ki, const uint32_t *vi, uint32_t n, int shift, uint32_t tiles,
                 uint32_t *counts, ScanScratch ss, uint32_t *ko, uint32_t *vo, hipStream_t st) {
  constexpr int RADIX = 1 << DB;
  kt_begin(st, KID_HIST);
  k_digit_hist<T, I, DB><<<tiles, T, 0, st>>>(ki, n, shift, tiles, counts);
  kt_end(st, KID_HIST, 4.0 * n);  // keys read once
  const uint32_t nb = (tiles + ROWS - 1) / ROWS;
  uint32_t *part = ss.block_sums;  // nb * RADIX words
  uint32_t *dtot = part + (size_t)nb * RADIX;
  k_col_partial<DB><<<nb, RADIX, 0, st>>>(counts, tiles, part);
  k_col_digit<DB><<<RADIX, 256, 0, st>>>(part, nb, dtot);
  k_col_final<DB><<<nb, RADIX, 0, st>>>(counts, tiles, part, dtot);
  kt_begin(st, KID_SCATTER);
  k_digit_scatter<T, I, DB><<<tiles, T, 0, st>>>(ki, vi, n, shift, tiles, counts, ko, vo);
  kt_end(st, KID_SCATTER, (vi ? 16.0 : 12.0) * n);  // key (+value) read, key+value written
}

// widest digit (9 bits measured best at cfg3: 26-bit occupancy keys take 3
// passes instead of 4); RK_RADIX_BITS (8..10) overrides it, for measurements
int max_digit_bits() {
  static const int v = [] {
    const char *e = getenv("RK_RADIX_BITS");
    const int b = e ? atoi(e) : 9;
    return b < 8 ? 8 : b > MAX_DB ? MAX_DB : b;
  }();
  return v;
}

}  // namespace

thread_local KernelTimer *g_ktimer = nullptr;

size_t radix_scratch_words(uint32_t n) {
  const size_t tiles = (n + RTILE - 1) / RTILE;
  constexpr size_t RADIX = 1u << MAX_DB;
  const size_t cnt = tiles * RADIX + 1;
  const size_t part = ((tiles + ROWS - 1) / ROWS + 1) * RADIX;  // column-scan partials, totals
  return ((cnt + 3) & ~(size_t)3) + part + 64;
}

// Sorts by the low `bits` bits of key.  key_in/val_in are not modified unless
// they alias the ping-pong buffers; the result lands in key_out/val_out.
// key_tmp/val_tmp: n-word ping-pong buffers.  val_in == nullptr => values are
// the input positions 0..n-1.
void radix_sort_pairs(const uint32_t *key_in, const uint32_t *val_in, uint32_t *key_out,
                      uint32_t *val_out, uint32_t *key_tmp, uint32_t *val_tmp, uint32_t n,
                      int bits, uint32_t *scratch, size_t scratch_words, hipStream_t st,
                      int max_digit) {
  if (n == 0) return;
  if (bits < 1) bits = 1;
  // as few passes as the widest digit allows, widths as even as possible
  const int maxdb = max_digit >= 8 && max_digit <= MAX_DB ? max_digit : max_digit_bits();
  const int passes = (bits + maxdb - 1) / maxdb;
  const uint32_t tiles = (n + RTILE - 1) / RTILE;
  const size_t cnt = (size_t)tiles * (1u << MAX_DB) + 1;
  uint32_t *counts = scratch;
  ScanScratch ss{scratch + ((cnt + 3) & ~(size_t)3),
                 scratch_words - ((cnt + 3) & ~(size_t)3)};
  // ping-pong so that the last pass writes key_out/val_out
  const uint32_t *ki = key_in, *vi = val_in;
  int shift = 0;
  for (int p = 0; p < passes; ++p) {
    // pass p writes out when (passes-1-p) is even, tmp otherwise
    uint32_t *ko = ((passes - 1 - p) % 2 == 0) ? key_out : key_tmp;
    uint32_t *vo = ((passes - 1 - p) % 2 == 0) ? val_out : val_tmp;
    const int left = bits - shift, w0 = (left + (passes - p) - 1) / (passes - p);
    const int db = w0 < 8 ? 8 : w0;  // a narrower digit still uses 256 bins
    switch (db) {
      case 8: launch_pass<RT, RITEMS, 8>(ki, vi, n, shift, tiles, counts, ss, ko, vo, st); break;
      case 9: launch_pass<RT, RITEMS, 9>(ki, vi, n, shift, tiles, counts, ss, ko, vo, st); break;
      case 10: launch_pass<RT, RITEMS, 10>(ki, vi, n, shift, tiles, counts, ss, ko, vo, st); break;
      default: launch_pass<RT, RITEMS, 10>(ki, vi, n, shift, tiles, counts, ss, ko, vo, st); break;
    }
    shift += w0;
    ki = ko;
    vi = vo;
  }
}

}  // namespace rk
