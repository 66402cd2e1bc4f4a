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

namespace rk {
namespace {

constexpr int RADIX = 256;

template <int T, int ITEMS>
__global__ void __launch_bounds__(T) k_digit_hist(const uint32_t *__restrict__ key, uint32_t n,
                                                  int shift, uint32_t tiles,
                                                  uint32_t *__restrict__ counts) {
  constexpr int TILE = T * ITEMS;
  __shared__ uint32_t hist[RADIX];
  if (threadIdx.x < RADIX) hist[threadIdx.x] = 0;
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
  if (threadIdx.x < RADIX) counts[(size_t)blockIdx.x * RADIX + threadIdx.x] = hist[threadIdx.x];
}

// Column scan of the [tiles][256] digit counts: thread d of block b sums
// digit d over the rows [b*ROWS, (b+1)*ROWS) (each row read coalesced)...
constexpr uint32_t ROWS = 16;
__global__ void __launch_bounds__(RADIX) k_col_partial(const uint32_t *__restrict__ counts,
                                                       uint32_t tiles,
                                                       uint32_t *__restrict__ part) {
  const uint32_t t0 = blockIdx.x * ROWS, t1 = min(t0 + ROWS, tiles);
  uint32_t s = 0;
  for (uint32_t t = t0; t < t1; ++t) s += counts[(size_t)t * RADIX + threadIdx.x];
  part[blockIdx.x * RADIX + threadIdx.x] = s;
}
// ...block d scans digit d's partial sums over the row blocks (exclusive) and
// stores the digit total...
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t *tot) {
  __shared__ uint32_t wsum[RADIX / 64];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t inc = v;
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t o = __shfl_up(inc, off);
    if ((int)lane >= off) inc += o;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t pre = 0, all = 0;
  for (uint32_t k = 0; k < RADIX / 64; ++k) {
    pre += k < w ? wsum[k] : 0u;
    all += wsum[k];
  }
  __syncthreads();
  *tot = all;
  return pre + inc - v;
}
__global__ void __launch_bounds__(RADIX) k_col_digit(uint32_t *__restrict__ part, uint32_t nb,
                                                     uint32_t *__restrict__ dtot) {
  const uint32_t d = blockIdx.x;
  uint32_t carry = 0;
  for (uint32_t b0 = 0; b0 < nb; b0 += RADIX) {
    const uint32_t b = b0 + threadIdx.x;
    const uint32_t v = b < nb ? part[(size_t)b * RADIX + d] : 0u;
    uint32_t tot;
    const uint32_t e = block_excl_scan256(v, &tot);
    if (b < nb) part[(size_t)b * RADIX + d] = carry + e;
    carry += tot;
  }
  if (threadIdx.x == 0) dtot[d] = carry;
}
// ...and every block rewrites its rows with running offsets (in place).
// (the digit base -- keys of all smaller digits -- is re-derived per block
// from the 256 digit totals)
__global__ void __launch_bounds__(RADIX) k_col_final(uint32_t *__restrict__ counts, uint32_t tiles,
                                                     const uint32_t *__restrict__ part,
                                                     const uint32_t *__restrict__ dtot) {
  const uint32_t t0 = blockIdx.x * ROWS, t1 = min(t0 + ROWS, tiles);
  uint32_t all;
  const uint32_t base = block_excl_scan256(dtot[threadIdx.x], &all);
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
// 8 ballots give each key's peers (same digit) in the round, so
// rank = counter[d] + #peers in lower lanes.  One barrier then turns the
// waves' digit counts into tile-local offsets; every key is placed at its
// tile-local sorted slot in LDS and the tile is written out slot by slot
// (consecutive lanes -> consecutive addresses of one digit segment).
// Tile order = (wave, round, lane) = index order, hence stable.  Every load of
// the tile is issued before the first ballot (2*ITEMS loads in flight/lane).
template <int T, int ITEMS>
__global__ void __launch_bounds__(T) k_digit_scatter(const uint32_t *__restrict__ key_in,
                                                     const uint32_t *__restrict__ val_in,
                                                     uint32_t n, int shift, uint32_t tiles,
                                                     const uint32_t *__restrict__ offs,
                                                     uint32_t *__restrict__ key_out,
                                                     uint32_t *__restrict__ val_out) {
  constexpr int NW = T / 64, TILE = T * ITEMS, DW = RADIX / 64;
  static_assert(T >= RADIX, "one thread per digit in the tile scan");
  __shared__ uint32_t sk[TILE];
  __shared__ uint32_t sv[TILE];
  __shared__ uint32_t wcnt[NW][RADIX];  // per-wave digit counters, then per-wave starts
  __shared__ uint32_t lbase[RADIX];     // tile-local start of digit d
  __shared__ uint32_t wsum[DW];
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
    for (int b = 0; b < 8; ++b) {
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
  // digit d (threads 0..255): tile total -> exclusive scan (lbase); wave starts
  // inside the digit
  uint32_t run = 0, inc = 0;
  if (threadIdx.x < RADIX) {
    const uint32_t d = threadIdx.x;
#pragma unroll
    for (int k2 = 0; k2 < NW; ++k2) {
      const uint32_t c = wcnt[k2][d];
      wcnt[k2][d] = run;
      run += c;
    }
    inc = run;
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t o = __shfl_up(inc, off);
      if (lane >= off) inc += o;
    }
    if (lane == 63) wsum[w] = inc;
  }
  __syncthreads();
  if (threadIdx.x < RADIX) {
    uint32_t pre = 0;
    for (int k2 = 0; k2 < w; ++k2) pre += wsum[k2];
    lbase[threadIdx.x] = pre + inc - run;
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
// per pass): 256x16 0.181 ms, 512x16 0.184, 256x32 0.229, 1024x16 0.252,
// 1024x8 0.282 -- four 37-KB blocks per CU beat fewer, larger tiles.
constexpr int RT = 256, RITEMS = 16;
constexpr uint32_t RTILE = RT * RITEMS;

template <int T, int I>
void launch_pass(const uint32_t *ki, const uint32_t *vi, uint32_t n, int shift, uint32_t tiles,
                 uint32_t *counts, ScanScratch ss, uint32_t *ko, uint32_t *vo, hipStream_t st) {
  kt_begin(st);
  k_digit_hist<T, I><<<tiles, T, 0, st>>>(ki, n, shift, tiles, counts);
  kt_end(st, KID_HIST, 4.0 * n);  // keys read once
  const uint32_t nb = (tiles + ROWS - 1) / ROWS;
  uint32_t *part = ss.block_sums;  // nb * 256 words
  uint32_t *dtot = part + (size_t)nb * RADIX;
  k_col_partial<<<nb, RADIX, 0, st>>>(counts, tiles, part);
  k_col_digit<<<RADIX, RADIX, 0, st>>>(part, nb, dtot);
  k_col_final<<<nb, RADIX, 0, st>>>(counts, tiles, part, dtot);
  kt_begin(st);
  k_digit_scatter<T, I><<<tiles, T, 0, st>>>(ki, vi, n, shift, tiles, counts, ko, vo);
  kt_end(st, KID_SCATTER, (vi ? 16.0 : 12.0) * n);  // key (+value) read, key+value written
}

}  // namespace

thread_local KernelTimer *g_ktimer = nullptr;

size_t radix_scratch_words(uint32_t n) {
  const size_t tiles = (n + RTILE - 1) / RTILE;
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
                      int bits, uint32_t *scratch, size_t scratch_words, hipStream_t st) {
  if (n == 0) return;
  if (bits < 1) bits = 1;
  const int passes = (bits + 7) / 8;
  const uint32_t tiles = (n + RTILE - 1) / RTILE;
  const size_t cnt = (size_t)tiles * RADIX + 1;
  uint32_t *counts = scratch;
  ScanScratch ss{scratch + ((cnt + 3) & ~(size_t)3),
                 scratch_words - ((cnt + 3) & ~(size_t)3)};
  // ping-pong so that the last pass writes key_out/val_out
  const uint32_t *ki = key_in, *vi = val_in;
  for (int p = 0; p < passes; ++p) {
    // pass p writes out when (passes-1-p) is even, tmp otherwise
    uint32_t *ko = ((passes - 1 - p) % 2 == 0) ? key_out : key_tmp;
    uint32_t *vo = ((passes - 1 - p) % 2 == 0) ? val_out : val_tmp;
    launch_pass<RT, RITEMS>(ki, vi, n, 8 * p, tiles, counts, ss, ko, vo, st);
    ki = ko;
    vi = vo;
  }
}

}  // namespace rk
