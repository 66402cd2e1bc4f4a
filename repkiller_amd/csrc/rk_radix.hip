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
//                  written digit-major: counts[digit * tiles + tile]
//   exclusive scan over counts (rk_sort.hip, DPP wave scan)
//   k_digit_scatter  re-reads the tile in index order, ranks every key among
//                  equal digits (8 wave ballots -> peer mask -> popcount against
//                  a wave-private counter), places it at its tile-local sorted
//                  slot in LDS, then writes the tile out slot by slot
//                  (coalesced per digit segment).
// Tiles: 256 threads x 16 keys; wave w owns keys [1024w, 1024w+1024) of the
// tile, read 64 at a time -- coalesced, and rank order == index order.
#include "rk_internal.h"

namespace rk {
namespace {

constexpr int RT = 256;             // threads per block
constexpr int RITEMS = 16;          // keys per thread
constexpr int RTILE = RT * RITEMS;  // 4096 keys per tile
constexpr int RADIX = 256;

__global__ void __launch_bounds__(RT) k_digit_hist(const uint32_t *__restrict__ key, uint32_t n,
                                                   int shift, uint32_t tiles,
                                                   uint32_t *__restrict__ counts) {
  __shared__ uint32_t hist[RADIX];
  hist[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t base = blockIdx.x * (uint32_t)RTILE;
#pragma unroll
  for (int r = 0; r < RITEMS; ++r) {
    const uint32_t i = base + r * RT + threadIdx.x;
    if (i < n) atomicAdd(&hist[(key[i] >> shift) & (RADIX - 1)], 1u);
  }
  __syncthreads();
  counts[threadIdx.x * tiles + blockIdx.x] = hist[threadIdx.x];
}

// Stable scatter of one tile through LDS.  Each wavefront ranks its own
// contiguous quarter of the tile (1024 keys, 16 rounds of 64) against a
// wave-private digit counter in LDS -- no workgroup barrier inside the rounds;
// 8 ballots give each key's peers (same digit) in the round, so
// rank = counter[d] + #peers in lower lanes.  One barrier then turns the four
// waves' digit counts into tile-local offsets; every key is placed at its
// tile-local sorted slot in LDS and the tile is written out slot by slot
// (consecutive lanes -> consecutive addresses of one digit segment).
// Tile order = (wave, round, lane) = index order, hence stable.
__global__ void __launch_bounds__(RT) k_digit_scatter(const uint32_t *__restrict__ key_in,
                                                      const uint32_t *__restrict__ val_in,
                                                      uint32_t n, int shift, uint32_t tiles,
                                                      const uint32_t *__restrict__ offs,
                                                      uint32_t *__restrict__ key_out,
                                                      uint32_t *__restrict__ val_out) {
  constexpr int NW = RT / 64;
  __shared__ uint32_t sk[RTILE];
  __shared__ uint32_t sv[RTILE];
  __shared__ uint32_t wcnt[NW][RADIX];  // per-wave digit counters, then per-wave starts
  __shared__ uint32_t lbase[RADIX];     // tile-local start of digit d
  __shared__ uint32_t wsum[NW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
  const uint32_t tile0 = blockIdx.x * (uint32_t)RTILE;
  const uint32_t cnt = n - tile0 < (uint32_t)RTILE ? n - tile0 : (uint32_t)RTILE;
#pragma unroll
  for (int k2 = 0; k2 < NW; ++k2) wcnt[k2][threadIdx.x] = 0;
  __syncthreads();

  uint32_t kk[RITEMS], rk[RITEMS];
  uint32_t *mycnt = wcnt[w];
#pragma unroll
  for (int r = 0; r < RITEMS; ++r) {
    const uint32_t i = (uint32_t)w * (RTILE / NW) + r * 64 + lane;
    const bool live = i < cnt;
    const uint32_t k = live ? key_in[tile0 + i] : 0u;
    const uint32_t d = (k >> shift) & (RADIX - 1);
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
    kk[r] = k;
    rk[r] = live ? before + below : 0xFFFFFFFFu;
  }
  __syncthreads();
  {  // digit d: tile total -> exclusive block scan (lbase); wave starts inside the digit
    const uint32_t d = threadIdx.x;
    uint32_t run = 0;
#pragma unroll
    for (int k2 = 0; k2 < NW; ++k2) {
      const uint32_t c = wcnt[k2][d];
      wcnt[k2][d] = run;
      run += c;
    }
    uint32_t inc = run;
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t o = __shfl_up(inc, off);
      if (lane >= off) inc += o;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t pre = 0;
    for (int k2 = 0; k2 < w; ++k2) pre += wsum[k2];
    lbase[d] = pre + inc - run;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < RITEMS; ++r) {
    if (rk[r] == 0xFFFFFFFFu) continue;
    const uint32_t d = (kk[r] >> shift) & (RADIX - 1);
    const uint32_t pos = lbase[d] + mycnt[d] + rk[r];
    const uint32_t i = (uint32_t)w * (RTILE / NW) + r * 64 + lane;
    sk[pos] = kk[r];
    sv[pos] = val_in ? val_in[tile0 + i] : tile0 + i;
  }
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < cnt; j += RT) {
    const uint32_t k = sk[j];
    const uint32_t d = (k >> shift) & (RADIX - 1);
    const uint32_t gpos = offs[d * tiles + blockIdx.x] + (j - lbase[d]);
    key_out[gpos] = k;
    val_out[gpos] = sv[j];
  }
}

}  // namespace

thread_local KernelTimer *g_ktimer = nullptr;

size_t radix_scratch_words(uint32_t n) {
  const size_t tiles = (n + RTILE - 1) / RTILE;
  const size_t cnt = tiles * RADIX + 1;
  return ((cnt + 3) & ~(size_t)3) + scan_blocks(cnt) + 64;
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
    k_digit_hist<<<tiles, RT, 0, st>>>(ki, n, 8 * p, tiles, counts);
    exclusive_scan_u32(counts, counts, (size_t)tiles * RADIX, ss, st);
    KernelTimer *kt = g_ktimer;
    const bool timed = kt && kt->n < KernelTimer::MAX;
    if (timed) (void)hipEventRecord(kt->ev[2 * kt->n], st);
    k_digit_scatter<<<tiles, RT, 0, st>>>(ki, vi, n, 8 * p, tiles, counts, ko, vo);
    if (timed) {
      (void)hipEventRecord(kt->ev[2 * kt->n + 1], st);
      kt->elems[kt->n++] = n;
    }
    ki = ko;
    vi = vo;
  }
}

}  // namespace rk
