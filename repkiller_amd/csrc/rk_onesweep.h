// rk_onesweep.h -- the one-sweep LSD radix pass of the record pipeline
// (rk_narrow.hip: 12- and 16-B records; its only user -- the generic
// pipeline's pair sort in rk_radix.hip keeps its three-kernel passes, see
// DESIGN.md).  Included inside namespace rk { namespace { ... } }.
//
// Src: rec_t (the record type), load(i) -> record i, key(rec) -> the sort key
// word.  Dst: store(pos, rec); kWave / wave(rec, live) (see rk_narrow.hip).
#pragma once

#include <type_traits>

// ---------------------------------------------------------------------------
// tile status words of the decoupled look-backs: 2 flag bits + a 30-bit count
constexpr uint32_t SW_AGG = 1u << 30, SW_INC = 2u << 30, SW_VAL = (1u << 30) - 1;

__device__ __forceinline__ uint32_t sw_load(const uint32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void sw_store(uint32_t *p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Exclusive prefix of slot `slot` over tiles [0, tile): walk back over the
// published words (AGG: that tile's own count, keep walking; INC: the prefix
// through that tile, stop), then publish this tile's inclusive prefix.  Tile
// ids come from an atomic counter in dispatch order, so every earlier tile is
// resident or done and publishes its AGG before it waits on anything.
// The walk reads LB_BATCH predecessors per round trip (hundreds of tiles are
// resident; the nearest INC is often dozens back; fewer words per trip keep
// the status traffic down).  Measured per tile at cfg3
// (RK_NW_TRACE): the look-back is ~9-10 us of ~16 us at 32; 64 reads per round
// trip made it 13 us (the status traffic itself), a wave per digit reading 64
// tiles per load (status[digit][tile]) 36-47 us.
// RK_LB_BATCH (compile time): predecessors read per round trip.  With
// 6144-record tiles, cfg3 step 8 / 12 / 16 / 24 / 32 / 48: 12.00-12.03 /
// 12.04-12.10 / 12.00-12.08 / 12.05-12.21 / 12.29-12.32 / 12.51-12.54 ms;
// after the 12-B Y/member passes, 8 / 16 / 24: 11.31-11.36 / 11.32-11.45 /
// 11.51-11.54 ms (same box); with the 7-bit passes, record passes per step at
// 4 / 8 / 12 / 16 / 24: 6.09-6.22 / 6.11-6.25 / 6.15-6.29 / 6.18-6.31 /
// 6.38-6.42 ms (RK_LIB builds, interleaved; the spread is the box's); with
// the late-Y schedule, k_onesweep per step at 8 / 16: 4.157-4.173 /
// 4.229-4.232 ms (three interleaved runs each, profiles/r3_lb_batch.json);
// later, 4 / 6 / 8 / 12: 4.138-4.141 / 4.138 / 4.151-4.155 / 4.191-4.193 ms.
#ifndef RK_LB_BATCH
#define RK_LB_BATCH 6
#endif
// RK_LB_SLEEP: s_sleep units between polls of unpublished tiles (0 / 1 / 4:
// 12.09-12.10 / 12.12-12.14 / 12.10-12.18 ms, neutral)
#ifndef RK_LB_SLEEP
#define RK_LB_SLEEP 1
#endif
constexpr uint32_t LB_BATCH = RK_LB_BATCH;

// Tile loads.  Every lane loads (dead ones a copy of the tile's last record):
// no branch around a load, which made the compiler wait for each item's
// round trip before issuing the next (SrcYX12's merged X-hit bit: 14 serial
// HBM round trips in the tile prologue).  A Src with kPerRow keeps the
// guarded per-item form (SrcFile: computing the records from every item's
// raw columns at once spills 22-53 VGPRs under the 128-VGPR bound; per item
// it waits for each item's round trip, in the first order pass only).  A Src
// with kFixup adds per-wave extras after the loads (SrcYX12: the X-hit
// bitmask words, one vector load for all items).
template <class S, class = void>
struct has_per_row : std::false_type {};
template <class S>
struct has_per_row<S, std::void_t<decltype(S::kPerRow)>> : std::true_type {};
template <class S, class = void>
struct has_fixup : std::false_type {};
template <class S>
struct has_fixup<S, std::void_t<decltype(S::kFixup)>> : std::true_type {};
template <int ITEMS, class Src, class R>
__device__ __forceinline__ void load_items(const Src &src, R (&rec)[ITEMS], uint32_t base,
                                           uint32_t wbase, uint32_t cnt) {
  if constexpr (has_per_row<Src>::value) {
    if (cnt == (uint32_t)(ITEMS * blockDim.x)) {  // a full tile: one base, constant offsets
#pragma unroll
      for (int r = 0; r < ITEMS; ++r) rec[r] = src.load(base + wbase + r * 64);
    } else {
#pragma unroll
      for (int r = 0; r < ITEMS; ++r) {
        const uint32_t i = wbase + r * 64;
        rec[r] = i < cnt ? src.load(base + i) : R{};
      }
    }
  } else {
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t i = wbase + r * 64;
      rec[r] = src.load(base + (i < cnt ? i : cnt - 1));
    }
  }
  if constexpr (has_fixup<Src>::value) src.template fixup<ITEMS>(rec, base, wbase);
}

__device__ __forceinline__ uint32_t look_back(uint32_t *status, uint32_t tile, uint32_t stride,
                                              uint32_t slot, uint32_t mine) {
  uint32_t acc = 0;
  uint32_t j = tile;  // tiles [0, j) not yet accounted for
  while (j > 0) {
    const uint32_t cnt = j < LB_BATCH ? j : LB_BATCH;
    uint32_t v[LB_BATCH];
#pragma unroll
    for (uint32_t k = 0; k < LB_BATCH; ++k)
      v[k] = k < cnt ? sw_load(&status[(size_t)(j - 1 - k) * stride + slot]) : 0u;
    uint32_t k = 0;
    bool done = false;
#pragma unroll
    for (uint32_t q = 0; q < LB_BATCH; ++q) {
      if (done || q != k || q >= cnt) continue;
      const uint32_t f = v[q] & ~SW_VAL;
      if (f == 0) continue;  // not published yet: poll again from here
      acc += v[q] & SW_VAL;
      ++k;
      done = f == SW_INC;
    }
    if (done) break;
    j -= k;
    if (RK_LB_SLEEP && k < cnt) __builtin_amdgcn_s_sleep(RK_LB_SLEEP);
  }
  sw_store(&status[(size_t)tile * stride + slot], SW_INC | (acc + mine));
  return acc;
}

// ---------------------------------------------------------------------------
// One LSD pass, persistent: each block claims tiles (T threads x ITEMS
// records) from an atomic counter in dispatch order and, per tile:
//   1 ranks its records (held in registers) -- wave w ranks its contiguous
//     slice, ITEMS rounds of 64, against a wave-private digit counter by DB
//     ballots (index order = rank order: stable);
//   2 publishes the tile's digit counts for the look-back, turns the counts
//     into tile-local starts and places the records at their sorted LDS slot;
//   3 issues the loads of its NEXT tile, then walks the look-back (the global
//     start of each digit in this tile) -- the next tile's loads are in
//     flight during the look-back, whose cross-CU round trips (~2-5 us each
//     under streaming load) made it half of a tile's time when every tile
//     was its own block;
//   4 writes the tile out slot by slot (consecutive lanes -> consecutive
//     addresses of one digit segment).
// Deadlock-free: a block holds at most its current tile and the claimed next
// one, and a tile's look-back only waits for smaller tiles, each of which is
// held by a running block that publishes it without waiting for larger ones.
// Src: load(i) -> record i, key(rec); Dst: store(pos, rec).
// (two blocks per CU: 4 waves per SIMD at 512 threads -- at most 128 VGPRs,
// which the branch-free tile loads would exceed unbounded)
template <int T, int ITEMS, int DB, bool PERSIST, class Src, class Dst>
__global__ void __launch_bounds__(T)
__attribute__((amdgpu_waves_per_eu(T >= 512 && ITEMS <= 14 ? 4 : 1)))
k_onesweep(Src src, Dst dst, uint32_t n, uint32_t tiles,
                                                int shift, const uint32_t *__restrict__ ghist,
                                                uint32_t *__restrict__ status,
                                                uint32_t *__restrict__ tile_ctr,
                                                uint64_t *__restrict__ trace,
                                                uint32_t *__restrict__ clear_next) {
  // thread t < RADIX / DPT owns digits [t*DPT, (t+1)*DPT)
  constexpr int RADIX = 1 << DB, NW = T / 64, TILE = T * ITEMS;
  constexpr int DPT = RADIX >= T ? RADIX / T : 1, OWNERS = RADIX / DPT;
  static_assert(RADIX % T == 0 || T % RADIX == 0, "whole digits per thread");
  const bool owner = (int)threadIdx.x < OWNERS;
  // sorted records staged in LDS, LSLOTS slots at a time (tiles above 64 KB of
  // records are placed and written out in rounds)
  using R = typename Src::rec_t;  // uint4 (16-B records) or uint2 (key, value pairs)
  // (48 KB with 9-bit and wider digits, whose counters take the rest: two
  // blocks per CU)
  constexpr int LBYTES = DB >= 9 ? 49152 : 65536;
  constexpr int LSLOTS = TILE < (int)(LBYTES / sizeof(R)) ? TILE : (int)(LBYTES / sizeof(R));
  static_assert(!PERSIST || LSLOTS == TILE, "persistent tiles reload rec[] before the write-out");
  __shared__ R srec[LSLOTS];
  __shared__ uint32_t wcnt[NW][RADIX];  // per-wave digit counters, then per-wave starts
  __shared__ uint32_t lbase[RADIX];     // tile-local start of digit d
  __shared__ uint32_t gpos[RADIX];      // global position of the tile's first digit-d record
  __shared__ uint32_t wsum[NW], gsum[NW];
  __shared__ uint32_t s_tile[2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
  const uint64_t tr_entry = trace ? __builtin_amdgcn_s_memrealtime() : 0;
  if (threadIdx.x == 0) s_tile[0] = atomicAdd(tile_ctr, 1u);
  // this owner's digits' counts over the whole pass: their exclusive scan (the
  // digits' global starts) rides on the tile-local scan of step 2, so the
  // block's start waits only for its ticket
  uint32_t gh[DPT];
#pragma unroll
  for (int j = 0; j < DPT; ++j) gh[j] = owner ? ghist[threadIdx.x * DPT + j] : 0u;
  __syncthreads();
  uint32_t tile = s_tile[0];
  if (tile >= tiles) return;
  const uint32_t wbase = (uint32_t)w * (TILE / NW) + lane;
  R rec[ITEMS];
  uint32_t rk[ITEMS];
  {
    const uint32_t tile0 = tile * (uint32_t)TILE;
    const uint32_t cnt = n - tile0 < (uint32_t)TILE ? n - tile0 : (uint32_t)TILE;
    load_items<ITEMS>(src, rec, tile0, wbase, cnt);
  }
  uint32_t *mycnt = wcnt[w];
  for (uint32_t it = 0;; ++it) {
    const uint64_t tr0 = trace ? __builtin_amdgcn_s_memrealtime() : 0;
    const uint32_t tile0 = tile * (uint32_t)TILE;
    const uint32_t cnt = n - tile0 < (uint32_t)TILE ? n - tile0 : (uint32_t)TILE;
    if (PERSIST && threadIdx.x == 0) s_tile[(it + 1) & 1] = atomicAdd(tile_ctr, 1u);
    // the next pass' status row of this tile (same tiles, same radix), zeroed
    // here instead of by a memset between the passes
    if (clear_next)
      for (uint32_t d = threadIdx.x; d < (uint32_t)RADIX; d += T) clear_next[(size_t)tile * RADIX + d] = 0;
    // 1: rank (the wave's own counter row: no block barrier before it)
    for (uint32_t d = lane; d < RADIX; d += 64) mycnt[d] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t i = wbase + r * 64;
      const bool live = i < cnt;
      const uint32_t d = (src.key(rec[r]) >> shift) & (RADIX - 1);
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
    const uint64_t tr1 = trace ? __builtin_amdgcn_s_memrealtime() : 0;
    // 2: thread t owns digits [t*DPT, (t+1)*DPT): tile totals (published at
    // once: later tiles may be waiting for them), wave starts, tile-local starts
    uint32_t run[DPT], tsum = 0, gs = 0;
#pragma unroll
    for (int j = 0; j < DPT; ++j) {
      run[j] = 0;
      gs += gh[j];
      if (!owner) continue;
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
      sw_store(&status[(size_t)tile * RADIX + d], (tile ? SW_AGG : SW_INC) | r0);
    }
    uint32_t inc = tsum, ginc = gs;
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t o = __shfl_up(inc, off), go = __shfl_up(ginc, off);
      if (lane >= off) inc += o, ginc += go;
    }
    if (lane == 63) wsum[w] = inc, gsum[w] = ginc;
    __syncthreads();
    uint32_t gb[DPT];  // the global start of each owned digit
    {
      uint32_t at = inc - tsum, gat = ginc - gs;
      for (int k2 = 0; k2 < w; ++k2) at += wsum[k2], gat += gsum[k2];
#pragma unroll
      for (int j = 0; j < DPT; ++j) {
        gb[j] = gat, gat += gh[j];
        if (owner) lbase[threadIdx.x * DPT + j] = at, at += run[j];
      }
    }
    __syncthreads();
    // sorted slot of every record (round 0's placed at once)
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      if (rk[r] == 0xFFFFFFFFu) continue;
      const uint32_t d = (src.key(rec[r]) >> shift) & (RADIX - 1);
      rk[r] += lbase[d] + mycnt[d];
      if (LSLOTS == TILE || rk[r] < (uint32_t)LSLOTS) srec[rk[r]] = rec[r];
    }
    // 3: the next tile's loads, then the look-back
    const uint32_t next = PERSIST ? s_tile[(it + 1) & 1] : tiles;
    if (next < tiles) {
      const uint32_t n0 = next * (uint32_t)TILE;
      const uint32_t ncnt = n - n0 < (uint32_t)TILE ? n - n0 : (uint32_t)TILE;
      load_items<ITEMS>(src, rec, n0, wbase, ncnt);
    }
    if (owner) {
#pragma unroll
      for (int j = 0; j < DPT; ++j) {
        const uint32_t d = threadIdx.x * DPT + j;
        gpos[d] = gb[j] + (tile ? look_back(status, tile, RADIX, d, run[j]) : 0u);
      }
    }
    __syncthreads();
    const uint64_t tr2 = trace ? __builtin_amdgcn_s_memrealtime() : 0;
    // 4: write-out (the next iteration's LDS writes follow its first barrier,
    // which every thread reaches only after this loop)
    for (uint32_t h0 = 0; h0 < cnt; h0 += LSLOTS) {
      if (LSLOTS < TILE && h0 > 0) {  // the next round of sorted slots
        __syncthreads();
#pragma unroll
        for (int r = 0; r < ITEMS; ++r)
          if (rk[r] != 0xFFFFFFFFu && rk[r] - h0 < (uint32_t)LSLOTS) srec[rk[r] - h0] = rec[r];
        __syncthreads();
      }
      const uint32_t h1 = cnt - h0 < (uint32_t)LSLOTS ? cnt : h0 + LSLOTS;
      if constexpr (Dst::kPre) {
        // the Dst's dependent per-record load issued one slot round ahead
        uint32_t j = h0 + threadIdx.x;
        R r = j < h1 ? srec[j - h0] : R{};
        uint32_t pv = j < h1 ? dst.pre(r) : 0u;
        for (uint32_t j0 = h0; j0 < h1; j0 += T, j += T) {
          const uint32_t jn = j + T;
          const R rn = jn < h1 ? srec[jn - h0] : R{};
          const uint32_t pn = jn < h1 ? dst.pre(rn) : 0u;
          if (j < h1) {
            const uint32_t d = (src.key(r) >> shift) & (RADIX - 1);
            dst.store(gpos[d] + (j - lbase[d]), r, pv);
          }
          r = rn;
          pv = pn;
        }
      } else {
        for (uint32_t j0 = h0; j0 < h1; j0 += T) {  // wave-uniform trip count (Dst::wave)
          const uint32_t j = j0 + threadIdx.x;
          const bool live = j < h1;
          const R r = live ? srec[j - h0] : R{};
          if (live) {
            const uint32_t d = (src.key(r) >> shift) & (RADIX - 1);
            dst.store(gpos[d] + (j - lbase[d]), r);
          }
          if (Dst::kWave) dst.wave(r, live);
        }
      }
    }
    if (trace && threadIdx.x == 0) {  // RK_NW_TRACE: phase timestamps of this tile
      uint32_t xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      uint64_t *o = trace + (size_t)tile * 8;
      o[0] = tr0;
      o[1] = tr1;
      o[2] = tr2;
      o[3] = __builtin_amdgcn_s_memrealtime();
      o[4] = xcc & 15u;
      o[5] = blockIdx.x;
      o[6] = tr_entry;  // block start (the ticket, the digit starts, the loads' issue)
      o[7] = 0;
    }
    tile = next;
    if (tile >= tiles) break;
  }
}

