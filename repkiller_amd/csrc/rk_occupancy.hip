// rk_occupancy.hip -- the SequenceOcupationList replacement (gfx950).
//
// Reference semantics (/root/reference/src):
//   * four push-front lists per 100-bp bucket of fragment centres
//     (SequenceOcupationList.h:11,15-24; .cpp:93-96), {forward, other} x {X, Y};
//   * get_associated_group (.cpp:33-91) scans its own bucket, then the buckets
//     of c-1, c+1, c-2, c+2 (guards: c>0, c<max_index, c>1, c<max_index-1 with
//     max_index = seq_size/100 -- a bucket COUNT compared with a position), and
//     returns the group of the first strictly-greatest deviation (> 0);
//   * generate_fragment_groups (commonFunctions.cpp:51-77): X query; on a hit
//     the fragment is inserted into Y only; else Y query, on a hit inserted into
//     X only; else a new group, inserted into both.
//
// Data-parallel restatement.  A fragment sits in the X list iff it did NOT hit
// on X, and in the Y list iff it did not hit on Y; only fragments that missed
// on X query Y.  So per axis, "hit" of fragment i depends only on the states of
// earlier fragments (processing index j < i) in i's probe buckets: a greedy,
// order-dependent fixpoint.  Rescanning a bucket under the strict `>` is a
// no-op, so a query's effective scan is: its own bucket newest-first, then at
// most ONE neighbour bucket newest-first restricted to j < i -- bucket B-1 when
// c % 100 in {0,1} and c >= 100, bucket B+1 when (c % 100 == 99 && c < max) or
// (c % 100 == 98 && c < max - 1).
//
// Layout: the axis' entries are radix-sorted by bucket key (strand * nbs +
// centre/100), stable, so each bucket is a contiguous RUN of positions holding
// its fragments in processing order, and buckets B-1 / B+1 are the runs just
// before / after it when non-empty.  Centre, length, state and winner live in
// that CSR order, so a bucket walk reads contiguous memory.
//
// Each sweep walks every listed run in processing order (one lane per run, or
// one wavefront per run of >= WAVE_MIN entries), deciding an entry when the
// states of all its candidates with deviation > 0 are known: any ACTIVE
// candidate => HIT (winner = first strict maximum in scan order), else all
// candidates inactive => ACTIVE.  Own-run candidates are decided earlier in the
// same walk; neighbour-run states come from global memory (monotone: UNKNOWN ->
// decided, so a stale read only delays).  The smallest undecided processing
// index is always decidable, so sweeps terminate; on real inputs neighbour
// dependencies are rare and 2-3 sweeps suffice.
//
// deviation (SequenceOcupationList.cpp:20-31) is evaluated in IEEE f64 with
// the reference's expression shape; this TU is built with -ffp-contract=off so
// 0.4*sl + 0.6*sp is never fused (the reference binary is baseline x86-64).
#include "rk_internal.h"

namespace rk {
namespace {

constexpr uint32_t WAVE_MIN = 48;  // runs at least this long get a whole wavefront

__device__ __forceinline__ double deviation(uint64_t c, uint64_t L, uint64_t oc, uint64_t oL,
                                            double lr, double pr) {
  uint64_t dl = L > oL ? L - oL : oL - L;
  double sl = -fabs((double)dl / ((double)L * lr)) + 1.0;
  if (sl < 0) return 0.0;
  uint64_t dc = c > oc ? c - oc : oc - c;
  double sp = -fabs((double)dc / ((double)L * pr)) + 1.0;
  if (sp < 0) return 0.0;
  return sl * 0.4 + sp * 0.6;
}

// -1: bucket B-1, +1: bucket B+1, 0: none
__device__ __forceinline__ int neighbour_dir(uint64_t c, uint64_t max_index) {
  const uint64_t r = c % 100;
  if (r <= 1 && c >= 100) return -1;
  if ((r == 99 && c < max_index) || (r == 98 && c < max_index - 1)) return 1;
  return 0;
}

__device__ __forceinline__ uint8_t load_state(const uint8_t *s) {
  return __hip_atomic_load(s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void store_state(uint8_t *s, uint8_t v) {
  __hip_atomic_store(s, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct Scan {
  double best;
  uint32_t win;  // CSR position of the best ACTIVE candidate
  uint32_t pos;  // its scan-order rank (wave path only)
  bool any_active, any_unknown;
};

__device__ __forceinline__ void consider(const Axis &ax, Scan &s, uint32_t q, uint64_t c,
                                         uint64_t L) {
  const uint8_t sj = load_state(&ax.state[q]);
  if (sj >= ST_HIT_PENDING) return;  // not in the list
  const double d = deviation(c, L, ax.cen[q], ax.len[q], ax.len_ratio, ax.pos_ratio);
  if (!(d > 0)) return;
  if (sj == ST_ACTIVE) {
    s.any_active = true;
    if (d > s.best) {
      s.best = d;
      s.win = q;
    }
  } else {
    s.any_unknown = true;
  }
}

__device__ __forceinline__ uint8_t decide(const Scan &s) {
  if (s.any_unknown) return s.any_active ? ST_HIT_PENDING : ST_UNKNOWN;
  return s.any_active ? ST_HIT : ST_ACTIVE;
}

// Append `item` to list when pred; called by EVERY thread of the block (uniform
// control flow).  One global atomic per block instead of one per item: a single
// hot counter serialises at ~88 increments/us (MI355X_MICROARCH.md "dequeue").
__device__ __forceinline__ void block_append(uint32_t *list, uint32_t *count, uint32_t item,
                                             bool pred) {
  __shared__ uint32_t wtot[16];
  __shared__ uint32_t gbase;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  const uint64_t b = __ballot(pred);
  if (lane == 0) wtot[w] = __popcll(b);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int k = 0; k < nw; ++k) {
      const uint32_t c = wtot[k];
      wtot[k] = t;
      t += c;
    }
    gbase = t ? atomicAdd(count, t) : 0u;
  }
  __syncthreads();
  if (pred) list[gbase + wtot[w] + __popcll(b & ((1ull << lane) - 1ull))] = item;
  __syncthreads();
}

// bounds of the run holding key +-1 adjacent to [beg, end) on side `dir`
__device__ __forceinline__ bool neighbour_run(const Axis &ax, uint32_t beg, uint32_t end,
                                              uint32_t key, int dir, uint32_t &nb,
                                              uint32_t &ne) {
  if (dir < 0) {
    if (beg == 0 || ax.key[beg - 1] != key - 1) return false;
    ne = beg;
    nb = beg - 1;
    while (nb > 0 && ax.key[nb - 1] == key - 1) --nb;
    return true;
  }
  if (end >= ax.m || ax.key[end] != key + 1) return false;
  nb = end;
  ne = end + 1;
  while (ne < ax.m && ax.key[ne] == key + 1) ++ne;
  return true;
}

// ---- one lane walks one run ----------------------------------------------
__global__ void __launch_bounds__(256) k_sweep_lane(Axis ax, const uint32_t *work, uint32_t nwork,
                                                    uint32_t *next_work, uint32_t *next_count,
                                                    uint32_t *big_work, uint32_t *big_count) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  bool pending = false, big = false;
  uint32_t beg = 0;
  if (w < nwork) {
    beg = work[w];
    const uint32_t key = ax.key[beg];
    uint32_t end = beg + 1;
    while (end < ax.m && ax.key[end] == key) ++end;
    if (end - beg >= WAVE_MIN) {
      big = true;
    } else {
      // neighbour runs, found lazily: 0 = not looked up, 1 = absent, 2 = present
      int lo_st = 0, hi_st = 0;
      uint32_t lo_b = 0, lo_e = 0, hi_b = 0, hi_e = 0;
      for (uint32_t t = beg; t < end; ++t) {
        const uint8_t st = ax.state[t];
        if (st == ST_ACTIVE || st == ST_HIT) continue;
        const uint64_t c = ax.cen[t], L = ax.len[t];
        Scan s{0.0, NONE, 0, false, false};
        for (uint32_t q = t; q-- > beg;) consider(ax, s, q, c, L);
        const int dir = neighbour_dir(c, ax.max_index);
        if (dir) {
          int &nst = dir < 0 ? lo_st : hi_st;
          uint32_t &nb = dir < 0 ? lo_b : hi_b;
          uint32_t &ne = dir < 0 ? lo_e : hi_e;
          if (nst == 0) nst = neighbour_run(ax, beg, end, key, dir, nb, ne) ? 2 : 1;
          if (nst == 2) {
            const uint32_t i = ax.ent[t];
            uint32_t q = ne;
            while (q > nb && ax.ent[q - 1] > i) --q;  // only entries inserted before i
            while (q-- > nb) consider(ax, s, q, c, L);
          }
        }
        const uint8_t ns = decide(s);
        if (ns == ST_HIT) ax.win[t] = ax.ent[s.win];
        if (ns != st) store_state(&ax.state[t], ns);
        pending |= ns == ST_UNKNOWN || ns == ST_HIT_PENDING;
      }
    }
  }
  block_append(big_work, big_count, beg, big);
  block_append(next_work, next_count, beg, pending);
}

// ---- one wavefront walks one long run --------------------------------------
// Entries are decided one after another (the walk is inherently ordered); the
// 64 lanes split each entry's candidate scan and combine with a wave argmax
// that keeps the reference's tie rule (earliest in scan order wins).
__device__ __forceinline__ void consider_ranked(const Axis &ax, Scan &s, uint32_t q, uint32_t p,
                                                uint64_t c, uint64_t L) {
  const uint8_t sj = load_state(&ax.state[q]);
  if (sj >= ST_HIT_PENDING) return;
  const double d = deviation(c, L, ax.cen[q], ax.len[q], ax.len_ratio, ax.pos_ratio);
  if (!(d > 0)) return;
  if (sj == ST_ACTIVE) {
    s.any_active = true;
    if (d > s.best || (d == s.best && p < s.pos)) {
      s.best = d;
      s.win = q;
      s.pos = p;
    }
  } else {
    s.any_unknown = true;
  }
}

__device__ __forceinline__ void wave_combine(Scan &s) {
  for (int off = 32; off > 0; off >>= 1) {
    const double ob = __shfl_xor(s.best, off);
    const uint32_t ow = __shfl_xor(s.win, off);
    const uint32_t op = __shfl_xor(s.pos, off);
    const int oa = __shfl_xor((int)s.any_active, off);
    const int ou = __shfl_xor((int)s.any_unknown, off);
    if (ob > s.best || (ob == s.best && op < s.pos)) {
      s.best = ob;
      s.win = ow;
      s.pos = op;
    }
    s.any_active |= oa != 0;
    s.any_unknown |= ou != 0;
  }
}

__global__ void __launch_bounds__(256) k_sweep_wave(Axis ax, const uint32_t *work,
                                                    const uint32_t *nwork_ptr, uint32_t *next_work,
                                                    uint32_t *next_count) {
  const uint32_t nwork = *nwork_ptr;
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < nwork;
       w += (gridDim.x * blockDim.x) >> 6) {
    const uint32_t beg = work[w];
    const uint32_t key = ax.key[beg];
    uint32_t end = beg + 1;
    while (end < ax.m && ax.key[end] == key) ++end;
    uint32_t lo_b = 0, lo_e = 0, hi_b = 0, hi_e = 0;
    const bool has_lo = neighbour_run(ax, beg, end, key, -1, lo_b, lo_e);
    const bool has_hi = neighbour_run(ax, beg, end, key, 1, hi_b, hi_e);
    bool pending = false;
    for (uint32_t t = beg; t < end; ++t) {
      const uint8_t st = load_state(&ax.state[t]);
      if (st == ST_ACTIVE || st == ST_HIT) continue;
      const uint64_t c = ax.cen[t], L = ax.len[t];
      const uint32_t i = ax.ent[t];
      Scan s{0.0, NONE, 0xFFFFFFFFu, false, false};
      for (uint32_t q0 = beg; q0 < t; q0 += 64) {  // own run, newest first: rank t-1-q
        const uint32_t q = q0 + lane;
        if (q < t) consider_ranked(ax, s, q, t - 1 - q, c, L);
      }
      const int dir = neighbour_dir(c, ax.max_index);
      if ((dir < 0 && has_lo) || (dir > 0 && has_hi)) {
        const uint32_t nb = dir < 0 ? lo_b : hi_b, ne = dir < 0 ? lo_e : hi_e;
        const uint32_t own = t - beg;
        for (uint32_t q0 = nb; q0 < ne; q0 += 64) {
          const uint32_t q = q0 + lane;
          if (q < ne && ax.ent[q] < i) consider_ranked(ax, s, q, own + (ne - 1 - q), c, L);
        }
      }
      wave_combine(s);
      const uint8_t ns = decide(s);
      if (lane == 0) {
        if (ns == ST_HIT) ax.win[t] = ax.ent[s.win];
        if (ns != st) store_state(&ax.state[t], ns);
      }
      pending |= ns == ST_UNKNOWN || ns == ST_HIT_PENDING;
    }
    if (pending && lane == 0) next_work[atomicAdd(next_count, 1u)] = beg;
  }
}

// run starts of a sorted key array: p == 0 || key[p] != key[p-1]
__global__ void __launch_bounds__(256) k_run_starts(const uint32_t *key, uint32_t m,
                                                    uint32_t *list, uint32_t *count) {
  for (uint32_t b0 = blockIdx.x * blockDim.x; b0 < m; b0 += gridDim.x * blockDim.x) {
    const uint32_t p = b0 + threadIdx.x;
    const bool start = p < m && (p == 0 || key[p] != key[p - 1]);
    block_append(list, count, p, start);
  }
}

}  // namespace

void run_starts(const uint32_t *key, uint32_t m, uint32_t *list, uint32_t *count,
                hipStream_t st) {
  (void)hipMemsetAsync(count, 0, sizeof(uint32_t), st);
  if (!m) return;
  uint32_t g = (m + 255) / 256;
  if (g > 8192) g = 8192;
  k_run_starts<<<g, 256, 0, st>>>(key, m, list, count);
}

void occupancy_sweep(const Axis &ax, const uint32_t *work, uint32_t nwork, uint32_t *next_work,
                     uint32_t *next_count, uint32_t *big_work, uint32_t *big_count,
                     hipStream_t st) {
  if (!nwork) return;
  (void)hipMemsetAsync(big_count, 0, sizeof(uint32_t), st);
  k_sweep_lane<<<(nwork + 255) / 256, 256, 0, st>>>(ax, work, nwork, next_work, next_count,
                                                     big_work, big_count);
  unsigned blocks = (nwork + 3) / 4;  // one wave per long run (upper bound), grid-strided
  if (blocks > 2048) blocks = 2048;
  k_sweep_wave<<<blocks, 256, 0, st>>>(ax, big_work, big_count, next_work, next_count);
}

}  // namespace rk
