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
// Each sweep walks every listed bucket in processing order (one lane per
// bucket, or one wavefront per bucket of >= WAVE_MIN entries), deciding an
// entry when the states of all its candidates with deviation > 0 are known:
// any ACTIVE candidate => HIT (winner = first strict maximum in scan order),
// else all candidates inactive => ACTIVE.  Own-bucket candidates are decided
// earlier in the same walk; neighbour-bucket states come from global memory
// (monotone: UNKNOWN -> decided, so a stale read only delays).  The smallest
// undecided index is always decidable, so sweeps terminate; on real inputs
// neighbour dependencies are rare and two or three sweeps suffice.
//
// deviation (SequenceOcupationList.cpp:20-31) is evaluated in IEEE f64 with
// the reference's expression shape; this TU is built with -ffp-contract=off so
// 0.4*sl + 0.6*sp is never fused (the reference binary is baseline x86-64).
#include "rk_internal.h"

namespace rk {
namespace {

constexpr uint32_t WAVE_MIN = 48;  // buckets at least this big get a whole wavefront

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

// neighbour bucket of centre c (same strand), or NONE
__device__ __forceinline__ uint32_t neighbour_bin(uint32_t bin, uint64_t c, uint64_t max_index) {
  const uint64_t r = c % 100;
  if (r <= 1 && c >= 100) return bin - 1;
  if ((r == 99 && c < max_index) || (r == 98 && c < max_index - 1)) return bin + 1;
  return NONE;
}

struct Scan {
  double best;
  uint32_t win;
  bool any_active, any_unknown;
};

__device__ __forceinline__ void consider(const Axis &ax, Scan &s, uint32_t j, uint64_t c,
                                         uint64_t L) {
  uint8_t sj = __hip_atomic_load(&ax.state[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (sj >= ST_HIT_PENDING) return;  // not in the list
  double d = deviation(c, L, ax.cen[j], ax.len[j], ax.len_ratio, ax.pos_ratio);
  if (!(d > 0)) return;
  if (sj == ST_ACTIVE) {
    s.any_active = true;
    if (d > s.best) {
      s.best = d;
      s.win = j;
    }
  } else {
    s.any_unknown = true;
  }
}

// ---- one lane walks one bucket ------------------------------------------
__global__ void __launch_bounds__(256) k_sweep_lane(Axis ax, const uint32_t *work, uint32_t nwork,
                                                    uint32_t *next_work, uint32_t *next_count,
                                                    uint32_t *big_work, uint32_t *big_count) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= nwork) return;
  const uint32_t bin = work[w];
  const uint32_t beg = ax.off[bin], end = ax.off[bin + 1];
  if (big_work && end - beg >= WAVE_MIN) {  // hand big buckets to the wave kernel
    big_work[atomicAdd(big_count, 1u)] = bin;
    return;
  }
  bool pending = false;
  for (uint32_t t = beg; t < end; ++t) {
    const uint32_t i = ax.ent[t];
    const uint8_t st = ax.state[i];
    if (st == ST_ACTIVE || st == ST_HIT) continue;
    const uint64_t c = ax.cen[i], L = ax.len[i];
    Scan s{0.0, NONE, false, false};
    for (uint32_t q = t; q-- > beg;) consider(ax, s, ax.ent[q], c, L);
    const uint32_t nb = neighbour_bin(bin, c, ax.max_index);
    if (nb != NONE) {
      const uint32_t nbeg = ax.off[nb];
      uint32_t q = ax.off[nb + 1];
      while (q > nbeg && ax.ent[q - 1] > i) --q;
      while (q-- > nbeg) consider(ax, s, ax.ent[q], c, L);
    }
    uint8_t ns;
    if (s.any_unknown) ns = s.any_active ? ST_HIT_PENDING : ST_UNKNOWN;
    else ns = s.any_active ? ST_HIT : ST_ACTIVE;
    if (ns == ST_HIT) ax.win[i] = s.win;
    if (ns != st) __hip_atomic_store(&ax.state[i], ns, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    pending |= ns == ST_UNKNOWN || ns == ST_HIT_PENDING;
  }
  if (pending) next_work[atomicAdd(next_count, 1u)] = bin;
}

// ---- one wavefront walks one big bucket ----------------------------------
// Entries are decided one after another (the walk is inherently ordered);
// the 64 lanes split each entry's candidate scan and combine with a wave
// argmax that keeps the reference's tie rule (earliest in scan order wins).
__device__ __forceinline__ void wave_combine(Scan &s, uint32_t &pos) {
  // pos = scan-order position of s.win (smaller = scanned earlier)
  for (int off = 32; off > 0; off >>= 1) {
    double ob = __shfl_xor(s.best, off);
    uint32_t ow = __shfl_xor(s.win, off);
    uint32_t op = __shfl_xor(pos, off);
    bool oa = __shfl_xor((int)s.any_active, off);
    bool ou = __shfl_xor((int)s.any_unknown, off);
    if (ob > s.best || (ob == s.best && op < pos)) {
      s.best = ob;
      s.win = ow;
      pos = op;
    }
    s.any_active |= oa;
    s.any_unknown |= ou;
  }
}

__device__ __forceinline__ void consider_pos(const Axis &ax, Scan &s, uint32_t &pos, uint32_t j,
                                             uint32_t p, uint64_t c, uint64_t L) {
  uint8_t sj = __hip_atomic_load(&ax.state[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (sj >= ST_HIT_PENDING) return;
  double d = deviation(c, L, ax.cen[j], ax.len[j], ax.len_ratio, ax.pos_ratio);
  if (!(d > 0)) return;
  if (sj == ST_ACTIVE) {
    s.any_active = true;
    if (d > s.best || (d == s.best && p < pos)) {  // lanes scan out of order: keep earliest
      s.best = d;
      s.win = j;
      pos = p;
    }
  } else {
    s.any_unknown = true;
  }
}

__global__ void __launch_bounds__(256) k_sweep_wave(Axis ax, const uint32_t *work,
                                                    const uint32_t *nwork_ptr, uint32_t *next_work,
                                                    uint32_t *next_count) {
  const uint32_t nwork = *nwork_ptr;
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < nwork;
       w += (gridDim.x * blockDim.x) >> 6) {
    const uint32_t bin = work[w];
    const uint32_t beg = ax.off[bin], end = ax.off[bin + 1];
    bool pending = false;
    for (uint32_t t = beg; t < end; ++t) {
      const uint32_t i = ax.ent[t];
      const uint8_t st = __hip_atomic_load(&ax.state[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (st == ST_ACTIVE || st == ST_HIT) continue;
      const uint64_t c = ax.cen[i], L = ax.len[i];
      Scan s{0.0, NONE, false, false};
      uint32_t pos = 0xFFFFFFFFu;
      // own bucket newest first: scan position p = t-1-q
      for (uint32_t q0 = beg; q0 < t; q0 += 64) {
        uint32_t q = q0 + lane;
        if (q < t) consider_pos(ax, s, pos, ax.ent[q], t - 1 - q, c, L);
      }
      const uint32_t nb = neighbour_bin(bin, c, ax.max_index);
      if (nb != NONE) {
        const uint32_t nbeg = ax.off[nb], nend = ax.off[nb + 1];
        const uint32_t own = t - beg;
        for (uint32_t q0 = nbeg; q0 < nend; q0 += 64) {
          uint32_t q = q0 + lane;
          if (q < nend) {
            uint32_t j = ax.ent[q];
            if (j < i) consider_pos(ax, s, pos, j, own + (nend - 1 - q), c, L);
          }
        }
      }
      wave_combine(s, pos);
      uint8_t ns;
      if (s.any_unknown) ns = s.any_active ? ST_HIT_PENDING : ST_UNKNOWN;
      else ns = s.any_active ? ST_HIT : ST_ACTIVE;
      if (lane == 0) {
        if (ns == ST_HIT) ax.win[i] = s.win;
        if (ns != st) __hip_atomic_store(&ax.state[i], ns, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      pending |= ns == ST_UNKNOWN || ns == ST_HIT_PENDING;
    }
    if (pending && lane == 0) next_work[atomicAdd(next_count, 1u)] = bin;
  }
}

}  // namespace

void occupancy_sweep(const Axis &ax, const uint32_t *work, uint32_t nwork, uint32_t *next_work,
                     uint32_t *next_count, uint32_t *big_work, uint32_t *big_count,
                     hipStream_t st) {
  if (!nwork) return;
  (void)hipMemsetAsync(big_count, 0, sizeof(uint32_t), st);
  k_sweep_lane<<<(nwork + 255) / 256, 256, 0, st>>>(ax, work, nwork, next_work, next_count,
                                                     big_work, big_count);
  // big buckets: one wavefront each (grid sized for the upper bound)
  uint32_t max_big = nwork;
  unsigned blocks = (unsigned)((max_big + 3) / 4);
  if (blocks > 4096) blocks = 4096;
  k_sweep_wave<<<blocks, 256, 0, st>>>(ax, big_work, big_count, next_work, next_count);
}

}  // namespace rk
