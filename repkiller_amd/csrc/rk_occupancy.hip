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
// Each sweep walks every run in processing order (the short runs of a
// 64-position window by one wavefront, k_sweep_tile; each run longer than
// LONG_RUN by a wavefront of its own, k_sweep_wave), deciding an entry when the
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
#include <algorithm>
#include <cstdio>
#include <cstdlib>

namespace rk {
namespace {

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

// "deviation > 0" without the two divisions.  For a double a >= 0 (an exactly
// converted integer) and a double b > 0, fl(a/b) > 1 exactly when a > b and
// fl(a/b) == 1 exactly when a == b: two doubles that differ have a quotient at
// least 2^-53 (relative) away from 1, which never rounds to 1.  So with
// bl = fl(L*lr): sl < 0 <=> (double)dl > bl and sl == 0 <=> (double)dl == bl,
// likewise for sp, and d = 0.4*sl + 0.6*sp > 0 <=> sl >= 0, sp >= 0 and not
// both zero.  A zero query length or a NaN ratio makes every reference
// quotient inf/NaN, and such a query never matches.
struct Query {
  uint64_t c, L;
  uint64_t tl, tc;  // floor(bl), floor(bc) when both are < 2^53 (`fast`)
  double bl, bc;
  bool ok, fast, eq;  // eq: bl and bc are both integral
};
__device__ __forceinline__ Query make_query(uint64_t c, uint64_t L, double lr, double pr) {
  Query q;
  q.c = c;
  q.L = L;
  q.bl = (double)L * lr;
  q.bc = (double)L * pr;
  q.ok = L != 0 && q.bl == q.bl && q.bc == q.bc;
  // below 2^53 every integer converts exactly: (double)d <= b <=> d <= floor(b)
  q.fast = q.bl < 9007199254740992.0 && q.bc < 9007199254740992.0;
  q.tl = q.fast ? (uint64_t)q.bl : 0;
  q.tc = q.fast ? (uint64_t)q.bc : 0;
  q.eq = q.fast && (double)q.tl == q.bl && (double)q.tc == q.bc;
  return q;
}
__device__ __forceinline__ bool matches(const Query &q, uint64_t oc, uint64_t oL) {
  const uint64_t dl = q.L > oL ? q.L - oL : oL - q.L;
  const uint64_t dc = q.c > oc ? q.c - oc : oc - q.c;
  if (q.fast) return q.ok && dl <= q.tl && dc <= q.tc && !(q.eq && dl == q.tl && dc == q.tc);
  const double al = (double)dl, ac = (double)dc;
  return q.ok && al <= q.bl && ac <= q.bc && !(al == q.bl && ac == q.bc);
}


// States only move UNKNOWN -> decided (and HIT_PENDING -> HIT), so a stale
// read of another run's state is always conservative: it can only postpone a
// decision to the next sweep, never change one.  Plain loads and stores are
// therefore enough (agent-scope sc1 byte stores are one fabric write each);
// every sweep is its own launch, which makes all states coherent between sweeps.
__device__ __forceinline__ uint8_t load_state(const uint8_t *s) { return *(const volatile uint8_t *)s; }
__device__ __forceinline__ void store_state(uint8_t *s, uint8_t v) { *s = v; }

// A final decision (ST_HIT with winner `win`, or ST_ACTIVE) of entry i
// (processing index).  X axis: the X result goes into i's Y record (winner,
// or NONE: the entry queries Y next) and a hit's parent is its X winner
// (commonFunctions.cpp:55-61).  Y axis (X misses): the parent is the Y
// winner, or i itself -- a new group (:63-76).
__device__ __forceinline__ void record_decision(const Axis &ax, uint32_t i, uint8_t st,
                                                uint32_t win) {
  if (ax.xres) {
    ax.xres[4 * (size_t)i + 3] = st == ST_HIT ? win : NONE;
    if (st == ST_HIT) ax.par[i] = win;
  } else {
    ax.par[i] = st == ST_HIT ? win : i;
  }
}

struct Scan {
  double best;
  uint32_t win;  // CSR position of the best ACTIVE candidate
  uint32_t pos;  // its scan-order rank (wave path only)
  bool any_active, any_unknown;
};

__device__ __forceinline__ void consider(const Axis &ax, Scan &s, uint32_t q, const Query &qy) {
  const uint8_t sj = load_state(&ax.state[q]);
  if (sj >= ST_HIT_PENDING) return;  // not in the list
  const uint64_t oc = ax.cen[q], oL = ax.len[q];
  if (!matches(qy, oc, oL)) return;
  if (sj == ST_ACTIVE) {
    s.any_active = true;
    const double d = deviation(qy.c, qy.L, oc, oL, ax.len_ratio, ax.pos_ratio);
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

// bounds of the run holding key +-1 adjacent to [beg, end) on side `dir`:
// one lookup each in the per-position run tables (rlen_at at run starts,
// rbeg_at at run ends) instead of a walk over the neighbour's keys
__device__ __forceinline__ bool neighbour_run(const Axis &ax, uint32_t beg, uint32_t end,
                                              uint32_t key, int dir, uint32_t &nb,
                                              uint32_t &ne) {
  if (dir < 0) {
    if (beg == 0 || ax.key[beg - 1] != key - 1) return false;
    ne = beg;
    nb = ax.rbeg_at[beg - 1];
    return true;
  }
  if (end >= ax.m || ax.key[end] != key + 1) return false;
  nb = end;
  ne = end + ax.rlen_at[end];
  return true;
}


// pending-run counters are spread over PEND_WORDS words (one hot word
// serialises at ~88 atomics/us); the host sums them
constexpr uint32_t PEND_SLOTS = PEND_WORDS;

__device__ __forceinline__ void count_pending(uint32_t *counters, bool pending) {
  const uint64_t b = __ballot(pending);
  if ((threadIdx.x & 63) == 0 && b)
    atomicAdd(&counters[(blockIdx.x * 4 + (threadIdx.x >> 6)) % PEND_SLOTS], (uint32_t)__popcll(b));
}

// ---- one wavefront decides the short runs that start in a 64-position window
// Window w = positions [64w, 64w+64).  The wave OWNS every run of at most
// LONG_RUN entries that starts in its window, so everything it owns lies in
// [64w, 64w+128): lane l holds slot 0 (position 64w+l) and slot 1 (64w+64+l).
// Loads are coalesced, and each entry's centre/length/id sit in LDS for the
// other lanes.  Every undecided owned entry first records its candidates with
// deviation > 0 as bit masks over the 128 window positions: earlier entries
// of its own run, and the entries inserted before it of the neighbour run when
// that run is owned by the wave too.  A neighbour run owned elsewhere (an
// earlier window's run, a later window's run, or a long run) is scanned once
// from global memory into a fixed summary.  Decisions then proceed in rounds
// of four ballots: an entry with an ACTIVE candidate has hit (it leaves the
// list); one whose candidates are all decided is final -- a hit takes the
// first strict maximum in scan order (own run newest first, then the
// neighbour run newest first), a miss becomes ACTIVE.  Rounds repeat while
// anything changes; what is still open waits for the next sweep.
constexpr uint32_t LONG_RUN = 64;  // runs longer than this take a whole wavefront each

struct M128 {
  uint64_t lo, hi;
};
__device__ __forceinline__ void set_bit(M128 &m, int u) {
  if (u < 64) m.lo |= 1ull << u;
  else m.hi |= 1ull << (u - 64);
}
__device__ __forceinline__ bool any_and(const M128 &a, const M128 &b) {
  return ((a.lo & b.lo) | (a.hi & b.hi)) != 0;
}
// highest set bit <= P (-1 if none) / lowest set bit > P (128 if none);
// P is per lane (0..127): selects, no branches (both halves are cheap)
__device__ __forceinline__ int hs_le(uint64_t s0, uint64_t s1, int P) {
  const bool up = P >= 64;
  const int p1 = (P - 64) & 63;
  const uint64_t m1 = up ? s1 & ((2ull << p1) - 1ull) : 0ull;
  const uint64_t m0 = s0 & (up ? ~0ull : (2ull << (P & 63)) - 1ull);
  return m1 ? 127 - (int)__clzll(m1) : m0 ? 63 - (int)__clzll(m0) : -1;
}
__device__ __forceinline__ int ls_gt(uint64_t s0, uint64_t s1, int P) {
  const bool up = P >= 64;
  const uint64_t m0 = up ? 0ull : s0 & ~((2ull << (P & 63)) - 1ull);
  const uint64_t m1 = up ? s1 & ~((2ull << ((P - 64) & 63)) - 1ull) : s1;
  return m0 ? (int)__builtin_ctzll(m0) : m1 ? 64 + (int)__builtin_ctzll(m1) : 128;
}

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ void __launch_bounds__(256) k_sweep_tile(Axis ax, uint8_t *wpend, uint32_t nwin,
                                                    uint32_t *counters) {
  __shared__ uint64_t s_cen[4][128], s_len[4][128];
  __shared__ uint32_t s_ent[4][128], s_key[4][128];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t w = blockIdx.x * 4 + wv;
  bool pending = false;
  if (w < nwin && wpend[w]) {
    uint64_t *cen = s_cen[wv], *len = s_len[wv];
    uint32_t *ent = s_ent[wv], *key = s_key[wv];
    const uint32_t base = w * 64, m = ax.m;
    // run starts over the 128 positions (positions >= m count as starts)
    uint64_t S[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const uint32_t p = base + 64 * s + lane;
      const uint32_t k = p < m ? ax.key[p] : NONE;
      key[64 * s + lane] = k;
      S[s] = __ballot(p >= m || p == 0 || ax.key[p - 1] != k);
    }
    // ownership: the run starts in [0, 64) and ends within LONG_RUN entries
    bool own[2];
    int rs[2], re[2];
    uint8_t st[2], st0[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int P = 64 * s + lane;
      rs[s] = hs_le(S[0], S[1], P);
      re[s] = ls_gt(S[0], S[1], P);
      own[s] = base + P < m && rs[s] >= 0 && rs[s] < 64 && re[s] - rs[s] <= (int)LONG_RUN;
      st[s] = ST_HIT;
      if (own[s]) {
        const uint32_t p = base + P;
        cen[P] = ax.cen[p];
        len[P] = ax.len[p];
        ent[P] = ax.ent[p];
        st[s] = ax.state[p];
      }
      st0[s] = st[s];
    }
    wave_sync_lds();
    // candidates (deviation > 0) of every undecided owned entry, as masks:
    // earlier entries of its own run (rown), entries of an owned neighbour
    // run inserted before it (rnb, a prefix: ids ascend inside a run); a
    // foreign neighbour run is scanned once from global memory into fs
    M128 rown[2], rnb[2];
    Query qy[2];
    Scan fs[2];
    uint32_t fwin_ent[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      rown[s] = rnb[s] = M128{0, 0};
      fs[s] = Scan{0.0, NONE, 0, false, false};
      fwin_ent[s] = NONE;
      if (!own[s] || (st[s] != ST_UNKNOWN && st[s] != ST_HIT_PENDING)) continue;
      const int P = 64 * s + lane;
      const uint64_t c = cen[P], L = len[P];
      const uint32_t i = ent[P], k = key[P];
      qy[s] = make_query(c, L, ax.len_ratio, ax.pos_ratio);
      for (int u = rs[s]; u < P; ++u)
        if (matches(qy[s], cen[u], len[u])) set_bit(rown[s], u);
      const int dir = neighbour_dir(c, ax.max_index);
      if (!dir) continue;
      uint32_t gb = 0, ge = 0;
      bool foreign = false;
      int nb = -1, ne = -1;
      if (dir < 0) {
        const int q = rs[s] - 1;
        if (q >= 0) {
          if (key[q] == k - 1) {
            const int b2 = hs_le(S[0], S[1], q);
            if (b2 >= 0) nb = b2, ne = rs[s];
            else foreign = true, ge = base + rs[s], gb = ax.rbeg_at[ge - 1];
          }
        } else if (base > 0 && ax.key[base - 1] == k - 1) {
          foreign = true, ge = base, gb = ax.rbeg_at[base - 1];
        }
      } else {
        const int q = re[s];
        const uint32_t gq = base + q;
        if (gq < m) {
          const uint32_t kq = q < 128 ? key[q] : ax.key[gq];
          if (kq == k + 1) {
            const int e2 = q < 127 ? ls_gt(S[0], S[1], q) : 128;
            if (q < 64 && e2 - q <= (int)LONG_RUN && e2 < 128) nb = q, ne = e2;
            else foreign = true, gb = gq, ge = gq + ax.rlen_at[gq];
          }
        }
      }
      if (nb >= 0) {
        for (int u = nb; u < ne && ent[u] < i; ++u)
          if (matches(qy[s], cen[u], len[u])) set_bit(rnb[s], u);
      } else if (foreign) {
        for (uint32_t q = ge; q-- > gb;)  // newest first, only entries inserted before i
          if (ax.ent[q] < i) consider(ax, fs[s], q, qy[s]);
        if (fs[s].win != NONE) fwin_ent[s] = ax.ent[fs[s].win];
      }
    }
    // rounds of ballots: an ACTIVE candidate means a hit; an UNKNOWN one
    // blocks the final decision (it may still become ACTIVE and win)
    // (the round structure of sweep_window32 below)
    for (;;) {
      const M128 A{__ballot(own[0] && st[0] == ST_ACTIVE), __ballot(own[1] && st[1] == ST_ACTIVE)};
      const M128 U{__ballot(own[0] && st[0] == ST_UNKNOWN), __ballot(own[1] && st[1] == ST_UNKNOWN)};
      bool changed = false;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if (!own[s] || st[s] != ST_UNKNOWN) continue;
        const bool has_act = any_and(rown[s], A) || any_and(rnb[s], A) || fs[s].any_active;
        const bool has_unk = any_and(rown[s], U) || any_and(rnb[s], U) || fs[s].any_unknown;
        if (has_act) st[s] = ST_HIT_PENDING, changed = true;
        else if (!has_unk) st[s] = ST_ACTIVE, changed = true;
      }
      const M128 V{__ballot(own[0] && st[0] == ST_UNKNOWN), __ballot(own[1] && st[1] == ST_UNKNOWN)};
      bool left = false;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if (!own[s]) continue;
        if (st[s] == ST_HIT_PENDING && !any_and(rown[s], V) && !any_and(rnb[s], V) &&
            !fs[s].any_unknown)
          st[s] = ST_HIT, changed = true;
        left |= st[s] == ST_UNKNOWN || st[s] == ST_HIT_PENDING;
      }
      if (!__ballot(changed) || !__ballot(left)) break;
    }
    const M128 A{__ballot(own[0] && st[0] == ST_ACTIVE), __ballot(own[1] && st[1] == ST_ACTIVE)};
    // winners (the matching ACTIVE candidates in scan order) and write-back
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (!own[s]) continue;
      pending |= st[s] == ST_UNKNOWN || st[s] == ST_HIT_PENDING;
      if (st[s] == st0[s]) continue;
      const int P = 64 * s + lane;
      const uint32_t p = base + P;
      if (st[s] == ST_HIT) {
        const uint64_t c = cen[P], L = len[P];
        double best = 0.0;
        uint32_t win = NONE;
#pragma unroll
        for (int part = 0; part < 2; ++part) {  // own run newest first, then the neighbour's
          const M128 r = part ? rnb[s] : rown[s];
          uint64_t b[2] = {A.lo & r.lo, A.hi & r.hi};
          for (int half = 1; half >= 0; --half) {
            while (b[half]) {
              const int v = 63 - __clzll(b[half]);
              b[half] &= ~(1ull << v);
              const int u = v + 64 * half;
              const double d = deviation(c, L, cen[u], len[u], ax.len_ratio, ax.pos_ratio);
              if (d > best) best = d, win = ent[u];
            }
          }
        }
        if (fs[s].any_active && fs[s].best > best) best = fs[s].best, win = fwin_ent[s];
        record_decision(ax, ent[P], ST_HIT, win);
      } else if (st[s] == ST_ACTIVE) {
        record_decision(ax, ent[P], ST_ACTIVE, NONE);
      }
      store_state(&ax.state[p], st[s]);
    }
    const bool wp = __ballot(pending) != 0;
    if (lane == 0) wpend[w] = wp;
  }
  count_pending(counters, pending);
}

// 64 bits of a 128-bit window mask starting at bit a (0 <= a < 128)
// m << a as a 128-bit window mask (0 <= a < 128); selects, no branches
__device__ __forceinline__ M128 shl128(uint64_t m, int a) {
  const int b = a & 63;
  const uint64_t sh = m << b, carry = b ? m >> (64 - b) : 0ull;
  return a >= 64 ? M128{0ull, sh} : M128{sh, carry};
}
__device__ __forceinline__ uint64_t bits_from(uint64_t lo, uint64_t hi, int a) {
  const int b = a & 63;
  const uint64_t hs = hi >> b, ls = b ? (lo >> b) | (hi << (64 - b)) : lo;
  return a >= 64 ? hs : ls;
}

// ---- 32-bit fast path of the window sweep --------------------------------
// When every length is below 2^31 (checked once per call in k_prep_keys), the
// length difference of two entries fits 31 bits and the centre difference of
// two entries in the same or adjacent 100-bp buckets is below 200, so the
// candidate test and the deviation run on 32-bit operands (the values, and
// therefore every f64 result, are identical).  Thresholds saturate at 2^32-1,
// which no 31-bit difference reaches.
struct Q32 {
  uint32_t c, L, tl, tc;
  bool ok, eq;
};
__device__ __forceinline__ Q32 make_q32(uint32_t c, uint32_t L, double lr, double pr) {
  Q32 q;
  const double bl = (double)L * lr, bc = (double)L * pr;
  q.c = c;
  q.L = L;
  q.ok = L != 0 && bl == bl && bc == bc;
  q.tl = bl >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)bl;
  q.tc = bc >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)bc;
  q.eq = (double)q.tl == bl && (double)q.tc == bc;
  return q;
}
__device__ __forceinline__ void diffs32(const Q32 &q, uint2 o, uint32_t &dl, uint32_t &dc) {
  dl = q.L > o.y ? q.L - o.y : o.y - q.L;
  const int32_t d = (int32_t)(q.c - o.x);
  dc = (uint32_t)(d < 0 ? -d : d);
}
// (bitwise, not short-circuit: the `&&` form compiled to a branch around the
// centre test of every candidate)
__device__ __forceinline__ bool m32(const Q32 &q, uint2 o) {
  uint32_t dl, dc;
  diffs32(q, o, dl, dc);
  const bool at_both = (dl == q.tl) & (dc == q.tc);
  return q.ok & (dl <= q.tl) & (dc <= q.tc) & !(q.eq & at_both);
}
// deviation (SequenceOcupationList.cpp:20-31) from the same integer operands
__device__ __forceinline__ double dev32(const Q32 &q, uint2 o, double lr, double pr) {
  uint32_t dl, dc;
  diffs32(q, o, dl, dc);
  const double sl = -fabs((double)dl / ((double)q.L * lr)) + 1.0;
  if (sl < 0) return 0.0;
  const double sp = -fabs((double)dc / ((double)q.L * pr)) + 1.0;
  if (sp < 0) return 0.0;
  return sl * 0.4 + sp * 0.6;
}

// A neighbour run owned elsewhere, scanned from global memory from g0 in
// direction `step` while the key is `want` (no run-table lookup; key, id,
// state and packed record of an entry are loaded together); only entries
// inserted before i count.  Ties go to the higher position (newest first, the
// reference's scan order).  fs.win receives the winner's id.  The packed
// 32-bit records suffice: lengths are < 2^31 and a centre in an adjacent
// bucket differs by less than 200.
__device__ __forceinline__ void foreign_scan32(const Axis &ax, uint32_t g0, int step,
                                               uint32_t want, uint32_t i, const Q32 &q, Scan &fs) {
  uint32_t bestpos = 0;
  for (uint32_t g = g0;; g += step) {
    if (step < 0 ? g == NONE : g >= ax.m) return;
    const uint32_t kg = ax.key[g], eg = ax.ent[g];
    const uint8_t sg = load_state(&ax.state[g]);
    const uint2 o = ax.pk[g];
    if (kg != want) return;
    if (eg >= i || sg >= ST_HIT_PENDING || !m32(q, o)) continue;
    if (sg != ST_ACTIVE) {
      // an undecided candidate: this query cannot be final in this sweep, and
      // HIT_PENDING needs only one ACTIVE candidate, so the rest of the run
      // (a long run of hundreds in the first sweep) need not be read now
      fs.any_unknown = true;
      return;
    }
    const double d = dev32(q, o, ax.len_ratio, ax.pos_ratio);
    if (!fs.any_active || d > fs.best || (d == fs.best && g > bestpos))
      fs.best = d, fs.win = eg, bestpos = g;
    fs.any_active = true;
  }
}

#ifndef RK_OWN_U
#define RK_OWN_U 4
#endif
constexpr int OWN_U = RK_OWN_U;
#ifdef RK_SWEEP_PROF
// measurement build only: per-phase shader cycles of the first window sweep,
// sampled over every 64th window (the atomics of every window slowed the
// memory phases they were timing)
__device__ unsigned long long g_sweep_prof[16];
#define SP_T(k) const uint64_t _t##k = __builtin_amdgcn_s_memtime()
#define SP_ADD(slot, v) do { if (lflag && lane == 0 && (w & 63) == 0) atomicAdd(&g_sweep_prof[slot], (unsigned long long)(v)); } while (0)
#else
#define SP_T(k)
#define SP_ADD(slot, v)
#endif
// Window masks (bit P = window position P, two 64-bit words) of a per-lane
// predicate.  NSLOT == 2: lane l holds positions l (slot 0) and 64 + l (slot
// 1).  NSLOT == 1: lanes below t hold positions 64 + lane -- the tail of the
// window's last run --, the others position `lane` (t <= the first run start
// f of the window, and lanes [t, f) own nothing, so no position is doubled).
template <int NSLOT>
__device__ __forceinline__ void win_ballot(bool c0, bool c1, uint64_t lowt, uint64_t &lo,
                                           uint64_t &hi) {
  if (NSLOT == 2) {
    lo = __ballot(c0);
    hi = __ballot(c1);
  } else {
    const uint64_t b = __ballot(c0);
    lo = b & ~lowt;
    hi = b & lowt;
  }
}

// One window (64 positions) of the 32-bit sweep; LDS scratch of the calling
// wavefront in pk / ent / key; the window's keys are already in `key` and its
// run starts in S0 / S1.  Returns (wave-uniformly) whether the window still
// owns undecided entries, and records that in wpend[w].  NSLOT == 1 serves
// the windows whose last run's tail fits in the lanes before the first run
// start (most windows): every slot's code runs once instead of twice.
template <int NSLOT, bool PAR>
__device__ __forceinline__ bool sweep_core32(const Axis &ax, uint32_t w, uint8_t *wpend,
                                             uint8_t *lflag, uint8_t *rpend, uint2 *pk,
                                             uint32_t *ent, uint32_t *key, double *dev,
                                             int lane, uint64_t S0, uint64_t S1,
                                             int t, uint2 pk0, uint32_t ent0, uint8_t st00,
                                             uint8_t nd00, uint2 pk1, uint32_t ent1, uint8_t st01,
                                             uint8_t nd01) {
  bool pending = false;
  SP_T(0);
  {
    const uint32_t base = w * 64, m = ax.m;
    const uint64_t lowt = NSLOT == 1 ? (1ull << t) - 1ull : 0ull;  // t < 64 here
    int P[2];
    bool own[2];
    int rs[2];
    uint8_t st[2], st0[2], nd[2];
#pragma unroll
    for (int s = 0; s < NSLOT; ++s) {
      P[s] = NSLOT == 2 ? 64 * s + lane : (lane < t ? 64 + lane : lane);
      rs[s] = hs_le(S0, S1, P[s]);
      const int re = ls_gt(S0, S1, P[s]);
      own[s] = base + P[s] < m && rs[s] >= 0 && rs[s] < 64 && re - rs[s] <= (int)LONG_RUN;
      if (s == 0 && lflag) {  // first sweep: flag a long run that starts here
        const bool lng = base + P[s] < m && rs[0] == P[s] && re - P[s] > (int)LONG_RUN;
        const uint64_t bb = __ballot(lng);
        if (lane == 0) lflag[w] = bb != 0;
        if (lng) rpend[base + P[s]] = 1;  // the long-run kernel's "still open" flag
      }
      st[s] = ST_HIT;
      nd[s] = 0;
      if (own[s]) {
        // both slots' records came with the keys (lane l: positions l and 64 + l)
        if (P[s] < 64) {
          pk[P[s]] = pk0, ent[P[s]] = ent0, st[s] = st00, nd[s] = nd00;
        } else {
          pk[P[s]] = pk1, ent[P[s]] = ent1, st[s] = st01, nd[s] = nd01;
        }
      }
      st0[s] = st[s];
    }
    wave_sync_lds();
    SP_T(1);
    // matching candidates: own run (bit j = entry rs + j), owned neighbour run
    // (bit j = entry nbs + j); a foreign neighbour run is summarised in fs
    uint64_t rown[2], rnb[2];
    int nbs[2];
    Scan fs[2];
    Q32 qs[2];
    bool open[2];
#pragma unroll
    for (int s = 0; s < NSLOT; ++s) {
      rown[s] = rnb[s] = 0;
      nbs[s] = 0;
      fs[s] = Scan{0.0, NONE, 0, false, false};
      open[s] = own[s] && (st[s] == ST_UNKNOWN || st[s] == ST_HIT_PENDING);
      if (!open[s]) continue;
      const uint2 me = pk[P[s]];
      const Q32 q = make_q32(me.x, me.y, ax.len_ratio, ax.pos_ratio);
      qs[s] = q;
      const int n = P[s] - rs[s];
      // OWN_U independent LDS reads per step (pk is padded past position 127)
      for (int j = 0; j < n; j += OWN_U) {
        uint2 o[OWN_U];
#pragma unroll
        for (int u = 0; u < OWN_U; ++u) o[u] = pk[rs[s] + j + u];
        uint64_t b4 = 0;
#pragma unroll
        for (int u = 0; u < OWN_U; ++u) b4 |= (uint64_t)m32(q, o[u]) << u;
        if (n - j < OWN_U) b4 &= (1ull << (n - j)) - 1ull;
        rown[s] |= b4 << j;
      }
    }
    SP_T(2);
#ifdef RK_SWEEP_PROF
    uint32_t nbl = 0, nfor = 0;  // neighbour-run entries in LDS / foreign scans of this lane
    uint64_t fcyc = 0;           // cycles the wavefront spent in foreign scans
#endif
#pragma unroll
    for (int s = 0; s < NSLOT; ++s) {
      if (!open[s] || !nd[s]) continue;
      const Q32 q = qs[s];
      const int dir = nd[s] == 1 ? -1 : 1;
      const uint32_t i = ent[P[s]], k = key[P[s]];
      uint32_t g0 = 0;  // first position of a foreign neighbour scan
      bool foreign = false;
      int nb = -1, ne = -1;
      if (dir < 0) {
        const int q2 = rs[s] - 1;
        if (q2 >= 0) {
          if (key[q2] == k - 1) {
            const int b2 = hs_le(S0, S1, q2);
            if (b2 >= 0) nb = b2, ne = rs[s];
            else foreign = true, g0 = base + q2;
          }
        } else if (base > 0) {
          foreign = true, g0 = base - 1;  // the key test happens in the scan
        }
      } else {
        const int q2 = ls_gt(S0, S1, P[s]);
        const uint32_t gq = base + q2;
        if (gq < m) {
          const uint32_t kq = q2 < 128 ? key[q2] : k + 1;  // q2 == 128: tested in the scan
          if (kq == k + 1) {
            const int e2 = q2 < 127 ? ls_gt(S0, S1, q2) : 128;
            if (q2 < 64 && e2 - q2 <= (int)LONG_RUN && e2 < 128) nb = q2, ne = e2;
            else foreign = true, g0 = gq;
          }
        }
      }
      if (nb >= 0) {
        nbs[s] = nb;
#ifdef RK_SWEEP_PROF
        nbl += ne - nb;
#endif
        for (int u = nb; u < ne && ent[u] < i; ++u) rnb[s] |= (uint64_t)m32(q, pk[u]) << (u - nb);
      } else if (foreign) {
#ifdef RK_SWEEP_PROF
        ++nfor;
#endif
#ifdef RK_SWEEP_PROF
        const uint64_t _f0 = __builtin_amdgcn_s_memtime();
#endif
        foreign_scan32(ax, g0, dir, k + dir, i, q, fs[s]);
#ifdef RK_SWEEP_PROF
        fcyc += __builtin_amdgcn_s_memtime() - _f0;
#endif
      }
    }
    // all candidates of a slot as one mask in window positions, so a round
    // is two ANDs per ballot word
    M128 cm[2];
#pragma unroll
    for (int s = 0; s < NSLOT; ++s) {
      const M128 o = shl128(rown[s], rs[s]), q = shl128(rnb[s], nbs[s]);
      cm[s] = M128{o.lo | q.lo, o.hi | q.hi};
    }
    // rounds of ballots: a matching ACTIVE candidate means a hit; a matching
    // UNKNOWN one blocks the final decision (it may still become ACTIVE and win)
    // A round: UNKNOWN entries with an ACTIVE candidate become HIT_PENDING and
    // those with only decided, inactive candidates ACTIVE; then, against the
    // UNKNOWN set left after that, pending hits whose candidates are all
    // decided become final.  Rounds stop when nothing changes or nothing is
    // left open.
    SP_T(3);
#define RK_SLOT_IS(s, v) ((s) < NSLOT && own[(s) < NSLOT ? (s) : 0] && st[(s) < NSLOT ? (s) : 0] == (v))
    uint64_t A0, A1;
#ifdef RK_SWEEP_PROF
    uint32_t nrounds = 0;
#endif
    for (;;) {
#ifdef RK_SWEEP_PROF
      ++nrounds;
#endif
      uint64_t U0, U1;
      win_ballot<NSLOT>(RK_SLOT_IS(0, ST_ACTIVE), RK_SLOT_IS(1, ST_ACTIVE), lowt, A0, A1);
      win_ballot<NSLOT>(RK_SLOT_IS(0, ST_UNKNOWN), RK_SLOT_IS(1, ST_UNKNOWN), lowt, U0, U1);
      bool changed = false;
#pragma unroll
      for (int s = 0; s < NSLOT; ++s) {
        if (!own[s] || st[s] != ST_UNKNOWN) continue;
        const bool has_act = ((A0 & cm[s].lo) | (A1 & cm[s].hi)) != 0 || fs[s].any_active;
        const bool has_unk = ((U0 & cm[s].lo) | (U1 & cm[s].hi)) != 0 || fs[s].any_unknown;
        if (has_act) st[s] = ST_HIT_PENDING, changed = true;
        else if (!has_unk) st[s] = ST_ACTIVE, changed = true;
      }
      uint64_t V0, V1;
      win_ballot<NSLOT>(RK_SLOT_IS(0, ST_UNKNOWN), RK_SLOT_IS(1, ST_UNKNOWN), lowt, V0, V1);
      bool left = false;
#pragma unroll
      for (int s = 0; s < NSLOT; ++s) {
        if (!own[s]) continue;
        if (st[s] == ST_HIT_PENDING && ((V0 & cm[s].lo) | (V1 & cm[s].hi)) == 0 &&
            !fs[s].any_unknown)
          st[s] = ST_HIT, changed = true;
        left |= st[s] == ST_UNKNOWN || st[s] == ST_HIT_PENDING;
      }
      if (!__ballot(changed) || !__ballot(left)) break;
    }
    SP_T(4);
    win_ballot<NSLOT>(RK_SLOT_IS(0, ST_ACTIVE), RK_SLOT_IS(1, ST_ACTIVE), lowt, A0, A1);
#undef RK_SLOT_IS
    // winners: the first strict maximum in scan order among the matching
    // ACTIVE candidates (own run newest first, then the neighbour run); a
    // single candidate needs no deviation
#ifdef RK_SWEEP_PROF
    uint32_t ndev = 0;  // deviations computed by this lane
#endif
    bool multi[2] = {false, false};
    uint64_t aov[2] = {0, 0}, anv[2] = {0, 0};
    uint32_t winv[2] = {NONE, NONE};
    double bestv[2] = {0.0, 0.0};
#pragma unroll
    for (int s = 0; s < NSLOT; ++s) {
      if (!own[s]) continue;
      pending |= st[s] == ST_UNKNOWN || st[s] == ST_HIT_PENDING;
      if (st[s] == st0[s] || st[s] != ST_HIT) continue;
      const uint64_t ao = bits_from(A0, A1, rs[s]) & rown[s];
      const uint64_t an = rnb[s] ? bits_from(A0, A1, nbs[s]) & rnb[s] : 0;
      if (__popcll(ao) + __popcll(an) + (fs[s].any_active ? 1 : 0) == 1) {
        winv[s] = ao ? ent[rs[s] + 63 - __clzll(ao)]
                     : an ? ent[nbs[s] + 63 - __clzll(an)] : fs[s].win;
      } else {
        multi[s] = true;
        aov[s] = ao;
        anv[s] = an;
      }
    }
    // deviations of the lanes with several candidates: lane-parallel over all
    // (query, candidate) pairs of the wavefront when some lane has three or
    // more (a serial loop would run to the longest list), serial otherwise
    const uint32_t c0 = multi[0] ? __popcll(aov[0]) + __popcll(anv[0]) : 0u;
    const uint32_t c1 = NSLOT == 2 && multi[1 % NSLOT] ? __popcll(aov[1 % NSLOT]) + __popcll(anv[1 % NSLOT]) : 0u;
    const uint32_t ct = c0 + c1;
#ifdef RK_SWEEP_PROF
    ndev = ct;
#endif
    uint32_t cmax = ct;
    for (int off = 32; off > 0; off >>= 1) {
      const uint32_t o = __shfl_xor(cmax, off);
      cmax = o > cmax ? o : cmax;
    }
#ifndef RK_DEV_PAR_MIN
#define RK_DEV_PAR_MIN 3
#endif
    if (PAR && cmax >= RK_DEV_PAR_MIN) {
      const uint32_t incl = wave_incl_scan(ct);  // inclusive prefix of the pair counts
      const uint32_t start = incl - ct, T = __builtin_amdgcn_readlane(incl, 63);
      uint32_t *owner_at = key;  // the keys are done with (64 words used)
      for (uint32_t cb = 0; cb < T; cb += 64) {
        // owners mark their pairs inside this chunk
        {
          const uint32_t j0 = start > cb ? start : cb, j1e = start + ct, j1 = j1e < cb + 64 ? j1e : cb + 64;
          for (uint32_t j = j0; j < j1; ++j) owner_at[j - cb] = lane;
        }
        wave_sync_lds();
        const uint32_t i = cb + lane;
        const bool live = i < T;
        const uint32_t o = live ? owner_at[lane] : 0u;
        // the owner's lists, pulled from its lane (every lane takes part)
        const uint32_t so = __shfl(start, (int)o), c0o = __shfl(c0, (int)o);
        const uint32_t k = i - so;
        const bool second = NSLOT == 2 && k >= c0o;
        const uint32_t kk = second ? k - c0o : k;
        uint64_t ao = 0, an = 0;
        int rso = 0, nbo = 0, Po = 0;
#pragma unroll
        for (int s = 0; s < NSLOT; ++s) {
          const uint64_t a = (uint64_t)(uint32_t)__shfl((int)(uint32_t)aov[s], (int)o) |
                             (uint64_t)(uint32_t)__shfl((int)(uint32_t)(aov[s] >> 32), (int)o) << 32;
          const uint64_t n = (uint64_t)(uint32_t)__shfl((int)(uint32_t)anv[s], (int)o) |
                             (uint64_t)(uint32_t)__shfl((int)(uint32_t)(anv[s] >> 32), (int)o) << 32;
          const int r = __shfl(rs[s], (int)o), nb = __shfl(nbs[s], (int)o), pp = __shfl(P[s], (int)o);
          if (s == (second ? 1 : 0)) ao = a, an = n, rso = r, nbo = nb, Po = pp;
        }
        // the kk-th candidate in scan order: the (kk)-th highest bit of ao, then of an
        const uint32_t na = __popcll(ao);
        const bool in_own = kk < na;
        uint64_t msk = in_own ? ao : an;
        uint32_t r = (uint32_t)__popcll(msk) - 1u - (in_own ? kk : kk - na);  // rank from the bottom
        int bpos = 0;
#pragma unroll
        for (int wdt = 32; wdt > 0; wdt >>= 1) {
          const uint32_t lowc = __popcll(msk & ((1ull << wdt) - 1ull));
          if (r >= lowc) {
            r -= lowc;
            msk >>= wdt;
            bpos += wdt;
          }
        }
        const int cpos = (in_own ? rso : nbo) + bpos;
        double d = 0.0;
        if (live) {
          const uint2 qp = pk[Po];
          const Q32 q = make_q32(qp.x, qp.y, ax.len_ratio, ax.pos_ratio);
          d = dev32(q, pk[cpos], ax.len_ratio, ax.pos_ratio);
          dev[lane] = d;
          owner_at[64 + lane] = ent[cpos];  // the candidate's id
        }
        wave_sync_lds();
        // every owner takes its pairs of this chunk in scan order, four per
        // step (independent LDS reads; the longest list sets the pace)
        {
          const uint32_t j0 = start > cb ? start : cb, j1e = start + ct, j1 = j1e < cb + 64 ? j1e : cb + 64;
          for (uint32_t j = j0; j < j1; j += 4) {
            double dj[4];
            uint32_t ej[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const uint32_t x = (j + u < j1 ? j + u : j0) - cb;
              dj[u] = dev[x];
              ej[u] = owner_at[64 + x];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              if (j + u >= j1) break;
              const uint32_t kj = j + u - start;
              if (NSLOT == 2 && kj >= c0) {
                if (dj[u] > bestv[1 % NSLOT]) bestv[1 % NSLOT] = dj[u], winv[1 % NSLOT] = ej[u];
              } else {
                if (dj[u] > bestv[0]) bestv[0] = dj[u], winv[0] = ej[u];
              }
            }
          }
        }
        wave_sync_lds();
      }
    } else {
#pragma unroll
      for (int s = 0; s < NSLOT; ++s) {
        if (!multi[s]) continue;
        const Q32 q = make_q32(pk[P[s]].x, pk[P[s]].y, ax.len_ratio, ax.pos_ratio);
        uint64_t b = aov[s];
        while (b) {
          const int v = 63 - __clzll(b);
          b &= ~(1ull << v);
          const double d = dev32(q, pk[rs[s] + v], ax.len_ratio, ax.pos_ratio);
          if (d > bestv[s]) bestv[s] = d, winv[s] = ent[rs[s] + v];
        }
        b = anv[s];
        while (b) {
          const int v = 63 - __clzll(b);
          b &= ~(1ull << v);
          const double d = dev32(q, pk[nbs[s] + v], ax.len_ratio, ax.pos_ratio);
          if (d > bestv[s]) bestv[s] = d, winv[s] = ent[nbs[s] + v];
        }
      }
    }
    SP_T(45);
#pragma unroll
    for (int s = 0; s < NSLOT; ++s) {
      if (!own[s] || st[s] == st0[s]) continue;
      if (st[s] == ST_HIT) {
        uint32_t win = winv[s];
        if (multi[s] && fs[s].any_active && fs[s].best > bestv[s]) win = fs[s].win;
        record_decision(ax, ent[P[s]], ST_HIT, win);
      } else if (st[s] == ST_ACTIVE) {
        record_decision(ax, ent[P[s]], ST_ACTIVE, NONE);
      }
      store_state(&ax.state[base + P[s]], st[s]);
    }
    const bool wp = __ballot(pending) != 0;
    if (lane == 0) wpend[w] = wp;
#ifdef RK_SWEEP_PROF
    SP_T(5);
    const uint64_t o1 = __ballot(NSLOT == 2 && own[NSLOT - 1]);
    SP_ADD(0, _t1 - _t0);
    SP_ADD(1, _t2 - _t1);
    SP_ADD(2, _t3 - _t2);
    SP_ADD(3, _t4 - _t3);
    SP_ADD(4, _t45 - _t4);
    SP_ADD(14, _t5 - _t45);
    SP_ADD(15, __builtin_amdgcn_readfirstlane((uint32_t)fcyc));
    SP_ADD(5, nrounds);
    SP_ADD(6, 1);
    SP_ADD(7, o1 != 0);
    SP_ADD(8, NSLOT == 1);
    {
      uint32_t mx = ndev, sm = ndev;
      for (int off = 32; off > 0; off >>= 1) {
        const uint32_t o = __shfl_xor(mx, off);
        mx = o > mx ? o : mx;
        sm += __shfl_xor(sm, off);
      }
      SP_ADD(9, mx);   // the longest deviation list of a lane
      SP_ADD(10, sm);  // deviations computed
      uint32_t m2 = nbl, s2 = nbl, f2 = nfor;
      for (int off = 32; off > 0; off >>= 1) {
        const uint32_t o = __shfl_xor(m2, off);
        m2 = o > m2 ? o : m2;
        s2 += __shfl_xor(s2, off);
        f2 += __shfl_xor(f2, off);
      }
      SP_ADD(11, m2);  // the longest LDS neighbour run of a lane
      SP_ADD(12, s2);  // LDS neighbour entries tested
      SP_ADD(13, f2);  // foreign neighbour scans
    }
#endif
    return wp;
  }
}

// One window: the keys and slot-0 records in one memory round trip, the run
// starts, then the one-slot core when the last run's tail (t entries past
// position 63) fits in the lanes before the window's first run start f.
template <bool PAR>
__device__ __forceinline__ bool sweep_window32(const Axis &ax, uint32_t w, uint8_t *wpend,
                                               uint8_t *lflag, uint8_t *rpend, uint2 *pk,
                                               uint32_t *ent, uint32_t *key, double *dev,
                                               int lane) {
  const uint32_t base = w * 64, m = ax.m;
  uint64_t S0, S1;
  const uint32_t p0 = base + lane;
  uint2 pk0 = make_uint2(0, 0);
  uint32_t ent0 = 0;
  uint8_t st00 = ST_HIT, nd00 = 0;
  if (p0 < m) pk0 = ax.pk[p0], ent0 = ax.ent[p0], st00 = ax.state[p0], nd00 = ax.nbd[p0];
  // the records at 64 + lane too, in the same memory round trip: 74 % of the
  // windows own the tail of a run past position 63 (the next window's slot 0,
  // mostly served by L2)
  uint2 pk1 = make_uint2(0, 0);
  uint32_t ent1 = 0;
  uint8_t st01 = ST_HIT, nd01 = 0;
  {
    const uint32_t p1 = base + 64 + lane;
    if (p1 < m) pk1 = ax.pk[p1], ent1 = ax.ent[p1], st01 = ax.state[p1], nd01 = ax.nbd[p1];
  }
  {
    const uint32_t p1 = base + 64 + lane;
    const uint32_t k0 = p0 < m ? ax.key[p0] : NONE, k1 = p1 < m ? ax.key[p1] : NONE;
    const uint32_t q0 = p0 < m && p0 > 0 ? ax.key[p0 - 1] : NONE;
    const uint32_t q1 = p1 < m ? ax.key[p1 - 1] : NONE;
    key[lane] = k0;
    key[64 + lane] = k1;
    S0 = __ballot(p0 >= m || p0 == 0 || q0 != k0);
    S1 = __ballot(p1 >= m || q1 != k1);
  }
  // f: first run start of the window; t: how far the last run that starts in
  // the window reaches past position 63 (0 when it does not, or is long)
  const int f = S0 ? __builtin_ctzll(S0) : 64;
  int t = 0;
  if (S0) {
    const int L = 63 - __clzll(S0);
    const int re = S1 ? 64 + __builtin_ctzll(S1) : 128;
    if (re > 64 && re - L <= (int)LONG_RUN && base + L < m) t = re - 64;
  }
  if (t <= f && t < 64)
    return sweep_core32<1, PAR>(ax, w, wpend, lflag, rpend, pk, ent, key, dev, lane, S0, S1, t, pk0, ent0,
                           st00, nd00, pk1, ent1, st01, nd01);
  return sweep_core32<2, PAR>(ax, w, wpend, lflag, rpend, pk, ent, key, dev, lane, S0, S1, t, pk0, ent0,
                         st00, nd00, pk1, ent1, st01, nd01);
}

// first sweep: one wavefront per window, every window (wpend and rpend are
// written here, not read)
#ifndef RK_SWEEP_WPE
#define RK_SWEEP_WPE 8
#endif
#ifndef RK_SWEEP_WPE_PAR
#define RK_SWEEP_WPE_PAR 7  // 71 VGPRs, no spills (neutral against 8 waves with 44 B of scratch)
#endif
template <bool PAR>
__global__ void __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(PAR ? RK_SWEEP_WPE_PAR : RK_SWEEP_WPE)))
k_sweep_fast(Axis ax, uint8_t *wpend, uint32_t nwin, uint32_t *counters, uint8_t *lflag,
             uint8_t *rpend) {
  __shared__ uint2 s_pk[4][128 + OWN_U];  // {centre low 32 bits, length}; read padding
  __shared__ uint32_t s_ent[4][128], s_key[4][128];
  __shared__ double s_dev[4][PAR ? 64 : 1];  // the lane-parallel winner deviations
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t w = blockIdx.x * 4 + wv;
  bool pending = false;
  if (w < nwin)
    pending = sweep_window32<PAR>(ax, w, wpend, lflag, rpend, s_pk[wv], s_ent[wv], s_key[wv],
                             s_dev[wv], lane);
  count_pending(counters, pending && lane == 0);
}

// later sweeps: one wavefront per 64 windows, which reads their flags with
// one coalesced load and handles the still-pending ones in turn
template <bool PAR>
__global__ void __launch_bounds__(256) k_sweep_fast_more(Axis ax, uint8_t *wpend, uint32_t nwin, uint32_t *counters) {
  __shared__ uint2 s_pk[4][128 + OWN_U];
  __shared__ uint32_t s_ent[4][128], s_key[4][128];
  __shared__ double s_dev[4][PAR ? 64 : 1];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t g = blockIdx.x * 4 + wv, w0 = g * 64;
  bool pending = false;
  if (w0 < nwin) {
    uint64_t todo = __ballot(w0 + lane < nwin && wpend[w0 + lane]);
    while (todo) {
      const int b = __builtin_ctzll(todo);
      todo &= todo - 1;
      wave_sync_lds();  // the previous window's LDS reads are done
      pending |= sweep_window32<PAR>(ax, w0 + b, wpend, nullptr, nullptr, s_pk[wv], s_ent[wv],
                                s_key[wv], s_dev[wv], lane);
    }
  }
  count_pending(counters, pending && lane == 0);
}

// ---- one wavefront walks one long run --------------------------------------
// Entries are decided one after another (the walk is inherently ordered); the
// 64 lanes split each entry's candidate scan and combine with a wave argmax
// that keeps the reference's tie rule (earliest in scan order wins).
__device__ __forceinline__ void consider_ranked(const Axis &ax, Scan &s, uint32_t q, uint32_t p,
                                                const Query &qy) {
  const uint8_t sj = load_state(&ax.state[q]);
  if (sj >= ST_HIT_PENDING) return;
  const uint64_t oc = ax.cen[q], oL = ax.len[q];
  if (!matches(qy, oc, oL)) return;
  if (sj == ST_ACTIVE) {
    s.any_active = true;
    const double d = deviation(qy.c, qy.L, oc, oL, ax.len_ratio, ax.pos_ratio);
    if (d > s.best || (d == s.best && p < s.pos)) {
      s.best = d;
      s.win = q;
      s.pos = p;
    }
  } else {
    s.any_unknown = true;
  }
}

// the same on the packed 32-bit records (RunList::fast32)
__device__ __forceinline__ void consider_ranked32(const Axis &ax, Scan &s, uint32_t q, uint32_t p,
                                                  const Q32 &qy) {
  const uint8_t sj = load_state(&ax.state[q]);
  if (sj >= ST_HIT_PENDING) return;
  const uint2 o = ax.pk[q];
  if (!m32(qy, o)) return;
  if (sj == ST_ACTIVE) {
    s.any_active = true;
    const double d = dev32(qy, o, ax.len_ratio, ax.pos_ratio);
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

// first position >= from whose key is not `key` (or m), 64 keys per step
__device__ __forceinline__ uint32_t wave_scan_end(const Axis &ax, uint32_t from, uint32_t key,
                                                  uint32_t lane) {
  for (uint32_t b = from;; b += 64) {
    const uint32_t q = b + lane;
    const uint64_t e = __ballot(q >= ax.m || ax.key[q] != key);
    if (e) return b + __builtin_ctzll(e);
  }
}
// smallest p with key `key` on all of [p, before), 64 keys per step
__device__ __forceinline__ uint32_t wave_scan_begin(const Axis &ax, uint32_t before, uint32_t key,
                                                    uint32_t lane) {
  for (uint32_t b = before;;) {
    const uint32_t q0 = b >= 64 ? b - 64 : 0;
    const uint32_t q = q0 + lane;
    const uint64_t e = __ballot(q < b && ax.key[q] != key);
    if (e) return q0 + 64 - __clzll(e);
    if (q0 == 0) return 0;
    b = q0;
  }
}

// 64-bit lengths (k_sweep_tile's long runs): one wavefront per listed run,
// entries decided one after another; big = the starts of the runs of more
// than LONG_RUN entries (k_run_bounds), run and neighbour bounds from the run
// tables
__global__ void __launch_bounds__(256) k_sweep_wave(Axis ax, const uint32_t *big, uint32_t nbig,
                                                    uint8_t *rpend, uint32_t *counters) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < nbig;
       w += (gridDim.x * blockDim.x) >> 6) {
    const uint32_t beg = big[w];
    if (!rpend[beg]) continue;
    const uint32_t key = ax.key[beg];
    const uint32_t end = beg + ax.rlen_at[beg];
    uint32_t lo_b = 0, lo_e = 0, hi_b = 0, hi_e = 0;
    const bool has_lo = neighbour_run(ax, beg, end, key, -1, lo_b, lo_e);
    const bool has_hi = neighbour_run(ax, beg, end, key, 1, hi_b, hi_e);
    bool pending = false;
    for (uint32_t t = beg; t < end; ++t) {
      const uint8_t st = load_state(&ax.state[t]);
      if (st == ST_ACTIVE || st == ST_HIT) continue;
      const uint32_t i = ax.ent[t];
      const uint64_t c = ax.cen[t];
      const Query qy = make_query(c, ax.len[t], ax.len_ratio, ax.pos_ratio);
      const int dir = neighbour_dir(c, ax.max_index);
      Scan s{0.0, NONE, 0xFFFFFFFFu, false, false};
      for (uint32_t q0 = beg; q0 < t; q0 += 64) {  // own run, newest first: rank t-1-q
        const uint32_t q = q0 + lane;
        if (q < t) consider_ranked(ax, s, q, t - 1 - q, qy);
      }
      if ((dir < 0 && has_lo) || (dir > 0 && has_hi)) {
        const uint32_t nb = dir < 0 ? lo_b : hi_b, ne = dir < 0 ? lo_e : hi_e;
        const uint32_t own = t - beg;
        for (uint32_t q0 = nb; q0 < ne; q0 += 64) {
          const uint32_t q = q0 + lane;
          if (q < ne && ax.ent[q] < i) consider_ranked(ax, s, q, own + (ne - 1 - q), qy);
        }
      }
      wave_combine(s);
      const uint8_t ns = decide(s);
      if (lane == 0) {
        if (ns != st && (ns == ST_HIT || ns == ST_ACTIVE))
          record_decision(ax, i, ns, ns == ST_HIT ? ax.ent[s.win] : NONE);
        if (ns != st) store_state(&ax.state[t], ns);
      }
      pending |= ns == ST_UNKNOWN || ns == ST_HIT_PENDING;
    }
    if (lane == 0) {
      rpend[beg] = pending;
      if (pending) atomicAdd(&counters[w % PEND_SLOTS], 1u);
    }
  }
}

// ---- long runs on the 32-bit records: 64 entries at a time -----------------
// k_sweep_wave decides a long run's entries one after another, each with a
// wave-wide scan of every earlier entry: O(run^2 / 64) dependent steps, which
// dominates repeat-rich sets (cfg5: ~93 % of the entries sit in runs of
// 100-800).  Here lane l owns entry cb + l of the chunk [cb, cb + 64), and the
// chunk is decided like a short-run window (sweep_window32): each open entry
// gathers its candidates as
//   * a bit mask over the earlier lanes of its chunk,
//   * a summary of the run's earlier chunks, read from an LDS list that keeps
//     only their ACTIVE and UNKNOWN entries (a HIT or HIT_PENDING entry is
//     never in the reference's list again; a run's states change only in this
//     walk, so the list is exact),
//   * a summary of the neighbour run's entries inserted before it, read from
//     an LDS list of that run's ACTIVE / UNKNOWN entries made once per run
//     (states only leave that set; they are re-read at every chunk),
// then rounds of ballots decide the chunk.  Scan order and tie rule are the
// reference's: own run newest first (this chunk, then the list, newest
// first), then the neighbour run newest first; the first strict maximum wins.
// A list that would overflow hands the rest of the run to the entry-by-entry
// walk (own list) or to a per-entry global scan (neighbour list).
__device__ __forceinline__ int below_count(uint64_t m) {  // set bits below this lane
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                        __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

#ifndef RK_LCAP
#define RK_LCAP 128
#endif
constexpr int LCAP = RK_LCAP;  // own-run list
constexpr int NCAP = 64;   // neighbour-run list, per side

struct LongLds {
  uint2 cpk[64 + OWN_U];
  uint32_t cent[64];
  uint2 lpk[LCAP];
  uint32_t lpos[LCAP], lent[LCAP];
  uint8_t lst[LCAP];
  uint2 npk[2][NCAP];
  uint32_t npos[2][NCAP], nent[2][NCAP];
  uint8_t nst[2][NCAP];
  uint32_t ht[2][256];  // list_dedup's two hash tables (zero between calls)
};

// the entry-by-entry walk (k_sweep_wave's, on the 32-bit records) over
// [from, end) of run [beg, end)
__device__ bool walk_entries32(const Axis &ax, uint32_t beg, uint32_t from, uint32_t end,
                               bool has_lo, uint32_t lo_b, uint32_t lo_e, bool has_hi,
                               uint32_t hi_b, uint32_t hi_e, uint32_t lane) {
  bool pending = false;
  for (uint32_t t = from; t < end; ++t) {
    const uint8_t st = load_state(&ax.state[t]);
    if (st == ST_ACTIVE || st == ST_HIT) continue;
    const uint32_t i = ax.ent[t];
    const uint2 me = ax.pk[t];
    const Q32 q32 = make_q32(me.x, me.y, ax.len_ratio, ax.pos_ratio);
    const int dir = ax.nbd[t] == 1 ? -1 : ax.nbd[t] == 2 ? 1 : 0;
    Scan s{0.0, NONE, 0xFFFFFFFFu, false, false};
    for (uint32_t q0 = beg; q0 < t; q0 += 64) {
      const uint32_t q = q0 + lane;
      if (q < t) consider_ranked32(ax, s, q, t - 1 - q, q32);
    }
    if ((dir < 0 && has_lo) || (dir > 0 && has_hi)) {
      const uint32_t nb = dir < 0 ? lo_b : hi_b, ne = dir < 0 ? lo_e : hi_e;
      const uint32_t own = t - beg;
      for (uint32_t q0 = nb; q0 < ne; q0 += 64) {
        const uint32_t q = q0 + lane;
        if (q < ne && ax.ent[q] < i) consider_ranked32(ax, s, q, own + (ne - 1 - q), q32);
      }
    }
    wave_combine(s);
    const uint8_t ns = decide(s);
    if (lane == 0) {
      if (ns != st && (ns == ST_HIT || ns == ST_ACTIVE))
        record_decision(ax, i, ns, ns == ST_HIT ? ax.ent[s.win] : NONE);
      if (ns != st) store_state(&ax.state[t], ns);
    }
    pending |= ns == ST_UNKNOWN || ns == ST_HIT_PENDING;
  }
  return pending;
}

// the neighbour run [nb, ne)'s ACTIVE / UNKNOWN entries into side `sd` of the
// LDS lists; returns their count, or -1 when they do not fit
__device__ int neighbour_list(const Axis &ax, uint32_t nb, uint32_t ne, LongLds &L, int sd,
                              uint32_t lane) {
  int n = 0;
  for (uint32_t q0 = nb; q0 < ne; q0 += 128) {  // two chunks' loads in flight
    uint8_t s[2];
    uint2 pk[2];
    uint32_t en[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const uint32_t q = q0 + 64 * u + lane;
      s[u] = ST_HIT, pk[u] = make_uint2(0, 0), en[u] = 0;
      if (q < ne) s[u] = load_state(&ax.state[q]), pk[u] = ax.pk[q], en[u] = ax.ent[q];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bool keep = s[u] < ST_HIT_PENDING;
      const uint64_t b = __ballot(keep);
      const int at = n + below_count(b);
      if (n + __popcll(b) > NCAP) return -1;
      if (keep) {
        L.npk[sd][at] = pk[u];
        L.npos[sd][at] = q0 + 64 * u + lane;
        L.nent[sd][at] = en[u];
        L.nst[sd][at] = s[u];
      }
      n += __popcll(b);
    }
  }
  return n;
}

// run bounds for long runs: 64 probes 64 positions apart, then one window
// (two memory round trips for a run of up to 4096 instead of one per 64)
// first position >= from whose key is not `key` (or m)
__device__ uint32_t wave_find_end(const Axis &ax, uint32_t from, uint32_t key, uint32_t lane) {
  for (uint64_t b = from;; b += 64 * 64) {
    const uint64_t q = b + 64 * lane;
    const uint64_t e = __ballot(q >= ax.m || ax.key[q] != key);
    if (e) {
      const uint32_t j = (uint32_t)__builtin_ctzll(e);
      return j == 0 ? (uint32_t)b : wave_scan_end(ax, (uint32_t)b + 64 * (j - 1) + 1, key, lane);
    }
  }
}
// smallest p with key `key` on all of [p, before), key[before - 1] == key
__device__ uint32_t wave_find_begin(const Axis &ax, uint32_t before, uint32_t key,
                                    uint32_t lane) {
  for (int64_t b = (int64_t)before - 1;; b -= 64 * 64) {
    const int64_t q = b - 64 * (int64_t)lane;
    const uint64_t e = __ballot(q < 0 || ax.key[q] != key);
    if (e) {  // lane j's probe is the first miss; lane j-1's position is in the run
      const uint32_t j = (uint32_t)__builtin_ctzll(e);
      return j == 0 ? (uint32_t)(b + 1)
                    : wave_scan_begin(ax, (uint32_t)(b - 64 * (int64_t)(j - 1)) + 1, key, lane);
    }
  }
}

// lflag[w] = 1: a run of more than LONG_RUN entries starts in window w (at
// most one can); the first sweep's window kernel sets the flags, so no
// shared list (and no hot atomic counter) is needed.  One wavefront takes 64
// windows and walks their long runs in turn.
// Compacts the own-run list [0, nl) in place, dropping every ACTIVE entry
// whose packed record equals that of a newer ACTIVE entry -- a later list
// entry or an ACTIVE lane of the current chunk (act, rec: this lane) --; an
// ACTIVE lane of the chunk with a newer twin in the chunk clears *keep.
// Returns the new list length (the order of the survivors is kept).
__device__ int list_dedup(LongLds &L, int nl, uint32_t lane, bool act, uint2 rec, bool &keep) {
  constexpr int LS = LCAP / 64;  // list entries per lane: k = lane + 64 s
  bool lk[LS];
  uint2 lp[LS];
  uint32_t lq[LS], le[LS];
  uint8_t ls[LS];
#pragma unroll
  for (int s = 0; s < LS; ++s) {
    const int k = (int)lane + 64 * s;
    lk[s] = k < nl;
    lp[s] = lk[s] ? L.lpk[k] : make_uint2(0, 0);
    lq[s] = lk[s] ? L.lpos[k] : 0u;
    le[s] = lk[s] ? L.lent[k] : 0u;
    ls[s] = lk[s] ? L.lst[k] : (uint8_t)ST_HIT;
  }
#ifndef RK_LDEDUP_HASH
#define RK_LDEDUP_HASH 1
#endif
#if RK_LDEDUP_HASH
  // Every ACTIVE entry by age (list position k: k; chunk lane: nl + lane; the
  // larger the newer) into two 256-slot tables under two hashes of its
  // record, the newest age per slot winning (atomicMax); an entry whose winner
  // in either table is a newer entry with the same record is an older twin.
  // A slot shared by two records can hide a twin -- it then stays, which is
  // always allowed (only the list's room depends on the drops).  ~40
  // instructions per entry where the rounds below took one round trip per
  // distinct record (~2/3 of the cfg5 Y walk's cycles)
  {
    const auto h1 = [](uint2 r) { return (r.x * 0x9E3779B1u ^ r.y * 0x85EBCA77u) >> 24; };
    const auto h2 = [](uint2 r) { return ((r.x ^ (r.y * 0xC2B2AE3Du)) * 0x27D4EB2Fu) >> 24; };
    L.cpk[lane] = rec;  // (the chunk's records, for the winners' lookups)
    wave_sync_lds();
    const uint32_t ca = (uint32_t)nl + lane + 1;  // ages + 1 (0: an empty slot)
    if (act) atomicMax(&L.ht[0][h1(rec)], ca), atomicMax(&L.ht[1][h2(rec)], ca);
#pragma unroll
    for (int s = 0; s < LS; ++s)
      if (lk[s] && ls[s] == ST_ACTIVE) {
        const uint32_t a = (uint32_t)((int)lane + 64 * s) + 1;
        atomicMax(&L.ht[0][h1(lp[s])], a);
        atomicMax(&L.ht[1][h2(lp[s])], a);
      }
    wave_sync_lds();
    const auto twin = [&](uint2 r, uint32_t age1) {  // a newer ACTIVE entry with record r
      bool t = false;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const uint32_t w = L.ht[k][k ? h2(r) : h1(r)];
        if (w > age1) {
          const uint2 o = w - 1 < (uint32_t)nl ? L.lpk[w - 1] : L.cpk[w - 1 - (uint32_t)nl];
          t |= o.x == r.x && o.y == r.y;
        }
      }
      return t;
    };
    if (act && twin(rec, ca)) keep = false;
#pragma unroll
    for (int s = 0; s < LS; ++s)
      if (lk[s] && ls[s] == ST_ACTIVE && twin(lp[s], (uint32_t)((int)lane + 64 * s) + 1)) lk[s] = false;
    wave_sync_lds();  // every table read is done: clear the slots written
    if (act) L.ht[0][h1(rec)] = 0, L.ht[1][h2(rec)] = 0;
#pragma unroll
    for (int s = 0; s < LS; ++s)
      if (ls[s] == ST_ACTIVE && (int)lane + 64 * s < nl) L.ht[0][h1(lp[s])] = 0, L.ht[1][h2(lp[s])] = 0;
  }
#else
  // one round per distinct record among the newest entries: the chunk's ACTIVE
  // lanes, newest first, then the list's ACTIVE entries newest first
  uint64_t a = __ballot(act);
  while (a) {
    const int v = 63 - __clzll(a);
    const uint32_t px = (uint32_t)__builtin_amdgcn_readlane((int)rec.x, v),
                   py = (uint32_t)__builtin_amdgcn_readlane((int)rec.y, v);
    const bool same = act && rec.x == px && rec.y == py;
    if (same && (int)lane != v) keep = false;  // (lanes below v: older)
#pragma unroll
    for (int s = 0; s < LS; ++s)
      lk[s] = lk[s] && !(ls[s] == ST_ACTIVE && lp[s].x == px && lp[s].y == py);
    a &= ~__ballot(same);
  }
#pragma unroll
  for (int s = LS - 1; s >= 0; --s) {
    uint64_t b = __ballot(lk[s] && ls[s] == ST_ACTIVE);
    while (b) {
      const int v = 63 - __clzll(b);
      const uint32_t px = (uint32_t)__builtin_amdgcn_readlane((int)lp[s].x, v),
                     py = (uint32_t)__builtin_amdgcn_readlane((int)lp[s].y, v);
      // older list entries with the same record (list position v + 64 s)
#pragma unroll
      for (int s2 = 0; s2 < LS; ++s2) {
        const int k2 = (int)lane + 64 * s2, kv = v + 64 * s;
        lk[s2] = lk[s2] && !(k2 < kv && ls[s2] == ST_ACTIVE && lp[s2].x == px && lp[s2].y == py);
      }
      b &= ~__ballot(lk[s] && ls[s] == ST_ACTIVE && lp[s].x == px && lp[s].y == py);
      b &= (v > 0 ? (1ull << v) - 1ull : 0ull);  // (continue below v)
    }
  }
#endif
  uint64_t lb[LS];
  int nk = 0;
#pragma unroll
  for (int s = 0; s < LS; ++s) lb[s] = __ballot(lk[s]), nk += __popcll(lb[s]);
  wave_sync_lds();  // every list read is done
  int base = 0;
#pragma unroll
  for (int s = 0; s < LS; ++s) {
    if (lk[s]) {
      const int at = base + below_count(lb[s]);
      L.lpk[at] = lp[s];
      L.lpos[at] = lq[s];
      L.lent[at] = le[s];
      L.lst[at] = ls[s];
    }
    base += __popcll(lb[s]);
  }
  return nk;
}

#ifdef RK_SWEEP_PROF
// measurement build only: the long-run walk's counters (first sweep) --
// [0] runs, [1] entries, [2] chunks, [3] open lanes, [4] list length at the
// chunks, [5] runs handed to the entry walk, [6] entries walked there, [7]
// cycles in chunks, [8] cycles in the entry walk, [9] list entries dropped
// as duplicates
__device__ unsigned long long g_long_prof[24];
// (accumulated per wave in lpacc, flushed once at the end of the kernel)
#define LP_ADD(slot, v) do { lpacc[slot] += (unsigned long long)(v); } while (0)
#else
#define LP_ADD(slot, v)
#endif
// 5 wavefronts per SIMD (96 VGPRs, a few spilled; 119 without the bound, 4
// per SIMD): the walk is latency-bound, and its LDS (28.8 KB per block)
// allows 5 blocks per CU.  cfg5: 66.1 -> 63.7 ms per step (two A/B pairs,
// `tools/gpu_tasks.sh abw5`).  RK_LONG_WPE=0 at build time: unbounded
#ifndef RK_LONG_WPE
#define RK_LONG_WPE 5
#endif
#if RK_LONG_WPE > 0
#define RK_LONG_ATTR __attribute__((amdgpu_waves_per_eu(RK_LONG_WPE)))
#else
#define RK_LONG_ATTR
#endif
__global__ void __launch_bounds__(256) RK_LONG_ATTR k_sweep_long32(Axis ax, uint8_t *lflag,
                                                      uint32_t nwin, uint8_t *rpend,
                                                      uint32_t *counters, uint32_t *work) {
  __shared__ LongLds s_l[4];
  const uint32_t lane = threadIdx.x & 63;
  LongLds &L = s_l[threadIdx.x >> 6];
  for (uint32_t j = lane; j < 2 * 256; j += 64) (&L.ht[0][0])[j] = 0;
  const uint32_t ngrp = (nwin + 63) / 64;
  uint32_t walked = 0;  // (one atomic per wave at the end: 4.6 M same-word atomics per
                        // launch at cfg5 cost the timed launch ~20 ms)
#ifdef RK_SWEEP_PROF
  unsigned long long lpacc[24] = {};
#endif
  for (uint32_t gi = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; gi < ngrp;
       gi += (gridDim.x * blockDim.x) >> 6) {
    uint64_t todo = __ballot(gi * 64 + lane < nwin && lflag[gi * 64 + lane]);
    while (todo) {
#ifdef RK_SWEEP_PROF
      const uint64_t lp_tr = __builtin_amdgcn_s_memtime();
#endif
      const uint32_t w = gi * 64 + (uint32_t)__builtin_ctzll(todo);
      todo &= todo - 1;
      const uint32_t pw = w * 64 + lane;
      const uint32_t kp = pw < ax.m ? ax.key[pw] : NONE;
      const uint64_t sb = __ballot(pw < ax.m && (pw == 0 || ax.key[pw - 1] != kp) &&
                                   pw + LONG_RUN < ax.m && ax.key[pw + LONG_RUN] == kp);
      if (!sb) continue;
      const uint32_t beg = w * 64 + (uint32_t)__builtin_ctzll(sb);
      if (!rpend[beg]) continue;
      const uint32_t key = ax.key[beg];
      const uint32_t end = wave_find_end(ax, beg + LONG_RUN, key, lane);
      walked += end - beg;  // entries walked (the kernel timer's units)
      LP_ADD(0, 1);
      LP_ADD(1, end - beg);
#ifdef RK_SWEEP_PROF
      const uint64_t lp_ta = __builtin_amdgcn_s_memtime();
      LP_ADD(16, lp_ta - lp_tr);
#endif
      // the run's open entries (UNKNOWN / HIT_PENDING): first fo, last lo.
      // Entries after lo are decided and no later query reads them, entries
      // before fo only join the list; a run without one is done (repeat-rich
      // sets: most Y runs -- their X hits sit ACTIVE in the Y lists -- and
      // many X runs).  Four states per lane and load round
      uint32_t fo = NONE, lo = 0;
      for (uint32_t c = beg; c < end; c += 256) {
        uint32_t bits = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t p = c + 4 * lane + j;
          const uint8_t sp = p < end ? load_state(&ax.state[p]) : (uint8_t)ST_HIT;
          bits |= (uint32_t)(sp == ST_UNKNOWN || sp == ST_HIT_PENDING) << j;
        }
        const uint64_t any = __ballot(bits != 0);
        if (any) {
          const int lf = __builtin_ctzll(any), ll = 63 - __clzll(any);
          const uint32_t bf = (uint32_t)__builtin_amdgcn_readlane((int)bits, lf),
                         bl = (uint32_t)__builtin_amdgcn_readlane((int)bits, ll);
          if (fo == NONE) fo = c + 4 * lf + __builtin_ctz(bf);
          lo = c + 4 * ll + 31 - __clz(bl);
        }
      }
#ifdef RK_SWEEP_PROF
      const uint64_t lp_tb = __builtin_amdgcn_s_memtime();
      LP_ADD(12, lp_tb - lp_ta);
#endif
      if (fo == NONE) {
        LP_ADD(10, 1);
        if (lane == 0) rpend[beg] = 0, lflag[w] = 0;  // (later sweeps skip the window)
        continue;
      }
      uint32_t lo_b = 0, lo_e = 0, hi_b = 0, hi_e = 0;
      const bool has_lo = beg > 0 && ax.key[beg - 1] == key - 1;
      if (has_lo) lo_e = beg, lo_b = wave_find_begin(ax, beg, key - 1, lane);
      const bool has_hi = end < ax.m && ax.key[end] == key + 1;
      if (has_hi) hi_b = end, hi_e = wave_find_end(ax, end + 1, key + 1, lane);
      wave_sync_lds();  // the previous run's LDS reads are done
#ifdef RK_SWEEP_PROF
      const uint64_t lp_tc = __builtin_amdgcn_s_memtime();
      LP_ADD(13, lp_tc - lp_tb);
#endif
      const int nn0 = has_lo ? neighbour_list(ax, lo_b, lo_e, L, 0, lane) : 0;
      const int nn1 = has_hi ? neighbour_list(ax, hi_b, hi_e, L, 1, lane) : 0;
      LP_ADD(15, (nn0 < 0 ? 1 : 0) + (nn1 < 0 ? 1 : 0));
#ifdef RK_SWEEP_PROF
      const uint64_t lp_t0 = __builtin_amdgcn_s_memtime();
      LP_ADD(14, lp_t0 - lp_tc);
#endif
      int nl = 0;
      bool pending = false;
      uint32_t cb = beg;
      // a chunk's entries (and the neighbour states) are loaded one chunk
      // ahead: only this walk changes them
      uint2 nme;
      uint32_t ni;
      uint8_t nst, nnd, ns0 = ST_HIT, ns1 = ST_HIT;
      auto fetch = [&](uint32_t c) {
        const uint32_t t = c + lane;
        nme = make_uint2(0, 0), ni = 0, nst = ST_HIT, nnd = 0;
        if (t < end) nme = ax.pk[t], ni = ax.ent[t], nst = load_state(&ax.state[t]), nnd = ax.nbd[t];
        if ((int)lane < nn0) ns0 = load_state(&ax.state[L.npos[0][lane]]);
        if ((int)lane < nn1) ns1 = load_state(&ax.state[L.npos[1][lane]]);
      };
      // this chunk's ACTIVE / UNKNOWN entries join the list: false when it
      // would overflow even without its redundant entries
      auto join_list = [&](bool keep, bool act, uint2 me, uint32_t t, uint32_t i, uint8_t st) {
        uint64_t kb = __ballot(keep);
        if (nl + __popcll(kb) > LCAP) {
          // First drop the redundant entries.  An ACTIVE entry stays ACTIVE,
          // so every OLDER ACTIVE entry with the same packed record {centre,
          // length} -- the same match and the same deviation for every later
          // query, later in scan order (newest first) -- can neither win (the
          // first strict maximum) nor decide anything the newer one does not.
          // Repeat-family runs hold a few dozen distinct records over hundreds
          // of entries.  RK_LDEDUP=0: off
          int nk = nl;
#ifndef RK_LDEDUP
#define RK_LDEDUP 1
#endif
          if (RK_LDEDUP) nk = list_dedup(L, nl, lane, act, me, keep);
          kb = __ballot(keep);
          LP_ADD(9, nl - nk);
          nl = nk;
          if (nl + __popcll(kb) > LCAP) return false;
        }
        wave_sync_lds();  // the list reads of this chunk are done
        if (keep) {
          const int at = nl + below_count(kb);
          L.lpk[at] = me;
          L.lpos[at] = t;
          L.lent[at] = i;
          L.lst[at] = st;
        }
        nl += __popcll(kb);
        return true;
      };
      fetch(beg);
      for (; cb <= lo; cb += 64) {
        const uint32_t t = cb + lane;
        const bool in = t < end;
        const uint2 me = nme;
        const uint32_t i = ni;
        uint8_t st = nst;
        const uint8_t nd = nnd, s0 = ns0, s1 = ns1;
        if (cb + 64 <= lo) fetch(cb + 64);
        if (cb + 64 <= fo) {  // no open entry here: the ACTIVE ones only join the list
          LP_ADD(11, 1);
          const bool act = in && st == ST_ACTIVE;
          if (!join_list(act, act, me, t, i, st)) {
            cb += 64;
            break;
          }
          continue;
        }
        wave_sync_lds();  // the previous chunk's LDS reads are done
        L.cpk[lane] = me;
        L.cent[lane] = i;
        if ((int)lane < nn0) L.nst[0][lane] = s0;
        if ((int)lane < nn1) L.nst[1][lane] = s1;
        wave_sync_lds();
        const uint8_t st0 = st;
        const bool open = in && (st == ST_UNKNOWN || st == ST_HIT_PENDING);
        LP_ADD(2, 1);
#ifdef RK_SWEEP_PROF
        const uint32_t nopen = (uint32_t)__popcll(__ballot(open));  // (outside the lane-0 branch)
        LP_ADD(3, nopen);
#endif
        LP_ADD(4, nl);
        uint64_t rown = 0;
        Scan fl{0.0, NONE, 0, false, false}, fn{0.0, NONE, 0, false, false};
        Q32 q{};
        bool coop = false;  // a neighbour query for the wavefront-wide scan
        // few open entries (cfg5's Y runs: ~1 per chunk, the list holding ~54
        // ACTIVE X hits): the wavefront scans the chunk, the list and the
        // neighbour list for each of them together, as below for an
        // overflowed neighbour run; many (X: ~55 per chunk): a lane each
        const uint64_t openm = __ballot(open);
        const bool wide = __popcll(openm) <= 8;
        if (open) q = make_q32(me.x, me.y, ax.len_ratio, ax.pos_ratio);
        if (wide) {
          for (uint64_t om = openm; om; om &= om - 1) {
            const int v = __builtin_ctzll(om);
            const uint32_t iv = __shfl(i, v);
            const int ndv = __shfl((int)nd, v);
            const Q32 qv{(uint32_t)__shfl((int)q.c, v), (uint32_t)__shfl((int)q.L, v),
                         (uint32_t)__shfl((int)q.tl, v), (uint32_t)__shfl((int)q.tc, v),
                         __shfl(q.ok ? 1 : 0, v) != 0, __shfl(q.eq ? 1 : 0, v) != 0};
            // the chunk's earlier entries: one ballot
            const uint64_t ro = __ballot((int)lane < v && m32(qv, L.cpk[lane]));
            // the list (older chunks), newest first: the first strict maximum
            // is the largest d, then the largest position
            const auto best_of = [&](bool act, double d, int k, Scan &out, const uint32_t *ids) {
              d = act ? d : -1.0;
              k = act ? k : -1;
              for (int o = 32; o > 0; o >>= 1) {
                const double od = __shfl_xor(d, o);
                const int ok = __shfl_xor(k, o);
                if (od > d || (od == d && ok > k)) d = od, k = ok;
              }
              if (k >= 0) out.best = d, out.win = ids[k], out.any_active = true;
            };
            Scan sl{0.0, NONE, 0, false, false}, sn{0.0, NONE, 0, false, false};
            {
              bool unk = false, act = false;
              double d = -1.0;
              int kb = -1;
#pragma unroll
              for (int s2 = 0; s2 < LCAP / 64; ++s2) {
                const int k = (int)lane + 64 * s2;
                if (k >= nl) continue;
                const uint2 o = L.lpk[k];
                if (!m32(qv, o)) continue;
                if (L.lst[k] != ST_ACTIVE) {
                  unk = true;
                  continue;
                }
                const double dk = dev32(qv, o, ax.len_ratio, ax.pos_ratio);
                if (!act || dk > d || (dk == d && k > kb)) d = dk, kb = k;
                act = true;
              }
              sl.any_unknown = __ballot(unk) != 0;
              best_of(act, d, kb, sl, L.lent);
            }
            const int dir = ndv == 1 ? -1 : ndv == 2 ? 1 : 0;
            const int sd = dir < 0 ? 0 : 1;
            const int nn = dir < 0 ? nn0 : nn1;
            if (dir != 0 && (dir < 0 ? has_lo : has_hi) && nn >= 0) {
              bool unk = false, act = false;
              double d = -1.0;
              int kb = -1;
              static_assert(NCAP == 64, "one neighbour-list entry per lane");
              const int k = (int)lane;
              if (k < nn && L.nent[sd][k] < iv && L.nst[sd][k] < ST_HIT_PENDING) {
                const uint2 o = L.npk[sd][k];
                if (m32(qv, o)) {
                  if (L.nst[sd][k] != ST_ACTIVE) unk = true;
                  else act = true, d = dev32(qv, o, ax.len_ratio, ax.pos_ratio), kb = k;
                }
              }
              sn.any_unknown = __ballot(unk) != 0;
              best_of(act, d, kb, sn, L.nent[sd]);
            } else if (dir != 0 && (dir < 0 ? has_lo : has_hi)) {
              if ((int)lane == v) coop = true;  // (overflowed: the scan below)
            }
            if ((int)lane == v) rown = ro, fl = sl, fn = sn;
          }
        } else if (open) {
          for (int j = 0; j < (int)lane; j += OWN_U) {
            uint64_t b4 = 0;
  #pragma unroll
            for (int u = 0; u < OWN_U; ++u) b4 |= (uint64_t)m32(q, L.cpk[j + u]) << u;
            if ((int)lane - j < OWN_U) b4 &= (1ull << ((int)lane - j)) - 1ull;
            rown |= b4 << j;
          }
          for (int k = nl - 1; k >= 0; --k) {  // earlier chunks, newest first
            const uint8_t sk = L.lst[k];
            const uint2 o = L.lpk[k];
            if (!m32(q, o)) continue;
            if (sk != ST_ACTIVE) {
              fl.any_unknown = true;
              continue;
            }
            const double d = dev32(q, o, ax.len_ratio, ax.pos_ratio);
            if (d > fl.best) fl.best = d, fl.win = L.lent[k];
            fl.any_active = true;
          }
          const int dir = nd == 1 ? -1 : nd == 2 ? 1 : 0;
          const int sd = dir < 0 ? 0 : 1;
          const int nn = dir < 0 ? nn0 : nn1;
          if (dir != 0 && (dir < 0 ? has_lo : has_hi)) {
            if (nn >= 0) {
              // newest first, four entries per step (their LDS reads together)
              for (int k0 = nn - 1; k0 >= 0; k0 -= 4) {
                uint32_t ek[4];
                uint8_t sk[4];
                uint2 ok[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                  const int k = k0 - u >= 0 ? k0 - u : 0;
                  ek[u] = L.nent[sd][k], sk[u] = L.nst[sd][k], ok[u] = L.npk[sd][k];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                  if (k0 - u < 0 || ek[u] >= i || sk[u] >= ST_HIT_PENDING || !m32(q, ok[u])) continue;
                  if (sk[u] != ST_ACTIVE) {
                    fn.any_unknown = true;
                    continue;
                  }
                  const double d = dev32(q, ok[u], ax.len_ratio, ax.pos_ratio);
                  if (d > fn.best) fn.best = d, fn.win = ek[u];
                  fn.any_active = true;
                }
              }
            } else {  // list overflow: the wavefront scans the neighbour run (below)
              coop = true;
            }
          }
        }
        // Queries whose neighbour run overflowed its list: the whole wavefront
        // scans that run for each of them, 64 entries per load, newest first.
        // (A lane walking it alone -- foreign_scan32 -- waits for one load per
        // entry: on cfg5's Y axis, where a family copy's runs straddle bucket
        // bounds and hold hundreds of ACTIVE X hits, that walk took most of
        // the kernel's time.)
#ifdef RK_SWEEP_PROF
        const uint64_t lp_c0 = __builtin_amdgcn_s_memtime();
        LP_ADD(18, __popcll(__ballot(coop)));
#endif
        for (uint64_t cm = __ballot(coop); cm; cm &= cm - 1) {
          const int v = __builtin_ctzll(cm);
          const int dv = __shfl(nd == 1 ? -1 : 1, v);
          const uint32_t iv = __shfl(i, v);
          const Q32 qv{(uint32_t)__shfl((int)q.c, v), (uint32_t)__shfl((int)q.L, v),
                       (uint32_t)__shfl((int)q.tl, v), (uint32_t)__shfl((int)q.tc, v),
                       __shfl(q.ok ? 1 : 0, v) != 0, __shfl(q.eq ? 1 : 0, v) != 0};
          const uint32_t nb = dv < 0 ? lo_b : hi_b, ne = dv < 0 ? lo_e : hi_e;
          Scan cs{0.0, NONE, 0, false, false};
          uint32_t bestg = 0;
          for (uint32_t top = ne; top > nb;) {  // positions [top - 64, top), newest first
            const uint32_t g = top - 1 - lane;
            const bool ing = g + 1 > nb && top >= 1 + lane;  // g >= nb, no wrap
            const uint32_t eg = ing ? ax.ent[g] : 0xFFFFFFFFu;
            const uint8_t sg = ing ? load_state(&ax.state[g]) : (uint8_t)ST_HIT;
            const uint2 og = ing ? ax.pk[g] : make_uint2(0, 0);
            const bool cand = ing && eg < iv && sg < ST_HIT_PENDING && m32(qv, og);
            if (__ballot(cand && sg != ST_ACTIVE)) {  // an undecided candidate: not final now
              cs.any_unknown = true;
              break;
            }
            const bool act = cand && sg == ST_ACTIVE;
            double d = act ? dev32(qv, og, ax.len_ratio, ax.pos_ratio) : -1.0;
            uint32_t gg = act ? g : 0u;
            // the first strict maximum, newest first: the larger d, then the larger g
            for (int o = 32; o > 0; o >>= 1) {
              const double od = __shfl_xor(d, o);
              const uint32_t og2 = (uint32_t)__shfl_xor((int)gg, o);
              if (od > d || (od == d && og2 > gg)) d = od, gg = og2;
            }
            if (__ballot(act) && (!cs.any_active || d > cs.best))
              cs.best = d, bestg = gg, cs.any_active = true;
            top = top > 64 ? top - 64 : 0;
          }
          if (cs.any_active) cs.win = ax.ent[bestg];
          if ((int)lane == v) fn = cs;
        }
#ifdef RK_SWEEP_PROF
        LP_ADD(17, __builtin_amdgcn_s_memtime() - lp_c0);
#endif
        const bool out_act = fl.any_active || fn.any_active;
        const bool out_unk = fl.any_unknown || fn.any_unknown;
        for (;;) {
          const uint64_t A = __ballot(in && st == ST_ACTIVE);
          const uint64_t U = __ballot(in && st == ST_UNKNOWN);
          bool changed = false;
          if (open && st == ST_UNKNOWN) {
            if ((A & rown) || out_act) st = ST_HIT_PENDING, changed = true;
            else if (!(U & rown) && !out_unk) st = ST_ACTIVE, changed = true;
          }
          const uint64_t V = __ballot(in && st == ST_UNKNOWN);
          if (open && st == ST_HIT_PENDING && !(V & rown) && !out_unk) st = ST_HIT, changed = true;
          const bool left = open && (st == ST_UNKNOWN || st == ST_HIT_PENDING);
          if (!__ballot(changed) || !__ballot(left)) break;
        }
        const uint64_t A = __ballot(in && st == ST_ACTIVE);
        pending |= open && (st == ST_UNKNOWN || st == ST_HIT_PENDING);
        if (open && st != st0) {
          if (st == ST_HIT) {
            double best = 0.0;
            uint32_t win = NONE;
            uint64_t b = A & rown;
            while (b) {  // this chunk, newest first
              const int v = 63 - __clzll(b);
              b &= ~(1ull << v);
              const double d = dev32(q, L.cpk[v], ax.len_ratio, ax.pos_ratio);
              if (d > best) best = d, win = L.cent[v];
            }
            if (fl.any_active && fl.best > best) best = fl.best, win = fl.win;
            if (fn.any_active && fn.best > best) win = fn.win;
            record_decision(ax, i, ST_HIT, win);
          } else if (st == ST_ACTIVE) {
            record_decision(ax, i, ST_ACTIVE, NONE);
          }
          store_state(&ax.state[t], st);
        }
        // this chunk's ACTIVE / UNKNOWN entries join the list
        if (!join_list(in && (st == ST_ACTIVE || st == ST_UNKNOWN), in && st == ST_ACTIVE, me, t, i,
                       st)) {
          cb += 64;
          break;
        }
      }
#ifdef RK_SWEEP_PROF
      const uint64_t lp_t1 = __builtin_amdgcn_s_memtime();
      LP_ADD(7, lp_t1 - lp_t0);
#endif
      if (cb <= lo) {  // own list overflow: the rest (up to the last open entry) one by one
        LP_ADD(5, 1);
        LP_ADD(6, lo + 1 - cb);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        pending |= walk_entries32(ax, beg, cb, lo + 1, has_lo, lo_b, lo_e, has_hi, hi_b, hi_e,
                                  lane);
#ifdef RK_SWEEP_PROF
        LP_ADD(8, __builtin_amdgcn_s_memtime() - lp_t1);
#endif
      }
      const bool pend = __ballot(pending) != 0;
      if (lane == 0) {
        rpend[beg] = pend;
        if (pend) atomicAdd(&counters[w % PEND_SLOTS], 1u);
        else lflag[w] = 0;  // a decided run: later sweeps skip its window at the flag load
      }
    }
  }
  if (work && lane == 0 && walked) atomicAdd(work, walked);
#ifdef RK_SWEEP_PROF
  if (lane == 0)
    for (int k = 0; k < 24; ++k)
      if (lpacc[k]) atomicAdd(&g_long_prof[k], lpacc[k]);
#endif
}

// Run bounds of every bucket run, one wavefront per 64 positions: rlen_at at
// each run start, rbeg_at at each run end, and the starts of the runs longer
// than LONG_RUN appended to `big` (one atomic per wave).  A run crossing the
// window is finished by a wave-wide search 64 keys at a time; each wave
// searches at most once in each direction, so the kernel is O(m).
__device__ __forceinline__ bool is_start(const Axis &ax, uint32_t p) {
  return p == 0 || p >= ax.m || ax.key[p] != ax.key[p - 1];
}
__global__ void __launch_bounds__(256) k_run_bounds(Axis ax, uint32_t nwin, uint32_t *big,
                                                    uint32_t *nbig) {
  const int lane = threadIdx.x & 63;
  const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (w >= nwin) return;
  const uint32_t base = w * 64, p = base + lane, m = ax.m;
  const bool in = p < m;
  const bool st = in && is_start(ax, p);
  const bool en = in && is_start(ax, p + 1);  // p + 1 == m counts as a start
  const uint64_t S = __ballot(st), E = __ballot(en);
  const uint64_t le = (2ull << lane) - 1ull;  // bits <= lane
  // the run that started before the window and ends inside it (an end comes
  // before the window's first start)
  uint32_t first_beg = base;
  const int fs = S ? __builtin_ctzll(S) : 64, fe = E ? __builtin_ctzll(E) : 64;
  if (fe < fs) {  // base > 0 here: position 0 is always a start
    uint32_t b = base;
    for (;;) {  // wave-wide backward search
      const uint32_t q0 = b - 64;
      const uint64_t s2 = __ballot(is_start(ax, q0 + lane));
      if (s2) {
        first_beg = q0 + 63 - __clzll(s2);
        break;
      }
      b = q0;
    }
  }
  // the run that starts inside the window and ends after it
  uint32_t last_end = 0;  // exclusive
  {
    const int hi_start = S ? 63 - __clzll(S) : 0;
    const bool open = S && (E >> hi_start) == 0;
    if (open) {
      uint32_t b = base + 64;
      for (;;) {  // wave-wide forward search
        const uint32_t q = b + lane;
        const uint64_t e2 = __ballot(q < m && is_start(ax, q + 1));
        if (e2) {
          last_end = b + __builtin_ctzll(e2) + 1;
          break;
        }
        b += 64;
      }
    }
  }
  bool isbig = false;
  if (st) {
    const uint64_t e_after = E & ~((1ull << lane) - 1ull);
    const uint32_t end = e_after ? base + __builtin_ctzll(e_after) + 1 : last_end;
    ax.rlen_at[p] = end - p;
    isbig = end - p > LONG_RUN;
  }
  if (en) {
    const uint64_t s_before = S & le;
    ax.rbeg_at[p] = s_before ? base + 63 - __clzll(s_before) : first_beg;
  }
  const uint64_t bb = __ballot(isbig);
  uint32_t at = 0;
  if (lane == 0 && bb) at = atomicAdd(nbig, (uint32_t)__popcll(bb));
  at = __shfl(at, 0);
  if (isbig) big[at + __popcll(bb & ((1ull << lane) - 1ull))] = p;
}

}  // namespace

#ifdef RK_SWEEP_PROF
static void *g_sweep_prof_ptr() {
  void *p = nullptr;
  (void)hipGetSymbolAddress(&p, HIP_SYMBOL(g_sweep_prof));
  return p;
}
#endif
size_t runs_scratch_words(uint32_t m) { return (size_t)m / (LONG_RUN + 1) + 64; }

void build_runs(const Axis &ax, RunList &rl, uint32_t *dev_count, uint32_t *host_words,
                hipStream_t st) {
  rl.nbig = 0;
  rl.nwin = (ax.m + 63) / 64;
  if (!ax.m) return;
  if (rl.fast32) return;  // the first sweep flags the long runs and the windows itself
  (void)hipMemsetAsync(rl.wpend, 1, rl.nwin, st);
  (void)hipMemsetAsync(dev_count, 0, 4, st);
  kt_begin(st, KID_RUN_BOUNDS);
  k_run_bounds<<<(rl.nwin + 3) / 4, 256, 0, st>>>(ax, rl.nwin, rl.big, dev_count);
  kt_end(st, KID_RUN_BOUNDS, 4.0 * ax.m);  // keys read once (boundary writes not counted)
  (void)hipMemcpyAsync(host_words, dev_count, 4, hipMemcpyDeviceToHost, st);
  (void)hipStreamSynchronize(st);
  rl.nbig = host_words[0];
}

void occupancy_sweep(const Axis &ax, const RunList &rl, uint8_t *rpend, uint32_t *counters,
                     bool first, hipStream_t st, bool clear) {
  if (clear) (void)hipMemsetAsync(counters, 0, PEND_SLOTS * sizeof(uint32_t), st);
  // algorithmic bytes: the first sweep reads every entry's key, centre, length,
  // id and state and writes state (+ winner): 30 B (26 B with the packed 8-B
  // record and neighbour code of the 32-bit kernel); later sweeps only need
  // the window flags (their real work is what the first one left open)
  if (rl.nwin) {
    const int kid = rl.fast32 ? (first ? KID_SWEEP_FAST : KID_SWEEP_MORE) : KID_SWEEP_TILE;
    kt_begin(st, kid);
    if (rl.fast32 && first) {
      if (ax.par_dev)
        k_sweep_fast<true><<<(rl.nwin + 3) / 4, 256, 0, st>>>(
            ax, rl.wpend, rl.nwin, counters, reinterpret_cast<uint8_t *>(rl.big), rpend);
      else
        k_sweep_fast<false><<<(rl.nwin + 3) / 4, 256, 0, st>>>(
            ax, rl.wpend, rl.nwin, counters, reinterpret_cast<uint8_t *>(rl.big), rpend);
    } else if (rl.fast32) {
      if (ax.par_dev)
        k_sweep_fast_more<true><<<((rl.nwin + 63) / 64 + 3) / 4, 256, 0, st>>>(ax, rl.wpend,
                                                                             rl.nwin, counters);
      else
        k_sweep_fast_more<false><<<((rl.nwin + 63) / 64 + 3) / 4, 256, 0, st>>>(ax, rl.wpend,
                                                                              rl.nwin, counters);
    }
    else
      k_sweep_tile<<<(rl.nwin + 3) / 4, 256, 0, st>>>(ax, rl.wpend, rl.nwin, counters);
    kt_end(st, kid, first ? (rl.fast32 ? 26.0 : 30.0) * ax.m : (double)rl.nwin);
#ifdef RK_SWEEP_PROF
    if (rl.fast32 && first) {
      unsigned long long h[16];
      (void)hipStreamSynchronize(st);
      (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_sweep_prof), sizeof h);
      const double w = h[6] ? (double)h[6] : 1.0;
      fprintf(stderr, "SWEEPPROF m=%u windows=%llu cyc/win: setup %.0f own %.0f nb %.0f (foreign scans %.0f) rounds %.0f winners %.0f record %.0f | rounds/win %.2f slot1 %.3f one-slot windows %.3f | longest deviation list/win %.2f deviations/win %.2f | longest LDS neighbour run/win %.2f LDS neighbour entries/win %.2f foreign scans/win %.3f\n",
              ax.m, h[6], h[0] / w, h[1] / w, h[2] / w, h[15] / w, h[3] / w, h[4] / w, h[14] / w, h[5] / w, h[7] / w, h[8] / w, h[9] / w, h[10] / w, h[11] / w, h[12] / w, h[13] / w);
      (void)hipMemsetAsync(g_sweep_prof_ptr(), 0, sizeof h, st);
    }
#endif
  }
  if (rl.fast32) {  // the long-run count lives on the device: a fixed grid reads it
    // algorithmic bytes per entry of a walked run: its packed record (8 B),
    // id (4 B), state read and write (2 B) and winner (4 B)
    uint32_t *work = kt_units(st, KID_SWEEP_LONG);  // (its clear ahead of the start event)
    // blocks: the 64-window groups go round-robin over them, so a grid many
    // times the resident blocks (5 per CU) lets the hardware balance the
    // uneven groups -- one block per 8 groups, 2048 .. 32768 (cfg5: 2048 ->
    // 32768 blocks, 63.7 -> 55.6 ms per step; cfg3 keeps 2048).
    // RK_LONG_GRID: a fixed grid
    static const int long_env = [] {
      const char *e = getenv("RK_LONG_GRID");
      return e ? atoi(e) : 0;
    }();
    const int long_grid =
        long_env > 0 ? long_env
                     : (int)std::min(32768u, std::max(2048u, (rl.nwin + 63) / 64 / 8));
    kt_begin(st, KID_SWEEP_LONG);
    k_sweep_long32<<<long_grid, 256, 0, st>>>(ax, reinterpret_cast<uint8_t *>(rl.big), rl.nwin,
                                              rpend, counters, work);
    kt_end_units(st, KID_SWEEP_LONG, 18.0);
#ifdef RK_SWEEP_PROF
    {  // every sweep (first=1: the first of the axis)
      unsigned long long h[24];
      (void)hipStreamSynchronize(st);
      (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_long_prof), sizeof h);
      fprintf(stderr, "first=%d ", (int)first);
      const double c = h[2] ? (double)h[2] : 1.0;
      fprintf(stderr, "LONGPROF m=%u runs=%llu entries=%llu chunks=%llu open/chunk %.2f list/chunk %.1f overflow runs=%llu walked=%llu | Mcyc run-find %.1f prescan %.1f nbounds %.1f nlists %.1f chunks %.1f walk %.1f | dedup drops=%llu | runs without open entries %llu, list-only chunks %llu, overflowed neighbour lists %llu | wavefront neighbour scans %llu, %.1f Mcyc\n",
              ax.m, h[0], h[1], h[2], h[3] / c, h[4] / c, h[5], h[6], h[16] / 1e6, h[12] / 1e6,
              h[13] / 1e6, h[14] / 1e6, h[7] / 1e6, h[8] / 1e6, h[9], h[10], h[11], h[15], h[18],
              h[17] / 1e6);
      void *p = nullptr;
      (void)hipGetSymbolAddress(&p, HIP_SYMBOL(g_long_prof));
      (void)hipMemsetAsync(p, 0, sizeof h, st);
    }
#endif
  } else if (rl.nbig) {
    kt_begin(st, KID_SWEEP_WAVE);
    k_sweep_wave<<<grid_for(rl.nbig, 4, 2048), 256, 0, st>>>(ax, rl.big, rl.nbig, rpend,
                                                             counters);
    kt_end(st, KID_SWEEP_WAVE, 0.0);
  }
}

}  // namespace rk
