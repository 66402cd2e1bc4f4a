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

constexpr uint32_t WAVE_MIN = 48;  // runs at least this long get a whole wavefront (<= 64)

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

// States only move UNKNOWN -> decided (and HIT_PENDING -> HIT), so a stale
// read of another run's state is always conservative: it can only postpone a
// decision to the next sweep, never change one.  Plain loads and stores are
// therefore enough (agent-scope sc1 byte stores are one fabric write each);
// every sweep is its own launch, which makes all states coherent between sweeps.
__device__ __forceinline__ uint8_t load_state(const uint8_t *s) { return *(const volatile uint8_t *)s; }
__device__ __forceinline__ void store_state(uint8_t *s, uint8_t v) { *s = v; }

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

__device__ __forceinline__ bool run_start(const Axis &ax, uint32_t p) {
  return p == 0 || ax.key[p] != ax.key[p - 1];
}

// pending-run counters are spread over PEND_WORDS words (one hot word
// serialises at ~88 atomics/us); the host sums them
constexpr uint32_t PEND_SLOTS = PEND_WORDS;

__device__ __forceinline__ void count_pending(uint32_t *counters, bool pending) {
  const uint64_t b = __ballot(pending);
  if ((threadIdx.x & 63) == 0 && b)
    atomicAdd(&counters[(blockIdx.x * 4 + (threadIdx.x >> 6)) % PEND_SLOTS], (uint32_t)__popcll(b));
}

// ---- one lane walks one run ----------------------------------------------
// Work items: the short runs (< WAVE_MIN <= 64 entries), sorted by length
// class so the 64 lanes of a wave walk runs of similar length.  The run's own
// states live in two 64-bit masks (bit t = entry beg+t): `act` = in the list,
// `unk` = undecided, so entries that already hit are never touched again.
// While the run holds at most ACACHE list entries their centre and length
// stay in registers too: the typical run (a repeat copy's fragments -- one
// list entry, every later fragment hits it) then reads each entry from memory
// exactly once.
constexpr int ACACHE = 4;

__global__ void __launch_bounds__(256) k_sweep_lane(Axis ax, const uint32_t *run_beg,
                                                    uint32_t nruns, uint8_t *rpend,
                                                    uint32_t *counters) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  bool pending = false;
  if (w < nruns) {
    const uint32_t beg = run_beg[w];
    if (rpend[beg]) {
      const uint32_t len = ax.rlen_at[beg];
      const uint32_t key = ax.key[beg];
      uint64_t act = 0, unk = 0, todo = 0;
      for (uint32_t t = 0; t < len; ++t) {
        const uint8_t st = ax.state[beg + t];
        const uint64_t bit = 1ull << t;
        if (st == ST_ACTIVE) act |= bit;
        else if (st == ST_UNKNOWN) unk |= bit, todo |= bit;
        else if (st == ST_HIT_PENDING) todo |= bit;
      }
      // register cache of the list entries (ascending position)
      uint32_t cp[ACACHE];
      uint64_t cc[ACACHE], cl[ACACHE];
      int nc = 0;
      bool ovf = __popcll(act) > ACACHE;
#pragma unroll
      for (int j = 0; j < ACACHE; ++j) cp[j] = 64, cc[j] = 0, cl[j] = 0;
      if (!ovf) {
        uint64_t a = act;
#pragma unroll
        for (int j = 0; j < ACACHE; ++j) {
          if (a) {
            const uint32_t u = (uint32_t)__builtin_ctzll(a);
            a &= a - 1;
            cp[j] = u;
            cc[j] = ax.cen[beg + u];
            cl[j] = ax.len[beg + u];
            nc = j + 1;
          }
        }
      }
      // neighbour runs, found lazily: 0 = not looked up, 1 = absent, 2 = present
      int lo_st = 0, hi_st = 0;
      uint32_t lo_b = 0, lo_e = 0, hi_b = 0, hi_e = 0;
      while (todo) {
        const uint32_t t = (uint32_t)__builtin_ctzll(todo);
        const uint64_t bit = 1ull << t;
        todo &= todo - 1;
        const uint32_t q0 = beg + t;
        const uint64_t c = ax.cen[q0], L = ax.len[q0];
        Scan s{0.0, NONE, 0, false, false};
        const uint64_t below = bit - 1;
        if (!ovf && (unk & below) == 0) {
          // every candidate is a cached list entry: newest first
#pragma unroll
          for (int j = ACACHE - 1; j >= 0; --j) {
            if (j < nc && cp[j] < t) {
              const double d = deviation(c, L, cc[j], cl[j], ax.len_ratio, ax.pos_ratio);
              if (d > 0) {
                s.any_active = true;
                if (d > s.best) {
                  s.best = d;
                  s.win = beg + cp[j];
                }
              }
            }
          }
        } else {
          uint64_t cand = (act | unk) & below;
          while (cand) {  // newest first
            const uint32_t u = 63 - (uint32_t)__builtin_clzll(cand);
            cand &= ~(1ull << u);
            const uint32_t q = beg + u;
            const double d = deviation(c, L, ax.cen[q], ax.len[q], ax.len_ratio, ax.pos_ratio);
            if (!(d > 0)) continue;
            if ((act >> u) & 1ull) {
              s.any_active = true;
              if (d > s.best) {
                s.best = d;
                s.win = q;
              }
            } else {
              s.any_unknown = true;
            }
          }
        }
        const int dir = neighbour_dir(c, ax.max_index);
        if (dir) {
          int &nst = dir < 0 ? lo_st : hi_st;
          uint32_t &nb = dir < 0 ? lo_b : hi_b;
          uint32_t &ne = dir < 0 ? lo_e : hi_e;
          if (nst == 0) nst = neighbour_run(ax, beg, beg + len, key, dir, nb, ne) ? 2 : 1;
          if (nst == 2) {
            const uint32_t i = ax.ent[q0];
            for (uint32_t q = ne; q-- > nb;)  // newest first, only entries inserted before i
              if (ax.ent[q] < i) consider(ax, s, q, c, L);
          }
        }
        const uint8_t ns = decide(s);
        if (ns == ST_HIT) ax.win[q0] = ax.ent[s.win];
        if (ns != ST_UNKNOWN) {
          unk &= ~bit;
          if (ns == ST_ACTIVE) {
            act |= bit;
            // the cache must stay in ascending position (newest-first scans);
            // in a re-walk an entry may be decided behind a cached later one,
            // and a fifth list entry does not fit: both switch to memory reads
            if (!ovf) {
              uint32_t last = 0;
#pragma unroll
              for (int j = 0; j < ACACHE; ++j)
                if (j + 1 == nc) last = cp[j];
              if (nc < ACACHE && (nc == 0 || last < t)) {
#pragma unroll
                for (int j = 0; j < ACACHE; ++j)
                  if (j == nc) cp[j] = t, cc[j] = c, cl[j] = L;
                ++nc;
              } else {
                ovf = true;
              }
            }
          }
          store_state(&ax.state[q0], ns);
        }
        pending |= ns == ST_UNKNOWN || ns == ST_HIT_PENDING;
      }
      rpend[beg] = pending;
    }
  }
  count_pending(counters, pending);
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

__global__ void __launch_bounds__(256) k_sweep_wave(Axis ax, const uint32_t *big, uint32_t nbig,
                                                    uint8_t *rpend, uint32_t *counters) {
  // big = starts of the runs of >= WAVE_MIN entries
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
    if (lane == 0) {
      rpend[beg] = pending;
      if (pending) atomicAdd(&counters[w % PEND_SLOTS], 1u);
    }
  }
}

__global__ void k_run_flags(Axis ax, uint32_t *flag) {
  for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < ax.m; p += gridDim.x * blockDim.x)
    flag[p] = run_start(ax, p);
}

// run r starts at p (rank from the scan); its length key is filled next
__global__ void k_run_emit(Axis ax, const uint32_t *flag, const uint32_t *rank, uint32_t *beg) {
  for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < ax.m; p += gridDim.x * blockDim.x)
    if (flag[p]) beg[rank[p]] = p;
}

// length CLASS key (1, 2, 3-4, 5-8, ..., 33-47, >= WAVE_MIN): a stable sort by
// class keeps runs in position order inside a class, so the lanes of a wave
// walk runs of similar length that also sit close together in memory (a sort
// by exact length scatters them and every lane drags in its own cache lines).
// Counts runs shorter than WAVE_MIN (one atomic per block).
__global__ void __launch_bounds__(256) k_run_len(const uint32_t *beg, uint32_t nruns, uint32_t m,
                                                 uint32_t *lenkey, uint32_t *nshort) {
  uint32_t mine = 0;
  for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < nruns;
       r += gridDim.x * blockDim.x) {
    const uint32_t len = (r + 1 < nruns ? beg[r + 1] : m) - beg[r];
    lenkey[r] = len >= WAVE_MIN ? 7u : (uint32_t)(32 - __clz((int)(len - 1)));  // ceil(log2)
    mine += len < WAVE_MIN;
  }
  __shared__ uint32_t part[4];
  for (int off = 32; off > 0; off >>= 1) mine += __shfl_xor(mine, off);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = mine;
  __syncthreads();
  if (threadIdx.x == 0 && part[0] + part[1] + part[2] + part[3])
    atomicAdd(nshort, part[0] + part[1] + part[2] + part[3]);
}

// per-position run tables: length at each run start, start at each run end
__global__ void k_run_tables(Axis ax, const uint32_t *beg, uint32_t nruns, uint32_t *rlen_at,
                             uint32_t *rbeg_at) {
  for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < nruns;
       r += gridDim.x * blockDim.x) {
    const uint32_t b = beg[r], e = r + 1 < nruns ? beg[r + 1] : ax.m;
    rlen_at[b] = e - b;
    rbeg_at[e - 1] = b;
  }
}

}  // namespace

size_t runs_scratch_words(uint32_t m) { return 4 * ((size_t)m + 1) + 64; }

void build_runs(const Axis &ax, RunList &rl, uint32_t *scratch, uint32_t *radix_k_tmp,
                uint32_t *radix_v_tmp, uint32_t *radix_scratch, size_t radix_words,
                ScanScratch ss, uint32_t *dev_words, uint32_t *host_words, hipStream_t st) {
  rl.nruns = rl.nshort = 0;
  if (!ax.m) return;
  const size_t m1 = (size_t)ax.m + 1;
  uint32_t *flag = scratch, *rank = scratch + m1, *beg = rank + m1, *lenkey = beg + m1;
  k_run_flags<<<grid_for(ax.m, 256), 256, 0, st>>>(ax, flag);
  (void)hipMemsetAsync(flag + ax.m, 0, 4, st);
  exclusive_scan_u32(flag, rank, m1, ss, st);
  k_run_emit<<<grid_for(ax.m, 256), 256, 0, st>>>(ax, flag, rank, beg);
  (void)hipMemcpyAsync(host_words, rank + ax.m, 4, hipMemcpyDeviceToHost, st);
  (void)hipStreamSynchronize(st);
  rl.nruns = host_words[0];
  (void)hipMemsetAsync(dev_words, 0, 4, st);
  k_run_len<<<grid_for(rl.nruns, 256, 2048), 256, 0, st>>>(beg, rl.nruns, ax.m, lenkey, dev_words);
  k_run_tables<<<grid_for(rl.nruns, 256), 256, 0, st>>>(ax, beg, rl.nruns, ax.rlen_at, ax.rbeg_at);
  // ascending class: short runs first, long runs (class 7) last
  radix_sort_pairs(lenkey, beg, rl.len, rl.beg, radix_k_tmp, radix_v_tmp, rl.nruns, 3,
                   radix_scratch, radix_words, st);
  (void)hipMemcpyAsync(host_words, dev_words, 4, hipMemcpyDeviceToHost, st);
  (void)hipStreamSynchronize(st);
  rl.nshort = host_words[0];
}

void occupancy_sweep(const Axis &ax, const RunList &rl, uint8_t *rpend, uint32_t *counters,
                     hipStream_t st) {
  (void)hipMemsetAsync(counters, 0, PEND_SLOTS * sizeof(uint32_t), st);
  if (rl.nshort)
    k_sweep_lane<<<(rl.nshort + 255) / 256, 256, 0, st>>>(ax, rl.beg, rl.nshort, rpend,
                                                          counters);
  const uint32_t nbig = rl.nruns - rl.nshort;
  if (nbig)
    k_sweep_wave<<<grid_for(nbig, 4, 2048), 256, 0, st>>>(ax, rl.beg + rl.nshort, nbig, rpend,
                                                          counters);
}

}  // namespace rk
