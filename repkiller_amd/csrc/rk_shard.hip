// rk_shard.hip -- ONE fragment set classified across P GPUs (rk_classify_sharded).
//
// Produces exactly what rk_classify writes for the concatenated input
// (reference: generate_fragment_groups + generate_diagonal_func + sort_groups,
// commonFunctions.cpp:41-177), with every rank holding a contiguous share of
// each structure:
//
//   ingress     processing order = stable sort by xStart/10 (FragmentsDatabase
//               buckets, FragmentsDatabase.cpp:84-97); ranks own contiguous
//               xStart/10 ranges chosen from an all-gathered histogram (the
//               global coverage histogram) and receive their rows by all-to-all.
//               Blocks arrive in rank order = file order, so a stable local sort
//               gives the global processing order; global index = slice offset
//               + local index.
//   X axis      a query only sees EARLIER entries (SequenceOcupationList.cpp:33-91
//               over lists filled in processing order), so slice g needs the
//               entries of slices < g whose X centre bucket is >= its first
//               bucket - 1 ("relevant") -- plus a lead-in of `lead_in` more
//               buckets so that those entries' own decisions come out right
//               locally.  Each rank resolves [lead-in + own] with the
//               single-device sweeps, then the owners' final states of the
//               relevant entries are exchanged and compared; a rank whose halo
//               disagrees re-resolves with the halo FIXED to the owners' states
//               (only owner-ACTIVE relevant entries kept: they stay ACTIVE
//               locally, because the winner rule never lets an ACTIVE entry have
//               an ACTIVE earlier candidate with positive deviation).  Slice 0
//               is exact, and after round t slices <= t are, so this ends.
//   Y axis      X misses query the Y lists (commonFunctions.cpp:63-69); entries
//               are redistributed to Y-centre-bucket ranges (+ the same lead-in
//               halo on both sides), arrive in global processing order, and are
//               resolved and verified like X (halo neighbours on both sides; a
//               consistent assignment is unique, and the smallest wrong index
//               increases every round).
//   roots       parents (X winner, else Y winner, else self) go back to the
//               slice owners; chains are compressed inside each slice, the
//               remaining cross-slice links are resolved by request/response
//               rounds (pointer doubling); gid = global rank of the root among
//               new groups (slice offsets from an all-gather).
//   members     (in-group key, file row) records go to gid-range owners, which
//               run the exact libstdc++ introsort emulation and the emit of the
//               single-device path on their gid range = a contiguous range of
//               the global output.
//
// Every collective is an all-gather of small host metadata or an all-to-all of
// device blocks (rk_comm: RCCL send/recv over xGMI, or host callbacks).
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <initializer_list>
#include <string>
#include <vector>

#include "rk_comm.h"
#include "rk_ctx.h"

namespace rk {
namespace {

constexpr uint32_t MAXP = 32;
constexpr uint32_t NBINS = 4096;  // coarse histogram bins (LDS resident)

#define GRID_STRIDE(i, n)                                                      \
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < (n);           \
       i += gridDim.x * blockDim.x)

// owner q holds keys [b[q], b[q+1]); keys >= b[P] belong to nobody
struct Bounds {
  uint64_t b[MAXP + 1];
  uint32_t P;
};
__device__ __forceinline__ uint32_t owner_of(const Bounds &B, uint64_t key) {
  uint32_t lo = 0, hi = B.P;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (B.b[mid] <= key) lo = mid;
    else hi = mid;
  }
  return lo;
}

// ---------------------------------------------------------------- records --
// An input row on its way to its slice owner (32 B).  Received rows are used
// in place as the processing-order gather's records ({x, y}, {len, sr}):
// sr = strand byte | global file row << 32 (gather_proc reads the low byte).
struct ShardRow {
  uint64_t x, y, len, sr;
};
struct GhostX {  // an X-axis halo entry (24 B)
  uint64_t xc, len;
  uint32_t gidx, s;
};
struct YRec {  // a Y-axis entry on its way to its Y-range owner (24 B)
  uint64_t yc, len;
  uint32_t gidx, flags;  // bit 0: reverse strand, bit 1: X hit
};
struct ParRec {
  uint32_t gidx, par;
};

// ----------------------------------------------------- partition / exchange --
// An Op describes, per element i < n, the set of destination ranks (mask) and
// writes the record bound for rank d at send position pos (emit).  Positions
// are stable: rank-d records keep element order.
// mcache: masks of an earlier plan over the same elements (mread), or where
// this plan stores them (the scatter then reads them back)
// A block handles PART_TILE consecutive elements in PART_ROUNDS rounds of 256
// (round r: elements tile + 256 r + thread); per round and wave, only the
// destinations present in the wave (the OR of its masks) are balloted.
constexpr uint32_t PART_ROUNDS = 16, PART_TILE = 256 * PART_ROUNDS;
__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
  for (int off = 32; off > 0; off >>= 1) v |= (uint32_t)__shfl_xor((int)v, off);
  return v;
}
template <class Op>
__global__ void __launch_bounds__(256) k_part_count(Op op, uint32_t n, uint32_t P, uint32_t nblk,
                                                    uint32_t *cnt, uint32_t *mcache, bool mread) {
  __shared__ uint32_t bc[MAXP];
  if (threadIdx.x < MAXP) bc[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t t0 = blockIdx.x * PART_TILE + threadIdx.x;
  for (uint32_t r = 0; r < PART_ROUNDS; ++r) {
    const uint32_t i = t0 + 256 * r;
    uint32_t mask = 0u;
    if (i < n) {
      mask = mread ? mcache[i] : op.mask(i);
      if (mcache && !mread) mcache[i] = mask;
    }
    for (uint32_t any = wave_or(mask); any; any &= any - 1) {
      const uint32_t d = __builtin_ctz(any);
      const uint64_t b = __ballot((mask >> d) & 1u);
      if (lane == 0) atomicAdd(&bc[d], (uint32_t)__popcll(b));
    }
  }
  __syncthreads();
  if (threadIdx.x < P) cnt[(size_t)threadIdx.x * nblk + blockIdx.x] = bc[threadIdx.x];
}

// cap: positions at or past it are not written (a plan built from host-known
// counts whose device offsets disagree: *ovf is flagged instead)
template <class Op>
__global__ void __launch_bounds__(256) k_part_scatter(Op op, uint32_t n, uint32_t P,
                                                      uint32_t nblk, const uint32_t *off,
                                                      const uint32_t *mcache, uint32_t cap,
                                                      uint32_t *ovf) {
  // wc[r][w][d]: round r, wave w's count of destination d, then its first position
  __shared__ uint32_t wc[PART_ROUNDS][4][MAXP];
  for (uint32_t j = threadIdx.x; j < PART_ROUNDS * 4 * MAXP; j += 256) (&wc[0][0][0])[j] = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
  const uint32_t t0 = blockIdx.x * PART_TILE + threadIdx.x;
  uint32_t mask[PART_ROUNDS];
#pragma unroll
  for (uint32_t r = 0; r < PART_ROUNDS; ++r) {
    const uint32_t i = t0 + 256 * r;
    mask[r] = i < n ? (mcache ? mcache[i] : op.mask(i)) : 0u;
  }
#pragma unroll
  for (uint32_t r = 0; r < PART_ROUNDS; ++r)
    for (uint32_t any = wave_or(mask[r]); any; any &= any - 1) {
      const uint32_t d = __builtin_ctz(any);
      const uint64_t b = __ballot((mask[r] >> d) & 1u);
      if (lane == 0) wc[r][w][d] = (uint32_t)__popcll(b);
    }
  __syncthreads();
  if (threadIdx.x < P) {  // destination d: its positions in (round, wave) order
    const uint32_t d = threadIdx.x;
    uint32_t acc = off[(size_t)d * nblk + blockIdx.x];
    for (uint32_t r = 0; r < PART_ROUNDS; ++r)
      for (uint32_t v = 0; v < 4; ++v) {
        const uint32_t c = wc[r][v][d];
        wc[r][v][d] = acc;
        acc += c;
      }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t r = 0; r < PART_ROUNDS; ++r) {
    const uint32_t i = t0 + 256 * r;
    for (uint32_t any = wave_or(mask[r]); any; any &= any - 1) {
      const uint32_t d = __builtin_ctz(any);
      const uint64_t b = __ballot((mask[r] >> d) & 1u);
      if ((mask[r] >> d) & 1u) {
        const uint32_t pos = wc[r][w][d] + (uint32_t)__popcll(b & lt);
        if (pos < cap) op.emit(i, d, pos);
        else atomicOr(ovf, 1u);
      }
    }
  }
}

// a plan that keeps every element for rank 0 in element order (world size 1,
// nothing dropped): the emit at position i, no counts, scan or ballots
template <class Op>
__global__ void __launch_bounds__(256) k_part_identity(Op op, uint32_t n) {
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) op.emit(i, 0, i);
}

__global__ void k_totals(const uint32_t *off, uint32_t nblk, uint32_t P, uint32_t *tot) {
  const uint32_t d = threadIdx.x;
  if (d <= P) tot[d] = off[(size_t)d * nblk];
}

// a plan built from host-known counts: the device's own offsets must agree
// (else ERRB_INTERNAL, caught at the next agreement point; the send buffers
// of such plans are sized for every element, so a disagreement cannot write
// out of bounds)
struct Expect {
  uint32_t v[MAXP + 1];
};
__global__ void k_expect_totals(const uint32_t *off, uint32_t nblk, uint32_t P, Expect e,
                                uint32_t *flag, uint32_t bit) {
  const uint32_t d = threadIdx.x;
  if (d <= P && off[(size_t)d * nblk] != e.v[d]) atomicOr(flag, bit);
}

template <class Op>
__global__ void __launch_bounds__(256) k_hist(Op op, uint32_t n, uint32_t *hist) {
  __shared__ uint32_t h[NBINS];
  for (uint32_t b = threadIdx.x; b < NBINS; b += 256) h[b] = 0;
  __syncthreads();
  GRID_STRIDE(i, n) {
    const uint32_t b = op.bin(i);
    if (b < NBINS) atomicAdd(&h[b], 1u);
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < NBINS; b += 256)
    if (h[b]) atomicAdd(&hist[b], h[b]);
}

// -------------------------------------------------------------------- ops --
__device__ __forceinline__ uint32_t strand_code(uint64_t s) { return (uint8_t)s == 'f' ? 0u : 1u; }

struct RowOp {  // input rows -> slice owners (by xStart/10)
  const uint32_t *pkey;
  Frags f;  // this rank's rows (SoA, file order)
  Bounds B;
  uint32_t drop, shift, row_base;
  ShardRow *out;
  __device__ uint32_t bin(uint32_t i) const {
    const uint32_t k = pkey[i];
    return k < drop ? k >> shift : NBINS;
  }
  __device__ uint32_t mask(uint32_t i) const {
    const uint32_t k = pkey[i];
    return k < drop ? 1u << owner_of(B, k) : 0u;
  }
  __device__ void emit(uint32_t i, uint32_t, uint32_t pos) const {
    out[pos] = ShardRow{f.x[i], f.y[i], f.len[i],
                        (uint64_t)f.strand[i] | ((uint64_t)(row_base + i) << 32)};
  }
};

// own entries in processing order -> later slices whose lead-in they fall in.
// Only a suffix of the slice can reach a later slice (centre <= xStart +
// longest/2), so the op runs over entries base .. m-1.
struct GhostOp {
  const uint32_t *row;
  const ulonglong2 *rec;
  uint64_t thr[MAXP];  // lead-in start bucket of every slice (~0: none)
  uint32_t P, me, poff, base;
  GhostX *out;          // records, or
  uint8_t *sout;        // the entries' X states (1 = ACTIVE), same order
  const uint32_t *xg;
  __device__ uint32_t mask(uint32_t i) const {
    const uint32_t r = row[base + i];
    const uint64_t xc = rec[2 * (size_t)r].x + rec[2 * (size_t)r + 1].x / 2;
    const uint64_t bk = xc / 100;
    uint32_t m = 0;
    for (uint32_t g = me + 1; g < P; ++g)
      if (bk >= thr[g]) m |= 1u << g;
    return m;
  }
  __device__ void emit(uint32_t i, uint32_t, uint32_t pos) const {
    const uint32_t k = base + i;
    if (sout) {
      sout[pos] = xg[k] == NONE ? 1 : 0;
      return;
    }
    const uint32_t r = row[k];
    const ulonglong2 a = rec[2 * (size_t)r], b = rec[2 * (size_t)r + 1];
    out[pos] = GhostX{a.x + b.x / 2, b.x, poff + k, strand_code(b.y)};
  }
};

// relevant halo entries the owner calls ACTIVE (the fixed-halo X problem)
struct SelXOp {
  const GhostX *gh;
  const uint8_t *owner_state;
  uint64_t rel;
  GhostX *out;
  __device__ uint32_t mask(uint32_t j) const {
    return gh[j].xc / 100 >= rel && owner_state[j] ? 1u : 0u;
  }
  __device__ void emit(uint32_t j, uint32_t, uint32_t pos) const { out[pos] = gh[j]; }
};

struct YOp {  // own entries -> Y-range owners (+ their halos), processing order
  const ulonglong2 *yrec;  // {centre, length low 32 | ...} (gather_proc)
  const uint32_t *ylenhi;  // length high 32 bits (null: all lengths < 2^31)
  const uint32_t *keyy;    // strand * nby + bucket
  const uint32_t *xg;      // with xout: the X results, sent after X in the same order
  int64_t lo[MAXP], hi[MAXP];  // halo-extended ranges
  uint32_t P, poff, shift, nby;
  YRec *out;
  uint8_t *xout;
  __device__ uint32_t bin(uint32_t k) const { return (uint32_t)((yrec[k].x / 100) >> shift); }
  __device__ uint32_t mask(uint32_t k) const {
    const int64_t bk = (int64_t)(yrec[k].x / 100);
    uint32_t m = 0;
    for (uint32_t q = 0; q < P; ++q)
      if (bk >= lo[q] && bk < hi[q]) m |= 1u << q;
    return m;
  }
  __device__ void emit(uint32_t k, uint32_t, uint32_t pos) const {
    const ulonglong2 a = yrec[k];
    const uint64_t L = (a.y & 0xFFFFFFFFull) | (ylenhi ? (uint64_t)ylenhi[k] << 32 : 0ull);
    if (xout) {
      xout[pos] = xg[k] != NONE ? 1 : 0;
      return;
    }
    const uint32_t s = keyy[k] >= nby ? 1u : 0u;
    out[pos] = YRec{a.x, L, poff + k, s};  // the X-hit bit follows after X
  }
};

// One code byte per Y record held here (own range [lo, hi), relevant halo =
// buckets lo-1 and hi), written with the records' first fill; the verification
// and parent ops then read one byte per record instead of the 24-B record.
enum : uint8_t {
  YC_OWN = 0, YC_REL_LO = 1, YC_REL_HI = 2, YC_GHOST = 3,  // bits 0-1: class
  YC_FIRST = 4,   // own entry in bucket lo (a lower neighbour's relevant halo)
  YC_LAST = 8,    // own entry in bucket hi-1 (an upper neighbour's relevant halo)
  YC_XHIT = 16,   // the entry hit on X (set once X is final)
};
__device__ __forceinline__ uint8_t y_code(uint64_t b, uint64_t lo, uint64_t hi) {
  if (b >= lo && b < hi) return (b == lo ? YC_FIRST : 0) | (b + 1 == hi ? YC_LAST : 0);
  return b + 1 == lo ? YC_REL_LO : b == hi ? YC_REL_HI : YC_GHOST;
}

struct YStateOp {  // owner side: own entries in a neighbour's relevant halo
  const uint8_t *code;
  uint32_t first_mask, last_mask;  // ranks whose relevant halo holds my first / last bucket
  const uint8_t *ystate;
  uint8_t *out;
  __device__ uint32_t mask(uint32_t r) const {
    const uint8_t c = code[r];
    if (c & 3) return 0u;
    return (c & YC_FIRST ? first_mask : 0u) | (c & YC_LAST ? last_mask : 0u);
  }
  __device__ void emit(uint32_t r, uint32_t, uint32_t pos) const { out[pos] = ystate[r]; }
};

struct RelOp {  // receiver side: relevant halo entries grouped by owner
  const uint8_t *code;
  uint32_t lo_owner, hi_owner;  // owners of buckets lo-1 and hi
  uint32_t *out;
  __device__ uint32_t mask(uint32_t r) const {
    const uint8_t c = code[r] & 3;
    return c == YC_REL_LO ? 1u << lo_owner : c == YC_REL_HI ? 1u << hi_owner : 0u;
  }
  __device__ void emit(uint32_t r, uint32_t, uint32_t pos) const { out[pos] = r; }
};

struct SelYOp {  // the fixed-halo Y problem: own + relevant halo the owner calls ACTIVE
  const uint8_t *code;
  const uint8_t *used;
  uint32_t *out;
  __device__ uint32_t mask(uint32_t r) const {
    const uint8_t c = code[r], k = c & 3;
    if (k == YC_OWN) return 1u;
    return (k == YC_REL_LO || k == YC_REL_HI) && ((c & YC_XHIT) || used[r]) ? 1u : 0u;
  }
  __device__ void emit(uint32_t r, uint32_t, uint32_t pos) const { out[pos] = r; }
};

struct ParOp {  // Y decisions of own X misses -> slice owners
  const YRec *yr;
  const uint8_t *code;
  Bounds slices;
  const uint32_t *ywin;
  ParRec *out;
  __device__ uint32_t mask(uint32_t r) const {
    const uint8_t c = code[r];
    return !(c & 3) && !(c & YC_XHIT) ? 1u << owner_of(slices, yr[r].gidx) : 0u;
  }
  __device__ void emit(uint32_t r, uint32_t, uint32_t pos) const {
    out[pos] = ParRec{yr[r].gidx, ywin[r]};
  }
};

struct ReqOp {  // unresolved cross-slice roots -> the owner of their current target
  const uint32_t *lpar, *lab, *cur;
  Bounds slices;
  uint32_t *req, *src;
  __device__ uint32_t mask(uint32_t k) const {
    return lpar[k] == k && lab[k] == NONE ? 1u << owner_of(slices, cur[k]) : 0u;
  }
  __device__ void emit(uint32_t k, uint32_t, uint32_t pos) const {
    req[pos] = cur[k];
    src[pos] = k;
  }
};

struct MemOp {  // (in-group key, file row, gid) -> gid-range owners
  const uint32_t *gid;
  const ulonglong2 *hrec;  // {in-group key, GLOBAL file row}
  Bounds B;
  uint32_t shift;
  ulonglong2 *out;
  __device__ uint32_t bin(uint32_t k) const { return gid[k] >> shift; }
  __device__ uint32_t mask(uint32_t k) const { return 1u << owner_of(B, gid[k]); }
  __device__ void emit(uint32_t k, uint32_t, uint32_t pos) const {
    const ulonglong2 h = hrec[k];
    out[pos] = make_ulonglong2(h.x, (h.y & 0xFFFFFFFFull) | ((uint64_t)gid[k] << 32));
  }
};

// ---------------------------------------------------------- small kernels --
// processing keys of the received rows (used in place as records) and the
// longest length
__global__ void k_row_keys(const ulonglong2 *rec, uint32_t m, uint32_t *pkey,
                           unsigned long long *maxlen) {
  uint64_t lmax = 0;
  GRID_STRIDE(k, m) {
    pkey[k] = (uint32_t)(rec[2 * (size_t)k].x / 10);
    const uint64_t L = rec[2 * (size_t)k + 1].x;
    lmax = L > lmax ? L : lmax;
  }
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t o = __shfl_xor(lmax, off);
    lmax = o > lmax ? o : lmax;
  }
  // one atomic per block (the grid is capped): a per-wave atomic on one
  // address serialises ~m/64 updates
  __shared__ uint64_t wmax[4];
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = lmax;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t b = wmax[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) b = wmax[w] > b ? wmax[w] : b;
    if (b) atomicMax(maxlen, (unsigned long long)b);
  }
}

// Y records get their X-hit bit once X is final: the code byte and the Y
// problem's X-result word (which csr_fill_y turns into the initial state)
__global__ void k_merge_yx(uint8_t *code, const uint8_t *xh, uint32_t n, ulonglong2 *yrec) {
  GRID_STRIDE(r, n) {
    const bool h = xh[r] != 0;
    if (h) code[r] |= YC_XHIT;
    yrec[r].y = (yrec[r].y & 0xFFFFFFFFull) | ((uint64_t)(h ? 0u : NONE) << 32);
  }
}

// first k with key[k] >= v (key ascending)
__global__ void k_lower_bound(const uint32_t *key, uint32_t m, uint64_t v, uint32_t *out) {
  uint32_t lo = 0, hi = m;
  while (lo < hi) {
    const uint32_t mid = lo + (hi - lo) / 2;
    if (key[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  *out = lo;
}

__global__ void k_fill_ghost_x(const GhostX *gh, uint32_t G, ulonglong2 *xrec, uint32_t *keyx,
                               uint32_t nbx) {
  GRID_STRIDE(j, G) {
    const GhostX g = gh[j];
    xrec[j] = make_ulonglong2(g.xc, g.len);
    keyx[j] = g.s * nbx + (uint32_t)(g.xc / 100);
  }
}

// own X results (local winner ids in the Y records' high words) -> global ids
__global__ void k_x_own(const ulonglong2 *yrec_own, const GhostX *gh, uint32_t G, uint32_t poff,
                        uint32_t m, uint32_t *xg) {
  GRID_STRIDE(k, m) {
    const uint32_t w = (uint32_t)(yrec_own[k].y >> 32);
    xg[k] = w == NONE ? NONE : (w < G ? gh[w].gidx : poff + (w - G));
  }
}

__global__ void k_x_used(const ulonglong2 *yrec, uint32_t G, uint8_t *used) {
  GRID_STRIDE(j, G) used[j] = (uint32_t)(yrec[j].y >> 32) == NONE ? 1 : 0;
}

__device__ __forceinline__ void count_flag(bool f, uint32_t *cnt) {
  const uint64_t b = __ballot(f);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(cnt, (uint32_t)__popcll(b));
}

__global__ void k_cmp_x(const GhostX *gh, uint32_t G, uint64_t rel, const uint8_t *used,
                        const uint8_t *owner, uint32_t *mism) {
  for (uint32_t base = blockIdx.x * blockDim.x; base < G; base += gridDim.x * blockDim.x) {
    const uint32_t j = base + threadIdx.x;
    count_flag(j < G && gh[j].xc / 100 >= rel && used[j] != owner[j], mism);
  }
}

// the Y problem's records (all held records, or the selection ymap); the
// first fill (ymap null) also writes the code bytes
__global__ void k_fill_y(const YRec *yr, const uint32_t *ymap, uint32_t c, ulonglong2 *yrec,
                         uint32_t *ylenhi, uint32_t *keyy, uint32_t nby, uint8_t *code,
                         uint64_t lo, uint64_t hi_b) {
  GRID_STRIDE(k, c) {
    const uint32_t r = ymap ? ymap[k] : k;
    const YRec R = yr[r];
    if (!ymap) code[r] = y_code(R.yc / 100, lo, hi_b);
    const uint64_t hi = ymap && (code[r] & YC_XHIT) ? 0ull : (uint64_t)NONE;
    yrec[k] = make_ulonglong2(R.yc, (R.len & 0xFFFFFFFFull) | (hi << 32));
    if (ylenhi) ylenhi[k] = (uint32_t)(R.len >> 32);
    keyy[k] = (R.flags & 1u) * nby + (uint32_t)(R.yc / 100);
  }
}

__global__ void k_y_results(const YRec *yr, const uint8_t *code, const uint32_t *ymap, uint32_t c,
                            const uint32_t *par, uint8_t *ystate, uint32_t *ywin) {
  GRID_STRIDE(k, c) {
    const uint32_t r = ymap ? ymap[k] : k;
    if (code[r] & YC_XHIT) {
      ystate[r] = 1;
      ywin[r] = NONE;
    } else {
      const uint32_t p = par[k];
      ystate[r] = p == k ? 1 : 0;
      ywin[r] = yr[ymap ? ymap[p] : p].gidx;
    }
  }
}

__global__ void k_cmp_y(const uint32_t *relidx, uint32_t nrel, const uint8_t *used,
                        const uint8_t *owner, uint32_t *mism) {
  for (uint32_t base = blockIdx.x * blockDim.x; base < nrel; base += gridDim.x * blockDim.x) {
    const uint32_t i = base + threadIdx.x;
    count_flag(i < nrel && used[relidx[i]] != owner[i], mism);
  }
}

// used[relidx[i]] = src ? src[i] (owner states) : state[relidx[i]] (own decisions)
__global__ void k_set_used(const uint32_t *relidx, uint32_t nrel, const uint8_t *src,
                           const uint8_t *state, uint8_t *used) {
  GRID_STRIDE(i, nrel) {
    const uint32_t r = relidx[i];
    used[r] = src ? src[i] : state[r];
  }
}

__global__ void k_par_scatter(const ParRec *pr, uint32_t np, uint32_t poff, uint32_t m,
                              uint32_t *par, uint32_t *err) {
  GRID_STRIDE(i, np) {
    const ParRec p = pr[i];
    const uint32_t k = p.gidx - poff;
    if (k < m) par[k] = p.par;
    else atomicOr(err, ERRB_INTERNAL);
  }
}

// split parents into the slice-local part (for pointer jumping) and the
// cross-slice link; roots are the new groups
__global__ void k_local_par(const uint32_t *par, uint32_t m, uint32_t poff, uint32_t *lpar,
                            uint32_t *ext, uint32_t *isroot, uint32_t *err) {
  bool link = false;
  GRID_STRIDE(k, m) {
    uint32_t pg = par[k];
    if (pg == NONE || pg > poff + k) {  // parents are always earlier (or self)
      atomicOr(err, ERRB_INTERNAL);
      pg = poff + k;
    }
    const bool local = pg >= poff;
    lpar[k] = local ? pg - poff : k;
    ext[k] = local ? NONE : pg;
    link |= !local;
    isroot[k] = pg == poff + k ? 1u : 0u;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) isroot[m] = 0;
  if (__ballot(link) && (threadIdx.x & 63) == 0) atomicOr(&err[23], 1u);  // a cross-slice link
}

__global__ void k_init_labels(const uint32_t *lpar, const uint32_t *ext, const uint32_t *lrank,
                              uint32_t goff, uint32_t m, uint32_t *lab, uint32_t *cur) {
  GRID_STRIDE(k, m) {
    const bool root = lpar[k] == k;
    lab[k] = root && ext[k] == NONE ? goff + lrank[k] : NONE;
    cur[k] = root ? ext[k] : NONE;
  }
}

__global__ void k_respond(const uint32_t *rq, uint32_t nq, uint32_t poff, uint32_t m,
                          const uint32_t *lpar, const uint32_t *lab, const uint32_t *cur,
                          uint2 *resp, uint32_t *err) {
  GRID_STRIDE(i, nq) {
    const uint32_t t = rq[i] - poff;
    if (t >= m) {
      atomicOr(err, ERRB_INTERNAL);
      resp[i] = make_uint2(0, 1);
      continue;
    }
    const uint32_t r = lpar[t];
    resp[i] = lab[r] != NONE ? make_uint2(lab[r], 1u) : make_uint2(cur[r], 0u);
  }
}

__global__ void k_apply(const uint2 *back, const uint32_t *src, uint32_t n, uint32_t *lab,
                        uint32_t *cur) {
  GRID_STRIDE(i, n) {
    const uint2 b = back[i];
    const uint32_t k = src[i];
    if (b.y) lab[k] = b.x;
    else cur[k] = b.x;
  }
}

__global__ void k_final_gid(const uint32_t *lpar, const uint32_t *lab, uint32_t m,
                            uint32_t *gid, uint32_t *err) {
  GRID_STRIDE(k, m) {
    const uint32_t g = lab[lpar[k]];
    if (g == NONE) atomicOr(err, ERRB_INTERNAL);
    gid[k] = g;
  }
}

// no rank has a cross-slice link: every root is local, gid = goff + its rank
__global__ void k_final_gid_local(const uint32_t *lpar, const uint32_t *lrank, uint32_t goff,
                                  uint32_t m, uint32_t *gid) {
  GRID_STRIDE(k, m) gid[k] = goff + lrank[lpar[k]];
}

__global__ void k_mem_keys(const ulonglong2 *mem, uint32_t n, uint32_t g0, uint32_t *lg) {
  GRID_STRIDE(i, n) lg[i] = (uint32_t)(mem[i].y >> 32) - g0;
}

__global__ void k_add_u32(uint32_t *a, uint32_t n, uint32_t v) {
  GRID_STRIDE(i, n) a[i] += v;
}

// ------------------------------------------------------------- the driver --
enum Slot : int {
  SL_CTRL, SL_HIST, SL_PKEY_IN, SL_REC_IN, SL_PCNT, SL_POFF, SL_PSCAN, SL_SEND, SL_ROWS, SL_REC,
  SL_PKEY2, SL_GROW, SL_PKEY, SL_ROW, SL_TK, SL_TV, SL_RADIX, SL_SCAN, SL_GH, SL_GH2, SL_XREC,
  SL_YRECF, SL_KEYX, SL_PARF, SL_YS, SL_KEYY, SL_YLENHI, SL_XG, SL_XUSED, SL_XOWN, SL_CKEY,
  SL_CENT, SL_CCEN, SL_CLEN, SL_CSTATE, SL_CPK, SL_CNBD, SL_RUNS, SL_WPEND, SL_RPEND, SL_RLEN,
  SL_RBEG, SL_YR, SL_YMAP, SL_YRECL, SL_YLENHIL, SL_KEYYL, SL_PARL, SL_YSTATE, SL_YWIN,
  SL_YUSED, SL_RELIDX, SL_RYS, SL_PR, SL_PARG, SL_LPAR, SL_EXT, SL_ISROOT, SL_LRANK, SL_JUNK,
  SL_LAB, SL_CUR, SL_REQ, SL_SRC, SL_RQ, SL_RESP, SL_BACK, SL_HREC, SL_MEM, SL_LG, SL_SGID,
  SL_GMEM, SL_GOFF, SL_RECKEY, SL_TAG, SL_OTAG, SL_GSORT, SL_OGID, SL_OREP, SL_OORD, SL_CKEY_Y,
  SL_CENT_Y, SL_CSTATE_Y, SL_CPK_Y, SL_CNBD_Y, SL_CCEN_Y, SL_CLEN_Y, SL_TK2, SL_TV2, SL_RADIX2,
  SL_YXH, SL_YMASK, SL_YCODE, SL_GMSG, SL_JLIST, SL_COUNT
};

constexpr int kPoolSlots = 160;  // slots of both drivers (rk_shard_nw.h adds its own)

struct PartPlan {
  uint32_t n = 0, nblk = 1;
  uint32_t cap = 0xFFFFFFFFu;  // send positions written (plan_same: the expected total)
  uint32_t *off = nullptr;
  uint32_t *mcache = nullptr;  // set before plan(): masks cached there (mread: read)
  bool mread = false;
  uint64_t cnt[MAXP] = {};
  uint64_t total = 0;
};

// The driver's all-gather message (see Shard::allgather): a 16-B header whose
// first word is the sender's status, then up to GMAX payload bytes.
constexpr size_t GMAX = 2 * NBINS * 4 + 2048, GHDR = 16;  // two histograms + a few words
constexpr int STATUS_COMM_FAILED = 0x7fffffff;
int status_message(rk_comm *comm, hipStream_t st, int32_t status, const void *mine, void *all,
                   size_t bytes, uint32_t *who, std::string *err, std::vector<char> &snd,
                   std::vector<char> &rcv) {
  if (bytes > GMAX) {
    *err = "allgather payload above the fixed message size";
    return STATUS_COMM_FAILED;
  }
  const size_t P = (size_t)comm->size;
  snd.assign(GHDR + GMAX, 0);
  rcv.resize((GHDR + GMAX) * P);
  std::memcpy(snd.data(), &status, 4);
  if (bytes) std::memcpy(snd.data() + GHDR, mine, bytes);
  if (comm->allgather(snd.data(), rcv.data(), GHDR + GMAX, st)) {
    *err = "allgather: " + comm->err;
    return STATUS_COMM_FAILED;
  }
  int first = 0;
  for (size_t q = 0; q < P; ++q) {
    int32_t sq;
    std::memcpy(&sq, rcv.data() + (GHDR + GMAX) * q, 4);
    if (sq && !first) first = sq, *who = (uint32_t)q;
    if (bytes && all)
      std::memcpy((char *)all + bytes * q, rcv.data() + (GHDR + GMAX) * q + GHDR, bytes);
  }
  return first;
}

struct Shard {
  rk_ctx *ctx;
  rk_comm *comm;
  hipStream_t st;   // compute + exchanges
  hipStream_t st2;  // overlapped work (Y bucket order, in-group sort keys)
  uint32_t P, me;
  uint32_t *ctrl = nullptr;  // [0] err bits, [1] kept, [2] mismatches, [3] jump flag,
                            // [4] long-run count, [6] wide keys, [64..128) sweep
                            // counters, [128..161) partition totals
  uint64_t bytes_sent = 0;
  // elements every rank received in the last exchange (known to every rank
  // from that exchange's count all-gather: no further collective needed)
  uint64_t last_recv[MAXP] = {};
  uint32_t n_gathers = 0, n_a2a = 0, n_syncs = 0, n_agree_skipped = 0;  // (shard stats)
  uint64_t readbacks0 = 0;  // ctx->readbacks at the call's start
  // fast path (rk_shard_fast.h): plans from host-known counts flag a device
  // disagreement in *expect_flag (bit expect_bit) instead of the error word,
  // and write no send position past the expected total
  uint32_t *expect_flag = nullptr;
  uint32_t expect_bit = 0;
  // a stage whose sizes match the last completed call runs without agreement
  // points: no buffer may grow then (a growth is reported at the next gather)
  bool alloc_locked = false, alloc_violation = false;
  int sticky = 0;  // a local failure inside such a stage: reported at the next gather
  uint32_t max_sweeps[2] = {0, 0};  // the careful driver's sweeps per axis (X, Y)

  template <class T>
  T *take(int slot, size_t count) {
    rk_pool &pl = ctx->pool;
    if (pl.ptr.size() < (size_t)kPoolSlots) pl.ptr.resize(kPoolSlots, nullptr), pl.cap.resize(kPoolSlots, 0);
    const size_t need = align_up(count * sizeof(T) + 16);
    if (need > pl.cap[slot]) {
      if (alloc_locked) alloc_violation = true;
      if (pl.ptr[slot]) (void)hipFree(pl.ptr[slot]);
      pl.ptr[slot] = nullptr;
      pl.cap[slot] = 0;
      if (hipMalloc(&pl.ptr[slot], need) != hipSuccess) {
        ctx->err = "sharded workspace hipMalloc(" + std::to_string(need) + ") failed";
        throw RK_E_NOMEM;
      }
      pl.cap[slot] = need;
    }
    return reinterpret_cast<T *>(pl.ptr[slot]);
  }

  void check(int rc) {
    if (rc) throw rc;
  }
  void hip(hipError_t e, const char *what) {
    if (e != hipSuccess) {
      ctx->err = std::string(what) + ": " + hipGetErrorString(e);
      throw RK_E_HIP;
    }
  }
  void launched(const char *what) { hip(hipGetLastError(), what); }

  // Every all-gather of the driver is one fixed-size message per rank: a
  // status word plus up to GMAX payload bytes.  A rank that fails locally
  // (allocation, HIP error, consistency check) sends its status in ONE such
  // message from the top-level handler (fail_broadcast): its peers are then
  // inside their next all-gather (every all-to-all is preceded by one, see
  // exchange()), receive the status and fail together with RK_E_PEER instead
  // of waiting forever, and the comm stays in step for the next call.
  bool peer_failed = false;  // a collective reported a failure on some rank
  bool comm_broken = false;  // the comm itself failed: no further collectives
  std::vector<char> gsend, grecv;
  void allgather(const void *mine, void *all, size_t bytes) {
    if (status_gather(0, mine, all, bytes)) throw RK_E_PEER;
  }
  // returns the first non-zero status of any rank (0: every rank is fine)
  int status_gather(int32_t status, const void *mine, void *all, size_t bytes) {
    uint32_t who = 0;
    std::string cerr;
    ++n_gathers;
    const int first = status_message(comm, st, status, mine, all, bytes, &who, &cerr, gsend,
                                     grecv);
    if (first == STATUS_COMM_FAILED) {
      comm_broken = true;
      ctx->err = cerr;
      throw RK_E_HIP;
    }
    if (first) {
      peer_failed = true;
      if (!status)
        ctx->err = "rank " + std::to_string(who) + " failed (status " + std::to_string(first) +
                   "); every rank stops";
    }
    return first;
  }
  // ---- device-assembled messages (the fast path): the payload is written on
  // the device by the kernels that produce it (histograms, counts, flags) plus
  // a small host part at payload offset 0, then gathered in one collective
  // with one wait for the stream (RCCL: on the device, one copy down)
  static constexpr size_t MB = GHDR + GMAX;
  uint8_t *gdev = nullptr;
  // zeroes the header and the first dev_bytes of the payload (on the stream)
  // and returns the device payload
  uint8_t *msg_begin(size_t dev_bytes) {
    if (!gdev) gdev = take<uint8_t>(SL_GMSG, MB);
    const size_t hbytes = MB * (size_t)(P + 1);
    if (ctx->sh_msg_cap < hbytes) {
      if (ctx->sh_msg) (void)hipHostFree(ctx->sh_msg);
      ctx->sh_msg = nullptr;
      ctx->sh_msg_cap = 0;
      if (hipHostMalloc((void **)&ctx->sh_msg, hbytes, hipHostMallocDefault) != hipSuccess) {
        ctx->sh_msg = nullptr;
        ctx->err = "pinned message buffer";
        throw RK_E_NOMEM;
      }
      ctx->sh_msg_cap = hbytes;
    }
    zero(gdev, GHDR + (dev_bytes < GMAX ? dev_bytes : GMAX));
    return gdev + GHDR;
  }
  // every rank's message (payloads at msg_of(q)); returns the first non-zero
  // status (0: every rank is fine).  host: copied to payload offset 0.
  int msg_gather(int32_t status, const void *host = nullptr, size_t host_bytes = 0) {
    if (!status) status = sticky;
    if (!status && alloc_violation) {
      ctx->err = "fast path: a buffer grew inside a stage without agreement points";
      status = RK_E_INTERNAL;
    }
    char *snd = ctx->sh_msg;
    std::memset(snd, 0, GHDR);
    std::memcpy(snd, &status, 4);
    if (host_bytes) std::memcpy(snd + GHDR, host, host_bytes);
    hip(hipMemcpyAsync(gdev, snd, GHDR + host_bytes, hipMemcpyHostToDevice, st), "h2d");
    ++n_gathers;
    ++n_syncs;
    if (comm->allgather_dev(gdev, ctx->sh_msg + MB, MB, st)) {
      comm_broken = true;
      ctx->err = "allgather: " + comm->err;
      throw RK_E_HIP;
    }
    int first = 0;
    uint32_t who = 0;
    for (uint32_t q = 0; q < P; ++q) {
      int32_t sq;
      std::memcpy(&sq, ctx->sh_msg + MB * (1 + q), 4);
      if (sq && !first) first = sq, who = q;
    }
    if (first) {
      peer_failed = true;
      if (!status)
        ctx->err = "rank " + std::to_string(who) + " failed (status " + std::to_string(first) +
                   "); every rank stops";
    }
    return first;
  }
  const uint8_t *msg_of(uint32_t q) const { return (const uint8_t *)ctx->sh_msg + MB * (1 + q) + GHDR; }

  // a rank that failed outside a collective releases its peers (see allgather)
  void fail_broadcast(int code) {
    if (peer_failed || comm_broken) return;
    try {
      (void)status_gather(code ? code : RK_E_INTERNAL, nullptr, nullptr, 0);
    } catch (...) {
    }
  }
  // every rank's local status at an agreement point (before each all-to-all):
  // all continue or all fail
  void agree(int rc) {
    if (status_gather(rc, nullptr, nullptr, 0)) throw rc ? rc : (int)RK_E_PEER;
  }
  template <class T>
  std::vector<T> gather1(T v) {
    std::vector<T> all(P);
    allgather(&v, all.data(), sizeof(T));
    return all;
  }
  uint64_t sum_any(uint64_t v) {
    uint64_t s = 0;
    for (uint64_t x : gather1<uint64_t>(v)) s += x;
    return s;
  }
  std::vector<uint32_t> d2h(const uint32_t *dev, size_t count) {
    std::vector<uint32_t> h(count);
    if (count) {
      ++n_syncs;
      hip(hipMemcpyAsync(h.data(), dev, count * 4, hipMemcpyDeviceToHost, st), "d2h");
      hip(hipStreamSynchronize(st), "d2h sync");
    }
    return h;
  }
  uint32_t read1(const uint32_t *dev) { return d2h(dev, 1)[0]; }
  void zero(void *dev, size_t bytes) {
    if (bytes) hip(hipMemsetAsync(dev, 0, bytes, st), "memset");
  }

  ScanScratch scan_scratch(int slot, size_t n) {
    const size_t cap = scan_blocks(n + 1) + 64;
    return ScanScratch{take<uint32_t>(slot, cap), cap};
  }

  template <class Op>
  void plan(const Op &op, uint32_t n, PartPlan &pp) {
    pp.n = n;
    pp.nblk = n ? (n + PART_TILE - 1) / PART_TILE : 1;
    const size_t len = (size_t)P * pp.nblk + 1;
    uint32_t *cnt = take<uint32_t>(SL_PCNT, len);
    pp.off = take<uint32_t>(SL_POFF, len);
    zero(cnt + len - 1, 4);
    kt_begin(st, KID_PART);
    k_part_count<<<pp.nblk, 256, 0, st>>>(op, n, P, pp.nblk, cnt, pp.mcache, pp.mread);
    kt_end(st, KID_PART, 0.0);
    launched("k_part_count");
    exclusive_scan_u32(cnt, pp.off, len, scan_scratch(SL_PSCAN, len), st);
    k_totals<<<1, 64, 0, st>>>(pp.off, pp.nblk, P, ctrl + 128);
    launched("k_totals");
    std::vector<uint32_t> t = d2h(ctrl + 128, P + 1);
    for (uint32_t q = 0; q < P; ++q) pp.cnt[q] = t[q + 1] - t[q];
    pp.total = t[P];
  }
  // a plan whose per-destination counts are known on the host: the device
  // offsets are built, without a readback
  template <class Op>
  void plan_counts(const Op &op, uint32_t n, PartPlan &pp, const uint64_t *cnt) {
    PartPlan ref;
    ref.total = 0;
    for (uint32_t q = 0; q < MAXP; ++q) {
      ref.cnt[q] = q < P ? cnt[q] : 0;
      ref.total += ref.cnt[q];
    }
    plan_same(op, n, pp, ref);
  }
  // a plan whose host counts are known to equal `ref`'s (the same selection
  // in the same order): the device offsets are rebuilt, without a readback
  template <class Op>
  void plan_same(const Op &op, uint32_t n, PartPlan &pp, const PartPlan &ref) {
    pp.n = n;
    pp.nblk = n ? (n + PART_TILE - 1) / PART_TILE : 1;
    const size_t len = (size_t)P * pp.nblk + 1;
    uint32_t *cnt = take<uint32_t>(SL_PCNT, len);
    pp.off = take<uint32_t>(SL_POFF, len);
    zero(cnt + len - 1, 4);
    kt_begin(st, KID_PART);
    k_part_count<<<pp.nblk, 256, 0, st>>>(op, n, P, pp.nblk, cnt, pp.mcache, pp.mread);
    kt_end(st, KID_PART, 0.0);
    launched("k_part_count");
    exclusive_scan_u32(cnt, pp.off, len, scan_scratch(SL_PSCAN, len), st);
    for (uint32_t q = 0; q < MAXP; ++q) pp.cnt[q] = ref.cnt[q];
    pp.total = ref.total;
    Expect e{};
    for (uint32_t q = 0, acc = 0; q <= P; ++q) {
      e.v[q] = acc;
      if (q < P) acc += (uint32_t)ref.cnt[q];
    }
    k_expect_totals<<<1, 64, 0, st>>>(pp.off, pp.nblk, P, e, expect_flag ? expect_flag : ctrl,
                                      expect_flag ? expect_bit : (uint32_t)ERRB_INTERNAL);
    launched("k_expect_totals");
    if (expect_flag) pp.cap = (uint32_t)(ref.total < 0xFFFFFFFFull ? ref.total : 0xFFFFFFFFull);
  }
  // several device words in one round trip
  std::vector<uint32_t> d2h_words(std::initializer_list<const uint32_t *> src) {
    std::vector<uint32_t> h(src.size());
    size_t i = 0;
    for (const uint32_t *d : src)
      hip(hipMemcpyAsync(&h[i++], d, 4, hipMemcpyDeviceToHost, st), "d2h");
    ++n_syncs;
    hip(hipStreamSynchronize(st), "d2h sync");
    return h;
  }
  // world size 1 with every element selected (known on the host): the
  // identity plan, emitted by k_part_identity
  template <class Op>
  void emit_identity(const Op &op, uint32_t n, PartPlan &pp) {
    identity_plan(n, pp);
    kt_begin(st, KID_PART);
    k_part_identity<<<grid_for(n, 256, 4096), 256, 0, st>>>(op, n);
    kt_end(st, KID_PART, 0.0);
    launched("k_part_identity");
  }
  void identity_plan(uint32_t n, PartPlan &pp) {
    pp.n = n;
    pp.nblk = 1;
    for (uint32_t q = 0; q < MAXP; ++q) pp.cnt[q] = 0;
    pp.cnt[0] = n;
    pp.total = n;
  }
  // a plan that sends nothing (the op cannot select any element)
  void zero_plan(uint32_t n, PartPlan &pp) {
    pp.n = n;
    pp.nblk = 1;
    for (uint32_t q = 0; q < MAXP; ++q) pp.cnt[q] = 0;
    pp.total = 0;
  }
  template <class Op>
  void emit(const Op &op, const PartPlan &pp) {
    kt_begin(st, KID_PART);
    k_part_scatter<<<pp.nblk, 256, 0, st>>>(op, pp.n, P, pp.nblk, pp.off, pp.mcache, pp.cap,
                                            expect_flag ? expect_flag : ctrl + 7);
    kt_end(st, KID_PART, 0.0);
    launched("k_part_scatter");
  }

  // all-to-all of records (esz bytes each) laid out by plan pp in `send`;
  // returns the received count and the per-source counts
  template <class T>
  T *exchange(const void *send, const PartPlan &pp, int recv_slot, uint32_t *nrecv,
              uint64_t *from = nullptr) {
    const size_t esz = sizeof(T);
    // per destination the bytes sent, then this rank's receive-slot capacity
    const uint32_t W = P + 1;
    uint64_t msg[MAXP + 1], sb[MAXP], rb[MAXP];
    for (uint32_t q = 0; q < P; ++q) sb[q] = msg[q] = pp.cnt[q] * esz;
    {
      const rk_pool &pl = ctx->pool;
      msg[P] = (size_t)recv_slot < pl.cap.size() ? (uint64_t)pl.cap[recv_slot] : 0ull;
    }
    std::vector<uint64_t> all((size_t)P * W);
    allgather(msg, all.data(), W * sizeof(uint64_t));
    uint64_t tot = 0;
    for (uint32_t q = 0; q < P; ++q) rb[q] = all[(size_t)q * W + me], tot += rb[q];
    // every rank's receive total against its capacity -- the same data, so
    // the same decisions, on every rank
    bool too_many = false, grows = false;
    for (uint32_t r = 0; r < P; ++r) {
      uint64_t need = 0;
      for (uint32_t q = 0; q < P; ++q) need += all[(size_t)q * W + r];
      last_recv[r] = need / esz;
      too_many |= need / esz >= 0xFFFFFFFFull;
      grows |= align_up((size_t)(need / esz + 1) * esz + 16) > all[(size_t)r * W + P];
    }
    if (too_many) {
      ctx->err = "a rank would receive more than 2^32-1 records";
      throw RK_E_TOO_MANY;
    }
    // the receive buffer (its size depends on the other ranks' data: the
    // allocation most likely to fail under skew) is agreed before data moves
    // -- unless no rank has to allocate (a repeated call), when none can fail
    T *recv = nullptr;
    if (grows) {
      int rc = RK_OK;
      try {
        recv = take<T>(recv_slot, tot / esz + 1);
      } catch (int code) {
        rc = code;
      }
      agree(rc);
    } else {
      recv = take<T>(recv_slot, tot / esz + 1);  // (no allocation)
      ++n_agree_skipped;
    }
    run_a2a(send, sb, recv, rb);
    *nrecv = (uint32_t)(tot / esz);
    if (from)
      for (uint32_t q = 0; q < P; ++q) from[q] = rb[q] / esz;
    return recv;
  }
  void run_a2a(const void *send, const uint64_t *sb, void *recv, const uint64_t *rb) {
    for (uint32_t q = 0; q < P; ++q)
      if (q != me) bytes_sent += sb[q];
    double moved = 0;
    for (uint32_t q = 0; q < P; ++q) moved += (double)sb[q] + (double)rb[q];
    kt_begin(st, KID_EXCHANGE);
    ++n_a2a;
    const int rc = comm->alltoallv(send, sb, recv, rb, st);
    kt_end(st, KID_EXCHANGE, moved);  // bytes read + written (device time of the a2a)
    if (rc) {
      comm_broken = true;
      ctx->err = "alltoallv: " + comm->err;
      throw RK_E_HIP;
    }
  }

  // a bound on every rank's last received count, checked by every rank on
  // the same data (last_recv): all continue or all fail, no collective
  void check_recv_below(uint64_t lim, int code, const char *what) {
    for (uint32_t q = 0; q < P; ++q)
      if (last_recv[q] >= lim) {
        ctx->err = what;
        throw code;
      }
  }
  // device error bits agreed by every rank
  void agree_errors() { agree_error_bits(read1(ctrl)); }
  void agree_error_bits(uint32_t bits) {
    uint32_t any = 0;
    for (uint32_t b : gather1<uint32_t>(bits)) any |= b;
    check(err_status(ctx, any & ~(uint32_t)ERRB_WIDE_LENGTH));
  }
};

// Test hook: RK_TEST_FAULT=<stage> in one rank's environment makes that rank
// fail locally at <stage> (as an allocation failure would), so the tests can
// check that every peer still leaves the call with RK_E_PEER.
bool fault_here(rk_ctx *, const char *stage) {
  const char *e = std::getenv("RK_TEST_FAULT");
  return e && std::strcmp(e, stage) == 0;
}

uint32_t owner_of_host(const Bounds &B, uint64_t key) {
  uint32_t q = 0;
  while (q + 1 < B.P && B.b[q + 1] <= key) ++q;
  return q;
}

uint32_t bin_shift(uint64_t keys) {  // keys in [0, keys) -> < NBINS bins
  uint32_t s = 0;
  while (keys > 0 && ((keys - 1) >> s) >= NBINS) ++s;
  return s;
}

// balanced ownership bounds over [0, keymax) from a global bin histogram
Bounds split_bounds(const std::vector<uint64_t> &hist, uint32_t shift, uint64_t keymax,
                    uint32_t P) {
  Bounds B{};
  B.P = P;
  uint64_t total = 0;
  for (uint64_t h : hist) total += h;
  uint64_t acc = 0;
  size_t bin = 0;
  B.b[0] = 0;
  for (uint32_t q = 1; q < P; ++q) {
    const uint64_t target = (total * q + P - 1) / P;
    while (bin < hist.size() && acc < target) acc += hist[bin++];
    uint64_t v = (uint64_t)bin << shift;
    B.b[q] = v < keymax ? v : keymax;
  }
  B.b[P] = keymax;
  for (uint32_t q = P + 1; q <= MAXP; ++q) B.b[q] = keymax;
  return B;
}

// The global histogram of op's bins over every rank's n elements.  words: up
// to 16 device words read back with this rank's histogram and gathered in the
// same message (one readback, one all-gather); *gathered = every rank's words,
// rank-major
template <class Op>
std::vector<uint64_t> global_hist(Shard &S, const Op &op, uint32_t n,
                                  std::initializer_list<const uint32_t *> words = {},
                                  std::vector<uint32_t> *gathered = nullptr) {
  uint32_t *h = S.take<uint32_t>(SL_HIST, NBINS);
  S.zero(h, NBINS * 4);
  if (n) {
    k_hist<<<grid_for(n, 256, 512), 256, 0, S.st>>>(op, n, h);
    S.launched("k_hist");
  }
  const size_t K = words.size(), W = NBINS + K;
  std::vector<uint32_t> mine(W);
  S.hip(hipMemcpyAsync(mine.data(), h, NBINS * 4, hipMemcpyDeviceToHost, S.st), "d2h");
  size_t i = NBINS;
  for (const uint32_t *d : words)
    S.hip(hipMemcpyAsync(&mine[i++], d, 4, hipMemcpyDeviceToHost, S.st), "d2h");
  ++S.n_syncs;
  S.hip(hipStreamSynchronize(S.st), "d2h sync");
  std::vector<uint32_t> all((size_t)S.P * W);
  S.allgather(mine.data(), all.data(), W * 4);
  std::vector<uint64_t> g(NBINS, 0);
  for (uint32_t q = 0; q < S.P; ++q)
    for (uint32_t b = 0; b < NBINS; ++b) g[b] += all[(size_t)q * W + b];
  if (gathered) {
    gathered->resize((size_t)S.P * K);
    for (uint32_t q = 0; q < S.P; ++q)
      for (size_t k = 0; k < K; ++k) (*gathered)[q * K + k] = all[(size_t)q * W + NBINS + k];
  }
  return g;
}

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// One resolved occupancy axis over `n` entries (entry i's record in rec, its
// bucket key in key).  X: xres = the Y records (winner word), Y: xres null.
struct AxisIn {
  const ulonglong2 *rec;  // X: {centre, length}; Y: {centre, length lo | X result << 32}
  const uint32_t *ylenhi;
  uint32_t *key;
  uint32_t *par;
  uint32_t *xres;
  uint32_t n, bits;
  uint64_t max_index;
  bool is_x, fast32;
};

// device buffers of one axis' CSR and its radix sort (X and Y own separate
// sets: the Y axis is sorted on the second stream while X resolves)
struct AxisSlots {
  int key, ent, state, pk, nbd, cen, len, tk, tv, radix;
};
constexpr AxisSlots kXSlots{SL_CKEY, SL_CENT, SL_CSTATE, SL_CPK, SL_CNBD,
                           SL_CCEN, SL_CLEN, SL_TK, SL_TV, SL_RADIX};
constexpr AxisSlots kYSlots{SL_CKEY_Y, SL_CENT_Y, SL_CSTATE_Y, SL_CPK_Y, SL_CNBD_Y,
                           SL_CCEN_Y, SL_CLEN_Y, SL_TK2, SL_TV2, SL_RADIX2};

// the axis' bucket order (stable radix sort of the keys) on stream st
Csr sort_axis(Shard &S, const AxisIn &a, const AxisSlots &sl, hipStream_t st) {
  const uint32_t n = a.n;
  Csr c{};
  c.key = S.take<uint32_t>(sl.key, n + 1);
  c.ent = S.take<uint32_t>(sl.ent, n + 1);
  c.state = S.take<uint8_t>(sl.state, n + 1);
  c.pk = S.take<uint2>(sl.pk, n + 1);
  c.nbd = S.take<uint8_t>(sl.nbd, n + 1);
  c.cen = a.fast32 ? nullptr : S.take<uint64_t>(sl.cen, n + 1);
  c.len = a.fast32 ? nullptr : S.take<uint64_t>(sl.len, n + 1);
  const size_t rw = radix_scratch_words(n + 1);
  uint32_t *tk = S.take<uint32_t>(sl.tk, n + 1), *tv = S.take<uint32_t>(sl.tv, n + 1);
  uint32_t *rs = S.take<uint32_t>(sl.radix, rw);
  if (n) radix_sort_pairs(a.key, nullptr, c.key, c.ent, tk, tv, n, a.bits, rs, rw, st);
  return c;
}

// CSR columns (centre, length, neighbour code, states) and the sweeps, on the
// context stream
uint32_t sweep_axis(Shard &S, const AxisIn &a, const Csr &c, const rk_params &p) {
  const uint32_t n = a.n;
  if (!n) return 0;
  if (a.is_x) csr_fill_x(c, a.rec, n, a.max_index, S.st);
  else csr_fill_y(c, a.rec, a.ylenhi, n, a.max_index, S.st);
  S.launched("axis csr");
  Axis ax{c.key, c.ent, c.cen, c.len, c.state, a.xres, a.par, c.pk, c.nbd,
          S.take<uint32_t>(SL_RLEN, n), S.take<uint32_t>(SL_RBEG, n), n, a.max_index,
          p.len_ratio, p.pos_ratio};
  SweepScratch sc{S.take<uint32_t>(SL_RUNS, runs_scratch_words(n)),
                  S.take<uint8_t>(SL_WPEND, n / 64 + 1), S.take<uint8_t>(SL_RPEND, n),
                  S.ctrl + 64, S.ctrl + 4};
  uint32_t sweeps = 0;
  S.check(resolve_axis(S.ctx, ax, sc, a.fast32, &sweeps));
  return sweeps;
}

uint32_t resolve(Shard &S, const AxisIn &a, const AxisSlots &sl, const rk_params &p) {
  if (!a.n) return 0;
  const Csr c = sort_axis(S, a, sl, S.st);
  return sweep_axis(S, a, c, p);
}

// The Y halo check of both drivers: owners send the states of their entries in
// a neighbour's relevant halo (YStateOp); a rank whose local decisions
// disagree re-solves its Y problem with that halo fixed -- solve_y(ymap, c):
// the selected entries, arrival order -- until every rank agrees.
template <class SolveY>
void verify_y_halo(Shard &S, RelOp relop, const uint8_t *ycode, uint8_t *ystate, uint8_t *yused,
                   const Bounds &yb, uint32_t ny, SolveY &&solve_y) {
  rk_ctx *ctx = S.ctx;
  rk_shard_stats &ss = ctx->shard_stats;
  const uint32_t P = S.P, me = S.me;
  const uint64_t ylo = yb.b[me], yhi = yb.b[me + 1];
  PartPlan pp;
  // no neighbour range on either side (one rank): no relevant halo entries
  const bool lonely = ylo == 0 && yhi == yb.b[P];
  if (lonely) S.zero_plan(ny, pp);
  else S.plan(relop, ny, pp);
  const uint32_t nrel = (uint32_t)pp.total;
  uint32_t *relidx = S.take<uint32_t>(SL_RELIDX, nrel + 1);
  relop.out = relidx;
  if (!lonely) S.emit(relop, pp);
  if (nrel) {
    k_set_used<<<grid_for(nrel, 256), 256, 0, S.st>>>(relidx, nrel, nullptr, ystate, yused);
    S.launched("k_set_used");
  }
  YStateOp yso{};
  yso.code = ycode;
  yso.ystate = ystate;
  for (uint32_t q = 0; q < P; ++q) {  // whose relevant halo holds my first / last bucket
    if (q == me) continue;
    if (yb.b[q + 1] == ylo) yso.first_mask |= 1u << q;
    if (yb.b[q] == yhi) yso.last_mask |= 1u << q;
  }
  for (;;) {
    ++ss.y_rounds;
    if (ss.y_rounds > 64) {
      ctx->err = "Y halo verification did not converge";
      throw RK_E_INTERNAL;
    }
    const bool none = !yso.first_mask && !yso.last_mask;  // no neighbour reads my states
    if (none) S.zero_plan(ny, pp);
    else S.plan(yso, ny, pp);
    yso.out = S.take<uint8_t>(SL_SEND, pp.total + 1);
    if (!none) S.emit(yso, pp);
    uint32_t n2 = 0;
    uint8_t *rys = S.exchange<uint8_t>(yso.out, pp, SL_RYS, &n2);
    if (n2 != nrel) {
      ctx->err = "Y halo state count mismatch";
      throw RK_E_INTERNAL;
    }
    S.zero(S.ctrl + 2, 4);
    if (nrel) {
      k_cmp_y<<<grid_for(nrel, 256, 1024), 256, 0, S.st>>>(relidx, nrel, yused, rys,
                                                            S.ctrl + 2);
      S.launched("k_cmp_y");
    }
    const uint32_t mism = nrel ? S.read1(S.ctrl + 2) : 0u;  // no relevant halo: nothing to compare
    if (S.sum_any(mism) == 0) break;
    if (mism) {
      ++ss.y_reruns;
      k_set_used<<<grid_for(nrel, 256), 256, 0, S.st>>>(relidx, nrel, rys, nullptr, yused);
      S.launched("k_set_used");
      SelYOp sel{ycode, yused, nullptr};
      Shard S1 = S;
      S1.P = 1;
      S1.me = 0;
      PartPlan sp;
      S1.plan(sel, ny, sp);
      sel.out = S.take<uint32_t>(SL_YMAP, sp.total + 1);
      S1.emit(sel, sp);
      solve_y(sel.out, (uint32_t)sp.total);
    }
  }
}

// Roots and gids of both drivers: parents (own X winners in xg, the Y winners
// of own X misses received in prr) -> slice-local parent chains compressed by
// pointer jumping, cross-slice links by request/response rounds, gid = global
// rank of the root among new groups.  Returns the gid of every own entry
// (processing order); *Gtot = the number of groups.
const uint32_t *resolve_roots(Shard &S, uint32_t *xg, const ParRec *prr, uint32_t npar,
                              uint32_t m, uint32_t poff, const Bounds &slices, uint64_t *Gtot_out) {
  rk_ctx *ctx = S.ctx;
  rk_shard_stats &ss = ctx->shard_stats;
  const uint32_t P = S.P, me = S.me;
  PartPlan pp;
  uint32_t *parg = xg;  // X winners; the X misses' Y winners are scattered in
  uint32_t *lpar = S.take<uint32_t>(SL_LPAR, m + 1);
  uint32_t *ext = S.take<uint32_t>(SL_EXT, m + 1);
  uint32_t *isroot = S.take<uint32_t>(SL_ISROOT, m + 2);
  uint32_t *lrank = S.take<uint32_t>(SL_LRANK, m + 2);
  uint32_t *junk = S.take<uint32_t>(SL_JUNK, m + 1);
  uint32_t *lab = S.take<uint32_t>(SL_LAB, m + 1);
  uint32_t *cur = S.take<uint32_t>(SL_CUR, m + 1);
  if (m) {
    if (npar) {
      kt_begin(S.st, KID_SHARD_AUX);
      k_par_scatter<<<grid_for(npar, 256), 256, 0, S.st>>>(prr, npar, poff, m, parg, S.ctrl);
      kt_end(S.st, KID_SHARD_AUX, 0.0);
    }
    kt_begin(S.st, KID_SHARD_AUX);
    k_local_par<<<grid_for(m, 256), 256, 0, S.st>>>(parg, m, poff, lpar, ext, isroot, S.ctrl);
    kt_end(S.st, KID_SHARD_AUX, 0.0);
    S.launched("parents");
    Proc jp{};
    jp.par = lpar;
    for (uint32_t rounds = 0;; ++rounds) {
      if (rounds > 64) {
        ctx->err = "pointer jumping did not converge";
        throw RK_E_INTERNAL;
      }
      S.zero(S.ctrl + 3, 4);
      jump_round(jp, m, S.ctrl + 3, rounds == 0 ? junk : nullptr, S.ctrl, S.st);
      S.launched("jump_round");
      if (!S.read1(S.ctrl + 3)) break;
    }
    exclusive_scan_u32(isroot, lrank, (size_t)m + 1, S.scan_scratch(SL_SCAN, m + 1), S.st);
  }
  // the error bits, the root count and the cross-slice link flag: one readback
  uint32_t nroots = 0, xlink = 0, ebits = 0;
  if (m) {
    const std::vector<uint32_t> w = S.d2h_words({S.ctrl, lrank + m, S.ctrl + 23});
    ebits = w[0];
    nroots = w[1];
    xlink = w[2];
  } else {
    ebits = S.read1(S.ctrl);
  }
  // the error bits, the root count and whether this rank has a cross-slice
  // link: one all-gather
  uint64_t goff = 0, Gtot = 0;
  bool links = false;
  {
    const std::vector<uint3> rall = S.gather1<uint3>(make_uint3(ebits, nroots, xlink));
    uint32_t anyerr = 0;
    for (uint32_t q = 0; q < P; ++q) {
      anyerr |= rall[q].x;
      links |= rall[q].z != 0;
      Gtot += rall[q].y, goff += q < me ? rall[q].y : 0;
    }
    S.check(err_status(ctx, anyerr & ~(uint32_t)ERRB_WIDE_LENGTH));
  }
  if (!links) {  // every chain ends in its own slice: no label rounds
    if (m) {
      kt_begin(S.st, KID_SHARD_AUX);
      k_final_gid_local<<<grid_for(m, 256), 256, 0, S.st>>>(lpar, lrank, (uint32_t)goff, m, junk);
      kt_end(S.st, KID_SHARD_AUX, 12.0 * m);
      S.launched("k_final_gid_local");
    }
    // (no agreement point here: k_final_gid_local raises no error bits, and
    // the driver's last agreement follows)
    *Gtot_out = Gtot;
    return junk;
  }
  if (m) {
    kt_begin(S.st, KID_SHARD_AUX);
    k_init_labels<<<grid_for(m, 256), 256, 0, S.st>>>(lpar, ext, lrank, (uint32_t)goff, m, lab,
                                                        cur);
    kt_end(S.st, KID_SHARD_AUX, 0.0);
    S.launched("k_init_labels");
  }
  for (;;) {  // cross-slice links: request/response rounds (the owner answers
              // with its current knowledge, so chains halve every round)
    ReqOp rq{lpar, lab, cur, slices, nullptr, nullptr};
    S.plan(rq, m, pp);
    if (S.sum_any(pp.total) == 0) break;
    if (++ss.root_rounds > 64) {
      ctx->err = "cross-slice root resolution did not converge";
      throw RK_E_INTERNAL;
    }
    rq.req = S.take<uint32_t>(SL_REQ, pp.total + 1);
    rq.src = S.take<uint32_t>(SL_SRC, pp.total + 1);
    S.emit(rq, pp);
    uint32_t nq = 0;
    uint64_t from[MAXP];
    const uint32_t *rqs = S.exchange<uint32_t>(rq.req, pp, SL_RQ, &nq, from);
    // the response all-to-all needs its own agreement point: both buffers are
    // sized by skewed counts and the launch can fail on one rank alone
    uint2 *resp = nullptr, *back = nullptr;
    int rrc = RK_OK;
    try {
      resp = S.take<uint2>(SL_RESP, nq + 1);
      back = S.take<uint2>(SL_BACK, pp.total + 1);
      if (fault_here(ctx, "k_respond")) throw (int)RK_E_NOMEM;
      if (nq) {
        k_respond<<<grid_for(nq, 256), 256, 0, S.st>>>(rqs, nq, poff, m, lpar, lab, cur, resp,
                                                        S.ctrl);
        S.launched("k_respond");
      }
    } catch (int code) {
      rrc = code;
    }
    S.agree(rrc);
    uint64_t sb[MAXP], rb[MAXP];
    for (uint32_t q = 0; q < P; ++q) sb[q] = from[q] * sizeof(uint2), rb[q] = pp.cnt[q] * sizeof(uint2);
    S.run_a2a(resp, sb, back, rb);
    k_apply<<<grid_for((uint32_t)pp.total, 256), 256, 0, S.st>>>(back, rq.src, (uint32_t)pp.total,
                                                                  lab, cur);
    S.launched("k_apply");
  }
  uint32_t *gid_own = junk;  // the jump's scratch is free again
  if (m) {
    kt_begin(S.st, KID_SHARD_AUX);
    k_final_gid<<<grid_for(m, 256), 256, 0, S.st>>>(lpar, lab, m, gid_own, S.ctrl);
    kt_end(S.st, KID_SHARD_AUX, 0.0);
    S.launched("k_final_gid");
  }
  S.agree_errors();
  *Gtot_out = Gtot;
  return gid_own;
}

// the call's statistics and kernel timings (both drivers)
void finish_stats(Shard &S, uint32_t nl, const rk_shard_result *out,
                  std::chrono::steady_clock::time_point t0) {
  rk_ctx *ctx = S.ctx;
  rk_shard_stats &ss = ctx->shard_stats;
  if (ctx->profiling) collect_kernel_timing(ctx);
  ss.bytes_sent = S.bytes_sent;
  ss.gathers = S.n_gathers;
  ss.exchanges = S.n_a2a;
  ss.host_syncs = S.n_syncs + (uint32_t)(ctx->readbacks - S.readbacks0);
  ss.agree_skipped = S.n_agree_skipped;
  ss.ms_total = ms_since(t0);
  ctx->stats = rk_stats{};
  stats_numa_unknown(&ctx->stats);
  ctx->stats.n_in = nl;
  ctx->stats.n_proc = ss.n_slice;
  ctx->stats.n_groups = out->n_groups;
  ctx->stats.device_ms = ss.ms_total;
}

#include "rk_shard_nw.h"
#include "rk_shard_fast.h"

int classify_sharded_impl(Shard &S, const rk_frags_soa *in, const rk_params *prm,
                          int32_t lead_in, rk_shard_result *out, int pre) {
  rk_ctx *ctx = S.ctx;
  const auto t0 = std::chrono::steady_clock::now();
  rk_shard_stats &ss = ctx->shard_stats;
  std::memset(&ss, 0, sizeof ss);
  const uint32_t P = S.P, me = S.me;
  const uint64_t H = lead_in < 0 ? 2 : (uint64_t)lead_in;
  const rk_params p = pre ? rk_params{1000, 1000, 1, 1} : *prm;
  const uint64_t len_x = p.len_x_hdr + 1, len_y = p.len_y_hdr + 1;  // FragmentsDatabase.cpp:62,65
  const uint64_t vsize = 1 + len_x / 10;                             // :84
  const uint64_t max_x = len_x / 100, max_y = len_y / 100;           // SequenceOcupationList.cpp:4
  // local argument checks become this rank's status in the first collective,
  // so a rank that cannot run never leaves its peers waiting
  int rc = pre;
  if (!rc && ((!(p.len_ratio > 0) && !std::isnan(p.len_ratio)) ||
              (!(p.pos_ratio > 0) && !std::isnan(p.pos_ratio))))
    rc = RK_E_ARG;
  if (!rc && (vsize - 1 >= 0xFFFFFFF0ull || 2 * (max_x + 1) >= 0xFFFFFFF0ull ||
              2 * (max_y + 1) >= 0xFFFFFFF0ull)) {
    ctx->err = "sequence length too large for 32-bit bucket ids";
    rc = RK_E_ARG;
  }
  const uint32_t nbx = (uint32_t)(max_x + 1), nby = (uint32_t)(max_y + 1);
  const uint32_t drop = (uint32_t)(vsize - 1);  // the never-iterated last bucket

  if (!rc && ctx->profiling) {  // launch-level timing of the pipeline kernels
    ctx->kt.n = 0;
    g_ktimer = &ctx->kt;
  }
  if (!rc) {
    try {
      S.ctrl = S.take<uint32_t>(SL_CTRL, 256);
      S.zero(S.ctrl, 256 * 4);
    } catch (int code) {
      rc = code;
    }
  }

  // the record pipeline's internals when every row of every rank packs into a
  // 16-B record (rk_shard_nw.h); RK_SHARD_GENERIC=1 forces this driver
  static const bool generic_only = [] {
    const char *e = std::getenv("RK_SHARD_GENERIC");
    return e && e[0] == '1';
  }();
  // the fast path (rk_shard_fast.h) unless RK_SH_FAST=0 or the round-3 Y
  // schedule is asked for (RK_SH_YEARLY=1, the careful driver's option)
  static const bool fast_on = [] {
    const char *e = std::getenv("RK_SH_FAST"), *y = std::getenv("RK_SH_YEARLY");
    return !(e && e[0] == '0') && !(y && y[0] == '1');
  }();
  uint64_t row_base = 0, N = 0;
  if (!generic_only && fast_on) {
    int r;
    try {
      r = classify_sharded_fast(S, in, p, lead_in, out, rc, &N, &row_base);
    } catch (...) {
      std::memset(ctx->sh_fp, 0, sizeof ctx->sh_fp);
      throw;
    }
    S.expect_flag = nullptr;
    S.alloc_locked = false;
    if (r == RK_SHARD_RETRY) {
      // a halo disagreement, an axis left open, a chain longer than the
      // queued jumping rounds: every rank repeats the call the careful way
      // (with as many queued sweeps next time as it took)
      std::memset(ctx->sh_fp, 0, sizeof ctx->sh_fp);
      ss.fast_retry = 1;
      S.zero(S.ctrl, 256 * 4);
      r = classify_sharded_nw(S, in, p, P, me, N, row_base, lead_in, out, t0);
      for (int a = 0; a < 2; ++a)
        ctx->sh_blind[a] = S.max_sweeps[a] > 3 ? S.max_sweeps[a] : 3u;
    }
    if (r != RK_SHARD_FALLBACK) {
      if (r) std::memset(ctx->sh_fp, 0, sizeof ctx->sh_fp);
      finish_stats(S, (uint32_t)(rc ? 0 : in->n), out, t0);
      return r;
    }
    std::memset(ctx->sh_fp, 0, sizeof ctx->sh_fp);
    S.zero(S.ctrl, 256 * 4);
  } else {
    // ---- 0: global row numbering (rank blocks are consecutive in file
    // order); the first collective carries every rank's status
    const uint64_t n_mine = rc ? 0 : in->n;
    std::vector<uint64_t> nall(P);
    if (S.status_gather(rc, &n_mine, nall.data(), sizeof n_mine)) throw rc ? rc : (int)RK_E_PEER;
    for (uint32_t q = 0; q < P; ++q) N += nall[q], row_base += q < me ? nall[q] : 0;
  }
  if (N >= 0xFFFFFFFFull) return RK_E_TOO_MANY;  // every rank sees the same N
  const uint32_t nl = (uint32_t)in->n;
  ss.n_in = nl;
  ss.n_total = N;
  if (!generic_only && !fast_on) {
    const int r = classify_sharded_nw(S, in, p, P, me, N, row_base, lead_in, out, t0);
    if (r != RK_SHARD_FALLBACK) {
      finish_stats(S, nl, out, t0);
      return r;
    }
    S.zero(S.ctrl, 256 * 4);
  }
  ss.generic_driver = 1;

  // ---- 1: processing keys, slice bounds from the global xStart/10 histogram
  Frags f{in->x_start, in->y_start, in->length, in->strand, nl};
  uint32_t *pkey_in = S.take<uint32_t>(SL_PKEY_IN, nl + 1);
  prep_keys(f, vsize, max_x, max_y, pkey_in, nullptr, S.ctrl + 1, S.ctrl, S.st);
  S.launched("prep_keys");
  S.agree_errors();
  bool fast32 = true;
  for (uint32_t b : S.gather1<uint32_t>(S.read1(S.ctrl))) fast32 &= !(b & ERRB_WIDE_LENGTH);
  RowOp rop{pkey_in, f, {}, drop, bin_shift(drop), (uint32_t)row_base, nullptr};
  const Bounds slice_keys = split_bounds(global_hist(S, rop, nl), rop.shift, drop, P);
  rop.B = slice_keys;

  // ---- 2: rows -> slice owners; local processing order
  PartPlan pp;
  S.plan(rop, nl, pp);
  rop.out = S.take<ShardRow>(SL_SEND, pp.total + 1);
  S.emit(rop, pp);
  uint32_t m = 0;
  ShardRow *rows = S.exchange<ShardRow>(rop.out, pp, SL_ROWS, &m);
  ulonglong2 *rec = reinterpret_cast<ulonglong2 *>(rows);  // the records, in place
  uint32_t *pkey2 = S.take<uint32_t>(SL_PKEY2, m + 1);
  Proc pr{};
  pr.rec = rec;
  pr.pkey = S.take<uint32_t>(SL_PKEY, m + 1);
  pr.row = S.take<uint32_t>(SL_ROW, m + 1);
  if (m) {
    kt_begin(S.st, KID_SH_ROWKEYS);
    k_row_keys<<<grid_for(m, 256, 1024), 256, 0, S.st>>>(
        rec, m, pkey2, reinterpret_cast<unsigned long long *>(S.ctrl + 10));
    kt_end(S.st, KID_SH_ROWKEYS, 0.0);
    S.launched("k_row_keys");
    const size_t rw = radix_scratch_words(m);
    radix_sort_pairs(pkey2, nullptr, pr.pkey, pr.row, S.take<uint32_t>(SL_TK, m),
                     S.take<uint32_t>(SL_TV, m), m, bit_length(vsize - 1),
                     S.take<uint32_t>(SL_RADIX, rw), rw, S.st);
  }
  std::vector<uint64_t> mall = S.gather1<uint64_t>(m);
  uint64_t poff64 = 0, M = 0;
  for (uint32_t q = 0; q < P; ++q) M += mall[q], poff64 += q < me ? mall[q] : 0;
  const uint32_t poff = (uint32_t)poff64;
  Bounds slices{};
  slices.P = P;
  for (uint32_t q = 0, acc = 0; q <= MAXP; ++q) {
    slices.b[q] = acc;
    if (q < P) acc += (uint32_t)mall[q];
  }
  ss.n_slice = m;
  ss.ms_ingress = ms_since(t0);

  // ---- 3: X lead-in halos from earlier slices
  const auto tx = std::chrono::steady_clock::now();
  GhostOp gop{};
  gop.row = pr.row;
  gop.rec = rec;
  gop.P = P;
  gop.me = me;
  gop.poff = poff;
  for (uint32_t g = 0; g < MAXP; ++g) {
    gop.thr[g] = ~0ull;
    if (g < P && mall[g]) {
      const uint64_t bmin = slice_keys.b[g] / 10;  // xStart >= 10*key, centre >= xStart
      gop.thr[g] = bmin >= 1 + H ? bmin - 1 - H : 0;
    }
  }
  {  // the suffix of the slice whose centres can reach a later slice's lead-in
    uint64_t thr_min = ~0ull;
    for (uint32_t g = me + 1; g < P; ++g) thr_min = gop.thr[g] < thr_min ? gop.thr[g] : thr_min;
    uint32_t k0 = m;
    if (thr_min != ~0ull && m) {
      const std::vector<uint32_t> lw = S.d2h(S.ctrl + 10, 2);
      const uint64_t half = ((uint64_t)lw[0] | ((uint64_t)lw[1] << 32)) / 2;
      const uint64_t reach = thr_min * 100;  // centre >= reach is needed
      const uint64_t key0 = reach > half + 10 ? (reach - half) / 10 - 1 : 0;
      k_lower_bound<<<1, 1, 0, S.st>>>(pr.pkey, m, key0, S.ctrl + 12);
      S.launched("k_lower_bound");
      k0 = S.read1(S.ctrl + 12);
    }
    gop.base = k0;
  }
  const uint32_t nsuf = m - gop.base;
  const uint64_t bmin_me = slice_keys.b[me] / 10;
  const uint64_t rel_x = bmin_me >= 1 ? bmin_me - 1 : 0;  // relevant: probed by own queries
  S.plan(gop, nsuf, pp);
  gop.out = S.take<GhostX>(SL_SEND, pp.total + 1);
  S.emit(gop, pp);
  uint32_t G = 0;
  GhostX *gh = S.exchange<GhostX>(gop.out, pp, SL_GH, &G);
  ss.x_ghosts = G;

  // X problem = [halo (global order)] + own slice.  The own arrays sit at
  // offset G (the whole lead-in); a fixed-halo re-resolution with Gc <= G
  // halo entries uses the window [G - Gc, G + m).
  uint32_t *xg = S.take<uint32_t>(SL_XG, m + 1);
  uint8_t *xused = S.take<uint8_t>(SL_XUSED, G + 1);
  pr.ys = S.take<uint64_t>(SL_YS, m + 1);
  pr.keyy = S.take<uint32_t>(SL_KEYY, m + 1);
  pr.ylenhi = fast32 ? nullptr : S.take<uint32_t>(SL_YLENHI, m + 1);
  uint32_t *grow_proc = S.take<uint32_t>(SL_GROW, m + 1);  // global file row by processing index
  ulonglong2 *xrec_f = S.take<ulonglong2>(SL_XREC, G + m + 1);
  ulonglong2 *yrec_f = S.take<ulonglong2>(SL_YRECF, G + m + 1);
  uint32_t *keyx_f = S.take<uint32_t>(SL_KEYX, G + m + 1);
  uint32_t *par_f = S.take<uint32_t>(SL_PARF, G + m + 1);
  {
    Proc q = pr;
    q.xrec = xrec_f + G;
    q.yrec = yrec_f + G;
    q.keyx = keyx_f + G;
    q.grow = grow_proc;
    gather_proc(f, q, m, nbx, nby, S.st);
    S.launched("gather_proc");
  }
  const ulonglong2 *yrec_own = yrec_f + G;
  // the X problem's bucket order (lead-in + own) is sorted on stream 2 while
  // stream 1 exchanges the Y records
  const uint32_t xbits = (uint32_t)bit_length(2ull * nbx - 1);
  const AxisIn xa{xrec_f, nullptr, keyx_f, par_f, reinterpret_cast<uint32_t *>(yrec_f), G + m,
                  xbits, max_x, true, fast32};
  S.hip(hipEventRecord(ctx->fork, S.st), "fork");
  S.hip(hipStreamWaitEvent(S.st2, ctx->fork, 0), "fork wait");
  if (G) {
    kt_begin(S.st2, KID_SHARD_AUX);
    k_fill_ghost_x<<<grid_for(G, 256), 256, 0, S.st2>>>(gh, G, xrec_f, keyx_f, nbx);
    kt_end(S.st2, KID_SHARD_AUX, 0.0);
    S.launched("k_fill_ghost_x");
  }
  const Csr xcsr = sort_axis(S, xa, kXSlots, S.st2);
  S.hip(hipEventRecord(ctx->aux, S.st2), "x sorted");
  ss.ms_x = ms_since(tx);

  // ---- 4a: Y records -> Y-centre-bucket ranges (+ halos).  They do not depend
  // on X (the X-hit bit follows later in the same order), so the Y axis'
  // bucket order and the in-group sort keys are built on the second stream
  // while X resolves.
  const auto ty = std::chrono::steady_clock::now();
  YOp yop{};
  yop.yrec = yrec_own;
  yop.ylenhi = pr.ylenhi;
  yop.keyy = pr.keyy;
  yop.nby = nby;
  yop.xg = xg;
  yop.P = P;
  yop.poff = poff;
  yop.shift = bin_shift(nby);
  const Bounds yb = split_bounds(global_hist(S, yop, m), yop.shift, nby, P);
  for (uint32_t q = 0; q < MAXP; ++q) {
    yop.lo[q] = q < P ? (int64_t)yb.b[q] - 1 - (int64_t)H : 0;
    yop.hi[q] = q < P ? (int64_t)yb.b[q + 1] + 1 + (int64_t)H : 0;
  }
  PartPlan ypp;
  ypp.mcache = S.take<uint32_t>(SL_YMASK, m + 1);  // the X-hit bits follow the same masks
  S.plan(yop, m, ypp);
  yop.out = S.take<YRec>(SL_SEND, ypp.total + 1);
  S.emit(yop, ypp);
  uint32_t ny = 0;
  YRec *yr = S.exchange<YRec>(yop.out, ypp, SL_YR, &ny);
  ss.y_entries = ny;
  uint8_t *ycode = S.take<uint8_t>(SL_YCODE, ny + 1);
  uint8_t *ystate = S.take<uint8_t>(SL_YSTATE, ny + 1);
  uint32_t *ywin = S.take<uint32_t>(SL_YWIN, ny + 1);
  uint8_t *yused = S.take<uint8_t>(SL_YUSED, ny + 1);
  ulonglong2 *yrec_l = S.take<ulonglong2>(SL_YRECL, ny + 1);
  uint32_t *ylh_l = fast32 ? nullptr : S.take<uint32_t>(SL_YLENHIL, ny + 1);
  uint32_t *keyy_l = S.take<uint32_t>(SL_KEYYL, ny + 1);
  uint32_t *par_l = S.take<uint32_t>(SL_PARL, ny + 1);
  pr.hrec = S.take<ulonglong2>(SL_HREC, m + 1);
  const uint32_t ybits = (uint32_t)bit_length(2ull * nby - 1);
  const AxisIn ya{yrec_l, ylh_l, keyy_l, par_l, nullptr, ny, ybits, max_y, false, fast32};
  S.zero(S.ctrl + 6, 4);
  S.hip(hipEventRecord(ctx->fork, S.st), "fork");
  S.hip(hipStreamWaitEvent(S.st2, ctx->fork, 0), "fork wait");
  if (ny) {
    kt_begin(S.st2, KID_SH_FILLY);
    k_fill_y<<<grid_for(ny, 256), 256, 0, S.st2>>>(yr, nullptr, ny, yrec_l, ylh_l, keyy_l, nby,
                                                   ycode, yb.b[me], yb.b[me + 1]);
    kt_end(S.st2, KID_SH_FILLY, 0.0);
    S.launched("k_fill_y");
  }
  const Csr ycsr = sort_axis(S, ya, kYSlots, S.st2);
  {
    Proc q = pr;
    q.row = grow_proc;  // the member records carry global file rows
    sort_keys(q, m, S.ctrl + 6, S.st2);  // in-group keys, for the member stage
  }
  S.launched("stream-2 work");
  S.hip(hipEventRecord(ctx->join, S.st2), "join");
  ss.ms_y = ms_since(ty);

  // ---- 4b: X axis
  const auto tx2 = std::chrono::steady_clock::now();
  // a fixed-halo re-resolution: the selected halo in [G - Gc, G), all on stream 1
  auto solve_x = [&](const GhostX *halo, uint32_t Gc) {
    const uint32_t base = G - Gc, n = Gc + m;
    if (Gc) {
      kt_begin(S.st, KID_SHARD_AUX);
      k_fill_ghost_x<<<grid_for(Gc, 256), 256, 0, S.st>>>(halo, Gc, xrec_f + base,
                                                         keyx_f + base, nbx);
      kt_end(S.st, KID_SHARD_AUX, 0.0);
      S.launched("k_fill_ghost_x");
    }
    AxisIn a{xrec_f + base, nullptr, keyx_f + base, par_f + base,
             reinterpret_cast<uint32_t *>(yrec_f + base), n,
             (uint32_t)bit_length(2ull * nbx - 1), max_x, true, fast32};
    resolve(S, a, kXSlots, p);
    if (m) {
      kt_begin(S.st, KID_SH_XOWN);
      k_x_own<<<grid_for(m, 256), 256, 0, S.st>>>(yrec_f + G, halo, Gc, poff, m, xg);
      kt_end(S.st, KID_SH_XOWN, 0.0);
      S.launched("k_x_own");
    }
  };
  S.hip(hipStreamWaitEvent(S.st, ctx->aux, 0), "x sorted wait");
  sweep_axis(S, xa, xcsr, p);
  if (m) {
    kt_begin(S.st, KID_SH_XOWN);
    k_x_own<<<grid_for(m, 256), 256, 0, S.st>>>(yrec_f + G, gh, G, poff, m, xg);
    kt_end(S.st, KID_SH_XOWN, 0.0);
    S.launched("k_x_own");
  }
  if (G) {
    k_x_used<<<grid_for(G, 256), 256, 0, S.st>>>(yrec_f, G, xused);
    S.launched("k_x_used");
  }
  for (;;) {  // verify the relevant halo against its owners' decisions
    ++ss.x_rounds;
    if (ss.x_rounds > P + 2) {
      ctx->err = "X halo verification did not converge";
      throw RK_E_INTERNAL;
    }
    GhostOp sop = gop;
    sop.out = nullptr;
    sop.xg = xg;
    S.plan(sop, nsuf, pp);
    sop.sout = S.take<uint8_t>(SL_SEND, pp.total + 1);
    S.emit(sop, pp);
    uint32_t G2 = 0;
    uint8_t *xown = S.exchange<uint8_t>(sop.sout, pp, SL_XOWN, &G2);
    if (G2 != G) {
      ctx->err = "X halo state count mismatch";
      throw RK_E_INTERNAL;
    }
    S.zero(S.ctrl + 2, 4);
    if (G) {
      k_cmp_x<<<grid_for(G, 256, 1024), 256, 0, S.st>>>(gh, G, rel_x, xused, xown, S.ctrl + 2);
      S.launched("k_cmp_x");
    }
    const uint32_t mism = S.read1(S.ctrl + 2);
    if (S.sum_any(mism) == 0) break;
    if (mism) {  // re-resolve with the halo fixed to the owners' states
      ++ss.x_reruns;
      SelXOp sel{gh, xown, rel_x, nullptr};
      PartPlan sp;
      Shard S1 = S;
      S1.P = 1;
      S1.me = 0;
      S1.plan(sel, G, sp);
      sel.out = S.take<GhostX>(SL_GH2, sp.total + 1);
      S1.emit(sel, sp);
      solve_x(sel.out, (uint32_t)sp.total);
      hipError_t e = hipMemcpyAsync(xused, xown, G, hipMemcpyDeviceToDevice, S.st);
      S.hip(e, "xused copy");
    }
  }
  ss.ms_x += ms_since(tx2);

  // ---- 4c: the X-hit bits follow the Y records (same plan, same order); the
  // Y axis resolves on the bucket order stream 2 built
  const auto ty2 = std::chrono::steady_clock::now();
  {
    YOp xop = yop;
    xop.out = nullptr;
    PartPlan xpp;
    xpp.mcache = ypp.mcache;
    xpp.mread = true;
    S.plan(xop, m, xpp);
    xop.xout = S.take<uint8_t>(SL_SEND, xpp.total + 1);
    S.emit(xop, xpp);
    uint32_t n2 = 0;
    const uint8_t *xh = S.exchange<uint8_t>(xop.xout, xpp, SL_YXH, &n2);
    if (n2 != ny) {
      ctx->err = "Y X-hit count mismatch";
      throw RK_E_INTERNAL;
    }
    S.hip(hipStreamWaitEvent(S.st, ctx->join, 0), "join wait");
    if (ny) {
      kt_begin(S.st, KID_SH_MERGE);
      k_merge_yx<<<grid_for(ny, 256), 256, 0, S.st>>>(ycode, xh, ny, yrec_l);
      kt_end(S.st, KID_SH_MERGE, 0.0);
      S.launched("k_merge_yx");
    }
  }
  auto y_results = [&](const uint32_t *ymap, uint32_t c, const uint32_t *par) {
    if (!c) return;
    kt_begin(S.st, KID_SH_YRES);
    k_y_results<<<grid_for(c, 256), 256, 0, S.st>>>(yr, ycode, ymap, c, par, ystate, ywin);
    kt_end(S.st, KID_SH_YRES, 0.0);
    S.launched("k_y_results");
  };
  sweep_axis(S, ya, ycsr, p);
  y_results(nullptr, ny, par_l);
  // a fixed-halo re-resolution: the selected records, sorted again on stream 1
  auto solve_y = [&](const uint32_t *ymap, uint32_t c) {
    if (!c) return;
    kt_begin(S.st, KID_SH_FILLY);
    k_fill_y<<<grid_for(c, 256), 256, 0, S.st>>>(yr, ymap, c, yrec_l, ylh_l, keyy_l, nby,
                                                  ycode, 0, 0);
    kt_end(S.st, KID_SH_FILLY, 0.0);
    S.launched("k_fill_y");
    AxisIn a{yrec_l, ylh_l, keyy_l, par_l, nullptr, c, ybits, max_y, false, fast32};
    resolve(S, a, kYSlots, p);
    y_results(ymap, c, par_l);
  };
  // relevant halo entries grouped by owner (the order owners send their states in)
  const uint64_t ylo = yb.b[me], yhi = yb.b[me + 1];
  const RelOp relop{ycode, ylo ? owner_of_host(yb, ylo - 1) : 0u,
                    yhi < nby ? owner_of_host(yb, yhi) : 0u, nullptr};
  verify_y_halo(S, relop, ycode, ystate, yused, yb, ny, solve_y);
  ss.ms_y += ms_since(ty2);


  // ---- 5: parents back to the slice owners; roots; gids
  const auto tr = std::chrono::steady_clock::now();
  ParOp pop{yr, ycode, slices, ywin, nullptr};
  S.plan(pop, ny, pp);
  pop.out = S.take<ParRec>(SL_SEND, pp.total + 1);
  S.emit(pop, pp);
  uint32_t npar = 0;
  const ParRec *prr = S.exchange<ParRec>(pop.out, pp, SL_PR, &npar);
  uint64_t Gtot = 0;
  const uint32_t *gid_own = resolve_roots(S, xg, prr, npar, m, poff, slices, &Gtot);
  ss.ms_roots = ms_since(tr);

  // ---- 6: members -> gid-range owners; exact in-group order; emit
  const auto tm = std::chrono::steady_clock::now();
  bool narrow = true;  // the sort keys came from stream 2 (joined before the Y sweeps)
  for (uint32_t w : S.gather1<uint32_t>(S.read1(S.ctrl + 6))) narrow &= w == 0;
  MemOp mop{gid_own, pr.hrec, {}, bin_shift(Gtot), nullptr};
  const Bounds gb = split_bounds(global_hist(S, mop, m), mop.shift, Gtot, P);
  mop.B = gb;
  S.plan(mop, m, pp);
  mop.out = S.take<ulonglong2>(SL_SEND, pp.total + 1);
  S.emit(mop, pp);
  uint32_t mr = 0;
  ulonglong2 *mem = S.exchange<ulonglong2>(mop.out, pp, SL_MEM, &mr);
  const uint32_t g0 = (uint32_t)gb.b[me], Gl = (uint32_t)(gb.b[me + 1] - gb.b[me]);
  uint32_t *ogid = S.take<uint32_t>(SL_OGID, mr + 1);
  uint8_t *orep = S.take<uint8_t>(SL_OREP, mr + 1);
  uint32_t *oord = S.take<uint32_t>(SL_OORD, mr + 1);
  if (mr) {
    uint32_t *lg = S.take<uint32_t>(SL_LG, mr + 1);
    uint32_t *sgid = S.take<uint32_t>(SL_SGID, mr + 1);
    uint32_t *gmem = S.take<uint32_t>(SL_GMEM, mr + 1);
    uint32_t *goffs = S.take<uint32_t>(SL_GOFF, (size_t)Gl + 2);
    uint64_t *reckey = S.take<uint64_t>(SL_RECKEY, mr + 1);
    uint32_t *tag = S.take<uint32_t>(SL_TAG, mr + 1);
    uint32_t *otag = S.take<uint32_t>(SL_OTAG, mr + 1);
    void *gsort = S.take<uint8_t>(SL_GSORT, groupsort_scratch_bytes(mr));
    kt_begin(S.st, KID_SHARD_AUX);
    k_mem_keys<<<grid_for(mr, 256), 256, 0, S.st>>>(mem, mr, g0, lg);
    kt_end(S.st, KID_SHARD_AUX, 0.0);
    S.launched("k_mem_keys");
    const size_t rw = radix_scratch_words(mr);
    radix_sort_pairs(lg, nullptr, sgid, gmem, S.take<uint32_t>(SL_TK, mr),
                     S.take<uint32_t>(SL_TV, mr), mr, bit_length(Gl ? Gl - 1 : 0),
                     S.take<uint32_t>(SL_RADIX, rw), rw, S.st);
    group_offsets(sgid, mr, Gl, goffs, S.st);
    build_records(gmem, mem, mr, reckey, tag, S.st);
    // the group-sort tiers on both streams, as in the single-device path
    S.check(sort_groups_exact(sgid, goffs, Gl, mr, reckey, tag, otag, gsort,
                              S.scan_scratch(SL_SCAN, mr + Gl + 2), ctx->host + 128, narrow, S.st,
                              S.st2 != S.st ? S.st2 : nullptr, ctx->fork, ctx->join));
    emit_result(otag, sgid, goffs, gmem, mr, ogid, orep, oord, S.st);
    if (g0) k_add_u32<<<grid_for(mr, 256), 256, 0, S.st>>>(ogid, mr, g0);
    S.launched("member order");
  }
  std::vector<uint64_t> oall = S.gather1<uint64_t>(mr);
  uint64_t ooff = 0, otot = 0;
  for (uint32_t q = 0; q < P; ++q) otot += oall[q], ooff += q < me ? oall[q] : 0;
  S.hip(hipStreamSynchronize(S.st), "final sync");
  S.agree_errors();
  ss.ms_members = ms_since(tm);

  out->out_order = oord;
  out->gid = ogid;
  out->repval = orep;
  out->n_out = mr;
  out->out_offset = ooff;
  out->n_out_total = otot;
  out->n_groups = Gtot;
  finish_stats(S, nl, out, t0);
  (void)M;
  return RK_OK;
}

// A rank that cannot run the call at all joins its peers' first collective
// with a failure status, so that they stop too.
int status_broadcast(rk_comm *comm, int status) {
  std::vector<char> a, b;
  uint32_t who = 0;
  std::string err;
  const int r = status_message(comm, nullptr, status, nullptr, nullptr, 0, &who, &err, a, b);
  return r == STATUS_COMM_FAILED ? RK_E_HIP : RK_OK;
}

// A failure on one rank becomes a failure of every rank (Shard::allgather):
// `pre` is a status this rank already has (e.g. its input upload failed).
int classify_sharded(rk_ctx *ctx, rk_comm *comm, const rk_frags_soa *in, const rk_params *prm,
                     int32_t lead_in, rk_shard_result *out, int pre) {
  if (!comm || comm->size < 1 || (uint32_t)comm->size > MAXP) return RK_E_ARG;
  if (!ctx) {
    (void)status_broadcast(comm, RK_E_ARG);
    return RK_E_ARG;
  }
  int rc = pre;
  if (!rc && (!in || !prm || !out)) rc = RK_E_ARG;
  if (!rc && in->n && (!in->x_start || !in->y_start || !in->length || !in->strand))
    rc = RK_E_ARG;
  if (hipSetDevice(ctx->device) != hipSuccess) {
    ctx->err = "hipSetDevice failed";
    if (!rc) rc = RK_E_HIP;
  }
  Shard S{ctx, comm, ctx->stream, ctx->stream2, (uint32_t)comm->size, (uint32_t)comm->rank};
  S.readbacks0 = ctx->readbacks;
  try {
    return classify_sharded_impl(S, in, prm, lead_in, out, rc);
  } catch (int code) {
    S.fail_broadcast(code);  // no-op when the failure is already shared
    throw;
  } catch (...) {
    S.fail_broadcast(RK_E_INTERNAL);
    throw;
  }
}

}  // namespace
}  // namespace rk

static int classify_sharded_entry(rk_ctx *ctx, rk_comm *comm, const rk_frags_soa *in_dev,
                                  const rk_params *p, int32_t lead_in, rk_shard_result *out,
                                  int pre) {
  int rc;
  try {
    rc = rk::classify_sharded(ctx, comm, in_dev, p, lead_in, out, pre);
  } catch (int code) {
    rc = code;
  } catch (...) {
    ctx->err = "unexpected C++ exception";
    rc = RK_E_INTERNAL;
  }
  rk::g_ktimer = nullptr;
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->stream2) (void)hipStreamSynchronize(ctx->stream2);
  return rc;
}

extern "C" int rk_classify_sharded(rk_ctx *ctx, rk_comm *comm, const rk_frags_soa *in_dev,
                                   const rk_params *p, int32_t lead_in, rk_shard_result *out) {
  if (!ctx) return rk::classify_sharded(ctx, comm, in_dev, p, lead_in, out, RK_E_ARG);
  ctx->err.clear();
  return classify_sharded_entry(ctx, comm, in_dev, p, lead_in, out, RK_OK);
}

extern "C" int rk_get_shard_stats(const rk_ctx *ctx, rk_shard_stats *st) {
  if (!ctx || !st) return RK_E_ARG;
  *st = ctx->shard_stats;
  return RK_OK;
}

extern "C" int rk_shard_copy_result(rk_ctx *ctx, const rk_shard_result *res, uint32_t *out_order,
                                    uint32_t *gid, uint8_t *repval) {
  if (!ctx || !res) return RK_E_ARG;
  const size_t n = res->n_out;
  if (!n) return RK_OK;
  if (!out_order || !gid || !repval) return RK_E_ARG;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  HIPCHK(ctx, hipMemcpyAsync(out_order, res->out_order, n * 4, hipMemcpyDefault, ctx->stream));
  HIPCHK(ctx, hipMemcpyAsync(gid, res->gid, n * 4, hipMemcpyDefault, ctx->stream));
  HIPCHK(ctx, hipMemcpyAsync(repval, res->repval, n, hipMemcpyDefault, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return RK_OK;
}

extern "C" int rk_classify_sharded_host(rk_ctx *ctx, rk_comm *comm, const rk_frags_soa *in,
                                        const rk_params *p, int32_t lead_in,
                                        rk_shard_result *out) {
  if (!ctx) return rk::classify_sharded(ctx, comm, in, p, lead_in, out, RK_E_ARG);
  ctx->err.clear();
  // a failure here is this rank's status in the first collective of
  // classify_sharded, so the peers stop with it instead of waiting
  int pre = RK_OK;
  const size_t n = in ? in->n : 0;
  if (!in || (n && (!in->x_start || !in->y_start || !in->length || !in->strand))) pre = RK_E_ARG;
  if (!pre && hipSetDevice(ctx->device) != hipSuccess) pre = RK_E_HIP;
  const size_t need = rk::align_up(n * 8 + 16) * 3 + rk::align_up(n + 16);
  if (!pre && need > ctx->io_cap) {
    if (ctx->io) (void)hipFree(ctx->io);
    ctx->io = nullptr;
    ctx->io_cap = 0;
    if (hipMalloc(&ctx->io, need) != hipSuccess) {
      ctx->err = "sharded input hipMalloc(" + std::to_string(need) + ") failed";
      pre = RK_E_NOMEM;
    } else {
      ctx->io_cap = need;
    }
  }
  rk_frags_soa din{nullptr, nullptr, nullptr, nullptr, 0};
  if (!pre) {
    rk::Carve c{(char *)ctx->io};
    uint64_t *dx = c.take<uint64_t>(n), *dy = c.take<uint64_t>(n), *dl = c.take<uint64_t>(n);
    uint8_t *ds = c.take<uint8_t>(n);
    if (n && (hipMemcpyAsync(dx, in->x_start, n * 8, hipMemcpyHostToDevice, ctx->stream) ||
              hipMemcpyAsync(dy, in->y_start, n * 8, hipMemcpyHostToDevice, ctx->stream) ||
              hipMemcpyAsync(dl, in->length, n * 8, hipMemcpyHostToDevice, ctx->stream) ||
              hipMemcpyAsync(ds, in->strand, n, hipMemcpyHostToDevice, ctx->stream))) {
      ctx->err = "sharded input upload failed";
      pre = RK_E_HIP;
    }
    din = rk_frags_soa{dx, dy, dl, ds, n};
  }
  return classify_sharded_entry(ctx, comm, &din, p, lead_in, out, pre);
}

extern "C" int rk_comm_abandon(rk_comm *comm, int status) {
  if (!comm) return RK_E_ARG;
  return rk::status_broadcast(comm, status ? status : RK_E_INTERNAL);
}
