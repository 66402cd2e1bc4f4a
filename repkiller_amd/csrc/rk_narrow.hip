// rk_narrow.hip -- the record-carrying single-device pipeline (gfx950).
//
// The same classification as the generic pipeline (rk_groups.hip +
// rk_radix.hip: generate_fragment_groups + generate_diagonal_func +
// sort_groups, commonFunctions.cpp:41-177), laid out to move as few HBM bytes
// as possible.  It applies when every fragment packs into a 16-B record
// ("narrow": length < 2^24, yStart < 2^35; n < 2^30) -- every BASELINE config
// does; anything else takes the generic pipeline.
//
// What moves instead of random gathers:
//   * processing order (FragmentsDatabase buckets, FragmentsDatabase.cpp:84-97)
//     is a stable LSD sort of 16-B records {xStart/10, row, yStart lo,
//     length | strand | yStart hi | xStart%10} straight from the file-order
//     SoA: the records carry everything later stages read, so nothing is
//     gathered back by row;
//   * every sort is a one-sweep LSD radix: ONE histogram for all of its digits
//     (fused into the kernel that produces the keys), then per pass one kernel
//     that ranks a tile in LDS by wave ballots, gets each digit's global
//     offset by a decoupled look-back over the preceding tiles' published
//     counts, and writes the tile out digit segment by digit segment;
//   * the X occupancy axis (SequenceOcupationList buckets of centre/100,
//     SequenceOcupationList.cpp:17,95) is NOT sorted at all: a centre lies at
//     most max(len)/2 after xStart, so in processing order (sorted by
//     xStart/10) every chunk of W buckets is fed by a contiguous row range
//     plus a short halo; one kernel orders each chunk's entries in LDS (stable
//     by processing index) and places them by a look-back over the chunks;
//     the same kernel computes each row's in-group sort key
//     |yStart - diag_func[xStart/10]| (diag_func[b] = yStart of the LAST row
//     of bucket b, commonFunctions.cpp:161-177) from the bucket runs it holds;
//   * the Y axis records (12 B: {bucket key, processing index, length |
//     centre%100 << 24}) are written by the last processing-order pass and sorted on the second
//     stream while X resolves; the X results reach the Y axis through one
//     byte per fragment (xhit);
//   * group members {gid, row, sort key} are sorted by gid with the records
//     carried (12 B when every sort key fits 32 bits, else 16 B), straight
//     into the arrays the in-group sort reads.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <utility>

#include "rk_ctx.h"

namespace rk {
namespace {

#include "rk_onesweep.h"

// ---------------------------------------------------------------------------
// the 16-B processing-order record
//   x: xStart / 10 (the processing key; the dropped last bucket -> vsize - 1)
//   y: file row
//   z: yStart low 32 bits
//   w: length (24) | strand != 'f' (1) | yStart >> 32 (3) | xStart % 10 (4)
__device__ __forceinline__ uint64_t rec_x(const uint4 &r) {
  return (uint64_t)r.x * 10 + (r.w >> 28);
}
__device__ __forceinline__ uint64_t rec_y(const uint4 &r) {
  return ((uint64_t)((r.w >> 25) & 7u) << 32) | r.z;
}
__device__ __forceinline__ uint32_t rec_len(const uint4 &r) { return r.w & 0xFFFFFFu; }
__device__ __forceinline__ uint32_t rec_strand(const uint4 &r) { return (r.w >> 24) & 1u; }

__device__ __forceinline__ uint8_t nbd_code_nw(uint64_t c, uint64_t max_index) {
  const int d = neighbour_dir(c, max_index);
  return d < 0 ? 1 : d > 0 ? 2 : 0;
}

// largest bucket index get_associated_group touches for centre c
__device__ __forceinline__ uint64_t probe_max_bucket_nw(uint64_t c, uint64_t max_index) {
  if (c < (1ull << 32) - 2 && max_index != 0 && max_index < (1ull << 32)) {
    // the same in 32 bits (no wrap of c + 2 or max_index - 1 here)
    const uint32_t c32 = (uint32_t)c, m32 = (uint32_t)max_index;
    uint32_t b = c32 / 100u;
    if (c32 < m32 && (c32 + 1) / 100u > b) b = (c32 + 1) / 100u;
    if (c32 < m32 - 1 && (c32 + 2) / 100u > b) b = (c32 + 2) / 100u;
    return b;
  }
  uint64_t b = c / 100;
  if (c < max_index && (c + 1) / 100 > b) b = (c + 1) / 100;
  if (c < max_index - 1 && (c + 2) / 100 > b) b = (c + 2) / 100;
  return b;
}
__device__ __forceinline__ uint64_t div_small(uint64_t v, uint32_t d) {  // 32-bit when it fits
  return v < (1ull << 32) ? (uint64_t)((uint32_t)v / d) : v / d;
}

// digits of one LSD sort: pass p sorts by (key >> shift[p]) & (2^db[p] - 1)
struct Digits {
  int passes;
  int shift[4], db[4];
  __device__ __forceinline__ uint32_t digit(int p, uint32_t key) const {
    return (key >> shift[p]) & ((1u << db[p]) - 1u);
  }
};

// per-block LDS histogram of every digit of a sort (HW = 4 x 1024 words), flushed
// with one global atomic per non-zero bin
struct HistLds {
  uint32_t h[4 * 1024];
};
__device__ __forceinline__ void hist_init(HistLds &L) {
  for (uint32_t j = threadIdx.x; j < 4 * 1024; j += blockDim.x) L.h[j] = 0;
}
__device__ __forceinline__ void hist_add(HistLds &L, const Digits &D, uint32_t key) {
  for (int p = 0; p < D.passes; ++p) atomicAdd(&L.h[p * 1024 + D.digit(p, key)], 1u);
}
__device__ __forceinline__ void hist_flush(HistLds &L, const Digits &D, uint32_t *g) {
  for (int p = 0; p < D.passes; ++p)
    for (uint32_t j = threadIdx.x; j < (1u << D.db[p]); j += blockDim.x)
      if (L.h[p * 1024 + j]) atomicAdd(&g[p * 1024 + j], L.h[p * 1024 + j]);
}

// records in a uint4 array, key = .x (streamed once: nontemporal loads)
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
struct SrcRec {
  using rec_t = uint4;
  const uint4 *in;
  uint32_t sub = 0;  // key base (the sharded driver's slice-relative coarse keys)
  __device__ __forceinline__ uint4 load(uint32_t i) const {
    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(in + i));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  __device__ __forceinline__ uint32_t key(const uint4 &r) const { return r.x - sub; }
};
// 12-B records (the Y axis' records, and the member records when every sort
// key fits 32 bits), key = .x
struct SrcRec12 {
  using rec_t = uint3;
  const uint3 *in;
  __device__ __forceinline__ uint3 load(uint32_t i) const {
    const uint32_t *p = reinterpret_cast<const uint32_t *>(in + i);
    return make_uint3(__builtin_nontemporal_load(p), __builtin_nontemporal_load(p + 1),
                      __builtin_nontemporal_load(p + 2));
  }
  __device__ __forceinline__ uint32_t key(const uint3 &r) const { return r.x; }
};
// the member records of the X chunk kernel ({row, key low} + key high) with
// the gid from its own array, as 12-B {gid, row, key} or 16-B {gid, row, key
// low, key high} records
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
struct SrcMem12 {
  using rec_t = uint3;
  const uint2 *erk;
  const uint32_t *gid;
  __device__ __forceinline__ uint3 load(uint32_t i) const {
    const v2u v = __builtin_nontemporal_load(reinterpret_cast<const v2u *>(erk + i));
    return make_uint3(__builtin_nontemporal_load(gid + i), v.x, v.y);
  }
  __device__ __forceinline__ uint32_t key(const uint3 &r) const { return r.x; }
};
struct SrcMem16 {
  using rec_t = uint4;
  const uint2 *erk;
  const uint32_t *ehi, *gid;
  __device__ __forceinline__ uint4 load(uint32_t i) const {
    const v2u v = __builtin_nontemporal_load(reinterpret_cast<const v2u *>(erk + i));
    return make_uint4(__builtin_nontemporal_load(gid + i), v.x, v.y,
                      __builtin_nontemporal_load(ehi + i));
  }
  __device__ __forceinline__ uint32_t key(const uint4 &r) const { return r.x; }
};
// Dst::wave(rec, live): called by every lane of a wave for consecutive
// sorted slots of the tile (kWave = false: not at all)
#define RK_NO_WAVE                   \
  static constexpr bool kWave = false; \
  static constexpr bool kPre = false;  \
  template <class R_>                  \
  __device__ __forceinline__ void wave(const R_ &, bool) const {}
struct DstRec {
  RK_NO_WAVE
  uint4 *out;
  __device__ __forceinline__ void store(uint32_t pos, const uint4 &r) const { out[pos] = r; }
};
struct DstRec12 {
  RK_NO_WAVE
  uint3 *out;
  __device__ __forceinline__ void store(uint32_t pos, const uint3 &r) const {
    uint32_t *p = reinterpret_cast<uint32_t *>(out + pos);
    p[0] = r.x, p[1] = r.y, p[2] = r.z;
  }
};

// arr[v] += the length of every run of equal v != NONE over consecutive lanes
// (one atomic per run: sorted records repeat their chunk ids; arr in LDS)
__device__ __forceinline__ void wave_run_add(uint32_t v, uint32_t *arr) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t pv = __shfl_up(v, 1), nv = __shfl_down(v, 1);
  const bool head = v != NONE && (lane == 0 || pv != v);
  const uint64_t tails = __ballot(v != NONE && (lane == 63 || nv != v));
  if (head) {
    const uint32_t e = __builtin_ctzll(tails & ~((1ull << lane) - 1ull));
    atomicAdd(&arr[v], e - lane + 1);
  }
}

// --- processing order, pass 1: the file-order rows become records ---------
// A row source gives row i's (xStart, yStart, length, strand != 'f'): the
// caller's SoA in HBM, or the 12-B wire rows rk_classify uploads (packed on
// the host: {xStart lo 32, yStart lo 32, length (24) | reverse (1) | yStart
// >> 32 (3) | xStart >> 32 (4)}, rk_io.hip)
// (raw: the row's loads only; unpack: what is computed from them -- a Src
// with raw_t has every item's loads issued before any is used, see k_onesweep)
struct RowSoA {
  const uint64_t *x, *y, *len;
  const uint8_t *strand;
  struct raw_t {
    uint64_t x, y, L;
    uint8_t s;
  };
  __device__ __forceinline__ raw_t raw(uint32_t i) const { return raw_t{x[i], y[i], len[i], strand[i]}; }
  __device__ __forceinline__ void unpack(const raw_t &r, uint64_t &xs, uint64_t &ys, uint64_t &L,
                                         uint32_t &s) const {
    xs = r.x, ys = r.y, L = r.L;
    s = r.s != 'f' ? 1u : 0u;
  }
  __device__ __forceinline__ void row(uint32_t i, uint64_t &xs, uint64_t &ys, uint64_t &L,
                                      uint32_t &s) const {
    unpack(raw(i), xs, ys, L, s);
  }
};
struct RowWire {
  const uint3 *w;
  using raw_t = uint3;
  __device__ __forceinline__ raw_t raw(uint32_t i) const {
    const uint32_t *p = reinterpret_cast<const uint32_t *>(w + i);
    return make_uint3(__builtin_nontemporal_load(p), __builtin_nontemporal_load(p + 1),
                      __builtin_nontemporal_load(p + 2));
  }
  __device__ __forceinline__ void unpack(const raw_t &r, uint64_t &xs, uint64_t &ys, uint64_t &L,
                                         uint32_t &s) const {
    xs = (uint64_t)(r.z >> 28) << 32 | r.x;
    ys = (uint64_t)((r.z >> 25) & 7u) << 32 | r.y;
    L = r.z & 0xFFFFFFu;
    s = (r.z >> 24) & 1u;
  }
  __device__ __forceinline__ void row(uint32_t i, uint64_t &xs, uint64_t &ys, uint64_t &L,
                                      uint32_t &s) const {
    unpack(raw(i), xs, ys, L, s);
  }
};
template <class Rows>
struct SrcFile {
  using rec_t = uint4;
  static constexpr bool kPerRow = true;  // see load_items (rk_onesweep.h)
  Rows rows;
  uint64_t vsize;
  __device__ __forceinline__ uint4 load(uint32_t i) const {
    uint64_t xs, ys, L;
    uint32_t s;
    rows.row(i, xs, ys, L, s);
    return pack(xs, ys, L, s, i);
  }
  __device__ __forceinline__ uint4 pack(uint64_t xs, uint64_t ys, uint64_t L, uint32_t s,
                                        uint32_t i) const {
    // xs / 10 without a branch (div_small's 32-bit test waited for each row's
    // load before the next one issued): ceil(2^67 / 10) * xs >> 67 is exact
    // for every 64-bit xs
    const uint64_t pk = __umul64hi(xs, 0xCCCCCCCCCCCCCCCDull) >> 3;
    const uint32_t key = (uint32_t)(pk < vsize - 1 ? pk : vsize - 1);
    // (rows that do not pack were flagged by k_nw_order_hist: the generic
    // pipeline takes over then)
    return make_uint4(key, i, (uint32_t)ys,
                      (uint32_t)(L & 0xFFFFFFu) | s << 24 | (uint32_t)((ys >> 32) & 7u) << 25 |
                          (uint32_t)(xs - pk * 10) << 28);
  }
  __device__ __forceinline__ uint32_t key(const uint4 &r) const { return r.x; }
};
// --- processing order, last pass: the records, and the Y axis' input -------
// Yrec: {strand * nby + centre/100, processing index, centre low 32, length}
// 12-B Yrec: {strand * nby + centre/100, processing index, length (24) |
// centre % 100 (7) << 24}; the centre is the bucket * 100 + the remainder
struct DstProc {
  RK_NO_WAVE
  uint4 *out;
  uint3 *yrec;
  uint32_t nby;
  uint32_t base;  // processing index of position 0 (the sharded driver's slice offset)
  __device__ __forceinline__ void store(uint32_t pos, const uint4 &r) const {
    out[pos] = r;
    const uint64_t ys = rec_y(r);
    const uint32_t len = rec_len(r), s = rec_strand(r);
    const uint64_t yc = ys + len / 2;
    yrec[pos] = make_uint3(s * nby + (uint32_t)(yc / 100), base + pos,
                           len | (uint32_t)(yc % 100) << 24);
  }
};

// --- sharded driver: records as received from other ranks -------------------
// the Y records in arrival order: the entry id becomes the arrival index (the
// global processing index stays in the received array)
struct SrcIdx12 {
  using rec_t = uint3;
  const uint3 *in;
  __device__ __forceinline__ uint3 load(uint32_t i) const {
    const uint32_t *p = reinterpret_cast<const uint32_t *>(in + i);
    return make_uint3(__builtin_nontemporal_load(p), i, __builtin_nontemporal_load(p + 2));
  }
  __device__ __forceinline__ uint32_t key(const uint3 &r) const { return r.x; }
};
// member records {gid, row, key ...} with the gid made local to the rank's range
struct SrcSub12 {
  using rec_t = uint3;
  const uint3 *in;
  uint32_t sub;
  __device__ __forceinline__ uint3 load(uint32_t i) const {
    const uint32_t *p = reinterpret_cast<const uint32_t *>(in + i);
    return make_uint3(__builtin_nontemporal_load(p) - sub, __builtin_nontemporal_load(p + 1),
                      __builtin_nontemporal_load(p + 2));
  }
  __device__ __forceinline__ uint32_t key(const uint3 &r) const { return r.x; }
};
struct SrcSub16 {
  using rec_t = uint4;
  const uint4 *in;
  uint32_t sub;
  __device__ __forceinline__ uint4 load(uint32_t i) const {
    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(in + i));
    return make_uint4(v.x - sub, v.y, v.z, v.w);
  }
  __device__ __forceinline__ uint32_t key(const uint4 &r) const { return r.x; }
};

// digit histograms of every pass of a sort over records whose key is their
// first word (minus `sub`); STRIDE = record size in words
template <int STRIDE>
__global__ void __launch_bounds__(256) k_nw_rec_hist(const uint32_t *__restrict__ recs, uint32_t n,
                                                     uint32_t sub, Digits D,
                                                     uint32_t *__restrict__ ghist) {
  __shared__ HistLds L;
  hist_init(L);
  __syncthreads();
  if (STRIDE == 1) {
    // 4-B keys (the sharded driver's group ids by processing index) come in
    // long runs of equal high digits: one LDS atomic per run of a wavefront
    // instead of one per key on the same counter
    const uint32_t step = gridDim.x * blockDim.x;
    for (uint32_t b = blockIdx.x * blockDim.x + (threadIdx.x & ~63u); b < n; b += step) {
      const uint32_t i = b + (threadIdx.x & 63);
      const bool in = i < n;
      const uint32_t key = in ? recs[i] - sub : 0u;
      for (int p = 0; p < D.passes; ++p)
        wave_run_add(in ? (uint32_t)p * 1024u + D.digit(p, key) : NONE, L.h);
    }
  } else {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
      hist_add(L, D, recs[(size_t)i * STRIDE] - sub);
  }
  __syncthreads();
  hist_flush(L, D, ghist);
}

// --- Y axis, last pass: the CSR arrays the sweeps read -----------------------
// The X-hit lookup is a dependent load per record; with kPre the write-out
// issues it one slot round ahead (pre), and store() takes the loaded word.
struct DstCsr {
  static constexpr bool kPre = true;
  uint32_t *key, *ent;
  uint2 *pk;
  uint8_t *nbd;
  uint32_t nb;
  uint64_t max_index;
  const uint32_t *xbits;  // null: the states are filled later (k_nw_fill_y)
  uint8_t *state;
  __device__ __forceinline__ uint32_t pre(const uint3 &r) const {
    return xbits ? xbits[r.y >> 5] : 0u;
  }
  bool hit_bit;  // the X-hit bit travels in bit 31 of the record (SrcYX12): no lookup
  __device__ __forceinline__ void store(uint32_t pos, const uint3 &r, uint32_t xw) const {
    key[pos] = r.x;
    ent[pos] = r.y;
    const uint32_t b = r.x >= nb ? r.x - nb : r.x, rem = (r.z >> 24) & 0x7Fu;
    const uint64_t c = (uint64_t)b * 100 + rem;  // bucket * 100 + remainder
    pk[pos] = make_uint2((uint32_t)c, r.z & 0xFFFFFFu);
    // nbd_code_nw(c, max_index) with c % 100 == rem and c >= 100 <=> b >= 1
    // (no 64-bit remainder per record)
    nbd[pos] = rem <= 1 && b >= 1 ? 1
               : (rem == 99 && c < max_index) || (rem == 98 && c < max_index - 1) ? 2
                                                                                   : 0;
    // with the X results: the Y states -- X hits sit in the Y lists
    // (commonFunctions.cpp:59), X misses query them
    if (hit_bit) state[pos] = (r.z >> 31) ? ST_ACTIVE : ST_UNKNOWN;
    else if (xbits) state[pos] = (xw >> (r.y & 31)) & 1u ? ST_ACTIVE : ST_UNKNOWN;
  }
};
// the Y records in processing order with their fragment's X-hit bit in bit
// 31 of the third word.  Record i is fragment i (DstProc, one device), and a
// wave loads 64 consecutive records from a multiple of 64 (k_onesweep's
// layout: the tile and every wave's slice are multiples of 64 records), so
// the wave's 64 bits are one uniform 8-B load
// The bits come after the record loads (fixup): lane l < ITEMS loads the
// word of the wave's item l (its 64 records are 64 consecutive fragments from
// a multiple of 64), and item r takes its word by a lane read; lane j of
// every item group is record j of the group.
template <int ITEMS>
__device__ __forceinline__ void merge_xhit(uint3 (&rec)[ITEMS], const uint64_t *xbits64,
                                           uint32_t nwords, uint32_t base, uint32_t wbase) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t w0 = (base + wbase - lane) >> 6;  // the wave's first item group
  const uint64_t wd = lane < (uint32_t)ITEMS && w0 + lane < nwords ? xbits64[w0 + lane] : 0ull;
  const uint32_t lo = (uint32_t)wd, hi = (uint32_t)(wd >> 32);
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const uint32_t l = __builtin_amdgcn_readlane(lo, r), h = __builtin_amdgcn_readlane(hi, r);
    const uint32_t bit = ((lane < 32 ? l >> lane : h >> (lane - 32)) & 1u);
    rec[r].z |= bit << 31;
  }
}
struct SrcYX12 {
  using rec_t = uint3;
  static constexpr bool kFixup = true;
  const uint3 *in;
  const uint64_t *xbits64;
  uint32_t nwords;  // bitmask words: (records + 63) / 64
  __device__ __forceinline__ uint3 load(uint32_t i) const {
    const uint32_t *p = reinterpret_cast<const uint32_t *>(in + i);
    return make_uint3(__builtin_nontemporal_load(p), __builtin_nontemporal_load(p + 1),
                      __builtin_nontemporal_load(p + 2));
  }
  template <int ITEMS>
  __device__ __forceinline__ void fixup(uint3 (&rec)[ITEMS], uint32_t base, uint32_t wbase) const {
    merge_xhit<ITEMS>(rec, xbits64, nwords, base, wbase);
  }
  __device__ __forceinline__ uint32_t key(const uint3 &r) const { return r.x; }
};

// the same for the sharded driver's received Y records: the entry id becomes
// the arrival index (SrcIdx12) and the bit comes by arrival index
struct SrcIdxYX12 {
  using rec_t = uint3;
  static constexpr bool kFixup = true;
  const uint3 *in;
  const uint64_t *xbits64;
  uint32_t nwords;  // bitmask words: (records + 63) / 64
  __device__ __forceinline__ uint3 load(uint32_t i) const {
    const uint32_t *p = reinterpret_cast<const uint32_t *>(in + i);
    return make_uint3(__builtin_nontemporal_load(p), i, __builtin_nontemporal_load(p + 2));
  }
  template <int ITEMS>
  __device__ __forceinline__ void fixup(uint3 (&rec)[ITEMS], uint32_t base, uint32_t wbase) const {
    merge_xhit<ITEMS>(rec, xbits64, nwords, base, wbase);
  }
  __device__ __forceinline__ uint32_t key(const uint3 &r) const { return r.x; }
};

// --- processing order in two stages --------------------------------------
// (nw_order_sort with a split plan, nw_order_split): the one-sweep passes
// sort the records by the COARSE key K >> F only (C = b - F bits: cfg3's
// 29-bit key as 14 bits in two 7-bit passes instead of four passes), the last
// of them also counting the records of every coarse key (DstRecHist: one
// global atomic per run of equal keys in a wave's consecutive sorted slots);
// the counts' scan places every segment (the records of one coarse key, ~3000
// at cfg3).  k_seg_fine then sorts each segment by its F fine bits in
// LDS -- one block per segment, LSD by digits of up to 8 bits ranked by wave
// ballots, stable like a record pass -- and writes the final records, the Y
// records (DstProc's job) and the X-chunk counts (k_nw_xcount's job, which
// needs the final order).  A segment above the LDS capacity is sorted by the
// same block through global memory (chunks of OF_CAP in order: stable) --
// correct for any input, slow only for pathological ones.
struct DstRecHist {
  static constexpr bool kWave = true;
  static constexpr bool kPre = false;
  uint4 *out;
  uint32_t *chist;  // records per coarse key
  int F;
  uint32_t sub = 0;  // key base (as SrcRec::sub)
  __device__ __forceinline__ void store(uint32_t pos, const uint4 &r) const { out[pos] = r; }
  __device__ __forceinline__ void wave(const uint4 &r, bool live) const {
    wave_run_add(live ? (r.x - sub) >> F : NONE, chist);
  }
};

// the same coarse-key counts over 12-B records (the member sort by gid)
struct DstRec12Hist {
  static constexpr bool kWave = true;
  static constexpr bool kPre = false;
  uint3 *out;
  uint32_t *chist;
  int F;
  __device__ __forceinline__ void store(uint32_t pos, const uint3 &r) const {
    uint32_t *p = reinterpret_cast<uint32_t *>(out + pos);
    p[0] = r.x, p[1] = r.y, p[2] = r.z;
  }
  __device__ __forceinline__ void wave(const uint3 &r, bool live) const {
    wave_run_add(live ? r.x >> F : NONE, chist);
  }
};

constexpr int OF_T = 512, OF_ITEMS = 8, OF_NW = OF_T / 64, OF_CAP = OF_T * OF_ITEMS;
// the records inside the segment kernels as plain structs (kept in HIP's
// vector types, the 16-B records' y/z/w went through a scratch array)
struct P4 {
  uint32_t x, y, z, w;
};
struct P3 {
  uint32_t x, y, z;
};
template <class R>
struct PodOf;
template <>
struct PodOf<uint4> {
  using type = P4;
  __device__ static __forceinline__ P4 from(const uint4 &v) { return P4{v.x, v.y, v.z, v.w}; }
  __device__ static __forceinline__ uint4 to(const P4 &v) { return make_uint4(v.x, v.y, v.z, v.w); }
};
template <>
struct PodOf<uint3> {
  using type = P3;
  __device__ static __forceinline__ P3 from(const uint3 &v) { return P3{v.x, v.y, v.z}; }
  __device__ static __forceinline__ uint3 to(const P3 &v) { return make_uint3(v.x, v.y, v.z); }
};
template <class R>
struct FineLds {
  typename PodOf<R>::type srec[OF_CAP];
  uint32_t wcnt[OF_NW][256];  // per-wave digit counters, then per-wave starts
  uint32_t lbase[256];        // block-local digit starts
  uint32_t run[256];          // global path: running digit offsets
  uint32_t tot[256];          // global path: digit totals of a chunk / histogram
  uint32_t wsum[OF_NW];
};

// Stable ranks of the block's records by digit d = (x >> shift) & (2^db - 1)
// (x = the record's fine key): rec[r] sits at block index wbase + 64 r, live
// below cnt.  Returns in rk[r] the record's slot among the wave's records of
// its digit; afterwards L.wcnt[w][d] = wave w's start inside digit d, L.lbase[d]
// = digit d's start in the block, L.tot[d] = its count.
template <class R, class V>
__device__ __forceinline__ void fine_rank(FineLds<R> &L, const V (&rec)[OF_ITEMS],
                                          uint32_t (&rk)[OF_ITEMS], uint32_t (&dg)[OF_ITEMS],
                                          uint32_t wbase, uint32_t cnt, uint32_t fmask, int shift,
                                          int db) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
  uint32_t *mycnt = L.wcnt[w];
  for (uint32_t d = lane; d < 256; d += 64) mycnt[d] = 0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int r = 0; r < OF_ITEMS; ++r) {
    const bool live = wbase + 64 * r < cnt;
    const uint32_t d = live ? ((rec[r].x & fmask) >> shift) & ((1u << db) - 1u) : 0u;
    dg[r] = d;
    uint64_t peer = __ballot(live);
    for (int b = 0; b < db; ++b) {
      const bool bit = (d >> b) & 1u;
      const uint64_t bb = __ballot(bit);
      peer &= bit ? bb : ~bb;
    }
    const uint32_t below = __popcll(peer & lt);
    const uint32_t before = live ? mycnt[d] : 0u;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    if (live && below == 0) mycnt[d] = before + __popcll(peer);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    rk[r] = before + below;
  }
  __syncthreads();
  // thread t < 256 owns digit t: the waves' starts inside it, then the block scan
  const uint32_t t = threadIdx.x;
  uint32_t tot = 0;
  if (t < 256) {
#pragma unroll
    for (int k = 0; k < OF_NW; ++k) {
      const uint32_t c = L.wcnt[k][t];
      L.wcnt[k][t] = tot;
      tot += c;
    }
  }
  uint32_t inc = tot;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(inc, o);
    if ((int)lane >= o) inc += v;
  }
  if (lane == 63) L.wsum[w] = inc;
  __syncthreads();
  if (t < 256) {
    uint32_t at = inc - tot;
    for (uint32_t k = 0; k < w; ++k) at += L.wsum[k];
    L.lbase[t] = at;
    L.tot[t] = tot;
  }
  __syncthreads();
}

// The processing order's emit: a position of the final order -- the record
// and its Y record (DstProc), the X-chunk counts (k_nw_xcount's layout).
// Every lane of the wave calls emit (first: the record's key differs from the
// previous position's).
// The X counts go to an LDS window of OE_WIN chunks from the segment's first
// owner chunk (a segment spans 2^F xStart/10 keys: a few chunks), flushed with
// one global atomic per non-zero bin after the segment (begin / end); a chunk
// outside the window (a centre far past its xStart) takes a global atomic.
// (The emit objects stay const: a kernel argument written to lives in scratch.)
constexpr uint32_t OE_WIN = 256;
struct OrderEmit {
  static constexpr int kWin = 3 * OE_WIN;
  DstProc dst;
  uint32_t m;      // kept rows: the X counts take positions below m
  uint32_t *cnts;  // X-chunk counts, or null
  uint32_t lgW, nch, kdiv;
  // the window's first chunk, after clearing the window
  __device__ __forceinline__ uint32_t begin(uint32_t *win, uint32_t key0) const {
    for (uint32_t j = threadIdx.x; j < (uint32_t)kWin; j += blockDim.x) win[j] = 0;
    __syncthreads();
    return cnts ? key0 / kdiv : 0u;
  }
  __device__ __forceinline__ void emit(uint32_t *win, uint32_t w0, uint32_t pos, const uint4 &r,
                                       bool live, bool) const {
    if (live) dst.store(pos, r);
    if (cnts) {
      const bool kept = live && pos < m;
      uint32_t vx = NONE, vo = NONE;
      if (kept) {
        const uint32_t cx = (uint32_t)((rec_x(r) + rec_len(r) / 2) / 100) >> lgW;
        const uint32_t co = r.x / kdiv, st = rec_strand(r);
        if (cx - w0 < OE_WIN) vx = st * OE_WIN + (cx - w0);
        else atomicAdd(&cnts[st * nch + cx], 1u);
        if (co - w0 < OE_WIN) vo = 2 * OE_WIN + (co - w0);
        else atomicAdd(&cnts[2 * nch + co], 1u);
      }
      wave_run_add(vx, win);
      wave_run_add(vo, win);
    }
  }
  __device__ __forceinline__ void end(uint32_t *win, uint32_t w0) const {
    __syncthreads();
    if (!cnts) return;
    for (uint32_t j = threadIdx.x; j < (uint32_t)kWin; j += blockDim.x) {
      const uint32_t v = win[j];
      if (!v) continue;
      const uint32_t part = j / OE_WIN, ch = w0 + (j - part * OE_WIN);
      atomicAdd(&cnts[part * nch + ch], v);
    }
  }
};
// The member sort's emit: the in-group sort arrays (DstMembers) and the group
// starts (k_group_offsets' job: a group starts where the gid changes; the
// last position closes goff[G] = m)
struct MemberEmit {
  static constexpr int kWin = 1;
  uint32_t *sgid, *tag, *mrow;
  uint64_t *key;
  uint32_t *goff;
  uint32_t G, m;
  __device__ __forceinline__ uint32_t begin(uint32_t *, uint32_t) const { return 0; }
  __device__ __forceinline__ void end(uint32_t *, uint32_t) const {}
  __device__ __forceinline__ void emit(uint32_t *, uint32_t, uint32_t pos, const uint3 &r,
                                       bool live, bool first) const {
    if (!live) return;
    sgid[pos] = r.x;
    mrow[pos] = r.y;
    key[pos] = r.z;
    if (first) goff[r.x] = pos;
    if (pos + 1 == m) goff[G] = m;
  }
};

// The Y axis' emit: the occupancy CSR arrays and the Y states (DstCsr, the
// X-hit bit carried in bit 31 of the record); a segment's positions are
// consecutive, so the five arrays are written as whole lines
struct CsrEmit {
  static constexpr int kWin = 1;
  DstCsr dc;
  __device__ __forceinline__ uint32_t begin(uint32_t *, uint32_t) const { return 0; }
  __device__ __forceinline__ void end(uint32_t *, uint32_t) const {}
  __device__ __forceinline__ void emit(uint32_t *, uint32_t, uint32_t pos, const uint3 &r,
                                       bool live, bool) const {
    if (live) dc.store(pos, r, 0u);
  }
};

// One block per segment: the F fine bits of its records, LSD by digits of up
// to 8 bits, in LDS (at most OF_CAP records).  A larger segment is listed in
// big (big[0] = count) for k_seg_big: kept apart, the LDS kernel's registers
// hold no global-memory path (with it inline the records spilled to scratch).
template <class R>
struct SegArgs {
  const R *in;          // sorted by coarse key, stable
  R *A, *B;             // k_seg_big's buffers, its last pass landing in A
  const uint32_t *off;  // nseg + 1 segment starts
  uint32_t nseg;
  int F;                // fine bits (>= 1)
  uint32_t *big;        // [0] count, then the segments above OF_CAP
};
template <class R, class E>
__global__ void __launch_bounds__(OF_T) __attribute__((amdgpu_waves_per_eu(4)))
k_seg_fine(const SegArgs<R> a, const E e) {
  __shared__ FineLds<R> L;
  __shared__ uint32_t ewin[E::kWin];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6, t = threadIdx.x;
  const uint32_t wbase = w * (OF_CAP / OF_NW) + lane;
  const uint32_t fmask = a.F >= 32 ? 0xFFFFFFFFu : (1u << a.F) - 1u;
  const int np = (a.F + 7) / 8;
  using P = PodOf<R>;
  typename P::type rec[OF_ITEMS];
  uint32_t rk[OF_ITEMS], dg[OF_ITEMS];
  for (uint32_t sg = blockIdx.x; sg < a.nseg; sg += gridDim.x) {
    const uint32_t s0 = a.off[sg], cnt = a.off[sg + 1] - s0;
    if (cnt == 0) continue;
    if (cnt > (uint32_t)OF_CAP) {
      if (t == 0) a.big[1 + atomicAdd(&a.big[0], 1u)] = sg;
      continue;
    }
#pragma unroll
    for (int r = 0; r < OF_ITEMS; ++r) {
      const uint32_t i = wbase + 64 * r;
      rec[r] = P::from(a.in[s0 + (i < cnt ? i : cnt - 1)]);  // (dead lanes: a copy, no branch)
    }
    // LSD passes over the fine key; the last placement is the final order
    for (int q = 0; q < np; ++q) {
      const int shift = 8 * q, db = a.F - shift < 8 ? a.F - shift : 8;
      fine_rank(L, rec, rk, dg, wbase, cnt, fmask, shift, db);
#pragma unroll
      for (int r = 0; r < OF_ITEMS; ++r)
        if (wbase + 64 * r < cnt) L.srec[L.lbase[dg[r]] + L.wcnt[w][dg[r]] + rk[r]] = rec[r];
      __syncthreads();
      if (q + 1 < np) {
#pragma unroll
        for (int r = 0; r < OF_ITEMS; ++r) {
          const uint32_t i = wbase + 64 * r;
          rec[r] = L.srec[i < cnt ? i : cnt - 1];  // (unconditional: the array stays in VGPRs)
        }
        __syncthreads();
      }
    }
    const uint32_t w0 = e.begin(ewin, L.srec[0].x);
    for (uint32_t j0 = 0; j0 < cnt; j0 += OF_T) {
      const uint32_t j = j0 + t;
      const bool live = j < cnt;
      const R r = P::to(L.srec[live ? j : cnt - 1]);
      const bool first = live && (j == 0 || L.srec[j - 1].x != r.x);
      e.emit(ewin, w0, s0 + j, r, live, first);
    }
    e.end(ewin, w0);
    __syncthreads();  // the next segment reuses the LDS
  }
}

// The listed segments above OF_CAP, one block each: the same passes through
// global memory, chunk by chunk in order (stable); the last lands in A.  A
// segment whose fine keys are all equal (one huge group of the member sort)
// is already in order.
template <class R, class E>
__global__ void __launch_bounds__(OF_T) k_seg_big(const SegArgs<R> a, const E e) {
  __shared__ FineLds<R> L;
  __shared__ uint32_t ewin[E::kWin];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6, t = threadIdx.x;
  const uint32_t wbase = w * (OF_CAP / OF_NW) + lane;
  const uint32_t fmask = a.F >= 32 ? 0xFFFFFFFFu : (1u << a.F) - 1u;
  const int np = (a.F + 7) / 8;
  using P = PodOf<R>;
  typename P::type rec[OF_ITEMS];
  uint32_t rk[OF_ITEMS], dg[OF_ITEMS];
  const uint32_t nbig = a.big[0];
  for (uint32_t k = blockIdx.x; k < nbig; k += gridDim.x) {
    const uint32_t sg = a.big[1 + k];
    const uint32_t s0 = a.off[sg], cnt = a.off[sg + 1] - s0;
    const R *src = a.in + s0;
    uint32_t lo = 0xFFFFFFFFu, hi = 0;
    for (uint32_t j = t; j < cnt; j += OF_T) {
      const uint32_t x = src[j].x & fmask;
      lo = x < lo ? x : lo;
      hi = x > hi ? x : hi;
    }
    if (t == 0) L.run[0] = 0xFFFFFFFFu, L.run[1] = 0;
    __syncthreads();
    atomicMin(&L.run[0], lo);
    atomicMax(&L.run[1], hi);
    __syncthreads();
    const bool sorted = L.run[0] == L.run[1];
    __syncthreads();
    for (int q = 0; q < (sorted ? 0 : np); ++q) {
      const int shift = 8 * q, db = a.F - shift < 8 ? a.F - shift : 8;
      R *dst = ((np - 1 - q) % 2 == 0) ? a.A + s0 : a.B + s0;
      // the pass' digit histogram over the segment, its scan into running starts
      if (t < 256) L.tot[t] = 0;
      __syncthreads();
      for (uint32_t j = t; j < cnt; j += OF_T)
        atomicAdd(&L.tot[((src[j].x & fmask) >> shift) & ((1u << db) - 1u)], 1u);
      __syncthreads();
      {
        const uint32_t tot = t < 256 ? L.tot[t] : 0u;
        uint32_t inc = tot;
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t v = __shfl_up(inc, o);
          if ((int)lane >= o) inc += v;
        }
        if (lane == 63) L.wsum[w] = inc;
        __syncthreads();
        if (t < 256) {
          uint32_t at = inc - tot;
          for (uint32_t k2 = 0; k2 < w; ++k2) at += L.wsum[k2];
          L.run[t] = at;
        }
        __syncthreads();
      }
      for (uint32_t c0 = 0; c0 < cnt; c0 += OF_CAP) {
        const uint32_t cc = cnt - c0 < (uint32_t)OF_CAP ? cnt - c0 : (uint32_t)OF_CAP;
#pragma unroll
        for (int r = 0; r < OF_ITEMS; ++r) {
          const uint32_t i = wbase + 64 * r;
          rec[r] = P::from(src[c0 + (i < cc ? i : cc - 1)]);
        }
        fine_rank(L, rec, rk, dg, wbase, cc, fmask, shift, db);
#pragma unroll
        for (int r = 0; r < OF_ITEMS; ++r)
          if (wbase + 64 * r < cc) dst[L.run[dg[r]] + L.wcnt[w][dg[r]] + rk[r]] = P::to(rec[r]);
        __syncthreads();
        if (t < 256) L.run[t] += L.tot[t];
        __syncthreads();
      }
      // this block's global writes before its next reads of them: one CU,
      // one L1 -- the barrier's workgroup-scope release/acquire suffices (an
      // agent-scope fence would write the L2 back)
      __syncthreads();
      src = dst;
    }
    const R *fin = sorted ? a.in + s0 : a.A + s0;
    const uint32_t w0 = e.begin(ewin, fin[0].x);
    for (uint32_t j0 = 0; j0 < cnt; j0 += OF_T) {
      const uint32_t j = j0 + t;
      const bool live = j < cnt;
      const R r = fin[live ? j : cnt - 1];
      const bool first = live && (j == 0 || fin[j - 1].x != r.x);
      e.emit(ewin, w0, s0 + j, r, live, first);
    }
    e.end(ewin, w0);
    __syncthreads();
  }
}

template <class R, class E>
static void launch_seg(const SegArgs<R> &a, const E &e, hipStream_t st) {
  // (a.big[0], the list count, is the segment counts' first word: the scan
  // that placed the segments cleared it, exclusive_scan_u32_clear0)
  k_seg_fine<<<a.nseg < 65536u ? a.nseg : 65536u, OF_T, 0, st>>>(a, e);
  k_seg_big<<<256, OF_T, 0, st>>>(a, e);  // (returns at once when none is listed)
}

// --- group members, last pass: gid order (stable: processing order inside) -
// members {gid, row, sort key lo, hi} -> group of every slot, sort key, tag =
// slot, file row
struct DstMembers {
  RK_NO_WAVE
  uint32_t *sgid, *tag, *mrow;
  uint64_t *key;
  // (no tags: sort_groups_exact takes tag[x] == x without reading them)
  __device__ __forceinline__ void store(uint32_t pos, const uint4 &r) const {
    sgid[pos] = r.x;
    mrow[pos] = r.y;
    key[pos] = (uint64_t)r.w << 32 | r.z;
  }
  __device__ __forceinline__ void store(uint32_t pos, const uint3 &r) const {
    sgid[pos] = r.x;
    mrow[pos] = r.y;
    key[pos] = r.z;
  }
};

// ---------------------------------------------------------------------------
// One read of the file-order SoA before the sort: the digit histograms of the
// processing key (all passes) and of the Y axis key of every kept row, the
// kept-row and forward-strand counts, the longest kept length, the
// out-of-bounds checks (xStart/10 >= vsize; probes past an occupancy array)
// and whether every row packs into a record.  ctrl: [0] error bits, [1] kept
// rows, [3] some row does not pack, [4] longest kept length, [8] forward kept.
template <class Rows>
struct OrderHistArgs {
  Rows rows;
  uint32_t n;
  uint64_t vsize, max_x, max_y;
  uint32_t nby;
  Digits D, yd;
  uint32_t *ghist, *yhist, *ctrl;
};
template <class Rows>
__global__ void __launch_bounds__(256) k_nw_order_hist(OrderHistArgs<Rows> a) {
  __shared__ HistLds L, LY;
  __shared__ uint32_t red[4];
  hist_init(L);
  hist_init(LY);
  if (threadIdx.x < 4) red[threadIdx.x] = 0;
  __syncthreads();
  uint32_t kept = 0, fwd = 0, maxlen = 0;
  bool ub = false, ubc = false, wide = false;
  const uint64_t drop = a.vsize - 1;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += gridDim.x * blockDim.x) {
    uint64_t xs, ys, L0;
    uint32_t s;
    a.rows.row(i, xs, ys, L0, s);
    const uint64_t pk = div_small(xs, 10);
    ub |= pk >= a.vsize;
    wide |= L0 >= (1ull << 24) || ys >= (1ull << 35);
    const uint32_t key = (uint32_t)(pk < drop ? pk : drop);
    hist_add(L, a.D, key);
    if (key == drop) continue;  // the never-iterated last bucket
    ++kept;
    fwd += s == 0;
    const uint32_t len = (uint32_t)(L0 & 0xFFFFFFu);  // exact whenever the row packs
    maxlen = len > maxlen ? len : maxlen;
    const uint64_t h = len / 2;
    ubc |= probe_max_bucket_nw(xs + h, a.max_x) > a.max_x ||
           probe_max_bucket_nw(ys + h, a.max_y) > a.max_y;
    hist_add(LY, a.yd, s * a.nby + (uint32_t)div_small(ys + h, 100));
  }
  for (int off = 32; off > 0; off >>= 1) {
    kept += __shfl_xor(kept, off);
    fwd += __shfl_xor(fwd, off);
    const uint32_t o = __shfl_xor(maxlen, off);
    maxlen = o > maxlen ? o : maxlen;
  }
  const uint64_t bub = __ballot(ub), bubc = __ballot(ubc), bwide = __ballot(wide);
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&red[0], kept);
    atomicAdd(&red[1], fwd);
    atomicMax(&red[2], maxlen);
    atomicOr(&red[3], (bub ? 1u : 0u) | (bubc ? 2u : 0u) | (bwide ? 4u : 0u));
  }
  __syncthreads();
  hist_flush(L, a.D, a.ghist);
  hist_flush(LY, a.yd, a.yhist);
  if (threadIdx.x == 0) {
    if (red[0]) atomicAdd(&a.ctrl[1], red[0]);
    if (red[1]) atomicAdd(&a.ctrl[8], red[1]);
    if (red[2]) atomicMax(&a.ctrl[4], red[2]);
    if (red[3] & 1u) atomicOr(&a.ctrl[0], ERRB_UB_BUCKET);
    if (red[3] & 2u) atomicOr(&a.ctrl[0], ERRB_UB_CENTER);
    if (red[3] & 4u) atomicOr(&a.ctrl[3], 1u);
  }
}

// ---------------------------------------------------------------------------
// X axis by chunks of W centre buckets (both strands), from the processing
// order, one wavefront per chunk.  Chunk c owns buckets [cW, (c+1)W); its
// entries are the rows whose centre falls in the chunk: the rows it OWNS
// (xStart/100 in the chunk: [kO, kB), from the owner counts of the last order
// pass) plus a halo of earlier rows (centre <= xStart + H, H = longest length
// / 2), found by a backward ballot scan from kO.  The wave counts its entries
// per (strand, bucket) bin in LDS, scans the counts into bin starts, and
// places every entry at chunk offset (strand-major scan of the per-chunk
// counts, also from the last order pass) + bin start + its rank among the
// bin's entries in row order (= processing order: stable).  No look-back, no
// block barrier.  The same wave writes every owned row's member record
// {0, row, sort key}: the sort key |yStart - diag_func[xStart/10]| needs the
// yStart of the LAST row of the row's xStart/10 run (commonFunctions.cpp:
// 161-177), and chunk borders are run borders.
// Per-chunk counts for the X axis, from the processing order (sorted by
// xStart/10, so a block's rows cover a narrow window of chunks): cnts[s * nch
// + chunk of the row's X bucket] (strand s) and cnts[2 nch + owner chunk]
// (xStart/10 / 10W).  Runs of equal ids are added per wave into an LDS window
// of chunks, flushed with one global atomic per non-zero bin.
// The processing order the X axis is built from: G halo records (the sharded
// driver's lead-in from earlier slices, rk_shard_nw.h) ahead of the own
// records; G = 0 on one device.
struct RecView {
  const uint4 *h;
  uint32_t G;
  const uint4 *o;
  __device__ __forceinline__ uint4 operator[](uint32_t k) const { return k < G ? h[k] : o[k - G]; }
};

constexpr int XN_T = 256, XN_ITEMS = 16, XN_WIN = 1024;
__global__ void __launch_bounds__(XN_T) k_nw_xcount(const RecView R, uint32_t m,
                                                    uint32_t lgW, uint32_t nch, uint32_t kdiv,
                                                    uint32_t *__restrict__ cnts) {
  __shared__ uint32_t win[3 * XN_WIN];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t r0 = blockIdx.x * (XN_T * XN_ITEMS);
  for (uint32_t j = threadIdx.x; j < 3 * XN_WIN; j += XN_T) win[j] = 0;
  const uint32_t w0 = R[r0].x / kdiv;  // the block's first owner chunk
  __syncthreads();
  const uint32_t wb = r0 + wv * 64 * XN_ITEMS;
  uint4 rr[XN_ITEMS];
#pragma unroll
  for (int i = 0; i < XN_ITEMS; ++i) {
    const uint32_t k = wb + i * 64 + lane;
    rr[i] = k < m ? R[k] : make_uint4(NONE, 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < XN_ITEMS; ++i) {
    const uint4 r = rr[i];
    const bool live = wb + i * 64 + lane < m;
    uint32_t vx = NONE, vo = NONE;
    if (live) {
      const uint32_t cx = (uint32_t)((rec_x(r) + rec_len(r) / 2) / 100) >> lgW;
      const uint32_t co = r.x / kdiv, st = rec_strand(r);
      if (cx - w0 < XN_WIN) vx = st * XN_WIN + (cx - w0);
      else atomicAdd(&cnts[st * nch + cx], 1u);  // outside the window: rare
      if (co - w0 < XN_WIN) vo = 2 * XN_WIN + (co - w0);
      else atomicAdd(&cnts[2 * nch + co], 1u);
    }
    wave_run_add(vx, win);
    wave_run_add(vo, win);
  }
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < 3 * XN_WIN; j += XN_T) {
    const uint32_t v = win[j];
    if (!v) continue;
    const uint32_t part = j / XN_WIN, ch = w0 + (j - part * XN_WIN);
    atomicAdd(&cnts[part * nch + ch], v);
  }
}

constexpr int XC_WAVES = 4, XC_SLOTS = 8;  // rows per batch: XC_SLOTS x 64
struct XChunkArgs {
  RecView R;             // processing order
  uint32_t m;            // kept rows
  uint32_t W, lgW, nch;  // chunk width in buckets (power of two), chunks
  uint32_t halo;         // ceil(H / 10) in xStart/10 units
  uint64_t max_x;
  uint32_t nbx;
  const uint32_t *xoff;  // [2 nch] strand-major entry offsets, [nch + 1] owner row starts (+ m)
  Csr out;
  uint32_t *xpos;        // X position of every fragment (processing index)
  uint2 *erk;            // member records (processing order): {file row, sort key low 32}
  uint32_t *ehi;         // ... and the sort key's high 32 bits
  uint32_t *ctrl;        // [6] some sort key >= 2^32
};

__global__ void __launch_bounds__(64 * XC_WAVES) k_nw_xchunk(XChunkArgs a) {
  extern __shared__ uint32_t xc_lds[];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t c = blockIdx.x * XC_WAVES + wv;
  if (c >= a.nch) return;  // whole waves; nothing below synchronises the block
  const uint32_t nb2 = 2 * a.W;
  uint32_t *bin_at = xc_lds + (size_t)wv * nb2;  // counts, then running positions
  for (uint32_t j = lane; j < nb2; j += 64) bin_at[j] = 0;
  const uint32_t *orow = a.xoff + 2 * a.nch;
  const uint32_t kO = orow[c] - a.m, kB = orow[c + 1] - a.m;
  const uint64_t b0 = (uint64_t)a.W * c;
  // halo rows: the suffix of [0, kO) with xStart/10 >= 10Wc - halo
  const uint64_t own_key = (uint64_t)10 * a.W * c;
  const uint64_t hk = own_key > a.halo ? own_key - a.halo : 0;
  uint32_t kA = kO;
  while (kA > 0) {
    const uint32_t lo = kA >= 64 ? kA - 64 : 0;
    const uint32_t k = lo + lane;
    const bool in = k < kA && a.R[k].x >= hk;
    const uint32_t nin = (uint32_t)__popcll(__ballot(in));
    const bool all = nin == kA - lo;
    kA -= nin;
    if (!all) break;
  }
  const uint32_t nrows = kB - kA, nbatch = (nrows + 64 * XC_SLOTS - 1) / (64 * XC_SLOTS);
  uint4 rr[XC_SLOTS];
  // pass 1, batches and slots backwards: bin counts, owned rows' sort keys
  // (carry: key and run-end yStart of the row just after the current slot)
  uint32_t carry_key = NONE;
  uint64_t carry_end = 0;
  bool wide = false;
  for (uint32_t bi = nbatch; bi-- > 0;) {
    const uint32_t base = kA + bi * 64 * XC_SLOTS;
#pragma unroll
    for (int s = 0; s < XC_SLOTS; ++s) {
      const uint32_t k = base + s * 64 + lane;
      rr[s] = k < kB ? a.R[k] : make_uint4(NONE, 0, 0, 0);
    }
#pragma unroll
    for (int s = XC_SLOTS - 1; s >= 0; --s) {
      const uint32_t k = base + s * 64 + lane;
      const bool live = k < kB;
      const uint4 r = rr[s];
      const uint64_t xs = rec_x(r), ys = rec_y(r);
      const uint32_t len = rec_len(r), st = rec_strand(r);
      const uint64_t bk = (xs + len / 2) / 100;
      if (live && bk >= b0 && bk < b0 + a.W) atomicAdd(&bin_at[st * a.W + (uint32_t)(bk - b0)], 1u);
      // run ends inside the slot; the last row's successor is the carry
      const uint32_t key = live ? r.x : NONE;
      uint32_t nk = __shfl_down(key, 1);
      if (lane == 63) nk = carry_key;
      const uint64_t ends = __ballot(live && nk != key);
      const uint64_t above = ends & ~((1ull << lane) - 1ull);
      const uint64_t end_ys =
          above ? __shfl(ys, (int)__builtin_ctzll(above)) : carry_end;  // all lanes shuffle
      if (live && k >= kO) {
        const uint64_t h = ys > end_ys ? ys - end_ys : end_ys - ys;
        a.erk[k] = make_uint2(r.y, (uint32_t)h);
        a.ehi[k] = (uint32_t)(h >> 32);
        wide |= (h >> 32) != 0;
      }
      carry_key = __shfl(key, 0);
      carry_end = __shfl(end_ys, 0);
    }
  }
  if (__ballot(wide) && lane == 0) atomicOr(&a.ctrl[6], 1u);
  // bin starts (exclusive scan over the 2W bins, W/32 per lane)
  {
    const uint32_t per = nb2 / 64;
    uint32_t tot = 0;
    for (uint32_t j = 0; j < per; ++j) tot += bin_at[lane * per + j];
    uint32_t inc = tot;
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t o = __shfl_up(inc, off);
      if ((int)lane >= off) inc += o;
    }
    uint32_t at = inc - tot;
    for (uint32_t j = 0; j < per; ++j) {
      const uint32_t cn = bin_at[lane * per + j];
      bin_at[lane * per + j] = at;
      at += cn;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const uint32_t nf = bin_at[a.W];  // forward entries of the chunk
  const uint32_t off_f = a.xoff[c], off_r = a.xoff[a.nch + c];
  const int bits = (int)a.lgW + 1;
  // pass 2, forwards: rank within bin (ballots over the bin bits), place
  for (uint32_t bi = 0; bi < nbatch; ++bi) {
    const uint32_t base = kA + bi * 64 * XC_SLOTS;
    if (nbatch > 1) {
#pragma unroll
      for (int s = 0; s < XC_SLOTS; ++s) {
        const uint32_t k = base + s * 64 + lane;
        rr[s] = k < kB ? a.R[k] : make_uint4(NONE, 0, 0, 0);
      }
    }
#pragma unroll
    for (int s = 0; s < XC_SLOTS; ++s) {
      const uint32_t k = base + s * 64 + lane;
      const uint4 r = rr[s];
      const uint64_t xs = rec_x(r);
      const uint32_t len = rec_len(r), st = rec_strand(r);
      const uint64_t xc = xs + len / 2, bk = xc / 100;
      const bool mine = k < kB && bk >= b0 && bk < b0 + a.W;
      if (!__ballot(mine)) continue;
      const uint32_t bin = mine ? st * a.W + (uint32_t)(bk - b0) : 0u;
      uint64_t peer = __ballot(mine);
      for (int b = 0; b < bits; ++b) {
        const bool bit = (bin >> b) & 1u;
        const uint64_t bb = __ballot(bit);
        peer &= bit ? bb : ~bb;
      }
      const uint32_t below = __popcll(peer & ((1ull << lane) - 1ull));
      const uint32_t before = mine ? bin_at[bin] : 0u;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      if (mine && below == 0) bin_at[bin] = before + __popcll(peer);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (!mine) continue;
      const uint32_t loc = before + below;
      const uint32_t q = st == 0 ? off_f + loc : off_r + (loc - nf);
      a.out.key[q] = st * a.nbx + (uint32_t)bk;
      a.out.ent[q] = k;
      a.out.pk[q] = make_uint2((uint32_t)xc, len);
      a.out.nbd[q] = nbd_code_nw(xc, a.max_x);
      a.out.state[q] = ST_UNKNOWN;
      a.xpos[k] = q;
    }
  }
}

// X hits as a bitmask by processing index, a wave per 64 fragments (their X
// positions are a narrow window of the X axis: the state reads stay local)
__global__ void k_nw_x_bits(const uint32_t *__restrict__ xpos, const uint8_t *__restrict__ xstate,
                            uint32_t m, uint32_t *__restrict__ bits) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k - lane < m;
       k += gridDim.x * blockDim.x) {
    const bool hit = k < m && xstate[xpos[k]] == ST_HIT;
    const uint64_t b = __ballot(hit);
    if (lane == 0) bits[k >> 5] = (uint32_t)b;
    if (lane == 32 && k < m) bits[k >> 5] = (uint32_t)(b >> 32);
  }
}

// Y states: X hits sit in the Y lists (commonFunctions.cpp:59), X misses query
// them; the 6-MB bitmask (cfg3) is served from L2 / Infinity Cache
__global__ void k_nw_fill_y(const uint32_t *__restrict__ ent, const uint32_t *__restrict__ bits,
                            uint8_t *__restrict__ state, uint32_t m) {
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < m; q += gridDim.x * blockDim.x) {
    const uint32_t e = ent[q];
    state[q] = (bits[e >> 5] >> (e & 31)) & 1u ? ST_ACTIVE : ST_UNKNOWN;
  }
}

// gid of every member (its root's rank among new groups) into its record,
// and the member sort's digit histograms
__global__ void __launch_bounds__(256) k_nw_assign(const uint32_t *__restrict__ par,
                                                   const uint32_t *__restrict__ newrank,
                                                   uint32_t *__restrict__ gidp, uint32_t m,
                                                   Digits D, uint32_t *__restrict__ ghist) {
  __shared__ HistLds L;
  hist_init(L);
  __syncthreads();
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < m; k += gridDim.x * blockDim.x) {
    const uint32_t g = newrank[par[k]];
    gidp[k] = g;  // (a word per fragment: the member records take it in the sort's first pass)
    hist_add(L, D, g);
  }
  __syncthreads();
  hist_flush(L, D, ghist);
}

// The roots and the gids in one pass (the new-group ranks already scanned from
// the parents' root flags, exclusive_scan_roots): each member chases its
// parent chain up to `steps` steps, writes the root back as its parent (so
// later chases are short), and its gid = newrank[root] with the member sort's
// digit histograms; a longer chain is listed for k_nw_assign_rest.  Replaces
// k_jump's first round + the flag scan + k_nw_assign (their flag array
// written and read, the parents read twice).
//
// Every gid written is below G = newrank[m], whatever happens: each of the G
// roots (par[r] == r, never rewritten) takes its own rank, so no group is
// empty and the member sort and the group sort downstream stay in bounds even
// when a chain is left open (*open: the caller then classifies again the
// round-by-round way) or a parent is corrupt (ERRB_INTERNAL: the call fails).

// chase from `a` at most `steps` steps; stops at a root (true) or at a parent
// not before its child (error bit; `a` is then taken as the end)
__device__ __forceinline__ bool chase_root(const uint32_t *par, uint32_t &a, int steps,
                                           uint32_t *err) {
  for (int step = 0; step < steps; ++step) {
    const uint32_t b = par[a];
    if (b == a) return true;
    if (b > a) {  // parents are always earlier
      atomicOr(err, ERRB_INTERNAL);
      return true;
    }
    a = b;
  }
  return par[a] == a;
}
__device__ __forceinline__ uint32_t gid_of(const uint32_t *newrank, uint32_t a, uint32_t G) {
  const uint32_t g = newrank[a];
  return g < G ? g : G - 1u;  // (only a corrupt parent or an open chain needs the clamp)
}

__global__ void __launch_bounds__(256) k_nw_assign_jump(uint32_t *__restrict__ par,
                                                        const uint32_t *__restrict__ newrank,
                                                        uint32_t *__restrict__ gidp, uint32_t m,
                                                        Digits D, uint32_t *__restrict__ ghist,
                                                        uint32_t *__restrict__ list,
                                                        uint32_t *__restrict__ count,
                                                        uint32_t *__restrict__ err, int steps) {
  __shared__ HistLds L;
  hist_init(L);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t G = newrank[m];  // >= 1: the first fragment always opens a group
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k - lane < m;
       k += gridDim.x * blockDim.x) {
    bool open = false;
    if (k < m) {
      const uint32_t a0 = par[k];
      uint32_t a = a0;
      bool done;
      if (a0 > k) {  // corrupt: taken as its own root
        atomicOr(err, ERRB_INTERNAL);
        a = k;
        done = true;
      } else {
        done = chase_root(par, a, steps, err);
        if (a != a0) par[k] = a;
      }
      open = !done;
      if (done) {
        const uint32_t g = gid_of(newrank, a, G);
        gidp[k] = g;
        hist_add(L, D, g);
      }
    }
    const uint64_t b = __ballot(open);
    if (b) {
      uint32_t at = 0;
      if (lane == 0) at = atomicAdd(count, (uint32_t)__popcll(b));
      at = (uint32_t)__shfl((int)at, 0);
      if (open) list[at + __popcll(b & ((1ull << lane) - 1ull))] = k;
    }
  }
  __syncthreads();
  hist_flush(L, D, ghist);
}

// the listed chains, followed further (up to `steps` more); a chain still open
// sets *open and takes a clamped gid (the caller classifies again)
__global__ void k_nw_assign_rest(uint32_t *par, const uint32_t *newrank, uint32_t *gidp,
                                 uint32_t m, Digits D, uint32_t *ghist, const uint32_t *list,
                                 const uint32_t *count, uint32_t *open, uint32_t *err,
                                 int steps) {
  const uint32_t n = *count, G = newrank[m];
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t k = list[i];
    uint32_t a = par[k];
    if (!chase_root(par, a, steps, err)) *open = 1u;
    par[k] = a;
    const uint32_t g = gid_of(newrank, a, G);
    gidp[k] = g;
    for (int p = 0; p < D.passes; ++p) atomicAdd(&ghist[p * 1024 + D.digit(p, g)], 1u);
  }
}

// ---------------------------------------------------------------------------
// widest digit of the record sorts (RK_NW_BITS=8..10 for measurements): 8-bit
// digits measured fastest at cfg3 (a 16-B record pass 0.49 ms against 0.69 ms
// at 9 bits and 1.44 ms at 10: wider digits leave fewer records per digit
// segment of a tile and fewer resident tiles)
int nw_max_bits() {
  static const int v = [] {
    const char *e = getenv("RK_NW_BITS");
    const int b = e ? atoi(e) : 8;
    return b < 8 ? 8 : b > 10 ? 10 : b;
  }();
  return v;
}

// narrowest radix of a pass (RK_NW_MINBITS=7..8): a pass whose balanced
// digit width is 7 bits sorts over 128 digits instead of 256 (cfg3's 29-bit
// processing key: 8 + 7 + 7 + 7) -- one ballot less per record and half the
// counters and look-back walks per tile
int nw_min_bits() {
  static const int v = [] {
    const char *e = getenv("RK_NW_MINBITS");
    const int b = e ? atoi(e) : 7;
    return b < 7 ? 7 : b > 8 ? 8 : b;
  }();
  return v;
}

Digits plan_digits(int bits, int max_bits = 0) {
  Digits D{};
  if (bits < 1) bits = 1;
  const int mb = max_bits ? max_bits : nw_max_bits();
  const int lo = nw_min_bits();
  D.passes = (bits + mb - 1) / mb;
  int shift = 0;
  for (int p = 0; p < D.passes; ++p) {
    const int left = bits - shift, w0 = (left + (D.passes - p) - 1) / (D.passes - p);
    D.shift[p] = shift;
    D.db[p] = w0 < lo ? lo : w0;
    shift += w0;
  }
  return D;
}

constexpr int OS_T = 256;
// 12-B record passes (the Y axis; the members when every sort key fits 32
// bits): 512 threads x RK_NW_ITEMS12 records, placed through LDS in rounds of
// 5461 slots.  14 (7168 per tile, 128 VGPRs: two blocks per CU): cfg3 step
// 11.54-11.58 ms; 12: 11.59-11.66; 16 (142 VGPRs, one block per CU) not run;
// the same passes on 16-B records: 12.14-12.16 ms
#ifndef RK_NW_ITEMS12
#define RK_NW_ITEMS12 14
#endif
// SrcYX12: a wave's slice of a tile starts at a multiple of 64 records
static_assert(512 * RK_NW_ITEMS12 % 64 == 0 && 512 * 12 % 64 == 0, "waves load from multiples of 64");
int nw_shape();
// records per tile of a pass with DB-bit digits over rec_bytes-B records (the
// shape of launch_pass_db)
uint32_t tile_records(int db, int rec_bytes = 16) {
  if (rec_bytes == 12 && db <= 9) return 512 * RK_NW_ITEMS12;
  if (db == 7) return 512 * 12;
  if (db != 8) return OS_T * (db >= 10 ? 12 : 16);
  switch (nw_shape()) {
    case 2: return 256 * 8;
    case 3: return 256 * 12;
    case 5: case 6: return 512 * 16;
    case 7: return 512 * 12;
    case 8: return 1024 * 8;
    default: return 4096;  // 0, 1: 256 x 16; 4: 512 x 8
  }
}
uint32_t tiles_for(uint32_t n, int db, int rec_bytes = 16) {
  const uint32_t tile = tile_records(db, rec_bytes);
  return (n + tile - 1) / tile;
}

// RK_NW_TRACE=<file>: per-tile phase timestamps of every record pass, written
// to <file> after each classification (measurement only)
struct NwTrace {
  uint64_t *buf = nullptr;
  size_t cap = 0, used = 0;
  std::vector<std::pair<size_t, uint32_t>> passes;  // (offset, tiles)
};
NwTrace &nw_trace() {
  static NwTrace t;
  return t;
}
const char *nw_trace_path() {
  static const char *p = getenv("RK_NW_TRACE");
  return p;
}
uint64_t *trace_slot(uint32_t tiles) {
  if (!nw_trace_path()) return nullptr;
  NwTrace &t = nw_trace();
  if (!t.buf) {
    t.cap = (size_t)8 << 20;  // words
    if (hipMalloc(&t.buf, t.cap * 8) != hipSuccess) return t.buf = nullptr;
  }
  const size_t need = (size_t)tiles * 8;
  if (t.used + need > t.cap) return nullptr;
  uint64_t *p = t.buf + t.used;
  t.passes.push_back({t.used, tiles});
  t.used += need;
  return p;
}

// persistent grid: as many blocks as stay resident (occupancy x CUs)
template <class K>
uint32_t resident_blocks(K kernel, int threads) {
  int dev = 0, cus = 0, per = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, threads, 0);
  const int b = (cus > 0 ? cus : 256) * (per > 0 ? per : 1);
  return (uint32_t)b;
}

// RK_NW_SHAPE (measurements; 8-bit digits): 0 = 256 threads x 16 records per
// block, one tile each; 1 = the same, persistent blocks, the next tile's loads
// issued before the look-back; 2 = 256 x 8; 3 = 256 x 12; 4 = 512 x 8; 5, 6 =
// 512 x 16; 7 = 512 x 12 (default); 8 = 1024 x 8.  Tiles above 4096 records
// are staged through LDS in rounds of 4096 sorted slots, so a 6144-record tile
// keeps two blocks per CU (125 VGPRs, 2 x ~75 KB of LDS) and pays one look-back
// per 6144 records.  cfg3 step, two streams: 13.75 / - / 14.39 / - / 13.28 /
// 13.49 ms (round 2, earlier code: 5 had 128 KB of LDS, one block per CU;
// shape 1 was slower: the look-back's loads queue behind the next tile's in the
// same wave's memory counter); now 4 / 6 / 7 / 8: 12.78 / 13.01 / 12.27 / 12.59
// ms (6: 158 VGPRs, one block per CU; 8: one 1024-thread block per CU)
int nw_shape() {
  static const int v = [] {
    const char *e = getenv("RK_NW_SHAPE");
    return e ? atoi(e) : 7;
  }();
  return v;
}

template <int T, int ITEMS, int DB, bool PERSIST, class Src, class Dst>
void launch_shape(const Src &src, const Dst &dst, uint32_t n, int shift, const uint32_t *ghist,
                  uint32_t *status, uint32_t *ctr, hipStream_t st, uint32_t *clear_next) {
  const uint32_t tiles = (n + T * ITEMS - 1) / (T * ITEMS);
  auto kern = k_onesweep<T, ITEMS, DB, PERSIST, Src, Dst>;
  uint32_t grid = tiles;
  if (PERSIST) {
    static const uint32_t resident = resident_blocks(kern, T);
    grid = tiles < resident ? tiles : resident;
  }
  kern<<<grid, T, 0, st>>>(src, dst, n, tiles, shift, ghist, status, ctr, trace_slot(tiles),
                           clear_next);
}
template <int DB, class Src, class Dst>
void launch_pass_db(const Src &src, const Dst &dst, uint32_t n, int shift, const uint32_t *ghist,
                    uint32_t *status, uint32_t *ctr, hipStream_t st, uint32_t *clear_next) {
  constexpr int ITEMS = DB >= 10 ? 12 : 16;
  if constexpr (DB == 7 && sizeof(typename Src::rec_t) == 12) {
    launch_shape<512, RK_NW_ITEMS12, 7, false>(src, dst, n, shift, ghist, status, ctr, st,
                                               clear_next);
    return;
  } else if constexpr (DB == 7) {
    launch_shape<512, 12, 7, false>(src, dst, n, shift, ghist, status, ctr, st, clear_next);
    return;
  } else if constexpr (DB == 9 && sizeof(typename Src::rec_t) == 12) {
    launch_shape<512, RK_NW_ITEMS12, 9, false>(src, dst, n, shift, ghist, status, ctr, st,
                                               clear_next);
    return;
  } else if constexpr (DB == 8 && sizeof(typename Src::rec_t) == 12) {
    // 12-B records: RK_NW_ITEMS12 per thread (LDS rounds of 5461 slots)
    launch_shape<512, RK_NW_ITEMS12, 8, false>(src, dst, n, shift, ghist, status, ctr, st,
                                               clear_next);
    return;
  } else if constexpr (DB == 8) {
    switch (nw_shape()) {
      case 1: launch_shape<OS_T, 16, 8, true>(src, dst, n, shift, ghist, status, ctr, st, clear_next); return;
      case 2: launch_shape<256, 8, 8, false>(src, dst, n, shift, ghist, status, ctr, st, clear_next); return;
      case 3: launch_shape<256, 12, 8, false>(src, dst, n, shift, ghist, status, ctr, st, clear_next); return;
      case 4: launch_shape<512, 8, 8, false>(src, dst, n, shift, ghist, status, ctr, st, clear_next); return;
      case 5: case 6: launch_shape<512, 16, 8, false>(src, dst, n, shift, ghist, status, ctr, st, clear_next); return;
      case 7: launch_shape<512, 12, 8, false>(src, dst, n, shift, ghist, status, ctr, st, clear_next); return;
      case 8: launch_shape<1024, 8, 8, false>(src, dst, n, shift, ghist, status, ctr, st, clear_next); return;
      default: break;
    }
  }
  launch_shape<OS_T, ITEMS, DB, false>(src, dst, n, shift, ghist, status, ctr, st, clear_next);
}
template <class Src, class Dst>
void launch_pass(const Src &src, const Dst &dst, uint32_t n, int shift, int db,
                 const uint32_t *ghist, uint32_t *status, uint32_t *ctr, hipStream_t st,
                 double bytes, uint32_t *clear_next = nullptr) {
  if (!n) return;
  kt_begin(st, KID_ONESWEEP);
  switch (db) {
    case 7: launch_pass_db<7>(src, dst, n, shift, ghist, status, ctr, st, clear_next); break;
    case 8: launch_pass_db<8>(src, dst, n, shift, ghist, status, ctr, st, clear_next); break;
    case 9: launch_pass_db<9>(src, dst, n, shift, ghist, status, ctr, st, clear_next); break;
    default: launch_pass_db<10>(src, dst, n, shift, ghist, status, ctr, st, nullptr); break;
  }
  kt_end(st, KID_ONESWEEP, bytes);
}

// one launch clears up to ZR_MAX regions (blockIdx.y = region): 16-B stores
// where the region is 16-B aligned, 4-B stores for the rest
constexpr int ZR_MAX = 8;
struct ZeroArgs {
  uint32_t *p[ZR_MAX];
  uint32_t words[ZR_MAX];
};
__global__ void __launch_bounds__(256) k_zero_regions(const ZeroArgs a) {
  uint32_t *p = a.p[blockIdx.y];
  const uint32_t n = a.words[blockIdx.y];
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, stride = gridDim.x * blockDim.x;
  uint32_t head = 0;
  if ((reinterpret_cast<uintptr_t>(p) & 15) == 0) {
    const uint32_t nv = n / 4;
    uint4 *v = reinterpret_cast<uint4 *>(p);
    for (uint32_t i = t; i < nv; i += stride) v[i] = make_uint4(0, 0, 0, 0);
    head = nv * 4;
  }
  for (uint32_t i = head + t; i < n; i += stride) p[i] = 0;
}

}  // namespace

void zero_regions(hipStream_t st, std::initializer_list<ZeroRegion> regs) {
  ZeroArgs a{};
  int k = 0;
  uint32_t most = 0;
  for (const ZeroRegion &r : regs) {
    if (!r.ptr || !r.bytes) continue;
    if (k == ZR_MAX || (r.bytes & 3) || r.bytes / 4 > 0xFFFFFFFFull) {
      (void)hipMemsetAsync(r.ptr, 0, r.bytes, st);
      continue;
    }
    a.p[k] = reinterpret_cast<uint32_t *>(r.ptr);
    a.words[k] = (uint32_t)(r.bytes / 4);
    most = a.words[k] > most ? a.words[k] : most;
    ++k;
  }
  if (!k) return;
  const uint32_t bx = (most / 4 + 255) / 256;
  k_zero_regions<<<dim3(bx < 1 ? 1 : bx > 256 ? 256 : bx, (uint32_t)k), 256, 0, st>>>(a);
}

// ===========================================================================
// host side
void nw_trace_dump(hipStream_t st) {
  if (!nw_trace_path()) return;
  NwTrace &t = nw_trace();
  if (!t.buf || t.passes.empty()) return;
  (void)hipStreamSynchronize(st);
  std::vector<uint64_t> h(t.used);
  if (hipMemcpy(h.data(), t.buf, t.used * 8, hipMemcpyDeviceToHost) == hipSuccess) {
    if (FILE *f = fopen(nw_trace_path(), "wb")) {
      const uint64_t np = t.passes.size();
      fwrite(&np, 8, 1, f);
      for (auto &p : t.passes) {
        const uint64_t hdr[2] = {p.first, p.second};
        fwrite(hdr, 8, 2, f);
      }
      fwrite(h.data(), 8, h.size(), f);
      fclose(f);
    }
  }
  t.used = 0;
  t.passes.clear();
}

size_t nw_status_words(uint32_t n) {
  // the largest pass: tiles of 3072 records x 1024 digits, + per-pass tile counters
  return (size_t)((n + 3071) / 3072 + 1) * 1024 + 64;
}

NwDigits nw_plan(int bits, int max_bits) {
  const Digits D = plan_digits(bits, max_bits);
  NwDigits o{};
  o.passes = D.passes;
  for (int p = 0; p < 4; ++p) o.shift[p] = D.shift[p], o.db[p] = D.db[p];
  return o;
}

static const uint32_t *ghist_of(const uint32_t *h, int pass) { return h + pass * 1024; }

static Digits to_digits(const NwDigits &o) {
  Digits D{};
  D.passes = o.passes;
  for (int p = 0; p < 4; ++p) D.shift[p] = o.shift[p], D.db[p] = o.db[p];
  return D;
}

// Status words of one sort.  When every pass has the same tiles and no pass
// has more digits than the one before (8-bit digits, or 9-bit ones over 12-B
// records), the buffer is used as two halves: pass p publishes into half p & 1
// and zeroes, tile by tile, its own rows of the other half for pass p + 1
// (k_onesweep's clear_next), so a sort needs one memset instead of one per
// pass; otherwise one buffer, cleared before each pass.
struct PassStatus {
  uint32_t *base;
  size_t half;
  bool ahead;
  int rec_bytes;
  uint32_t *use(int p) const { return ahead ? base + (size_t)(p & 1) * half : base; }
  uint32_t *next(int p, int passes) const {
    return ahead && p + 1 < passes ? base + (size_t)((p + 1) & 1) * half : nullptr;
  }
  // before pass p: the words it still needs cleared (none after a clear-ahead
  // pass: {nullptr, 0})
  ZeroRegion region(int p, uint32_t n, const Digits &D) const {
    if (ahead && p > 0) return ZeroRegion{nullptr, 0};
    const size_t words =
        ahead ? half : (size_t)tiles_for(n, D.db[p], rec_bytes) * ((size_t)1 << D.db[p]);
    return ZeroRegion{use(p), words * 4};
  }
  void prepare(int p, uint32_t n, const Digits &D, hipStream_t st) const {
    const ZeroRegion r = region(p, n, D);
    if (r.bytes) (void)hipMemsetAsync(r.ptr, 0, r.bytes, st);
  }
};
static PassStatus pass_status(uint32_t *status, uint32_t n, const Digits &D, int rec_bytes = 16) {
  const uint32_t tiles = tiles_for(n, D.db[0], rec_bytes);
  bool same = true;
  for (int p = 1; p < D.passes; ++p)
    same &= D.db[p] <= D.db[p - 1] && tiles_for(n, D.db[p], rec_bytes) == tiles;
  const size_t half = (size_t)tiles << D.db[0];
  return PassStatus{status, half, same && 2 * half + 64 <= nw_status_words(n), rec_bytes};
}

template <class Rows>
static void order_hist(const Rows &rows, uint32_t n, double row_bytes, uint64_t vsize,
                       uint64_t max_x, uint64_t max_y, uint32_t nby, const NwDigits &a,
                       const NwDigits &y, uint32_t *ghist, uint32_t *yhist, uint32_t *ctrl,
                       hipStream_t st) {
  if (!n) return;
  OrderHistArgs<Rows> args{rows, n, vsize, max_x, max_y, nby, to_digits(a), to_digits(y), ghist,
                           yhist, ctrl};
  kt_begin(st, KID_NW_HIST);
  k_nw_order_hist<Rows><<<grid_for(n, 256, 2048), 256, 0, st>>>(args);
  kt_end(st, KID_NW_HIST, row_bytes * n);  // the rows read once
}
void nw_order_hist(const rk_frags_soa &in, uint64_t vsize, uint64_t max_x, uint64_t max_y,
                   uint32_t nby, const NwDigits &a, const NwDigits &y, uint32_t *ghist,
                   uint32_t *yhist, uint32_t *ctrl, hipStream_t st, const uint3 *wire) {
  if (wire)
    order_hist(RowWire{wire}, (uint32_t)in.n, 12.0, vsize, max_x, max_y, nby, a, y, ghist, yhist,
               ctrl, st);
  else
    order_hist(RowSoA{in.x_start, in.y_start, in.length, in.strand}, (uint32_t)in.n, 25.0, vsize,
               max_x, max_y, nby, a, y, ghist, yhist, ctrl, st);
}

// the processing order: passes over records, the first one from `first`
// (the file SoA, or records received by the sharded driver); the Y records
// carry processing index base + position
template <class Src1>
static void nw_order_passes(const Src1 &first, double in_bytes, uint32_t n, uint32_t nby,
                            uint32_t base, const NwDigits &a, const uint32_t *ghist,
                            uint32_t *status, uint4 *Ra, uint4 *Rb, uint4 *yrec, hipStream_t st) {
  const Digits D = to_digits(a);
  const size_t sw = nw_status_words(n);
  (void)hipMemsetAsync(status + sw - 64, 0, 64 * 4, st);  // the passes' tile counters
  const PassStatus ps = pass_status(status, n, D);
  // the final pass lands in Ra
  for (int p = 0; p < D.passes; ++p) {
    uint4 *out = ((D.passes - 1 - p) % 2 == 0) ? Ra : Rb;
    const uint4 *src = ((D.passes - p) % 2 == 0) ? Ra : Rb;  // the previous pass' output
    ps.prepare(p, n, D, st);
    uint32_t *stp = ps.use(p), *nxt = ps.next(p, D.passes);
    uint32_t *ctr = status + sw - 64 + p;
    const uint32_t *gh = ghist + p * 1024;
    const bool last = p == D.passes - 1;
    const DstProc dp{out, reinterpret_cast<uint3 *>(yrec), nby, base};
    if (p == 0) {
      if (last)
        launch_pass(first, dp, n, D.shift[p], D.db[p], gh, stp, ctr, st, in_bytes * n + 28.0 * n,
                    nxt);
      else
        launch_pass(first, DstRec{out}, n, D.shift[p], D.db[p], gh, stp, ctr, st,
                    in_bytes * n + 16.0 * n, nxt);
    } else if (last) {
      launch_pass(SrcRec{src}, dp, n, D.shift[p], D.db[p], gh, stp, ctr, st, 44.0 * n, nxt);
    } else {
      launch_pass(SrcRec{src}, DstRec{out}, n, D.shift[p], D.db[p], gh, stp, ctr, st,
                  32.0 * n, nxt);
    }
  }
}
void nw_order_sort(const rk_frags_soa &in, uint64_t vsize, uint32_t nby, const NwDigits &a,
                   const uint32_t *ghist, uint32_t *status, uint4 *Ra, uint4 *Rb, uint4 *yrec,
                   hipStream_t st, const uint3 *wire) {
  if (wire)
    nw_order_passes(SrcFile<RowWire>{RowWire{wire}, vsize}, 12.0, (uint32_t)in.n, nby, 0u, a,
                    ghist, status, Ra, Rb, yrec, st);
  else
    nw_order_passes(
        SrcFile<RowSoA>{RowSoA{in.x_start, in.y_start, in.length, in.strand}, vsize}, 25.0,
        (uint32_t)in.n, nby, 0u, a, ghist, status, Ra, Rb, yrec, st);
}
void nw_order_sort_recs(const uint4 *in, uint32_t m, uint32_t nby, uint32_t base,
                        const NwDigits &a, const uint32_t *ghist, uint32_t *status, uint4 *Ra,
                        uint4 *Rb, uint4 *yrec, hipStream_t st) {
  nw_order_passes(SrcRec{in}, 16.0, m, nby, base, a, ghist, status, Ra, Rb, yrec, st);
}

// The two-stage plan (see k_seg_fine): F fine bits for the segment
// kernel -- as many as keep the average segment (n rows over the nkeys key
// values, 2^F keys per segment) at most NW_SEG_TARGET rows, 3/4 of the LDS
// capacity (cfg3: ~2730 rows; the global-memory path stays rare) -- and
// C = b - F coarse bits for the one-sweep passes.  passes = 0: the LSD passes
// over all b bits (too few rows, or RK_NW_SPLIT=0).
constexpr uint32_t NW_SEG_TARGET = OF_CAP * 3 / 4;
NwOrderPlan nw_order_split(uint32_t n, uint64_t nkeys, int b) {
  NwOrderPlan o{};
  static const bool on = [] {
    const char *e = getenv("RK_NW_SPLIT");
    return !(e && e[0] == '0');
  }();
  int F = 0;
  while (F < b && (double)n * (double)(2ull << F) <= (double)NW_SEG_TARGET * (double)nkeys) ++F;
  const int C = b - F;
  // (2^C + 1 segment counts must fit nw_seg_words(n): 2^C < 4n / NW_SEG_TARGET)
  if (!on || F < 1 || C < 1 || C > 24 || ((size_t)1 << C) + 1 > nw_seg_words(n)) return o;
  o.F = F;
  o.C = C;
  o.coarse = nw_plan(C);
  for (int p = 0; p < o.coarse.passes; ++p) o.coarse.shift[p] += o.F;
  o.nseg = (uint32_t)1 << C;
  return o;
}
// the same over the keys [klo, khi) of one slice (the sharded driver): the
// coarse keys are (key - kbase) >> F with kbase = klo rounded down to 2^F, so
// the segments cover the slice's span, not the whole key space, and the fine
// bits stay the key's own low F bits
NwOrderPlan nw_order_split_range(uint32_t n, uint64_t klo, uint64_t khi) {
  if (khi <= klo) return NwOrderPlan{};
  // F as nw_order_split picks it (capped by the absolute key's bits)
  const int b = bit_length(khi - 1);
  int F = 0;
  while (F < b && (double)n * (double)(2ull << F) <= (double)NW_SEG_TARGET * (double)(khi - klo))
    ++F;
  const uint64_t kbase = klo & ~((1ull << F) - 1);
  NwOrderPlan o = nw_order_split(n, khi - klo, bit_length(khi - 1 - kbase));
  // (its F is at most this F -- the same density test, a smaller cap -- so
  // kbase stays a multiple of 2^o.F)
  if (o.nseg && (kbase & ((1ull << o.F) - 1))) return NwOrderPlan{};
  o.kbase = (uint32_t)kbase;
  return o;
}

// the coarse passes (the last writes Rb and counts the coarse keys into
// chist, 2^C + 1 words, zeroed here), the scan into segment starts, the fine
// kernel into Ra (+ Y records, + the X-chunk counts into cc.cnts when given,
// zeroed here)
// the first half: the clears (tile counters, coarse-key counts, the first
// pass' status words, `extra`) and the coarse passes, the last one counting
// the coarse keys into chist
// what the coarse order passes need cleared before they start: the passes'
// tile counters, the coarse-key counts, the first pass' status words, `extra`
void nw_order_coarse_regions(uint32_t n, const NwOrderPlan &op, uint32_t *status, uint32_t *chist,
                             ZeroRegion extra, ZeroRegion out[4]) {
  const Digits D = to_digits(op.coarse);
  const size_t sw = nw_status_words(n);
  const PassStatus ps = pass_status(status, n, D);
  out[0] = ZeroRegion{status + sw - 64, 64 * 4};
  out[1] = ZeroRegion{chist, ((size_t)op.nseg + 1) * 4};
  out[2] = ps.region(0, n, D);
  out[3] = extra;
}
template <class Src1>
static void nw_order_coarse(const Src1 &first, double in_bytes, uint32_t n, const NwOrderPlan &op,
                            const uint32_t *ghist, uint32_t *status, uint4 *Ra, uint4 *Rb,
                            uint32_t *chist, ZeroRegion extra, hipStream_t st,
                            bool zeroed = false) {
  const Digits D = to_digits(op.coarse);
  const size_t sw = nw_status_words(n);
  const PassStatus ps = pass_status(status, n, D);
  if (!zeroed) {
    ZeroRegion r[4];
    nw_order_coarse_regions(n, op, status, chist, extra, r);
    zero_regions(st, {r[0], r[1], r[2], r[3]});
  }
  for (int p = 0; p < D.passes; ++p) {
    uint4 *out = ((D.passes - 1 - p) % 2 == 0) ? Rb : Ra;  // the last coarse pass lands in Rb
    const uint4 *src = ((D.passes - p) % 2 == 0) ? Rb : Ra;
    if (p > 0) ps.prepare(p, n, D, st);
    uint32_t *stp = ps.use(p), *nxt = ps.next(p, D.passes);
    uint32_t *ctr = status + sw - 64 + p;
    const uint32_t *gh = ghist + p * 1024;
    const bool last = p == D.passes - 1;
    const DstRecHist dh{out, chist, op.F, op.kbase};
    const double bytes = (p == 0 ? in_bytes : 16.0) * n + 16.0 * n;
    if (p == 0 && last) launch_pass(first, dh, n, D.shift[p], D.db[p], gh, stp, ctr, st, bytes, nxt);
    else if (p == 0) launch_pass(first, DstRec{out}, n, D.shift[p], D.db[p], gh, stp, ctr, st, bytes, nxt);
    else if (last) launch_pass(SrcRec{src, op.kbase}, dh, n, D.shift[p], D.db[p], gh, stp, ctr, st, bytes, nxt);
    else launch_pass(SrcRec{src, op.kbase}, DstRec{out}, n, D.shift[p], D.db[p], gh, stp, ctr, st, bytes, nxt);
  }
}
// the second half: the counts' scan into segment starts, the segment kernel
// into Ra (+ Y records, + the X-chunk counts into cc->cnts when given, which
// the first half cleared)
static void nw_order_fine(uint32_t n, uint32_t m, uint32_t nby, uint32_t base,
                          const NwOrderPlan &op, uint4 *Ra, uint4 *Rb, uint4 *yrec, uint4 *tmp,
                          uint32_t *chist, uint32_t *coff, ScanScratch ss,
                          const NwChunkCounts *cc, hipStream_t st) {
  exclusive_scan_u32_clear0(chist, coff, (size_t)op.nseg + 1, ss, st);
  OrderEmit oe{DstProc{Ra, reinterpret_cast<uint3 *>(yrec), nby, base}, m, nullptr, 0, 0, 0};
  if (cc) {
    oe.cnts = cc->cnts;
    oe.lgW = cc->lgW;
    oe.nch = cc->nch;
    oe.kdiv = 10 * cc->W;
  }
  kt_begin(st, KID_NW_FINE);
  // (the counts are free after the scan: the list of segments above OF_CAP)
  launch_seg(SegArgs<uint4>{Rb, Ra, tmp, coff, op.nseg, op.F, chist}, oe, st);
  // records in and out, Y records out (the X counts: no extra reads)
  kt_end(st, KID_NW_FINE, 44.0 * n);
}
static ZeroRegion counts_region(const NwChunkCounts *cc) {
  return ZeroRegion{cc ? cc->cnts : nullptr, cc ? ((size_t)3 * cc->nch + 1) * 4 : 0};
}
void nw_order_sort_split_coarse(const rk_frags_soa &in, const NwOrderPlan &op,
                                const uint32_t *ghist, uint32_t *status, uint4 *Ra, uint4 *Rb,
                                uint32_t *chist, ZeroRegion extra, uint64_t vsize,
                                hipStream_t st, const uint3 *wire, bool zeroed) {
  if (wire)
    nw_order_coarse(SrcFile<RowWire>{RowWire{wire}, vsize}, 12.0, (uint32_t)in.n, op, ghist,
                    status, Ra, Rb, chist, extra, st, zeroed);
  else
    nw_order_coarse(SrcFile<RowSoA>{RowSoA{in.x_start, in.y_start, in.length, in.strand}, vsize},
                    25.0, (uint32_t)in.n, op, ghist, status, Ra, Rb, chist, extra, st, zeroed);
}
void nw_order_sort_split_fine(uint32_t n, uint32_t m, uint32_t nby, const NwOrderPlan &op,
                              uint4 *Ra, uint4 *Rb, uint4 *yrec, uint4 *tmp, uint32_t *chist,
                              uint32_t *coff, ScanScratch ss, const NwChunkCounts *cc,
                              hipStream_t st) {
  nw_order_fine(n, m, nby, 0u, op, Ra, Rb, yrec, tmp, chist, coff, ss, cc, st);
}
void nw_order_sort_split(const rk_frags_soa &in, uint32_t m, uint32_t nby, const NwOrderPlan &op,
                         const uint32_t *ghist, uint32_t *status, uint4 *Ra, uint4 *Rb,
                         uint4 *yrec, uint4 *tmp, uint32_t *chist, uint32_t *coff,
                         ScanScratch ss, const NwChunkCounts *cc, uint64_t vsize, hipStream_t st,
                         const uint3 *wire) {
  nw_order_sort_split_coarse(in, op, ghist, status, Ra, Rb, chist, counts_region(cc), vsize, st,
                             wire);
  nw_order_fine((uint32_t)in.n, m, nby, 0u, op, Ra, Rb, yrec, tmp, chist, coff, ss, cc, st);
}
void nw_order_sort_recs_split(const uint4 *in, uint32_t m, uint32_t nby, uint32_t base,
                              const NwOrderPlan &op, const uint32_t *ghist, uint32_t *status,
                              uint4 *Ra, uint4 *Rb, uint4 *yrec, uint4 *tmp, uint32_t *chist,
                              uint32_t *coff, ScanScratch ss, const NwChunkCounts *cc,
                              hipStream_t st) {
  nw_order_coarse(SrcRec{in, op.kbase}, 16.0, m, op, ghist, status, Ra, Rb, chist,
                  counts_region(cc), st);
  nw_order_fine(m, m, nby, base, op, Ra, Rb, yrec, tmp, chist, coff, ss, cc, st);
}

void nw_rec_hist(const void *recs, int rec_bytes, uint32_t n, uint32_t sub, const NwDigits &d,
                 uint32_t *ghist, hipStream_t st) {
  if (!n) return;
  const uint32_t *w = reinterpret_cast<const uint32_t *>(recs);
  kt_begin(st, KID_NW_HIST);
  if (rec_bytes == 16)
    k_nw_rec_hist<4><<<grid_for(n, 256, 2048), 256, 0, st>>>(w, n, sub, to_digits(d), ghist);
  else if (rec_bytes == 12)
    k_nw_rec_hist<3><<<grid_for(n, 256, 2048), 256, 0, st>>>(w, n, sub, to_digits(d), ghist);
  else  // a plain key array
    k_nw_rec_hist<1><<<grid_for(n, 256, 2048), 256, 0, st>>>(w, n, sub, to_digits(d), ghist);
  kt_end(st, KID_NW_HIST, (double)rec_bytes * n);  // the records' lines are read whole
}


// The Y axis sort in two parts: every pass but the last (on the second stream,
// beside the X axis), then the last one, which writes the CSR arrays and --
// given the X-hit bitmask -- the Y states (no separate fill pass).  Pass p
// reads yrec (p = 0) or the previous pass' output; intermediates alternate
// tmp, yrec (yrec is free once the first pass read it).
void nw_y_sort_head(const uint4 *yrec, uint4 *tmp, uint32_t m, const NwDigits &y,
                    const uint32_t *yhist, uint32_t *status, hipStream_t st, bool arrival_ids,
                    const uint4 *src0) {
  const Digits D = to_digits(y);
  const size_t sw = nw_status_words(m);
  (void)hipMemsetAsync(status + sw - 64, 0, 64 * 4, st);  // the passes' tile counters
  const PassStatus ps = pass_status(status, m, D, 12);  // the tail pass' half is cleared here
  // 12-B records (DstProc); the buffers are uint4 arrays, large enough
  const uint3 *src = reinterpret_cast<const uint3 *>(src0 ? src0 : yrec);
  for (int p = 0; p + 1 < D.passes; ++p) {
    ps.prepare(p, m, D, st);
    uint3 *out = reinterpret_cast<uint3 *>(p % 2 == 0 ? tmp : const_cast<uint4 *>(yrec));
    if (p == 0 && arrival_ids)
      launch_pass(SrcIdx12{src}, DstRec12{out}, m, D.shift[p], D.db[p], ghist_of(yhist, p),
                  ps.use(p), status + sw - 64 + p, st, 24.0 * m, ps.next(p, D.passes));
    else
      launch_pass(SrcRec12{src}, DstRec12{out}, m, D.shift[p], D.db[p], ghist_of(yhist, p),
                  ps.use(p), status + sw - 64 + p, st, 24.0 * m, ps.next(p, D.passes));
    src = out;
  }
}
void nw_y_sort_tail(const uint4 *yrec, const uint4 *tmp, uint32_t m, const NwDigits &y,
                    const uint32_t *yhist, uint32_t *status, Csr cy, uint32_t nby,
                    uint64_t max_y, const uint32_t *xbits, hipStream_t st, bool arrival_ids,
                    const uint4 *src0) {
  const Digits D = to_digits(y);
  const size_t sw = nw_status_words(m);
  const int p = D.passes - 1;
  const uint3 *src = reinterpret_cast<const uint3 *>(
      p == 0 ? (src0 ? src0 : yrec) : (p - 1) % 2 == 0 ? tmp : yrec);
  const PassStatus ps = pass_status(status, m, D, 12);
  ps.prepare(p, m, D, st);  // a no-op after the head's clear-ahead
  if (p == 0) (void)hipMemsetAsync(status + sw - 64, 0, 64 * 4, st);
  const DstCsr dc{cy.key, cy.ent, cy.pk, cy.nbd, nby, max_y, xbits, cy.state, false};
  const double bytes = 12.0 * m + 17.0 * m + (xbits ? 5.0 * m : 0.0);
  if (p == 0 && arrival_ids)
    launch_pass(SrcIdx12{src}, dc, m, D.shift[p], D.db[p], ghist_of(yhist, p), ps.use(p),
                status + sw - 64 + p, st, bytes);
  else
    launch_pass(SrcRec12{src}, dc, m, D.shift[p], D.db[p], ghist_of(yhist, p), ps.use(p),
                status + sw - 64 + p, st, bytes);
}

// The Y axis sort after the X axis is resolved (one device): the first pass
// reads the Y records in processing order together with their X-hit bits
// (sequential bitmask words) and carries the bit in the records, so the last
// pass writes the Y states from it instead of looking it up per record
template <class Src0>
static void y_after_x_first(const Src0 &s0, const DstCsr &dc, uint3 *out, bool last, uint32_t m,
                            const Digits &D, const uint32_t *gh, uint32_t *stp, uint32_t *ctr,
                            hipStream_t st, double bytes, uint32_t *nxt) {
  if (last) launch_pass(s0, dc, m, D.shift[0], D.db[0], gh, stp, ctr, st, bytes, nxt);
  else launch_pass(s0, DstRec12{out}, m, D.shift[0], D.db[0], gh, stp, ctr, st, bytes, nxt);
}
void nw_y_sort_after_x(const uint4 *yrec, uint4 *tmp, uint32_t m, const NwDigits &y,
                       const uint32_t *yhist, uint32_t *status, Csr cy, uint32_t nby,
                       uint64_t max_y, const uint32_t *xbits, hipStream_t st, const uint4 *src0) {
  const Digits D = to_digits(y);
  const size_t sw = nw_status_words(m);
  const PassStatus ps = pass_status(status, m, D, 12);
  // the passes' tile counters and the first pass' status words, one launch
  zero_regions(st, {{status + sw - 64, 64 * 4}, ps.region(0, m, D)});
  const DstCsr dc{cy.key, cy.ent, cy.pk, cy.nbd, nby, max_y, nullptr, cy.state, true};
  const uint3 *src = reinterpret_cast<const uint3 *>(src0 ? src0 : yrec);
  const uint64_t *bits64 = reinterpret_cast<const uint64_t *>(xbits);
  for (int p = 0; p < D.passes; ++p) {
    if (p > 0) ps.prepare(p, m, D, st);
    const bool last = p == D.passes - 1;
    uint3 *out = reinterpret_cast<uint3 *>(p % 2 == 0 ? tmp : const_cast<uint4 *>(yrec));
    uint32_t *stp = ps.use(p), *nxt = ps.next(p, D.passes), *ctr = status + sw - 64 + p;
    const uint32_t *gh = ghist_of(yhist, p);
    const double bytes = (p == 0 ? 12.0 + 0.125 : 12.0) * m + (last ? 18.0 : 12.0) * m;
    if (p == 0 && src0)
      y_after_x_first(SrcIdxYX12{src, bits64, (m + 63) / 64}, dc, out, last, m, D, gh, stp, ctr,
                      st, bytes, nxt);
    else if (p == 0)
      y_after_x_first(SrcYX12{src, bits64, (m + 63) / 64}, dc, out, last, m, D, gh, stp, ctr, st,
                      bytes, nxt);
    else if (last)
      launch_pass(SrcRec12{src}, dc, m, D.shift[p], D.db[p], gh, stp, ctr, st, bytes, nxt);
    else
      launch_pass(SrcRec12{src}, DstRec12{out}, m, D.shift[p], D.db[p], gh, stp, ctr, st, bytes,
                  nxt);
    src = out;
  }
}

// The same in two stages (round 5): the coarse passes over the Y key's top C
// bits (the first carrying the X-hit bits, the last counting each coarse
// key), then one block per coarse-key segment sorts the F fine bits in LDS
// and writes the CSR arrays and the Y states (CsrEmit).  The last record pass
// of the one-stage sort scattered the five CSR arrays over ~14-record digit
// segments (1-B stores: partial lines); a segment writes them whole.
// Buffers: yrec (records in processing order; later k_seg_big's A), tmp (the
// last coarse pass' output), tmp2 (scratch: the other coarse pass, k_seg_big's
// B); chist / coff: 2^C + 1 words each.
void nw_y_sort_split_after_x(uint4 *yrec, uint4 *tmp, uint4 *tmp2, uint32_t m,
                             const NwOrderPlan &yp, const uint32_t *yhist, uint32_t *status,
                             Csr cy, uint32_t nby, uint64_t max_y, const uint32_t *xbits,
                             uint32_t *chist, uint32_t *coff, ScanScratch ss, hipStream_t st) {
  const Digits D = to_digits(yp.coarse);
  const size_t sw = nw_status_words(m);
  const PassStatus ps = pass_status(status, m, D, 12);
  // the passes' tile counters, the first pass' status words, the coarse-key counts
  zero_regions(st, {{status + sw - 64, 64 * 4},
                    ps.region(0, m, D),
                    {chist, ((size_t)yp.nseg + 1) * 4}});
  uint3 *a = reinterpret_cast<uint3 *>(tmp), *b = reinterpret_cast<uint3 *>(tmp2);
  const uint3 *src = reinterpret_cast<const uint3 *>(yrec);
  const uint64_t *bits64 = reinterpret_cast<const uint64_t *>(xbits);
  for (int p = 0; p < D.passes; ++p) {
    if (p > 0) ps.prepare(p, m, D, st);
    const bool last = p == D.passes - 1;
    uint3 *out = ((D.passes - 1 - p) % 2 == 0) ? a : b;  // the last coarse pass lands in a
    uint32_t *stp = ps.use(p), *nxt = ps.next(p, D.passes), *ctr = status + sw - 64 + p;
    const uint32_t *gh = ghist_of(yhist, p);
    const double bytes = (p == 0 ? 12.0 + 0.125 : 12.0) * m + 12.0 * m;
    const DstRec12Hist dh{out, chist, yp.F};
    if (p == 0) {
      const SrcYX12 s0{src, bits64, (m + 63) / 64};
      if (last) launch_pass(s0, dh, m, D.shift[p], D.db[p], gh, stp, ctr, st, bytes, nxt);
      else launch_pass(s0, DstRec12{out}, m, D.shift[p], D.db[p], gh, stp, ctr, st, bytes, nxt);
    } else if (last) {
      launch_pass(SrcRec12{src}, dh, m, D.shift[p], D.db[p], gh, stp, ctr, st, bytes, nxt);
    } else {
      launch_pass(SrcRec12{src}, DstRec12{out}, m, D.shift[p], D.db[p], gh, stp, ctr, st, bytes,
                  nxt);
    }
    src = out;
  }
  exclusive_scan_u32_clear0(chist, coff, (size_t)yp.nseg + 1, ss, st);
  const DstCsr dc{cy.key, cy.ent, cy.pk, cy.nbd, nby, max_y, nullptr, cy.state, true};
  kt_begin(st, KID_NW_YFINE);
  // (the counts are free after the scan: the list of segments above OF_CAP)
  launch_seg(SegArgs<uint3>{a, reinterpret_cast<uint3 *>(yrec), b, coff, yp.nseg, yp.F, chist},
             CsrEmit{dc}, st);
  // records in; key, entry, packed record, neighbour code and state out
  kt_end(st, KID_NW_YFINE, 30.0 * m);
}

// The member sort by gid: 12-B records {gid, row, key} when every sort key
// fits 32 bits, else 16-B {gid, row, key low, key high}; pass 1 reads the X
// chunk kernel's {row, key low} (+ key high) and the gids.
template <class Rec, class Src1, class SrcN, class DstN>
static void nw_member_passes(const Src1 &s1, Rec *t0, Rec *t1, uint32_t m, const NwDigits &dg,
                             const uint32_t *ghist, uint32_t *status, const DstMembers &fin,
                             hipStream_t st) {
  const Digits D = to_digits(dg);
  const size_t sw = nw_status_words(m);
  const PassStatus ps = pass_status(status, m, D, (int)sizeof(Rec));
  // the passes' tile counters and the first pass' status words, one launch
  zero_regions(st, {{status + sw - 64, 64 * 4}, ps.region(0, m, D)});
  const double rb = sizeof(Rec), in1 = sizeof(Rec) == 12 ? 12.0 : 16.0;
  const Rec *src = nullptr;
  for (int p = 0; p < D.passes; ++p) {
    if (p > 0) ps.prepare(p, m, D, st);
    uint32_t *stp = ps.use(p), *nxt = ps.next(p, D.passes);
    uint32_t *ctr = status + sw - 64 + p;
    const uint32_t *gh = ghist + p * 1024;
    const bool last = p == D.passes - 1;
    Rec *out = p % 2 == 0 ? t0 : t1;
    const double in_b = p == 0 ? in1 : rb, out_b = last ? 20.0 : rb;
    if (p == 0) {
      if (last) launch_pass(s1, fin, m, D.shift[p], D.db[p], gh, stp, ctr, st, (in_b + out_b) * m, nxt);
      else launch_pass(s1, DstN{out}, m, D.shift[p], D.db[p], gh, stp, ctr, st, (in_b + out_b) * m, nxt);
    } else if (last) {
      launch_pass(SrcN{src}, fin, m, D.shift[p], D.db[p], gh, stp, ctr, st, (in_b + out_b) * m, nxt);
    } else {
      launch_pass(SrcN{src}, DstN{out}, m, D.shift[p], D.db[p], gh, stp, ctr, st, (in_b + out_b) * m, nxt);
    }
    src = out;
  }
}
void nw_member_sort(const uint4 *erec, const uint32_t *gidp, uint4 *t0, uint4 *t1, uint32_t m,
                    const NwDigits &e, const uint32_t *ehist, uint32_t *status, uint32_t *sgid,
                    uint64_t *key, uint32_t *tag, uint32_t *mrow, bool narrow_keys,
                    hipStream_t st) {
  const uint2 *erk = reinterpret_cast<const uint2 *>(erec);
  const uint32_t *ehi = reinterpret_cast<const uint32_t *>(erk + m);
  const DstMembers fin{sgid, tag, mrow, key};
  if (narrow_keys)
    nw_member_passes<uint3, SrcMem12, SrcRec12, DstRec12>(
        SrcMem12{erk, gidp}, reinterpret_cast<uint3 *>(t0), reinterpret_cast<uint3 *>(t1), m, e,
        ehist, status, fin, st);
  else
    nw_member_passes<uint4, SrcMem16, SrcRec, DstRec>(SrcMem16{erk, ehi, gidp}, t0, t1, m, e,
                                                      ehist, status, fin, st);
}

void nw_member_sort_split(const uint4 *erec, const uint32_t *gidp, uint4 *t0, uint4 *t1,
                          uint4 *t2, uint32_t m, uint32_t G, const NwOrderPlan &mp,
                          const uint32_t *ehist, uint32_t *status, uint32_t *sgid, uint64_t *key,
                          uint32_t *tag, uint32_t *mrow, uint32_t *goff, uint32_t *chist,
                          uint32_t *coff, ScanScratch ss, hipStream_t st) {
  const uint2 *erk = reinterpret_cast<const uint2 *>(erec);
  uint3 *a = reinterpret_cast<uint3 *>(t0), *b = reinterpret_cast<uint3 *>(t1),
        *c = reinterpret_cast<uint3 *>(t2);
  const Digits D = to_digits(mp.coarse);
  const size_t sw = nw_status_words(m);
  (void)hipMemsetAsync(status + sw - 64, 0, 64 * 4, st);  // the passes' tile counters
  (void)hipMemsetAsync(chist, 0, ((size_t)mp.nseg + 1) * 4, st);
  const PassStatus ps = pass_status(status, m, D, 12);
  const SrcMem12 s1{erk, gidp};
  const uint3 *src = nullptr;
  for (int p = 0; p < D.passes; ++p) {
    uint3 *out = ((D.passes - 1 - p) % 2 == 0) ? b : a;  // the last coarse pass lands in b
    ps.prepare(p, m, D, st);
    uint32_t *stp = ps.use(p), *nxt = ps.next(p, D.passes);
    uint32_t *ctr = status + sw - 64 + p;
    const uint32_t *gh = ehist + p * 1024;
    const bool last = p == D.passes - 1;
    const DstRec12Hist dh{out, chist, mp.F};
    const double bytes = 24.0 * m;
    if (p == 0 && last) launch_pass(s1, dh, m, D.shift[p], D.db[p], gh, stp, ctr, st, bytes, nxt);
    else if (p == 0) launch_pass(s1, DstRec12{out}, m, D.shift[p], D.db[p], gh, stp, ctr, st, bytes, nxt);
    else if (last) launch_pass(SrcRec12{src}, dh, m, D.shift[p], D.db[p], gh, stp, ctr, st, bytes, nxt);
    else launch_pass(SrcRec12{src}, DstRec12{out}, m, D.shift[p], D.db[p], gh, stp, ctr, st, bytes, nxt);
    src = out;
  }
  exclusive_scan_u32_clear0(chist, coff, (size_t)mp.nseg + 1, ss, st);
  kt_begin(st, KID_NW_MFINE);
  launch_seg(SegArgs<uint3>{b, a, c, coff, mp.nseg, mp.F, chist},
             MemberEmit{sgid, tag, mrow, key, goff, G, m}, st);
  // records in; gid, row, key (8 B), tag out; the group starts
  kt_end(st, KID_NW_MFINE, 32.0 * m + 4.0 * G);
}

// the member sort of the sharded driver: received {gid, row, key ...} records
// (12 B when every sort key fits 32 bits, else 16 B), gids made local (- g0)
void nw_member_sort_recv(const void *recs, bool narrow_keys, uint32_t m, uint32_t g0,
                         const NwDigits &e, const uint32_t *ehist, uint32_t *status, uint4 *t0,
                         uint4 *t1, uint32_t *sgid, uint64_t *key, uint32_t *tag, uint32_t *mrow,
                         hipStream_t st) {
  const DstMembers fin{sgid, tag, mrow, key};
  if (narrow_keys)
    nw_member_passes<uint3, SrcSub12, SrcRec12, DstRec12>(
        SrcSub12{reinterpret_cast<const uint3 *>(recs), g0}, reinterpret_cast<uint3 *>(t0),
        reinterpret_cast<uint3 *>(t1), m, e, ehist, status, fin, st);
  else
    nw_member_passes<uint4, SrcSub16, SrcRec, DstRec>(
        SrcSub16{reinterpret_cast<const uint4 *>(recs), g0}, t0, t1, m, e, ehist, status, fin, st);
}

uint32_t nw_chunk_width(uint32_t m, uint32_t nbx) {
  // about 256-512 rows per chunk (one batch of the chunk kernel), 64..1024 buckets
  const double per_bucket = (double)m / (double)(nbx ? nbx : 1);
  uint32_t W = 64;
  while (W < 1024 && per_bucket * (2 * W) <= 64.0 * XC_SLOTS) W *= 2;
  return W;
}

uint32_t nw_chunks(uint32_t nbx, uint32_t W) { return (nbx + W - 1) / W; }

void nw_x_count(const uint4 *R, uint32_t m, const NwChunkCounts &cc, hipStream_t st,
                const uint4 *halo, uint32_t G) {
  (void)hipMemsetAsync(cc.cnts, 0, ((size_t)3 * cc.nch + 1) * 4, st);
  if (!m) return;
  kt_begin(st, KID_NW_XCOUNT);
  k_nw_xcount<<<(m + XN_T * XN_ITEMS - 1) / (XN_T * XN_ITEMS), XN_T, 0, st>>>(
      RecView{halo, G, R}, m, cc.lgW, cc.nch, 10 * cc.W, cc.cnts);
  kt_end(st, KID_NW_XCOUNT, 16.0 * m);
}

void nw_x_count_add(const uint4 *halo, uint32_t G, const NwChunkCounts &cc, hipStream_t st) {
  if (!G) return;
  kt_begin(st, KID_NW_XCOUNT);
  k_nw_xcount<<<(G + XN_T * XN_ITEMS - 1) / (XN_T * XN_ITEMS), XN_T, 0, st>>>(
      RecView{halo, G, halo}, G, cc.lgW, cc.nch, 10 * cc.W, cc.cnts);
  kt_end(st, KID_NW_XCOUNT, 16.0 * G);
}

void nw_x_chunks(const uint4 *R, uint32_t m, uint32_t nbx, uint64_t max_x, uint32_t maxlen,
                 const uint32_t *xoff, Csr cx, uint32_t *xpos, uint4 *erec, uint32_t *ctrl,
                 uint32_t W, hipStream_t st, const uint4 *halo, uint32_t G) {
  if (!m) return;
  uint32_t lgW = 0;
  while ((1u << lgW) < W) ++lgW;
  const uint32_t nch = nw_chunks(nbx, W);
  // the member records take the erec buffer (16 B per row) as two arrays
  uint2 *erk = reinterpret_cast<uint2 *>(erec);
  XChunkArgs a{RecView{halo, G, R}, m, W, lgW, nch, (maxlen / 2 + 9) / 10, max_x, nbx, xoff, cx,
               xpos, erk, reinterpret_cast<uint32_t *>(erk + m), ctrl};
  kt_begin(st, KID_NW_XCHUNK);
  k_nw_xchunk<<<(nch + XC_WAVES - 1) / XC_WAVES, 64 * XC_WAVES,
                XC_WAVES * 2 * W * sizeof(uint32_t), st>>>(a);
  // records in (+ halo), X entries (key, id, packed record, code, state), their
  // positions by fragment and member records out
  kt_end(st, KID_NW_XCHUNK, 16.0 * m + 22.0 * m + 12.0 * m);  // records in; X CSR + position out; member records ({row, key lo} + key hi)
}

void nw_x_bits(const uint32_t *xpos, const uint8_t *xstate, uint32_t m, uint32_t *bits,
               hipStream_t st) {
  if (!m) return;
  kt_begin(st, KID_NW_XBITS);
  k_nw_x_bits<<<grid_for(m, 256), 256, 0, st>>>(xpos, xstate, m, bits);
  kt_end(st, KID_NW_XBITS, 5.0 * m);
}

void nw_fill_y(const uint32_t *ent, const uint32_t *bits, uint8_t *state, uint32_t m,
               hipStream_t st) {
  if (!m) return;
  kt_begin(st, KID_NW_FILLY);
  k_nw_fill_y<<<grid_for(m, 256), 256, 0, st>>>(ent, bits, state, m);
  kt_end(st, KID_NW_FILLY, 5.0 * m);
}

void nw_assign_jump(uint32_t *par, const uint32_t *newrank, uint32_t *gidp, uint32_t m,
                    const NwDigits &e, uint32_t *ehist, uint32_t *list, uint32_t *ctrl,
                    hipStream_t st) {
  if (!m) return;
  // the step budgets (RK_ROOTS_STEPS / RK_ROOTS_REST_STEPS: test hooks for the
  // listed chains and the round-by-round fallback)
  static const int steps1 = [] {
    const char *e = getenv("RK_ROOTS_STEPS");
    return e ? std::max(1, atoi(e)) : 32;
  }();
  static const int steps2 = [] {
    const char *e = getenv("RK_ROOTS_REST_STEPS");
    return e ? std::max(1, atoi(e)) : 4096;
  }();
  kt_begin(st, KID_NW_ASSIGN);
  k_nw_assign_jump<<<grid_for(m, 256, 2048), 256, 0, st>>>(par, newrank, gidp, m, to_digits(e),
                                                           ehist, list, ctrl + 12, ctrl, steps1);
  // parent, root (+ its parent), parent back, root's rank, gid
  kt_end(st, KID_NW_ASSIGN, 20.0 * m);
  k_nw_assign_rest<<<256, 256, 0, st>>>(par, newrank, gidp, m, to_digits(e), ehist, list,
                                        ctrl + 12, ctrl + 13, ctrl, steps2);
}

void nw_assign(const uint32_t *par, const uint32_t *newrank, uint32_t *gidp, uint32_t m,
               const NwDigits &e, uint32_t *ehist, hipStream_t st) {
  if (!m) return;
  kt_begin(st, KID_NW_ASSIGN);
  k_nw_assign<<<grid_for(m, 256, 2048), 256, 0, st>>>(par, newrank, gidp, m, to_digits(e),
                                                      ehist);
  kt_end(st, KID_NW_ASSIGN, 12.0 * m);
}

}  // namespace rk
