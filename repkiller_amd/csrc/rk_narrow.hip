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
//   * the Y axis records {bucket key, processing index, centre lo, length} are
//     written by the last processing-order pass and sorted on the second
//     stream while X resolves; the X results reach the Y axis through one
//     byte per fragment (xhit);
//   * group members {gid, row, sort key} are sorted by gid with the records
//     carried, straight into the arrays the in-group sort reads.
#include "rk_ctx.h"

namespace rk {
namespace {

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
__device__ __forceinline__ uint32_t look_back(uint32_t *status, uint32_t tile, uint32_t stride,
                                              uint32_t slot, uint32_t mine) {
  uint32_t acc = 0;
  for (uint32_t j = tile; j-- > 0;) {
    uint32_t v;
    while (((v = sw_load(&status[(size_t)j * stride + slot])) & ~SW_VAL) == 0)
      __builtin_amdgcn_s_sleep(1);
    acc += v & SW_VAL;
    if ((v & ~SW_VAL) == SW_INC) break;
  }
  sw_store(&status[(size_t)tile * stride + slot], SW_INC | (acc + mine));
  return acc;
}

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
  uint64_t b = c / 100;
  if (c < max_index && (c + 1) / 100 > b) b = (c + 1) / 100;
  if (c < max_index - 1 && (c + 2) / 100 > b) b = (c + 2) / 100;
  return b;
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

// ---------------------------------------------------------------------------
// One LSD pass: tile = T threads x ITEMS records; wave w ranks its contiguous
// slice (ITEMS rounds of 64) against a wave-private digit counter by DB
// ballots (index order = rank order: stable), one barrier turns the counts
// into tile-local starts, the look-back gives the tile's global start per
// digit, the records are placed in LDS at their sorted slot and written out
// slot by slot (consecutive lanes -> consecutive addresses of one segment).
// Src: load(i, thr) -> record i (and folds per-thread side data into thr),
// key(rec); Dst: store(pos, rec); Side: extra per-block work on every loaded
// record (histograms of a later sort, flags), flushed at the end.
struct NoSide {
  struct Lds {
    uint32_t unused;
  };
  struct Thr {};
  __device__ void init(Lds &) const {}
  __device__ void add(Lds &, const uint4 &, Thr &) const {}
  __device__ void flush(Lds &, Thr &) const {}
};

template <int T, int ITEMS, int DB, class Src, class Dst, class Side>
__global__ void __launch_bounds__(T) k_onesweep(Src src, Dst dst, Side side, uint32_t n, int shift,
                                                const uint32_t *__restrict__ ghist,
                                                uint32_t *__restrict__ status,
                                                uint32_t *__restrict__ tile_ctr) {
  constexpr int RADIX = 1 << DB, NW = T / 64, TILE = T * ITEMS, DPT = RADIX / T;
  static_assert(RADIX % T == 0, "whole digits per thread");
  __shared__ uint4 srec[TILE];
  __shared__ uint32_t wcnt[NW][RADIX];  // per-wave digit counters, then per-wave starts
  __shared__ uint32_t lbase[RADIX];     // tile-local start of digit d
  __shared__ uint32_t gpos[RADIX];      // global position of the tile's first digit-d record
  __shared__ uint32_t wsum[2][NW];
  __shared__ uint32_t s_tile;
  __shared__ typename Side::Lds sl;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
  if (threadIdx.x == 0) s_tile = atomicAdd(tile_ctr, 1u);
  for (uint32_t j = threadIdx.x; j < NW * RADIX; j += T) (&wcnt[0][0])[j] = 0;
  side.init(sl);
  __syncthreads();
  const uint32_t tile = s_tile;
  const uint32_t tile0 = tile * (uint32_t)TILE;
  const uint32_t cnt = n - tile0 < (uint32_t)TILE ? n - tile0 : (uint32_t)TILE;

  uint4 rec[ITEMS];
  uint32_t rk[ITEMS];
  typename Side::Thr thr{};
  const uint32_t wbase = (uint32_t)w * (TILE / NW) + lane;
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const uint32_t i = wbase + r * 64;
    rec[r] = i < cnt ? src.load(tile0 + i, thr) : make_uint4(0, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < ITEMS; ++r)
    if (wbase + r * 64 < cnt) side.add(sl, rec[r], thr);
  uint32_t *mycnt = wcnt[w];
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const bool live = wbase + r * 64 < cnt;
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
  // thread t owns digits [t*DPT, (t+1)*DPT): tile totals, wave starts, and the
  // exclusive scans of the tile totals (lbase) and of the global totals
  uint32_t run[DPT], gtot[DPT], tsum = 0, gsum = 0;
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
    gtot[j] = ghist[d];
    gsum += gtot[j];
  }
  // publish this tile's counts first (later tiles may be waiting for them)
#pragma unroll
  for (int j = 0; j < DPT; ++j)
    sw_store(&status[(size_t)tile * RADIX + threadIdx.x * DPT + j],
             (tile ? SW_AGG : SW_INC) | run[j]);
  uint32_t inc = tsum, ginc = gsum;
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t o = __shfl_up(inc, off), go = __shfl_up(ginc, off);
    if (lane >= off) inc += o, ginc += go;
  }
  if (lane == 63) wsum[0][w] = inc, wsum[1][w] = ginc;
  __syncthreads();
  {
    uint32_t pre = 0, gpre = 0;
    for (int k2 = 0; k2 < w; ++k2) pre += wsum[0][k2], gpre += wsum[1][k2];
    uint32_t at = pre + inc - tsum, gat = gpre + ginc - gsum;
#pragma unroll
    for (int j = 0; j < DPT; ++j) {
      const uint32_t d = threadIdx.x * DPT + j;
      lbase[d] = at;
      at += run[j];
      const uint32_t before = tile ? look_back(status, tile, RADIX, d, run[j]) : 0u;
      gpos[d] = gat + before;
      gat += gtot[j];
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    if (rk[r] == 0xFFFFFFFFu) continue;
    const uint32_t d = (src.key(rec[r]) >> shift) & (RADIX - 1);
    srec[lbase[d] + mycnt[d] + rk[r]] = rec[r];
  }
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < cnt; j += T) {
    const uint4 r = srec[j];
    const uint32_t d = (src.key(r) >> shift) & (RADIX - 1);
    dst.store(gpos[d] + (j - lbase[d]), r);
  }
  side.flush(sl, thr);
}

// records in a uint4 array, key = .x (streamed once: nontemporal loads)
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
struct SrcRec {
  const uint4 *in;
  struct Thr0 {};
  template <class Thr>
  __device__ __forceinline__ uint4 load(uint32_t i, Thr &) const {
    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(in + i));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  __device__ __forceinline__ uint32_t key(const uint4 &r) const { return r.x; }
};
struct DstRec {
  uint4 *out;
  __device__ __forceinline__ void store(uint32_t pos, const uint4 &r) const { out[pos] = r; }
};

// --- processing order, pass 1: the file-order SoA becomes records ----------
struct SrcFile {
  const uint64_t *x, *y, *len;
  const uint8_t *strand;
  uint64_t vsize;
  template <class Thr>
  __device__ __forceinline__ uint4 load(uint32_t i, Thr &t) const {
    const uint64_t xs = x[i], ys = y[i], L = len[i];
    const uint32_t s = strand[i] != 'f' ? 1u : 0u;
    const uint64_t pk = xs / 10;
    const uint32_t key = (uint32_t)(pk < vsize - 1 ? pk : vsize - 1);
    // not representable: the generic pipeline takes over (flag)
    t.wide |= L >= (1ull << 24) || ys >= (1ull << 35);
    return make_uint4(key, i, (uint32_t)ys,
                      (uint32_t)(L & 0xFFFFFFu) | s << 24 | (uint32_t)((ys >> 32) & 7u) << 25 |
                          (uint32_t)(xs % 10) << 28);
  }
  __device__ __forceinline__ uint32_t key(const uint4 &r) const { return r.x; }
};
// ... and, on the side, the Y axis' digit histograms, the forward-strand
// count, the longest length and the probe-range checks of every kept row
struct SideFile {
  Digits yd;
  uint64_t drop, max_x, max_y;
  uint32_t nby;
  uint32_t *yhist;  // [4][1024]
  uint32_t *ctrl;   // [0] error bits, [3] narrow-failure flag, [4] max length, [8] forward kept
  struct Lds {
    HistLds h;
    uint32_t red[3];
  };
  struct Thr {
    bool wide = false, ub = false;
    uint32_t maxlen = 0, fwd = 0;
  };
  __device__ void init(Lds &L) const {
    hist_init(L.h);
    if (threadIdx.x < 3) L.red[threadIdx.x] = 0;
  }
  __device__ void add(Lds &L, const uint4 &r, Thr &t) const {
    if (r.x == drop) return;  // the never-iterated last bucket
    const uint64_t xs = rec_x(r), ys = rec_y(r);
    const uint32_t len = rec_len(r), s = rec_strand(r);
    const uint64_t h = len / 2;
    if (probe_max_bucket_nw(xs + h, max_x) > max_x || probe_max_bucket_nw(ys + h, max_y) > max_y)
      t.ub = true;
    t.maxlen = len > t.maxlen ? len : t.maxlen;
    t.fwd += s == 0;
    const uint64_t yc = ys + h;
    hist_add(L.h, yd, s * nby + (uint32_t)(yc / 100));
  }
  __device__ void flush(Lds &L, Thr &t) const {
    // every add() of this block precedes the kernel's last barrier
    const uint64_t wide = __ballot(t.wide), ub = __ballot(t.ub);
    uint32_t mx = t.maxlen, fw = t.fwd;
    for (int off = 32; off > 0; off >>= 1) {
      const uint32_t o = __shfl_xor(mx, off);
      mx = o > mx ? o : mx;
      fw += __shfl_xor(fw, off);
    }
    if ((threadIdx.x & 63) == 0) {
      if (wide) atomicOr(&L.red[0], 1u);
      if (ub) atomicOr(&L.red[0], 2u);
      atomicMax(&L.red[1], mx);
      atomicAdd(&L.red[2], fw);
    }
    __syncthreads();
    hist_flush(L.h, yd, yhist);
    if (threadIdx.x == 0) {
      if (L.red[0] & 1u) atomicOr(&ctrl[3], 1u);
      if (L.red[0] & 2u) atomicOr(&ctrl[0], ERRB_UB_CENTER);
      atomicMax(&ctrl[4], L.red[1]);
      if (L.red[2]) atomicAdd(&ctrl[8], L.red[2]);
    }
  }
};

// --- processing order, last pass: the records, and the Y axis' input -------
// Yrec: {strand * nby + centre/100, processing index, centre low 32, length}
struct DstProc {
  uint4 *out, *yrec;
  uint32_t nby;
  __device__ __forceinline__ void store(uint32_t pos, const uint4 &r) const {
    out[pos] = r;
    const uint64_t ys = rec_y(r);
    const uint32_t len = rec_len(r), s = rec_strand(r);
    const uint64_t yc = ys + len / 2;
    yrec[pos] = make_uint4(s * nby + (uint32_t)(yc / 100), pos, (uint32_t)yc, len);
  }
};

// --- Y axis, last pass: the CSR arrays the sweeps read -----------------------
struct DstCsr {
  uint32_t *key, *ent;
  uint2 *pk;
  uint8_t *nbd;
  uint32_t nb;
  uint64_t max_index;
  __device__ __forceinline__ void store(uint32_t pos, const uint4 &r) const {
    key[pos] = r.x;
    ent[pos] = r.y;
    pk[pos] = make_uint2(r.z, r.w);
    const uint32_t b = r.x >= nb ? r.x - nb : r.x;
    const uint64_t base = (uint64_t)b * 100;
    const uint64_t c = base + (uint32_t)(r.z - (uint32_t)base);  // centre from bucket + low bits
    nbd[pos] = nbd_code_nw(c, max_index);
  }
};

// --- group members, last pass: gid order (stable: processing order inside) -
// members {gid, row, sort key lo, hi} -> group of every slot, sort key, tag =
// slot, file row
struct DstMembers {
  uint32_t *sgid, *tag, *mrow;
  uint64_t *key;
  __device__ __forceinline__ void store(uint32_t pos, const uint4 &r) const {
    sgid[pos] = r.x;
    mrow[pos] = r.y;
    key[pos] = (uint64_t)r.w << 32 | r.z;
    tag[pos] = pos;
  }
};

// ---------------------------------------------------------------------------
// processing-order histograms from xStart alone; kept rows; xStart/10 >= vsize
__global__ void __launch_bounds__(256) k_nw_order_hist(const uint64_t *__restrict__ x, uint32_t n,
                                                       uint64_t vsize, Digits D,
                                                       uint32_t *__restrict__ ghist,
                                                       uint32_t *__restrict__ ctrl) {
  __shared__ HistLds L;
  __shared__ uint32_t part[4];
  hist_init(L);
  __syncthreads();
  uint32_t kept = 0;
  bool ub = false;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint64_t pk = x[i] / 10;
    ub |= pk >= vsize;
    const uint32_t key = (uint32_t)(pk < vsize - 1 ? pk : vsize - 1);
    kept += key != vsize - 1;
    hist_add(L, D, key);
  }
  for (int off = 32; off > 0; off >>= 1) kept += __shfl_xor(kept, off);
  const uint64_t any_ub = __ballot(ub);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = kept;
  if ((threadIdx.x & 63) == 0 && any_ub) atomicOr(&ctrl[0], ERRB_UB_BUCKET);
  __syncthreads();
  hist_flush(L, D, ghist);
  if (threadIdx.x == 0) {
    const uint32_t t = part[0] + part[1] + part[2] + part[3];
    if (t) atomicAdd(&ctrl[1], t);
  }
}

// ---------------------------------------------------------------------------
// X axis by chunks of W centre buckets (both strands), from the processing
// order.  Chunk c (dynamic id) owns buckets [cW, (c+1)W); its entries are the
// rows with xStart/10 in [10cW - ceil(H/10), 10(c+1)W) whose centre falls in
// the chunk (H = longest length / 2): a contiguous row range found by three
// wave-wide 64-ary searches.  Entries are collected in row order into LDS,
// ranked within their bucket in that order (stable = processing order),
// counted per strand and placed by a look-back over the chunks: forward
// entries at [0, M0), the others after.  The same pass writes every OWNED row's
// member record {0, row, sort key}: the sort key needs the yStart of the last
// row of its xStart/10 run, and chunk borders are run borders.
constexpr int XC_T = 256, XC_CAP = 2048;
struct XChunkArgs;

__device__ __forceinline__ uint32_t wave_lower_bound(const uint4 *R, uint32_t m, uint32_t T) {
  const uint32_t *key = reinterpret_cast<const uint32_t *>(R);
  const uint32_t lane = threadIdx.x & 63;
  uint32_t lo = 0, hi = m;  // answer in [lo, hi]: first row with key >= T
  while (hi - lo > 64) {
    const uint32_t step = (hi - lo + 63) / 64;
    const uint32_t p = lo + lane * step;
    const bool pred = p < hi && key[4 * (size_t)p] < T;
    const uint32_t c = __popcll(__ballot(pred));
    if (c == 0) return lo;
    const uint32_t nlo = lo + (c - 1) * step + 1;
    const uint32_t nhi = c < 64 ? min(hi, lo + c * step) : hi;
    lo = nlo;
    hi = nhi;
  }
  const uint32_t p = lo + lane;
  const bool pred = p < hi && key[4 * (size_t)p] < T;
  return lo + (uint32_t)__popcll(__ballot(pred));
}

struct XChunkArgs {
  const uint4 *R;     // processing order
  uint32_t m;         // kept rows
  uint32_t W, lgW;    // chunk width in buckets (power of two)
  uint32_t nchunks;
  uint32_t halo;      // ceil(H / 10) in xStart/10 units
  uint32_t nbx;
  uint64_t max_x;
  uint32_t M0;        // forward-strand entries (all chunks)
  Csr out;
  uint4 *erec;        // member records (processing order)
  uint32_t *status;   // [nchunks][2]
  uint32_t *ctr;
  uint32_t *ctrl;     // [0] err bits, [6] wide sort keys, [7] chunk overflow
};

// a chunk entry from its processing-order record (mine: its centre bucket is
// in the chunk)
struct XEnt {
  bool mine;
  uint32_t bin, s;
  uint64_t xc;
  uint32_t len;
};
__device__ __forceinline__ XEnt x_entry(const uint4 &r, bool in, uint64_t b0, uint32_t W) {
  XEnt e;
  const uint64_t xs = rec_x(r);
  e.len = rec_len(r);
  e.s = rec_strand(r);
  e.xc = xs + e.len / 2;
  const uint64_t bk = e.xc / 100;
  e.mine = in && bk >= b0 && bk < b0 + W;
  e.bin = (uint32_t)(e.s * W + (bk - b0));
  return e;
}

// Rank the LDS list ent[0, cnt) (row order) within each bin against the
// running per-bin counters rcnt, by one wavefront 64 entries at a time
// (DB ballots; stable), and place entry i at CSR position start[bin] + rank.
__device__ __forceinline__ void rank_and_write(const XChunkArgs &a, const uint4 *ent, uint32_t cnt,
                                               uint32_t *rcnt, const uint32_t *start, int bits,
                                               uint64_t b0, uint32_t off_f, uint32_t off_r,
                                               uint32_t nf) {
  const uint32_t lane = threadIdx.x & 63;
  if (threadIdx.x >= 64) return;
  for (uint32_t r0 = 0; r0 < cnt; r0 += 64) {
    const uint32_t i = r0 + lane;
    const bool live = i < cnt;
    const uint4 e = live ? ent[i] : make_uint4(0, 0, 0, 0);
    const uint32_t bin = e.x;
    uint64_t peer = __ballot(live);
    for (int b = 0; b < bits; ++b) {
      const bool bit = (bin >> b) & 1u;
      const uint64_t bb = __ballot(bit);
      peer &= bit ? bb : ~bb;
    }
    const uint32_t below = __popcll(peer & ((1ull << lane) - 1ull));
    const uint32_t before = live ? rcnt[bin] : 0u;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    if (live && below == 0) rcnt[bin] = before + __popcll(peer);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (!live) continue;
    const uint32_t loc = start[bin] + before + below;
    const uint32_t s = bin >= a.W ? 1u : 0u;
    const uint32_t q = s == 0 ? off_f + loc : a.M0 + off_r + (loc - nf);
    const uint64_t bk = b0 + (bin - s * a.W);
    const uint64_t cbase = bk * 100;
    const uint64_t xc = cbase + (uint32_t)(e.z - (uint32_t)cbase);
    a.out.key[q] = s * a.nbx + (uint32_t)bk;
    a.out.ent[q] = e.y;
    a.out.pk[q] = make_uint2(e.z, e.w);
    a.out.nbd[q] = nbd_code_nw(xc, a.max_x);
    a.out.state[q] = ST_UNKNOWN;
  }
}

__global__ void __launch_bounds__(XC_T) k_nw_xchunk(XChunkArgs a) {
  constexpr int NW = XC_T / 64;
  __shared__ uint4 ent[XC_CAP];      // {bin, row k, centre lo, length}, row order
  __shared__ uint32_t hcnt[2048];    // per-bin counts, then starts
  __shared__ uint32_t rcnt[2048];    // running per-bin ranks
  __shared__ uint32_t s_chunk, s_rng[3], s_n, s_nf, s_wofs[NW], s_hi, s_bad;
  __shared__ uint32_t s_off[2];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (threadIdx.x == 0) s_chunk = atomicAdd(a.ctr, 1u), s_n = 0, s_nf = 0, s_bad = 0;
  __syncthreads();
  const uint32_t c = s_chunk;
  const uint64_t own = (uint64_t)10 * a.W * c, nxt = own + (uint64_t)10 * a.W;
  if (w < 3) {
    const uint64_t t64 = w == 0 ? (own > a.halo ? own - a.halo : 0) : w == 1 ? own : nxt;
    const uint32_t t = t64 > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)t64;
    const uint32_t r = wave_lower_bound(a.R, a.m, t);
    if (lane == 0) s_rng[w] = r;
  }
  for (uint32_t j = threadIdx.x; j < 2 * a.W; j += XC_T) hcnt[j] = 0, rcnt[j] = 0;
  __syncthreads();
  const uint32_t kA = s_rng[0], kO = s_rng[1], kB = s_rng[2];
  const uint64_t b0 = (uint64_t)a.W * c;
  bool wide_key = false;
  // rows in order: X entries of this chunk -> per-bin counts and the LDS list
  // (while it fits); owned rows -> sort keys
  for (uint32_t base = kA; base < kB; base += XC_T) {
    const uint32_t k = base + threadIdx.x;
    const bool in = k < kB;
    const uint4 r = in ? a.R[k] : make_uint4(0, 0, 0, 0);
    const XEnt e = x_entry(r, in, b0, a.W);
    const uint64_t bal = __ballot(e.mine), fbal = __ballot(e.mine && e.s == 0);
    if (lane == 0) s_wofs[w] = __popcll(bal), atomicAdd(&s_nf, (uint32_t)__popcll(fbal));
    if (e.mine) atomicAdd(&hcnt[e.bin], 1u);
    __syncthreads();
    uint32_t at = s_n;
    for (uint32_t q = 0; q < w; ++q) at += s_wofs[q];
    at += __popcll(bal & ((1ull << lane) - 1ull));
    if (e.mine && at < XC_CAP) ent[at] = make_uint4(e.bin, k, (uint32_t)e.xc, e.len);
    // owned rows: |yStart - yStart(last row of the xStart/10 run)|
    const bool owned = in && k >= kO;
    if (__ballot(owned)) {
      const uint32_t key = r.x;
      const uint64_t ys = rec_y(r);
      const bool end = owned && (k + 1 >= kB || a.R[k + 1].x != key);
      const uint64_t ends = __ballot(end) & ~((1ull << lane) - 1ull);
      const int src = ends ? __ffsll((unsigned long long)ends) - 1 : 63;
      uint64_t d = __shfl(ys, src);
      if (__ballot(owned && !ends)) {  // the wave's last run continues past it
        const uint32_t klast = __shfl(key, 63);
        uint32_t eidx = 0;
        for (uint32_t b = base + (w + 1) * 64;; b += 64) {
          const uint32_t q = b + lane;
          const uint64_t stop = __ballot(q >= kB || a.R[q].x != klast);
          if (stop) {
            eidx = b + __builtin_ctzll(stop) - 1;
            break;
          }
        }
        if (owned && !ends) d = rec_y(a.R[eidx]);
      }
      if (owned) {
        const uint64_t h = ys > d ? ys - d : d - ys;
        a.erec[k] = make_uint4(0, r.y, (uint32_t)h, (uint32_t)(h >> 32));
        wide_key |= (h >> 32) != 0;
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t t = 0;
      for (uint32_t q = 0; q < NW; ++q) t += s_wofs[q];
      s_n += t;
    }
    __syncthreads();
  }
  const uint64_t any_wide = __ballot(wide_key);
  if ((threadIdx.x & 63) == 0 && any_wide && *(volatile uint32_t *)&a.ctrl[6] == 0)
    atomicOr(&a.ctrl[6], 1u);
  const uint32_t n = s_n, nf = s_nf;
  // place the chunk among the chunks (per strand)
  if (threadIdx.x < 2) {
    const uint32_t mine = threadIdx.x == 0 ? nf : n - nf;
    if (c == 0) {
      sw_store(&a.status[threadIdx.x], SW_INC | mine);
      s_off[threadIdx.x] = 0;
    } else {
      sw_store(&a.status[2 * (size_t)c + threadIdx.x], SW_AGG | mine);
      s_off[threadIdx.x] = look_back(a.status, c, 2, threadIdx.x, mine);
    }
  }
  // bin starts: exclusive scan of the 2W counts
  {
    const uint32_t per = (2 * a.W + XC_T - 1) / XC_T;
    uint32_t tot = 0;
    for (uint32_t j = 0; j < per; ++j) {
      const uint32_t bn = threadIdx.x * per + j;
      tot += bn < 2 * a.W ? hcnt[bn] : 0u;
    }
    uint32_t inc = tot;
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t o = __shfl_up(inc, off);
      if ((int)lane >= off) inc += o;
    }
    if (lane == 63) s_wofs[w] = inc;
    __syncthreads();
    uint32_t at = inc - tot;
    for (uint32_t q = 0; q < w; ++q) at += s_wofs[q];
    for (uint32_t j = 0; j < per; ++j) {
      const uint32_t bn = threadIdx.x * per + j;
      if (bn < 2 * a.W) {
        const uint32_t cn = hcnt[bn];
        hcnt[bn] = at;
        at += cn;
      }
    }
  }
  __syncthreads();
  const uint32_t off_f = s_off[0], off_r = s_off[1];
  const int bits = (int)a.lgW + 1;
  if (n <= XC_CAP) {
    rank_and_write(a, ent, n, rcnt, hcnt, bits, b0, off_f, off_r, nf);
    return;
  }
  // A chunk denser than the list: its bins in ranges of at most XC_CAP
  // entries, the rows re-read once per range.
  for (uint32_t blo = 0; blo < 2 * a.W;) {
    if (threadIdx.x == 0) {
      // the widest bin range [blo, hi) of at most XC_CAP entries (at least one bin;
      // bin starts are non-decreasing, the end of bin b is the start of b + 1)
      const uint32_t nb = 2 * a.W;
      auto end_of = [&](uint32_t b) { return b + 1 < nb ? hcnt[b + 1] : n; };
      uint32_t hi = blo + 1;
      while (hi < nb && end_of(hi) - hcnt[blo] <= XC_CAP) ++hi;
      // a single bin above the list capacity: the generic pipeline takes over
      if (end_of(blo) - hcnt[blo] > XC_CAP) s_bad = 1;
      s_hi = hi;
      s_n = 0;
    }
    __syncthreads();
    if (s_bad) break;
    const uint32_t bhi = s_hi;
    for (uint32_t base = kA; base < kB; base += XC_T) {
      const uint32_t k = base + threadIdx.x;
      const bool in = k < kB;
      const uint4 r = in ? a.R[k] : make_uint4(0, 0, 0, 0);
      const XEnt e = x_entry(r, in, b0, a.W);
      const bool take = e.mine && e.bin >= blo && e.bin < bhi;
      const uint64_t bal = __ballot(take);
      if (lane == 0) s_wofs[w] = __popcll(bal);
      __syncthreads();
      uint32_t at = s_n;
      for (uint32_t q = 0; q < w; ++q) at += s_wofs[q];
      at += __popcll(bal & ((1ull << lane) - 1ull));
      if (take) ent[at] = make_uint4(e.bin, k, (uint32_t)e.xc, e.len);
      __syncthreads();
      if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (uint32_t q = 0; q < NW; ++q) t += s_wofs[q];
        s_n += t;
      }
      __syncthreads();
    }
    rank_and_write(a, ent, s_n, rcnt, hcnt, bits, b0, off_f, off_r, nf);
    __syncthreads();
    blo = bhi;
  }
  if (s_bad && threadIdx.x == 0) atomicOr(&a.ctrl[7], 1u);
}

// Y states: X hits sit in the Y lists (commonFunctions.cpp:59), X misses query them
__global__ void k_nw_fill_y(const uint32_t *__restrict__ ent, const uint8_t *__restrict__ xhit,
                            uint8_t *__restrict__ state, uint32_t m) {
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < m; q += gridDim.x * blockDim.x)
    state[q] = xhit[ent[q]] ? ST_ACTIVE : ST_UNKNOWN;
}

// gid of every member (its root's rank among new groups) into its record,
// and the member sort's digit histograms
__global__ void __launch_bounds__(256) k_nw_assign(const uint32_t *__restrict__ par,
                                                   const uint32_t *__restrict__ newrank,
                                                   uint4 *__restrict__ erec, uint32_t m, Digits D,
                                                   uint32_t *__restrict__ ghist) {
  __shared__ HistLds L;
  hist_init(L);
  __syncthreads();
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < m; k += gridDim.x * blockDim.x) {
    const uint32_t g = newrank[par[k]];
    reinterpret_cast<uint32_t *>(erec)[4 * (size_t)k] = g;
    hist_add(L, D, g);
  }
  __syncthreads();
  hist_flush(L, D, ghist);
}

// ---------------------------------------------------------------------------
Digits plan_digits(int bits) {
  Digits D{};
  if (bits < 1) bits = 1;
  D.passes = (bits + 9) / 10;
  int shift = 0;
  for (int p = 0; p < D.passes; ++p) {
    const int left = bits - shift, w0 = (left + (D.passes - p) - 1) / (D.passes - p);
    D.shift[p] = shift;
    D.db[p] = w0 < 8 ? 8 : w0;
    shift += w0;
  }
  return D;
}

constexpr int OS_T = 256;
int items_for(int db) { return db >= 10 ? 12 : 16; }
uint32_t tiles_for(uint32_t n, int db) {
  const uint32_t tile = OS_T * items_for(db);
  return (n + tile - 1) / tile;
}

template <int DB, class Src, class Dst, class Side>
void launch_pass_db(const Src &src, const Dst &dst, const Side &side, uint32_t n, int shift,
                    const uint32_t *ghist, uint32_t *status, uint32_t *ctr, hipStream_t st) {
  constexpr int ITEMS = DB >= 10 ? 12 : 16;
  const uint32_t tiles = (n + OS_T * ITEMS - 1) / (OS_T * ITEMS);
  k_onesweep<OS_T, ITEMS, DB><<<tiles, OS_T, 0, st>>>(src, dst, side, n, shift, ghist, status,
                                                       ctr);
}
template <class Src, class Dst, class Side>
void launch_pass(const Src &src, const Dst &dst, const Side &side, uint32_t n, int shift, int db,
                 const uint32_t *ghist, uint32_t *status, uint32_t *ctr, hipStream_t st,
                 double bytes) {
  if (!n) return;
  kt_begin(st);
  switch (db) {
    case 8: launch_pass_db<8>(src, dst, side, n, shift, ghist, status, ctr, st); break;
    case 9: launch_pass_db<9>(src, dst, side, n, shift, ghist, status, ctr, st); break;
    default: launch_pass_db<10>(src, dst, side, n, shift, ghist, status, ctr, st); break;
  }
  kt_end(st, KID_ONESWEEP, bytes);
}

}  // namespace

// ===========================================================================
// host side
size_t nw_status_words(uint32_t n) {
  // the largest pass: tiles of 3072 records x 1024 digits, + per-pass tile counters
  return (size_t)((n + 3071) / 3072 + 1) * 1024 + 64;
}

NwDigits nw_plan(int bits) {
  const Digits D = plan_digits(bits);
  NwDigits o{};
  o.passes = D.passes;
  for (int p = 0; p < 4; ++p) o.shift[p] = D.shift[p], o.db[p] = D.db[p];
  return o;
}

static Digits to_digits(const NwDigits &o) {
  Digits D{};
  D.passes = o.passes;
  for (int p = 0; p < 4; ++p) D.shift[p] = o.shift[p], D.db[p] = o.db[p];
  return D;
}

void nw_order_hist(const rk_frags_soa &in, uint64_t vsize, const NwDigits &a, uint32_t *ghist,
                   uint32_t *ctrl, hipStream_t st) {
  const uint32_t n = (uint32_t)in.n;
  if (!n) return;
  kt_begin(st);
  k_nw_order_hist<<<grid_for(n, 256, 2048), 256, 0, st>>>(in.x_start, n, vsize, to_digits(a),
                                                          ghist, ctrl);
  kt_end(st, KID_NW_HIST, 8.0 * n);  // xStart read once
}

// the processing order: passes over records, the first one from the file SoA
void nw_order_sort(const rk_frags_soa &in, uint64_t vsize, uint64_t max_x, uint64_t max_y,
                   uint32_t nby, const NwDigits &a, const NwDigits &y, const uint32_t *ghist,
                   uint32_t *yhist, uint32_t *status, uint4 *Ra, uint4 *Rb, uint4 *yrec,
                   uint32_t *ctrl, hipStream_t st) {
  const uint32_t n = (uint32_t)in.n;
  const Digits D = to_digits(a);
  const size_t sw = nw_status_words(n);
  (void)hipMemsetAsync(status + sw - 64, 0, 64 * 4, st);  // the passes' tile counters
  // the final pass lands in Ra
  for (int p = 0; p < D.passes; ++p) {
    uint4 *out = ((D.passes - 1 - p) % 2 == 0) ? Ra : Rb;
    const uint4 *src = ((D.passes - p) % 2 == 0) ? Ra : Rb;  // the previous pass' output
    const size_t status_bytes = (size_t)tiles_for(n, D.db[p]) * ((size_t)1 << D.db[p]) * 4;
    (void)hipMemsetAsync(status, 0, status_bytes, st);
    uint32_t *ctr = status + sw - 64 + p;
    const uint32_t *gh = ghist + p * 1024;
    const bool last = p == D.passes - 1;
    if (p == 0) {
      SrcFile sf{in.x_start, in.y_start, in.length, in.strand, vsize};
      SideFile side{to_digits(y), vsize - 1, max_x, max_y, nby, yhist, ctrl};
      if (last)
        launch_pass(sf, DstProc{out, yrec, nby}, side, n, D.shift[p], D.db[p], gh, status, ctr,
                    st, 25.0 * n + 32.0 * n);
      else
        launch_pass(sf, DstRec{out}, side, n, D.shift[p], D.db[p], gh, status, ctr, st,
                    25.0 * n + 16.0 * n);
    } else if (last) {
      launch_pass(SrcRec{src}, DstProc{out, yrec, nby}, NoSide{}, n, D.shift[p], D.db[p], gh,
                  status, ctr, st, 48.0 * n);
    } else {
      launch_pass(SrcRec{src}, DstRec{out}, NoSide{}, n, D.shift[p], D.db[p], gh, status, ctr, st,
                  32.0 * n);
    }
  }
}

// a sort of m 16-B records by .x, the last pass writing through `final`
template <class Final>
static void nw_sort_records(const uint4 *in, uint4 *t0, uint4 *t1, uint32_t m, const NwDigits &dg,
                            const uint32_t *ghist, uint32_t *status, const Final &fin,
                            double final_bytes, hipStream_t st) {
  const Digits D = to_digits(dg);
  const size_t sw = nw_status_words(m);
  (void)hipMemsetAsync(status + sw - 64, 0, 64 * 4, st);  // the passes' tile counters
  const uint4 *src = in;
  for (int p = 0; p < D.passes; ++p) {
    const size_t status_bytes = (size_t)tiles_for(m, D.db[p]) * ((size_t)1 << D.db[p]) * 4;
    (void)hipMemsetAsync(status, 0, status_bytes, st);
    uint32_t *ctr = status + sw - 64 + p;
    const uint32_t *gh = ghist + p * 1024;
    if (p == D.passes - 1) {
      launch_pass(SrcRec{src}, fin, NoSide{}, m, D.shift[p], D.db[p], gh, status, ctr, st,
                  16.0 * m + final_bytes);
    } else {
      uint4 *out = p % 2 == 0 ? t0 : t1;
      launch_pass(SrcRec{src}, DstRec{out}, NoSide{}, m, D.shift[p], D.db[p], gh, status, ctr,
                  st, 32.0 * m);
      src = out;
    }
  }
}

void nw_y_sort(const uint4 *yrec, uint4 *tmp, uint32_t m, const NwDigits &y, const uint32_t *yhist,
               uint32_t *status, Csr cy, uint32_t nby, uint64_t max_y, hipStream_t st) {
  // intermediates alternate tmp, yrec (yrec is free once the first pass read it)
  nw_sort_records(yrec, tmp, const_cast<uint4 *>(yrec), m, y, yhist, status,
                  DstCsr{cy.key, cy.ent, cy.pk, cy.nbd, nby, max_y}, 17.0 * m, st);
}

void nw_member_sort(const uint4 *erec, uint4 *t0, uint4 *t1, uint32_t m, const NwDigits &e,
                    const uint32_t *ehist, uint32_t *status, uint32_t *sgid, uint64_t *key,
                    uint32_t *tag, uint32_t *mrow, hipStream_t st) {
  nw_sort_records(erec, t0, t1, m, e, ehist, status, DstMembers{sgid, tag, mrow, key}, 20.0 * m,
                  st);
}

uint32_t nw_chunk_width(uint32_t m, uint32_t nbx) {
  // about XC_CAP / 3 entries per chunk on average, 128..1024 buckets
  const double per_bucket = (double)m / (double)nbx;
  uint32_t W = 128;
  while (W < 1024 && per_bucket * (2 * W) <= XC_CAP / 3.0) W *= 2;
  return W;
}

void nw_x_chunks(const uint4 *R, uint32_t m, uint32_t nbx, uint64_t max_x, uint32_t maxlen,
                 uint32_t M0, Csr cx, uint4 *erec, uint32_t *status, uint32_t *ctrl,
                 uint32_t W, hipStream_t st) {
  if (!m) return;
  uint32_t lgW = 0;
  while ((1u << lgW) < W) ++lgW;
  const uint32_t nchunks = (nbx + W - 1) / W;
  (void)hipMemsetAsync(status, 0, ((size_t)nchunks * 2 + 64) * 4, st);
  XChunkArgs a{R, m, W, lgW, nchunks, (maxlen / 2 + 9) / 10, nbx, max_x, M0, cx, erec,
               status, status + (size_t)nchunks * 2 + 32, ctrl};
  kt_begin(st);
  k_nw_xchunk<<<nchunks, XC_T, 0, st>>>(a);
  // records in (+ halo), X entries (key, id, packed record, code, state) and
  // member records out
  kt_end(st, KID_NW_XCHUNK, 16.0 * m + 18.0 * m + 16.0 * m);
}

void nw_fill_y(const uint32_t *ent, const uint8_t *xhit, uint8_t *state, uint32_t m,
               hipStream_t st) {
  if (!m) return;
  kt_begin(st);
  k_nw_fill_y<<<grid_for(m, 256), 256, 0, st>>>(ent, xhit, state, m);
  kt_end(st, KID_NW_FILLY, 6.0 * m);
}

void nw_assign(const uint32_t *par, const uint32_t *newrank, uint4 *erec, uint32_t m,
               const NwDigits &e, uint32_t *ehist, hipStream_t st) {
  if (!m) return;
  kt_begin(st);
  k_nw_assign<<<grid_for(m, 256, 2048), 256, 0, st>>>(par, newrank, erec, m, to_digits(e),
                                                      ehist);
  kt_end(st, KID_NW_ASSIGN, 12.0 * m);
}

}  // namespace rk
