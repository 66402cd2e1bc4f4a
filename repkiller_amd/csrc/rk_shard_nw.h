// rk_shard_nw.h -- rk_classify_sharded on the record pipeline's internals.
// Part of rk_shard.hip's translation unit (included inside namespace rk {
// namespace { ... } } after the driver infrastructure: Shard, the partition
// plans, Bounds, the Y-halo codes and the root kernels).
//
// The same stages as the generic sharded driver (rk_shard.hip's header
// comment), with the single-device record pipeline (rk_narrow.hip) inside
// each stage instead of 32-B rows, pair sorts and gathers:
//   ingress   rows leave their rank as 16-B processing-order records {xStart/10,
//             global file row, yStart lo, length | strand | yStart hi |
//             xStart % 10}; the slice owner sorts them with the one-sweep
//             passes (the last pass also writes the 12-B Y records with GLOBAL
//             processing indices);
//   X axis    the lead-in halo arrives as the same 16-B records (the row word
//             replaced by the global processing index) and sits AHEAD of the
//             own records: the X-chunk kernel builds the axis straight from
//             [halo ; own], no sort;
//   Y axis    12-B Y records go to their Y-range owners and are sorted there
//             (the first pass numbers them by arrival: arrival order = global
//             processing order); the X-hit bits follow in the same order, as
//             one byte per record, and become the tail pass' state bitmask;
//   members   12-B {gid, global row, sort key} records (16 B when a sort key
//             needs more than 32 bits) go to gid-range owners and are sorted
//             by local gid with the one-sweep passes into the group sort.
// Every row has to pack into a record (length < 2^24, yStart < 2^35, as in
// the single-device record pipeline); otherwise every rank agrees to run the
// generic driver.  At world size 1 an exchange hands the send block over
// without a copy.
#pragma once

constexpr int RK_SHARD_FALLBACK = 1 << 20;  // not a status: run the generic driver

// largest bucket index get_associated_group touches for centre c
// (SequenceOcupationList.cpp:47-89; the same bound as rk_narrow.hip's)
__device__ __forceinline__ uint64_t probe_max_bucket_sh(uint64_t c, uint64_t max_index) {
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

// 16-B record fields (rk_narrow.hip's layout)
__device__ __forceinline__ uint64_t nwr_x(const uint4 &r) { return (uint64_t)r.x * 10 + (r.w >> 28); }
__device__ __forceinline__ uint32_t nwr_len(const uint4 &r) { return r.w & 0xFFFFFFu; }
__device__ __forceinline__ uint64_t nwr_xbucket(const uint4 &r) {
  return (nwr_x(r) + nwr_len(r) / 2) / 100;
}
// 12-B Y record: {strand * nby + bucket, id, length | centre % 100 << 24}
__device__ __forceinline__ uint32_t nwy_bucket(const uint3 &r, uint32_t nby) {
  return r.x >= nby ? r.x - nby : r.x;
}

// ---- source side: processing keys, the checks, the slice histogram --------
// ctrl: [0] error bits, [20] some kept row does not pack, [21] longest kept
// length, [25] kept rows
struct ShRowsArgs {
  Frags f;
  uint64_t vsize, max_x, max_y;
  uint32_t shift;
  uint32_t *hist, *ctrl;  // hist null: one rank owns everything, no bounds to find
  uint32_t *yhist = nullptr;  // (fast path) the Y-centre bucket histogram, bins >> yshift
  uint32_t yshift = 0;
};
__device__ __forceinline__ uint64_t div10_sh(uint64_t v) {  // 32-bit when it fits
  return v < (1ull << 32) ? (uint64_t)((uint32_t)v / 10u) : v / 10;
}
__global__ void __launch_bounds__(256) k_sh_rows(ShRowsArgs a) {
  __shared__ uint32_t h[NBINS], hy[NBINS];
  __shared__ uint32_t red[3];
  for (uint32_t b = threadIdx.x; b < NBINS; b += 256) h[b] = hy[b] = 0;
  if (threadIdx.x < 3) red[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t drop = a.vsize - 1;
  uint32_t maxlen = 0, kept = 0;
  bool ub = false, ubc = false, wide = false;
  GRID_STRIDE(i, a.f.n) {
    const uint64_t xs = a.f.x[i], ys = a.f.y[i], L0 = a.f.len[i];
    const uint64_t pk = div10_sh(xs);
    ub |= pk >= a.vsize;
    if (pk >= drop) continue;  // the never-iterated last bucket (or out of bounds)
    ++kept;
    wide |= L0 >= (1ull << 24) || ys >= (1ull << 35);
    const uint32_t len = (uint32_t)(L0 & 0xFFFFFFu);  // exact whenever the row packs
    maxlen = len > maxlen ? len : maxlen;
    const uint64_t hl = len / 2;
    ubc |= probe_max_bucket_sh(xs + hl, a.max_x) > a.max_x ||
           probe_max_bucket_sh(ys + hl, a.max_y) > a.max_y;
    if (a.hist) atomicAdd(&h[(uint32_t)pk >> a.shift], 1u);
    if (a.yhist) {  // the Y record's bucket (rk_narrow.hip DstProc): centre yStart + len / 2
      const uint64_t yb = ((ys + hl) / 100) >> a.yshift;
      if (yb < NBINS) atomicAdd(&hy[yb], 1u);
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t o = __shfl_xor(maxlen, off);
    maxlen = o > maxlen ? o : maxlen;
    kept += __shfl_xor(kept, off);
  }
  const uint64_t bub = __ballot(ub), bubc = __ballot(ubc), bwide = __ballot(wide);
  if ((threadIdx.x & 63) == 0) {
    atomicMax(&red[0], maxlen);
    atomicOr(&red[1], (bub ? 1u : 0u) | (bubc ? 2u : 0u) | (bwide ? 4u : 0u));
    atomicAdd(&red[2], kept);
  }
  __syncthreads();
  if (a.hist)
    for (uint32_t b = threadIdx.x; b < NBINS; b += 256)
      if (h[b]) atomicAdd(&a.hist[b], h[b]);
  if (a.yhist)
    for (uint32_t b = threadIdx.x; b < NBINS; b += 256)
      if (hy[b]) atomicAdd(&a.yhist[b], hy[b]);
  if (threadIdx.x == 0) {
    if (red[2]) atomicAdd(&a.ctrl[25], red[2]);
    if (red[0]) atomicMax(&a.ctrl[21], red[0]);
    if (red[1] & 1u) atomicOr(&a.ctrl[0], ERRB_UB_BUCKET);
    if (red[1] & 2u) atomicOr(&a.ctrl[0], ERRB_UB_CENTER);
    if (red[1] & 4u) atomicOr(&a.ctrl[20], 1u);
  }
}

// ---- partition ops ----------------------------------------------------------
struct RowOp16 {  // kept rows -> slice owners, as processing-order records
  Frags f;
  Bounds B;
  uint32_t drop, row_base;
  uint4 *out;
  __device__ uint32_t key(uint32_t i) const {
    const uint64_t pk = div10_sh(f.x[i]);
    return pk < drop ? (uint32_t)pk : drop;
  }
  __device__ uint32_t mask(uint32_t i) const {
    const uint32_t k = key(i);
    return k < drop ? 1u << owner_of(B, k) : 0u;
  }
  __device__ void emit(uint32_t i, uint32_t, uint32_t pos) const {
    const uint64_t xs = f.x[i], ys = f.y[i], L = f.len[i];
    const uint32_t s = f.strand[i] != 'f' ? 1u : 0u;
    const uint64_t pk = div10_sh(xs);
    out[pos] = make_uint4((uint32_t)pk, row_base + i, (uint32_t)ys,
                          (uint32_t)(L & 0xFFFFFFu) | s << 24 | (uint32_t)((ys >> 32) & 7u) << 25 |
                              (uint32_t)(xs - pk * 10) << 28);
  }
};

// own records (processing order, suffix from `base`) -> later slices whose
// lead-in they fall in; the row word carries the global processing index
struct GhostOp16 {
  const uint4 *R;
  uint64_t thr[MAXP];  // lead-in start bucket of every slice (~0: none)
  uint32_t P, me, poff, base;
  uint4 *out;          // records, or
  uint8_t *sout;       // the entries' X states (1 = ACTIVE), same order
  const uint32_t *xg;
  // (fast path) the suffix start on the device: the op runs over all m
  // entries, those before *dbase select nothing (base is then 0)
  const uint32_t *dbase = nullptr;
  __device__ uint32_t mask(uint32_t i) const {
    if (dbase && i < *dbase) return 0u;
    const uint64_t bk = nwr_xbucket(R[base + i]);
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
    uint4 r = R[k];
    r.y = poff + k;
    out[pos] = r;
  }
};

struct SelXOp16 {  // relevant halo entries the owner calls ACTIVE (fixed-halo X problem)
  const uint4 *gh;
  const uint8_t *owner_state;
  uint64_t rel;
  uint4 *out;
  __device__ uint32_t mask(uint32_t j) const {
    return nwr_xbucket(gh[j]) >= rel && owner_state[j] ? 1u : 0u;
  }
  __device__ void emit(uint32_t j, uint32_t, uint32_t pos) const { out[pos] = gh[j]; }
};

struct YOp12 {  // own Y records -> Y-range owners (+ their halos), processing order
  const uint3 *yrec;
  uint32_t nby, P, shift;
  int64_t lo[MAXP], hi[MAXP];  // halo-extended ranges
  const uint32_t *xg;          // with xout: the X results, sent after X in the same order
  uint3 *out;
  uint8_t *xout;
  __device__ uint32_t bin(uint32_t k) const { return nwy_bucket(yrec[k], nby) >> shift; }
  __device__ uint32_t mask(uint32_t k) const {
    const int64_t b = nwy_bucket(yrec[k], nby);
    uint32_t m = 0;
    for (uint32_t q = 0; q < P; ++q)
      if (b >= lo[q] && b < hi[q]) m |= 1u << q;
    return m;
  }
  __device__ void emit(uint32_t k, uint32_t, uint32_t pos) const {
    if (xout) xout[pos] = xg[k] != NONE ? 1 : 0;
    else out[pos] = yrec[k];
  }
};

struct ParOp12 {  // Y decisions of own X misses -> slice owners (other ranks)
  const uint3 *yr;
  const uint8_t *code;
  Bounds slices;
  const uint32_t *ywin;
  uint32_t me;
  ParRec *out;
  __device__ uint32_t mask(uint32_t r) const {
    const uint8_t c = code[r];
    if ((c & 3) || (c & YC_XHIT)) return 0u;
    const uint32_t q = owner_of(slices, yr[r].y);
    return q == me ? 0u : 1u << q;  // this rank's own slice: written in place
  }
  __device__ void emit(uint32_t r, uint32_t, uint32_t pos) const {
    out[pos] = ParRec{yr[r].y, ywin[r]};
  }
};

struct MemOpNw {  // {gid, global row, sort key} -> gid-range owners
  const uint32_t *gid;
  const uint2 *erk;     // {global row, sort key low 32} of own row k
  const uint32_t *ehi;  // sort key high 32
  Bounds B;
  uint32_t shift;
  bool narrow;
  void *out;
  __device__ uint32_t bin(uint32_t k) const { return gid[k] >> shift; }
  __device__ uint32_t mask(uint32_t k) const { return 1u << owner_of(B, gid[k]); }
  __device__ void emit(uint32_t k, uint32_t, uint32_t pos) const {
    const uint2 e = erk[k];
    if (narrow) reinterpret_cast<uint3 *>(out)[pos] = make_uint3(gid[k], e.x, e.y);
    else reinterpret_cast<uint4 *>(out)[pos] = make_uint4(gid[k], e.x, e.y, ehi[k]);
  }
};

// ---- small kernels ------------------------------------------------------------
// first k with R[k].x >= v (keys ascending)
__global__ void k_lower_bound16(const uint4 *R, uint32_t m, uint64_t v, uint32_t *out) {
  uint32_t lo = 0, hi = m;
  while (lo < hi) {
    const uint32_t mid = lo + (hi - lo) / 2;
    if (R[mid].x < v) lo = mid + 1;
    else hi = mid;
  }
  *out = lo;
}

// own X results -> global winner ids (NONE: X miss); the halo entries' local
// decisions (1 = in the X list)
__global__ void k_sh_x_own(const uint32_t *xpos, const uint8_t *state, const uint32_t *par,
                           const uint4 *halo, uint32_t G, uint32_t m, uint32_t poff,
                           uint32_t *xg, uint8_t *used) {
  GRID_STRIDE(k, G + m) {
    const bool hit = state[xpos[k]] == ST_HIT;
    if (k < G) {
      used[k] = hit ? 0 : 1;
      continue;
    }
    const uint32_t w = par[k];
    xg[k - G] = !hit ? NONE : w < G ? halo[w].y : poff + (w - G);
  }
}

__global__ void k_cmp_x16(const uint4 *gh, uint32_t G, uint64_t rel, const uint8_t *used,
                          const uint8_t *owner, uint32_t *mism) {
  for (uint32_t base = blockIdx.x * blockDim.x; base < G; base += gridDim.x * blockDim.x) {
    const uint32_t j = base + threadIdx.x;
    count_flag(j < G && nwr_xbucket(gh[j]) >= rel && used[j] != owner[j], mism);
  }
}

__global__ void k_sh_ycode(const uint3 *yr, uint32_t n, uint32_t nby, uint64_t lo, uint64_t hi,
                           uint8_t *code) {
  GRID_STRIDE(r, n) code[r] = y_code(nwy_bucket(yr[r], nby), lo, hi);
}

// the X-hit bytes (arrival order) -> code bits and the Y states' bitmask
__global__ void k_sh_xhit_bits(const uint8_t *xh, uint32_t n, uint8_t *code, uint32_t *bits) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r - lane < n;
       r += gridDim.x * blockDim.x) {
    const bool hit = r < n && xh[r] != 0;
    if (hit) code[r] |= YC_XHIT;
    const uint64_t b = __ballot(hit);
    if (lane == 0) bits[r >> 5] = (uint32_t)b;
    if (lane == 32 && r < n) bits[r >> 5] = (uint32_t)(b >> 32);
  }
}

// a fixed-halo Y problem's records (the selection ymap, in arrival order) and
// their X-hit bitmask
__global__ void k_sh_ysel(const uint3 *yr, const uint8_t *code, const uint32_t *ymap, uint32_t c,
                          uint3 *ysel, uint32_t *bits) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k - lane < c;
       k += gridDim.x * blockDim.x) {
    bool hit = false;
    if (k < c) {
      const uint32_t r = ymap[k];
      ysel[k] = yr[r];
      hit = (code[r] & YC_XHIT) != 0;
    }
    const uint64_t b = __ballot(hit);
    if (lane == 0) bits[k >> 5] = (uint32_t)b;
    if (lane == 32 && k < c) bits[k >> 5] = (uint32_t)(b >> 32);
  }
}

// (the Y winner of an X miss of this rank's own slice -- processing index in
// [poff, poff + m) -- goes straight into its parent word xpar)
__global__ void k_sh_y_results(const uint3 *yr, const uint8_t *code, const uint32_t *ymap,
                               uint32_t c, const uint32_t *par, uint8_t *ystate, uint32_t *ywin,
                               uint32_t poff, uint32_t m, uint32_t *xpar) {
  GRID_STRIDE(k, c) {
    const uint32_t r = ymap ? ymap[k] : k;
    const uint8_t cr = code[r];
    if (cr & YC_XHIT) {
      ystate[r] = 1;
      ywin[r] = NONE;
    } else {
      const uint32_t p = par[k];
      ystate[r] = p == k ? 1 : 0;
      const uint32_t w = yr[ymap ? ymap[p] : p].y;
      ywin[r] = w;
      if (!(cr & 3)) {
        const uint32_t own = yr[r].y - poff;
        if (own < m) xpar[own] = w;
      }
    }
  }
}

// ---- the driver -----------------------------------------------------------------
enum SlotNw : int {
  SN_HIST = SL_COUNT, SN_SROWS, SN_RIN, SN_RA, SN_RB, SN_YOWN, SN_STAT, SN_YSTAT, SN_SHALO, SN_HX,
  SN_HSEL, SN_SY, SN_YR, SN_YA, SN_YB, SN_XCNT, SN_XOFF, SN_XKEY, SN_XENT, SN_XPK, SN_XNBD,
  SN_XSTATE, SN_XPOS, SN_EREC, SN_PAR, SN_XGUSED, SN_YKEY, SN_YENT, SN_YPK, SN_YNBD, SN_YST,
  SN_XBITS, SN_PARL, SN_SMEM, SN_T0, SN_T1, SN_SGID, SN_MROW, SN_KEY, SN_TAG, SN_GOFF, SN_YSEL,
  SN_SXH, SN_CHIST, SN_COFF, SN_XCNT0, SN_COUNT
};
static_assert(SN_COUNT <= kPoolSlots, "rk_shard.hip kPoolSlots");

// Every record exchange of this driver has its own send slot, so a block that
// is handed over without a copy at world size 1 is never overwritten by a
// later exchange.
template <class T>
T *exchange_nw(Shard &S, const T *send, const PartPlan &pp, int recv_slot, uint32_t *nrecv,
               uint64_t *from = nullptr) {
  if (S.P == 1) {
    S.agree(RK_OK);  // the same collective sequence as with peers
    *nrecv = (uint32_t)pp.total;
    S.last_recv[0] = pp.total;
    if (from) from[0] = pp.total;
    return const_cast<T *>(send);
  }
  return S.exchange<T>(send, pp, recv_slot, nrecv, from);
}

// the largest slice's row count: at one rank the kept rows, else the global
// histogram's bins between each pair of slice bounds (the bounds lie on bins)
static uint64_t slice_max_rows(const std::vector<uint64_t> &gh, const Bounds &sk, uint32_t shift,
                               uint32_t P, uint64_t kept) {
  if (P == 1) return kept;
  const uint64_t unit = 1ull << shift;
  uint64_t most = 0;
  for (uint32_t q = 0; q < P; ++q) {
    const uint64_t b0 = (sk.b[q] + unit - 1) >> shift, b1 = (sk.b[q + 1] + unit - 1) >> shift;
    uint64_t c = 0;
    for (uint64_t b = b0; b < b1 && b < gh.size(); ++b) c += gh[b];
    most = c > most ? c : most;
  }
  return most;
}

int classify_sharded_nw(Shard &S, const rk_frags_soa *in, const rk_params &p, uint32_t P,
                        uint32_t me, uint64_t N, uint64_t row_base, int32_t lead_in,
                        rk_shard_result *out, std::chrono::steady_clock::time_point t0) {
  rk_ctx *ctx = S.ctx;
  rk_shard_stats &ss = ctx->shard_stats;
  const uint64_t H = lead_in < 0 ? 2 : (uint64_t)lead_in;
  const uint64_t len_x = p.len_x_hdr + 1, len_y = p.len_y_hdr + 1;  // FragmentsDatabase.cpp:62,65
  const uint64_t vsize = 1 + len_x / 10;                             // :84
  const uint64_t max_x = len_x / 100, max_y = len_y / 100;           // SequenceOcupationList.cpp:4
  const uint32_t nbx = (uint32_t)(max_x + 1), nby = (uint32_t)(max_y + 1);
  const uint32_t drop = (uint32_t)(vsize - 1);
  const uint32_t nl = (uint32_t)in->n;
  hipStream_t st = S.st, st2 = S.st2;

  // ---- 1: keys, checks and the slice histogram at the source; every rank
  // agrees on the record layout (or all run the generic driver)
  Frags f{in->x_start, in->y_start, in->length, in->strand, nl};
  const uint32_t shift = bin_shift(drop);
  uint32_t *hist = S.take<uint32_t>(SN_HIST, 3 * 4096);  // later the sorts' digit histograms
  S.zero(hist, NBINS * 4);
  S.zero(S.ctrl + 25, 4);
  // World size 1 (rows numbered from 0): the rows are read once, as on one
  // device -- k_nw_order_hist takes the checks, the kept count and the order
  // and Y digit histograms (into step 3's ahist / yhist) in the place of
  // k_sh_rows, and when no row is dropped the order sort's first pass reads
  // the rows themselves (no row records, no record histogram, no Y-record
  // histogram).  RK_SH_ONE=0: the record route at world size 1 too.
  static const bool one_on = [] {
    const char *e = getenv("RK_SH_ONE");
    return !(e && e[0] == '0');
  }();
  static const bool y_early_env = [] {
    const char *e = getenv("RK_SH_YEARLY");
    return e && e[0] == '1';
  }();
  const bool one = one_on && P == 1 && row_base == 0;
  const NwDigits ad = nw_plan(bit_length(vsize - 1));
  const NwDigits yd = nw_plan(bit_length(2ull * nby - 1), 9);
  const NwOrderPlan op1 = one ? nw_order_split_range(nl, 0, drop) : NwOrderPlan{};
  if (one) {
    S.zero(hist, 3 * 4096 * 4);
    S.zero(S.ctrl + 32, 16 * 4);
    if (nl)
      nw_order_hist(*in, vsize, max_x, max_y, nby, op1.nseg ? op1.coarse : ad, yd, hist,
                    hist + 4096, S.ctrl + 32, st);
  } else if (nl) {
    // more blocks when there is no slice histogram to flush (one rank)
    kt_begin(st, KID_SH_ROWKEYS);
    k_sh_rows<<<grid_for(nl, 256, P > 1 ? 1024 : 4096), 256, 0, st>>>(
        ShRowsArgs{f, vsize, max_x, max_y, shift, P > 1 ? hist : nullptr, S.ctrl});
    kt_end(st, KID_SH_ROWKEYS, 25.0 * nl);
    S.launched("k_sh_rows");
  }
  // the error bits (ctrl[0]), the pack flags (ctrl[20..21]), the kept count
  // (ctrl[25]) and the slice histogram in one readback, and the first two with
  // the histogram in one all-gather
  std::vector<uint32_t> flags(41);
  const uint32_t MW = 2 + (P > 1 ? NBINS : 0);  // message words
  std::vector<uint32_t> msg(MW);
  S.hip(hipMemcpyAsync(flags.data(), S.ctrl, (one ? 41 : 26) * 4, hipMemcpyDeviceToHost, st),
        "d2h");
  if (P > 1) S.hip(hipMemcpyAsync(msg.data() + 2, hist, NBINS * 4, hipMemcpyDeviceToHost, st), "d2h");
  ++S.n_syncs;
  S.hip(hipStreamSynchronize(st), "d2h sync");
  if (one) {  // k_nw_order_hist's words: [0] error bits, [1] kept, [3] no pack, [4] longest
    flags[0] = flags[32];
    flags[25] = flags[33];
    flags[20] = flags[35];
    flags[21] = flags[36];
  }
  msg[0] = flags[0];
  msg[1] = flags[20] | (flags[21] << 1);
  std::vector<uint32_t> allm((size_t)P * MW);
  S.allgather(msg.data(), allm.data(), MW * 4);
  uint32_t anyerr = 0, nopack = 0, maxlen = 0;
  std::vector<uint64_t> gh(NBINS, 0);
  for (uint32_t q = 0; q < P; ++q) {
    const uint32_t *mq = allm.data() + (size_t)q * MW;
    anyerr |= mq[0];
    nopack |= mq[1] & 1u;
    maxlen = (mq[1] >> 1) > maxlen ? (mq[1] >> 1) : maxlen;
    if (P > 1)
      for (uint32_t b = 0; b < NBINS; ++b) gh[b] += mq[2 + b];
  }
  S.check(err_status(ctx, anyerr & ~(uint32_t)ERRB_WIDE_LENGTH));
  if (nopack) return RK_SHARD_FALLBACK;
  const uint32_t *mine = msg.data() + 2;  // this rank's own bins (P > 1)
  const Bounds slice_keys = split_bounds(gh, shift, drop, P);
  // the one-sweep passes' status words carry a 30-bit count (SW_VAL,
  // rk_onesweep.h), as the single-device record pipeline's bound n < 2^30
  // (record_eligible): a slice of 2^30 or more rows takes the generic driver.
  // Every rank sees the same global histogram (the kept count at one rank), so
  // the decision is agreed
  if (slice_max_rows(gh, slice_keys, shift, P, flags[25]) >= (1ull << 30)) return RK_SHARD_FALLBACK;

  // ---- 2: rows -> slice owners as 16-B records (arrival order = file order);
  // the bounds lie on histogram bins (or at the end), so this rank's count per
  // owner is a sum of its own bins -- the plan needs no readback
  RowOp16 rop{f, slice_keys, drop, (uint32_t)row_base, nullptr};
  PartPlan pp;
  rop.out = S.take<uint4>(SN_SROWS, (size_t)nl + 1);  // room for every row (see plan_counts)
  // (fast: step 3 reads the rows, rop.out is the fine kernel's scratch)
  const bool fast = one && flags[25] == nl;
  if (fast) {
    S.identity_plan(nl, pp);
  } else if (P == 1 && flags[25] == nl) {  // one rank, no row dropped: the records in row order
    S.emit_identity(rop, nl, pp);
  } else {
    uint64_t cnt[MAXP] = {};
    if (P == 1) {
      cnt[0] = flags[25];
    } else {
      const uint64_t unit = 1ull << shift;
      for (uint32_t q = 0; q < P; ++q) {
        const uint64_t b0 = (slice_keys.b[q] + unit - 1) >> shift,
                       b1 = (slice_keys.b[q + 1] + unit - 1) >> shift;
        for (uint64_t b = b0; b < b1 && b < NBINS; ++b) cnt[q] += mine[b];
      }
    }
    S.plan_counts(rop, nl, pp, cnt);
    S.emit(rop, pp);
  }
  uint32_t m = 0;
  const uint4 *rin = exchange_nw<uint4>(S, rop.out, pp, SN_RIN, &m);
  // every rank's slice size: known from the exchange's count all-gather
  std::vector<uint64_t> mall(S.last_recv, S.last_recv + P);
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

  // ---- 3: the slice's processing order (one-sweep passes), its Y records
  uint32_t *ahist = S.take<uint32_t>(SN_HIST, 3 * 4096);  // order / Y / member digit histograms
  uint32_t *yhist = ahist + 4096, *ehist = ahist + 2 * 4096;
  if (!fast) S.zero(ahist, 3 * 4096 * 4);  // (fast: the order and Y ones are in, ehist zero)
  else if (y_early_env) S.zero(yhist, 4096 * 4);  // (that schedule counts the Y keys itself)
  const size_t sw = nw_status_words(m + 1);
  uint32_t *astat = S.take<uint32_t>(SN_STAT, sw);
  uint4 *Ra = S.take<uint4>(SN_RA, m + 1), *Rb = S.take<uint4>(SN_RB, m + 1);
  uint4 *yown = S.take<uint4>(SN_YOWN, (size_t)m * 3 / 4 + 2);  // 12-B records
  // the two-stage order sort (coarse passes, per-segment LDS sort) when the
  // slice's key density suits it: the slice holds m rows over its own key
  // span, and the coarse digits are slice-relative, (key - kbase) >> F, so the
  // segment table covers that span only
  const NwOrderPlan op = fast ? op1 : nw_order_split_range(m, slice_keys.b[me], slice_keys.b[me + 1]);
  ss.order_split = op.nseg ? 1u : 0u;
  // the X axis' chunk width (step 6) from the slice's own rows: the fine
  // kernel then counts the slice's X-chunk entries as it writes the order, and
  // step 6 adds the halo's (when its width comes out the same)
  const uint64_t span = (slice_keys.b[me + 1] - slice_keys.b[me]) / 10 + 2;
  NwChunkCounts own_cc{};
  own_cc.W = nw_chunk_width(m, (uint32_t)(span < nbx ? span : nbx));
  while ((1u << own_cc.lgW) < own_cc.W) ++own_cc.lgW;
  own_cc.nch = nw_chunks(nbx, own_cc.W);
  bool own_counts = false;
  if (m && op.nseg) {
    uint32_t *chist = S.take<uint32_t>(SN_CHIST, nw_seg_words(m));
    uint32_t *coff = S.take<uint32_t>(SN_COFF, nw_seg_words(m));
    own_cc.cnts = S.take<uint32_t>(SN_XCNT0, (size_t)3 * own_cc.nch + 2);
    if (fast) {  // the rows themselves (op == op1, whose histogram is in)
      nw_order_sort_split_coarse(*in, op, ahist, astat, Ra, Rb, chist,
                                 ZeroRegion{own_cc.cnts, ((size_t)3 * own_cc.nch + 1) * 4}, vsize,
                                 st, nullptr);
      nw_order_sort_split_fine(nl, m, nby, op, Ra, Rb, yown, rop.out, chist, coff,
                               S.scan_scratch(SL_PSCAN, (size_t)op.nseg + 1), &own_cc, st);
    } else {
      nw_rec_hist(rin, 16, m, op.kbase, op.coarse, ahist, st);
      // rin is read by the first coarse pass only: the fine kernel's scratch
      nw_order_sort_recs_split(rin, m, nby, poff, op, ahist, astat, Ra, Rb, yown,
                               const_cast<uint4 *>(rin), chist, coff,
                               S.scan_scratch(SL_PSCAN, (size_t)op.nseg + 1), &own_cc, st);
    }
    own_counts = true;
    S.launched("order sort");
  } else if (m) {
    if (fast) {
      nw_order_sort(*in, vsize, nby, ad, ahist, astat, Ra, Rb, yown, st);
    } else {
      nw_rec_hist(rin, 16, m, 0, ad, ahist, st);
      nw_order_sort_recs(rin, m, nby, poff, ad, ahist, astat, Ra, Rb, yown, st);
    }
    S.launched("order sort");
  }
  ss.ms_ingress = ms_since(t0);

  // ---- 4: Y records -> Y-range owners (+ halos); their sort starts on the
  // second stream while X resolves
  const auto ty = std::chrono::steady_clock::now();
  YOp12 yop{};
  yop.yrec = reinterpret_cast<const uint3 *>(yown);
  yop.nby = nby;
  yop.P = P;
  yop.shift = bin_shift(nby);
  const Bounds yb = split_bounds(P > 1 ? global_hist(S, yop, m) : std::vector<uint64_t>(NBINS, 0),
                                 yop.shift, nby, P);
  for (uint32_t q = 0; q < MAXP; ++q) {
    yop.lo[q] = q < P ? (int64_t)yb.b[q] - 1 - (int64_t)H : 0;
    yop.hi[q] = q < P ? (int64_t)yb.b[q + 1] + 1 + (int64_t)H : 0;
  }
  PartPlan ypp;
  if (P == 1) {  // one Y range, halos included: every record stays, in order
    S.identity_plan(m, ypp);
  } else {
    ypp.mcache = S.take<uint32_t>(SL_YMASK, m + 1);  // the X-hit bytes follow the same masks
    S.plan(yop, m, ypp);
  }
  // every own record stays here, once: the send layout is the records themselves
  const bool y_self = ypp.total == m && ypp.cnt[me] == m;
  if (!y_self) {
    yop.out = S.take<uint3>(SN_SY, ypp.total + 1);
    S.emit(yop, ypp);
  }
  uint32_t ny = 0;
  const uint3 *yr = exchange_nw<uint3>(S, y_self ? yop.yrec : yop.out, ypp, SN_YR, &ny);
  ss.y_entries = ny;
  // the Y ranges (+ halos) received: the same 30-bit bound on every rank's
  // sort (every rank knows every rank's count from the exchange)
  S.check_recv_below(1u << 30, RK_E_TOO_MANY, "a Y range of 2^30 or more records");
  const uint64_t ylo = yb.b[me], yhi = yb.b[me + 1];
  uint8_t *ycode = S.take<uint8_t>(SL_YCODE, ny + 1);
  uint8_t *ystate = S.take<uint8_t>(SL_YSTATE, ny + 1);
  uint32_t *ywin = S.take<uint32_t>(SL_YWIN, ny + 1);
  uint8_t *yused = S.take<uint8_t>(SL_YUSED, ny + 1);
  uint32_t *par_l = S.take<uint32_t>(SN_PARL, ny + 1);
  uint32_t *ystat = S.take<uint32_t>(SN_YSTAT, nw_status_words(ny + 1));
  uint4 *yA = S.take<uint4>(SN_YA, (size_t)ny * 3 / 4 + 2), *yB = S.take<uint4>(SN_YB, (size_t)ny * 3 / 4 + 2);
  Csr cy{};
  cy.key = S.take<uint32_t>(SN_YKEY, ny + 1);
  cy.ent = S.take<uint32_t>(SN_YENT, ny + 1);
  cy.pk = S.take<uint2>(SN_YPK, ny + 1);
  cy.nbd = S.take<uint8_t>(SN_YNBD, ny + 1);
  cy.state = S.take<uint8_t>(SN_YST, ny + 1);
  uint32_t *ybits = S.take<uint32_t>(SN_XBITS, ny / 32 + 2);
  // the Y sort's passes read the received records (first pass: arrival
  // numbering) and ping-pong through yA / yB; the received array stays whole
  // for the winners' global ids
  auto y_sort = [&](const uint3 *src, uint32_t n, const uint32_t *bits, hipStream_t s,
                    bool head, bool tail) {
    if (!n) return;
    if (head) {
      nw_rec_hist(src, 12, n, 0, yd, yhist, s);
      nw_y_sort_head(yB, yA, n, yd, yhist, ystat, s, true, reinterpret_cast<const uint4 *>(src));
    }
    if (tail)
      nw_y_sort_tail(yB, yA, n, yd, yhist, ystat, cy, nby, max_y, bits, s, true,
                     reinterpret_cast<const uint4 *>(src));
  };
  // The Y sort runs after X, as on one device (nw_y_sort_after_x): its first
  // pass carries the X-hit bit in the records, so no pass shares the device
  // with the X axis and the last one needs no lookup.  Beside X on the second
  // stream: the Y codes and the Y key histogram.  RK_SH_YEARLY=1: the round-3
  // schedule (the head passes beside X, the tail looking the bits up)
  static const bool y_early = [] {
    const char *e = getenv("RK_SH_YEARLY");
    return e && e[0] == '1';
  }();
  hipStream_t sy = st2;
  S.hip(hipEventRecord(ctx->fork, st), "fork");
  S.hip(hipStreamWaitEvent(st2, ctx->fork, 0), "fork wait");
  if (ny) {
    k_sh_ycode<<<grid_for(ny, 256), 256, 0, sy>>>(yr, ny, nby, ylo, yhi, ycode);
    S.launched("k_sh_ycode");
  }
  if (y_early) {
    y_sort(yr, ny, nullptr, sy, true, false);
    S.launched("Y sort head");
  } else if (ny && !fast) {  // (fast: counted by k_nw_order_hist over the same rows)
    nw_rec_hist(yr, 12, ny, 0, yd, yhist, sy);
  }
  S.hip(hipEventRecord(ctx->join, st2), "join");
  ss.ms_y = ms_since(ty);

  // ---- 5: X lead-in halo from earlier slices (16-B records, global ids)
  const auto tx = std::chrono::steady_clock::now();
  GhostOp16 gop{};
  gop.R = Ra;
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
      const uint64_t reach = thr_min * 100;  // centre >= reach is needed
      const uint64_t half = maxlen / 2;
      const uint64_t key0 = reach > half + 10 ? (reach - half) / 10 - 1 : 0;
      k_lower_bound16<<<1, 1, 0, st>>>(Ra, m, key0, S.ctrl + 22);
      S.launched("k_lower_bound16");
      k0 = S.read1(S.ctrl + 22);
    }
    gop.base = k0;
  }
  const uint32_t nsuf = m - gop.base;
  const uint64_t bmin_me = slice_keys.b[me] / 10;
  const uint64_t rel_x = bmin_me >= 1 ? bmin_me - 1 : 0;  // relevant: probed by own queries
  if (nsuf) S.plan(gop, nsuf, pp);
  else S.zero_plan(0, pp);  // no row can reach a later slice: nothing to send
  gop.out = S.take<uint4>(SN_SHALO, pp.total + 1);
  if (nsuf) S.emit(gop, pp);
  uint32_t G = 0;
  const uint4 *hx = exchange_nw<uint4>(S, gop.out, pp, SN_HX, &G);
  ss.x_ghosts = G;

  // ---- 6: X axis over [halo ; own] (the X-chunk kernel, no sort)
  uint32_t *xg = S.take<uint32_t>(SL_XG, m + 1);
  uint8_t *xused = S.take<uint8_t>(SN_XGUSED, G + 1);
  uint32_t Gfin = 0;            // the halo of the last X solve
  const uint4 *hfin = nullptr;  // (its records: member records sit behind it)
  auto solve_x = [&](const uint4 *halo, uint32_t Gc) {
    const uint32_t mx = Gc + m;
    Gfin = Gc;
    hfin = halo;
    if (!mx) return;
    NwChunkCounts cc{};
    cc.W = nw_chunk_width(mx, (uint32_t)(span < nbx ? span : nbx));
    while ((1u << cc.lgW) < cc.W) ++cc.lgW;
    cc.nch = nw_chunks(nbx, cc.W);
    cc.cnts = S.take<uint32_t>(SN_XCNT, (size_t)3 * cc.nch + 2);
    uint32_t *xoff = S.take<uint32_t>(SN_XOFF, (size_t)3 * cc.nch + 2);
    if (own_counts && cc.W == own_cc.W) {
      (void)hipMemcpyAsync(cc.cnts, own_cc.cnts, ((size_t)3 * cc.nch + 1) * 4,
                           hipMemcpyDeviceToDevice, st);
      nw_x_count_add(halo, Gc, cc, st);
    } else {
      nw_x_count(Ra, mx, cc, st, halo, Gc);
    }
    exclusive_scan_u32(cc.cnts, xoff, (size_t)3 * cc.nch + 1,
                       S.scan_scratch(SL_PSCAN, (size_t)3 * cc.nch + 1), st);
    Csr cx{};
    cx.key = S.take<uint32_t>(SN_XKEY, mx + 1);
    cx.ent = S.take<uint32_t>(SN_XENT, mx + 1);
    cx.pk = S.take<uint2>(SN_XPK, mx + 1);
    cx.nbd = S.take<uint8_t>(SN_XNBD, mx + 1);
    cx.state = S.take<uint8_t>(SN_XSTATE, mx + 1);
    uint32_t *xpos = S.take<uint32_t>(SN_XPOS, mx + 1);
    uint4 *erec = S.take<uint4>(SN_EREC, (size_t)mx * 3 / 4 + 2);
    uint32_t *par = S.take<uint32_t>(SN_PAR, mx + 1);
    nw_x_chunks(Ra, mx, nbx, max_x, maxlen, xoff, cx, xpos, erec, S.ctrl, cc.W, st, halo, Gc);
    S.launched("X chunks");
    Axis ax{cx.key, cx.ent, nullptr, nullptr, cx.state, nullptr, par, cx.pk, cx.nbd,
            S.take<uint32_t>(SL_RLEN, mx), S.take<uint32_t>(SL_RBEG, mx), mx, max_x,
            p.len_ratio, p.pos_ratio};
    SweepScratch sc{S.take<uint32_t>(SL_RUNS, runs_scratch_words(mx)),
                    S.take<uint8_t>(SL_WPEND, mx / 64 + 1), S.take<uint8_t>(SL_RPEND, mx),
                    S.ctrl + 64, S.ctrl + 4};
    uint32_t sweeps = 0;
    S.check(resolve_axis(ctx, ax, sc, true, &sweeps));
    S.max_sweeps[0] = sweeps > S.max_sweeps[0] ? sweeps : S.max_sweeps[0];
    kt_begin(st, KID_SH_XOWN);
    k_sh_x_own<<<grid_for(mx, 256), 256, 0, st>>>(xpos, cx.state, par, halo, Gc, m, poff, xg,
                                                  xused);
    kt_end(st, KID_SH_XOWN, 0.0);
    S.launched("k_sh_x_own");
  };
  S.zero(S.ctrl + 6, 4);
  solve_x(hx, G);
  // verify the relevant halo against its owners' decisions (one rank: there
  // are no later slices, so no halo was sent or received)
  for (; P > 1;) {
    ++ss.x_rounds;
    if (ss.x_rounds > P + 2) {
      ctx->err = "X halo verification did not converge";
      throw RK_E_INTERNAL;
    }
    GhostOp16 sop = gop;
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
      k_cmp_x16<<<grid_for(G, 256, 1024), 256, 0, st>>>(hx, G, rel_x, xused, xown, S.ctrl + 2);
      S.launched("k_cmp_x16");
    }
    const uint32_t mism = S.read1(S.ctrl + 2);
    if (S.sum_any(mism) == 0) break;
    if (mism) {  // re-resolve with the halo fixed to the owners' states
      ++ss.x_reruns;
      SelXOp16 sel{hx, xown, rel_x, nullptr};
      PartPlan sp;
      Shard S1 = S;
      S1.P = 1;
      S1.me = 0;
      S1.plan(sel, G, sp);
      sel.out = S.take<uint4>(SN_HSEL, sp.total + 1);
      S1.emit(sel, sp);
      solve_x(sel.out, (uint32_t)sp.total);
      S.hip(hipMemcpyAsync(xused, xown, G, hipMemcpyDeviceToDevice, st), "xused copy");
    }
  }
  ss.ms_x = ms_since(tx);

  // ---- 7: the X-hit bytes follow the Y records (same plan, same order); the
  // Y sort's last pass writes the CSR with the states
  const auto ty2 = std::chrono::steady_clock::now();
  {
    YOp12 xop = yop;
    xop.xg = xg;
    PartPlan xpp;
    xop.xout = S.take<uint8_t>(SN_SXH, (size_t)ypp.total + 1);
    if (P == 1) {
      S.emit_identity(xop, m, xpp);
    } else {
      xpp.mcache = ypp.mcache;
      xpp.mread = true;
      S.plan_same(xop, m, xpp, ypp);  // the Y records' own selection: counts known
      S.emit(xop, xpp);
    }
    uint32_t n2 = 0;
    const uint8_t *xh = exchange_nw<uint8_t>(S, xop.xout, xpp, SL_YXH, &n2);
    if (n2 != ny) {
      ctx->err = "Y X-hit count mismatch";
      throw RK_E_INTERNAL;
    }
    S.hip(hipStreamWaitEvent(st, ctx->join, 0), "join wait");
    if (ny) {
      kt_begin(st, KID_SH_MERGE);
      k_sh_xhit_bits<<<grid_for(ny, 256), 256, 0, st>>>(xh, ny, ycode, ybits);
      kt_end(st, KID_SH_MERGE, 0.0);
      S.launched("k_sh_xhit_bits");
    }
  }
  auto sweep_y = [&](uint32_t n) {
    if (!n) return;
    Axis ay{cy.key, cy.ent, nullptr, nullptr, cy.state, nullptr, par_l, cy.pk, cy.nbd,
            S.take<uint32_t>(SL_RLEN, n), S.take<uint32_t>(SL_RBEG, n), n, max_y, p.len_ratio,
            p.pos_ratio};
    ay.par_dev = true;
    SweepScratch sc{S.take<uint32_t>(SL_RUNS, runs_scratch_words(n)),
                    S.take<uint8_t>(SL_WPEND, n / 64 + 1), S.take<uint8_t>(SL_RPEND, n),
                    S.ctrl + 64, S.ctrl + 4};
    uint32_t sweeps = 0;
    S.check(resolve_axis(ctx, ay, sc, true, &sweeps));
    S.max_sweeps[1] = sweeps > S.max_sweeps[1] ? sweeps : S.max_sweeps[1];
  };
  auto y_results = [&](const uint32_t *ymap, uint32_t c) {
    if (!c) return;
    kt_begin(st, KID_SH_YRES);
    k_sh_y_results<<<grid_for(c, 256), 256, 0, st>>>(yr, ycode, ymap, c, par_l, ystate, ywin,
                                                      poff, m, xg);
    kt_end(st, KID_SH_YRES, 0.0);
    S.launched("k_sh_y_results");
  };
  if (y_early) {
    y_sort(yr, ny, ybits, st, false, true);
  } else if (ny) {
    nw_y_sort_after_x(yB, yA, ny, yd, yhist, ystat, cy, nby, max_y, ybits, st,
                      reinterpret_cast<const uint4 *>(yr));
  }
  S.launched("Y sort");
  sweep_y(ny);
  y_results(nullptr, ny);
  // a fixed-halo re-resolution: the selected records sorted again on stream 1
  auto solve_y = [&](const uint32_t *ymap, uint32_t c) {
    if (!c) return;
    uint3 *ysel = S.take<uint3>(SN_YSEL, c + 1);
    k_sh_ysel<<<grid_for(c, 256), 256, 0, st>>>(yr, ycode, ymap, c, ysel, ybits);
    S.launched("k_sh_ysel");
    S.zero(yhist, 4096 * 4);
    y_sort(ysel, c, ybits, st, true, true);
    sweep_y(c);
    y_results(ymap, c);
  };
  const RelOp relop{ycode, ylo ? owner_of_host(yb, ylo - 1) : 0u,
                    yhi < nby ? owner_of_host(yb, yhi) : 0u, nullptr};
  verify_y_halo(S, relop, ycode, ystate, yused, yb, ny, solve_y);
  ss.ms_y += ms_since(ty2);

  // ---- 8: parents back to the slice owners; roots; gids
  const auto tr = std::chrono::steady_clock::now();
  ParOp12 pop{yr, ycode, slices, ywin, me, nullptr};
  if (P == 1) S.zero_plan(ny, pp);  // every parent is local (written by k_sh_y_results)
  else S.plan(pop, ny, pp);
  pop.out = S.take<ParRec>(SL_SEND, pp.total + 1);
  if (P > 1) S.emit(pop, pp);
  uint32_t npar = 0;
  const ParRec *prr = S.exchange<ParRec>(pop.out, pp, SL_PR, &npar);
  uint64_t Gtot = 0;
  const uint32_t *gid_own = resolve_roots(S, xg, prr, npar, m, poff, slices, &Gtot);
  ss.ms_roots = ms_since(tr);

  // ---- 9: members -> gid-range owners; exact in-group order; emit
  const auto tm = std::chrono::steady_clock::now();
  bool narrow = true;  // every sort key fits 32 bits (the X-chunk kernel's flag)
  const uint32_t mx = Gfin + m;
  const uint2 *erk = reinterpret_cast<const uint2 *>(S.take<uint4>(SN_EREC, (size_t)mx * 3 / 4 + 2));
  MemOpNw mop{gid_own, erk + Gfin, reinterpret_cast<const uint32_t *>(erk + mx) + Gfin,
              {}, bin_shift(Gtot), true, nullptr};
  (void)hfin;
  // the gid histogram and the wide-key flags in one readback and one all-gather
  std::vector<uint32_t> wide;
  std::vector<uint64_t> ghist(NBINS, 0);
  if (P > 1) ghist = global_hist(S, mop, m, {S.ctrl + 6}, &wide);
  else wide = S.gather1<uint32_t>(S.read1(S.ctrl + 6));
  for (uint32_t w : wide) narrow &= w == 0;
  mop.narrow = narrow;
  const Bounds gb = split_bounds(ghist, mop.shift, Gtot, P);
  mop.B = gb;
  const size_t esz = narrow ? 12 : 16;
  // one rank: every member stays here and the X chunk's member arrays are
  // exactly the own rows (no halo): the member sort reads them in place, as on
  // one device (no plan needed)
  const bool m_self = P == 1 && Gfin == 0;
  if (!m_self) S.plan(mop, m, pp);
  if (!m_self) {
    mop.out = S.take<uint8_t>(SN_SMEM, (pp.total + 1) * esz);
    S.emit(mop, pp);
  }
  uint32_t mr = 0;
  const void *mem = nullptr;
  if (m_self) {
    S.agree(RK_OK);  // the exchange's agreement point
    mr = m;
  } else {
    mem = narrow ? (const void *)exchange_nw<uint3>(S, (const uint3 *)mop.out, pp, SL_MEM, &mr)
                 : (const void *)exchange_nw<uint4>(S, (const uint4 *)mop.out, pp, SL_MEM, &mr);
  }
  // the gid range's members: the same 30-bit bound on the member sort
  if (m_self) S.last_recv[0] = mr;
  S.check_recv_below(1u << 30, RK_E_TOO_MANY, "a gid range of 2^30 or more members");
  const uint32_t g0 = (uint32_t)gb.b[me], Gl = (uint32_t)(gb.b[me + 1] - gb.b[me]);
  uint32_t *ogid = S.take<uint32_t>(SL_OGID, mr + 1);
  uint8_t *orep = S.take<uint8_t>(SL_OREP, mr + 1);
  uint32_t *oord = S.take<uint32_t>(SL_OORD, mr + 1);
  if (mr) {
    const NwDigits ed = nw_plan(bit_length(Gl ? Gl - 1 : 0), narrow ? 9 : 8);
    uint32_t *sgid = S.take<uint32_t>(SN_SGID, mr + 1);
    uint32_t *mrow = S.take<uint32_t>(SN_MROW, mr + 1);
    uint64_t *reckey = S.take<uint64_t>(SN_KEY, mr + 1);
    uint32_t *tag = S.take<uint32_t>(SN_TAG, mr + 1);
    uint32_t *otag = S.take<uint32_t>(SL_OTAG, mr + 1);
    uint32_t *goffs = S.take<uint32_t>(SN_GOFF, (size_t)Gl + 2);
    uint4 *t0 = S.take<uint4>(SN_T0, mr + 1), *t1 = S.take<uint4>(SN_T1, mr + 1);
    uint32_t *mstat = S.take<uint32_t>(SN_STAT, nw_status_words(mr + 1));
    void *gsort = S.take<uint8_t>(SL_GSORT, groupsort_scratch_bytes(mr));
    S.zero(ehist, 4096 * 4);
    if (m_self) {
      nw_rec_hist(gid_own, 4, mr, g0, ed, ehist, st);
      nw_member_sort(reinterpret_cast<const uint4 *>(erk), gid_own, t0, t1, mr, ed, ehist, mstat,
                     sgid, reckey, tag, mrow, narrow, st);
    } else {
      nw_rec_hist(mem, (int)esz, mr, g0, ed, ehist, st);
      nw_member_sort_recv(mem, narrow, mr, g0, ed, ehist, mstat, t0, t1, sgid, reckey, tag, mrow,
                          st);
    }
    group_offsets(sgid, mr, Gl, goffs, st);
    // the group-sort tiers on both streams, as in the single-device path
    S.check(sort_groups_exact(sgid, goffs, Gl, mr, reckey, tag, otag, gsort,
                              S.scan_scratch(SL_SCAN, mr + Gl + 2), ctx->host + 128, narrow, st,
                              st2 != st ? st2 : nullptr, ctx->fork, ctx->join));
    emit_result(otag, sgid, goffs, mrow, mr, ogid, orep, oord, st);
    if (g0) k_add_u32<<<grid_for(mr, 256), 256, 0, st>>>(ogid, mr, g0);
    S.launched("member order");
  }
  // every rank's share of the output: its received members
  std::vector<uint64_t> oall(S.last_recv, S.last_recv + P);
  uint64_t ooff = 0, otot = 0;
  for (uint32_t q = 0; q < P; ++q) otot += oall[q], ooff += q < me ? oall[q] : 0;
  S.hip(hipStreamSynchronize(st), "final sync");
  S.agree_errors();
  ss.ms_members = ms_since(tm);

  out->out_order = oord;
  out->gid = ogid;
  out->repval = orep;
  out->n_out = mr;
  out->out_offset = ooff;
  out->n_out_total = otot;
  out->n_groups = Gtot;
  (void)N;
  (void)M;
  return RK_OK;
}
