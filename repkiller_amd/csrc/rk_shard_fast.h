// rk_shard_fast.h -- the record driver with its exchange sizes agreed up
// front (part of rk_shard.hip's translation unit, after rk_shard_nw.h).
//
// The careful record driver (rk_shard_nw.h) sizes every all-to-all by a
// device count read back to the host and all-gathered right before it, and
// reads back the occupancy sweeps' pending counts and every pointer-jumping
// round: ~20 host waits and ~21-24 all-gathers per call at 2-4 ranks.  Over
// RCCL an all-gather is itself a wait, so at 8 ranks (~1.2 ms of device work
// per rank at cfg3) the round trips would decide the time.  This driver makes
// the same exchanges, in the same order, with the same kernels, but learns
// their sizes from a few messages assembled ON THE DEVICE (histograms, count
// matrices, flags written by the kernels that produce them) and gathered in
// one collective with one wait each:
//   GA  every rank's row count, error / pack bits, longest length, the
//       xStart/10 histogram and the Y-centre bucket histogram of its rows
//       -> the slice bounds AND the Y-range bounds (the same multiset of
//       rows, so the same bounds the careful driver finds after its Y sort);
//   GB  one pass over the source rows counts, per (slice, destination), the
//       Y records (halos included), the X lead-in records and the rows in
//       every Y range's first / last bucket -> the sizes of the row, Y, halo,
//       X-state, X-hit and Y-state exchanges;
//   GC  after both axes: the verification mismatches, whether a queued sweep
//       left an axis open, the wide-key flag, and per slice the parents this
//       Y owner sends, its roots and its cross-slice links -> the parent
//       exchange, the gid offsets and the first request round;
//   GD  after each request round: the next round's request counts, the
//       pointer-jumping flag and the (speculative) gid histogram -> the
//       member exchange (its bounds lie on the histogram's bins);
//   GE  the error bits and the deferred heap segments.
// Five gathers and five waits per call when one request round settles the
// roots (two ranks), one more per further round.  A halo disagreement or an
// axis still open after its queued sweeps (the careful driver's rare
// re-resolution) makes every rank repeat the call on the careful driver.
//
// Receive buffers: a stage whose gathered counts (and so every size it takes)
// equal those of the last call that completed on this path runs without
// agreement points -- no rank can need a larger buffer; otherwise its
// exchanges go through Shard::exchange, whose count gather agrees on any
// growth before data moves (the first call, or a new input).
#pragma once

constexpr int RK_SHARD_RETRY = 1 << 21;  // not a status: repeat on the careful driver

// fast-path control words S.ctrl[FW + i]: [0] retry bits, [1] X halo
// mismatches, [2] Y halo mismatches, [3] X axis left open, [4] Y axis left
// open, [5] deferred heap segments
constexpr uint32_t FW = 200;
enum : uint32_t { RETRY_EXPECT = 1u, RETRY_PARENT = 2u };

// message layouts (byte offsets into the payload)
constexpr size_t GA_HOST = 0;     // u64 rows of this rank, u64 fingerprints[8]
constexpr size_t GA_WORDS = 128;  // u32[32]: [0] error bits, [20] no pack, [21] longest, [25] kept
constexpr size_t GA_XH = 256, GA_YH = GA_XH + NBINS * 4, GA_END = GA_YH + NBINS * 4;
static_assert(GA_END <= GMAX, "GA message");
constexpr size_t GW_END = 64;  // GC / GD / GE: u32[16] head = ctrl[0..8) + ctrl[FW..FW+8)
static_assert(GW_END + (2 * MAXP + MAXP * MAXP + 2) * 4 <= GMAX, "GC message");
static_assert(GW_END + 256 + NBINS * 4 <= GMAX, "GD message");

inline uint64_t hmix(uint64_t h, uint64_t v) {
  uint64_t z = h + 0x9e3779b97f4a7c15ull + v;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
inline uint64_t hbytes(uint64_t h, const void *p, size_t n) {
  const uint8_t *b = (const uint8_t *)p;
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t v;
    std::memcpy(&v, b + i, 8);
    h = hmix(h, v);
  }
  uint64_t t = 0;
  for (size_t k = 0; i < n; ++i, ++k) t |= (uint64_t)b[i] << (8 * k);
  return hmix(h, t ^ n);
}

// ---- kernels ----------------------------------------------------------------
// the one-route's order-histogram words (k_nw_order_hist: [0] error bits, [1]
// kept, [3] no pack, [4] longest) in k_sh_rows' layout
__global__ void k_sh_one_words(const uint32_t *c, uint32_t *w) {
  if (threadIdx.x == 0) {
    w[0] = c[0];
    w[20] = c[3];
    w[21] = c[4];
    w[25] = c[1];
  }
}

// head of the GC / GD / GE messages: the error / flag words and the fast words
__global__ void k_msg_head(const uint32_t *ctrl, uint32_t *w) {
  const uint32_t t = threadIdx.x;
  if (t < 8) w[t] = ctrl[t];
  else if (t < 16) w[t] = ctrl[FW + t - 8];
}

// per source row, with the bounds of every slice, Y range and lead-in: the Y
// records each slice sends to each Y owner (YOp12's masks), the lead-in
// records each slice sends to each later slice (GhostOp16's), and the rows in
// every Y range's first / last bucket (YStateOp's selections)
struct ShCountArgs {
  Frags f;
  uint32_t drop, P;
  Bounds sk;
  int64_t ylo[MAXP], yhi[MAXP];
  uint64_t thr[MAXP];
  uint64_t fb[MAXP], lb[MAXP];  // ~0: an empty range
  uint32_t *out;                // [P * P] Y, [P * P] lead-in, [P] first, [P] last
};
__global__ void __launch_bounds__(256) k_sh_counts(ShCountArgs a) {
  __shared__ uint32_t c[2 * MAXP * MAXP + 2 * MAXP];
  const uint32_t P = a.P, W = 2 * P * P + 2 * P;
  for (uint32_t j = threadIdx.x; j < W; j += 256) c[j] = 0;
  __syncthreads();
  uint32_t *ym = c, *hm = c + P * P, *fc = c + 2 * P * P, *lc = fc + P;
  GRID_STRIDE(i, a.f.n) {
    const uint64_t xs = a.f.x[i];
    const uint64_t pk = div10_sh(xs);
    if (pk >= a.drop) continue;  // (the never-iterated last bucket: no record)
    const uint64_t ys = a.f.y[i];
    const uint32_t len = (uint32_t)(a.f.len[i] & 0xFFFFFFu);  // every row packs here
    const uint32_t s = owner_of(a.sk, pk);
    const uint64_t yb = (ys + len / 2) / 100, xb = (xs + len / 2) / 100;
    for (uint32_t q = 0; q < P; ++q) {
      if ((int64_t)yb >= a.ylo[q] && (int64_t)yb < a.yhi[q]) atomicAdd(&ym[s * P + q], 1u);
      if (yb == a.fb[q]) atomicAdd(&fc[q], 1u);
      if (yb == a.lb[q]) atomicAdd(&lc[q], 1u);
    }
    for (uint32_t g = s + 1; g < P; ++g)
      if (xb >= a.thr[g]) atomicAdd(&hm[s * P + g], 1u);
  }
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < W; j += 256)
    if (c[j]) atomicAdd(&a.out[j], c[j]);
}

// k_sh_x_own, counting the own X hits whose winner sits in an earlier slice
// (a cross-slice link per entry: lk[me * P + owner of the winner])
__global__ void k_sh_x_own_fast(const uint32_t *xpos, const uint8_t *state, const uint32_t *par,
                                const uint4 *halo, uint32_t G, uint32_t m, uint32_t poff,
                                uint32_t *xg, uint8_t *used, Bounds slices, uint32_t me,
                                uint32_t *lk) {
  __shared__ uint32_t c[MAXP];
  const uint32_t P = slices.P;
  if (threadIdx.x < MAXP) c[threadIdx.x] = 0;
  __syncthreads();
  GRID_STRIDE(k, G + m) {
    const bool hit = state[xpos[k]] == ST_HIT;
    if (k < G) {
      used[k] = hit ? 0 : 1;
      continue;
    }
    const uint32_t w = par[k];
    uint32_t g = NONE;
    if (hit) {
      if (w < G) {
        g = halo[w].y;
        atomicAdd(&c[owner_of(slices, g)], 1u);
      } else {
        g = poff + (w - G);
      }
    }
    xg[k - G] = g;
  }
  __syncthreads();
  if (threadIdx.x < P && c[threadIdx.x]) atomicAdd(&lk[me * P + threadIdx.x], c[threadIdx.x]);
}

// lanes with `on` add one to cnt[key]: one LDS atomic per distinct key in
// the wavefront (every lane of the wavefront must call it)
__device__ __forceinline__ void wave_count(bool on, uint32_t key, uint32_t *cnt) {
  uint64_t act = __ballot(on);
  while (act) {
    const int lead = __builtin_ctzll(act);
    const uint32_t k0 = (uint32_t)__shfl((int)key, lead);
    const uint64_t b = __ballot(on && key == k0);
    if ((int)(threadIdx.x & 63) == lead) atomicAdd(&cnt[k0], (uint32_t)__popcll(b));
    act &= ~b;
  }
}

// k_sh_y_results, counting per slice (the slice of the record's processing
// index) the parents this Y owner sends (X misses of its own range whose slice
// is another rank's), the roots (Y misses among them) and the cross-slice
// links (Y winner in another slice).  A winner outside the held records (an
// axis left open: the call is repeated) is not followed.
__global__ void __launch_bounds__(256) k_sh_y_results_fast(
    const uint3 *yr, const uint8_t *code, uint32_t c, const uint32_t *par, uint8_t *ystate,
    uint32_t *ywin, uint32_t poff, uint32_t m, uint32_t *xpar, Bounds slices, uint32_t me,
    uint32_t *pc, uint32_t *rc, uint32_t *lk, uint32_t *flag) {
  __shared__ uint32_t cnt[2 * MAXP + MAXP * MAXP];
  const uint32_t P = slices.P, lane = threadIdx.x & 63;
  for (uint32_t j = threadIdx.x; j < 2 * P + P * P; j += blockDim.x) cnt[j] = 0;
  __syncthreads();
  for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r - lane < c;
       r += gridDim.x * blockDim.x) {
    bool par_on = false, root_on = false, link_on = false;
    uint32_t s = 0, b = 0;
    if (r < c) {
      const uint8_t cr = code[r];
      if (cr & YC_XHIT) {
        ystate[r] = 1;
        ywin[r] = NONE;
      } else {
        uint32_t p = par[r];
        if (p >= c) {
          atomicOr(flag, RETRY_PARENT);
          p = r;
        }
        ystate[r] = p == r ? 1 : 0;
        const uint32_t w = yr[p].y, self = yr[r].y;
        ywin[r] = w;
        if (!(cr & 3)) {  // (a halo record: its owner decides it)
          const uint32_t own = self - poff;
          if (own < m) xpar[own] = w;
          s = owner_of(slices, self);
          par_on = s != me;
          if (p == r) {
            root_on = true;
          } else {
            b = owner_of(slices, w);
            link_on = b != s;
          }
        }
      }
    }
    wave_count(par_on, s, cnt);
    wave_count(root_on, P + s, cnt);
    wave_count(link_on, 2 * P + s * P + b, cnt);
  }
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < 2 * P + P * P; j += blockDim.x) {
    const uint32_t v = cnt[j];
    if (!v) continue;
    if (j < P) atomicAdd(&pc[j], v);
    else if (j < 2 * P) atomicAdd(&rc[j - P], v);
    else atomicAdd(&lk[j - 2 * P], v);
  }
}

// the root count of this slice against the one the Y owners counted
__global__ void k_expect1(const uint32_t *v, uint32_t want, uint32_t *flag, uint32_t bit) {
  if (threadIdx.x == 0 && *v != want) atomicOr(flag, bit);
}
__global__ void k_copy_word(const uint32_t *src, uint32_t *dst) {
  if (threadIdx.x == 0) *dst = *src;
}

// k_final_gid without the error bit: after a request round that may not be
// the last, the labels can still be open (the next gather says)
__global__ void k_final_gid_spec(const uint32_t *lpar, const uint32_t *lab, uint32_t m,
                                 uint32_t *gid) {
  GRID_STRIDE(k, m) {
    const uint32_t g = lab[lpar[k]];
    gid[k] = g == NONE ? 0u : g;
  }
}

// ---- host helpers --------------------------------------------------------------
// per source rank and slice, the rows of its gathered histogram in the slice
template <class T>
static uint64_t bins_in(const T *h, const Bounds &B, uint32_t q, uint32_t shift) {
  const uint64_t unit = 1ull << shift;
  const uint64_t b0 = (B.b[q] + unit - 1) >> shift, b1 = (B.b[q + 1] + unit - 1) >> shift;
  uint64_t c = 0;
  for (uint64_t b = b0; b < b1 && b < NBINS; ++b) c += h[b];
  return c;
}

// an exchange whose per-peer counts every rank knows: straight to the
// all-to-all (known: the stage's sizes match the last completed call, no rank
// grows a buffer), or through Shard::exchange's count gather and agreement
template <class T>
T *xchg(Shard &S, bool known, const void *send, const PartPlan &pp, const uint64_t *rcnt,
        int slot, uint32_t *nrecv) {
  const uint32_t P = S.P;
  if (P == 1) {  // one rank: the send block is the receive block
    *nrecv = (uint32_t)pp.total;
    return const_cast<T *>(reinterpret_cast<const T *>(send));
  }
  if (!known) {
    uint32_t n = 0;
    T *r = S.exchange<T>(send, pp, slot, &n);
    uint64_t want = 0;
    for (uint32_t q = 0; q < P; ++q) want += rcnt[q];
    if (n != want) {
      S.ctx->err = "fast path: exchange size differs from the agreed counts";
      throw RK_E_INTERNAL;
    }
    *nrecv = n;
    return r;
  }
  uint64_t sb[MAXP], rb[MAXP], tot = 0;
  for (uint32_t q = 0; q < P; ++q) {
    sb[q] = pp.cnt[q] * sizeof(T);
    rb[q] = rcnt[q] * sizeof(T);
    tot += rcnt[q];
  }
  T *recv = S.take<T>(slot, tot + 1);
  S.run_a2a(send, sb, recv, rb);
  ++S.n_agree_skipped;
  *nrecv = (uint32_t)tot;
  return recv;
}

// a plan whose per-destination counts come back in a message (the next
// request round): the counts and the scan on the device, the totals into the
// payload (k_totals' cumulative offsets), no readback
template <class Op>
void plan_to_msg(Shard &S, const Op &op, uint32_t n, PartPlan &pp, uint32_t *tot) {
  pp.n = n;
  pp.nblk = n ? (n + PART_TILE - 1) / PART_TILE : 1;
  const size_t len = (size_t)S.P * pp.nblk + 1;
  uint32_t *cnt = S.take<uint32_t>(SL_PCNT, len);
  pp.off = S.take<uint32_t>(SL_POFF, len);
  S.zero(cnt + len - 1, 4);
  kt_begin(S.st, KID_PART);
  k_part_count<<<pp.nblk, 256, 0, S.st>>>(op, n, S.P, pp.nblk, cnt, pp.mcache, pp.mread);
  kt_end(S.st, KID_PART, 0.0);
  S.launched("k_part_count");
  exclusive_scan_u32(cnt, pp.off, len, S.scan_scratch(SL_PSCAN, len), S.st);
  k_totals<<<1, 64, 0, S.st>>>(pp.off, pp.nblk, S.P, tot);
  S.launched("k_totals");
}

// ---- the driver ------------------------------------------------------------------
// Returns RK_OK, an error, RK_SHARD_FALLBACK (a row does not pack: the generic
// driver) or RK_SHARD_RETRY (the careful driver).  *N_out / *row_base_out:
// every rank's rows / this rank's first global row.
int classify_sharded_fast(Shard &S, const rk_frags_soa *in, const rk_params &p, int32_t lead_in,
                          rk_shard_result *out, int pre, uint64_t *N_out, uint64_t *row_base_out) {
  rk_ctx *ctx = S.ctx;
  rk_shard_stats &ss = ctx->shard_stats;
  const uint32_t P = S.P, me = S.me;
  const uint64_t H = lead_in < 0 ? 2 : (uint64_t)lead_in;
  const uint64_t len_x = p.len_x_hdr + 1, len_y = p.len_y_hdr + 1;  // FragmentsDatabase.cpp:62,65
  const uint64_t vsize = 1 + len_x / 10;                             // :84
  const uint64_t max_x = len_x / 100, max_y = len_y / 100;           // SequenceOcupationList.cpp:4
  const uint32_t nbx = (uint32_t)(max_x + 1), nby = (uint32_t)(max_y + 1);
  const uint32_t drop = (uint32_t)(vsize - 1);
  hipStream_t st = S.st, st2 = S.st2;
  if (pre) {  // this rank cannot run: its status in the peers' first gather (GA)
    (void)S.status_gather(pre, nullptr, nullptr, 0);
    throw pre;
  }
  uint32_t *F = S.ctrl + FW;
  S.expect_flag = F;
  S.expect_bit = RETRY_EXPECT;
  ss.fast_path = 1;
  const bool solo = P == 1;
  auto tphase = std::chrono::steady_clock::now();

  // ---- GA: rows, checks, the slice and Y-range histograms ---------------------
  const uint64_t n_mine = pre ? 0 : in->n;
  const uint32_t nl = (uint32_t)n_mine;
  const uint32_t shift = bin_shift(drop), yshift = bin_shift(nby);
  static const bool one_on = [] {
    const char *e = getenv("RK_SH_ONE");
    return !(e && e[0] == '0');
  }();
  const bool one = one_on && P == 1;
  const NwDigits ad = nw_plan(bit_length(vsize - 1));
  const NwDigits yd = nw_plan(bit_length(2ull * nby - 1), 9);
  const NwOrderPlan op1 = one ? nw_order_split_range(nl, 0, drop) : NwOrderPlan{};
  uint32_t *hist = S.take<uint32_t>(SN_HIST, 3 * 4096);  // order / Y / member digit histograms
  uint8_t *pay = S.msg_begin(P > 1 ? GA_END : GA_XH);
  uint32_t *wa = reinterpret_cast<uint32_t *>(pay + GA_WORDS);
  S.zero(F, 16 * 4);
  Frags f{pre ? nullptr : in->x_start, pre ? nullptr : in->y_start,
          pre ? nullptr : in->length, pre ? nullptr : in->strand, nl};
  if (!pre && nl) {
    if (one) {
      S.zero(hist, 3 * 4096 * 4);
      S.zero(S.ctrl + 32, 16 * 4);
      nw_order_hist(*in, vsize, max_x, max_y, nby, op1.nseg ? op1.coarse : ad, yd, hist,
                    hist + 4096, S.ctrl + 32, st);
      k_sh_one_words<<<1, 64, 0, st>>>(S.ctrl + 32, wa);
    } else {
      ShRowsArgs ra{f, vsize, max_x, max_y, shift,
                    P > 1 ? reinterpret_cast<uint32_t *>(pay + GA_XH) : nullptr, wa};
      if (P > 1) {
        ra.yhist = reinterpret_cast<uint32_t *>(pay + GA_YH);
        ra.yshift = yshift;
      }
      kt_begin(st, KID_SH_ROWKEYS);
      k_sh_rows<<<grid_for(nl, 256, P > 1 ? 1024 : 4096), 256, 0, st>>>(ra);
      kt_end(st, KID_SH_ROWKEYS, 25.0 * nl);
    }
    S.launched("rows");
  }
  {
    uint64_t hostp[9];
    hostp[0] = n_mine;
    for (int k = 0; k < 8; ++k) hostp[1 + k] = ctx->sh_fp[k];
    if (S.msg_gather(pre, hostp, sizeof hostp)) throw pre ? pre : (int)RK_E_PEER;
  }
  uint64_t N = 0, row_base = 0;
  std::vector<uint64_t> nall(P), kept(P), fps((size_t)P * 8);
  uint32_t anyerr = 0, nopack = 0, maxlen = 0;
  std::vector<uint64_t> gh(NBINS, 0), gy(NBINS, 0);
  std::vector<uint32_t> hx_all(P > 1 ? (size_t)P * NBINS : 0);  // every rank's own row bins
  uint64_t fp = hmix(0x5eedull, P);
  fp = hmix(hmix(hmix(fp, H), len_x), len_y);
  for (uint32_t q = 0; q < P; ++q) {
    const uint8_t *mq = S.msg_of(q);
    std::memcpy(&nall[q], mq + GA_HOST, 8);
    std::memcpy(&fps[(size_t)q * 8], mq + GA_HOST + 8, 64);
    const uint32_t *w = reinterpret_cast<const uint32_t *>(mq + GA_WORDS);
    N += nall[q];
    row_base += q < me ? nall[q] : 0;
    anyerr |= w[0];
    nopack |= w[20];
    maxlen = w[21] > maxlen ? w[21] : maxlen;
    kept[q] = w[25];
    fp = hmix(hmix(hmix(fp, nall[q]), kept[q]), w[21]);
    if (P > 1) {
      const uint32_t *hx = reinterpret_cast<const uint32_t *>(mq + GA_XH);
      const uint32_t *hy = reinterpret_cast<const uint32_t *>(mq + GA_YH);
      std::memcpy(&hx_all[(size_t)q * NBINS], hx, NBINS * 4);
      for (uint32_t b = 0; b < NBINS; ++b) gh[b] += hx[b], gy[b] += hy[b];
      fp = hbytes(hbytes(fp, hx, NBINS * 4), hy, NBINS * 4);
    }
  }
  *N_out = N;
  *row_base_out = row_base;
  if (N >= 0xFFFFFFFFull) return RK_E_TOO_MANY;  // every rank sees the same N
  ss.n_in = nl;
  ss.n_total = N;
  S.check(err_status(ctx, anyerr & ~(uint32_t)ERRB_WIDE_LENGTH));
  if (nopack) return RK_SHARD_FALLBACK;
  // the fingerprints every rank holds for each stage (a stage runs without
  // agreement points when every rank holds the same one and it matches)
  const auto fp_known = [&](int k, uint64_t want) {
    for (uint32_t q = 0; q < P; ++q)
      if (fps[(size_t)q * 8 + k] != want || !want) return false;
    return true;
  };
  uint64_t new_fp[8] = {};
  uint64_t kept_all = 0;
  for (uint32_t q = 0; q < P; ++q) kept_all += kept[q];
  const Bounds slice_keys = split_bounds(gh, shift, drop, P);
  if (slice_max_rows(gh, slice_keys, shift, P, kept_all) >= (1ull << 30)) return RK_SHARD_FALLBACK;
  std::vector<uint64_t> mall(P, 0);  // every slice: the global histogram's bins between its bounds
  for (uint32_t q = 0; q < P; ++q)
    mall[q] = P == 1 ? kept_all : bins_in(gh.data(), slice_keys, q, shift);
  const uint32_t m = (uint32_t)mall[me];
  uint64_t poff64 = 0;
  for (uint32_t q = 0; q < me; ++q) poff64 += mall[q];
  const uint32_t poff = (uint32_t)poff64;
  Bounds slices{};
  slices.P = P;
  for (uint32_t q = 0, acc = 0; q <= MAXP; ++q) {
    slices.b[q] = acc;
    if (q < P) acc += (uint32_t)mall[q];
  }
  ss.n_slice = m;
  const Bounds yb = split_bounds(gy, yshift, nby, P);
  const uint64_t ylo = yb.b[me], yhi = yb.b[me + 1];
  int64_t ylo_ext[MAXP] = {}, yhi_ext[MAXP] = {};
  for (uint32_t q = 0; q < P; ++q) {
    ylo_ext[q] = (int64_t)yb.b[q] - 1 - (int64_t)H;
    yhi_ext[q] = (int64_t)yb.b[q + 1] + 1 + (int64_t)H;
  }
  uint64_t thr[MAXP];
  for (uint32_t g = 0; g < MAXP; ++g) {
    thr[g] = ~0ull;
    if (g < P && mall[g]) {
      const uint64_t bmin = slice_keys.b[g] / 10;  // xStart >= 10*key, centre >= xStart
      thr[g] = bmin >= 1 + H ? bmin - 1 - H : 0;
    }
  }
  uint64_t fbk[MAXP], lbk[MAXP];  // every Y range's first and last bucket
  for (uint32_t q = 0; q < MAXP; ++q) {
    const bool ne = q < P && yb.b[q] < yb.b[q + 1];
    fbk[q] = ne ? yb.b[q] : ~0ull;
    lbk[q] = ne ? yb.b[q + 1] - 1 : ~0ull;
  }

  // ---- GB: the exchange sizes, counted over the source rows -------------------
  std::vector<uint64_t> Ym((size_t)P * P, 0), Hm((size_t)P * P, 0), Fc(P, 0), Lc(P, 0);
  if (P > 1) {
    pay = S.msg_begin((size_t)(2 * P * P + 2 * P) * 4);
    if (nl) {
      ShCountArgs ca{};
      ca.f = f;
      ca.drop = drop;
      ca.P = P;
      ca.sk = slice_keys;
      for (uint32_t q = 0; q < MAXP; ++q) {
        ca.ylo[q] = ylo_ext[q];
        ca.yhi[q] = yhi_ext[q];
        ca.thr[q] = thr[q];
        ca.fb[q] = fbk[q];
        ca.lb[q] = lbk[q];
      }
      ca.out = reinterpret_cast<uint32_t *>(pay);
      kt_begin(st, KID_SHARD_AUX);
      k_sh_counts<<<grid_for(nl, 256, 1024), 256, 0, st>>>(ca);
      kt_end(st, KID_SHARD_AUX, 25.0 * nl);
      S.launched("k_sh_counts");
    }
    if (S.msg_gather(0)) throw (int)RK_E_PEER;
    for (uint32_t q = 0; q < P; ++q) {
      const uint32_t *w = reinterpret_cast<const uint32_t *>(S.msg_of(q));
      for (size_t j = 0; j < (size_t)P * P; ++j) Ym[j] += w[j], Hm[j] += w[P * P + j];
      for (uint32_t k = 0; k < P; ++k) Fc[k] += w[2 * P * P + k], Lc[k] += w[2 * P * P + P + k];
    }
  }
  const auto Yat = [&](uint32_t s, uint32_t q) { return Ym[(size_t)s * P + q]; };
  const auto Hat = [&](uint32_t s, uint32_t g) { return Hm[(size_t)s * P + g]; };
  // the Y-state counts owner q -> rank r: YStateOp sends q's first-bucket
  // entries to every rank whose range ends at q's start, its last-bucket ones
  // to every rank whose range starts at q's end (once to a rank in both)
  std::vector<uint64_t> Ys((size_t)P * P, 0);
  for (uint32_t q = 0; q < P; ++q)
    for (uint32_t r = 0; r < P; ++r) {
      if (r == q) continue;
      const bool fm = yb.b[r + 1] == yb.b[q], lm = yb.b[r] == yb.b[q + 1];
      uint64_t c = (fm ? Fc[q] : 0) + (lm ? Lc[q] : 0);
      if (fm && lm && fbk[q] == lbk[q] && fbk[q] != ~0ull) c -= Fc[q];
      Ys[(size_t)q * P + r] = c;
    }
  uint64_t ny64 = P == 1 ? m : 0, G64 = 0;
  for (uint32_t s = 0; P > 1 && s < P; ++s) ny64 += Yat(s, me), G64 += Hat(s, me);
  for (uint32_t r = 0; P > 1 && r < P; ++r) {  // every rank's Y range under the 30-bit bound
    uint64_t c = 0;
    for (uint32_t s = 0; s < P; ++s) c += Yat(s, r);
    if (c >= (1ull << 30)) {
      ctx->err = "a Y range of 2^30 or more records";
      throw RK_E_TOO_MANY;
    }
  }
  fp = hbytes(hbytes(fp, Ym.data(), Ym.size() * 8), Hm.data(), Hm.size() * 8);
  fp = hbytes(hbytes(fp, Fc.data(), Fc.size() * 8), Lc.data(), Lc.size() * 8);
  new_fp[0] = fp;
  const bool knownA = P > 1 && fp_known(0, fp);
  S.alloc_locked = knownA;
  ss.fast_stages |= knownA ? 1u : 0u;
  // the GC message collects the axes' flags and counts from here on
  uint32_t *gc = reinterpret_cast<uint32_t *>(S.msg_begin(GW_END + (size_t)(2 * P + P * P) * 4));
  uint32_t *gc_pc = gc + GW_END / 4, *gc_rc = gc_pc + P, *gc_lk = gc_rc + P;
  ss.ms_ingress = ms_since(tphase);

  // ---- 2: rows -> slice owners as 16-B records ----------------------------------
  tphase = std::chrono::steady_clock::now();
  RowOp16 rop{f, slice_keys, drop, (uint32_t)row_base, nullptr};
  PartPlan pp;
  rop.out = S.take<uint4>(SN_SROWS, (size_t)nl + 1);
  const bool fast = one && kept[0] == nl;  // the order sort reads the rows themselves
  if (fast) {
    S.identity_plan(nl, pp);
  } else if (P == 1 && kept[0] == nl) {
    S.emit_identity(rop, nl, pp);
  } else {
    uint64_t cnt[MAXP] = {};
    for (uint32_t q = 0; q < P; ++q)
      cnt[q] = P == 1 ? kept[0] : bins_in(&hx_all[(size_t)me * NBINS], slice_keys, q, shift);
    S.plan_counts(rop, nl, pp, cnt);
    S.emit(rop, pp);
  }
  uint64_t rfrom[MAXP] = {};
  for (uint32_t q = 0; q < P; ++q)
    rfrom[q] = P == 1 ? pp.total : bins_in(&hx_all[(size_t)q * NBINS], slice_keys, me, shift);
  uint32_t mrecv = 0;
  const uint4 *rin = xchg<uint4>(S, knownA, rop.out, pp, rfrom, SN_RIN, &mrecv);
  if (mrecv != m) {
    ctx->err = "fast path: slice size differs from the histogram's";
    throw RK_E_INTERNAL;
  }

  // ---- 3: the slice's processing order, its Y records ---------------------------
  uint32_t *ahist = hist, *yhist = hist + 4096, *ehist = hist + 2 * 4096;
  if (!fast) S.zero(ahist, 3 * 4096 * 4);
  const size_t sw = nw_status_words(m + 1);
  uint32_t *astat = S.take<uint32_t>(SN_STAT, sw);
  uint4 *Ra = S.take<uint4>(SN_RA, m + 1), *Rb = S.take<uint4>(SN_RB, m + 1);
  uint4 *yown = S.take<uint4>(SN_YOWN, (size_t)m * 3 / 4 + 2);
  const NwOrderPlan op = fast ? op1 : nw_order_split_range(m, slice_keys.b[me], slice_keys.b[me + 1]);
  ss.order_split = op.nseg ? 1u : 0u;
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
    if (fast) {
      nw_order_sort_split_coarse(*in, op, ahist, astat, Ra, Rb, chist,
                                 ZeroRegion{own_cc.cnts, ((size_t)3 * own_cc.nch + 1) * 4}, vsize,
                                 st, nullptr);
      nw_order_sort_split_fine(nl, m, nby, op, Ra, Rb, yown, rop.out, chist, coff,
                               S.scan_scratch(SL_PSCAN, (size_t)op.nseg + 1), &own_cc, st);
    } else {
      nw_rec_hist(rin, 16, m, op.kbase, op.coarse, ahist, st);
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

  // ---- 4: Y records -> Y-range owners (+ halos) ----------------------------------
  YOp12 yop{};
  yop.yrec = reinterpret_cast<const uint3 *>(yown);
  yop.nby = nby;
  yop.P = P;
  yop.shift = yshift;
  for (uint32_t q = 0; q < MAXP; ++q) {
    yop.lo[q] = q < P ? ylo_ext[q] : 0;
    yop.hi[q] = q < P ? yhi_ext[q] : 0;
  }
  PartPlan ypp;
  if (P == 1) {
    S.identity_plan(m, ypp);
  } else {
    uint64_t cnt[MAXP] = {};
    for (uint32_t q = 0; q < P; ++q) cnt[q] = Yat(me, q);
    ypp.mcache = S.take<uint32_t>(SL_YMASK, m + 1);  // the X-hit bytes follow the same masks
    S.plan_counts(yop, m, ypp, cnt);
  }
  const bool y_self = ypp.total == m && ypp.cnt[me] == m;
  if (!y_self) {
    yop.out = S.take<uint3>(SN_SY, ypp.total + 1);
    S.emit(yop, ypp);
  }
  uint64_t yfrom[MAXP] = {};
  for (uint32_t q = 0; q < P; ++q) yfrom[q] = P == 1 ? m : Yat(q, me);
  uint32_t ny = 0;
  const uint3 *yr = xchg<uint3>(S, knownA, y_self ? yop.yrec : yop.out, ypp, yfrom, SN_YR, &ny);
  if (ny != ny64) {
    ctx->err = "fast path: Y range size differs from the counts";
    throw RK_E_INTERNAL;
  }
  ss.y_entries = ny;
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
  S.hip(hipEventRecord(ctx->fork, st), "fork");
  S.hip(hipStreamWaitEvent(st2, ctx->fork, 0), "fork wait");
  if (ny) {
    if (!solo) {  // (one rank: no halo classes, no verification, no parents to send)
      k_sh_ycode<<<grid_for(ny, 256), 256, 0, st2>>>(yr, ny, nby, ylo, yhi, ycode);
      S.launched("k_sh_ycode");
    }
    if (!fast) nw_rec_hist(yr, 12, ny, 0, yd, yhist, st2);
  }
  S.hip(hipEventRecord(ctx->join, st2), "join");
  ss.ms_y = ms_since(tphase);

  // ---- 5: X lead-in halo from earlier slices -------------------------------------
  tphase = std::chrono::steady_clock::now();
  GhostOp16 gop{};
  gop.R = Ra;
  gop.P = P;
  gop.me = me;
  gop.poff = poff;
  gop.base = 0;
  for (uint32_t g = 0; g < MAXP; ++g) gop.thr[g] = thr[g];
  uint64_t hsend[MAXP] = {}, hfrom[MAXP] = {};
  uint64_t hsend_tot = 0;
  for (uint32_t q = 0; q < P; ++q) {
    hsend[q] = P > 1 ? Hat(me, q) : 0;
    hfrom[q] = P > 1 ? Hat(q, me) : 0;
    hsend_tot += hsend[q];
  }
  PartPlan hpp;
  if (hsend_tot && m) {
    // the suffix of the slice whose centres can reach a later slice's lead-in
    // starts on the device (no readback): entries before it select nothing
    uint64_t thr_min = ~0ull;
    for (uint32_t g = me + 1; g < P; ++g) thr_min = thr[g] < thr_min ? thr[g] : thr_min;
    const uint64_t reach = thr_min * 100, half = maxlen / 2;
    const uint64_t key0 = reach > half + 10 ? (reach - half) / 10 - 1 : 0;
    k_lower_bound16<<<1, 1, 0, st>>>(Ra, m, key0, S.ctrl + 22);
    S.launched("k_lower_bound16");
    gop.dbase = S.ctrl + 22;
    S.plan_counts(gop, m, hpp, hsend);
  } else {
    S.zero_plan(0, hpp);
  }
  gop.out = S.take<uint4>(SN_SHALO, hpp.total + 1);
  if (hpp.n) S.emit(gop, hpp);
  uint32_t G = 0;
  const uint4 *hx = xchg<uint4>(S, knownA, gop.out, hpp, hfrom, SN_HX, &G);
  if (G != G64) {
    ctx->err = "fast path: lead-in size differs from the counts";
    throw RK_E_INTERNAL;
  }
  ss.x_ghosts = G;

  // ---- 6: X axis over [halo ; own], its sweeps queued -----------------------------
  uint32_t *xg = S.take<uint32_t>(SL_XG, m + 1);
  uint8_t *xused = S.take<uint8_t>(SN_XGUSED, G + 1);
  S.zero(S.ctrl + 6, 4);
  const uint32_t mx = G + m;
  if (mx) {
    NwChunkCounts cc{};
    cc.W = nw_chunk_width(mx, (uint32_t)(span < nbx ? span : nbx));
    while ((1u << cc.lgW) < cc.W) ++cc.lgW;
    cc.nch = nw_chunks(nbx, cc.W);
    cc.cnts = S.take<uint32_t>(SN_XCNT, (size_t)3 * cc.nch + 2);
    uint32_t *xoff = S.take<uint32_t>(SN_XOFF, (size_t)3 * cc.nch + 2);
    if (own_counts && cc.W == own_cc.W) {
      S.hip(hipMemcpyAsync(cc.cnts, own_cc.cnts, ((size_t)3 * cc.nch + 1) * 4,
                           hipMemcpyDeviceToDevice, st), "counts copy");
      nw_x_count_add(hx, G, cc, st);
    } else {
      nw_x_count(Ra, mx, cc, st, hx, G);
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
    // one rank: entry ids are processing indices, and both axes write their
    // decisions straight into the parent words (as on one device)
    uint32_t *par = solo ? xg : S.take<uint32_t>(SN_PAR, mx + 1);
    nw_x_chunks(Ra, mx, nbx, max_x, maxlen, xoff, cx, xpos, erec, S.ctrl, cc.W, st, hx, G);
    S.launched("X chunks");
    Axis ax{cx.key, cx.ent, nullptr, nullptr, cx.state, nullptr, par, cx.pk, cx.nbd,
            S.take<uint32_t>(SL_RLEN, mx), S.take<uint32_t>(SL_RBEG, mx), mx, max_x,
            p.len_ratio, p.pos_ratio};
    SweepScratch sc{S.take<uint32_t>(SL_RUNS, runs_scratch_words(mx)),
                    S.take<uint8_t>(SL_WPEND, mx / 64 + 1), S.take<uint8_t>(SL_RPEND, mx),
                    S.ctrl + 64, S.ctrl + 4};
    S.check(resolve_axis_queued(ctx, ax, sc, ctx->sh_blind[0], F + 3));
    if (solo) {  // the X hits as the Y sort's bitmask (k_nw_x_bits, as on one device)
      nw_x_bits(xpos, cx.state, m, ybits, st);
      S.launched("k_nw_x_bits");
    } else {
      kt_begin(st, KID_SH_XOWN);
      k_sh_x_own_fast<<<grid_for(mx, 256, 4096), 256, 0, st>>>(xpos, cx.state, par, hx, G, m,
                                                               poff, xg, xused, slices, me, gc_lk);
      kt_end(st, KID_SH_XOWN, 0.0);
      S.launched("k_sh_x_own_fast");
    }
  }
  // the owners' final states of the lead-in (the same selection as the records)
  if (P > 1) {
    GhostOp16 sop = gop;
    sop.out = nullptr;
    sop.xg = xg;
    PartPlan spp;
    if (hpp.n) S.plan_counts(sop, m, spp, hsend);
    else S.zero_plan(0, spp);
    sop.sout = S.take<uint8_t>(SL_SEND, spp.total + 1);
    if (spp.n) S.emit(sop, spp);
    uint32_t G2 = 0;
    const uint8_t *xown = xchg<uint8_t>(S, knownA, sop.sout, spp, hfrom, SL_XOWN, &G2);
    const uint64_t bmin_me = slice_keys.b[me] / 10;
    const uint64_t rel_x = bmin_me >= 1 ? bmin_me - 1 : 0;  // relevant: probed by own queries
    if (G) {
      k_cmp_x16<<<grid_for(G, 256, 1024), 256, 0, st>>>(hx, G, rel_x, xused, xown, F + 1);
      S.launched("k_cmp_x16");
    }
    ss.x_rounds = 1;
  }
  ss.ms_x = ms_since(tphase);

  // ---- 7: X-hit bytes after the Y records, the Y sort, its sweeps ----------------
  tphase = std::chrono::steady_clock::now();
  if (solo) {
    S.hip(hipStreamWaitEvent(st, ctx->join, 0), "join wait");
  } else {
    YOp12 xop = yop;
    xop.xg = xg;
    PartPlan xpp;
    xop.xout = S.take<uint8_t>(SN_SXH, (size_t)ypp.total + 1);
    if (P == 1) {
      S.emit_identity(xop, m, xpp);
    } else {
      xpp.mcache = ypp.mcache;
      xpp.mread = true;
      S.plan_same(xop, m, xpp, ypp);
      S.emit(xop, xpp);
    }
    uint32_t n2 = 0;
    const uint8_t *xh = xchg<uint8_t>(S, knownA, xop.xout, xpp, yfrom, SL_YXH, &n2);
    S.hip(hipStreamWaitEvent(st, ctx->join, 0), "join wait");
    if (ny) {
      kt_begin(st, KID_SH_MERGE);
      k_sh_xhit_bits<<<grid_for(ny, 256), 256, 0, st>>>(xh, ny, ycode, ybits);
      kt_end(st, KID_SH_MERGE, 0.0);
      S.launched("k_sh_xhit_bits");
    }
  }
  if (ny) {
    nw_y_sort_after_x(yB, yA, ny, yd, yhist, ystat, cy, nby, max_y, ybits, st,
                      reinterpret_cast<const uint4 *>(yr));
    S.launched("Y sort");
    Axis ay{cy.key, cy.ent, nullptr, nullptr, cy.state, nullptr, solo ? xg : par_l, cy.pk, cy.nbd,
            S.take<uint32_t>(SL_RLEN, ny), S.take<uint32_t>(SL_RBEG, ny), ny, max_y, p.len_ratio,
            p.pos_ratio};
    ay.par_dev = true;
    SweepScratch sc{S.take<uint32_t>(SL_RUNS, runs_scratch_words(ny)),
                    S.take<uint8_t>(SL_WPEND, ny / 64 + 1), S.take<uint8_t>(SL_RPEND, ny),
                    S.ctrl + 64, S.ctrl + 4};
    S.check(resolve_axis_queued(ctx, ay, sc, ctx->sh_blind[1], F + 4));
  }
  if (ny && !solo) {
    kt_begin(st, KID_SH_YRES);
    // (a grid of at most 2048 blocks: each block adds its counts with global
    // atomics on a few shared words, and 65536 blocks serialised them there)
    k_sh_y_results_fast<<<grid_for(ny, 256, 2048), 256, 0, st>>>(yr, ycode, ny, par_l, ystate, ywin,
                                                           poff, m, xg, slices, me, gc_pc, gc_rc,
                                                           gc_lk, F);
    kt_end(st, KID_SH_YRES, 0.0);
    S.launched("k_sh_y_results_fast");
  }
  // the owners' states of the relevant Y halo entries
  if (P > 1) {
    const RelOp relop0{ycode, ylo ? owner_of_host(yb, ylo - 1) : 0u,
                       yhi < nby ? owner_of_host(yb, yhi) : 0u, nullptr};
    RelOp relop = relop0;
    uint64_t ysend[MAXP] = {}, yrecv[MAXP] = {};
    for (uint32_t q = 0; q < P; ++q) {
      ysend[q] = Ys[(size_t)me * P + q];
      yrecv[q] = Ys[(size_t)q * P + me];
    }
    const bool lonely = ylo == 0 && yhi == yb.b[P];
    PartPlan rp;
    if (lonely) S.zero_plan(ny, rp);
    else S.plan_counts(relop, ny, rp, yrecv);
    const uint32_t nrel = (uint32_t)rp.total;
    uint32_t *relidx = S.take<uint32_t>(SL_RELIDX, nrel + 1);
    relop.out = relidx;
    if (!lonely) S.emit(relop, rp);
    if (nrel) {
      k_set_used<<<grid_for(nrel, 256), 256, 0, st>>>(relidx, nrel, nullptr, ystate, yused);
      S.launched("k_set_used");
    }
    YStateOp yso{};
    yso.code = ycode;
    yso.ystate = ystate;
    for (uint32_t q = 0; q < P; ++q) {
      if (q == me) continue;
      if (yb.b[q + 1] == ylo) yso.first_mask |= 1u << q;
      if (yb.b[q] == yhi) yso.last_mask |= 1u << q;
    }
    const bool none = !yso.first_mask && !yso.last_mask;
    PartPlan sp;
    if (none) S.zero_plan(ny, sp);
    else S.plan_counts(yso, ny, sp, ysend);
    yso.out = S.take<uint8_t>(SL_SEND, sp.total + 1);
    if (!none) S.emit(yso, sp);
    uint32_t n2 = 0;
    const uint8_t *rys = xchg<uint8_t>(S, knownA, yso.out, sp, yrecv, SL_RYS, &n2);
    if (n2 != nrel) {
      ctx->err = "fast path: Y halo state count mismatch";
      throw RK_E_INTERNAL;
    }
    if (nrel) {
      k_cmp_y<<<grid_for(nrel, 256, 1024), 256, 0, st>>>(relidx, nrel, yused, rys, F + 2);
      S.launched("k_cmp_y");
    }
    ss.y_rounds = 1;
  }
  ss.ms_y += ms_since(tphase);

  // ---- 8: roots -------------------------------------------------------------------
  tphase = std::chrono::steady_clock::now();
  uint32_t *lpar = S.take<uint32_t>(SL_LPAR, m + 1);
  uint32_t *ext = S.take<uint32_t>(SL_EXT, m + 1);
  uint32_t *isroot = S.take<uint32_t>(SL_ISROOT, m + 2);
  uint32_t *lrank = S.take<uint32_t>(SL_LRANK, m + 2);
  uint32_t *junk = S.take<uint32_t>(SL_JUNK, m + 1);
  uint32_t *lab = S.take<uint32_t>(SL_LAB, m + 1);
  uint32_t *cur = S.take<uint32_t>(SL_CUR, m + 1);
  // local parents (X winners; the X misses' Y winners of this rank's slice
  // are in place, the other ranks' arrive with the parent exchange), chains
  // compressed inside the slice by a jumping pass and a pass over the chains
  // it left open (no readback between them; a chain still open after both is
  // a crafted input: its flag, checked with the next gather, repeats the call
  // the careful way)
  auto local_roots = [&](const ParRec *prr, uint32_t npar) {
    if (!m) return;
    if (npar) {
      kt_begin(st, KID_SHARD_AUX);
      k_par_scatter<<<grid_for(npar, 256), 256, 0, st>>>(prr, npar, poff, m, xg, S.ctrl);
      kt_end(st, KID_SHARD_AUX, 0.0);
    }
    kt_begin(st, KID_SHARD_AUX);
    k_local_par<<<grid_for(m, 256), 256, 0, st>>>(xg, m, poff, lpar, ext, isroot, S.ctrl);
    kt_end(st, KID_SHARD_AUX, 0.0);
    S.launched("parents");
    Proc jp{};
    jp.par = lpar;
    S.zero(S.ctrl + 3, 4);
    jump_listed(jp, m, junk, S.ctrl, S.take<uint32_t>(SL_JLIST, m + 1), S.ctrl + 10, S.ctrl + 3,
                st);
    S.launched("jump_listed");
    exclusive_scan_u32(isroot, lrank, (size_t)m + 1, S.scan_scratch(SL_SCAN, m + 1), st);
  };
  if (P == 1) {
    local_roots(nullptr, 0);
    if (m) {  // the slice's roots: its new groups
      k_copy_word<<<1, 64, 0, st>>>(lrank + m, gc_rc);
      S.launched("k_copy_word");
    }
  }
  k_msg_head<<<1, 64, 0, st>>>(S.ctrl, gc);
  S.launched("k_msg_head");
  if (S.msg_gather(S.sticky)) throw S.sticky ? S.sticky : (int)RK_E_PEER;
  uint32_t anyerr2 = 0, retry = 0, wide = 0;
  std::vector<uint64_t> Pm((size_t)P * P, 0), R(P, 0), Lm((size_t)P * P, 0);
  for (uint32_t q = 0; q < P; ++q) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(S.msg_of(q));
    anyerr2 |= w[0];
    wide |= w[6];
    retry |= w[8] | w[9] | w[10] | w[11] | w[12] | (P == 1 ? w[3] : 0u);
    const uint32_t *pc = w + GW_END / 4, *rc = pc + P, *lk = rc + P;
    for (uint32_t s = 0; s < P; ++s) {
      Pm[(size_t)q * P + s] = pc[s];
      R[s] += rc[s];
    }
    for (size_t j = 0; j < (size_t)P * P; ++j) Lm[j] += lk[j];
    fp = hbytes(fp, w, GW_END + (size_t)(2 * P + P * P) * 4);
  }
  if (retry) return RK_SHARD_RETRY;
  S.check(err_status(ctx, anyerr2 & ~(uint32_t)ERRB_WIDE_LENGTH));
  const bool narrow = wide == 0;  // every in-group sort key fits 32 bits
  uint64_t Gtot = 0, goff = 0;
  for (uint32_t q = 0; q < P; ++q) Gtot += R[q], goff += q < me ? R[q] : 0;
  bool links = false;
  for (uint64_t v : Lm) links |= v != 0;
  new_fp[1] = fp;
  const bool knownB = knownA && fp_known(1, fp);
  S.alloc_locked = knownB;
  ss.fast_stages |= knownB ? 2u : 0u;

  uint32_t *gid_own = junk;
  const uint32_t gshift = bin_shift(Gtot);
  MemOpNw mop{};
  // the member records: the X chunk kernel wrote them behind the halo's
  const uint2 *erk = reinterpret_cast<const uint2 *>(S.take<uint4>(SN_EREC, (size_t)mx * 3 / 4 + 2));
  mop.gid = gid_own;
  mop.erk = erk + G;
  mop.ehi = reinterpret_cast<const uint32_t *>(erk + mx) + G;
  mop.shift = gshift;
  mop.narrow = narrow;
  bool knownC = knownB;
  std::vector<uint32_t> ghist_all;  // every rank's gid histogram (the last GD)
  if (P > 1) {
    // the parent exchange: the sizes every Y owner counted
    ParOp12 pop{yr, ycode, slices, ywin, me, nullptr};
    uint64_t psend[MAXP] = {}, pfrom[MAXP] = {};
    for (uint32_t q = 0; q < P; ++q) {
      psend[q] = Pm[(size_t)me * P + q];
      pfrom[q] = Pm[(size_t)q * P + me];
    }
    PartPlan ppp;
    S.plan_counts(pop, ny, ppp, psend);
    pop.out = S.take<ParRec>(SL_SEND, ppp.total + 1);
    S.emit(pop, ppp);
    uint32_t npar = 0;
    const ParRec *prr = xchg<ParRec>(S, knownB, pop.out, ppp, pfrom, SL_PR, &npar);
    local_roots(prr, npar);
    if (m) {
      k_expect1<<<1, 64, 0, st>>>(lrank + m, (uint32_t)R[me], F, RETRY_EXPECT);
      S.launched("k_expect1");
    }
    // cross-slice links: request rounds, the first sized by the links the Y
    // owners and the X lead-in counted, each later one by the last GD message
    uint64_t rq_send[MAXP] = {}, rq_recv[MAXP] = {};
    for (uint32_t q = 0; q < P; ++q) {
      rq_send[q] = Lm[(size_t)me * P + q];
      rq_recv[q] = Lm[(size_t)q * P + me];
    }
    if (links && m) {
      kt_begin(st, KID_SHARD_AUX);
      k_init_labels<<<grid_for(m, 256), 256, 0, st>>>(lpar, ext, lrank, (uint32_t)goff, m, lab,
                                                      cur);
      kt_end(st, KID_SHARD_AUX, 0.0);
      S.launched("k_init_labels");
    }
    PartPlan rpp;
    bool planned = false;  // rpp already planned on the device (a later round)
    for (uint32_t round = 0;; ++round) {
      if (round > 64) {
        ctx->err = "cross-slice root resolution did not converge";
        throw RK_E_INTERNAL;
      }
      if (links) {
        ++ss.root_rounds;
        ReqOp rq{lpar, lab, cur, slices, nullptr, nullptr};
        if (!planned) S.plan_counts(rq, m, rpp, rq_send);
        rq.req = S.take<uint32_t>(SL_REQ, rpp.total + 1);
        rq.src = S.take<uint32_t>(SL_SRC, rpp.total + 1);
        S.emit(rq, rpp);
        uint32_t nq = 0;
        const uint32_t *rqs = xchg<uint32_t>(S, knownC, rq.req, rpp, rq_recv, SL_RQ, &nq);
        uint2 *resp = nullptr, *back = nullptr;
        int rrc = RK_OK;
        try {
          resp = S.take<uint2>(SL_RESP, nq + 1);
          back = S.take<uint2>(SL_BACK, rpp.total + 1);
          if (fault_here(ctx, "k_respond")) throw (int)RK_E_NOMEM;
          if (nq) {
            k_respond<<<grid_for(nq, 256), 256, 0, st>>>(rqs, nq, poff, m, lpar, lab, cur, resp,
                                                          S.ctrl);
            S.launched("k_respond");
          }
        } catch (int code) {
          rrc = code;
        }
        if (!knownC) {
          S.agree(rrc);  // the response buffers were sized by skewed counts
        } else if (rrc) {
          S.sticky = rrc;  // (no agreement point here: reported by the next gather)
          ctx->err = "a local failure before the response exchange";
        }
        uint64_t sb[MAXP], rb[MAXP];
        for (uint32_t q = 0; q < P; ++q) sb[q] = rq_recv[q] * sizeof(uint2), rb[q] = rpp.cnt[q] * sizeof(uint2);
        S.run_a2a(resp, sb, back, rb);
        if (rpp.total) {
          k_apply<<<grid_for((uint32_t)rpp.total, 256), 256, 0, st>>>(back, rq.src,
                                                                      (uint32_t)rpp.total, lab, cur);
          S.launched("k_apply");
        }
      }
      // GD: the next round's request counts, the jumping flag, the gid histogram
      uint32_t *gd = reinterpret_cast<uint32_t *>(S.msg_begin(GW_END + 256 + NBINS * 4));
      uint32_t *gd_tot = gd + GW_END / 4, *gd_hist = gd + (GW_END + 256) / 4;
      if (links) {
        ReqOp rq{lpar, lab, cur, slices, nullptr, nullptr};
        plan_to_msg(S, rq, m, rpp, gd_tot);
        if (m) {
          k_final_gid_spec<<<grid_for(m, 256), 256, 0, st>>>(lpar, lab, m, gid_own);
          S.launched("k_final_gid_spec");
        }
      } else if (m) {
        kt_begin(st, KID_SHARD_AUX);
        k_final_gid_local<<<grid_for(m, 256), 256, 0, st>>>(lpar, lrank, (uint32_t)goff, m,
                                                            gid_own);
        kt_end(st, KID_SHARD_AUX, 12.0 * m);
        S.launched("k_final_gid_local");
      }
      if (m) {
        k_hist<<<grid_for(m, 256, 512), 256, 0, st>>>(mop, m, gd_hist);
        S.launched("k_hist");
      }
      k_msg_head<<<1, 64, 0, st>>>(S.ctrl, gd);
      S.launched("k_msg_head");
      if (S.msg_gather(S.sticky)) throw S.sticky ? S.sticky : (int)RK_E_PEER;
      uint32_t anyerr3 = 0, jflag = 0, rflag = 0;
      bool more = false;
      std::vector<uint64_t> C((size_t)P * P, 0);
      for (uint32_t q = 0; q < P; ++q) {
        const uint32_t *w = reinterpret_cast<const uint32_t *>(S.msg_of(q));
        anyerr3 |= w[0];
        jflag |= w[3];
        rflag |= w[8];
        if (links) {
          const uint32_t *t = w + GW_END / 4;
          for (uint32_t d = 0; d < P; ++d) {
            C[(size_t)q * P + d] = t[d + 1] - t[d];
            more |= C[(size_t)q * P + d] != 0;
          }
        }
        fp = hbytes(fp, w, GW_END + 256);
      }
      if (jflag || rflag) return RK_SHARD_RETRY;  // a chain longer than two jumping rounds
      S.check(err_status(ctx, anyerr3 & ~(uint32_t)ERRB_WIDE_LENGTH));
      if (!more) {  // every label is final: the histogram stands
        ghist_all.resize((size_t)P * NBINS);
        for (uint32_t q = 0; q < P; ++q) {
          std::memcpy(&ghist_all[(size_t)q * NBINS], S.msg_of(q) + GW_END + 256, NBINS * 4);
          fp = hbytes(fp, &ghist_all[(size_t)q * NBINS], NBINS * 4);
        }
      }
      if (round + 2 < 8) {
        new_fp[2 + round] = fp;
        knownC = knownC && fp_known(2 + round, fp);
      } else {
        knownC = false;
      }
      S.alloc_locked = knownC;
      if (!more) break;
      for (uint32_t q = 0; q < P; ++q) {
        rq_send[q] = C[(size_t)me * P + q];
        rq_recv[q] = C[(size_t)q * P + me];
      }
      uint64_t tot = 0;
      for (uint32_t q = 0; q < MAXP; ++q) {
        rpp.cnt[q] = q < P ? rq_send[q] : 0;
        tot += rpp.cnt[q];
      }
      rpp.total = tot;
      rpp.cap = (uint32_t)tot;
      planned = true;
    }
  } else {
    // one rank: gid = the root's rank (every chain ends in the slice)
    if (m) {
      kt_begin(st, KID_SHARD_AUX);
      k_final_gid_local<<<grid_for(m, 256), 256, 0, st>>>(lpar, lrank, 0u, m, gid_own);
      kt_end(st, KID_SHARD_AUX, 12.0 * m);
      S.launched("k_final_gid_local");
    }
  }
  S.alloc_locked = knownC;
  ss.fast_stages |= knownC ? 4u : 0u;
  ss.ms_roots = ms_since(tphase);

  // ---- 9: members -> gid-range owners; exact in-group order; emit -----------------
  tphase = std::chrono::steady_clock::now();
  Bounds gb{};
  std::vector<uint64_t> mr_all(P, 0);
  uint64_t msend[MAXP] = {}, mfrom[MAXP] = {};
  if (P > 1) {
    std::vector<uint64_t> gsum(NBINS, 0);
    for (uint32_t q = 0; q < P; ++q)
      for (uint32_t b = 0; b < NBINS; ++b) gsum[b] += ghist_all[(size_t)q * NBINS + b];
    gb = split_bounds(gsum, gshift, Gtot, P);
    for (uint32_t q = 0; q < P; ++q) {
      msend[q] = bins_in(&ghist_all[(size_t)me * NBINS], gb, q, gshift);
      mfrom[q] = bins_in(&ghist_all[(size_t)q * NBINS], gb, me, gshift);
      for (uint32_t r = 0; r < P; ++r) mr_all[r] += bins_in(&ghist_all[(size_t)q * NBINS], gb, r, gshift);
    }
  } else {
    gb.P = 1;
    gb.b[0] = 0;
    for (uint32_t q = 1; q <= MAXP; ++q) gb.b[q] = Gtot;
    mr_all[0] = m;
  }
  for (uint32_t r = 0; r < P; ++r)
    if (mr_all[r] >= (1ull << 30)) {
      ctx->err = "a gid range of 2^30 or more members";
      throw RK_E_TOO_MANY;
    }
  mop.B = gb;
  const size_t esz = narrow ? 12 : 16;
  const bool m_self = P == 1;  // one rank, no halo: the X chunk's member arrays are the rows
  uint32_t mr = 0;
  const void *mem = nullptr;
  if (m_self) {
    mr = m;
  } else {
    PartPlan mpp;
    S.plan_counts(mop, m, mpp, msend);
    mop.out = S.take<uint8_t>(SN_SMEM, (mpp.total + 1) * esz);
    S.emit(mop, mpp);
    mem = narrow ? (const void *)xchg<uint3>(S, knownC, mop.out, mpp, mfrom, SL_MEM, &mr)
                 : (const void *)xchg<uint4>(S, knownC, mop.out, mpp, mfrom, SL_MEM, &mr);
  }
  const uint32_t g0 = (uint32_t)gb.b[me], Gl = (uint32_t)(gb.b[me + 1] - gb.b[me]);
  uint32_t *ogid = S.take<uint32_t>(SL_OGID, mr + 1);
  uint8_t *orep = S.take<uint8_t>(SL_OREP, mr + 1);
  uint32_t *oord = S.take<uint32_t>(SL_OORD, mr + 1);
  uint32_t *sgid = nullptr, *mrow = nullptr, *otag = nullptr, *goffs = nullptr, *tag = nullptr;
  uint64_t *reckey = nullptr;
  void *gsort = nullptr;
  if (mr) {
    const NwDigits ed = nw_plan(bit_length(Gl ? Gl - 1 : 0), narrow ? 9 : 8);
    sgid = S.take<uint32_t>(SN_SGID, mr + 1);
    mrow = S.take<uint32_t>(SN_MROW, mr + 1);
    reckey = S.take<uint64_t>(SN_KEY, mr + 1);
    tag = S.take<uint32_t>(SN_TAG, mr + 1);
    otag = S.take<uint32_t>(SL_OTAG, mr + 1);
    goffs = S.take<uint32_t>(SN_GOFF, (size_t)Gl + 2);
    uint4 *t0 = S.take<uint4>(SN_T0, mr + 1), *t1 = S.take<uint4>(SN_T1, mr + 1);
    uint32_t *mstat = S.take<uint32_t>(SN_STAT, nw_status_words(mr + 1));
    gsort = S.take<uint8_t>(SL_GSORT, groupsort_scratch_bytes(mr));
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
    // the group-sort tiers on both streams; the depth-limit heap segments
    // (crafted inputs only) are counted into F[5] and sorted after GE
    (void)sort_groups_exact(sgid, goffs, Gl, mr, reckey, tag, otag, gsort,
                            S.scan_scratch(SL_SCAN, mr + Gl + 2), ctx->host + 128, narrow, st,
                            st2 != st ? st2 : nullptr, ctx->fork, ctx->join, F + 5);
    emit_result(otag, sgid, goffs, mrow, mr, ogid, orep, oord, st);
    if (g0) k_add_u32<<<grid_for(mr, 256), 256, 0, st>>>(ogid, mr, g0);
    S.launched("member order");
  }
  S.alloc_locked = false;

  // ---- GE: the error bits and the heap segments ---------------------------------
  uint32_t *ge = reinterpret_cast<uint32_t *>(S.msg_begin(GW_END));
  k_msg_head<<<1, 64, 0, st>>>(S.ctrl, ge);
  S.launched("k_msg_head");
  if (S.msg_gather(S.sticky)) throw S.sticky ? S.sticky : (int)RK_E_PEER;
  uint32_t anyerr4 = 0, heap_me = 0, retry4 = 0;
  bool heap_any = false;
  for (uint32_t q = 0; q < P; ++q) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(S.msg_of(q));
    anyerr4 |= w[0];
    retry4 |= w[8];  // a member plan whose device counts disagreed
    heap_any |= w[8 + 5] != 0;
    if (q == me) heap_me = w[8 + 5];
  }
  if (retry4) return RK_SHARD_RETRY;
  S.check(err_status(ctx, anyerr4 & ~(uint32_t)ERRB_WIDE_LENGTH));
  int hrc = RK_OK;
  if (heap_me && mr) {  // sorted now, then the result again
    hrc = sort_groups_heap_deferred(Gl, mr, reckey, tag, otag, gsort, heap_me, ctx->host + 128, st);
    if (!hrc) {
      emit_result(otag, sgid, goffs, mrow, mr, ogid, orep, oord, st);
      if (g0) k_add_u32<<<grid_for(mr, 256), 256, 0, st>>>(ogid, mr, g0);
      if (hipGetLastError() != hipSuccess) hrc = RK_E_HIP;
    } else {
      ctx->err = "depth-limit heap segments: buffer allocation failed";
    }
  }
  if (heap_any) {  // every rank agrees on the heap segments' outcome
    if (!hrc && hipStreamSynchronize(st) != hipSuccess) hrc = RK_E_HIP;
    S.agree(hrc);
    S.agree_errors();
  }
  ss.ms_members = ms_since(tphase);
  uint64_t ooff = 0, otot = 0;
  for (uint32_t q = 0; q < P; ++q) otot += mr_all[q], ooff += q < me ? mr_all[q] : 0;
  out->out_order = oord;
  out->gid = ogid;
  out->repval = orep;
  out->n_out = mr;
  out->out_offset = ooff;
  out->n_out_total = otot;
  out->n_groups = Gtot;
  for (int k = 0; k < 8; ++k) ctx->sh_fp[k] = new_fp[k];
  return RK_OK;
}
