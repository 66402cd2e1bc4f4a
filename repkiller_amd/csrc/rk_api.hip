// rk_api.hip -- C ABI (include/repkiller_amd.h) and the device pipeline driver.
//
// One rk_ctx = one device + two HIP streams + one grow-only workspace in HBM,
// mirroring the reference's one-private-state-per-worker model
// (repkiller.cpp:60-72).  rk_classify_device runs, on the context stream
// (the Y-axis sort and the in-group sort keys on the second stream, overlapped
// with the X sweeps):
//
//   1 prep_keys        xStart/10 keys, last-bucket drop, probe validation
//   2 counting_sort    -> processing order (stable bucket order of FragmentsDatabase)
//   3 gather_proc      processing-order SoA + 100-bp bucket keys + sort key
//   4 counting_sort x2 -> X and Y occupancy CSRs (SequenceOcupationList buckets)
//   5 sweeps on X, then Y (rk_occupancy.hip) until every fragment is decided;
//     X decisions write X hits' parents and every X result (into the Y
//     records) as they are made; X misses get their parent from the Y sweeps
//   6 pointer jumping -> new-group rank (DPP scan) -> gid
//   7 counting_sort    -> group member lists in processing order
//   8 sort_groups      libstdc++ introsort per group; 9 emit flags / order
//
// Host synchronisation happens only where a data-dependent count decides the
// next launch (kept rows, work-list sizes, jump convergence, group count).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rk_ctx.h"

namespace rk {
const char *const kKernelNames[KID_COUNT] = {
    "k_prep_keys",     "k_digit_hist",      "k_digit_scatter", "k_gather_proc",
    "k_sort_keys",     "k_csr_fill_x",      "k_run_bounds",    "k_sweep_tile",
    "k_sweep_fast",    "k_sweep_fast_more", "k_sweep_wave",    "k_csr_fill_y",    "k_jump",
    "k_assign_gid",    "k_group_offsets",   "k_build_records",
    "k_sort_small",    "k_sort_groups_reg", "k_sort_groups_lds", "k_sort_groups_split",
    "k_emit",          "k_part (sharded)", "exchange (sharded)", "k_aux (sharded)",
    "k_row_keys (sharded)", "k_fill_y (sharded)", "k_y_results (sharded)", "k_x_own (sharded)",
    "k_merge_yx (sharded)", "k_sort_segments", "k_sweep_long32", "k_nw_order_hist",
    "k_onesweep", "k_nw_xchunk", "k_nw_fill_y", "k_nw_assign", "k_nw_xcount", "k_nw_x_bits",
    "k_heap_segments", "k_seg_fine (order)", "k_seg_fine (members)", "k_seg_fine (Y)",
};
}  // namespace rk

namespace rk {

void collect_kernel_timing(rk_ctx *ctx) {
  g_ktimer = nullptr;
  if (ctx->kt.n) (void)hipEventSynchronize(ctx->kt.ev[2 * ctx->kt.n - 1]);
  if (ctx->kt.tier_counts) {  // the group-sort tiers' algorithmic bytes
    const uint32_t nb = ctx->kt.tier_nblk;
    std::vector<uint32_t> h((size_t)KernelTimer::TIERS * nb);
    if (hipMemcpy(h.data(), ctx->kt.tier_counts, (size_t)GS_NTIER * nb * 4,
                  hipMemcpyDeviceToHost) == hipSuccess) {
      for (int u = 0; u < GS_NTIER; ++u) {
        double mem = 0;
        for (uint32_t b = 0; b < nb; ++b) mem += h[(size_t)u * nb + b];
        const int sl = ctx->kt.tier_slot[u];
        if (sl >= 0 && sl < ctx->kt.n) ctx->kt.bytes[sl] = 12.0 * mem;
        const int s2 = u == GS_NTIER - 1 ? ctx->kt.tier_slot[GS_NTIER] : -1;  // phase B
        if (s2 >= 0 && s2 < ctx->kt.n) ctx->kt.bytes[s2] = 12.0 * mem;
      }
    }
    ctx->kt.tier_counts = nullptr;
  }
  bool any_units = false;
  for (int i = 0; i < ctx->kt.n; ++i) any_units |= ctx->kt.unit_bytes[i] > 0.0;
  if (any_units) {  // launches that counted their work on the device
    std::vector<uint32_t> u(ctx->kt.n);
    if (hipMemcpy(u.data(), ctx->kt.units, (size_t)ctx->kt.n * 4, hipMemcpyDeviceToHost) ==
        hipSuccess)
      for (int i = 0; i < ctx->kt.n; ++i)
        if (ctx->kt.unit_bytes[i] > 0.0) ctx->kt.bytes[i] = ctx->kt.unit_bytes[i] * u[i];
  }
  for (int i = 0; i < ctx->kt.n; ++i) {
    float ms = 0;
    if (hipEventElapsedTime(&ms, ctx->kt.ev[2 * i], ctx->kt.ev[2 * i + 1]) == hipSuccess) {
      const int k = ctx->kt.kid[i];
      ctx->kt_ms[k] += ms;
      ctx->kt_bytes[k] += ctx->kt.bytes[i];
      ctx->kt_launches[k]++;
    }
  }
  ctx->kt.n = 0;
}

int readback(rk_ctx *ctx, const uint32_t *dev, uint32_t count) {
  ++ctx->readbacks;
  HIPCHK(ctx, hipMemcpyAsync(ctx->host, dev, count * sizeof(uint32_t), hipMemcpyDeviceToHost,
                             ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return RK_OK;
}

int err_status(rk_ctx *ctx, uint32_t bits) {
  if (bits & ERRB_UB_BUCKET) {
    ctx->err = "xStart/10 >= vsize: the reference indexes FragmentsDatabase out of bounds "
               "(FragmentsDatabase.cpp:96-97)";
    return RK_E_UB_BUCKET;
  }
  if (bits & ERRB_UB_CENTER) {
    ctx->err = "a fragment centre probes past an occupancy array "
               "(SequenceOcupationList.cpp:17,80)";
    return RK_E_UB_CENTER;
  }
  if (bits & ERRB_INTERNAL) {
    ctx->err = "device consistency check failed";
    return RK_E_INTERNAL;
  }
  return RK_OK;
}

// run sweeps on one axis until no bucket has undecided entries
int resolve_axis(rk_ctx *ctx, const Axis &ax, SweepScratch sc, bool fast32, uint32_t *sweeps) {
  uint32_t *counters = sc.counters;
  uint8_t *rpend = sc.rpend;
  RunList rl{sc.runs, sc.wpend, 0, 0, fast32};
  build_runs(ax, rl, sc.dev_count, ctx->host + 128, ctx->stream);
  HIPCHK(ctx, hipGetLastError());
  // the 32-bit path's first sweep sets the open flag of every long run itself
  if (!fast32) HIPCHK(ctx, hipMemsetAsync(rpend, 1, ax.m, ctx->stream));
  *sweeps = 0;
  for (;;) {
    if (*sweeps > ax.m + 2) {
      ctx->err = "occupancy sweeps did not converge";
      return RK_E_INTERNAL;
    }
    occupancy_sweep(ax, rl, rpend, counters, *sweeps == 0, ctx->stream);
    HIPCHK(ctx, hipGetLastError());
    ++*sweeps;
    // the first sweep practically never finishes an axis: the next ones (up to
    // RK_SWEEP_BLIND sweeps in all, default 3) are queued without a host round
    // trip (on a finished axis a sweep only reads the window flags).  cfg3's X
    // axis takes 3 sweeps, its Y axis 2: 3 queued saves the X axis' first
    // readback (sweep_x phase 1.246 -> 1.226 ms; the Y axis' extra sweep reads
    // flags only)
    static const uint32_t blind = [] {
      const char *e = getenv("RK_SWEEP_BLIND");
      const int v = e ? atoi(e) : 3;
      return (uint32_t)(v < 1 ? 1 : v > 8 ? 8 : v);
    }();
    if (*sweeps < blind && ax.m > 0) continue;
    int rc = readback(ctx, counters, PEND_WORDS);
    if (rc) return rc;
    uint64_t pending = 0;
    for (uint32_t k = 0; k < PEND_WORDS; ++k) pending += ctx->host[k];
    if (!pending) break;
  }
  return RK_OK;
}

__global__ void k_pend_flag(const uint32_t *counters, uint32_t *pend) {
  uint32_t s = 0;
  for (uint32_t k = threadIdx.x; k < PEND_WORDS; k += 64) s |= counters[k];
  if (__ballot(s != 0) && threadIdx.x == 0) *pend = 1u;
}

// `sweeps` sweeps of a 32-bit axis queued without a host round trip, then the
// pending count folded into *pend (left alone when the axis is final): the
// sharded driver's fast path reads it with its next all-gather and repeats the
// call the careful way if any axis was left open
int resolve_axis_queued(rk_ctx *ctx, const Axis &ax, SweepScratch sc, uint32_t sweeps,
                        uint32_t *pend, uint32_t *junk) {
  if (!ax.m) return RK_OK;
  RunList rl{sc.runs, sc.wpend, 0, 0, true};
  build_runs(ax, rl, sc.dev_count, ctx->host + 128, ctx->stream);  // (32-bit: no readback)
  // junk: the sweeps before the last count into words nobody reads, and the
  // last one into sc.counters, already zero (no clear launched per sweep)
  for (uint32_t s = 0; s < sweeps; ++s)
    occupancy_sweep(ax, rl, sc.rpend, junk && s + 1 < sweeps ? junk : sc.counters, s == 0,
                    ctx->stream, !junk);
  if (pend) k_pend_flag<<<1, 64, 0, ctx->stream>>>(sc.counters, pend);
  HIPCHK(ctx, hipGetLastError());
  return RK_OK;
}

}  // namespace rk

static const char *kPhaseNames[RK_N_PHASES] = {
    "prep_keys",      "order_csr",  "gather_proc", "occupancy_csr", "sweep_x", "sweep_y",
    "group_roots",    "member_csr", "group_sort",  "emit",
};

namespace {

using rk::align_up;
using rk::Carve;
using rk::readback;
using rk::err_status;

struct Plan {
  uint64_t n, vsize, max_x, max_y;
  uint32_t nbx, nby;
};

struct Work {
  uint32_t *ctrl;  // [0] err bits, [1] kept rows, [2..7] counters
  uint32_t *pkey_in, *tk, *tv, *tk2, *tv2;
  uint32_t *radix, *radix2;
  size_t radix_words;
  rk::Proc p;
  rk::Csr cx, cy;
  uint32_t *isnew, *newrank, *sgid, *gmem, *goff, *tag, *otag;
  void *gsort;
  uint64_t *reckey;
  uint32_t *rpend, *runs, *rlen_at, *rbeg_at;
  uint8_t *wpend;
  uint32_t *scan;
  size_t scan_cap;
};

size_t carve(Carve &c, const Plan &pl, Work &w) {
  const size_t n = pl.n + 1;
  w.ctrl = c.take<uint32_t>(64 + rk::PEND_WORDS);
  w.pkey_in = c.take<uint32_t>(n);
  w.tk = c.take<uint32_t>(n);
  w.tv = c.take<uint32_t>(n);
  w.tk2 = c.take<uint32_t>(n);
  w.tv2 = c.take<uint32_t>(n);
  w.radix_words = rk::radix_scratch_words((uint32_t)n);
  w.radix = c.take<uint32_t>(w.radix_words);
  w.radix2 = c.take<uint32_t>(w.radix_words);
  // the file-order records are dead once gather_proc has read them: the
  // in-group sort keys and the member stage's arrays reuse their 32 B / entry
  w.p.rec = c.take<ulonglong2>(2 * n + 64);
  {
    char *r = reinterpret_cast<char *>(w.p.rec);
    const size_t o1 = rk::align_up(16 * n + 64), o2 = o1 + rk::align_up(8 * n + 64),
                 o3 = o2 + rk::align_up(4 * n + 64);  // + slack, like every take()
    w.p.hrec = reinterpret_cast<ulonglong2 *>(r);
    w.reckey = reinterpret_cast<uint64_t *>(r + o1);
    w.tag = reinterpret_cast<uint32_t *>(r + o2);
    w.otag = reinterpret_cast<uint32_t *>(r + o3);
  }
  w.p.ys = c.take<uint64_t>(n);
  w.p.pkey = c.take<uint32_t>(n);
  w.p.row = c.take<uint32_t>(n);
  w.p.xrec = c.take<ulonglong2>(n);
  w.p.yrec = c.take<ulonglong2>(n);
  w.p.ylenhi = nullptr;  // 64-bit lengths only: ensure_wide
  w.p.keyx = c.take<uint32_t>(n);
  w.p.keyy = c.take<uint32_t>(n);
  w.p.par = c.take<uint32_t>(n);
  w.p.gid = c.take<uint32_t>(n);
  w.p.grow = nullptr;  // the sharded driver's global rows; unused here
  for (rk::Csr *cs : {&w.cx, &w.cy}) {
    cs->key = c.take<uint32_t>(n);
    cs->ent = c.take<uint32_t>(n);
    cs->cen = cs->len = nullptr;  // 64-bit lengths only: ensure_wide
    cs->state = c.take<uint8_t>(n);
    cs->pk = c.take<uint2>(n);
    cs->nbd = c.take<uint8_t>(n);
  }
  w.isnew = c.take<uint32_t>(n);
  w.newrank = c.take<uint32_t>(n);
  w.sgid = c.take<uint32_t>(n);
  w.gmem = c.take<uint32_t>(n);
  w.goff = c.take<uint32_t>(n);
  w.gsort = c.take<uint8_t>(rk::groupsort_scratch_bytes((uint32_t)n));
  w.rpend = c.take<uint32_t>(n / 4 + 1);
  w.wpend = c.take<uint8_t>(n / 64 + 1);
  w.runs = c.take<uint32_t>(rk::runs_scratch_words((uint32_t)n));
  w.rlen_at = c.take<uint32_t>(n);
  w.rbeg_at = c.take<uint32_t>(n);
  w.scan_cap = rk::scan_blocks(n + 1) + 64;
  w.scan = c.take<uint32_t>(w.scan_cap);
  return c.off;
}

int ensure_ws(rk_ctx *ctx, const Plan &pl, Work &w) {
  Carve probe{nullptr};
  size_t need = carve(probe, pl, w);
  if (need > ctx->ws_cap) {
    if (ctx->ws) (void)hipFree(ctx->ws);
    ctx->ws = nullptr;
    ctx->ws_cap = 0;
    hipError_t e = hipMalloc(&ctx->ws, need);
    if (e != hipSuccess) {
      ctx->err = std::string("workspace hipMalloc(") + std::to_string(need) + "): " +
                 hipGetErrorString(e);
      return e == hipErrorOutOfMemory ? RK_E_NOMEM : RK_E_HIP;
    }
    ctx->ws_cap = need;
  }
  Carve real{(char *)ctx->ws};
  carve(real, pl, w);
  return RK_OK;
}

rk::SweepScratch sweep_scratch(const Work &w) {
  return rk::SweepScratch{w.runs, w.wpend, reinterpret_cast<uint8_t *>(w.rpend), w.ctrl + 64,
                          w.ctrl + 2};
}

// The 64-bit centre/length copies of both axes and the Y lengths' high words,
// needed only when some length is >= 2^31 (the generic sweep kernel): a
// second grow-only buffer, so the common case does not carry 36 B per entry.
int ensure_wide(rk_ctx *ctx, size_t n1, Work &w) {
  const size_t n = n1 + 1;
  auto carve_wide = [&](Carve &c) {
    w.p.ylenhi = c.take<uint32_t>(n);
    w.cx.cen = c.take<uint64_t>(n);
    w.cx.len = c.take<uint64_t>(n);
    w.cy.cen = c.take<uint64_t>(n);
    w.cy.len = c.take<uint64_t>(n);
  };
  Carve probe{nullptr};
  carve_wide(probe);
  const size_t need = probe.off;  // with take()'s slack
  if (need > ctx->ws_wide_cap) {
    if (ctx->ws_wide) (void)hipFree(ctx->ws_wide);
    ctx->ws_wide = nullptr;
    ctx->ws_wide_cap = 0;
    hipError_t e = hipMalloc(&ctx->ws_wide, need);
    if (e != hipSuccess) {
      ctx->err = std::string("64-bit workspace hipMalloc: ") + hipGetErrorString(e);
      return e == hipErrorOutOfMemory ? RK_E_NOMEM : RK_E_HIP;
    }
    ctx->ws_wide_cap = need;
  }
  Carve c{(char *)ctx->ws_wide};
  carve_wide(c);
  return RK_OK;
}

// mark the START of phase `ph` (ph == RK_N_PHASES marks the end of the last)
void mark(rk_ctx *ctx, int ph) {
  if (!ctx->profiling) return;
  if (ph == RK_PH_PREP) {
    ctx->kt.n = 0;
    rk::g_ktimer = &ctx->kt;
  }
  (void)hipEventRecord(ctx->pev[ph], ctx->stream);
  ctx->pev_used[ph] = true;
}

void collect_phases(rk_ctx *ctx) {
  if (!ctx->profiling) return;
  rk::collect_kernel_timing(ctx);
  (void)hipEventSynchronize(ctx->pev[RK_N_PHASES]);
  for (int ph = 0; ph < RK_N_PHASES; ++ph) {
    if (!ctx->pev_used[ph]) continue;
    int nx = ph + 1;
    while (nx <= RK_N_PHASES && !ctx->pev_used[nx]) ++nx;
    if (nx > RK_N_PHASES) break;
    float ms = 0;
    if (hipEventElapsedTime(&ms, ctx->pev[ph], ctx->pev[nx]) == hipSuccess) {
      ctx->phase_ms[ph] += ms;
      ctx->phase_calls[ph]++;
    }
  }
  for (auto &u : ctx->pev_used) u = false;
}

// ---------------------------------------------------------------------------
// The record pipeline (rk_narrow.hip): used when every row packs into a
// 16-B record; returns with *fallback set when the input turns out not to (a
// length >= 2^24 or a yStart >= 2^35, found by the upfront pass before the
// workspace is sized; n >= 2^30 never gets here) -- the generic pipeline then
// classifies from scratch.
struct NWork {
  uint32_t *ctrl, *ahist, *yhist, *ehist;
  uint32_t *astatus, *ystatus, *xcnt, *xoff;
  uint4 *Ra, *Rb, *yrec, *erec;
  rk::Csr cx, cy;
  uint32_t *xpos, *xbits;
  uint32_t *par, *isnew, *newrank, *sgid, *tag, *otag, *mrow, *goff;
  uint64_t *reckey;
  void *gsort;
  uint32_t *rpend, *runs, *rlen_at, *rbeg_at;
  uint8_t *wpend;
  uint32_t *scan;
  size_t scan_cap;
  uint32_t *chist, *coff;  // the two-stage order sort's segment counts and starts
};

size_t carve_nw(Carve &c, uint64_t n1, uint32_t nbx, NWork &w) {
  const size_t n = n1 + 1;
  const size_t sw = rk::nw_status_words((uint32_t)n);
  w.astatus = c.take<uint32_t>(sw);
  w.ystatus = c.take<uint32_t>(sw);
  // X-chunk counts and their scan (chunks of >= 64 buckets)
  w.xcnt = c.take<uint32_t>((size_t)3 * (nbx / 64 + 2) + 64);
  w.xoff = c.take<uint32_t>((size_t)3 * (nbx / 64 + 2) + 64);
  w.Ra = c.take<uint4>(n);
  w.Rb = c.take<uint4>(n);
  w.yrec = c.take<uint4>(n);
  w.erec = c.take<uint4>(n);
  for (rk::Csr *cs : {&w.cx, &w.cy}) {
    cs->key = c.take<uint32_t>(n);
    cs->ent = c.take<uint32_t>(n);
    cs->cen = cs->len = nullptr;
    cs->state = c.take<uint8_t>(n);
    cs->pk = c.take<uint2>(n);
    cs->nbd = c.take<uint8_t>(n);
  }
  w.xpos = c.take<uint32_t>(n);
  w.xbits = c.take<uint32_t>(n / 32 + 2);
  w.par = c.take<uint32_t>(n);
  w.isnew = c.take<uint32_t>(n);
  w.newrank = c.take<uint32_t>(n);
  w.sgid = c.take<uint32_t>(n);
  w.tag = c.take<uint32_t>(n);
  w.otag = c.take<uint32_t>(n);
  w.mrow = c.take<uint32_t>(n);
  w.goff = c.take<uint32_t>(n);
  w.reckey = c.take<uint64_t>(n);
  w.gsort = c.take<uint8_t>(rk::groupsort_scratch_bytes((uint32_t)n));
  w.rpend = c.take<uint32_t>(n / 4 + 1);
  w.wpend = c.take<uint8_t>(n / 64 + 1);
  w.runs = c.take<uint32_t>(rk::runs_scratch_words((uint32_t)n));
  w.rlen_at = c.take<uint32_t>(n);
  w.rbeg_at = c.take<uint32_t>(n);
  w.scan_cap = rk::scan_blocks(n + 1) + 64;
  w.scan = c.take<uint32_t>(w.scan_cap);
  // the two-stage order sort's segment counts and starts (<= n / 1536 + 1 each)
  w.chist = c.take<uint32_t>(rk::nw_seg_words(n));
  w.coff = c.take<uint32_t>(rk::nw_seg_words(n));
  return c.off;
}

// control words and digit histograms (ctrl, ahist / yhist / ehist), size
// independent of n: the upfront pass that decides whether every row packs
// writes only these, so an input that falls back never sizes the workspace
// ctrl: 64 words, the X and the Y axis' pending counters (zeroed with the
// words), a third counter block the earlier queued sweeps count into (never
// read), then the order / Y / member histograms
constexpr size_t NW_CTRL_WORDS = 64 + 3 * rk::PEND_WORDS;
constexpr size_t NW_SMALL_WORDS = NW_CTRL_WORDS + 3 * 4096;

int ensure_nw_small(rk_ctx *ctx, NWork &w) {
  if (!ctx->nw_small) {
    const hipError_t e = hipMalloc(&ctx->nw_small, NW_SMALL_WORDS * sizeof(uint32_t));
    if (e != hipSuccess) {
      ctx->nw_small = nullptr;
      ctx->err = std::string("record-pipeline control hipMalloc: ") + hipGetErrorString(e);
      return e == hipErrorOutOfMemory ? RK_E_NOMEM : RK_E_HIP;
    }
  }
  w.ctrl = static_cast<uint32_t *>(ctx->nw_small);
  w.ahist = w.ctrl + NW_CTRL_WORDS;
  w.yhist = w.ahist + 4096;
  w.ehist = w.ahist + 8192;
  return RK_OK;
}

int ensure_nw(rk_ctx *ctx, uint64_t n, uint32_t nbx, NWork &w) {
  Carve probe{nullptr};
  const size_t need = carve_nw(probe, n, nbx, w);
  if (need > ctx->ws_nw_cap) {
    if (ctx->ws_nw) (void)hipFree(ctx->ws_nw);
    ctx->ws_nw = nullptr;
    ctx->ws_nw_cap = 0;
    hipError_t e = hipMalloc(&ctx->ws_nw, need);
    if (e == hipErrorOutOfMemory && (ctx->ws || ctx->ws_wide)) {
      // the generic pipeline's buffers (a previous fallback) give way
      (void)hipGetLastError();
      if (ctx->ws) (void)hipFree(ctx->ws);
      if (ctx->ws_wide) (void)hipFree(ctx->ws_wide);
      ctx->ws = ctx->ws_wide = nullptr;
      ctx->ws_cap = ctx->ws_wide_cap = 0;
      e = hipMalloc(&ctx->ws_nw, need);
    }
    if (e != hipSuccess) {
      ctx->err = std::string("record-pipeline workspace hipMalloc(") + std::to_string(need) +
                 "): " + hipGetErrorString(e);
      return e == hipErrorOutOfMemory ? RK_E_NOMEM : RK_E_HIP;
    }
    ctx->ws_nw_cap = need;
  }
  Carve real{(char *)ctx->ws_nw};
  carve_nw(real, n, nbx, w);
  return RK_OK;
}

// RK_RECORD_PIPELINE=0 forces the generic pipeline (A/B measurements)
bool record_pipeline_enabled() {
  static const bool on = [] {
    const char *e = std::getenv("RK_RECORD_PIPELINE");
    return !(e && e[0] == '0');
  }();
  return on;
}

int classify_narrow(rk_ctx *ctx, const rk_frags_soa *in, const rk_params *prms, uint32_t npairs,
                    rk_result *outs, const Plan &pl, bool *fallback, const uint3 *wire,
                    bool fused_roots = true) {
  *fallback = false;
  // The roots and gids in one pass after a scan of the parents' root flags
  // (k_nw_assign_jump; RK_ROOTS_FUSED=0: pointer-jumping rounds, each read
  // back, then the flag scan and k_nw_assign).  A chain still open after 4128
  // steps (none in the BASELINE configs) makes the call classify again the
  // round-by-round way.
  static const bool fused_on = [] {
    const char *e = getenv("RK_ROOTS_FUSED");
    return !(e && e[0] == '0');
  }();
  fused_roots = fused_roots && fused_on;
  const uint32_t n = (uint32_t)pl.n;
  NWork w{};
  int rc = ensure_nw_small(ctx, w);
  if (rc) return rc;
  hipStream_t st = ctx->stream, st2 = ctx->stream2;
  ctx->stats.n_in = n;
  const rk::NwDigits ad = rk::nw_plan(rk::bit_length(pl.vsize - 1));
  // the processing order in two stages (coarse one-sweep passes + the segment
  // kernel) when the rows are many enough; else LSD passes over every bit
  const rk::NwOrderPlan op = rk::nw_order_split(n, pl.vsize, rk::bit_length(pl.vsize - 1));
  const bool split = op.coarse.passes > 0;
  // the widest digit of the 12-B record sorts (Y axis, narrow members): 9
  // bits (7168 records per tile: 14 per digit segment) takes cfg3's 26-bit Y
  // key in 3 passes instead of 4 (RK_NW_YBITS=8 for measurements)
  static const int bits12 = [] {
    const char *e = getenv("RK_NW_YBITS");
    const int b = e ? atoi(e) : 9;
    return b < 8 ? 8 : b > 9 ? 9 : b;
  }();
  const rk::NwDigits yd = rk::nw_plan(rk::bit_length(2ull * pl.nby - 1), bits12);
  // The Y sort in two stages too (coarse passes + the segment kernel writing
  // the CSR arrays) -- RK_NW_YSPLIT=0 restores the one-stage passes
  static const bool ysplit_on = [] {
    const char *e = getenv("RK_NW_YSPLIT");
    return !(e && e[0] == '0');
  }();
  static const bool y_overlap = [] {
    const char *e = getenv("RK_Y_OVERLAP");
    return e && e[0] == '1';
  }();
  const rk::NwOrderPlan yp = ysplit_on && !y_overlap
                                 ? rk::nw_order_split(n, 2ull * pl.nby,
                                                      rk::bit_length(2ull * pl.nby - 1))
                                 : rk::NwOrderPlan{};
  const bool ysplit = yp.coarse.passes > 0;

  // The control words (errors, kept rows, pack flag, longest length) come back
  // while the split sort's coarse passes run -- they need only n -- when the
  // workspace is already large enough (a repeated call; the first call
  // allocates it after the pack check, so an input that falls back to the
  // generic pipeline never holds both).  A fallback or an error then leaves
  // the coarse passes' output unused.
  // (not after a call on this context fell back: an input that does not pack
  // would run the coarse passes for nothing and book them to the order phase)
  bool early = false;
  if (split && !ctx->nw_fell_back) {
    Carve probe{nullptr};
    NWork tmpw = w;
    early = carve_nw(probe, pl.n, pl.nbx, tmpw) <= ctx->ws_nw_cap;
  }
  rk::ZeroRegion cr[4] = {};
  if (early) {
    if ((rc = ensure_nw(ctx, pl.n, pl.nbx, w))) return rc;  // (no allocation)
    // what the coarse passes need cleared (the X-chunk counts for the widest
    // chunking, 64 buckets a chunk, among it) joins the call's first clear
    rk::nw_order_coarse_regions(
        (uint32_t)pl.n, op, w.astatus, w.chist,
        rk::ZeroRegion{w.xcnt, ((size_t)3 * (pl.nbx / 64 + 2) + 1) * sizeof(uint32_t)}, cr);
  }
  HIPCHK(ctx, hipEventRecord(ctx->ev0, st));
  // the control words and the order / Y / member digit histograms (ehist stays
  // zero until the first pair's k_nw_assign), one launch
  rk::zero_regions(st, {{w.ctrl, (64 + 2 * rk::PEND_WORDS) * sizeof(uint32_t)},
                        {w.ahist, 3 * 4096 * sizeof(uint32_t)}, cr[0], cr[1], cr[2], cr[3]});
  mark(ctx, RK_PH_PREP);
  rk::nw_order_hist(*in, pl.vsize, pl.max_x, pl.max_y, pl.nby, split ? op.coarse : ad,
                    ysplit ? yp.coarse : yd, w.ahist, w.yhist, w.ctrl, st, wire);
  HIPCHK(ctx, hipGetLastError());
  if (early) {
    HIPCHK(ctx, hipMemcpyAsync(ctx->host, w.ctrl, 9 * sizeof(uint32_t), hipMemcpyDeviceToHost,
                               st));
    HIPCHK(ctx, hipEventRecord(ctx->aux, st));
    mark(ctx, RK_PH_ORDER);
    rk::nw_order_sort_split_coarse(*in, op, w.ahist, w.astatus, w.Ra, w.Rb, w.chist,
                                   rk::ZeroRegion{}, pl.vsize, st, wire, true);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipEventSynchronize(ctx->aux));
  } else if ((rc = readback(ctx, w.ctrl, 9))) {
    return rc;
  }
  if ((rc = err_status(ctx, ctx->host[0]))) return rc;
  if (ctx->host[3]) {  // some row does not pack into a record
    *fallback = true;
    ctx->stats.record_fallback = 1;
    ctx->nw_fell_back = true;
    return RK_OK;
  }
  ctx->nw_fell_back = false;
  // every row packs: now the workspace (~190 B per row)
  if (!early && (rc = ensure_nw(ctx, pl.n, pl.nbx, w))) return rc;
  rk::ScanScratch ss{w.scan, w.scan_cap};
  const uint32_t m = ctx->host[1], maxlen = ctx->host[4];
  ctx->stats.n_proc = m;
  for (uint32_t q = 0; q < npairs; ++q) outs[q].n_out = m, outs[q].n_groups = 0;
  if (m == 0) {
    mark(ctx, RK_N_PHASES);
    collect_phases(ctx);
    HIPCHK(ctx, hipEventRecord(ctx->ev1, st));
    HIPCHK(ctx, hipStreamSynchronize(st));
    return RK_OK;
  }
  // X chunks: entries per (strand, chunk) and owned rows per chunk, counted
  // over the processing order; one scan turns the counts into offsets
  rk::NwChunkCounts cc{};
  cc.W = rk::nw_chunk_width(m, pl.nbx);
  while ((1u << cc.lgW) < cc.W) ++cc.lgW;
  cc.nch = rk::nw_chunks(pl.nbx, cc.W);
  cc.cnts = w.xcnt;
  if (!early) mark(ctx, RK_PH_ORDER);
  if (early) {
    // (the member records' buffer is free until the X chunk kernel)
    rk::nw_order_sort_split_fine((uint32_t)pl.n, m, pl.nby, op, w.Ra, w.Rb, w.yrec, w.erec,
                                 w.chist, w.coff, ss, &cc, st);
  } else if (split) {
    rk::nw_order_sort_split(*in, m, pl.nby, op, w.ahist, w.astatus, w.Ra, w.Rb, w.yrec, w.erec,
                            w.chist, w.coff, ss, &cc, pl.vsize, st, wire);
  } else {
    rk::nw_order_sort(*in, pl.vsize, pl.nby, ad, w.ahist, w.astatus, w.Ra, w.Rb, w.yrec, st, wire);
    rk::nw_x_count(w.Ra, m, cc, st);
  }
  rk::exclusive_scan_u32(w.xcnt, w.xoff, (size_t)3 * cc.nch + 1, ss, st);
  HIPCHK(ctx, hipGetLastError());
  // The Y axis is sorted once X is resolved (default): its first pass reads
  // each record's X-hit bit in processing order and the last writes the Y
  // states from it -- no per-record lookup, and no record pass shares the
  // device with the X sweeps.  RK_Y_OVERLAP=1: the earlier schedule, every Y
  // pass but the last on the second stream beside the X axis, the last one
  // looking up the X-hit bits (cfg3 11.0 ms against 11.2 with those passes
  // serial before X).
  if (y_overlap) {
    HIPCHK(ctx, hipEventRecord(ctx->fork, st));
    HIPCHK(ctx, hipStreamWaitEvent(st2, ctx->fork, 0));
    rk::nw_y_sort_head(w.yrec, w.Rb, m, yd, w.yhist, w.ystatus, st2);
    HIPCHK(ctx, hipEventRecord(ctx->join, st2));
  }
  mark(ctx, RK_PH_GATHER);
  rk::nw_x_chunks(w.Ra, m, pl.nbx, pl.max_x, maxlen, w.xoff, w.cx, w.xpos, w.erec, w.ctrl, cc.W,
                  st);
  HIPCHK(ctx, hipGetLastError());
  mark(ctx, RK_PH_OCC_CSR);
  // pending counters: the X axis' at ctrl[64..), the Y axis' after them (both
  // zero from the call's start), a third block for the queued sweeps before
  // each axis' last (never read)
  rk::SweepScratch sc{w.runs, w.wpend, reinterpret_cast<uint8_t *>(w.rpend), w.ctrl + 64,
                      w.ctrl + 2};
  rk::SweepScratch scy = sc;
  scy.counters = w.ctrl + 64 + rk::PEND_WORDS;
  uint32_t *const junk = w.ctrl + 64 + 2 * rk::PEND_WORDS;
  // Both axes' sweeps are queued without a host round trip (RK_SWEEP_QUEUED=0:
  // the readback after each axis' third sweep); whether either axis was left
  // open comes back with the roots' first readback (the two axes' pending
  // counters; with RK_ROOTS_FUSED=0 a flag per axis in ctrl[10], ctrl[11],
  // which the first jumping round checks), and a pair left open repeats its
  // axes the careful way (no input of the BASELINE configs needs more than
  // three sweeps an axis)
  static const bool queued_on = [] {
    const char *e = getenv("RK_SWEEP_QUEUED");
    return !(e && e[0] == '0');
  }();
  static const uint32_t blind = [] {
    const char *e = getenv("RK_SWEEP_BLIND");
    const int v = e ? atoi(e) : 3;
    return (uint32_t)(v < 1 ? 1 : v > 8 ? 8 : v);
  }();
  for (uint32_t q = 0; q < npairs; ++q) {
    const rk_params &pq = prms[q];
    rk_result *out = &outs[q];
    const bool prof = q == 0;
    uint32_t rounds = 0, G = 0;
    bool narrow_keys = true;
    for (int attempt = 0; attempt < 2; ++attempt) {
    const bool queued = queued_on && attempt == 0;
    if (q > 0 || attempt > 0) HIPCHK(ctx, hipMemsetAsync(w.cx.state, rk::ST_UNKNOWN, m, st));
    // (the open flags and the counters: zero from the call's start for the first pair)
    if (queued && q > 0)
      rk::zero_regions(st, {{w.ctrl + 10, 2 * sizeof(uint32_t)},
                            {w.ctrl + 64, 2 * rk::PEND_WORDS * sizeof(uint32_t)}});
    if (prof) mark(ctx, RK_PH_SWEEP_X);
    // X decisions: hits' parents (X winner); the X states become a bitmask after
    rk::Axis ax{w.cx.key, w.cx.ent, nullptr, nullptr, w.cx.state, nullptr, w.par,
                w.cx.pk, w.cx.nbd, w.rlen_at, w.rbeg_at, m, pl.max_x, pq.len_ratio,
                pq.pos_ratio};
    uint32_t sweeps = blind;
    if ((rc = queued ? rk::resolve_axis_queued(ctx, ax, sc, blind,
                                               fused_roots ? nullptr : w.ctrl + 10, junk)
                     : rk::resolve_axis(ctx, ax, sc, true, &sweeps)))
      return rc;
    ctx->stats.x_sweeps = sweeps;
    if (prof) mark(ctx, RK_PH_SWEEP_Y);
    rk::nw_x_bits(w.xpos, w.cx.state, m, w.xbits, st);
    if (q == 0 && attempt == 0 && y_overlap) {  // the Y sort's last pass writes the CSR and the Y states
      HIPCHK(ctx, hipStreamWaitEvent(st, ctx->join, 0));
      rk::nw_y_sort_tail(w.yrec, w.Rb, m, yd, w.yhist, w.ystatus, w.cy, pl.nby, pl.max_y,
                         w.xbits, st);
    } else if (q == 0 && attempt == 0 && ysplit) {
      // (the order records are done with after the X chunk kernel; the order
      // sort's segment counts after its segment kernel)
      rk::nw_y_sort_split_after_x(w.yrec, w.Rb, w.Ra, m, yp, w.yhist, w.ystatus, w.cy, pl.nby,
                                  pl.max_y, w.xbits, w.chist, w.coff, ss, st);
    } else if (q == 0 && attempt == 0) {
      rk::nw_y_sort_after_x(w.yrec, w.Rb, m, yd, w.yhist, w.ystatus, w.cy, pl.nby, pl.max_y,
                            w.xbits, st);
    } else  // later ratio pairs, or a repeat: the same CSR, new X results
      rk::nw_fill_y(w.cy.ent, w.xbits, w.cy.state, m, st);
    rk::Axis ay{w.cy.key, w.cy.ent, nullptr, nullptr, w.cy.state, nullptr, w.par,
                w.cy.pk, w.cy.nbd, w.rlen_at, w.rbeg_at, m, pl.max_y, pq.len_ratio,
                pq.pos_ratio};
    ay.par_dev = true;
    sweeps = blind;
    if ((rc = queued ? rk::resolve_axis_queued(ctx, ay, scy, blind,
                                               fused_roots ? nullptr : w.ctrl + 11, junk)
                     : rk::resolve_axis(ctx, ay, sc, true, &sweeps)))
      return rc;
    ctx->stats.y_sweeps = sweeps;

    // group roots and ids
    if (prof) mark(ctx, RK_PH_ROOTS);
    rk::Proc pr{};
    pr.par = w.par;
    rounds = 0;
    G = 0;
    bool open_axes = false;
    if (fused_roots) {
      // the new-group ranks from the parents' root flags (G straight into
      // ctrl[32]); the wide-key flag, G and the queued axes' pending counters
      // back in one readback; later pairs' member histograms and listed-chain
      // count cleared first
      rk::zero_regions(st, {{q > 0 ? w.ehist : nullptr, 4096 * sizeof(uint32_t)},
                            {q > 0 ? w.ctrl + 12 : nullptr, sizeof(uint32_t)}});
      rk::exclusive_scan_roots(w.par, m, w.newrank, ss, st, w.ctrl + 32);
      if ((rc = readback(ctx, w.ctrl + 5, 64 - 5 + 2 * rk::PEND_WORDS))) return rc;
      uint32_t pending = 0;
      for (uint32_t k = 0; k < 2 * rk::PEND_WORDS; ++k) pending |= ctx->host[64 - 5 + k];
      if (queued && pending) {
        open_axes = true;  // an axis was left open: this pair again, the careful way
      } else {
        G = ctx->host[27];
        narrow_keys = ctx->host[1] == 0;
        rounds = 1;
      }
    } else {
    // (the first round's changed-count with the scan's end word, one launch;
    // later pairs' member histograms too -- the first pair's are still zero)
    rk::zero_regions(st, {{w.isnew + m, sizeof(uint32_t)},
                          {w.ctrl + 5, sizeof(uint32_t)},
                          {q > 0 ? w.ehist : nullptr, 4096 * sizeof(uint32_t)}});
    for (;;) {
      if (rounds > 0) HIPCHK(ctx, hipMemsetAsync(w.ctrl + 5, 0, sizeof(uint32_t), st));
      rk::jump_round(pr, m, w.ctrl + 5, rounds == 0 ? w.isnew : nullptr, w.ctrl, st,
                     queued && rounds == 0 ? w.ctrl + 10 : nullptr);
      if (rounds == 0) {
        // the new-group flags are final after the first round: their scan
        // (the group count G, in ctrl[32]) shares the round's readback
        rk::exclusive_scan_u32(w.isnew, w.newrank, (size_t)m + 1, ss, st);
        HIPCHK(ctx, hipMemcpyAsync(w.ctrl + 32, w.newrank + m, sizeof(uint32_t),
                                   hipMemcpyDeviceToDevice, st));
      }
      // + the wide-key flag, the queued axes' open flags, G
      if ((rc = readback(ctx, w.ctrl + 5, 28))) return rc;
      if (rounds == 0 && queued && (ctx->host[5] || ctx->host[6])) {
        open_axes = true;  // an axis was left open: this pair again, the careful way
        break;
      }
      if (rounds == 0) G = ctx->host[27];
      ++rounds;
      narrow_keys = ctx->host[1] == 0;
      if (!ctx->host[0]) break;
      if (rounds > 64) {
        ctx->err = "pointer jumping did not converge";
        return RK_E_INTERNAL;
      }
    }
    }
    if (!open_axes) break;
    ++ctx->stats.sweep_repeats;
    }
    ctx->stats.jump_rounds = rounds;
    out->n_groups = G;
    ctx->stats.n_groups = G;
    // 12-B member records take 9-bit digits too (a 25..27-bit gid in 3
    // passes); 16-B ones keep 8-bit digits
    const rk::NwDigits ed = rk::nw_plan(rk::bit_length(G ? G - 1 : 0), narrow_keys ? bits12 : 8);
    // 12-B member records: the sort by gid in two stages (coarse passes, then
    // the segment kernel, which also writes the group starts)
    // RK_NW_MSPLIT=1 (measurement): the member sort in two stages
    static const bool msplit_on = [] {
      const char *e = getenv("RK_NW_MSPLIT");
      return e && e[0] == '1';
    }();
    const rk::NwOrderPlan mp = narrow_keys && msplit_on
                                   ? rk::nw_order_split(m, G, rk::bit_length(G ? G - 1 : 0))
                                   : rk::NwOrderPlan{};
    const bool msplit = mp.coarse.passes > 0;
    // (ehist: zero -- cleared at the start, or with the roots' words for q > 0)
    // gids into isnew's words (dead after the scan)
    if (fused_roots)  // (otag: free until the group sort)
      rk::nw_assign_jump(w.par, w.newrank, w.isnew, m, msplit ? mp.coarse : ed, w.ehist, w.otag,
                         w.ctrl, st);
    else
      rk::nw_assign(w.par, w.newrank, w.isnew, m, msplit ? mp.coarse : ed, w.ehist, st);

    // members (stable by gid => processing order), in-group order, flags
    if (prof) mark(ctx, RK_PH_MEMBERS);
    if (msplit) {
      // (the order records and the Y records are done with)
      rk::nw_member_sort_split(w.erec, w.isnew, w.Ra, w.Rb, w.yrec, m, G, mp, w.ehist, w.astatus,
                               w.sgid, w.reckey, w.tag, w.mrow, w.goff, w.chist, w.coff, ss, st);
    } else {
      rk::nw_member_sort(w.erec, w.isnew, w.Ra, w.Rb, m, ed, w.ehist, w.astatus, w.sgid,
                         w.reckey, w.tag, w.mrow, narrow_keys, st);
      rk::group_offsets(w.sgid, m, G, w.goff, st);
    }
    if (prof) mark(ctx, RK_PH_GROUP_SORT);
    // one pair: the depth-limit heap segments' count (crafted inputs only)
    // comes back with the final status word (ctrl[33]) instead of a wait of
    // its own (several pairs share the scratch: each waits)
    if ((rc = rk::sort_groups_exact(w.sgid, w.goff, G, m, w.reckey, w.tag, w.otag, w.gsort, ss,
                                    ctx->host + 128, narrow_keys, st, st2, ctx->fork, ctx->join,
                                    npairs == 1 ? w.ctrl + 33 : nullptr))) {
      ctx->err = "depth-limit heap segments: buffer allocation failed";
      return rc;
    }
    if (prof) mark(ctx, RK_PH_EMIT);
    rk::emit_result(w.otag, w.sgid, w.goff, w.mrow, m, out->gid, out->repval, out->out_order,
                    st);
    HIPCHK(ctx, hipGetLastError());
    if (prof) mark(ctx, RK_N_PHASES);
  }
  HIPCHK(ctx, hipEventRecord(ctx->ev1, st));
  if ((rc = readback(ctx, w.ctrl, npairs == 1 ? 34 : 14))) return rc;
  if (fused_roots && ctx->host[13]) {  // a parent chain above 4128 steps: round by round
    collect_phases(ctx);
    return classify_narrow(ctx, in, prms, npairs, outs, pl, fallback, wire, false);
  }
  if (npairs == 1 && m && ctx->host[33]) {  // heap segments: sorted now, then the result again
    const uint32_t G = outs[0].n_groups;
    if ((rc = rk::sort_groups_heap_deferred(G, m, w.reckey, w.tag, w.otag, w.gsort, ctx->host[33],
                                            ctx->host + 128, st))) {
      ctx->err = "depth-limit heap segments: buffer allocation failed";
      return rc;
    }
    rk::emit_result(w.otag, w.sgid, w.goff, w.mrow, m, outs[0].gid, outs[0].repval,
                    outs[0].out_order, st);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipEventRecord(ctx->ev1, st));
    if ((rc = readback(ctx, w.ctrl, 1))) return rc;
  }
  collect_phases(ctx);
  if ((rc = err_status(ctx, ctx->host[0]))) return rc;
  float ms = 0;
  HIPCHK(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
  ctx->stats.device_ms = ms;
  ctx->stats.pipeline = 1;
  rk::nw_trace_dump(st);
  return RK_OK;
}

// All pairs share one fragment set: the ratio-independent part (processing
// order, the two occupancy axes, the in-group sort keys) is built once, then
// every (len_ratio, pos_ratio) pair runs the sweeps, groups and in-group order
// (repkiller.cpp:60-72 runs each pair through the whole path).  Phase
// profiling covers the shared part and the first pair.
// The record pipeline takes this input (and the generic one is not forced).
bool record_eligible(const rk_ctx *ctx, uint64_t n) {
  return ctx->pipeline == RK_PIPELINE_AUTO && record_pipeline_enabled() && n > 0 &&
         n < (1ull << 30);
}

// wire: the rows as 12-B wire records in HBM (rk_classify's compact upload,
// rk_io.hip); only in->n is read then, and the input must be record-eligible
int classify_device(rk_ctx *ctx, const rk_frags_soa *in, const rk_params *prms, uint32_t npairs,
                    rk_result *outs, const uint3 *wire = nullptr) {
  if (!ctx || !in || !prms || !outs || npairs == 0) return RK_E_ARG;
  if (in->n >= 0xFFFFFFFFull) return RK_E_TOO_MANY;
  for (uint32_t q = 0; q < npairs; ++q) {
    const rk_params &pq = prms[q];
    if (pq.len_ratio <= 0 || pq.pos_ratio <= 0) {  // NaN passes, as in the reference
      ctx->err = "ratios must be greater than zero (commonFunctions.cpp:26-27)";
      return RK_E_ARG;
    }
    if (pq.len_x_hdr != prms[0].len_x_hdr || pq.len_y_hdr != prms[0].len_y_hdr) {
      ctx->err = "all pairs must describe the same fragment set (header lengths differ)";
      return RK_E_ARG;
    }
    if (in->n && (!outs[q].gid || !outs[q].repval || !outs[q].out_order)) return RK_E_ARG;
  }
  if (in->n && !wire && (!in->x_start || !in->y_start || !in->length || !in->strand))
    return RK_E_ARG;
  if (wire && !record_eligible(ctx, in->n)) {
    ctx->err = "wire rows need the record pipeline";
    return RK_E_INTERNAL;
  }
  HIPCHK(ctx, hipSetDevice(ctx->device));
  std::memset(&ctx->stats, 0, sizeof ctx->stats);
  rk::stats_numa_unknown(&ctx->stats);
  hipStream_t st = ctx->stream;
  const rk_params *prm = &prms[0];

  Plan pl{};
  pl.n = in->n;
  const uint64_t len_x = prm->len_x_hdr + 1, len_y = prm->len_y_hdr + 1;  // FragmentsDatabase.cpp:62,65
  pl.vsize = 1 + len_x / 10;                                                // :84
  pl.max_x = len_x / 100;                                                   // SequenceOcupationList.cpp:4
  pl.max_y = len_y / 100;
  if (pl.vsize - 1 >= 0xFFFFFFF0ull || 2 * (pl.max_x + 1) >= 0xFFFFFFF0ull ||
      2 * (pl.max_y + 1) >= 0xFFFFFFF0ull) {
    ctx->err = "sequence length too large for 32-bit bucket ids";
    return RK_E_ARG;
  }
  pl.nbx = (uint32_t)(pl.max_x + 1);
  pl.nby = (uint32_t)(pl.max_y + 1);
  int rc;
  if (record_eligible(ctx, pl.n)) {
    bool fallback = false;
    rc = classify_narrow(ctx, in, prms, npairs, outs, pl, &fallback, wire);
    if (rc || !fallback) return rc;
    if (wire) {  // wire rows always pack (checked on the host)
      ctx->err = "wire rows did not pack";
      return RK_E_INTERNAL;
    }
    // the generic pipeline needs its own ~200 B per row: give the HBM back
    (void)hipStreamSynchronize(ctx->stream2);
    (void)hipFree(ctx->ws_nw);
    ctx->ws_nw = nullptr;
    ctx->ws_nw_cap = 0;
    if (ctx->profiling) ctx->kt.n = 0;  // the timings of the abandoned attempt
    const uint32_t why = ctx->stats.record_fallback;
    std::memset(&ctx->stats, 0, sizeof ctx->stats);
    rk::stats_numa_unknown(&ctx->stats);
    ctx->stats.record_fallback = why;
  }
  Work w{};  // value-initialised: optional Proc columns (grow, ...) stay null
  rc = ensure_ws(ctx, pl, w);
  if (rc) return rc;
  const uint32_t n = (uint32_t)pl.n;
  rk::ScanScratch ss{w.scan, w.scan_cap};
  ctx->stats.n_in = n;

  HIPCHK(ctx, hipEventRecord(ctx->ev0, st));
  HIPCHK(ctx, hipMemsetAsync(w.ctrl, 0, (64 + rk::PEND_WORDS) * sizeof(uint32_t), st));
  rk::Frags f{in->x_start, in->y_start, in->length, in->strand, n};
  mark(ctx, RK_PH_PREP);

  // 1-2: processing order = stable sort of rows by xStart/10 (dropped bucket last)
  rk::prep_keys(f, pl.vsize, pl.max_x, pl.max_y, w.pkey_in, w.p.rec, w.ctrl + 1, w.ctrl, st);
  mark(ctx, RK_PH_ORDER);
  rk::radix_sort_pairs(w.pkey_in, nullptr, w.p.pkey, w.p.row, w.tk, w.tv, n,
                       rk::bit_length(pl.vsize - 1), w.radix, w.radix_words, st);
  HIPCHK(ctx, hipGetLastError());
  if ((rc = readback(ctx, w.ctrl, 2))) return rc;
  if ((rc = err_status(ctx, ctx->host[0]))) return rc;
  const bool fast32 = !(ctx->host[0] & rk::ERRB_WIDE_LENGTH);
  const uint32_t m = ctx->host[1];
  ctx->stats.n_proc = m;
  for (uint32_t q = 0; q < npairs; ++q) outs[q].n_out = m, outs[q].n_groups = 0;
  if (m == 0) {
    mark(ctx, RK_N_PHASES);
    collect_phases(ctx);
    HIPCHK(ctx, hipEventRecord(ctx->ev1, st));
    HIPCHK(ctx, hipStreamSynchronize(st));
    return RK_OK;
  }

  // 3: processing-order SoA, bucket keys, in-group sort keys
  mark(ctx, RK_PH_GATHER);
  if (!fast32 && (rc = ensure_wide(ctx, pl.n, w))) return rc;  // some length >= 2^31
  rk::gather_proc(f, w.p, m, pl.nbx, pl.nby, st);

  // 4: the two occupancy axes as bucket runs (stable: processing order inside).
  // The Y sort and the in-group sort keys run on the second stream, overlapped
  // with the X sort and sweeps; the Y fill waits for them.
  HIPCHK(ctx, hipEventRecord(ctx->fork, st));
  HIPCHK(ctx, hipStreamWaitEvent(ctx->stream2, ctx->fork, 0));
  rk::radix_sort_pairs(w.p.keyy, nullptr, w.cy.key, w.cy.ent, w.tk2, w.tv2, m,
                       rk::bit_length(2ull * pl.nby - 1), w.radix2, w.radix_words, ctx->stream2);
  rk::sort_keys(w.p, m, w.ctrl + 6, ctx->stream2);
  HIPCHK(ctx, hipEventRecord(ctx->join, ctx->stream2));
  mark(ctx, RK_PH_OCC_CSR);
  rk::radix_sort_pairs(w.p.keyx, nullptr, w.cx.key, w.cx.ent, w.tk, w.tv, m,
                       rk::bit_length(2ull * pl.nbx - 1), w.radix, w.radix_words, st);
  rk::csr_fill_x(w.cx, w.p.xrec, m, pl.max_x, st);
  HIPCHK(ctx, hipGetLastError());

  for (uint32_t q = 0; q < npairs; ++q) {
    const rk_params &pq = prms[q];
    rk_result *out = &outs[q];
    const bool prof = q == 0;
    if (q > 0) HIPCHK(ctx, hipMemsetAsync(w.cx.state, rk::ST_UNKNOWN, m, st));

    // 5: X, then Y (X hits join the Y lists; X misses query Y)
    if (prof) mark(ctx, RK_PH_SWEEP_X);
    // X decisions write X results into the Y records and X hits' parents
    rk::Axis ax{w.cx.key, w.cx.ent, w.cx.cen, w.cx.len, w.cx.state,
                reinterpret_cast<uint32_t *>(w.p.yrec), w.p.par,
                w.cx.pk, w.cx.nbd, w.rlen_at, w.rbeg_at, m, pl.max_x, pq.len_ratio,
                pq.pos_ratio};
    uint32_t sweeps = 0;
    if ((rc = rk::resolve_axis(ctx, ax, sweep_scratch(w), fast32, &sweeps))) return rc;
    ctx->stats.x_sweeps = sweeps;
    if (prof) mark(ctx, RK_PH_SWEEP_Y);
    if (q == 0) HIPCHK(ctx, hipStreamWaitEvent(st, ctx->join, 0));
    rk::csr_fill_y(w.cy, w.p.yrec, w.p.ylenhi, m, pl.max_y, st);
    // X misses: the Y sweeps write parent = Y winner, or itself (new group)
    rk::Axis ay{w.cy.key, w.cy.ent, w.cy.cen, w.cy.len, w.cy.state, nullptr, w.p.par,
                w.cy.pk, w.cy.nbd, w.rlen_at, w.rbeg_at, m, pl.max_y, pq.len_ratio,
                pq.pos_ratio};
    ay.par_dev = true;
    if ((rc = rk::resolve_axis(ctx, ay, sweep_scratch(w), fast32, &sweeps))) return rc;
    ctx->stats.y_sweeps = sweeps;

    // 6: group roots and ids
    if (prof) mark(ctx, RK_PH_ROOTS);
    HIPCHK(ctx, hipMemsetAsync(w.isnew + m, 0, sizeof(uint32_t), st));
    uint32_t rounds = 0;
    for (;;) {
      HIPCHK(ctx, hipMemsetAsync(w.ctrl + 5, 0, sizeof(uint32_t), st));
      rk::jump_round(w.p, m, w.ctrl + 5, rounds == 0 ? w.isnew : nullptr, w.ctrl, st);
      if ((rc = readback(ctx, w.ctrl + 5, 2))) return rc;  // + the wide-key flag
      ++rounds;
      if (!ctx->host[0]) break;
      if (rounds > 64) {
        ctx->err = "pointer jumping did not converge";
        return RK_E_INTERNAL;
      }
    }
    ctx->stats.jump_rounds = rounds;
    const bool narrow_keys = ctx->host[1] == 0;
    rk::exclusive_scan_u32(w.isnew, w.newrank, (size_t)m + 1, ss, st);
    if ((rc = readback(ctx, w.newrank + m, 1))) return rc;
    const uint32_t G = ctx->host[0];
    out->n_groups = G;
    ctx->stats.n_groups = G;
    rk::assign_gid(w.p, m, w.newrank, st);

    // 7-9: members (stable by gid => processing order), in-group order, flags
    if (prof) mark(ctx, RK_PH_MEMBERS);
    rk::radix_sort_pairs(w.p.gid, nullptr, w.sgid, w.gmem, w.tk, w.tv, m,
                         rk::bit_length(G - 1), w.radix, w.radix_words, st);
    rk::group_offsets(w.sgid, m, G, w.goff, st);
    rk::build_records(w.gmem, w.p.hrec, m, w.reckey, w.tag, st);
    if (prof) mark(ctx, RK_PH_GROUP_SORT);
    if ((rc = rk::sort_groups_exact(w.sgid, w.goff, G, m, w.reckey, w.tag, w.otag, w.gsort, ss,
                                    ctx->host + 128, narrow_keys, st, ctx->stream2, ctx->fork,
                                    ctx->join))) {
      ctx->err = "depth-limit heap segments: buffer allocation failed";
      return rc;
    }
    if (prof) mark(ctx, RK_PH_EMIT);
    rk::emit_result(w.otag, w.sgid, w.goff, w.gmem, m, out->gid, out->repval,
                    out->out_order, st);
    HIPCHK(ctx, hipGetLastError());
    if (prof) mark(ctx, RK_N_PHASES);
  }
  HIPCHK(ctx, hipEventRecord(ctx->ev1, st));
  if ((rc = readback(ctx, w.ctrl, 1))) return rc;
  collect_phases(ctx);
  if ((rc = err_status(ctx, ctx->host[0]))) return rc;
  float ms = 0;
  HIPCHK(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
  ctx->stats.device_ms = ms;
  ctx->stats.pipeline = 2;
  return RK_OK;
}

}  // namespace

// The second stream carries the Y axis sort, the longer branch of the fork:
// it is created at the highest stream priority (cfg3 step 12.70-12.83 ms
// against 12.90-13.15 at the default priority); RK_S2_PRIO=0 turns that off.
static hipError_t create_stream2(hipStream_t *s) {
  const char *e = std::getenv("RK_S2_PRIO");
  if (!(e && e[0] == '0')) {
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess)
      return hipStreamCreateWithPriority(s, hipStreamNonBlocking, greatest);
  }
  return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}

extern "C" int rk_create(rk_ctx **out, int device) {
  if (!out) return RK_E_ARG;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0 || device < 0 || device >= count)
    return RK_E_NODEVICE;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return RK_E_NODEVICE;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return RK_E_NODEVICE;
  auto ctx = new (std::nothrow) rk_ctx;
  if (!ctx) return RK_E_NOMEM;
  ctx->device = device;
  // RK_ONE_STREAM=1 (profiling only): the overlapped work runs on the main
  // stream too, so per-kernel times are not shared with a concurrent kernel
  const char *one = std::getenv("RK_ONE_STREAM");
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
      (one && one[0] == '1' ? (ctx->stream2 = ctx->stream, hipSuccess)
                            : create_stream2(&ctx->stream2)) !=
          hipSuccess ||
      hipEventCreate(&ctx->ev0) != hipSuccess || hipEventCreate(&ctx->ev1) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->join, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->aux, hipEventDisableTiming) != hipSuccess ||
      hipHostMalloc((void **)&ctx->host, 256 * sizeof(uint32_t), hipHostMallocDefault) !=
          hipSuccess) {
    rk_destroy(ctx);
    return RK_E_HIP;
  }
  if (hipMalloc((void **)&ctx->kt.units, rk::KernelTimer::MAX * sizeof(uint32_t)) != hipSuccess) {
    rk_destroy(ctx);
    return RK_E_HIP;
  }
  // timing-only events: no system-scope fence at record (HIP's recommendation
  // for pure timing events; it keeps the instrumentation's own cost low)
  for (auto &e : ctx->kt.ev)
    if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) {
      rk_destroy(ctx);
      return RK_E_HIP;
    }
  for (auto &e : ctx->pev)
    if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) {
    rk_destroy(ctx);
    return RK_E_HIP;
  }
  *out = ctx;
  return RK_OK;
}

extern "C" void rk_destroy(rk_ctx *ctx) {
  if (!ctx) return;
  if (ctx->device >= 0) (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->stream2) (void)hipStreamSynchronize(ctx->stream2);
  rk::io_destroy(ctx);
  if (ctx->ws) (void)hipFree(ctx->ws);
  if (ctx->io) (void)hipFree(ctx->io);
  if (ctx->ws_wide) (void)hipFree(ctx->ws_wide);
  if (ctx->kt.units) (void)hipFree(ctx->kt.units);
  if (ctx->ws_nw) (void)hipFree(ctx->ws_nw);
  if (ctx->nw_small) (void)hipFree(ctx->nw_small);
  for (void *p : ctx->pool.ptr)
    if (p) (void)hipFree(p);
  if (ctx->host) (void)hipHostFree(ctx->host);
  if (ctx->sh_msg) (void)hipHostFree(ctx->sh_msg);
  if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
  if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
  for (auto &e : ctx->pev)
    if (e) (void)hipEventDestroy(e);
  for (auto &e : ctx->kt.ev)
    if (e) (void)hipEventDestroy(e);
  if (ctx->fork) (void)hipEventDestroy(ctx->fork);
  if (ctx->join) (void)hipEventDestroy(ctx->join);
  if (ctx->aux) (void)hipEventDestroy(ctx->aux);
  if (ctx->stream2 && ctx->stream2 != ctx->stream) (void)hipStreamDestroy(ctx->stream2);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

extern "C" const char *rk_last_error(const rk_ctx *ctx) { return ctx ? ctx->err.c_str() : ""; }

extern "C" int rk_set_profiling(rk_ctx *ctx, int enable) {
  if (!ctx) return RK_E_ARG;
  if (enable >= 2 + rk::KID_COUNT) return RK_E_ARG;
  ctx->profiling = enable != 0;
  ctx->kt.only = enable >= 2 ? enable - 2 : -1;  // 2 + k: kernel k's launches only
  return RK_OK;
}

extern "C" int rk_get_phase_ms(const rk_ctx *ctx, double *ms, uint32_t *calls) {
  if (!ctx || !ms) return RK_E_ARG;
  for (int i = 0; i < RK_N_PHASES; ++i) {
    ms[i] = ctx->phase_ms[i];
    if (calls) calls[i] = ctx->phase_calls[i];
  }
  return RK_OK;
}

extern "C" int rk_get_kernel_timing(const rk_ctx *ctx, int kernel, double *total_ms,
                                    double *algo_bytes, uint64_t *launches) {
  if (!ctx || kernel < 0 || kernel >= rk::KID_COUNT) return RK_E_ARG;
  if (total_ms) *total_ms = ctx->kt_ms[kernel];
  if (algo_bytes) *algo_bytes = ctx->kt_bytes[kernel];
  if (launches) *launches = ctx->kt_launches[kernel];
  return RK_OK;
}

extern "C" int rk_kernel_count(void) { return rk::KID_COUNT; }

extern "C" const char *rk_kernel_name(int kernel) {
  return kernel >= 0 && kernel < rk::KID_COUNT ? rk::kKernelNames[kernel] : "";
}

extern "C" int rk_reset_phases(rk_ctx *ctx) {
  if (!ctx) return RK_E_ARG;
  for (int k = 0; k < rk::KID_COUNT; ++k)
    ctx->kt_ms[k] = ctx->kt_bytes[k] = 0, ctx->kt_launches[k] = 0;
  for (int i = 0; i < RK_N_PHASES; ++i) ctx->phase_ms[i] = 0, ctx->phase_calls[i] = 0;
  return RK_OK;
}

extern "C" const char *rk_phase_name(int phase) {
  return phase >= 0 && phase < RK_N_PHASES ? kPhaseNames[phase] : "";
}

extern "C" int rk_set_pipeline(rk_ctx *ctx, int pipeline) {
  if (!ctx || (pipeline != RK_PIPELINE_AUTO && pipeline != RK_PIPELINE_GENERIC)) return RK_E_ARG;
  ctx->pipeline = pipeline;
  return RK_OK;
}

extern "C" int rk_get_stats(const rk_ctx *ctx, rk_stats *st) {
  if (!ctx || !st) return RK_E_ARG;
  *st = ctx->stats;
  return RK_OK;
}

extern "C" int rk_classify_device_pairs(rk_ctx *ctx, const rk_frags_soa *in_dev,
                                        const rk_params *p, uint32_t npairs,
                                        rk_result *out_dev) {
  if (!ctx) return RK_E_ARG;
  ctx->err.clear();
  int rc;
  try {
    rc = classify_device(ctx, in_dev, p, npairs, out_dev);
  } catch (...) {
    ctx->err = "unexpected C++ exception";
    rc = RK_E_INTERNAL;
  }
  rk::g_ktimer = nullptr;  // never leave the kernel timer pointing at this context
  // an early error return may leave the second stream's work in flight
  if (ctx->stream2) (void)hipStreamSynchronize(ctx->stream2);
  return rc;
}

extern "C" int rk_classify_device(rk_ctx *ctx, const rk_frags_soa *in_dev, const rk_params *p,
                                  rk_result *out_dev) {
  return rk_classify_device_pairs(ctx, in_dev, p, 1, out_dev);
}

extern "C" int rk_std_sort_segments(rk_ctx *ctx, const uint64_t *keys, uint64_t n,
                                    const uint32_t *seg_off, uint32_t nseg, uint32_t *perm) {
  if (!ctx || (n && (!keys || !perm)) || !seg_off || n >= 0xFFFFFFFFull) return RK_E_ARG;
  if (seg_off[0] != 0 || seg_off[nseg] != n) return RK_E_ARG;
  for (uint32_t s = 0; s < nseg; ++s)
    if (seg_off[s + 1] <= seg_off[s]) return RK_E_ARG;  // segments must be non-empty
  if (!n) return RK_OK;
  ctx->err.clear();
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const uint32_t m = (uint32_t)n;
  std::vector<uint32_t> sg(m), tags(m);
  for (uint32_t s = 0; s < nseg; ++s)
    for (uint32_t x = seg_off[s]; x < seg_off[s + 1]; ++x) sg[x] = s, tags[x] = x;
  const size_t gs = rk::groupsort_scratch_bytes(m), sc = rk::scan_blocks(nseg + 2) + 64;
  const size_t M = m;  // byte sizes in 64 bits: m * 8 wraps a uint32_t from m = 2^29
  const size_t bytes = align_up(M * 8 + 16) + align_up(M * 4 + 16) * 3 +
                       align_up(((size_t)nseg + 1) * 4 + 16) + align_up(gs) + align_up(sc * 4);
  void *buf = nullptr;
  HIPCHK(ctx, hipMalloc(&buf, bytes));
  Carve c{(char *)buf};
  uint64_t *dk = c.take<uint64_t>(m);
  uint32_t *dt = c.take<uint32_t>(m), *dot = c.take<uint32_t>(m), *dg = c.take<uint32_t>(m);
  uint32_t *doff = c.take<uint32_t>(nseg + 1);
  void *dgs = c.take<uint8_t>(gs);
  uint32_t *dsc = c.take<uint32_t>(sc);
  hipStream_t st = ctx->stream;
  int rc = RK_OK;
  if (hipMemcpyAsync(dk, keys, M * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
      hipMemcpyAsync(dt, tags.data(), M * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
      hipMemcpyAsync(dg, sg.data(), M * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
      hipMemcpyAsync(doff, seg_off, ((size_t)nseg + 1) * 4, hipMemcpyHostToDevice, st) !=
          hipSuccess) {
    rc = RK_E_HIP;
  } else {
    bool narrow = true;
    for (uint32_t x = 0; x < m; ++x) narrow &= (keys[x] >> 32) == 0;
    // one-element segments are not written by the group sort: their slot stays
    (void)hipMemcpyAsync(dot, dt, M * 4, hipMemcpyDeviceToDevice, st);
    rc = rk::sort_groups_exact(dg, doff, nseg, m, dk, dt, dot, dgs, rk::ScanScratch{dsc, sc},
                               ctx->host + 128, narrow, st);
    if (!rc && (hipGetLastError() != hipSuccess ||
                hipMemcpyAsync(perm, dot, M * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess))
      rc = RK_E_HIP;
  }
  (void)hipStreamSynchronize(st);
  (void)hipFree(buf);
  if (rc == RK_E_NOMEM) ctx->err = "rk_std_sort_segments: heap-segment buffer allocation failed";
  else if (rc) ctx->err = "rk_std_sort_segments: HIP failure";
  return rc;
}

// rk_classify through the compact wire format; RK_WIRE_UNPACKABLE when some
// row does not fit a wire record (nothing was classified: the caller uploads
// the SoA columns instead)
constexpr int RK_WIRE_UNPACKABLE = 1 << 20;
static int classify_wire(rk_ctx *ctx, const rk_frags_soa *in, const rk_params *p, uint32_t npairs,
                         rk_result *out) {
  const size_t n = in->n;
  const size_t need = align_up(n * 12 + 16) +
                      (size_t)npairs * (align_up(n + 16) + align_up(n * 4 + 16) * 2);
  if (need > ctx->io_cap) {
    if (ctx->io) (void)hipFree(ctx->io);
    ctx->io = nullptr;
    ctx->io_cap = 0;
    HIPCHK(ctx, hipMalloc(&ctx->io, need));
    ctx->io_cap = need;
  }
  Carve c{(char *)ctx->io};
  uint3 *rows = c.take<uint3>(n);
  std::vector<rk_result> dres(npairs);
  for (uint32_t q = 0; q < npairs; ++q) {
    uint8_t *drep = c.take<uint8_t>(n);
    uint32_t *dgid = c.take<uint32_t>(n), *dord = c.take<uint32_t>(n);
    dres[q] = rk_result{dord, dgid, drep, 0, 0};
  }
  const double t0 = rk::wall_ms();
  int rc = rk::io_h2d_rows(ctx, *in, rows);
  if (rc) return rc == 1 ? RK_WIRE_UNPACKABLE : rc;
  const double t1 = rk::wall_ms();
  const rk_frags_soa din{nullptr, nullptr, nullptr, nullptr, n};
  rc = classify_device(ctx, &din, p, npairs, dres.data(), rows);
  if (rc) return rc;
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  const double t2 = rk::wall_ms();
  // the flags first; then the output order comes down while other threads
  // rebuild the gids from the flags
  std::vector<rk::IoPiece> flags, orders;
  for (uint32_t q = 0; q < npairs; ++q) {
    out[q].n_out = dres[q].n_out;
    out[q].n_groups = dres[q].n_groups;
    flags.push_back({out[q].repval, dres[q].repval, dres[q].n_out});
    orders.push_back({out[q].out_order, dres[q].out_order, dres[q].n_out * 4});
  }
  if ((rc = rk::io_d2h(ctx, flags))) return rc;
  {
    rk::GidJob job;
    for (uint32_t q = 0; q < npairs; ++q)
      rk::gids_from_flags_async(out[q].repval, out[q].n_out, out[q].gid, 8, job);
    rc = rk::io_d2h(ctx, orders);
    job.wait();
  }
  if (rc) return rc;
  ctx->stats.h2d_ms = t1 - t0;
  ctx->stats.d2h_ms = rk::wall_ms() - t2;
  ctx->stats.wire = 1;
  rk::io_numa_stats(ctx, &ctx->stats);
  return RK_OK;
}

extern "C" int rk_classify_pairs(rk_ctx *ctx, const rk_frags_soa *in, const rk_params *p,
                                 uint32_t npairs, rk_result *out) {
  if (!ctx || !in || !p || !out || npairs == 0) return RK_E_ARG;
  ctx->err.clear();
  const size_t n = in->n;
  if (n >= 0xFFFFFFFFull) return RK_E_TOO_MANY;
  if (n && (!in->x_start || !in->y_start || !in->length || !in->strand)) return RK_E_ARG;
  for (uint32_t q = 0; q < npairs; ++q)
    if (n && (!out[q].gid || !out[q].repval || !out[q].out_order)) return RK_E_ARG;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  // The compact wire format (RK_WIRE=0: off): rows go up as 12-B records
  // packed by the host threads (25 B per row as SoA columns), and results come
  // down as order + flag (5 B per row instead of 9): a new group starts at
  // every row whose flag is not 2, so the gids are a host prefix count.
  static const bool wire_on = [] {
    const char *e = getenv("RK_WIRE");
    return !e || e[0] != '0';
  }();
  if (wire_on && record_eligible(ctx, n)) {
    const int rc = classify_wire(ctx, in, p, npairs, out);
    if (rc != RK_WIRE_UNPACKABLE) return rc;
  }
  // device staging: x, y, len (u64), strand (u8) in; per pair gid, order (u32), rep (u8) out
  size_t need = align_up(n * 8 + 16) * 3 + align_up(n + 16) +
                (size_t)npairs * (align_up(n + 16) + align_up(n * 4 + 16) * 2);
  if (need > ctx->io_cap) {
    if (ctx->io) (void)hipFree(ctx->io);
    ctx->io = nullptr;
    ctx->io_cap = 0;
    HIPCHK(ctx, hipMalloc(&ctx->io, need));
    ctx->io_cap = need;
  }
  Carve c{(char *)ctx->io};
  uint64_t *dx = c.take<uint64_t>(n), *dy = c.take<uint64_t>(n), *dl = c.take<uint64_t>(n);
  uint8_t *ds = c.take<uint8_t>(n);
  std::vector<rk_result> dres(npairs);
  for (uint32_t q = 0; q < npairs; ++q) {
    uint8_t *drep = c.take<uint8_t>(n);
    uint32_t *dgid = c.take<uint32_t>(n), *dord = c.take<uint32_t>(n);
    dres[q] = rk_result{dord, dgid, drep, 0, 0};
  }
  // 1: upload (copy stream; pinned buffers by DMA, pageable ones staged)
  const double t0 = rk::wall_ms();
  int rc = rk::io_h2d(ctx, {{(void *)in->x_start, dx, n * 8},
                            {(void *)in->y_start, dy, n * 8},
                            {(void *)in->length, dl, n * 8},
                            {(void *)in->strand, ds, n}});
  if (rc) return rc;
  const double t1 = rk::wall_ms();
  // 2: classify
  rk_frags_soa din{dx, dy, dl, ds, n};
  rc = rk_classify_device_pairs(ctx, &din, p, npairs, dres.data());
  if (rc) return rc;
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  // 3: download
  const double t2 = rk::wall_ms();
  std::vector<rk::IoPiece> down;
  for (uint32_t q = 0; q < npairs; ++q) {
    out[q].n_out = dres[q].n_out;
    out[q].n_groups = dres[q].n_groups;
    const size_t k = n ? dres[q].n_out : 0;
    down.push_back({out[q].out_order, dres[q].out_order, k * 4});
    down.push_back({out[q].gid, dres[q].gid, k * 4});
    down.push_back({out[q].repval, dres[q].repval, k});
  }
  if ((rc = rk::io_d2h(ctx, down))) return rc;
  ctx->stats.h2d_ms = t1 - t0;
  ctx->stats.d2h_ms = rk::wall_ms() - t2;
  rk::io_numa_stats(ctx, &ctx->stats);
  return RK_OK;
}

extern "C" int rk_classify(rk_ctx *ctx, const rk_frags_soa *in, const rk_params *p,
                           rk_result *out) {
  return rk_classify_pairs(ctx, in, p, 1, out);
}
