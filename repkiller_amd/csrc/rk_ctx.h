// rk_ctx.h -- the context object behind the C ABI and the host-side helpers
// shared by the single-device driver (rk_api.hip) and the sharded driver
// (rk_shard.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/repkiller_amd.h"
#include "rk_internal.h"

namespace rk {
struct IoEngine;  // rk_io.hip: copy stream, pinned staging ring, host copy threads
}

// Grow-only device buffers of the sharded driver, one per slot (the exchange
// sizes are only known mid-call, so they cannot share the single carve).
struct rk_pool {
  std::vector<void *> ptr;
  std::vector<size_t> cap;
};

struct rk_ctx {
  int device = -1;
  bool nw_fell_back = false;  // the last record-pipeline call handed over to the generic one
  uint64_t readbacks = 0;     // readback() calls over the context's life (host waits)
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;             // Y-axis sort, overlapped with the X sweeps
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  hipEvent_t aux = nullptr;  // sharded driver: the X bucket order is ready (stream 2)
  void *ws = nullptr;  // device workspace
  size_t ws_cap = 0;
  void *ws_wide = nullptr;  // 64-bit length columns, only when a length is >= 2^31
  size_t ws_wide_cap = 0;
  int pipeline = RK_PIPELINE_AUTO;
  void *ws_nw = nullptr;  // workspace of the record pipeline (rk_narrow.hip)
  size_t ws_nw_cap = 0;
  void *nw_small = nullptr;  // its control words + digit histograms: allocated once, so
                             // the pack check runs before the workspace is sized
  uint32_t *host = nullptr;  // pinned readback words
  // device copies for rk_classify (host-buffer entry point)
  void *io = nullptr;
  size_t io_cap = 0;
  rk::IoEngine *ioe = nullptr;
  rk_pool pool;  // rk_classify_sharded buffers
  // the sharded driver's fast path (rk_shard_fast.h): its all-gather messages
  // (pinned, every rank's), the stage fingerprints of the last call that
  // completed on it (a stage whose gathered counts match needs no agreement
  // before its exchanges: every buffer it takes already has its size), and the
  // sweeps it queues per axis before one deferred pending check
  char *sh_msg = nullptr;
  size_t sh_msg_cap = 0;
  uint64_t sh_fp[8] = {};
  uint32_t sh_blind[2] = {3, 3};
  rk_stats stats{};
  rk_shard_stats shard_stats{};
  std::string err;
  // phase profiling (rk_set_profiling): one event per phase boundary, on the
  // context stream, accumulated over calls until rk_reset_phases
  bool profiling = false;
  hipEvent_t pev[RK_N_PHASES + 1] = {};
  bool pev_used[RK_N_PHASES + 1] = {};
  double phase_ms[RK_N_PHASES] = {};
  uint32_t phase_calls[RK_N_PHASES] = {};
  rk::KernelTimer kt{};   // timed launches of the current call
  double kt_ms[rk::KID_COUNT] = {}, kt_bytes[rk::KID_COUNT] = {};
  uint64_t kt_launches[rk::KID_COUNT] = {};
};

namespace rk {

#define HIPCHK(ctx, call)                                                          \
  do {                                                                             \
    hipError_t e_ = (call);                                                        \
    if (e_ != hipSuccess) {                                                        \
      (ctx)->err = std::string(#call) + ": " + hipGetErrorString(e_);              \
      return RK_E_HIP;                                                             \
    }                                                                              \
  } while (0)

constexpr size_t ALIGN = 256;
inline size_t align_up(size_t v) { return (v + ALIGN - 1) & ~(ALIGN - 1); }

// bump allocator over a workspace (sizes first with a null base, then pointers)
struct Carve {
  char *base;
  size_t off = 0;
  template <class T>
  T *take(size_t count) {
    T *p = base ? reinterpret_cast<T *>(base + off) : nullptr;
    off += align_up(count * sizeof(T) + 16);  // +16: uint4 tails of the scan
    return p;
  }
};

// rk_io.hip: host <-> device pieces of rk_classify on the copy stream
// (pinned host buffers by DMA, pageable ones through the staging ring);
// both return when the transfer is complete
struct IoPiece {
  void *host;
  void *dev;
  size_t bytes;
};
int io_h2d(rk_ctx *ctx, const std::vector<IoPiece> &pieces);
int io_d2h(rk_ctx *ctx, const std::vector<IoPiece> &pieces);
// the rows of a host SoA as 12-B wire records {xStart lo, yStart lo, length
// (24) | reverse (1) | yStart >> 32 (3) | xStart >> 32 (4)} at `dev`, packed by
// the host threads into the staging ring; 1 when some row does not fit
// (length >= 2^24, yStart >= 2^35 or xStart >= 2^36)
int io_h2d_rows(rk_ctx *ctx, const rk_frags_soa &in, void *dev);
// gid[k] = (rows j <= k with flag[j] != 2) - 1: a new group starts at every
// row whose repeat flag is not 2; on `threads` threads of its own, started
// now and joined by job.wait(), so it runs beside a transfer that keeps the
// host pool busy
struct GidJob {
  std::vector<std::thread> th;
  void wait() {
    for (auto &t : th) t.join();
    th.clear();
  }
  ~GidJob() { wait(); }
};
void gids_from_flags_async(const uint8_t *flag, size_t n, uint32_t *gid, int threads, GidJob &job);
void io_destroy(rk_ctx *ctx);
// the NUMA nodes of the last upload (rk_stats numa_*)
void io_numa_stats(const rk_ctx *ctx, rk_stats *st);
// a call without an upload of its own: every NUMA field unknown (-1)
inline void stats_numa_unknown(rk_stats *st) {
  st->numa_input = st->numa_threads = st->numa_staging = st->numa_gpu = -1;
}
bool host_pinned(const void *p);
double wall_ms();

// copy `count` device words into ctx->host and wait
int readback(rk_ctx *ctx, const uint32_t *dev, uint32_t count);
// fold the launches timed during the current call into the per-kernel totals
void collect_kernel_timing(rk_ctx *ctx);
// device error bits (ERRB_*) -> status + message
int err_status(rk_ctx *ctx, uint32_t bits);

// Device scratch of the occupancy sweeps for an axis of up to m entries.
struct SweepScratch {
  uint32_t *runs;      // runs_scratch_words(m)
  uint8_t *wpend;      // m / 64 + 1
  uint8_t *rpend;      // m
  uint32_t *counters;  // PEND_WORDS
  uint32_t *dev_count; // 1
};
// run sweeps on one axis until no bucket has undecided entries
int resolve_axis(rk_ctx *ctx, const Axis &ax, SweepScratch sc, bool fast32, uint32_t *sweeps);
// `sweeps` sweeps of a 32-bit axis with no host round trip; *pend = 1 (device,
// when pend is given) when entries are still undecided after them.  junk:
// PEND_WORDS words the sweeps before the last count into, sc.counters then
// already zero (no clear per sweep); null: every sweep clears sc.counters
int resolve_axis_queued(rk_ctx *ctx, const Axis &ax, SweepScratch sc, uint32_t sweeps,
                        uint32_t *pend, uint32_t *junk = nullptr);

}  // namespace rk
