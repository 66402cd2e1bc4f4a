// rk_io.hip -- the host side of rk_classify: host buffers <-> HBM.
//
// The reference classifies fragments that live in host memory
// (FragmentsDatabase, FragmentsDatabase.cpp:84-97) and writes host-side
// results (save_frag_pair, commonFunctions.cpp:119-129).  rk_classify keeps
// that boundary: caller-owned host SoA in, caller-owned host results out.
//
// Transfers run on a dedicated copy stream.  Page-locked caller buffers
// (hipHostMalloc / hipHostRegister, e.g. the rk_db loader's columns) are
// copied by DMA directly.  Pageable buffers go through a ring of pinned
// staging slots: host threads copy chunk k into a free slot while the DMA
// engine moves chunk k-1 (and, for results, the DMA of chunk k+NS overlaps the
// host copy of chunk k out of its slot).  HIP's own pageable path stages
// through one thread; the parallel host copy is what lifts it to PCIe rate.
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "rk_ctx.h"

namespace rk {

// A fixed set of worker threads running one job at a time: job(t) on every
// worker t in [0, n); run() returns when all have finished.
class HostPool {
 public:
  explicit HostPool(int n) : n_(n) {
    for (int t = 0; t < n_; ++t) th_.emplace_back([this, t] { loop(t); });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : th_) t.join();
  }
  int size() const { return n_; }
  void run(const std::function<void(int)> &job) {
    std::unique_lock<std::mutex> g(mu_);
    job_ = &job;
    left_ = n_;
    ++gen_;
    cv_.notify_all();
    done_.wait(g, [this] { return left_ == 0; });
    job_ = nullptr;
  }

 private:
  void loop(int t) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)> *job;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        job = job_;
      }
      (*job)(t);
      std::lock_guard<std::mutex> g(mu_);
      if (--left_ == 0) done_.notify_one();
    }
  }
  int n_;
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  const std::function<void(int)> *job_ = nullptr;
  uint64_t gen_ = 0;
  int left_ = 0;
  bool stop_ = false;
};

namespace {

constexpr int NSLOT = 4;
constexpr size_t PF_ROWS = 512;  // rows of u64 columns in one 4-KB page
constexpr size_t SLOT = (size_t)32 << 20;

int io_threads() {
  const char *e = std::getenv("RK_IO_THREADS");
  int n = e ? std::atoi(e) : 0;
  if (n <= 0) {
    const char *o = std::getenv("OMP_NUM_THREADS");  // the box's CPU share
    n = o ? std::atoi(o) : 0;
  }
  if (n <= 0) n = (int)std::thread::hardware_concurrency();
  return std::max(1, std::min(n, 16));
}

// copy len bytes with every pool worker (pieces of at least 1 MiB)
void par_copy(HostPool *pool, void *dst, const void *src, size_t len) {
  const size_t piece = std::max<size_t>((len + pool->size() - 1) / pool->size(), (size_t)1 << 20);
  const std::function<void(int)> job = [&](int t) {
    const size_t a = (size_t)t * piece;
    if (a >= len) return;
    std::memcpy((char *)dst + a, (const char *)src + a, std::min(piece, len - a));
  };
  if (len <= piece) std::memcpy(dst, src, len);
  else pool->run(job);
}

// ---- NUMA placement of the host side (a two-socket host: the caller's pages,
// the packing threads, the staging slots and the GPU may sit on different
// nodes).  No libnuma: move_pages(2) with no target nodes reports the node of
// each page, sysfs the CPUs of a node and the node of the GPU's PCI device.

// the majority node of up to 16 pages sampled over [p, p + bytes); -1 when
// none is resident (or the query is unavailable)
int range_node(const void *p, size_t bytes) {
  if (!p || !bytes) return -1;
  constexpr int K = 16;
  void *pages[K];
  int status[K];
  const long psz = sysconf(_SC_PAGESIZE);
  for (int k = 0; k < K; ++k) {
    const uintptr_t a = (uintptr_t)p + (uintptr_t)(bytes / K) * (uintptr_t)k;
    pages[k] = (void *)(a & ~(uintptr_t)(psz - 1));
  }
  if (syscall(SYS_move_pages, 0, (unsigned long)K, pages, nullptr, status, 0) != 0) return -1;
  int best = -1, bestc = 0;
  for (int k = 0; k < K; ++k) {
    if (status[k] < 0) continue;
    int c = 0;
    for (int j = 0; j < K; ++j) c += status[j] == status[k];
    if (c > bestc) best = status[k], bestc = c;
  }
  return best;
}

// CPUs of NUMA node `node` (sysfs cpulist "0-15,64-79"); false when unknown
static bool node_cpus(int node, cpu_set_t *set) {
  CPU_ZERO(set);
  char path[96];
  std::snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
  FILE *f = std::fopen(path, "r");
  if (!f) return false;
  char buf[4096];
  const size_t len = std::fread(buf, 1, sizeof buf - 1, f);
  std::fclose(f);
  buf[len] = 0;
  bool any = false;
  for (char *q = buf; *q;) {
    if (!std::isdigit((unsigned char)*q)) {
      ++q;
      continue;
    }
    long a = std::strtol(q, &q, 10), b = a;
    if (*q == '-') b = std::strtol(q + 1, &q, 10);
    for (long c = a; c <= b && c < CPU_SETSIZE; ++c) CPU_SET((int)c, set), any = true;
  }
  return any;
}

// the node of the device's PCI function (sysfs), -1 when unknown
static int device_node(int device) {
  char bus[64] = {};
  if (hipDeviceGetPCIBusId(bus, sizeof bus, device) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  for (char *c = bus; *c; ++c) *c = (char)std::tolower((unsigned char)*c);
  char path[160];
  std::snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
  FILE *f = std::fopen(path, "r");
  if (!f) return -1;
  int node = -1;
  if (std::fscanf(f, "%d", &node) != 1) node = -1;
  std::fclose(f);
  return node;
}

// RK_IO_NUMA=0: leave the packing threads where the scheduler puts them
bool numa_bind_enabled() {
  static const bool on = [] {
    const char *e = std::getenv("RK_IO_NUMA");
    return !(e && e[0] == '0');
  }();
  return on;
}

}  // namespace

struct IoEngine {
  hipStream_t io = nullptr;
  char *slot[NSLOT] = {};
  hipEvent_t ev[NSLOT] = {};
  HostPool *pool = nullptr;
  cpu_set_t allowed;      // the process' CPUs when the engine was built
  int bound = -1;         // node the pool threads are bound to (-1: not bound)
  int last_input = -1;    // node of the last upload's input pages
  int staging = -1;       // node of the pinned staging slots
  int gpu = -1;           // node of the device
  // bind the pool's threads to the CPUs of `node` that this process may use
  // (nothing to bind to, or RK_IO_NUMA=0: they stay unbound)
  void bind(int node) {
    if (node == bound || !numa_bind_enabled()) return;
    cpu_set_t set;
    if (node < 0 || !node_cpus(node, &set)) return;
    CPU_AND(&set, &set, &allowed);
    if (CPU_COUNT(&set) == 0) return;
    const std::function<void(int)> job = [&](int) {
      (void)sched_setaffinity(0, sizeof set, &set);  // (0: the calling thread)
    };
    pool->run(job);
    bound = node;
  }
  // before packing the caller's rows / copying its pages: the threads go to
  // the node that holds them
  void place(const void *p, size_t bytes) {
    last_input = range_node(p, bytes);
    bind(last_input);
  }
  ~IoEngine() {
    if (io) (void)hipStreamSynchronize(io);
    for (auto &e : ev)
      if (e) (void)hipEventDestroy(e);
    for (auto &s : slot)
      if (s) (void)hipHostFree(s);
    if (io) (void)hipStreamDestroy(io);
    delete pool;
  }
};

void io_destroy(rk_ctx *ctx) {
  delete ctx->ioe;
  ctx->ioe = nullptr;
}

// The engine is built aside and published only when every resource exists: a
// failed pinned allocation returns RK_E_HIP now and is retried by the next
// call, instead of leaving a half-built engine (null slots / stream) behind.
static int io_build(rk_ctx *ctx, IoEngine *e) {
  HIPCHK(ctx, hipStreamCreateWithFlags(&e->io, hipStreamNonBlocking));
  for (int k = 0; k < NSLOT; ++k) {
    HIPCHK(ctx, hipHostMalloc((void **)&e->slot[k], SLOT, hipHostMallocDefault));
    HIPCHK(ctx, hipEventCreateWithFlags(&e->ev[k], hipEventDisableTiming));
  }
  e->pool = new HostPool(io_threads());
  CPU_ZERO(&e->allowed);
  if (sched_getaffinity(0, sizeof e->allowed, &e->allowed) != 0) CPU_ZERO(&e->allowed);
  e->staging = range_node(e->slot[0], SLOT);
  e->gpu = device_node(ctx->device);
  return RK_OK;
}

void io_numa_stats(const rk_ctx *ctx, rk_stats *st) {
  const IoEngine *e = ctx->ioe;
  st->numa_input = e ? e->last_input : -1;
  st->numa_threads = e ? e->bound : -1;
  st->numa_staging = e ? e->staging : -1;
  st->numa_gpu = e ? e->gpu : -1;
}

static int io_ready(rk_ctx *ctx) {
  if (ctx->ioe) return RK_OK;
  auto *e = new IoEngine;
  const int rc = io_build(ctx, e);
  if (rc) {
    delete e;  // the destructor skips the members that were never created
    return rc;
  }
  ctx->ioe = e;
  return RK_OK;
}

bool host_pinned(const void *p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // an unregistered pointer: pageable
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

// Host -> device for several (dst, src, bytes) pieces, one pipeline; returns
// when the last byte has landed.
int io_h2d(rk_ctx *ctx, const std::vector<IoPiece> &pieces) {
  int rc = io_ready(ctx);
  if (rc) return rc;
  IoEngine &e = *ctx->ioe;
  for (const IoPiece &pc : pieces)
    if (pc.bytes && !host_pinned(pc.host)) {
      e.place(pc.host, pc.bytes);  // (the first pageable column decides)
      break;
    }
  bool busy[NSLOT] = {};
  int k = 0;
  for (const IoPiece &pc : pieces) {
    if (!pc.bytes) continue;
    if (host_pinned(pc.host)) {
      HIPCHK(ctx, hipMemcpyAsync(pc.dev, pc.host, pc.bytes, hipMemcpyHostToDevice, e.io));
      continue;
    }
    for (size_t off = 0; off < pc.bytes; off += SLOT) {
      const size_t len = std::min(SLOT, pc.bytes - off);
      if (busy[k]) HIPCHK(ctx, hipEventSynchronize(e.ev[k]));
      par_copy(e.pool, e.slot[k], (const char *)pc.host + off, len);
      HIPCHK(ctx, hipMemcpyAsync((char *)pc.dev + off, e.slot[k], len, hipMemcpyHostToDevice,
                                 e.io));
      HIPCHK(ctx, hipEventRecord(e.ev[k], e.io));
      busy[k] = true;
      k = (k + 1) % NSLOT;
    }
  }
  HIPCHK(ctx, hipStreamSynchronize(e.io));
  return RK_OK;
}

// Device -> host: the DMA of up to NSLOT chunks runs ahead of the host copies
// out of the slots.
int io_d2h(rk_ctx *ctx, const std::vector<IoPiece> &pieces) {
  int rc = io_ready(ctx);
  if (rc) return rc;
  IoEngine &e = *ctx->ioe;
  struct Chunk {
    void *host;
    const void *dev;
    size_t len;
  };
  std::vector<Chunk> ch;
  for (const IoPiece &pc : pieces) {
    if (!pc.bytes) continue;
    if (host_pinned(pc.host)) {
      HIPCHK(ctx, hipMemcpyAsync(pc.host, pc.dev, pc.bytes, hipMemcpyDeviceToHost, e.io));
      continue;
    }
    for (size_t off = 0; off < pc.bytes; off += SLOT)
      ch.push_back({(char *)pc.host + off, (const char *)pc.dev + off,
                    std::min(SLOT, pc.bytes - off)});
  }
  const size_t nc = ch.size();
  auto issue = [&](size_t i) -> int {
    const int k = (int)(i % NSLOT);
    HIPCHK(ctx, hipMemcpyAsync(e.slot[k], ch[i].dev, ch[i].len, hipMemcpyDeviceToHost, e.io));
    HIPCHK(ctx, hipEventRecord(e.ev[k], e.io));
    return RK_OK;
  };
  for (size_t i = 0; i < nc && i < (size_t)NSLOT; ++i)
    if ((rc = issue(i))) return rc;
  for (size_t i = 0; i < nc; ++i) {
    const int k = (int)(i % NSLOT);
    HIPCHK(ctx, hipEventSynchronize(e.ev[k]));
    par_copy(e.pool, ch[i].host, e.slot[k], ch[i].len);
    if (i + NSLOT < nc && (rc = issue(i + NSLOT))) return rc;
  }
  HIPCHK(ctx, hipStreamSynchronize(e.io));
  return RK_OK;
}

int io_h2d_rows(rk_ctx *ctx, const rk_frags_soa &in, void *dev) {
  int rc = io_ready(ctx);
  if (rc) return rc;
  IoEngine &e = *ctx->ioe;
  const size_t n = in.n, per = SLOT / 12;
  e.place(in.x_start, n * 8);  // the threads read the caller's columns
  bool busy[NSLOT] = {};
  int k = 0;
  std::atomic<bool> bad{false};
  for (size_t a = 0; a < n; a += per) {
    const size_t cnt = std::min(per, n - a);
    if (busy[k]) HIPCHK(ctx, hipEventSynchronize(e.ev[k]));
    uint32_t *slot = reinterpret_cast<uint32_t *>(e.slot[k]);
    const size_t share = (cnt + e.pool->size() - 1) / e.pool->size();
    const std::function<void(int)> job = [&](int t) {
      const size_t lo = (size_t)t * share, hi = std::min(cnt, lo + share);
      bool ok = true;
      for (size_t i = lo; i < hi; ++i) {
        // software prefetch one 4-KB page ahead in each column: the hardware
        // streamers stop at page boundaries, and page-locked buffers (torch
        // pin_memory, hipHostMalloc) come in 4-KB pages where pageable ones
        // are mostly transparent huge pages
        if ((i & 7) == 0) {
          const size_t f = a + i + PF_ROWS;
          __builtin_prefetch(in.x_start + f);
          __builtin_prefetch(in.y_start + f);
          __builtin_prefetch(in.length + f);
          if ((i & 63) == 0) __builtin_prefetch(in.strand + f);
        }
        const uint64_t x = in.x_start[a + i], y = in.y_start[a + i], L = in.length[a + i];
        ok &= L < (1ull << 24) && y < (1ull << 35) && x < (1ull << 36);
        const uint32_t s = in.strand[a + i] != 'f' ? 1u : 0u;
        uint32_t *r = slot + 3 * i;
        r[0] = (uint32_t)x;
        r[1] = (uint32_t)y;
        r[2] = (uint32_t)(L & 0xFFFFFFu) | s << 24 | (uint32_t)((y >> 32) & 7u) << 25 |
               (uint32_t)((x >> 32) & 15u) << 28;
      }
      if (!ok) bad = true;
    };
    e.pool->run(job);
    if (bad) {
      HIPCHK(ctx, hipStreamSynchronize(e.io));
      return 1;
    }
    HIPCHK(ctx, hipMemcpyAsync((char *)dev + a * 12, slot, cnt * 12, hipMemcpyHostToDevice, e.io));
    HIPCHK(ctx, hipEventRecord(e.ev[k], e.io));
    busy[k] = true;
    k = (k + 1) % NSLOT;
  }
  HIPCHK(ctx, hipStreamSynchronize(e.io));
  return RK_OK;
}

// two phases on `threads` threads (counts per range, then the fill); the
// phases meet at a spin barrier on an atomic counter
void gids_from_flags_async(const uint8_t *flag, size_t n, uint32_t *gid, int threads, GidJob &job) {
  if (!n) return;
  const int T = threads < 1 ? 1 : threads;
  const size_t share = (n + T - 1) / T;
  auto cnt = std::make_shared<std::vector<uint32_t>>(T + 1, 0u);
  auto arrived = std::make_shared<std::atomic<int>>(0);
  int started = 0;
  try {
    for (int t = 0; t < T; ++t, ++started)
      job.th.emplace_back([=] {
      const size_t lo = std::min(n, (size_t)t * share), hi = std::min(n, lo + share);
      uint32_t c = 0;
      for (size_t i = lo; i < hi; ++i) c += flag[i] != 2;
      (*cnt)[t + 1] = c;
      arrived->fetch_add(1, std::memory_order_acq_rel);
      while (arrived->load(std::memory_order_acquire) < T) std::this_thread::yield();
      uint32_t g = 0;
      for (int k = 0; k <= t; ++k) g += (*cnt)[k];
      for (size_t i = lo; i < hi; ++i) {
        g += flag[i] != 2;
        gid[i] = g - 1;
      }
    });
  } catch (...) {
    // a thread could not be started: release the ones already waiting at the
    // barrier (their partial counts give wrong gids), join them, and rebuild
    // every gid here -- no exception crosses the C ABI, nothing spins forever
    arrived->fetch_add(T - started, std::memory_order_acq_rel);
    job.wait();
    uint32_t g = 0;
    for (size_t i = 0; i < n; ++i) {
      g += flag[i] != 2;
      gid[i] = g - 1;
    }
  }
}

double wall_ms() {
  return std::chrono::duration<double, std::milli>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

}  // namespace rk
