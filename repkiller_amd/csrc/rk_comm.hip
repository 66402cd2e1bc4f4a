// rk_comm.hip -- rk_comm implementations: RCCL over xGMI and host callbacks.
//
// RCCL: one communicator per rank/GPU.  The all-to-all of device blocks is a
// grouped ncclSend/ncclRecv per peer (point-to-point over the xGMI links; the
// self block is a device copy); the small host all-gather is staged through a
// device buffer.  librccl.so.1 is opened on first use (RTLD_NOLOAD first, so a
// process that already loaded torch's copy shares it) -- the library itself
// has no link-time dependency on RCCL.
//
// Host callbacks: the caller's allgather / alltoallv (e.g. torch.distributed
// gloo) on host buffers; device blocks are staged through host memory.  Used by
// the multi-rank tests, which run several ranks on one GPU.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>

#include "rk_comm.h"

namespace {

// ------------------------------------------------------------------ RCCL --
struct RcclApi {
  bool ok = false;
  std::string why;
  ncclResult_t (*GetUniqueId)(ncclUniqueId *);
  ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int);
  ncclResult_t (*CommDestroy)(ncclComm_t);
  ncclResult_t (*Send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
  ncclResult_t (*Recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
  ncclResult_t (*GroupStart)();
  ncclResult_t (*GroupEnd)();
  ncclResult_t (*AllGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t,
                            hipStream_t);
  const char *(*GetErrorString)(ncclResult_t);
};

const RcclApi &rccl() {
  static RcclApi api;
  static std::once_flag once;
  std::call_once(once, [] {
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW);
    if (!h) {
      api.why = std::string("cannot load librccl.so.1: ") + dlerror();
      return;
    }
    bool all = true;
    auto sym = [&](const char *name) {
      void *p = dlsym(h, name);
      if (!p) all = false;
      return p;
    };
    api.GetUniqueId = (decltype(api.GetUniqueId))sym("ncclGetUniqueId");
    api.CommInitRank = (decltype(api.CommInitRank))sym("ncclCommInitRank");
    api.CommDestroy = (decltype(api.CommDestroy))sym("ncclCommDestroy");
    api.Send = (decltype(api.Send))sym("ncclSend");
    api.Recv = (decltype(api.Recv))sym("ncclRecv");
    api.GroupStart = (decltype(api.GroupStart))sym("ncclGroupStart");
    api.GroupEnd = (decltype(api.GroupEnd))sym("ncclGroupEnd");
    api.AllGather = (decltype(api.AllGather))sym("ncclAllGather");
    api.GetErrorString = (decltype(api.GetErrorString))sym("ncclGetErrorString");
    api.ok = all;
    if (!all) api.why = "librccl.so.1 lacks a required symbol";
  });
  return api;
}

struct RcclComm final : rk_comm {
  ncclComm_t comm = nullptr;
  int device = 0;
  void *stage = nullptr;  // all-gather staging (send block + size blocks)
  size_t stage_cap = 0;

  ~RcclComm() override {
    if (comm) (void)rccl().CommDestroy(comm);
    if (stage) (void)hipFree(stage);
  }
  int fail(const char *what, ncclResult_t r) {
    err = std::string(what) + ": " + rccl().GetErrorString(r);
    return RK_E_HIP;
  }
  int fail_hip(const char *what, hipError_t e) {
    err = std::string(what) + ": " + hipGetErrorString(e);
    return RK_E_HIP;
  }

  int allgather(const void *send, void *recv, size_t bytes, hipStream_t st) override {
    if (!bytes) return RK_OK;
    if (size == 1) {  // no peers: the gathered block is our own (no device round trip)
      std::memcpy(recv, send, bytes);
      return RK_OK;
    }
    const size_t need = bytes * (size_t)(size + 1);
    if (need > stage_cap) {
      if (stage) (void)hipFree(stage);
      stage = nullptr;
      stage_cap = 0;
      hipError_t e = hipMalloc(&stage, need);
      if (e != hipSuccess) return fail_hip("hipMalloc", e);
      stage_cap = need;
    }
    char *s = (char *)stage;
    hipError_t e = hipMemcpyAsync(s, send, bytes, hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return fail_hip("hipMemcpyAsync", e);
    ncclResult_t r = rccl().AllGather(s, s + bytes, bytes, ncclUint8, comm, st);
    if (r != ncclSuccess) return fail("ncclAllGather", r);
    e = hipMemcpyAsync(recv, s + bytes, bytes * size, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return fail_hip("hipMemcpyAsync", e);
    return RK_OK;
  }

  // the message is gathered on the device (no host-to-device leg) and comes
  // down in one copy: a single wait for the stream
  int allgather_dev(const void *dsend, void *recv, size_t bytes, hipStream_t st) override {
    if (!bytes) return RK_OK;
    hipError_t e;
    if (size == 1) {
      e = hipMemcpyAsync(recv, dsend, bytes, hipMemcpyDeviceToHost, st);
    } else {
      const size_t need = bytes * (size_t)size;
      if (need > stage_cap) {
        if (stage) (void)hipFree(stage);
        stage = nullptr;
        stage_cap = 0;
        e = hipMalloc(&stage, need);
        if (e != hipSuccess) return fail_hip("hipMalloc", e);
        stage_cap = need;
      }
      ncclResult_t r = rccl().AllGather(dsend, stage, bytes, ncclUint8, comm, st);
      if (r != ncclSuccess) return fail("ncclAllGather", r);
      e = hipMemcpyAsync(recv, stage, need, hipMemcpyDeviceToHost, st);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return fail_hip("hipMemcpyAsync", e);
    return RK_OK;
  }

  int alltoallv(const void *send, const uint64_t *sb, void *recv, const uint64_t *rb,
                hipStream_t st) override {
    const RcclApi &api = rccl();
    size_t so = 0, ro = 0;
    ncclResult_t r = api.GroupStart();
    if (r != ncclSuccess) return fail("ncclGroupStart", r);
    for (int q = 0; q < size; ++q) {
      if (q != rank) {
        if (sb[q] && (r = api.Send((const char *)send + so, sb[q], ncclUint8, q, comm, st)) !=
                         ncclSuccess)
          break;
        if (rb[q] && (r = api.Recv((char *)recv + ro, rb[q], ncclUint8, q, comm, st)) !=
                         ncclSuccess)
          break;
      }
      so += sb[q];
      ro += rb[q];
    }
    ncclResult_t r2 = api.GroupEnd();
    if (r != ncclSuccess) return fail("ncclSend/ncclRecv", r);
    if (r2 != ncclSuccess) return fail("ncclGroupEnd", r2);
    // the block to ourselves
    so = ro = 0;
    for (int q = 0; q < rank; ++q) so += sb[q], ro += rb[q];
    if (sb[rank] != rb[rank]) {
      err = "alltoallv: self block sizes differ";
      return RK_E_INTERNAL;
    }
    if (sb[rank]) {
      hipError_t e = hipMemcpyAsync((char *)recv + ro, (const char *)send + so, sb[rank],
                                    hipMemcpyDeviceToDevice, st);
      if (e != hipSuccess) return fail_hip("hipMemcpyAsync", e);
    }
    return RK_OK;
  }
};

// -------------------------------------------------------- host callbacks --
struct HostComm final : rk_comm {
  rk_comm_host_ops ops{};
  std::vector<char> hs, hr;

  int allgather(const void *send, void *recv, size_t bytes, hipStream_t) override {
    if (ops.allgather(ops.user, send, recv, bytes) != 0) {
      err = "host allgather callback failed";
      return RK_E_INTERNAL;
    }
    return RK_OK;
  }

  int alltoallv(const void *send, const uint64_t *sb, void *recv, const uint64_t *rb,
                hipStream_t st) override {
    size_t ts = 0, tr = 0;
    for (int q = 0; q < size; ++q) ts += sb[q], tr += rb[q];
    hs.resize(ts + 1);
    hr.resize(tr + 1);
    hipError_t e = hipSuccess;
    if (ts) e = hipMemcpyAsync(hs.data(), send, ts, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
      err = std::string("alltoallv staging: ") + hipGetErrorString(e);
      return RK_E_HIP;
    }
    if (ops.alltoallv(ops.user, hs.data(), sb, hr.data(), rb) != 0) {
      err = "host alltoallv callback failed";
      return RK_E_INTERNAL;
    }
    if (tr) e = hipMemcpyAsync(recv, hr.data(), tr, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
      err = std::string("alltoallv staging: ") + hipGetErrorString(e);
      return RK_E_HIP;
    }
    return RK_OK;
  }
};

// ------------------------------------------------------ in-process group --
// P threads of one process, one GPU each (or all on one GPU): every rank
// publishes its buffer, a barrier, every rank copies what it needs from the
// others' buffers (device blocks: hipMemcpyDefault, peer copies over xGMI when
// the ranks sit on different GPUs), a second barrier frees the buffers.
struct LocalShared {
  int size;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t generation = 0;
  std::vector<const void *> ptr;
  std::vector<const uint64_t *> counts;
  explicit LocalShared(int p) : size(p), ptr(p), counts(p) {}
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    const uint64_t g = generation;
    if (++arrived == size) {
      arrived = 0;
      ++generation;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return generation != g; });
    }
  }
};

struct LocalComm final : rk_comm {
  std::shared_ptr<LocalShared> sh;

  int allgather(const void *send, void *recv, size_t bytes, hipStream_t) override {
    sh->ptr[rank] = send;
    sh->barrier();
    for (int q = 0; q < size; ++q)
      if (bytes) std::memcpy((char *)recv + (size_t)q * bytes, sh->ptr[q], bytes);
    sh->barrier();
    return RK_OK;
  }

  int alltoallv(const void *send, const uint64_t *sb, void *recv, const uint64_t *rb,
                hipStream_t st) override {
    // the send blocks were written by kernels on this rank's stream: complete
    // them before another rank copies out of them
    hipError_t e = hipStreamSynchronize(st);
    sh->ptr[rank] = send;
    sh->counts[rank] = sb;
    sh->barrier();
    size_t ro = 0;
    for (int q = 0; q < size && e == hipSuccess; ++q) {
      const uint64_t *qsb = sh->counts[q];
      size_t so = 0;
      for (int r = 0; r < rank; ++r) so += qsb[r];
      if (qsb[rank] != rb[q]) {
        e = hipErrorInvalidValue;
        break;
      }
      if (rb[q])
        e = hipMemcpyAsync((char *)recv + ro, (const char *)sh->ptr[q] + so, rb[q],
                           hipMemcpyDefault, st);
      ro += rb[q];
    }
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    sh->barrier();  // every rank has copied out of every send buffer
    if (e != hipSuccess) {
      err = std::string("local alltoallv: ") + hipGetErrorString(e);
      return RK_E_HIP;
    }
    return RK_OK;
  }
};

}  // namespace

extern "C" int rk_comm_create_local(int size, rk_comm **comms) {
  if (!comms || size < 1 || size > 32) return RK_E_ARG;
  auto sh = std::make_shared<LocalShared>(size);
  for (int r = 0; r < size; ++r) {
    auto c = new (std::nothrow) LocalComm;
    if (!c) {
      for (int q = 0; q < r; ++q) delete comms[q];
      return RK_E_NOMEM;
    }
    c->rank = r;
    c->size = size;
    c->sh = sh;
    comms[r] = c;
  }
  return RK_OK;
}

extern "C" int rk_comm_create_host(int rank, int size, const rk_comm_host_ops *ops,
                                   rk_comm **comm) {
  if (!comm || !ops || !ops->allgather || !ops->alltoallv || size < 1 || size > 32 ||
      rank < 0 || rank >= size)
    return RK_E_ARG;
  auto c = new (std::nothrow) HostComm;
  if (!c) return RK_E_NOMEM;
  c->rank = rank;
  c->size = size;
  c->ops = *ops;
  *comm = c;
  return RK_OK;
}

extern "C" int rk_comm_rccl_id(uint8_t id[RK_COMM_ID_BYTES]) {
  static_assert(sizeof(ncclUniqueId) == RK_COMM_ID_BYTES, "ncclUniqueId size");
  if (!id) return RK_E_ARG;
  const RcclApi &api = rccl();
  if (!api.ok) return RK_E_NODEVICE;
  ncclUniqueId u;
  if (api.GetUniqueId(&u) != ncclSuccess) return RK_E_HIP;
  std::memcpy(id, &u, sizeof u);
  return RK_OK;
}

extern "C" int rk_comm_create_rccl(int rank, int size, int device,
                                   const uint8_t id[RK_COMM_ID_BYTES], rk_comm **comm) {
  if (!comm || !id || size < 1 || size > 32 || rank < 0 || rank >= size) return RK_E_ARG;
  *comm = nullptr;
  const RcclApi &api = rccl();
  if (!api.ok) return RK_E_NODEVICE;
  if (hipSetDevice(device) != hipSuccess) return RK_E_NODEVICE;
  auto c = new (std::nothrow) RcclComm;
  if (!c) return RK_E_NOMEM;
  c->rank = rank;
  c->size = size;
  c->device = device;
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof u);
  const ncclResult_t r = api.CommInitRank(&c->comm, size, u, rank);
  std::fflush(stdout);  // RCCL's init banner, while the caller may redirect stdout
  if (r != ncclSuccess) {
    c->comm = nullptr;
    delete c;
    return RK_E_HIP;
  }
  *comm = c;
  return RK_OK;
}

extern "C" void rk_comm_destroy(rk_comm *comm) { delete comm; }

extern "C" const char *rk_comm_last_error(const rk_comm *comm) {
  return comm ? comm->err.c_str() : "";
}
