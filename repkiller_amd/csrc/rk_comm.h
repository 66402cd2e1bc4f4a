// rk_comm.h -- collectives behind rk_comm (internal).
//
// The sharded driver needs two collectives: an all-gather of small HOST
// metadata (counts, histograms, flags) and an all-to-all of variable-size
// DEVICE byte blocks (fragment rows, halo records, parents, members).  RCCL
// implements the all-to-all as grouped point-to-point send/recv over xGMI;
// the host-callback flavour stages through host memory for tests.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/repkiller_amd.h"

struct rk_comm {
  int rank = 0, size = 1;
  std::string err;
  virtual ~rk_comm() {}
  // recv (size * bytes host bytes) = every rank's `send`, in rank order
  virtual int allgather(const void *send, void *recv, size_t bytes, hipStream_t st) = 0;
  // the same with `send` in DEVICE memory, written by work queued on st: one
  // wait for the stream in all (RCCL gathers on the device and copies the
  // result down; the host flavours copy the block down and gather on the host)
  virtual int allgather_dev(const void *dsend, void *recv, size_t bytes, hipStream_t st) {
    std::vector<char> h(bytes);
    hipError_t e = hipMemcpyAsync(h.data(), dsend, bytes, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
      err = std::string("allgather_dev staging: ") + hipGetErrorString(e);
      return RK_E_HIP;
    }
    return allgather(h.data(), recv, bytes, st);
  }
  // device blocks; send_bytes / recv_bytes have `size` entries, blocks packed
  // in rank order; enqueued on / synchronised with st
  virtual int alltoallv(const void *send, const uint64_t *send_bytes, void *recv,
                        const uint64_t *recv_bytes, hipStream_t st) = 0;
};
