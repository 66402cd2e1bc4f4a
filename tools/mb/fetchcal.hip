// fetchcal.hip -- calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950
// for the access widths of the record pipeline (MI355X_MICROARCH.md: only
// 16-B/lane streaming reads and stores are calibrated there).  Every kernel
// moves a KNOWN byte count (1 GiB, well past the 256-MiB Infinity Cache, so
// nothing is served on-die); tools/pmc_summary.py --calib divides the counter
// by it.
//
//   r16   16-B/lane reads (uint4)            -- the guide's reference case
//   r12   12-B records, three dword loads per lane (rk_narrow.hip SrcRec12)
//   r8    8-B/lane reads (the file-order SoA columns)
//   r4    4-B/lane reads
//   r1    1-B/lane reads (the strand column)
//   r4a   4-B/lane agent-scope atomic loads (the look-back's status words)
//   w16   16-B/lane stores
//   w12   12-B records, three dword stores per lane (DstRec12)
//   w4    4-B/lane stores
//   w1    1-B/lane stores
//   seg16 16-B records written as digit segments of ~24 records each at
//         scattered offsets (the one-sweep write-out's pattern)
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/mb/fetchcal.hip -o tools/mb/fetchcal
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                  \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));               \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

template <class T>
__global__ void k_read(const T *__restrict__ in, size_t n, uint32_t *__restrict__ sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const T v = __builtin_nontemporal_load(in + i);
    acc ^= (uint32_t)v;
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;  // keeps the loads
}
__global__ void k_read16(const v4u *__restrict__ in, size_t n, uint32_t *__restrict__ sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const v4u v = __builtin_nontemporal_load(in + i);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}
__global__ void k_read12(const uint32_t *__restrict__ in, size_t n, uint32_t *__restrict__ sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const uint32_t *p = in + 3 * i;
    acc ^= __builtin_nontemporal_load(p) ^ __builtin_nontemporal_load(p + 1) ^
           __builtin_nontemporal_load(p + 2);
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}
// 4-B/lane agent-scope atomic loads (the one-sweep look-back's status reads)
__global__ void k_read4a(const uint32_t *__restrict__ in, size_t n, uint32_t *__restrict__ sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    acc ^= __hip_atomic_load(in + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (acc == 0x9e3779b9u) sink[0] = acc;
}
template <class T>
__global__ void k_write(T *__restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    out[i] = (T)i;
}
__global__ void k_write16(v4u *__restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const uint32_t v = (uint32_t)i;
    out[i] = v4u{v, v + 1, v + 2, v + 3};
  }
}
__global__ void k_write12(uint32_t *__restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    uint32_t *p = out + 3 * i;
    p[0] = (uint32_t)i, p[1] = (uint32_t)i + 1, p[2] = (uint32_t)i + 2;
  }
}
// digit segments: segment s (SEG records) goes to a pseudo-random slot of the
// output, every record once (a permutation of segments)
constexpr int SEG = 24;
__global__ void k_seg16(v4u *__restrict__ out, size_t nseg) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nseg * SEG;
       i += (size_t)gridDim.x * blockDim.x) {
    const size_t s = i / SEG, j = i % SEG;
    const size_t d = (s * 7919ull) % nseg;  // nseg coprime with 7919: a bijection
    const uint32_t v = (uint32_t)i;
    out[d * SEG + j] = v4u{v, v, v, v};
  }
}

int main() {
  const size_t bytes = (size_t)1 << 30;  // 1 GiB per kernel
  void *a = nullptr;
  uint32_t *sink = nullptr;
  CHK(hipMalloc(&a, bytes + 4096));
  CHK(hipMalloc(&sink, 64));
  CHK(hipMemset(a, 1, bytes + 4096));
  const int grid = 256 * 32, blk = 256;
  for (int rep = 0; rep < 2; ++rep) {  // the second repetition is the one to read
    k_read16<<<grid, blk>>>((const v4u *)a, bytes / 16, sink);
    k_read12<<<grid, blk>>>((const uint32_t *)a, bytes / 12, sink);
    k_read<uint64_t><<<grid, blk>>>((const uint64_t *)a, bytes / 8, sink);
    k_read<uint32_t><<<grid, blk>>>((const uint32_t *)a, bytes / 4, sink);
    k_read<uint8_t><<<grid, blk>>>((const uint8_t *)a, bytes, sink);
    k_read4a<<<grid, blk>>>((const uint32_t *)a, bytes / 4, sink);
    k_write16<<<grid, blk>>>((v4u *)a, bytes / 16);
    k_write12<<<grid, blk>>>((uint32_t *)a, bytes / 12);
    k_write<uint32_t><<<grid, blk>>>((uint32_t *)a, bytes / 4);
    k_write<uint8_t><<<grid, blk>>>((uint8_t *)a, bytes);
    size_t nseg = bytes / 16 / SEG;
    while (nseg % 7919 == 0) --nseg;
    k_seg16<<<grid, blk>>>((v4u *)a, nseg);
  }
  CHK(hipDeviceSynchronize());
  std::printf("{\"bytes_per_kernel\": %zu}\n", bytes);
  return 0;
}
