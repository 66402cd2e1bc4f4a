// micro-benchmark: unstable bin scatter of 16-B records by returning atomics
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cstdint>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_gen(uint4 *r, uint32_t n, uint32_t keymax) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    uint64_t z = (uint64_t)i * 0x9e3779b97f4a7c15ull + 12345;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull; z = (z ^ (z >> 27)) * 0x94d049bb133111ebull; z ^= z >> 31;
    r[i] = make_uint4((uint32_t)(z % keymax), i, (uint32_t)(z >> 32), 7);
  }
}
__global__ void k_hist(const uint4 *r, uint32_t n, int s, uint32_t *cnt) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    atomicAdd(&cnt[r[i].x >> s], 1u);
}
__global__ void k_scatter(const uint4 *r, uint32_t n, int s, uint32_t *cur, uint4 *out) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint4 v = r[i];
    const uint32_t p = atomicAdd(&cur[v.x >> s], 1u);
    out[p] = v;
  }
}
// wave-aggregated: lanes with the same bin share one atomic (match by ballots)
__global__ void k_scatter_agg(const uint4 *r, uint32_t n, int s, int bb, uint32_t *cur, uint4 *out) {
  const int lane = threadIdx.x & 63;
  for (uint32_t i0 = blockIdx.x * blockDim.x; i0 < n; i0 += gridDim.x * blockDim.x) {
    const uint32_t i = i0 + threadIdx.x;
    const bool live = i < n;
    const uint4 v = live ? r[i] : make_uint4(0, 0, 0, 0);
    const uint32_t b = v.x >> s;
    uint64_t peer = __ballot(live);
    for (int k = 0; k < bb; ++k) { const bool bit = (b >> k) & 1; const uint64_t m = __ballot(bit); peer &= bit ? m : ~m; }
    const int leader = __builtin_ctzll(peer);
    const uint32_t below = __popcll(peer & ((1ull << lane) - 1));
    uint32_t base = 0;
    if (live && lane == leader) base = atomicAdd(&cur[b], (uint32_t)__popcll(peer));
    base = __shfl(base, leader);
    if (live) out[base + below] = v;
  }
}
__global__ void k_copy(const uint4 *r, uint32_t n, uint4 *out) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) out[i] = r[i];
}
int main(int argc, char **argv) {
  const uint32_t n = 50000000, keymax = 300000000;
  uint4 *a, *b; uint32_t *cnt, *cur;
  CK(hipMalloc(&a, (size_t)n * 16)); CK(hipMalloc(&b, (size_t)n * 16));
  CK(hipMalloc(&cnt, 4u << 20)); CK(hipMalloc(&cur, 4u << 20));
  k_gen<<<4096, 256>>>(a, n, keymax);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  float ms;
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0); k_copy<<<8192, 256>>>(a, n, b); hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1); printf("copy %.3f ms\n", ms);
  }
  for (int s = 11; s <= 15; ++s) {
    const uint32_t nb = (keymax >> s) + 1;
    CK(hipMemset(cnt, 0, nb * 4));
    hipEventRecord(e0); k_hist<<<8192, 256>>>(a, n, s, cnt); hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<uint32_t> h(nb); CK(hipMemcpy(h.data(), cnt, nb * 4, hipMemcpyDeviceToHost));
    uint32_t mx = 0, acc = 0; for (uint32_t j = 0; j < nb; ++j) { uint32_t c = h[j]; h[j] = acc; acc += c; if (c > mx) mx = c; }
    printf("s=%d bins=%u avg=%.0f max=%u hist %.3f ms\n", s, nb, (double)n / nb, mx, ms);
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipMemcpy(cur, h.data(), nb * 4, hipMemcpyHostToDevice));
      hipEventRecord(e0); k_scatter<<<8192, 256>>>(a, n, s, cur, b); hipEventRecord(e1); hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1); printf("  scatter %.3f ms\n", ms);
    }
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipMemcpy(cur, h.data(), nb * 4, hipMemcpyHostToDevice));
      int bb = 0; while ((1u << bb) < nb) ++bb;
      hipEventRecord(e0); k_scatter_agg<<<8192, 256>>>(a, n, s, bb, cur, b); hipEventRecord(e1); hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1); printf("  scatter_agg %.3f ms\n", ms);
    }
  }
  CK(hipDeviceSynchronize());
  return 0;
}
