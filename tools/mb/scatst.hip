// micro-benchmark: 16-B stores, coalesced vs scattered inside a 4096-record tile
// (each tile's slots permuted: lane writes to a random slot of its tile), 50M records
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void k_copy(const uint4 *a, uint4 *b, uint32_t n) {
  const uint32_t i = blockIdx.x * 512 + threadIdx.x;
  for (int r = 0; r < 8; ++r) { uint32_t j = blockIdx.x * 4096 + r * 512 + threadIdx.x; if (j < n) b[j] = a[j]; }
}
// perm: a random permutation of 0..4095 per tile (same for every tile, rotated by tile)
__global__ void k_scat(const uint4 *a, uint4 *b, uint32_t n, const uint16_t *perm, int spread) {
  for (int r = 0; r < 8; ++r) {
    uint32_t k = r * 512 + threadIdx.x;
    uint32_t j = blockIdx.x * 4096 + k;
    if (j >= n) continue;
    uint4 v = a[j];
    uint32_t s = perm[(k + blockIdx.x * 37) & 4095];
    // spread: 256 segments of 16 slots; segment d of tile t lands at d * (n/256) + t*16 (like a radix pass)
    uint64_t dst;
    if (spread) { uint32_t d = s >> 4, o = s & 15; dst = (uint64_t)d * (n / 256 + 64) + (uint64_t)blockIdx.x * 16 + o; }
    else dst = (uint64_t)blockIdx.x * 4096 + s;
    if (dst < (uint64_t)n + 256 * 64) b[dst] = v;
  }
}
int main() {
  const uint32_t n = 50000000; uint4 *a, *b; uint16_t *p;
  (void)hipMalloc(&a, (size_t)n * 16); (void)hipMalloc(&b, (size_t)(n + 256 * 64) * 16); (void)hipMalloc(&p, 8192);
  uint16_t hp[4096]; for (int i = 0; i < 4096; ++i) hp[i] = i;
  uint64_t z = 88172645463325252ull;
  for (int i = 4095; i > 0; --i) { z ^= z << 13; z ^= z >> 7; z ^= z << 17; int j = z % (i + 1); uint16_t t = hp[i]; hp[i] = hp[j]; hp[j] = t; }
  (void)hipMemcpy(p, hp, 8192, hipMemcpyHostToDevice);
  (void)hipMemset(a, 1, (size_t)n * 16);
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1); float ms;
  const uint32_t g = (n + 4095) / 4096;
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(e0); k_copy<<<g, 512>>>(a, b, n); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1); printf("copy %.3f ms\n", ms);
    (void)hipEventRecord(e0); k_scat<<<g, 512>>>(a, b, n, p, 0); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1); printf("scatter-in-tile %.3f ms\n", ms);
    (void)hipEventRecord(e0); k_scat<<<g, 512>>>(a, b, n, p, 1); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1); printf("scatter-256-segments %.3f ms\n", ms);
  }
  return 0;
}
