// Shader clock seen by a lone wavefront vs a full grid: s_memtime (shader
// clock) against s_memrealtime (100 MHz) around a chain of dependent VALU and
// SALU adds.  Build: hipcc --offload-arch=gfx950 -O3 clockprobe.hip -o clockprobe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_probe(unsigned long long *out, int iters, int salu) {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  unsigned v = threadIdx.x;
  if (salu) {
    unsigned s = __builtin_amdgcn_readfirstlane(v);
    for (int i = 0; i < iters; ++i) asm volatile("s_mul_i32 %0, %0, 3" : "+s"(s));  // (no SCC write: the loop branch reads SCC)
    v += s;
  } else {
    for (int i = 0; i < iters; ++i) asm volatile("v_add_u32 %0, %0, 1" : "+v"(v));
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    out[0] = t1 - t0;
    out[1] = r1 - r0;
    out[2] = v;
  }
}

int main() {
  unsigned long long *d, h[3];
  (void)hipMalloc(&d, sizeof h);
  const int iters = 1 << 16;
  for (int salu = 0; salu < 2; ++salu)
    for (int grid : {1, 256, 2048}) {
      for (int rep = 0; rep < 2; ++rep) {
        k_probe<<<grid, 64>>>(d, iters, salu);
        (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
      }
      const double us = h[1] / 100.0;
      printf("{\"op\": \"%s\", \"grid\": %d, \"shader_cycles\": %llu, \"us\": %.1f, \"MHz\": %.0f, \"cycles_per_op\": %.2f}\n",
             salu ? "s_mul" : "v_add", grid, h[0], us, h[0] / us, (double)h[0] / iters);
      fflush(stdout);
    }
  return 0;
}
