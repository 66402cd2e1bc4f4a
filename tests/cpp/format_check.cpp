// Compares rk::put_float (repkiller_amd/csrc/rk_format.h) with the snprintf
// "%.6g" that ostream << float performs, on every "%.2f" similarity 0..1000,
// identity percentages ident*100/length, and random float bit patterns.
#include <cstdio>
#include <cstring>
#include <random>
#include <string>

#include "rk_format.h"

int main(int argc, char **argv) {
  const long nrand = argc > 1 ? std::atol(argv[1]) : 2000000;
  char a[64], b[64];
  long bad = 0, n = 0;
  auto chk = [&](float f) {
    *rk::put_float(a, f) = 0;
    *rk::put_float_slow(b, f) = 0;
    ++n;
    if (std::strcmp(a, b)) {
      if (bad < 10) std::printf("%.9g: %s vs %s\n", f, a, b);
      ++bad;
    }
  };
  for (int i = 0; i <= 100000; ++i) {
    char t[32];
    std::snprintf(t, sizeof t, "%d.%02d", i / 100, i % 100);
    chk(std::strtof(t, nullptr));
  }
  for (uint32_t id = 1; id < 2000; ++id)
    for (uint32_t L = id; L < 2000; L += 3) chk((float)id * 100 / (float)L);
  std::mt19937 r(1);
  std::uniform_int_distribution<uint32_t> u(0, 0xFFFFFFFFu);
  for (long i = 0; i < nrand; ++i) {
    const uint32_t x = u(r);
    float f;
    std::memcpy(&f, &x, 4);
    chk(f);
  }
  std::uniform_real_distribution<float> v(1e-3f, 1e6f);
  for (long i = 0; i < nrand; ++i) chk(v(r));
  std::printf("checked %ld, mismatches %ld\n", n, bad);
  return bad != 0;
}
