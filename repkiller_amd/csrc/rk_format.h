// rk_format.h -- number formatting of the reference's output rows
// (commonFunctions.cpp:101-104: ofstream << uint64_t, << float).
//
// ostream << float widens to double and prints "%.*g" with precision 6.
// put_float reproduces that exactly without snprintf for the range the
// output actually holds (similarity and identity percentages): positive
// finite floats in [1e-3, 1e6).  There the float is m * 2^k with m < 2^24 and
// -34 <= k <= 0... and v * 10^(5-e) (e = the decimal exponent) is an exact
// rational num / 2^s with num < 2^63, so the 6-significant-digit integer is
// rounded to nearest-even on the exact binary value, as glibc's printf does.
// Everything else (0, negatives, NaN/inf, tiny or huge values) goes to
// snprintf.  tests/test_format.py compares both paths over every value the
// generator can write and millions of random floats.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>

namespace rk {

inline char *put_u64(char *o, uint64_t v) {
  char t[24];
  int k = 0;
  do {
    t[k++] = (char)('0' + v % 10);
    v /= 10;
  } while (v);
  while (k) *o++ = t[--k];
  return o;
}

inline char *put_float_slow(char *o, float f) {
  return o + std::snprintf(o, 40, "%.6g", (double)f);
}

inline char *put_float(char *o, float f) {
  if (!(f >= 1e-3f && f < 1e6f)) return put_float_slow(o, f);
  uint32_t bits;
  std::memcpy(&bits, &f, 4);
  const int ebin = (int)((bits >> 23) & 0xFF);
  const uint64_t m = (bits & 0x7FFFFFu) | 0x800000u;  // normal: f >= 1e-3
  const int k = ebin - 150;                            // f = m * 2^k
  // decimal exponent e (f in [10^e, 10^(e+1))), e in [-3, 5]
  static const float p10[] = {1e-3f, 1e-2f, 1e-1f, 1e0f, 1e1f, 1e2f, 1e3f, 1e4f, 1e5f, 1e6f};
  int e = -3;
  while (e < 5 && f >= p10[e + 4]) ++e;
  const int q = 5 - e;  // 0..8: N = round(f * 10^q), 6 digits
  static const uint64_t t10[] = {1ull, 10ull, 100ull, 1000ull, 10000ull, 100000ull,
                                 1000000ull, 10000000ull, 100000000ull};
  // f * 10^q = m * 10^q * 2^k; k < 0 here unless f >= 2^23 (not in range)
  uint64_t num = m * t10[q];
  uint64_t N;
  if (k >= 0) {
    N = num << k;
  } else {
    const int s = -k;
    if (s >= 64) return put_float_slow(o, f);
    N = num >> s;
    const uint64_t rem = num & ((1ull << s) - 1ull), half = 1ull << (s - 1);
    if (rem > half || (rem == half && (N & 1ull))) ++N;
  }
  if (N >= 1000000ull) {  // rounded up to the next decade
    N /= 10;              // exact: N == 1000000
    ++e;
    if (e >= 6) return put_float_slow(o, f);
  }
  // %g: fixed notation for -4 <= e < 6 with 6 significant digits, trailing
  // zeros (and a trailing point) removed
  char d[6];
  for (int i = 5; i >= 0; --i) d[i] = (char)('0' + N % 10), N /= 10;
  int last = 5;
  while (last > 0 && d[last] == '0') --last;
  if (e >= 0) {
    for (int i = 0; i <= e; ++i) *o++ = d[i];
    if (last > e) {
      *o++ = '.';
      for (int i = e + 1; i <= last; ++i) *o++ = d[i];
    }
  } else {
    *o++ = '0';
    *o++ = '.';
    for (int i = 0; i < -e - 1; ++i) *o++ = '0';
    for (int i = 0; i <= last; ++i) *o++ = d[i];
  }
  return o;
}

// The common spelling of the similarity column ("93.45": optional leading
// blanks and sign, digits, an optional '.' and digits, nothing after) with at
// most 7 significant digits: the decimal mantissa m < 2^24 and 10^k (k <= 10)
// are exact floats, so m / 10^k in float arithmetic is the correctly rounded
// value strtof returns (Clinger's fast path).  Anything else returns false
// and the caller uses strtof (tests/cpp/stof_check.cpp compares the two).
inline bool fast_stof(const char *p, const char *e, float *out) {
  while (p < e && (*p == ' ' || (*p >= '\t' && *p <= '\r'))) ++p;
  bool neg = false;
  if (p < e && (*p == '+' || *p == '-')) neg = *p++ == '-';
  uint32_t m = 0;
  int digits = 0, frac = 0;
  bool any = false, dot = false;
  for (; p < e; ++p) {
    const char c = *p;
    if (c >= '0' && c <= '9') {
      any = true;
      if (m == 0 && c == '0') {  // leading zeros add no significant digit
        if (dot) ++frac;
        continue;
      }
      if (++digits > 7) return false;
      m = m * 10 + (uint32_t)(c - '0');
      if (dot) ++frac;
    } else if (c == '.' && !dot) {
      dot = true;
    } else {
      return false;
    }
  }
  if (!any || frac > 10) return false;
  static const float p10[] = {1e0f, 1e1f, 1e2f, 1e3f, 1e4f, 1e5f, 1e6f, 1e7f, 1e8f, 1e9f, 1e10f};
  const float v = (float)m / p10[frac];
  *out = neg ? -v : v;
  return true;
}

}  // namespace rk
