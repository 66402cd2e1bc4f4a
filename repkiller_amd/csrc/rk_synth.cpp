// rk_synth.cpp -- deterministic synthetic fragment sets (SURVEY.md §8d model).
//
// Host-side input maker for tests and bench.py: splitmix64 stream, seed =
// config number.  A share `family_frac` of the fragments come from repeat
// families (k copies of a length-l element; every ordered copy pair a != b
// gives one fragment x = pos_a + U[-3,3], y = pos_b, len = max(20, l + U[-10,10]));
// the rest are background fragments at uniform positions.  File order is a
// Fisher-Yates shuffle.  Same seed + params => bit-identical arrays.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "repkiller_amd.h"

namespace {

constexpr uint64_t GOLDEN = 0x9e3779b97f4a7c15ull;

uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// splitmix64 is counter based: draw c (0-based) of seed s is mix(s + (c+1)G),
// so any row's draws can be made without the draws before it.
struct SplitMix64 {
  uint64_t s;
  uint64_t next() { return mix(s += GOLDEN); }
  // U[lo, hi) for hi > lo
  uint64_t range(uint64_t lo, uint64_t hi) { return lo + next() % (hi - lo); }
  double unit() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
  static SplitMix64 at(uint64_t seed, uint64_t draw) { return SplitMix64{seed + draw * GOLDEN}; }
};

struct Family {
  uint64_t row0, rows;  // output rows [row0, row0 + rows)
  uint64_t draw0;       // draw counter of its first pair
  uint64_t copies, ell, pos0;
};

unsigned pool_threads(uint64_t work) {
  unsigned t = std::thread::hardware_concurrency();
  if (t == 0) t = 1;
  if (t > 16) t = 16;  // the GPU boxes' CPU share
  const uint64_t cap = work / (1u << 20) + 1;  // ~1M rows per thread at least
  return (unsigned)std::min<uint64_t>(t, cap);
}

template <class F>
void parallel_for(uint64_t n, F f) {  // f(begin, end) over [0, n)
  const unsigned t = pool_threads(n);
  if (t <= 1) {
    f((uint64_t)0, n);
    return;
  }
  std::vector<std::thread> th;
  for (unsigned k = 0; k < t; ++k)
    th.emplace_back([=] { f(n * k / t, n * (k + 1) / t); });
  for (auto &x : th) x.join();
}

// permutation of Fisher-Yates over n rows (draws from `draw0` on): the
// sequential swaps run on a u32/u64 index array with the random partner
// prefetched a few dozen steps ahead (the draws do not depend on the data)
template <class I>
void fy_perm(I *perm, uint64_t n, uint64_t seed, uint64_t draw0) {
  parallel_for(n, [=](uint64_t a, uint64_t b) {
    for (uint64_t i = a; i < b; ++i) perm[i] = (I)i;
  });
  constexpr uint64_t AHEAD = 48;
  SplitMix64 pre = SplitMix64::at(seed, draw0), rng = pre;
  uint64_t ring[AHEAD];
  for (uint64_t d = 0; d < AHEAD && n > 1 + d; ++d) {
    ring[d] = pre.next() % (n - d);
    __builtin_prefetch(&perm[ring[d]], 1);
  }
  for (uint64_t i = n, t = 0; i > 1; --i, ++t) {
    const uint64_t j = ring[t % AHEAD];
    if (i > 1 + AHEAD) {  // draw of step t + AHEAD (i - AHEAD rows left then)
      const uint64_t jn = pre.next() % (i - AHEAD);
      ring[t % AHEAD] = jn;
      __builtin_prefetch(&perm[jn], 1);
    }
    std::swap(perm[i - 1], perm[j]);
  }
  (void)rng;
}

template <class T, class I>
void apply_perm(T *a, const I *perm, uint64_t n, std::vector<T> &tmp) {
  tmp.resize(n);
  T *t = tmp.data();
  parallel_for(n, [=](uint64_t lo, uint64_t hi) {
    for (uint64_t i = lo; i < hi; ++i) t[i] = a[perm[i]];
  });
  parallel_for(n, [=](uint64_t lo, uint64_t hi) {
    std::memcpy(a + lo, t + lo, (hi - lo) * sizeof(T));
  });
}

}  // namespace

// Same output as the sequential generator (one splitmix64 stream: families,
// then background rows, then a Fisher-Yates shuffle), made in parallel: a
// first pass walks the family headers to find every row's draw counter.
extern "C" int rk_synth_generate(const rk_synth_params *p, uint64_t *x_start, uint64_t *y_start,
                                 uint64_t *length, uint8_t *strand, uint64_t *ident) {
  if (!p || !x_start || !y_start || !length || !strand) return RK_E_ARG;
  const uint64_t n = p->n, L = p->genome_len, seed = p->seed;
  if (L < 1000 || p->copies_lo < 2 || p->copies_hi <= p->copies_lo) return RK_E_ARG;
  uint64_t fam_target = (uint64_t)std::llround((double)n * p->family_frac);
  if (fam_target > n) fam_target = n;
  // pass 1: family headers (copies, element length, copy positions)
  std::vector<Family> fams;
  std::vector<uint64_t> pos;
  SplitMix64 rng{seed};
  uint64_t draws = 0, k = 0;
  while (k < fam_target) {
    Family f{};
    f.copies = rng.range(p->copies_lo, p->copies_hi);
    f.ell = rng.range(40, 400);
    f.pos0 = pos.size();
    for (uint64_t c = 0; c < f.copies; ++c) pos.push_back(rng.range(1, L - 2 * f.ell));
    draws += 2 + f.copies;
    f.row0 = k;
    f.draw0 = draws;
    f.rows = std::min(f.copies * (f.copies - 1), fam_target - k);
    k += f.rows;
    draws += 4 * f.rows;  // jitter, length delta, strand, ident per pair
    rng = SplitMix64::at(seed, draws);
    fams.push_back(f);
  }
  const uint64_t bg_draw0 = draws, shuffle_draw0 = draws + 5 * (n - fam_target);
  auto emit = [&](SplitMix64 &r, uint64_t row, uint64_t x, uint64_t y, uint64_t len) {
    x_start[row] = x;
    y_start[row] = y;
    length[row] = len;
    strand[row] = r.unit() < 0.6 ? 'f' : 'r';
    const double u = 0.6 + 0.4 * r.unit();
    if (ident) ident[row] = (uint64_t)std::floor((double)len * u);
  };
  // pass 2: family rows (ordered copy pairs a != b), in parallel by family
  parallel_for(fams.size(), [&](uint64_t lo, uint64_t hi) {
    for (uint64_t fi = lo; fi < hi; ++fi) {
      const Family &f = fams[fi];
      SplitMix64 r = SplitMix64::at(seed, f.draw0);
      const uint64_t *ps = pos.data() + f.pos0;
      for (uint64_t t = 0; t < f.rows; ++t) {
        const uint64_t a = t / (f.copies - 1), bb = t % (f.copies - 1);
        const uint64_t b = bb < a ? bb : bb + 1;
        const int64_t jit = (int64_t)r.range(0, 7) - 3;
        const int64_t x = (int64_t)ps[a] + jit;
        const int64_t dl = (int64_t)r.range(0, 21) - 10;
        const int64_t len = (int64_t)f.ell + dl;
        emit(r, f.row0 + t, x < 0 ? 0 : (uint64_t)x, ps[b], len < 20 ? 20 : (uint64_t)len);
      }
    }
  });
  // background rows, in parallel by row range
  parallel_for(n - fam_target, [&](uint64_t lo, uint64_t hi) {
    SplitMix64 r = SplitMix64::at(seed, bg_draw0 + 5 * lo);
    for (uint64_t q = lo; q < hi; ++q) {
      const uint64_t len = r.range(20, 400);
      const uint64_t x = r.range(1, L - len), y = r.range(1, L - len);
      emit(r, fam_target + q, x, y, len);
    }
  });
  // Fisher-Yates, file order
  if (n > 1) {
    auto shuffle = [&](auto *perm) {
      fy_perm(perm, n, seed, shuffle_draw0);
      std::vector<uint64_t> t64;
      apply_perm(x_start, perm, n, t64);
      apply_perm(y_start, perm, n, t64);
      apply_perm(length, perm, n, t64);
      if (ident) apply_perm(ident, perm, n, t64);
      t64.clear();
      t64.shrink_to_fit();
      std::vector<uint8_t> t8;
      apply_perm(strand, perm, n, t8);
    };
    if (n <= 0xFFFFFFFFull) {
      std::vector<uint32_t> perm(n);
      shuffle(perm.data());
    } else {
      std::vector<uint64_t> perm(n);
      shuffle(perm.data());
    }
  }
  return RK_OK;
}

// GECKO-style CSV with the 16-line header FragmentsDatabase reads
// (lines 7/8/13 carry the two lengths and the fragment total).
extern "C" int rk_synth_write_csv(const char *path, uint64_t n, const uint64_t *x_start,
                                  const uint64_t *y_start, const uint64_t *length,
                                  const uint8_t *strand, const uint64_t *ident,
                                  uint64_t len_x_hdr, uint64_t len_y_hdr) {
  FILE *f = std::fopen(path, "wb");
  if (!f) return RK_E_IO;
  std::vector<char> buf(1 << 20);
  std::setvbuf(f, buf.data(), _IOFBF, buf.size());
  std::fprintf(f,
               "All by-Identity Ungapped Fragments (Hits based approach)\n"
               "[synthetic -- repkiller_amd rk_synth]\n"
               "SeqX filename\t: synthX.fasta\n"
               "SeqY filename\t: synthY.fasta\n"
               "SeqX name\t: synthX\n"
               "SeqY name\t: synthY\n"
               "SeqX length\t: %llu\n"
               "SeqY length\t: %llu\n"
               "Min.fragment.length\t: 0\n"
               "Min.Identity\t: 0\n"
               "Total hits\t: 0\n"
               "Total hits (used)\t: 0\n"
               "Total fragments\t: %llu\n"
               "========================================================\n"
               "Type,xStart,yStart,xEnd,yEnd,Strand(f/r),block,length,score,ident,similarity,%%ident,SeqX,SeqY\n"
               "========================================================\n",
               (unsigned long long)len_x_hdr, (unsigned long long)len_y_hdr,
               (unsigned long long)n);
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t len = length[i], id = ident ? ident[i] : len;
    double sim = len ? 100.0 * (double)id / (double)len : 0.0;
    std::fprintf(f, "Frag,%llu,%llu,%llu,%llu,%c,0,%llu,%llu,%llu,%.2f,%.2f,0,0\n",
                 (unsigned long long)x_start[i], (unsigned long long)y_start[i],
                 (unsigned long long)(x_start[i] + len - 1),
                 (unsigned long long)(y_start[i] + len - 1), (char)strand[i],
                 (unsigned long long)len, (unsigned long long)(4 * id),
                 (unsigned long long)id, sim, sim);
  }
  return std::fclose(f) == 0 ? RK_OK : RK_E_IO;
}
