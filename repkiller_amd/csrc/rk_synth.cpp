// rk_synth.cpp -- deterministic synthetic fragment sets (SURVEY.md §8d model).
//
// Host-side input maker for tests and bench.py: splitmix64 stream, seed =
// config number.  A share `family_frac` of the fragments come from repeat
// families (k copies of a length-l element; every ordered copy pair a != b
// gives one fragment x = pos_a + U[-3,3], y = pos_b, len = max(20, l + U[-10,10]));
// the rest are background fragments at uniform positions.  File order is a
// Fisher-Yates shuffle.  Same seed + params => bit-identical arrays.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "repkiller_amd.h"

namespace {

struct SplitMix64 {
  uint64_t s;
  uint64_t next() {
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  }
  // U[lo, hi) for hi > lo
  uint64_t range(uint64_t lo, uint64_t hi) { return lo + next() % (hi - lo); }
  double unit() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
};

}  // namespace

extern "C" int rk_synth_generate(const rk_synth_params *p, uint64_t *x_start, uint64_t *y_start,
                                 uint64_t *length, uint8_t *strand, uint64_t *ident) {
  if (!p || !x_start || !y_start || !length || !strand) return RK_E_ARG;
  const uint64_t n = p->n, L = p->genome_len;
  if (L < 1000 || p->copies_lo < 2 || p->copies_hi <= p->copies_lo) return RK_E_ARG;
  SplitMix64 rng{p->seed};
  uint64_t fam_target = (uint64_t)std::llround((double)n * p->family_frac);
  if (fam_target > n) fam_target = n;
  uint64_t k = 0;
  std::vector<uint64_t> pos;
  auto emit = [&](uint64_t x, uint64_t y, uint64_t len) {
    x_start[k] = x;
    y_start[k] = y;
    length[k] = len;
    strand[k] = rng.unit() < 0.6 ? 'f' : 'r';
    double u = 0.6 + 0.4 * rng.unit();
    if (ident) ident[k] = (uint64_t)std::floor((double)len * u);
    ++k;
  };
  while (k < fam_target) {
    uint64_t copies = rng.range(p->copies_lo, p->copies_hi);
    uint64_t ell = rng.range(40, 400);
    pos.resize(copies);
    for (auto &q : pos) q = rng.range(1, L - 2 * ell);
    for (uint64_t a = 0; a < copies && k < fam_target; ++a)
      for (uint64_t b = 0; b < copies && k < fam_target; ++b) {
        if (a == b) continue;
        int64_t jit = (int64_t)rng.range(0, 7) - 3;
        int64_t x = (int64_t)pos[a] + jit;
        int64_t dl = (int64_t)rng.range(0, 21) - 10;
        int64_t len = (int64_t)ell + dl;
        emit(x < 0 ? 0 : (uint64_t)x, pos[b], len < 20 ? 20 : (uint64_t)len);
      }
  }
  while (k < n) {
    uint64_t len = rng.range(20, 400);
    uint64_t x = rng.range(1, L - len), y = rng.range(1, L - len);
    emit(x, y, len);
  }
  for (uint64_t i = n; i > 1; --i) {  // Fisher-Yates, file order
    uint64_t j = rng.next() % i;
    std::swap(x_start[i - 1], x_start[j]);
    std::swap(y_start[i - 1], y_start[j]);
    std::swap(length[i - 1], length[j]);
    std::swap(strand[i - 1], strand[j]);
    if (ident) std::swap(ident[i - 1], ident[j]);
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
