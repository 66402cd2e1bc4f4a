/* rk_oracle.c -- sequential CPU restatement of estebanpw/repkiller v0.9.b.
 *
 * TEST INFRASTRUCTURE ONLY (see rk_oracle.h).  Every function cites the
 * reference code it restates; /root/reference/src is the path prefix.
 *
 * Parity of this restatement is pinned by tests/golden/ (fixtures produced by
 * the reference itself, built by oracle/ref.mk) -- tests/test_oracle.py.
 *
 * Build: make -f oracle/oracle.mk  (gcc -std=c11 -O2 -ffp-contract=off).
 * -ffp-contract=off matters: the reference binary targets baseline x86-64 and
 * never fuses 0.4*sl + 0.6*sp (SequenceOcupationList.cpp:30).
 */
#define _GNU_SOURCE
#include "rk_oracle.h"

#include <errno.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* std::getline emulation                                                     */
/* ------------------------------------------------------------------------- */
/* libstdc++'s getline() builds a sentry first: on a stream whose eof or fail
 * bit is already set the sentry fails, the target string is NOT cleared and
 * failbit is set.  Otherwise the string is cleared and characters up to the
 * delimiter are extracted; hitting end of input sets eofbit, and extracting
 * nothing at all (delimiter not even seen) sets failbit.  Both the file reader
 * (FragmentsDatabase.cpp:57-93) and the field splitter (:23-27, on an
 * istringstream) depend on this -- e.g. a 13-field line gets its last field
 * repeated as field 14.  */
typedef struct {
  const char *buf;
  size_t len, pos;
  int eof, fail;
} getline_state;

/* returns 1 if the output (ptr,len) was replaced, 0 if left stale */
static int gl_next(getline_state *s, char delim, const char **out, size_t *out_len) {
  if (s->eof || s->fail) {
    s->fail = 1;
    return 0;
  }
  const char *start = s->buf + s->pos;
  size_t avail = s->len - s->pos;
  const char *hit = avail ? memchr(start, delim, avail) : NULL;
  if (hit) {
    *out = start;
    *out_len = (size_t)(hit - start);
    s->pos += *out_len + 1;
  } else {
    *out = start;
    *out_len = avail;
    s->pos = s->len;
    s->eof = 1;
    if (avail == 0) s->fail = 1;
  }
  return 1;
}

/* ------------------------------------------------------------------------- */
/* field conversions                                                          */
/* ------------------------------------------------------------------------- */
static char *cstr_of(const char *p, size_t n, char *small, size_t small_cap, char **heap) {
  char *d = small;
  if (n + 1 > small_cap) {
    *heap = (char *)malloc(n + 1);
    d = *heap;
  }
  memcpy(d, p, n);
  d[n] = 0;
  return d;
}

/* atoll(str.c_str()) -- glibc atoll == strtoll(s, NULL, 10); the result is
 * stored into uint64 fields (FragmentsDatabase.cpp:30-38). */
static uint64_t field_atoll(const char *p, size_t n) {
  char small[64], *heap = NULL;
  char *s = cstr_of(p, n, small, sizeof small, &heap);
  long long v = atoll(s);
  free(heap);
  return (uint64_t)v;
}

/* std::stof (libstdc++ __stoa over strtof): no digits -> invalid_argument,
 * errno == ERANGE (overflow or underflow) -> out_of_range.  Either exception
 * makes readFragment return false (FragmentsDatabase.cpp:46-48). */
static int field_stof(const char *p, size_t n, float *out) {
  char small[64], *heap = NULL;
  char *s = cstr_of(p, n, small, sizeof small, &heap);
  char *end = NULL;
  int saved = errno;
  errno = 0;
  float v = strtof(s, &end);
  int ok = !(end == s || errno == ERANGE);
  if (errno == 0) errno = saved;
  free(heap);
  *out = v;
  return ok;
}

/* (uint64_t) of a float as the x86-64 reference binary computes it
 * (FragmentsDatabase.cpp:39).  Out-of-range/NaN conversions are undefined in
 * C++; g++ emits: x < 2^63 (ordered) ? cvttss2si(x) : cvttss2si(x - 2^63) ^ 2^63,
 * and cvttss2si yields 0x8000000000000000 for NaN or out-of-range input.
 * Pinned by the edge fixture E6 (nan -> 9223372036854775808). */
static uint64_t cvtt_i64(float x) {
  if (isnan(x) || x >= 9223372036854775808.0f || x < -9223372036854775808.0f)
    return 0x8000000000000000ull;
  return (uint64_t)(int64_t)x;
}
static uint64_t x86_float_to_u64(float x) {
  if (!(x >= 9223372036854775808.0f)) return cvtt_i64(x);
  return cvtt_i64(x - 9223372036854775808.0f) ^ 0x8000000000000000ull;
}

/* ------------------------------------------------------------------------- */
/* ingress: FragmentsDatabase (FragmentsDatabase.cpp:17-101)                  */
/* ------------------------------------------------------------------------- */
typedef struct {
  uint64_t *p;
  size_t n, cap;
} u64vec;

static int grow(rko_db *db, size_t *cap) {
  size_t nc = *cap ? *cap * 2 : 1024;
#define RK_GROW(f, T)                                  \
  do {                                                 \
    void *q = realloc(db->f, nc * sizeof(T));          \
    if (!q) return 0;                                  \
    db->f = (T *)q;                                    \
  } while (0)
  RK_GROW(x_start, uint64_t);
  RK_GROW(y_start, uint64_t);
  RK_GROW(x_end, uint64_t);
  RK_GROW(y_end, uint64_t);
  RK_GROW(length, uint64_t);
  RK_GROW(score, uint64_t);
  RK_GROW(ident, uint64_t);
  RK_GROW(similarity, float);
  RK_GROW(strand, uint8_t);
#undef RK_GROW
  *cap = nc;
  return 1;
}

/* readFragment (FragmentsDatabase.cpp:17-50) on one line */
static int parse_frag_line(const char *line, size_t len, rko_db *db, size_t i) {
  getline_state s = {line, len, 0, 0, 0};
  const char *fp[14];
  size_t fl[14];
  const char *cur = NULL;
  size_t cur_len = 0;
  for (int k = 0; k < 14; ++k) {
    gl_next(&s, ',', &cur, &cur_len);
    if (cur_len == 0) return 0;
    fp[k] = cur;
    fl[k] = cur_len;
  }
  if (!(fl[0] == 4 && memcmp(fp[0], "Frag", 4) == 0)) return 0;
  float sim;
  /* stof(v[10]) is evaluated for ident first and would throw there */
  if (!field_stof(fp[10], fl[10], &sim)) return 0;
  db->x_start[i] = field_atoll(fp[1], fl[1]);
  db->y_start[i] = field_atoll(fp[2], fl[2]);
  db->x_end[i] = field_atoll(fp[3], fl[3]);
  db->y_end[i] = field_atoll(fp[4], fl[4]);
  db->strand[i] = (uint8_t)fp[5][0];
  db->length[i] = field_atoll(fp[7], fl[7]);
  db->score[i] = field_atoll(fp[8], fl[8]);
  db->ident[i] = x86_float_to_u64(sim);
  db->similarity[i] = sim;
  return 1;
}

static uint64_t header_value(const char *line, size_t len) {
  /* atoll(line.substr(line.find(':') + 1).c_str()) -- npos + 1 == 0 */
  const char *c = len ? memchr(line, ':', len) : NULL;
  size_t off = c ? (size_t)(c - line) + 1 : 0;
  return field_atoll(line + off, len - off);
}

int rko_load_csv(const char *path, rko_db *db) {
  memset(db, 0, sizeof *db);
  FILE *f = fopen(path, "rb");
  if (!f) return RKO_E_IO;
  fseek(f, 0, SEEK_END);
  long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  char *buf = (char *)malloc((size_t)sz + 1);
  if (!buf) {
    fclose(f);
    return RKO_E_NOMEM;
  }
  size_t got = fread(buf, 1, (size_t)sz, f);
  fclose(f);
  getline_state s = {buf, got, 0, 0, 0};
  const char *line = "";
  size_t line_len = 0;
  size_t hcap = 256;
  db->header = (char *)malloc(hcap);
  db->header_len = 0;
  for (int k = 1; k <= 16; ++k) {
    gl_next(&s, '\n', &line, &line_len);
    while (db->header_len + line_len + 2 > hcap) {
      hcap *= 2;
      db->header = (char *)realloc(db->header, hcap);
    }
    memcpy(db->header + db->header_len, line, line_len);
    db->header_len += line_len;
    db->header[db->header_len++] = '\n';
    if (k == 7) db->len_x_hdr = header_value(line, line_len);
    if (k == 8) db->len_y_hdr = header_value(line, line_len);
    if (k == 13) db->total_hdr = header_value(line, line_len);
  }
  db->header[db->header_len] = 0;
  size_t cap = 0, n = 0;
  int rc = RKO_OK;
  while (!s.eof) {
    gl_next(&s, '\n', &line, &line_len);
    if (n == cap && !grow(db, &cap)) {
      rc = RKO_E_NOMEM;
      break;
    }
    if (!parse_frag_line(line, line_len, db, n)) continue;
    ++n;
    if (n > db->total_hdr) {   /* FragmentsDatabase.cpp:99 */
      rc = RKO_E_COUNT;
      break;
    }
  }
  db->n = n;
  free(buf);
  return rc;
}

void rko_free_db(rko_db *db) {
  free(db->x_start);
  free(db->y_start);
  free(db->x_end);
  free(db->y_end);
  free(db->length);
  free(db->score);
  free(db->ident);
  free(db->similarity);
  free(db->strand);
  free(db->header);
  memset(db, 0, sizeof *db);
}

/* ------------------------------------------------------------------------- */
/* libstdc++ (GCC 11, bits/stl_algo.h + bits/stl_heap.h) std::sort restated   */
/* ------------------------------------------------------------------------- */
/* Third-party algorithm the reference depends on (sort_groups,
 * commonFunctions.cpp:158).  Restated from libstdc++ 11's published source:
 * __sort / __introsort_loop (depth 2*floor(log2 n), threshold 16) /
 * __unguarded_partition_pivot (median-of-three moved to first) /
 * __unguarded_partition / heapsort fallback (__make_heap, __adjust_heap,
 * __push_heap, __pop_heap, __sort_heap) / __final_insertion_sort. */
#define LESS(a, b) ((a).key < (b).key)
static inline void rec_swap(rko_rec *a, rko_rec *b) {
  rko_rec t = *a;
  *a = *b;
  *b = t;
}

static void push_heap_(rko_rec *a, ptrdiff_t hole, ptrdiff_t top, rko_rec v) {
  ptrdiff_t parent = (hole - 1) / 2;
  while (hole > top && LESS(a[parent], v)) {
    a[hole] = a[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  a[hole] = v;
}

static void adjust_heap_(rko_rec *a, ptrdiff_t hole, ptrdiff_t len, rko_rec v) {
  const ptrdiff_t top = hole;
  ptrdiff_t child = hole;
  while (child < (len - 1) / 2) {
    child = 2 * (child + 1);
    if (LESS(a[child], a[child - 1])) child--;
    a[hole] = a[child];
    hole = child;
  }
  if ((len & 1) == 0 && child == (len - 2) / 2) {
    child = 2 * (child + 1);
    a[hole] = a[child - 1];
    hole = child - 1;
  }
  push_heap_(a, hole, top, v);
}

static void heapsort_(rko_rec *a, ptrdiff_t len) {
  if (len >= 2) { /* __make_heap */
    ptrdiff_t parent = (len - 2) / 2;
    for (;;) {
      adjust_heap_(a, parent, len, a[parent]);
      if (parent == 0) break;
      parent--;
    }
  }
  for (ptrdiff_t last = len; last > 1;) { /* __sort_heap */
    --last;
    rko_rec v = a[last];
    a[last] = a[0];
    adjust_heap_(a, 0, last, v);
  }
}

static void median_to_first_(rko_rec *r, rko_rec *a, rko_rec *b, rko_rec *c) {
  if (LESS(*a, *b)) {
    if (LESS(*b, *c)) rec_swap(r, b);
    else if (LESS(*a, *c)) rec_swap(r, c);
    else rec_swap(r, a);
  } else if (LESS(*a, *c)) rec_swap(r, a);
  else if (LESS(*b, *c)) rec_swap(r, c);
  else rec_swap(r, b);
}

static rko_rec *partition_(rko_rec *first, rko_rec *last, const rko_rec *pivot) {
  for (;;) {
    while (LESS(*first, *pivot)) ++first;
    --last;
    while (LESS(*pivot, *last)) --last;
    if (!(first < last)) return first;
    rec_swap(first, last);
    ++first;
  }
}

static void introsort_loop_(rko_rec *first, rko_rec *last, long depth) {
  while (last - first > 16) {
    if (depth == 0) {
      heapsort_(first, last - first);
      return;
    }
    --depth;
    rko_rec *mid = first + (last - first) / 2;
    median_to_first_(first, first + 1, mid, last - 1);
    rko_rec *cut = partition_(first + 1, last, first);
    introsort_loop_(cut, last, depth);
    last = cut;
  }
}

static void linear_insert_(rko_rec *last) {
  rko_rec v = *last;
  rko_rec *next = last - 1;
  while (LESS(v, *next)) {
    *last = *next;
    last = next;
    --next;
  }
  *last = v;
}

static void insertion_sort_(rko_rec *first, rko_rec *last) {
  if (first == last) return;
  for (rko_rec *i = first + 1; i != last; ++i) {
    if (LESS(*i, *first)) {
      rko_rec v = *i;
      memmove(first + 1, first, (size_t)(i - first) * sizeof *i);
      *first = v;
    } else {
      linear_insert_(i);
    }
  }
}

void rko_std_sort(rko_rec *a, size_t n) {
  if (n == 0) return;
  long lg = 63 - __builtin_clzll((unsigned long long)n);
  introsort_loop_(a, a + n, 2 * lg);
  if (n > 16) {
    insertion_sort_(a, a + 16);
    for (rko_rec *i = a + 16; i != a + n; ++i) linear_insert_(i);
  } else {
    insertion_sort_(a, a + n);
  }
}
#undef LESS

/* ------------------------------------------------------------------------- */
/* occupancy lists: SequenceOcupationList (SequenceOcupationList.cpp:3-96)    */
/* ------------------------------------------------------------------------- */
typedef struct {
  uint64_t center, length;
  uint32_t group;
  int64_t next; /* forward_list link, -1 = end */
} occ_node;

typedef struct {
  int64_t *head;      /* max_index + 1 bucket heads, newest first */
  uint64_t max_index; /* seq_size / DIVISOR (SequenceOcupationList.cpp:4) */
  double len_ratio, pos_ratio;
} occ_list;

typedef struct {
  occ_node *nodes;
  size_t n, cap;
} occ_pool;

/* SequenceOcupationList::deviation (SequenceOcupationList.cpp:20-31) */
static double deviation(const occ_list *ol, const occ_node *oc, uint64_t center, uint64_t length) {
  uint64_t dif_len = length > oc->length ? length - oc->length : oc->length - length;
  double sim_len = -fabs((double)dif_len / ((double)length * ol->len_ratio)) + 1.0;
  if (sim_len < 0) return 0.0;
  uint64_t dif_cen = center > oc->center ? center - oc->center : oc->center - center;
  double sim_pos = -fabs((double)dif_cen / ((double)length * ol->pos_ratio)) + 1.0;
  if (sim_pos < 0) return 0.0;
  return sim_len * 0.4 + sim_pos * 0.6;
}

static void scan_bucket(const occ_list *ol, const occ_pool *pool, uint64_t bucket,
                        uint64_t center, uint64_t length, double *d, int64_t *g) {
  for (int64_t e = ol->head[bucket]; e >= 0; e = pool->nodes[e].next) {
    double cd = deviation(ol, &pool->nodes[e], center, length);
    if (cd > *d) {
      *d = cd;
      *g = pool->nodes[e].group;
    }
  }
}

/* get_associated_group (SequenceOcupationList.cpp:33-91): own bucket, then
 * c-1, c+1, c-2, c+2 -- each guarded exactly as in the reference, including
 * the position-vs-bucket-count comparison against max_index and its size_t
 * wrap at max_index == 0 (callers have rejected inputs that would index out
 * of bounds). */
static int64_t occ_query(const occ_list *ol, const occ_pool *pool, uint64_t c, uint64_t len) {
  double d = 0;
  int64_t g = -1;
  scan_bucket(ol, pool, c / 100, c, len, &d, &g);
  if (c > 0) scan_bucket(ol, pool, (c - 1) / 100, c, len, &d, &g);
  if (c < ol->max_index) scan_bucket(ol, pool, (c + 1) / 100, c, len, &d, &g);
  if (c > 1) scan_bucket(ol, pool, (c - 2) / 100, c, len, &d, &g);
  if (c < ol->max_index - 1) scan_bucket(ol, pool, (c + 2) / 100, c, len, &d, &g);
  return g;
}

/* largest bucket index occ_query would touch for centre c */
static uint64_t probe_max_bucket(uint64_t c, uint64_t max_index) {
  uint64_t b = c / 100;
  if (c < max_index && (c + 1) / 100 > b) b = (c + 1) / 100;
  if (c < max_index - 1 && (c + 2) / 100 > b) b = (c + 2) / 100;
  return b;
}

/* SequenceOcupationList::insert (SequenceOcupationList.cpp:93-96): push_front */
static void occ_insert(occ_list *ol, occ_pool *pool, uint64_t c, uint64_t len, uint32_t group) {
  occ_node *nd = &pool->nodes[pool->n];
  nd->center = c;
  nd->length = len;
  nd->group = group;
  nd->next = ol->head[c / 100];
  ol->head[c / 100] = (int64_t)pool->n;
  pool->n++;
}

/* ------------------------------------------------------------------------- */
/* stable LSD radix sort of (key u64, value u32) -- processing-order helper   */
/* ------------------------------------------------------------------------- */
static int stable_sort_by_key(uint64_t *key, uint32_t *val, size_t n) {
  uint64_t maxk = 0;
  for (size_t i = 0; i < n; ++i)
    if (key[i] > maxk) maxk = key[i];
  uint64_t *k2 = (uint64_t *)malloc(n * sizeof *k2 + 1);
  uint32_t *v2 = (uint32_t *)malloc(n * sizeof *v2 + 1);
  size_t *cnt = (size_t *)malloc(65537 * sizeof *cnt);
  if (!k2 || !v2 || !cnt) {
    free(k2), free(v2), free(cnt);
    return 0;
  }
  for (int shift = 0; shift < 64 && (maxk >> shift) != 0; shift += 16) {
    memset(cnt, 0, 65537 * sizeof *cnt);
    for (size_t i = 0; i < n; ++i) cnt[((key[i] >> shift) & 0xffff) + 1]++;
    for (int b = 0; b < 65536; ++b) cnt[b + 1] += cnt[b];
    for (size_t i = 0; i < n; ++i) {
      size_t p = cnt[(key[i] >> shift) & 0xffff]++;
      k2[p] = key[i];
      v2[p] = val[i];
    }
    memcpy(key, k2, n * sizeof *key);
    memcpy(val, v2, n * sizeof *val);
  }
  free(k2), free(v2), free(cnt);
  return 1;
}

/* ------------------------------------------------------------------------- */
/* the hot path: generate_fragment_groups + generate_diagonal_func +          */
/* sort_groups + the repeat flag of save_frags_from_group                     */
/* ------------------------------------------------------------------------- */
int rko_classify(uint64_t n, const uint64_t *x_start, const uint64_t *y_start,
                 const uint64_t *length, const uint8_t *strand, uint64_t len_x_hdr,
                 uint64_t len_y_hdr, double len_ratio, double pos_ratio, uint32_t *gid,
                 uint8_t *repval, uint32_t *out_order, uint64_t *n_out, uint64_t *n_groups) {
  if (n >= 0xFFFFFFFFull) return RKO_E_ARG;
  /* sequence lengths are header value + 1 (FragmentsDatabase.cpp:62,65) */
  const uint64_t len_x = len_x_hdr + 1, len_y = len_y_hdr + 1;
  const uint64_t vsize = 1 + len_x / 10; /* FragmentsDatabase.cpp:84 */
  for (uint64_t i = 0; i < n; ++i)
    if (x_start[i] / 10 >= vsize) return RKO_E_UB_BUCKET; /* :96-97 out of bounds */
  /* processing order: buckets xStart/10 in file order; end() stops before
   * bucket vsize-1 (FragmentsDatabase.h:29-31) */
  uint64_t *pk = (uint64_t *)malloc(n * sizeof *pk + 1);
  uint32_t *order = (uint32_t *)malloc(n * sizeof *order + 1);
  if (!pk || !order) {
    free(pk), free(order);
    return RKO_E_NOMEM;
  }
  for (uint64_t i = 0; i < n; ++i) {
    pk[i] = x_start[i] / 10;
    order[i] = (uint32_t)i;
  }
  if (!stable_sort_by_key(pk, order, n)) {
    free(pk), free(order);
    return RKO_E_NOMEM;
  }
  uint64_t m = 0;
  while (m < n && pk[m] != vsize - 1) ++m;

  const uint64_t max_x = len_x / 100, max_y = len_y / 100;
  for (uint64_t k = 0; k < m; ++k) {
    uint32_t i = order[k];
    uint64_t h = length[i] / 2;
    if (probe_max_bucket(x_start[i] + h, max_x) > max_x ||
        probe_max_bucket(y_start[i] + h, max_y) > max_y) {
      free(pk), free(order);
      return RKO_E_UB_CENTER;
    }
  }

  /* four lists {f, other} x {X, Y} (commonFunctions.cpp:45-53) */
  occ_list lx[2], ly[2];
  occ_pool pool = {NULL, 0, 0};
  int rc = RKO_OK;
  uint32_t *grp = (uint32_t *)malloc(m * sizeof *grp + 1);
  pool.cap = 2 * m + 1;
  pool.nodes = (occ_node *)malloc(pool.cap * sizeof *pool.nodes);
  for (int s = 0; s < 2; ++s) {
    lx[s].max_index = max_x;
    ly[s].max_index = max_y;
    lx[s].len_ratio = ly[s].len_ratio = len_ratio;
    lx[s].pos_ratio = ly[s].pos_ratio = pos_ratio;
    lx[s].head = (int64_t *)malloc((max_x + 1) * sizeof(int64_t));
    ly[s].head = (int64_t *)malloc((max_y + 1) * sizeof(int64_t));
    if (lx[s].head) memset(lx[s].head, 0xff, (max_x + 1) * sizeof(int64_t));
    if (ly[s].head) memset(ly[s].head, 0xff, (max_y + 1) * sizeof(int64_t));
  }
  if (!grp || !pool.nodes || !lx[0].head || !lx[1].head || !ly[0].head || !ly[1].head) {
    rc = RKO_E_NOMEM;
    goto done;
  }

  /* generate_fragment_groups (commonFunctions.cpp:51-77) */
  uint32_t groups = 0;
  for (uint64_t k = 0; k < m; ++k) {
    uint32_t i = order[k];
    int s = strand[i] == 'f' ? 0 : 1;
    uint64_t L = length[i];
    uint64_t xc = x_start[i] + L / 2, yc = y_start[i] + L / 2;
    int64_t g = occ_query(&lx[s], &pool, xc, L);
    if (g >= 0) {
      grp[k] = (uint32_t)g;
      occ_insert(&ly[s], &pool, yc, L, (uint32_t)g);
      continue;
    }
    g = occ_query(&ly[s], &pool, yc, L);
    if (g >= 0) {
      grp[k] = (uint32_t)g;
      occ_insert(&lx[s], &pool, xc, L, (uint32_t)g);
      continue;
    }
    grp[k] = groups++;
    occ_insert(&lx[s], &pool, xc, L, grp[k]);
    occ_insert(&ly[s], &pool, yc, L, grp[k]);
  }

  /* members of each group in insertion (= processing) order */
  {
    uint64_t *gstart = (uint64_t *)calloc((size_t)groups + 1, sizeof *gstart);
    rko_rec *mem = (rko_rec *)malloc(m * sizeof *mem + 1);
    uint64_t *diag = (uint64_t *)malloc(m * sizeof *diag + 1);
    if (!gstart || !mem || !diag) {
      free(gstart), free(mem), free(diag);
      rc = RKO_E_NOMEM;
      goto done;
    }
    /* generate_diagonal_func (commonFunctions.cpp:161-177): `oh` is never
     * updated, so diag_func[b] = yStart of the LAST fragment of bucket b; the
     * carry-forward for empty buckets is never read by sort_groups. */
    for (uint64_t k = m; k-- > 0;) {
      if (k + 1 < m && pk[k + 1] == pk[k]) diag[k] = diag[k + 1];
      else diag[k] = y_start[order[k]];
    }
    for (uint64_t k = 0; k < m; ++k) gstart[grp[k] + 1]++;
    for (uint32_t g = 0; g < groups; ++g) gstart[g + 1] += gstart[g];
    uint64_t *fill = (uint64_t *)malloc(((size_t)groups + 1) * sizeof *fill);
    if (!fill) {
      free(gstart), free(mem), free(diag);
      rc = RKO_E_NOMEM;
      goto done;
    }
    memcpy(fill, gstart, ((size_t)groups + 1) * sizeof *fill);
    for (uint64_t k = 0; k < m; ++k) {
      uint32_t i = order[k];
      uint64_t y = y_start[i], d = diag[k];
      rko_rec r;
      r.key = y > d ? y - d : d - y; /* comparator key, commonFunctions.cpp:149-157 */
      r.tag = i;
      r.pad = 0;
      mem[fill[grp[k]]++] = r;
    }
    free(fill);
    /* sort_groups (commonFunctions.cpp:158) + flags (:106-115) */
    uint64_t w = 0;
    for (uint32_t g = 0; g < groups; ++g) {
      rko_rec *a = mem + gstart[g];
      size_t sz = (size_t)(gstart[g + 1] - gstart[g]);
      if (sz > 1) rko_std_sort(a, sz);
      for (size_t t = 0; t < sz; ++t, ++w) {
        out_order[w] = a[t].tag;
        gid[w] = g;
        repval[w] = sz == 1 ? 0 : (t == 0 ? 1 : 2);
      }
    }
    *n_out = w;
    *n_groups = groups;
    free(gstart), free(mem), free(diag);
  }

done:
  for (int s = 0; s < 2; ++s) {
    free(lx[s].head);
    free(ly[s].head);
  }
  free(pool.nodes);
  free(grp);
  free(pk);
  free(order);
  return rc;
}

/* ------------------------------------------------------------------------- */
/* egress: save_all_frag_pairs / save_frag_pair / store_frag                  */
/* (commonFunctions.cpp:101-146) -- ostream formats uint64 as %llu and float */
/* as (double) with %.6g.                                                     */
/* ------------------------------------------------------------------------- */
int rko_write_csv(const char *path, const rko_db *db, const uint32_t *gid,
                  const uint8_t *repval, const uint32_t *out_order, uint64_t n_out) {
  FILE *f = fopen(path, "wb");
  if (!f) return RKO_E_IO;
  static char iobuf[1 << 20];
  setvbuf(f, iobuf, _IOFBF, sizeof iobuf);
  fwrite(db->header, 1, db->header_len, f);
  for (uint64_t k = 0; k < n_out; ++k) {
    uint32_t i = out_order[k];
    float identity = (float)db->ident[i] * 100 / (float)db->length[i];
    fprintf(f, "Frag,%llu,%llu,%llu,%llu,%c,%llu,%llu,%llu,%llu,%g,%g,0,%u\n",
            (unsigned long long)db->x_start[i], (unsigned long long)db->y_start[i],
            (unsigned long long)db->x_end[i], (unsigned long long)db->y_end[i],
            (char)db->strand[i], (unsigned long long)gid[k],
            (unsigned long long)db->length[i], (unsigned long long)db->score[i],
            (unsigned long long)db->ident[i], (double)db->similarity[i], (double)identity,
            (unsigned)repval[k]);
  }
  return fclose(f) == 0 ? RKO_OK : RKO_E_IO;
}
