// rk_host.cpp -- host ingress (FragmentsDatabase) and egress (CSV writer +
// SaverQueue) around the device classifier.
//
// Ingress restates /root/reference/src/FragmentsDatabase.cpp:17-101 with the
// same acceptance rules, byte for byte:
//   * 16 header lines read with std::getline semantics (a getline on a stream
//     already at EOF fails and leaves the previous line in place); lines 7, 8
//     and 13 give SeqX length, SeqY length and the fragment total, parsed as
//     atoll(text after the first ':') (:57-77);
//   * every later line is split into 14 ','-fields with std::getline on an
//     istringstream: an empty field rejects the line, and a line with fewer
//     than 14 fields repeats its last field (the stale-string rule above) (:23-27);
//   * field 0 must be exactly "Frag" (:29); xStart/yStart/xEnd/yEnd/length/score
//     are atoll (:30-38); ident = (uint64_t)stof(field 10) and similarity =
//     stof(field 10) (:39-40); a stof exception (no digits, ERANGE) rejects the
//     line (:46-48);
//   * more accepted lines than the header total is an error (:99).
// The file is memory-mapped and parsed by several threads over line-aligned
// chunks; rows keep file order.
//
// Egress restates save_all_frag_pairs / save_frag_pair / store_frag
// (commonFunctions.cpp:101-146): header echo, then one line per member, group
// by group, in the order rk_classify returns; floats print as ostream does
// (%.6g of the value widened to double).  rk_saver_* mirrors SaverQueue
// (SaverQueue.cpp:4-51) without its races: the worker re-checks the queue
// after every wake-up and drains it before stop() returns.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <climits>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "repkiller_amd.h"
#include "rk_format.h"

struct rk_db {
  std::vector<uint64_t> x_start, y_start, x_end, y_end, length, score, ident;
  std::vector<float> similarity;
  std::vector<uint8_t> strand;
  std::string header;
  uint64_t len_x_hdr = 0, len_y_hdr = 0, total_hdr = 0;
};

namespace {

// ---------------------------------------------------------------- numbers --

inline bool c_isspace(unsigned char c) { return c == ' ' || (c >= '\t' && c <= '\r'); }

// atoll == strtoll(s, NULL, 10) on the field's c_str(): leading white space,
// optional sign, decimal digits; saturates at LLONG_MAX/LLONG_MIN; stops at
// the first non-digit (an embedded NUL included).
uint64_t parse_atoll(const char *p, const char *e) {
  while (p < e && c_isspace((unsigned char)*p)) ++p;
  bool neg = false;
  if (p < e && (*p == '+' || *p == '-')) neg = *p++ == '-';
  unsigned long long acc = 0;
  bool over = false;
  const unsigned long long lim = neg ? (unsigned long long)LLONG_MAX + 1ull : (unsigned long long)LLONG_MAX;
  for (; p < e && *p >= '0' && *p <= '9'; ++p) {
    unsigned d = (unsigned)(*p - '0');
    if (!over && acc > (lim - d) / 10) over = true;
    if (!over) acc = acc * 10 + d;
  }
  if (over) acc = lim;
  long long v = neg ? (long long)(0ull - acc) : (long long)acc;
  return (uint64_t)v;
}

// std::stof: strtof on the field's c_str(); throws (=> line rejected) when no
// characters convert or errno == ERANGE.
bool parse_stof(const char *p, const char *e, float *out) {
  if (rk::fast_stof(p, e, out)) return true;
  char small[96];
  std::string big;
  size_t n = (size_t)(e - p);
  const char *s;
  if (n < sizeof small) {
    std::memcpy(small, p, n);
    small[n] = 0;
    s = small;
  } else {
    big.assign(p, n);
    s = big.c_str();
  }
  char *end = nullptr;
  errno = 0;
  float v = std::strtof(s, &end);
  if (end == s || errno == ERANGE) return false;
  *out = v;
  return true;
}

// (uint64_t)float as the x86-64 reference binary evaluates it: below 2^63
// (ordered compare) -> cvttss2si; else cvttss2si(x - 2^63) ^ 2^63; cvttss2si of
// NaN / out of range -> 0x8000000000000000.
uint64_t cvtt_si64(float x) {
  if (std::isnan(x) || x >= 9223372036854775808.0f || x < -9223372036854775808.0f)
    return 0x8000000000000000ull;
  return (uint64_t)(int64_t)x;
}
uint64_t float_to_u64_x86(float x) {
  if (!(x >= 9223372036854775808.0f)) return cvtt_si64(x);
  return cvtt_si64(x - 9223372036854775808.0f) ^ 0x8000000000000000ull;
}

// ------------------------------------------------------------------ lines --

struct Row {
  uint64_t xs, ys, xe, ye, len, score, ident;
  float sim;
  uint8_t strand;
};

// One body line -> Row, or false if readFragment would return false.
bool parse_line(const char *b, const char *e, Row *r) {
  const char *fb[14], *fe[14];
  const char *p = b;
  int k = 0;
  bool at_eof = false;
  while (k < 14) {
    if (at_eof) {  // sentry fails: the previous field stays in the string
      fb[k] = fb[k - 1];
      fe[k] = fe[k - 1];
      ++k;
      continue;
    }
    const char *c = (const char *)std::memchr(p, ',', (size_t)(e - p));
    if (c) {
      fb[k] = p;
      fe[k] = c;
      p = c + 1;
    } else {
      fb[k] = p;
      fe[k] = e;
      p = e;
      at_eof = true;
    }
    if (fe[k] == fb[k]) return false;
    ++k;
  }
  if (fe[0] - fb[0] != 4 || std::memcmp(fb[0], "Frag", 4) != 0) return false;
  float sim;
  if (!parse_stof(fb[10], fe[10], &sim)) return false;
  r->xs = parse_atoll(fb[1], fe[1]);
  r->ys = parse_atoll(fb[2], fe[2]);
  r->xe = parse_atoll(fb[3], fe[3]);
  r->ye = parse_atoll(fb[4], fe[4]);
  r->strand = (uint8_t)fb[5][0];
  r->len = parse_atoll(fb[7], fe[7]);
  r->score = parse_atoll(fb[8], fe[8]);
  r->ident = float_to_u64_x86(sim);
  r->sim = sim;
  return true;
}

uint64_t header_number(const char *b, const char *e) {
  const char *c = (const char *)std::memchr(b, ':', (size_t)(e - b));
  return parse_atoll(c ? c + 1 : b, e);
}

struct Mapped {
  const char *p = nullptr;
  size_t n = 0;
  int fd = -1;
  ~Mapped() {
    if (p && n) munmap((void *)p, n);
    if (fd >= 0) close(fd);
  }
};

}  // namespace

extern "C" int rk_db_load_csv(const char *path, rk_db **out) {
  if (!path || !out) return RK_E_ARG;
  *out = nullptr;
  Mapped m;
  m.fd = open(path, O_RDONLY);
  if (m.fd < 0) return RK_E_IO;
  struct stat st;
  if (fstat(m.fd, &st) != 0) return RK_E_IO;
  m.n = (size_t)st.st_size;
  if (m.n) {
    void *q = mmap(nullptr, m.n, PROT_READ, MAP_PRIVATE, m.fd, 0);
    if (q == MAP_FAILED) return RK_E_IO;
    m.p = (const char *)q;
    madvise(q, m.n, MADV_SEQUENTIAL);
  }
  auto db = new (std::nothrow) rk_db;
  if (!db) return RK_E_NOMEM;

  // ---- header: 16 std::getline calls on the file stream
  const char *p = m.p, *end = m.p + m.n;
  bool eof = false;
  const char *lb = p, *le = p;  // current `line` contents
  for (int k = 1; k <= 16; ++k) {
    if (!eof) {
      const char *nl = (const char *)std::memchr(p, '\n', (size_t)(end - p));
      lb = p;
      if (nl) {
        le = nl;
        p = nl + 1;
      } else {
        le = end;
        p = end;
        eof = true;
      }
    }
    db->header.append(lb, (size_t)(le - lb)).push_back('\n');
    if (k == 7) db->len_x_hdr = header_number(lb, le);
    if (k == 8) db->len_y_hdr = header_number(lb, le);
    if (k == 13) db->total_hdr = header_number(lb, le);
  }

  // ---- body: line-aligned chunks parsed in parallel, concatenated in order
  if (!eof && p < end) {
    unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    size_t body = (size_t)(end - p);
    if (body < (size_t)(4u << 20)) nt = 1;
    std::vector<const char *> cut(nt + 1);
    cut[0] = p;
    cut[nt] = end;
    for (unsigned t = 1; t < nt; ++t) {
      const char *q = p + body / nt * t;
      if (q < cut[t - 1]) q = cut[t - 1];
      const char *nl = (const char *)std::memchr(q, '\n', (size_t)(end - q));
      cut[t] = nl ? nl + 1 : end;
    }
    std::vector<std::vector<Row>> parts(nt);
    auto work = [&](unsigned t) {
      const char *q = cut[t], *qe = cut[t + 1];
      auto &v = parts[t];
      v.reserve((size_t)(qe - q) / 48 + 16);
      while (q < qe) {
        const char *nl = (const char *)std::memchr(q, '\n', (size_t)(qe - q));
        const char *le2 = nl ? nl : qe;
        Row r;
        if (parse_line(q, le2, &r)) v.push_back(r);
        q = nl ? nl + 1 : qe;
      }
    };
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nt; ++t) th.emplace_back(work, t);
    work(0);
    for (auto &t : th) t.join();
    size_t n = 0;
    for (auto &v : parts) n += v.size();
    if (n > db->total_hdr) {
      delete db;
      return RK_E_COUNT;
    }
    db->x_start.resize(n), db->y_start.resize(n), db->x_end.resize(n), db->y_end.resize(n);
    db->length.resize(n), db->score.resize(n), db->ident.resize(n);
    db->similarity.resize(n), db->strand.resize(n);
    // every part into the columns at its offset, one thread per part
    std::vector<size_t> at(nt + 1, 0);
    for (unsigned t = 0; t < nt; ++t) at[t + 1] = at[t] + parts[t].size();
    auto place = [&](unsigned t) {
      size_t i = at[t];
      for (const Row &r : parts[t]) {
        db->x_start[i] = r.xs, db->y_start[i] = r.ys, db->x_end[i] = r.xe, db->y_end[i] = r.ye;
        db->length[i] = r.len, db->score[i] = r.score, db->ident[i] = r.ident;
        db->similarity[i] = r.sim, db->strand[i] = r.strand;
        ++i;
      }
      std::vector<Row>().swap(parts[t]);
    };
    std::vector<std::thread> th2;
    for (unsigned t = 1; t < nt; ++t) th2.emplace_back(place, t);
    place(0);
    for (auto &t : th2) t.join();
  }
  *out = db;
  return RK_OK;
}

// ------------------------------------------------------ binary SoA cache --
// the parse is the largest host cost of the file path
// (FragmentsDatabase.cpp:17-100, ~1.2 us per line in the reference, 2.8 s for
// cfg3's 4-GB file here), so a parsed database can be kept as its SoA columns:
//   "RKSOA001" | u64 n, len_x_hdr, len_y_hdr, total_hdr, header bytes |
//   header text | x_start, y_start, x_end, y_end, length, score, ident (u64),
//   similarity (f32), strand (u8) -- each section starting on a 4-KB boundary
//   | u64 checksum of the fixed fields and the header.
// The columns are exactly what rk_db_load_csv produced (rows accepted by the
// reference's rules, in file order), so classification and egress from a
// loaded cache are byte-identical to the CSV route.  Columns are written and
// read by several threads at their own file offsets (pwrite / pread).
namespace {

constexpr char kSoaMagic[8] = {'R', 'K', 'S', 'O', 'A', '0', '0', '1'};
constexpr size_t kSoaAlign = 4096;

struct SoaLayout {
  uint64_t n, header_bytes;
  size_t col_off[9];  // x_start .. strand
  size_t sum_off, total;
};

size_t soa_round(size_t v) { return (v + kSoaAlign - 1) & ~(kSoaAlign - 1); }

SoaLayout soa_layout(uint64_t n, uint64_t header_bytes) {
  SoaLayout L{};
  L.n = n;
  L.header_bytes = header_bytes;
  size_t o = soa_round(48 + header_bytes);
  const size_t width[9] = {8, 8, 8, 8, 8, 8, 8, 4, 1};
  for (int c = 0; c < 9; ++c) {
    L.col_off[c] = o;
    o = soa_round(o + (size_t)n * width[c]);
  }
  L.sum_off = o;
  L.total = o + 8;
  return L;
}

uint64_t soa_checksum(const uint64_t fixed[5], const std::string &header) {
  uint64_t h = 0xcbf29ce484222325ull;
  auto mix = [&](const void *p, size_t n) {
    const uint8_t *b = (const uint8_t *)p;
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 0x100000001b3ull;
  };
  mix(fixed, 40);
  mix(header.data(), header.size());
  return h;
}

// [off, off + bytes) of fd <-> buf, split over up to 16 threads
bool soa_io(int fd, void *buf, size_t bytes, size_t off, bool write) {
  if (!bytes) return true;
  const unsigned nt = (unsigned)std::max<size_t>(
      1, std::min<size_t>({16, std::max(1u, std::thread::hardware_concurrency()),
                           bytes / (8u << 20) + 1}));
  std::atomic<bool> ok{true};
  auto work = [&](unsigned t) {
    size_t a = bytes * t / nt, b = bytes * (t + 1) / nt;
    char *p = (char *)buf;
    while (a < b && ok) {
      const size_t chunk = std::min<size_t>(b - a, (size_t)1 << 30);
      const ssize_t r = write ? pwrite(fd, p + a, chunk, (off_t)(off + a))
                              : pread(fd, p + a, chunk, (off_t)(off + a));
      if (r <= 0) {
        if (r < 0 && errno == EINTR) continue;
        ok = false;
        break;
      }
      a += (size_t)r;
    }
  };
  std::vector<std::thread> th;
  for (unsigned t = 1; t < nt; ++t) th.emplace_back(work, t);
  work(0);
  for (auto &t : th) t.join();
  return ok;
}

}  // namespace

extern "C" int rk_db_save_soa(const rk_db *db, const char *path) {
  if (!db || !path) return RK_E_ARG;
  const uint64_t n = db->x_start.size();
  const SoaLayout L = soa_layout(n, db->header.size());
  const int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) return RK_E_IO;
  bool ok = ftruncate(fd, (off_t)L.total) == 0;
  const uint64_t fixed[5] = {n, db->len_x_hdr, db->len_y_hdr, db->total_hdr, L.header_bytes};
  std::vector<char> head(48 + db->header.size());
  std::memcpy(head.data(), kSoaMagic, 8);
  std::memcpy(head.data() + 8, fixed, 40);
  std::memcpy(head.data() + 48, db->header.data(), db->header.size());
  ok = ok && soa_io(fd, head.data(), head.size(), 0, true);
  const void *cols[9] = {db->x_start.data(), db->y_start.data(), db->x_end.data(),
                         db->y_end.data(),   db->length.data(),  db->score.data(),
                         db->ident.data(),   db->similarity.data(), db->strand.data()};
  const size_t width[9] = {8, 8, 8, 8, 8, 8, 8, 4, 1};
  for (int c = 0; c < 9 && ok; ++c)
    ok = soa_io(fd, const_cast<void *>(cols[c]), (size_t)n * width[c], L.col_off[c], true);
  uint64_t sum = soa_checksum(fixed, db->header);
  ok = ok && soa_io(fd, &sum, 8, L.sum_off, true);
  ok = (close(fd) == 0) && ok;
  return ok ? RK_OK : RK_E_IO;
}

extern "C" int rk_db_load_soa(const char *path, rk_db **out) {
  if (!path || !out) return RK_E_ARG;
  *out = nullptr;
  const int fd = open(path, O_RDONLY);
  if (fd < 0) return RK_E_IO;
  struct Closer {
    int fd;
    ~Closer() { close(fd); }
  } closer{fd};
  struct stat st;
  if (fstat(fd, &st) != 0) return RK_E_IO;
  char head[48];
  if ((size_t)st.st_size < 48 || !soa_io(fd, head, 48, 0, false)) return RK_E_IO;
  if (std::memcmp(head, kSoaMagic, 8) != 0) return RK_E_ARG;  // not a cache file
  uint64_t fixed[5];
  std::memcpy(fixed, head + 8, 40);
  const uint64_t n = fixed[0];
  if (n >= (1ull << 40) || fixed[4] >= (1ull << 32)) return RK_E_ARG;
  const SoaLayout L = soa_layout(n, fixed[4]);
  if ((size_t)st.st_size != L.total) return RK_E_ARG;  // truncated or foreign
  auto db = std::unique_ptr<rk_db>(new (std::nothrow) rk_db);
  if (!db) return RK_E_NOMEM;
  db->len_x_hdr = fixed[1];
  db->len_y_hdr = fixed[2];
  db->total_hdr = fixed[3];
  try {
    db->header.resize(fixed[4]);
    db->x_start.resize(n), db->y_start.resize(n), db->x_end.resize(n), db->y_end.resize(n);
    db->length.resize(n), db->score.resize(n), db->ident.resize(n);
    db->similarity.resize(n), db->strand.resize(n);
  } catch (...) {
    return RK_E_NOMEM;
  }
  if (!soa_io(fd, &db->header[0], fixed[4], 48, false)) return RK_E_IO;
  void *cols[9] = {db->x_start.data(), db->y_start.data(), db->x_end.data(),
                   db->y_end.data(),   db->length.data(),  db->score.data(),
                   db->ident.data(),   db->similarity.data(), db->strand.data()};
  const size_t width[9] = {8, 8, 8, 8, 8, 8, 8, 4, 1};
  for (int c = 0; c < 9; ++c)
    if (!soa_io(fd, cols[c], (size_t)n * width[c], L.col_off[c], false)) return RK_E_IO;
  uint64_t sum = 0;
  if (!soa_io(fd, &sum, 8, L.sum_off, false)) return RK_E_IO;
  if (sum != soa_checksum(fixed, db->header)) return RK_E_ARG;
  *out = db.release();
  return RK_OK;
}

extern "C" void rk_db_free(rk_db *db) { delete db; }

extern "C" int rk_db_view(const rk_db *db, rk_frags_soa *soa, uint64_t *len_x_hdr,
                          uint64_t *len_y_hdr, uint64_t *total_hdr) {
  if (!db) return RK_E_ARG;
  if (soa) {
    soa->x_start = db->x_start.data();
    soa->y_start = db->y_start.data();
    soa->length = db->length.data();
    soa->strand = db->strand.data();
    soa->n = db->x_start.size();
  }
  if (len_x_hdr) *len_x_hdr = db->len_x_hdr;
  if (len_y_hdr) *len_y_hdr = db->len_y_hdr;
  if (total_hdr) *total_hdr = db->total_hdr;
  return RK_OK;
}

// ------------------------------------------------------------------ egress --

namespace {

using rk::put_float;
using rk::put_u64;

// store_frag (commonFunctions.cpp:101-104)
inline char *format_row(char *o, const rk_db *db, uint32_t i, uint64_t gid, unsigned rep) {
  std::memcpy(o, "Frag,", 5);
  o += 5;
  o = put_u64(o, db->x_start[i]);
  *o++ = ',';
  o = put_u64(o, db->y_start[i]);
  *o++ = ',';
  o = put_u64(o, db->x_end[i]);
  *o++ = ',';
  o = put_u64(o, db->y_end[i]);
  *o++ = ',';
  *o++ = (char)db->strand[i];
  *o++ = ',';
  o = put_u64(o, gid);
  *o++ = ',';
  o = put_u64(o, db->length[i]);
  *o++ = ',';
  o = put_u64(o, db->score[i]);
  *o++ = ',';
  o = put_u64(o, db->ident[i]);
  *o++ = ',';
  o = put_float(o, db->similarity[i]);
  *o++ = ',';
  float identity = (float)db->ident[i] * 100 / (float)db->length[i];
  o = put_float(o, identity);
  std::memcpy(o, ",0,", 3);
  o += 3;
  o = put_u64(o, rep);
  *o++ = '\n';
  return o;
}

int write_csv(const rk_db *db, const char *path, const uint32_t *gid, const uint8_t *rep,
               const uint32_t *order, uint64_t n_out) {
  const int fd = ::open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) return RK_E_IO;
  const uint64_t n_rows = db->x_start.size();
  // every chunk of rows is formatted into its own buffer in parallel, then
  // the chunks are written in parallel at their prefix-sum offsets (pwrite)
  const uint64_t chunk = 1u << 16;
  const uint64_t n_chunks = (n_out + chunk - 1) / chunk;
  unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (n_out < 4 * chunk) nt = 1;
  // a row is at most 5 + 10 * 21 + 2 * 16 + 4 bytes < 256; the buffers are
  // not zero-filled (only the formatted bytes are ever touched)
  std::vector<std::unique_ptr<char[]>> bufs(n_chunks);
  std::vector<size_t> blen(n_chunks, 0);
  std::atomic<bool> bad{false};
  std::atomic<uint64_t> next{0};
  auto fmt = [&]() {
    for (uint64_t c; (c = next.fetch_add(1)) < n_chunks;) {
      const uint64_t k0 = c * chunk, k1 = std::min(n_out, k0 + chunk);
      bufs[c].reset(new (std::nothrow) char[(size_t)(k1 - k0) * 256]);
      if (!bufs[c]) {
        bad = true;
        break;
      }
      char *const b0 = bufs[c].get();
      char *o = b0;
      // the rows come in output order, i.e. scattered over the nine columns:
      // each row's column words are prefetched PF rows ahead, so a thread
      // keeps that many rows' cache misses in flight instead of one
      constexpr uint64_t PF = 12;
      auto prefetch_row = [&](uint64_t k) {
        const uint32_t i = order[k];
        if (i >= n_rows) return;
        __builtin_prefetch(&db->x_start[i]);
        __builtin_prefetch(&db->y_start[i]);
        __builtin_prefetch(&db->x_end[i]);
        __builtin_prefetch(&db->y_end[i]);
        __builtin_prefetch(&db->strand[i]);
        __builtin_prefetch(&db->length[i]);
        __builtin_prefetch(&db->score[i]);
        __builtin_prefetch(&db->ident[i]);
        __builtin_prefetch(&db->similarity[i]);
      };
      for (uint64_t k = k0; k < k1 && k < k0 + PF; ++k) prefetch_row(k);
      for (uint64_t k = k0; k < k1; ++k) {
        if (k + PF < k1) prefetch_row(k + PF);
        const uint32_t i = order[k];
        if (i >= n_rows) {
          bad = true;
          break;
        }
        o = format_row(o, db, i, gid[k], rep[k]);
      }
      blen[c] = (size_t)(o - b0);
    }
  };
  {
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nt; ++t) th.emplace_back(fmt);
    fmt();
    for (auto &t : th) t.join();
  }
  if (bad) {
    ::close(fd);
    return RK_E_ARG;
  }
  std::vector<uint64_t> off(n_chunks + 1);
  off[0] = db->header.size();
  for (uint64_t c = 0; c < n_chunks; ++c) off[c + 1] = off[c] + blen[c];
  auto put = [fd](const char *p, size_t len, uint64_t at) {
    while (len) {
      const ssize_t w = ::pwrite(fd, p, len, (off_t)at);
      if (w <= 0) {
        if (w < 0 && errno == EINTR) continue;
        return false;
      }
      p += w, len -= (size_t)w, at += (uint64_t)w;
    }
    return true;
  };
  std::atomic<bool> ok{put(db->header.data(), db->header.size(), 0)};
  next = 0;
  auto wr = [&]() {
    for (uint64_t c; (c = next.fetch_add(1)) < n_chunks;)
      if (!put(bufs[c].get(), blen[c], off[c])) ok = false;
  };
  {
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nt; ++t) th.emplace_back(wr);
    wr();
    for (auto &t : th) t.join();
  }
  if (::close(fd) != 0) ok = false;
  return ok ? RK_OK : RK_E_IO;
}

}  // namespace

extern "C" int rk_db_write_csv(const rk_db *db, const char *path, const rk_result *res) {
  if (!db || !path || !res || (res->n_out && (!res->gid || !res->repval || !res->out_order)))
    return RK_E_ARG;
  return write_csv(db, path, res->gid, res->repval, res->out_order, res->n_out);
}

// ------------------------------------------------------------- SaverQueue --

struct rk_saver {
  struct Req {
    std::string path;
    std::vector<uint32_t> gid, order;
    std::vector<uint8_t> rep;
    uint64_t n_out;
  };
  const rk_db *db;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<Req> q;
  bool running = true;
  size_t fallback_count = 0;
  int status = RK_OK;
  std::thread th;

  void run() {
    for (;;) {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return !q.empty() || !running; });
      if (q.empty()) return;  // stopped and drained
      Req r = std::move(q.front());
      q.pop_front();
      lk.unlock();
      int rc = write_csv(db, r.path.c_str(), r.gid.data(), r.rep.data(), r.order.data(), r.n_out);
      if (rc == RK_E_IO) {  // SaverQueue.cpp:16-20
        std::string alt = "represults-" + std::to_string(++fallback_count) + ".csv";
        std::fprintf(stderr, "Couldn't access %s, saving into %s\n", r.path.c_str(), alt.c_str());
        rc = write_csv(db, alt.c_str(), r.gid.data(), r.rep.data(), r.order.data(), r.n_out);
      }
      if (rc != RK_OK) {
        std::lock_guard<std::mutex> g(mu);
        status = rc;
      }
    }
  }
};

extern "C" int rk_saver_start(const rk_db *db, rk_saver **sq) {
  if (!db || !sq) return RK_E_ARG;
  auto s = new (std::nothrow) rk_saver;
  if (!s) return RK_E_NOMEM;
  s->db = db;
  s->th = std::thread([s] { s->run(); });
  *sq = s;
  return RK_OK;
}

extern "C" int rk_saver_add(rk_saver *sq, const char *path, const rk_result *res, uint64_t n) {
  if (!sq || !path || !res) return RK_E_ARG;
  rk_saver::Req r;
  r.path = path;
  (void)n;
  r.gid.assign(res->gid, res->gid + res->n_out);
  r.rep.assign(res->repval, res->repval + res->n_out);
  r.order.assign(res->out_order, res->out_order + res->n_out);
  r.n_out = res->n_out;
  {
    std::lock_guard<std::mutex> g(sq->mu);
    sq->q.push_back(std::move(r));
  }
  sq->cv.notify_all();
  return RK_OK;
}

extern "C" int rk_saver_stop(rk_saver *sq) {
  if (!sq) return RK_E_ARG;
  {
    std::lock_guard<std::mutex> g(sq->mu);
    sq->running = false;
  }
  sq->cv.notify_all();
  sq->th.join();
  int st = sq->status;
  delete sq;
  return st;
}
