/* rk_oracle.h -- CPU restatement of estebanpw/repkiller's classification path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load or call this library, and only as the
 * checker / CPU baseline -- never as the product path (the product is
 * repkiller_amd/librepkiller_amd.so, which has no CPU fallback).
 *
 * The restatement is sequential and literal: it keeps the reference's four
 * push-front occupancy lists and probe order, so it is an independent check of
 * the data-parallel formulation the HIP kernels use.  Parity is pinned against
 * the reference itself (oracle/_ref, built from /root/reference/src by
 * oracle/ref.mk) through the committed fixtures in tests/golden/.
 */
#ifndef RK_ORACLE_H
#define RK_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  RKO_OK = 0,
  RKO_E_IO = -1,        /* input/output file cannot be opened            */
  RKO_E_COUNT = -2,     /* more accepted Frag lines than the header total */
  RKO_E_UB_BUCKET = -3, /* xStart/10 >= vsize: reference writes out of bounds */
  RKO_E_UB_CENTER = -4, /* a probe would index past an occupancy array     */
  RKO_E_NOMEM = -5,
  RKO_E_ARG = -6,
};

/* One parsed fragment file, file order, the fields repkiller keeps
 * (FragmentsDatabase.cpp:30-43). */
typedef struct {
  uint64_t n;
  uint64_t *x_start, *y_start, *x_end, *y_end, *length, *score, *ident;
  float *similarity;
  uint8_t *strand;
  char *header;          /* the 16 header lines exactly as echoed on output */
  size_t header_len;
  uint64_t len_x_hdr, len_y_hdr, total_hdr; /* raw header values (no +1) */
} rko_db;

int rko_load_csv(const char *path, rko_db *db);
void rko_free_db(rko_db *db);

/* Classify n fragments given in FILE order.  Outputs (caller-allocated, n
 * entries each, the first *n_out valid), all in OUTPUT order: out_order[k] =
 * file row written k-th, gid[k] its group id (block column), repval[k] its
 * repeat flag.  Rows of the dropped last xStart/10 bucket are not written.
 * *n_groups = groups created. */
int rko_classify(uint64_t n, const uint64_t *x_start, const uint64_t *y_start,
                 const uint64_t *length, const uint8_t *strand, uint64_t len_x_hdr,
                 uint64_t len_y_hdr, double len_ratio, double pos_ratio, uint32_t *gid,
                 uint8_t *repval, uint32_t *out_order, uint64_t *n_out, uint64_t *n_groups);

/* Write the reference's output CSV (commonFunctions.cpp:101-146). */
int rko_write_csv(const char *path, const rko_db *db, const uint32_t *gid,
                  const uint8_t *repval, const uint32_t *out_order, uint64_t n_out);

/* libstdc++ (GCC 11) std::sort restated for (key, tag) records compared by key
 * only; exposed so tests can cross-check it against std::sort directly. */
typedef struct { uint64_t key; uint32_t tag; uint32_t pad; } rko_rec;
void rko_std_sort(rko_rec *a, size_t n);

#ifdef __cplusplus
}
#endif
#endif
