/* rk_oracle CLI -- TEST INFRASTRUCTURE ONLY.  Same positional interface as the
 * reference for one parameter pair (commonFunctions.cpp:5,9-30):
 *   rk_oracle <in.csv> <out.csv> <len_ratio> <pos_ratio>
 * Prints per-phase wall times as one JSON line on stderr. */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "rk_oracle.h"

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int main(int argc, char **argv) {
  if (argc != 5) {
    fprintf(stderr, "usage: %s in.csv out.csv len_ratio pos_ratio\n", argv[0]);
    return 2;
  }
  double lr = atof(argv[3]), pr = atof(argv[4]);
  if (lr <= 0 || pr <= 0) {  /* commonFunctions.cpp:26-27: NaN passes */
    fprintf(stderr, "ratios must be greater than zero\n");
    return 1;
  }
  double t0 = now_s();
  rko_db db;
  int rc = rko_load_csv(argv[1], &db);
  if (rc) {
    fprintf(stderr, "load failed: %d\n", rc);
    return 3;
  }
  double t1 = now_s();
  uint32_t *gid = malloc(db.n * sizeof *gid + 1), *order = malloc(db.n * sizeof *order + 1);
  uint8_t *rep = malloc(db.n + 1);
  uint64_t n_out = 0, n_groups = 0;
  rc = rko_classify(db.n, db.x_start, db.y_start, db.length, db.strand, db.len_x_hdr,
                    db.len_y_hdr, lr, pr, gid, rep, order, &n_out, &n_groups);
  if (rc) {
    fprintf(stderr, "classify failed: %d\n", rc);
    return 4;
  }
  double t2 = now_s();
  rc = rko_write_csv(argv[2], &db, gid, rep, order, n_out);
  double t3 = now_s();
  fprintf(stderr, "{\"frags\": %llu, \"grouped\": %llu, \"groups\": %llu, \"load_s\": %.6f, "
          "\"classify_s\": %.6f, \"save_s\": %.6f}\n", (unsigned long long)db.n,
          (unsigned long long)n_out, (unsigned long long)n_groups, t1 - t0, t2 - t1, t3 - t2);
  rko_free_db(&db);
  free(gid), free(order), free(rep);
  return rc ? 5 : 0;
}
