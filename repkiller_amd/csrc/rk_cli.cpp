// rk_repkiller -- command-line driver with the reference's interface
// (/root/reference/src/repkiller.cpp:26-97, commonFunctions.cpp:3-30):
//
//   rk_repkiller <input.csv> <output.csv> <len_ratio> <pos_ratio> [<len_ratio> <pos_ratio>]...
//
// Loads the CSV once (FragmentsDatabase), classifies every (len_ratio,
// pos_ratio) pair on the GPU and hands each result to the SaverQueue writer.
// Like the reference, every pair writes the same output path; here the pairs
// run in order, so the LAST pair's result is the file left behind (the
// reference's 3-thread pool makes that nondeterministic).
// Differences kept deliberately: an odd number of ratio arguments is a usage
// error (the reference throws std::out_of_range and aborts), and every failure
// exits non-zero with a message instead of std::terminate.
//
// Options (before the positional arguments): --device N, --timing (phase
// times as one JSON line on stderr).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "repkiller_amd.h"

static void print_help() {
  std::printf("Repkiller (MI355X) v0.9.b-compatible\n");
  std::printf("Usage: ./rk_repkiller [--device N] [--timing] <input_file_path> <output_file_path> "
              "<length_ratio> <position_ratio> [<length_ratio> <position_ratio>]...\n");
  std::fflush(stdout);
}

static double now_s() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

static bool parse_ratio(const char *s, double *v) {
  char *end = nullptr;
  *v = std::strtod(s, &end);
  return end != s;
}

int main(int argc, char **argv) {
  int device = 0;
  bool timing = false;
  std::vector<const char *> pos;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--device") && i + 1 < argc) device = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--timing")) timing = true;
    else pos.push_back(argv[i]);
  }
  // init_args (commonFunctions.cpp:14-29)
  if (pos.size() < 4 || (pos.size() - 2) % 2 != 0) {
    std::fprintf(stderr, "Invalid number of arguments.\n");
    print_help();
    return 1;
  }
  std::vector<std::pair<double, double>> params;
  for (size_t i = 2; i + 1 < pos.size(); i += 2) {
    double lr, pr;
    if (!parse_ratio(pos[i], &lr) || !parse_ratio(pos[i + 1], &pr)) {
      std::fprintf(stderr, "Invalid ratio argument.\n");
      print_help();
      return 1;
    }
    if (lr <= 0) {
      std::fprintf(stderr, "Ratio between length and position must be greater than zero\n");
      print_help();
      return 1;
    }
    if (pr <= 0) {
      std::fprintf(stderr, "Position proximity must be greater than zero\n");
      print_help();
      return 1;
    }
    params.emplace_back(lr, pr);
  }
  const std::string out_path = pos[1];
  if (out_path.empty()) {
    std::fprintf(stderr, "Output file name is missing\n");
    return 1;
  }

  std::printf("--- Running REPKILLER (MI355X) ---\n\n");
  std::fflush(stdout);
  double t0 = now_s();
  rk_db *db = nullptr;
  int rc = rk_db_load_csv(pos[0], &db);
  if (rc == RK_E_IO) {
    std::fprintf(stderr, "Could not open input file %s.\n", pos[0]);
    return 1;
  }
  if (rc == RK_E_COUNT) {
    std::fprintf(stderr, "Unexpected number of fragments\n");
    return 1;
  }
  if (rc) {
    std::fprintf(stderr, "loading %s failed (%d)\n", pos[0], rc);
    return 1;
  }
  double t1 = now_s();
  rk_frags_soa soa;
  uint64_t lx, ly, total;
  rk_db_view(db, &soa, &lx, &ly, &total);

  rk_ctx *ctx = nullptr;
  rc = rk_create(&ctx, device);
  if (rc) {
    std::fprintf(stderr, "no usable gfx950 device %d (%d)\n", device, rc);
    rk_db_free(db);
    return 1;
  }
  rk_saver *sq = nullptr;
  rk_saver_start(db, &sq);
  // every pair over the one fragment set in one call: the ratio-independent
  // work (processing order, occupancy axes, sort keys) is shared
  const size_t q = params.size();
  std::vector<uint32_t> gid(q * soa.n), order(q * soa.n);
  std::vector<uint8_t> rep(q * soa.n);
  std::vector<rk_params> ps(q);
  std::vector<rk_result> rs(q);
  for (size_t i = 0; i < q; ++i) {
    ps[i] = rk_params{lx, ly, params[i].first, params[i].second};
    rs[i] = rk_result{order.data() + i * soa.n, gid.data() + i * soa.n, rep.data() + i * soa.n,
                      0, 0};
  }
  double a = now_s();
  rc = rk_classify_pairs(ctx, &soa, ps.data(), (uint32_t)q, rs.data());
  const double t_class = now_s() - a;
  if (rc) {
    std::fprintf(stderr, "classification failed (%d): %s\n", rc, rk_last_error(ctx));
    rk_saver_stop(sq);
    rk_destroy(ctx);
    rk_db_free(db);
    return 1;
  }
  rk_stats stt;
  rk_get_stats(ctx, &stt);
  const double dev_ms = stt.device_ms;
  for (size_t i = 0; i < q; ++i) rk_saver_add(sq, out_path.c_str(), &rs[i], soa.n);
  double t2 = now_s();
  rc = rk_saver_stop(sq);
  double t3 = now_s();
  rk_destroy(ctx);
  if (timing)
    std::fprintf(stderr,
                 "{\"frags\": %llu, \"pairs\": %zu, \"load_s\": %.6f, \"classify_s\": %.6f, "
                 "\"device_ms\": %.3f, \"save_s\": %.6f}\n",
                 (unsigned long long)soa.n, params.size(), t1 - t0, t_class, dev_ms, t3 - t2);
  rk_db_free(db);
  if (rc) {
    std::fprintf(stderr, "writing output failed (%d)\n", rc);
    return 1;
  }
  std::printf("Repkiller finished with no errors\n");
  return 0;
}
