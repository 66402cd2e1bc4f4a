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
// times as one JSON line on stderr), --gpus P (one fragment set sharded over
// P GPUs, devices N..N+P-1, one thread each: rk_classify_sharded over RCCL),
// --same-device (all P ranks on device N -- a rehearsal of the sharded path
// on one GPU), --comm rccl|local (collectives: RCCL, or in-process device
// copies; default rccl, local with --same-device), --save-soa PATH (after the
// parse, keep the database as a binary SoA cache), --soa (the input is such a
// cache: no parse at all).
#include <chrono>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "repkiller_amd.h"

static void print_help() {
  std::printf("Repkiller (MI355X) v0.9.b-compatible\n");
  std::printf("Usage: ./rk_repkiller [--device N] [--gpus P [--same-device] [--comm rccl|local]] "
              "[--timing] [--save-soa cache.soa | --soa] <input_file_path> <output_file_path> "
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

// One fragment set over `gpus` ranks, one thread each; every pair in turn.
// The ranks hold consecutive blocks of rows; each copies its output share into
// the full result arrays at its offset.
static int classify_sharded_threads(const rk_frags_soa &soa, int device, int gpus,
                                    bool same_device, bool local, const std::vector<rk_params> &ps,
                                    std::vector<rk_result> &rs, std::string &err) {
  std::vector<rk_comm *> comms(gpus, nullptr);
  uint8_t id[RK_COMM_ID_BYTES];
  if (local) {
    if (rk_comm_create_local(gpus, comms.data())) {
      err = "rk_comm_create_local failed";
      return 1;
    }
  } else if (rk_comm_rccl_id(id)) {
    err = "RCCL is not available";
    return 1;
  }
  std::vector<int> status(gpus, 0);
  std::vector<std::string> msgs(gpus);
  std::vector<std::thread> th;
  for (int r = 0; r < gpus; ++r)
    th.emplace_back([&, r] {
      const int dev = same_device ? device : device + r;
      if (!local && rk_comm_create_rccl(r, gpus, dev, id, &comms[r])) {
        status[r] = RK_E_HIP;
        msgs[r] = "rk_comm_create_rccl failed";
        return;
      }
      rk_ctx *ctx = nullptr;
      if ((status[r] = rk_create(&ctx, dev))) {
        msgs[r] = "no usable gfx950 device " + std::to_string(dev);
        // the peers' first pair waits for this rank: release them
        (void)rk_comm_abandon(comms[r], status[r]);
        return;
      }
      const uint64_t a = soa.n * (uint64_t)r / gpus, b = soa.n * (uint64_t)(r + 1) / gpus;
      const rk_frags_soa mine{soa.x_start + a, soa.y_start + a, soa.length + a,
                              soa.strand + a, b - a};
      for (size_t i = 0; i < ps.size() && !status[r]; ++i) {
        rk_shard_result res;
        status[r] = rk_classify_sharded_host(ctx, comms[r], &mine, &ps[i], -1, &res);
        if (!status[r])
          status[r] = rk_shard_copy_result(ctx, &res, rs[i].out_order + res.out_offset,
                                           rs[i].gid + res.out_offset,
                                           rs[i].repval + res.out_offset);
        if (status[r]) msgs[r] = rk_last_error(ctx);
        if (r == 0 && !status[r]) rs[i].n_out = res.n_out_total, rs[i].n_groups = res.n_groups;
      }
      rk_destroy(ctx);
    });
  for (auto &t : th) t.join();
  for (rk_comm *c : comms) rk_comm_destroy(c);
  for (int r = 0; r < gpus; ++r)
    if (status[r]) {
      err = "rank " + std::to_string(r) + ": " + msgs[r] + " (" + std::to_string(status[r]) + ")";
      return status[r];
    }
  return 0;
}

int main(int argc, char **argv) {
  int device = 0, gpus = 1;
  bool timing = false, same_device = false, soa_in = false;
  const char *comm_kind = nullptr, *save_soa = nullptr;
  std::vector<const char *> pos;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--device") && i + 1 < argc) device = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--gpus") && i + 1 < argc) gpus = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--comm") && i + 1 < argc) comm_kind = argv[++i];
    else if (!std::strcmp(argv[i], "--same-device")) same_device = true;
    else if (!std::strcmp(argv[i], "--timing")) timing = true;
    else if (!std::strcmp(argv[i], "--soa")) soa_in = true;
    else if (!std::strcmp(argv[i], "--save-soa") && i + 1 < argc) save_soa = argv[++i];
    else pos.push_back(argv[i]);
  }
  if (gpus < 1 || gpus > 32 ||
      (comm_kind && std::strcmp(comm_kind, "rccl") && std::strcmp(comm_kind, "local"))) {
    std::fprintf(stderr, "Invalid --gpus / --comm.\n");
    print_help();
    return 1;
  }
  const bool local = comm_kind ? !std::strcmp(comm_kind, "local") : same_device;
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
  int rc = soa_in ? rk_db_load_soa(pos[0], &db) : rk_db_load_csv(pos[0], &db);
  if (rc == RK_E_ARG && soa_in) {
    std::fprintf(stderr, "%s is not a complete SoA cache file.\n", pos[0]);
    return 1;
  }
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
  if (save_soa && (rc = rk_db_save_soa(db, save_soa))) {
    std::fprintf(stderr, "writing the SoA cache %s failed (%d)\n", save_soa, rc);
    rk_db_free(db);
    return 1;
  }
  double t1 = now_s();
  rk_frags_soa soa;
  uint64_t lx, ly, total;
  rk_db_view(db, &soa, &lx, &ly, &total);

  rk_ctx *ctx = nullptr;
  if (gpus == 1) {
    rc = rk_create(&ctx, device);
    if (rc) {
      std::fprintf(stderr, "no usable gfx950 device %d (%d)\n", device, rc);
      rk_db_free(db);
      return 1;
    }
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
  std::string err;
  if (gpus == 1) {
    rc = rk_classify_pairs(ctx, &soa, ps.data(), (uint32_t)q, rs.data());
    if (rc) err = rk_last_error(ctx);
  } else {
    rc = classify_sharded_threads(soa, device, gpus, same_device, local, ps, rs, err);
  }
  const double t_class = now_s() - a;
  if (rc) {
    std::fprintf(stderr, "classification failed (%d): %s\n", rc, err.c_str());
    rk_saver_stop(sq);
    rk_destroy(ctx);
    rk_db_free(db);
    return 1;
  }
  rk_stats stt{};
  if (ctx) rk_get_stats(ctx, &stt);
  const double dev_ms = stt.device_ms;
  for (size_t i = 0; i < q; ++i) rk_saver_add(sq, out_path.c_str(), &rs[i], soa.n);
  double t2 = now_s();
  rc = rk_saver_stop(sq);
  double t3 = now_s();
  rk_destroy(ctx);
  if (timing)
    std::fprintf(stderr,
                 "{\"frags\": %llu, \"pairs\": %zu, \"load_s\": %.6f, \"classify_s\": %.6f, "
                 "\"device_ms\": %.3f, \"save_s\": %.6f, \"gpus\": %d}\n",
                 (unsigned long long)soa.n, params.size(), t1 - t0, t_class, dev_ms, t3 - t2, gpus);
  rk_db_free(db);
  if (rc) {
    std::fprintf(stderr, "writing output failed (%d)\n", rc);
    return 1;
  }
  std::printf("Repkiller finished with no errors\n");
  return 0;
}
