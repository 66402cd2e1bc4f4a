// Synchronous timing/parity driver for the reference repkiller.  TEST
// INFRASTRUCTURE ONLY -- linked against the reference's own translation units
// (FragmentsDatabase.cpp, SequenceOcupationList.cpp, commonFunctions.cpp,
// class_structs.cpp) compiled from /root/reference/src by oracle/ref.mk.
//
// It runs exactly the sequence of the reference's main()/execWithParams()
// (/root/reference/src/repkiller.cpp:31-96) for ONE (len_ratio, pos_ratio)
// pair, with save_all_frag_pairs() called directly instead of through the
// SaverQueue thread (whose pack(1) layout aborts on this glibc),
// and prints per-phase wall times as one JSON line on stderr.
//
//   usage: ref_driver <in.csv> <out.csv|-> <len_ratio> <pos_ratio>
//   out "-" skips the CSV write (timing runs).
#include <chrono>
#include <cstdio>
#include <string>
#include <vector>
#include <queue>

#include "FragmentsDatabase.h"
#include "commonFunctions.h"

static double now_s() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
  if (argc != 5) {
    std::fprintf(stderr, "usage: %s in.csv out.csv|- len_ratio pos_ratio\n", argv[0]);
    return 2;
  }
  std::string out_path, in_path;
  std::queue<std::pair<double, double>> params;
  std::ifstream frags_file;
  std::vector<std::string> args(argv, argv + argc);
  bool write_out = std::string(argv[2]) != "-";
  if (!write_out) args[2] = "unused";
  try {
    init_args(args, frags_file, out_path, in_path, params);   // commonFunctions.cpp:9
  } catch (const std::invalid_argument &e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 1;
  }
  double t0 = now_s();
  sequence_manager sm;
  FragmentsDatabase db(frags_file, sm);                         // FragmentsDatabase.cpp:54
  frags_file.close();
  double t1 = now_s();
  auto param = params.front();
  FGList *groups = new FGList;
  generate_fragment_groups(db, *groups, sm, param.first, param.second);  // commonFunctions.cpp:41
  double t2 = now_s();
  size_t *diag = new size_t[db.getA()];
  generate_diagonal_func(db, diag);                             // commonFunctions.cpp:161
  sort_groups(*groups, diag);                                   // commonFunctions.cpp:148
  delete[] diag;
  double t3 = now_s();
  if (write_out) save_all_frag_pairs(out_path, sm, *groups);    // commonFunctions.cpp:131
  double t4 = now_s();
  size_t members = 0;
  for (auto g : *groups) members += g->size();
  std::fprintf(stderr,
               "{\"frags\": %llu, \"grouped\": %zu, \"groups\": %zu, \"load_s\": %.6f, "
               "\"group_s\": %.6f, \"diag_sort_s\": %.6f, \"save_s\": %.6f}\n",
               (unsigned long long)db.getTotalFrags(), members, groups->size(), t1 - t0,
               t2 - t1, t3 - t2, t4 - t3);
  return 0;
}
