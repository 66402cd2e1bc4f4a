// shim_driver.cpp -- the reference's execWithParams with classify_on_gpu in
// place of its hot path, for ONE (len_ratio, pos_ratio) pair:
//   init_args -> FragmentsDatabase -> classify_on_gpu -> save_all_frag_pairs
// (repkiller.cpp:31-96 with the SaverQueue write done synchronously, as
// oracle/ref_driver.cpp does).  Linked against the reference's ingress/egress
// translation units and librepkiller_amd.so by oracle/shim.mk; the GPU suite
// checks its output against the reference's golden files byte for byte.
//
//   usage: shim_driver <in.csv> <out.csv> <len_ratio> <pos_ratio>
#include <cstdio>
#include <queue>
#include <string>
#include <vector>

#include "FragmentsDatabase.h"
#include "commonFunctions.h"
#include "rk_reference_shim.h"

int main(int argc, char **argv) {
  if (argc != 5) {
    std::fprintf(stderr, "usage: %s in.csv out.csv len_ratio pos_ratio\n", argv[0]);
    return 2;
  }
  std::string out_path, in_path;
  std::queue<std::pair<double, double>> params;
  std::ifstream frags_file;
  std::vector<std::string> args(argv, argv + argc);
  try {
    init_args(args, frags_file, out_path, in_path, params);  // commonFunctions.cpp:9
    sequence_manager sm;
    FragmentsDatabase db(frags_file, sm);  // FragmentsDatabase.cpp:54
    frags_file.close();
    const auto param = params.front();
    FGList *groups = classify_on_gpu(db, sm, param.first, param.second);
    save_all_frag_pairs(out_path, sm, *groups);  // commonFunctions.cpp:131
    for (auto *g : *groups) delete g;
    delete groups;
  } catch (const std::exception &e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 1;
  }
  return 0;
}
