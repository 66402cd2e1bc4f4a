// rk_reference_shim.cpp -- see rk_reference_shim.h.
#include "rk_reference_shim.h"

#include <stdexcept>
#include <string>
#include <vector>

#include "repkiller_amd.h"

namespace {

// One context per worker thread: the reference runs up to MAX_THREADS pairs
// concurrently (repkiller.cpp:60-72), each with private state.
rk_ctx *thread_ctx() {
  thread_local struct Holder {
    rk_ctx *c = nullptr;
    Holder() {
      if (rk_create(&c, 0) != RK_OK) throw std::runtime_error("no usable gfx950 device");
    }
    ~Holder() { rk_destroy(c); }
  } h;
  return h.c;
}

}  // namespace

FGList *classify_on_gpu(const FragmentsDatabase &frag_db, const sequence_manager &sm,
                        double len_ratio, double pos_ratio) {
  // FragmentsDatabase iterates its xStart/10 buckets in order, file order
  // inside a bucket, and stops before the last bucket (FragmentsDatabase.h:26-31):
  // that is already the processing order, and rk_classify's stable
  // re-bucketing leaves it unchanged.  Rows of the skipped last bucket are
  // never written by the reference either.
  std::vector<const FragFile *> rows;
  std::vector<uint64_t> xs, ys, ls;
  std::vector<uint8_t> st;
  for (const auto *bucket = frag_db.begin(); bucket != frag_db.end(); ++bucket)
    for (const FragFile &f : *bucket) {
      rows.push_back(&f);
      xs.push_back(f.xStart);
      ys.push_back(f.yStart);
      ls.push_back(f.length);
      st.push_back((uint8_t)f.strand);
    }
  const uint64_t n = rows.size();
  std::vector<uint32_t> order(n), gid(n);
  std::vector<uint8_t> rep(n);
  rk_frags_soa in{xs.data(), ys.data(), ls.data(), st.data(), n};
  // the header values WITHOUT the +1 FragmentsDatabase applies (FragmentsDatabase.cpp:62,65)
  rk_params p{sm.get_sequence_by_label(0).len - 1, sm.get_sequence_by_label(1).len - 1,
              len_ratio, pos_ratio};
  rk_result out{order.data(), gid.data(), rep.data(), 0, 0};
  rk_ctx *ctx = thread_ctx();
  if (int rc = rk_classify(ctx, &in, &p, &out))
    throw std::runtime_error(std::string("rk_classify: ") + rk_last_error(ctx) + " (" +
                             std::to_string(rc) + ")");
  // the FGList the SaverQueue expects: groups in creation order (gid
  // ascending), members in sorted order; save_frags_from_group derives the
  // same 0/1/2 flags out.repval carries (commonFunctions.cpp:106-115)
  FGList *fgl = new FGList;
  fgl->reserve(out.n_groups);
  for (uint64_t k = 0; k < out.n_out; ++k) {
    if (k == 0 || gid[k] != gid[k - 1]) fgl->push_back(new FragsGroup());
    fgl->back()->push_back(rows[order[k]]);
  }
  return fgl;
}
