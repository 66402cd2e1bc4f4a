// rk_internal.h -- shared declarations of the device pipeline (not part of
// the public C ABI).  Kernels live in rk_sort.hip / rk_occupancy.hip /
// rk_groups.hip; each TU exports host-side launchers only, so no relocatable
// device code is needed.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rk {

// per-fragment resolution state on one axis (X or Y occupancy lists)
enum : uint8_t {
  ST_UNKNOWN = 0,      // not decided yet
  ST_ACTIVE = 1,       // in the axis' occupancy list (did not hit on this axis)
  ST_HIT_PENDING = 2,  // hit on this axis; winner not final yet
  ST_HIT = 3,          // hit on this axis; winner final
};

// device error bits (ctx->err word)
enum : uint32_t {
  ERRB_UB_BUCKET = 1u,
  ERRB_UB_CENTER = 2u,
  ERRB_INTERNAL = 4u,
};

constexpr uint32_t SKIP = 0xFFFFFFFFu;
constexpr uint32_t NONE = 0xFFFFFFFFu;

// ------------------------------------------------------------ rk_sort.hip --
// Stable counting sort of indices [0, m) by key[i] in [0, nbins) (key SKIP =
// leave out).  Histogram (LDS-privatised when a block's keys span a narrow
// window), DPP wave scan -> block -> device exclusive scan, atomic scatter and
// an in-bin rank fix that restores ascending index order inside every bin.
//   off  : nbins + 1 entries (off[nbins] = number kept)
//   perm : kept indices, bin-major, ascending inside a bin
//   scratch_cnt : nbins + 1 u32;  scratch_tmp : m u32
struct ScanScratch {
  uint32_t *block_sums;  // >= scan_blocks(n) + 1
  size_t cap;
};
size_t scan_blocks(size_t n);
void exclusive_scan_u32(const uint32_t *in, uint32_t *out, size_t n, ScanScratch ss,
                        hipStream_t st);
void counting_sort(const uint32_t *key, uint32_t m, uint32_t nbins, uint32_t *off, uint32_t *perm,
                   uint32_t *scratch_cnt, uint32_t *scratch_tmp, ScanScratch ss, hipStream_t st);
// list of non-empty bins, in no particular order; count -> *d_count
void nonempty_bins(const uint32_t *key, const uint32_t *perm, const uint32_t *off, uint32_t nbins,
                   uint32_t m, uint32_t *list, uint32_t *d_count, hipStream_t st);

// ------------------------------------------------------- rk_occupancy.hip --
struct Axis {
  const uint32_t *off;   // bucket CSR offsets, 2 * nbs + 1
  const uint32_t *ent;   // bucket entries (processing indices, ascending per bucket)
  const uint64_t *cen;   // centre per processing index
  const uint64_t *len;   // length per processing index
  uint8_t *state;        // ST_* per processing index
  uint32_t *win;         // winner per processing index (valid when ST_HIT)
  uint64_t max_index;    // seq_size / 100 (SequenceOcupationList.cpp:4)
  uint32_t nbs;          // buckets per strand = max_index + 1
  double len_ratio, pos_ratio;
};
// one Gauss-Seidel sweep over the buckets in `work`; buckets that still hold
// undecided entries are appended to next_work (count in *next_count, which the
// caller zeroes).  big_work/big_count: scratch for the wavefront-per-bucket path.
void occupancy_sweep(const Axis &ax, const uint32_t *work, uint32_t nwork, uint32_t *next_work,
                     uint32_t *next_count, uint32_t *big_work, uint32_t *big_count,
                     hipStream_t st);

// ---------------------------------------------------------- rk_groups.hip --
struct Frags {  // file-order inputs
  const uint64_t *x, *y, *len;
  const uint8_t *strand;
  uint32_t n;
};
struct Proc {  // processing-order working set
  uint32_t *row;          // proc -> file row
  uint64_t *xc, *yc, *len, *ha;
  uint32_t *keyx, *keyy;
  uint8_t *xstate, *ystate;
  uint32_t *xwin, *ywin;
  uint32_t *par, *gid;
};
void prep_keys(const Frags &f, uint64_t vsize, uint64_t max_x, uint64_t max_y, uint32_t *pkey,
               uint32_t *err, hipStream_t st);
void gather_proc(const Frags &f, const uint32_t *pkey, const uint32_t *poff, Proc p, uint32_t m,
                 uint32_t nbx, uint32_t nby, hipStream_t st);
void init_ystate(Proc p, uint32_t m, hipStream_t st);
void make_parents(Proc p, uint32_t m, uint32_t *isnew, uint32_t *err, hipStream_t st);
void jump_round(Proc p, uint32_t m, uint32_t *changed, hipStream_t st);
void assign_gid(Proc p, uint32_t m, const uint32_t *newrank, hipStream_t st);
void build_records(const uint32_t *gmem, const uint64_t *ha, uint32_t m, uint64_t *key,
                   uint32_t *tag, hipStream_t st);
void sort_groups(const uint32_t *goff, uint32_t ngroups, uint64_t *key, uint32_t *tag,
                 hipStream_t st);
void emit_result(const uint32_t *tag, const uint32_t *gid_proc, const uint32_t *goff,
                 const uint32_t *row, uint32_t m, uint32_t *out_gid, uint8_t *out_rep,
                 uint32_t *out_order, hipStream_t st);
void fill_dropped(uint32_t n, uint32_t *out_gid, uint8_t *out_rep, hipStream_t st);

}  // namespace rk
