// rk_internal.h -- shared declarations of the device pipeline (not part of
// the public C ABI).  Kernels live in rk_sort.hip (scan), rk_radix.hip (stable
// radix sort), rk_occupancy.hip (bucket sweeps) and rk_groups.hip (processing
// order, groups, in-group order); each TU exports host-side launchers only, so
// no relocatable device code is needed.
#pragma once

#include <initializer_list>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/repkiller_amd.h"

namespace rk {

// per-fragment resolution state on one axis (X or Y occupancy lists)
enum : uint8_t {
  ST_UNKNOWN = 0,      // not decided yet
  ST_ACTIVE = 1,       // in the axis' occupancy list (did not hit on this axis)
  ST_HIT_PENDING = 2,  // hit on this axis; winner not final yet
  ST_HIT = 3,          // hit on this axis; winner final
};

// device error bits (ctrl[0])
enum : uint32_t {
  ERRB_UB_BUCKET = 1u,
  ERRB_UB_CENTER = 2u,
  ERRB_INTERNAL = 4u,
  ERRB_WIDE_LENGTH = 8u,  // not an error: some length >= 2^31 (generic sweep kernel)
};

constexpr uint32_t NONE = 0xFFFFFFFFu;

inline unsigned grid_for(size_t n, int threads, size_t cap = 65536) {
  size_t g = (n + threads - 1) / threads;
  if (g > cap) g = cap;
  return (unsigned)(g ? g : 1);
}

inline int bit_length(uint64_t v) { return v ? 64 - __builtin_clzll(v) : 0; }

// ------------------------------------------------------------ rk_sort.hip --
// Device-wide exclusive scan of u32 (DPP wave scan -> block -> tiles).
struct ScanScratch {
  uint32_t *block_sums;
  size_t cap;
};
size_t scan_blocks(size_t n);
void exclusive_scan_u32(const uint32_t *in, uint32_t *out, size_t n, ScanScratch ss,
                        hipStream_t st);
// the same, in[0] cleared once read (out != in)
void exclusive_scan_u32_clear0(uint32_t *in, uint32_t *out, size_t n, ScanScratch ss,
                               hipStream_t st);
// out[k] = number of roots (par[j] == j) among j < k, for k <= m: the
// new-group ranks straight from the parents (out[m] = the group count)
void exclusive_scan_roots(const uint32_t *par, uint32_t m, uint32_t *out, ScanScratch ss,
                          hipStream_t st, uint32_t *total = nullptr);

// Launch-level HIP-event timing of the pipeline's kernels, active only while a
// context profiles (rk_set_profiling): rk_classify_device points g_ktimer at
// its context's timer for the duration of the call.  Every timed launch is
// bracketed by kt_begin / kt_end on the launch stream and carries the
// ALGORITHMIC bytes of that launch (the minimum HBM traffic its job needs,
// DESIGN.md "Kernels and their rooflines").
enum KernelId : int {
  KID_PREP, KID_HIST, KID_SCATTER, KID_GATHER, KID_SORT_KEYS, KID_CSR_FILL_X, KID_RUN_BOUNDS,
  KID_SWEEP_TILE, KID_SWEEP_FAST, KID_SWEEP_MORE, KID_SWEEP_WAVE, KID_CSR_FILL_Y, KID_JUMP,
  KID_ASSIGN_GID, KID_GROUP_OFFSETS, KID_BUILD_RECORDS, KID_SORT_SMALL, KID_SORT_REG, KID_SORT_LDS,
  KID_SORT_GLOBAL, KID_EMIT, KID_PART, KID_EXCHANGE, KID_SHARD_AUX, KID_SH_ROWKEYS, KID_SH_FILLY,
  KID_SH_YRES, KID_SH_XOWN, KID_SH_MERGE, KID_SORT_SEGS, KID_SWEEP_LONG, KID_NW_HIST,
  KID_ONESWEEP, KID_NW_XCHUNK, KID_NW_FILLY, KID_NW_ASSIGN, KID_NW_XCOUNT, KID_NW_XBITS,
  KID_SORT_HEAP, KID_NW_FINE, KID_NW_MFINE, KID_NW_YFINE, KID_COUNT
};
extern const char *const kKernelNames[KID_COUNT];
// group-sort tiers (rk_groupsort.hip tier_of): <=16, <=32, <=64, four LDS caps, larger
constexpr int GS_NTIER = 8;

struct KernelTimer {
  static constexpr int MAX = 256;
  hipEvent_t ev[2 * MAX];
  int kid[MAX];
  double bytes[MAX];
  int n;
  // group-sort tiers: their member counts exist on the device only; they are
  // read back when the call's timings are collected (no sync inside the call)
  static constexpr int TIERS = GS_NTIER + 1;  // + the large tier's phase B
  const uint32_t *tier_counts;  // [tier][nblk] members per block, or null
  uint32_t tier_nblk;
  int tier_slot[TIERS];         // timer slot of each tier's launch (-1: none)
  int only = -1;                // >= 0: time only this kernel's launches (rk_set_profiling)
  // launches whose work is known on the device only (k_sweep_long32: the
  // entries of the long runs it walks): the kernel adds its units into
  // units[slot], and the slot's algorithmic bytes are unit_bytes[slot] x that
  // count, read back when the call's timings are collected
  uint32_t *units = nullptr;    // device, MAX words (rk_create)
  double unit_bytes[MAX];
};
extern thread_local KernelTimer *g_ktimer;
// Every launch site names its kernel in kt_begin and kt_end alike, so a timer
// restricted to one kernel (rk_set_profiling(ctx, 2 + k)) records both events
// of that kernel's launches and none of the others'
inline void kt_begin(hipStream_t st, int kid) {
  KernelTimer *t = g_ktimer;
  if (t && t->n < KernelTimer::MAX && (t->only < 0 || t->only == kid))
    (void)hipEventRecord(t->ev[2 * t->n], st);
}
inline void kt_end(hipStream_t st, int kid, double bytes) {
  KernelTimer *t = g_ktimer;
  if (t && t->n < KernelTimer::MAX && (t->only < 0 || t->only == kid)) {
    (void)hipEventRecord(t->ev[2 * t->n + 1], st);
    t->kid[t->n] = kid;
    t->bytes[t->n] = bytes;
    t->unit_bytes[t->n] = 0.0;
    t->n++;
  }
}
// the device word a launch adds its work units to (null when this launch is
// not timed); call before kt_begin (the word is cleared on the stream), then
// launch and kt_end_units
inline uint32_t *kt_units(hipStream_t st, int kid) {
  KernelTimer *t = g_ktimer;
  if (!t || !t->units || t->n >= KernelTimer::MAX || !(t->only < 0 || t->only == kid)) return nullptr;
  (void)hipMemsetAsync(t->units + t->n, 0, 4, st);
  return t->units + t->n;
}
inline void kt_end_units(hipStream_t st, int kid, double bytes_per_unit) {
  KernelTimer *t = g_ktimer;
  const int slot = t ? t->n : -1;
  kt_end(st, kid, 0.0);
  if (t && t->n == slot + 1 && t->units) t->unit_bytes[slot] = bytes_per_unit;
}

// ----------------------------------------------------------- rk_radix.hip --
size_t radix_scratch_words(uint32_t n);
// stable sort of (key, value) by the low `bits` bits of key; val_in null =>
// values are input positions.  Inputs must not alias outputs or tmp buffers.
void radix_sort_pairs(const uint32_t *key_in, const uint32_t *val_in, uint32_t *key_out,
                      uint32_t *val_out, uint32_t *key_tmp, uint32_t *val_tmp, uint32_t n,
                      int bits, uint32_t *scratch, size_t scratch_words, hipStream_t st,
                      int max_digit = 0);  // widest digit in bits (0: the default)

// ------------------------------------------------------- rk_occupancy.hip --
struct Axis {          // one axis' occupancy entries in CSR (bucket-run) order
  const uint32_t *key; // bucket key strand * nbs + centre/100, sorted
  const uint32_t *ent; // processing index of the entry (ascending inside a run)
  const uint64_t *cen; // centre
  const uint64_t *len; // length
  uint8_t *state;      // ST_*
  uint32_t *xres;      // X axis only: the Y records as 32-bit words; word 4k+3 of
                       // entry k receives its X result (winner id, or NONE)
  uint32_t *par;       // parent by processing index: X hits -> X winner; Y axis
                       // (X misses) -> Y winner, or itself for a new group
  const uint2 *pk;     // {centre low 32, length low 32}: the 32-bit sweep's record
  const uint8_t *nbd;  // neighbour_dir code per entry (0, 1 = -1, 2 = +1)
  uint32_t *rlen_at;   // run length, stored at each run's first position
  uint32_t *rbeg_at;   // run start, stored at each run's last position
  uint32_t m;          // entries
  uint64_t max_index;  // seq_size / 100 (SequenceOcupationList.cpp:4)
  double len_ratio, pos_ratio;
  // the first window sweep evaluates the winners' deviations lane-parallel
  // (the Y axis: ~24 deviations per window against ~2 on the X axis)
  bool par_dev = false;
};
// The axis' bucket runs: the 64-position windows (wpend[w] = window w still
// owns undecided entries) and the runs longer than 64 entries, which take a
// wavefront each.  32-bit path: `big` holds one byte per window, set by the
// first sweep when a long run starts there.  64-bit path: `big` lists the
// long runs' starts (nbig of them) and build_runs fills Axis::rlen_at/rbeg_at.
struct RunList {
  uint32_t *big;
  uint8_t *wpend;
  uint32_t nbig, nwin;
  bool fast32;          // every length < 2^31: the 32-bit window kernel applies
};
size_t runs_scratch_words(uint32_t m);
void build_runs(const Axis &ax, RunList &rl, uint32_t *dev_count, uint32_t *host_words,
                hipStream_t st);
// One sweep.  rpend[p] (start p of a long run) = run still has undecided
// entries; set to 1 before the first sweep.  counters: PEND_WORDS words, their
// sum is the number of waves/runs still pending after the sweep.
constexpr uint32_t PEND_WORDS = 64;
void occupancy_sweep(const Axis &ax, const RunList &rl, uint8_t *rpend, uint32_t *counters,
                     bool first, hipStream_t st, bool clear = true);

// ---------------------------------------------------------- rk_groups.hip --
struct Frags {  // file-order inputs
  const uint64_t *x, *y, *len;
  const uint8_t *strand;
  uint32_t n;
};
struct Proc {  // processing-order working set
  ulonglong2 *rec; // FILE order: {xStart, yStart}, {length, strand} (one 32-B gather per row)
  uint64_t *ys;    // yStart in processing order
  uint32_t *pkey;  // sorted xStart/10 key
  uint32_t *row;   // proc -> file row
  ulonglong2 *xrec;  // {x centre, length}
  ulonglong2 *yrec;  // {y centre, length low 32 | X result << 32} (X result: X winner or
                     // NONE, written by the X sweeps)
  uint32_t *ylenhi;  // length high 32 bits, only when some length >= 2^31 (else null)
  ulonglong2 *hrec;  // {in-group sort key, file row}: one gather per member
  uint32_t *keyx, *keyy;
  uint32_t *par, *gid;
  uint32_t *grow;  // optional (sharded driver): global file row, from rec's high word
};
struct Csr {  // one axis in CSR order (see Axis)
  uint32_t *key, *ent;
  uint64_t *cen, *len;
  uint8_t *state;
  uint2 *pk;     // {centre low 32 bits, length low 32 bits} (the 32-bit sweep)
  uint8_t *nbd;  // neighbour bucket probed: 0 none, 1 = B-1, 2 = B+1
};

// inclusive prefix sum over the 64 lanes of a wavefront by DPP row shifts and
// row broadcasts (no LDS round trip; lanes outside the shifted row read 0)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}

// The neighbour bucket get_associated_group effectively probes
// (SequenceOcupationList.cpp:47-89): rescanning a bucket under the strict `>`
// is a no-op, so only B-1 (c % 100 in {0, 1}, c >= 100) or B+1 (c % 100 == 99
// and c < max_index, or c % 100 == 98 and c < max_index - 1) can add
// candidates.  -1 / +1 / 0.
__device__ __forceinline__ int neighbour_dir(uint64_t c, uint64_t max_index) {
  const uint64_t r = c % 100;
  if (r <= 1 && c >= 100) return -1;
  if ((r == 99 && c < max_index) || (r == 98 && c < max_index - 1)) return 1;
  return 0;
}
// processing key per file row (dropped last bucket -> vsize-1, sorts last);
// counts kept rows into *kept; flags UB into *err
void prep_keys(const Frags &f, uint64_t vsize, uint64_t max_x, uint64_t max_y, uint32_t *pkey,
               ulonglong2 *rec, uint32_t *kept, uint32_t *err, hipStream_t st);
void gather_proc(const Frags &f, Proc p, uint32_t m, uint32_t nbx, uint32_t nby, hipStream_t st);
// in-group sort key |yStart - diag_func[xStart/10]| per fragment, with its
// file row (p.hrec); *wide |= 1 when a key needs more than 32 bits
void sort_keys(Proc p, uint32_t m, uint32_t *wide, hipStream_t st);
// X axis in CSR order: centre/length (+ packed record, neighbour code), state UNKNOWN
void csr_fill_x(Csr c, const ulonglong2 *xrec, uint32_t m, uint64_t max_index, hipStream_t st);
// Y axis in CSR order: centre/length, state ACTIVE for X hits (they sit in the
// Y list) else UNKNOWN
void csr_fill_y(Csr c, const ulonglong2 *yrec, const uint32_t *ylenhi, uint32_t m,
                uint64_t max_index, hipStream_t st);
// one pointer-jumping round; the first also writes isnew[k] = (par[k] == k).
// open (optional, device): when open[0] | open[1] is set the parents are not
// final (an axis was left open) and the round does nothing
void jump_round(Proc p, uint32_t m, uint32_t *changed, uint32_t *isnew, uint32_t *err,
                hipStream_t st, const uint32_t *open = nullptr);
// the compression in one pass plus a pass over the chains it left open
// (list: m words, count: one word; *changed = 1 only for a chain still open
// after 4096 more links), no host round trip
void jump_listed(Proc p, uint32_t m, uint32_t *isnew, uint32_t *err, uint32_t *list,
                 uint32_t *count, uint32_t *changed, hipStream_t st);
void assign_gid(Proc p, uint32_t m, const uint32_t *newrank, hipStream_t st);
void group_offsets(const uint32_t *sgid, uint32_t m, uint32_t ngroups, uint32_t *goff,
                   hipStream_t st);
// members (gmem, processing ids, group-major) -> sort keys, tags = member
// slots, and the members' file rows IN PLACE of gmem
void build_records(uint32_t *gmem, const ulonglong2 *hrec, uint32_t m, uint64_t *key,
                   uint32_t *tag, hipStream_t st);
// ------------------------------------------------------- rk_groupsort.hip --
size_t groupsort_scratch_bytes(uint32_t n);
// libstdc++ std::sort of every group's (key, tag) records; sorted tags -> otag
// (groups of one member are left unwritten: their slot holds its own tag).
// Every record's tag is its position (tag[x] == x): the tiers compute it, and
// `tag` is only the scratch array in which the groups above 2048 members move
// their tags (written there first), so callers need not fill it.
// gid_sorted: group id of every record; host_words: >= 16 pinned words;
// narrow_keys: every key fits 32 bits (LDS tiers stage 4-byte keys).
// side (optional): a second stream for the tiers of <= 64 members, forked
// and joined through ev_fork / ev_join.
// Returns RK_OK, or the status of the depth-limit heap segments' own buffers
// (RK_E_NOMEM / RK_E_HIP; only when they are sorted here, heap_count null).
int sort_groups_exact(const uint32_t *gid_sorted, const uint32_t *goff, uint32_t ngroups,
                      uint32_t m, uint64_t *key, uint32_t *tag, uint32_t *otag, void *scratch,
                      ScanScratch ss, uint32_t *host_words, bool narrow_keys, hipStream_t st,
                      hipStream_t side = nullptr, hipEvent_t ev_fork = nullptr,
                      hipEvent_t ev_join = nullptr, uint32_t *heap_count = nullptr);
// heap_count != nullptr: the depth-limit heap segments are not sorted, their
// number goes to heap_count (device), and the caller, having read it back,
// sorts them by this before using otag (RK_OK / RK_E_NOMEM / RK_E_HIP)
int sort_groups_heap_deferred(uint32_t ngroups, uint32_t m, uint64_t *key, uint32_t *tag,
                              uint32_t *otag, void *scratch, uint32_t nheap,
                              uint32_t *host_words, hipStream_t st);
// sorted member slots (otag), group of every slot (sgid), group bounds, the
// members' file rows -> the output columns
void emit_result(const uint32_t *otag, const uint32_t *sgid, const uint32_t *goff,
                 const uint32_t *mrow, uint32_t m, uint32_t *out_gid, uint8_t *out_rep,
                 uint32_t *out_order, hipStream_t st);

// -------------------------------------------------------- rk_narrow.hip --
// The record-carrying pipeline (16-B records, one-sweep radix sorts, X axis by
// chunks of the processing order).  ctrl words: [0] error bits, [1] kept rows,
// [3] not representable, [4] longest length, [6] wide sort keys, [8]
// forward-strand kept rows.
struct NwDigits {
  int passes;
  int shift[4], db[4];
};
NwDigits nw_plan(int bits, int max_bits = 0);  // max_bits 0: nw_max_bits()
void nw_trace_dump(hipStream_t st);  // RK_NW_TRACE (measurement only)
size_t nw_status_words(uint32_t n);
uint32_t nw_chunk_width(uint32_t m, uint32_t nbx);
uint32_t nw_chunks(uint32_t nbx, uint32_t W);
// the X-chunk counts (3 nch + 1 words: entries per strand and chunk, owned rows per chunk)
struct NwChunkCounts {
  uint32_t W, lgW, nch;
  uint32_t *cnts;
};
// wire: the rows as rk_classify's 12-B wire records (rk_io.hip) instead of
// the SoA columns of `in` (only in.n is read then)
void nw_order_hist(const rk_frags_soa &in, uint64_t vsize, uint64_t max_x, uint64_t max_y,
                   uint32_t nby, const NwDigits &a, const NwDigits &y, uint32_t *ghist,
                   uint32_t *yhist, uint32_t *ctrl, hipStream_t st, const uint3 *wire = nullptr);
void nw_order_sort(const rk_frags_soa &in, uint64_t vsize, uint32_t nby, const NwDigits &a,
                   const uint32_t *ghist, uint32_t *status, uint4 *Ra, uint4 *Rb, uint4 *yrec,
                   hipStream_t st, const uint3 *wire = nullptr);
// Sorts in two stages (rk_narrow.hip, k_seg_fine): C coarse bits by
// one-sweep passes (coarse: their digits, shifted past the F fine bits), then
// one block per coarse-key segment (nseg = 2^C) sorts its F fine bits in LDS.
// The processing order's segment kernel writes the final records, the Y
// records and -- given cc -- the X-chunk counts; the member sort's writes the
// in-group sort arrays and the group starts.  passes == 0 in `coarse`: not
// applicable (too few rows, or RK_NW_SPLIT=0).
struct NwOrderPlan {
  int C = 0, F = 0;
  uint32_t nseg = 0;
  NwDigits coarse{};
  uint32_t kbase = 0;  // subtracted from every key (a multiple of 2^F; 0 on one device)
};
// several regions cleared by one kernel launch (a memset launch each costs a
// dispatch gap of ~4-9 us); null or empty regions are skipped
struct ZeroRegion {
  void *ptr;
  size_t bytes;
};
void zero_regions(hipStream_t st, std::initializer_list<ZeroRegion> regs);
// what nw_order_sort_split_coarse clears first (four regions)
void nw_order_coarse_regions(uint32_t n, const NwOrderPlan &op, uint32_t *status, uint32_t *chist,
                             ZeroRegion extra, ZeroRegion out[4]);
NwOrderPlan nw_order_split(uint32_t n, uint64_t nkeys, int bits);  // nkeys: key values in use
NwOrderPlan nw_order_split_range(uint32_t n, uint64_t klo, uint64_t khi);  // keys in [klo, khi)
// the same in two halves: the clears (+ `extra`) and the coarse passes, then
// the scan and the segment kernel (cc->cnts cleared by the first half's
// `extra`) -- the host can read the order histogram's control words back in
// between, while the coarse passes run
// (zeroed: the caller already cleared nw_order_coarse_regions)
void nw_order_sort_split_coarse(const rk_frags_soa &in, const NwOrderPlan &op,
                                const uint32_t *ghist, uint32_t *status, uint4 *Ra, uint4 *Rb,
                                uint32_t *chist, ZeroRegion extra, uint64_t vsize,
                                hipStream_t st, const uint3 *wire = nullptr,
                                bool zeroed = false);
void nw_order_sort_split_fine(uint32_t n, uint32_t m, uint32_t nby, const NwOrderPlan &op,
                              uint4 *Ra, uint4 *Rb, uint4 *yrec, uint4 *tmp, uint32_t *chist,
                              uint32_t *coff, ScanScratch ss, const NwChunkCounts *cc,
                              hipStream_t st);
// words of each segment array (counts, starts) a split sort of n rows may use
inline size_t nw_seg_words(uint32_t n) { return (size_t)n / 512 + 64; }
// the same over records received by the sharded driver (processing index base
// + position; no X-chunk counts); tmp: m records of scratch
void nw_order_sort_recs_split(const uint4 *in, uint32_t m, uint32_t nby, uint32_t base,
                              const NwOrderPlan &op, const uint32_t *ghist, uint32_t *status,
                              uint4 *Ra, uint4 *Rb, uint4 *yrec, uint4 *tmp, uint32_t *chist,
                              uint32_t *coff, ScanScratch ss, const NwChunkCounts *cc,
                              hipStream_t st);
void nw_order_sort_split(const rk_frags_soa &in, uint32_t m, uint32_t nby, const NwOrderPlan &op,
                         const uint32_t *ghist, uint32_t *status, uint4 *Ra, uint4 *Rb,
                         uint4 *yrec, uint4 *tmp, uint32_t *chist, uint32_t *coff,
                         ScanScratch ss, const NwChunkCounts *cc, uint64_t vsize, hipStream_t st,
                         const uint3 *wire = nullptr);
// the member sort in two stages (12-B member records: every sort key fits 32
// bits): the in-group sort arrays as nw_member_sort writes them, and goff (G +
// 1 group starts, group_offsets' job); t0 / t1 / t2: three scratch arrays of
// m 12-B records
void nw_member_sort_split(const uint4 *erec, const uint32_t *gidp, uint4 *t0, uint4 *t1,
                          uint4 *t2, uint32_t m, uint32_t G, const NwOrderPlan &mp,
                          const uint32_t *ehist, uint32_t *status, uint32_t *sgid, uint64_t *key,
                          uint32_t *tag, uint32_t *mrow, uint32_t *goff, uint32_t *chist,
                          uint32_t *coff, ScanScratch ss, hipStream_t st);
// (halo, G): the sharded driver's G lead-in records ahead of R (R holds m - G)
// the halo's G records added to counts already in cc.cnts (no clearing)
void nw_x_count_add(const uint4 *halo, uint32_t G, const NwChunkCounts &cc, hipStream_t st);
void nw_x_count(const uint4 *R, uint32_t m, const NwChunkCounts &cc, hipStream_t st,
                const uint4 *halo = nullptr, uint32_t G = 0);
// arrival_ids: the first pass numbers the entries by position (the sharded
// driver's received Y records), instead of keeping their processing index;
// src0: the first pass reads these records instead of yrec (which then only
// takes the intermediates, with tmp)
void nw_y_sort_head(const uint4 *yrec, uint4 *tmp, uint32_t m, const NwDigits &y,
                    const uint32_t *yhist, uint32_t *status, hipStream_t st,
                    bool arrival_ids = false, const uint4 *src0 = nullptr);
void nw_y_sort_tail(const uint4 *yrec, const uint4 *tmp, uint32_t m, const NwDigits &y,
                    const uint32_t *yhist, uint32_t *status, Csr cy, uint32_t nby,
                    uint64_t max_y, const uint32_t *xbits, hipStream_t st,
                    bool arrival_ids = false, const uint4 *src0 = nullptr);
// the whole Y sort once the X axis is resolved: the X-hit bits (by processing
// index; with src0, by position in src0) ride in the records from the first
// pass; the last writes CSR + states.  src0: the sharded driver's received Y
// records, numbered by arrival in the first pass (yrec and tmp then only take
// the intermediates)
// the same in two stages (coarse passes + one block per coarse-key segment
// writing the CSR arrays); yp = nw_order_split over the Y key; tmp2: m
// records of scratch; chist / coff: 2^C + 1 words
void nw_y_sort_split_after_x(uint4 *yrec, uint4 *tmp, uint4 *tmp2, uint32_t m,
                             const NwOrderPlan &yp, const uint32_t *yhist, uint32_t *status,
                             Csr cy, uint32_t nby, uint64_t max_y, const uint32_t *xbits,
                             uint32_t *chist, uint32_t *coff, ScanScratch ss, hipStream_t st);
void nw_y_sort_after_x(const uint4 *yrec, uint4 *tmp, uint32_t m, const NwDigits &y,
                       const uint32_t *yhist, uint32_t *status, Csr cy, uint32_t nby,
                       uint64_t max_y, const uint32_t *xbits, hipStream_t st,
                       const uint4 *src0 = nullptr);
void nw_x_chunks(const uint4 *R, uint32_t m, uint32_t nbx, uint64_t max_x, uint32_t maxlen,
                 const uint32_t *xoff, Csr cx, uint32_t *xpos, uint4 *erec, uint32_t *ctrl,
                 uint32_t W, hipStream_t st, const uint4 *halo = nullptr, uint32_t G = 0);
// the sharded driver (rk_shard_nw.h): the processing order of received 16-B
// records (Y records numbered from `base`), digit histograms of records whose
// key is their first word (minus sub), the member sort of received records
void nw_order_sort_recs(const uint4 *in, uint32_t m, uint32_t nby, uint32_t base,
                        const NwDigits &a, const uint32_t *ghist, uint32_t *status, uint4 *Ra,
                        uint4 *Rb, uint4 *yrec, hipStream_t st);
void nw_rec_hist(const void *recs, int rec_bytes, uint32_t n, uint32_t sub, const NwDigits &d,
                 uint32_t *ghist, hipStream_t st);
void nw_member_sort_recv(const void *recs, bool narrow_keys, uint32_t m, uint32_t g0,
                         const NwDigits &e, const uint32_t *ehist, uint32_t *status, uint4 *t0,
                         uint4 *t1, uint32_t *sgid, uint64_t *key, uint32_t *tag, uint32_t *mrow,
                         hipStream_t st);
// X hits as a bitmask by processing index, from the resolved X axis (xpos[k] =
// X position of fragment k); then the Y states: X hits sit in the Y lists
void nw_x_bits(const uint32_t *xpos, const uint8_t *xstate, uint32_t m, uint32_t *bits,
               hipStream_t st);
void nw_fill_y(const uint32_t *ent, const uint32_t *bits, uint8_t *state, uint32_t m,
               hipStream_t st);
void nw_assign(const uint32_t *par, const uint32_t *newrank, uint32_t *gidp, uint32_t m,
               const NwDigits &e, uint32_t *ehist, hipStream_t st);
// the roots and gids in one pass after exclusive_scan_roots (list: m words of
// scratch; ctrl[12] its count (zero on entry), ctrl[13] = 1 when a chain stayed open after
// 4128 steps, ctrl[0] |= ERRB_INTERNAL on a parent after its child)
void nw_assign_jump(uint32_t *par, const uint32_t *newrank, uint32_t *gidp, uint32_t m,
                    const NwDigits &e, uint32_t *ehist, uint32_t *list, uint32_t *ctrl,
                    hipStream_t st);
void nw_member_sort(const uint4 *erec, const uint32_t *gidp, uint4 *t0, uint4 *t1, uint32_t m,
                    const NwDigits &e, const uint32_t *ehist, uint32_t *status, uint32_t *sgid,
                    uint64_t *key, uint32_t *tag, uint32_t *mrow, bool narrow_keys,
                    hipStream_t st);

}  // namespace rk
