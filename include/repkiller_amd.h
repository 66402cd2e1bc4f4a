/* repkiller_amd.h -- C ABI of the MI355X-native repeat-fragment classifier.
 *
 * Drop-in boundary for the hot path of estebanpw/repkiller v0.9.b.  The
 * reference has no FFI; its hot path is three in-process C++ calls made by
 * execWithParams (/root/reference/src/repkiller.cpp:80-97):
 *
 *   generate_fragment_groups(db, FGList&, seq_mgr, len_ratio, pos_ratio)
 *                                            commonFunctions.h:35 / .cpp:41-80
 *   generate_diagonal_func(db, size_t *diag)  commonFunctions.h:59 / .cpp:161-177
 *   sort_groups(FGList&, const size_t *diag)  commonFunctions.h:57 / .cpp:148-159
 *
 * plus the repeat flag chosen when a group is saved
 * (save_frags_from_group, commonFunctions.cpp:106-115).  rk_classify() replaces
 * all four: it takes the fragments as plain SoA arrays and returns, per input
 * row, the group id (the `block` column the reference writes, creation order)
 * and the repeat flag, plus the exact row order of the reference's output.
 * Ingress (FragmentsDatabase, FragmentsDatabase.cpp:17-101) and egress
 * (save_all_frag_pairs / SaverQueue, commonFunctions.cpp:101-146,
 * SaverQueue.cpp:4-51) are provided host-side by rk_db_* / rk_saver_*.
 *
 * Conventions: every function returns 0 (RK_OK) or a negative rk_status; no
 * exception crosses the ABI; all buffers are caller-owned; one rk_ctx per
 * host thread (the reference runs up to 3 concurrent pairs, repkiller.cpp:60-72,
 * each with private state -- contexts mirror that).  There is NO CPU fallback:
 * rk_create fails with RK_E_NODEVICE when no gfx950 device is usable.
 */
#ifndef REPKILLER_AMD_H
#define REPKILLER_AMD_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  RK_OK = 0,
  RK_E_ARG = -1,
  RK_E_IO = -2,          /* cannot open/read/write a file (reference: runtime_error) */
  RK_E_COUNT = -3,       /* more Frag lines than the header total (FragmentsDatabase.cpp:99) */
  RK_E_UB_BUCKET = -4,   /* xStart/10 >= vsize: the reference writes out of bounds (:96-97) */
  RK_E_UB_CENTER = -5,   /* a probe would index past an occupancy array
                            (SequenceOcupationList.cpp:17, :80 size_t wrap) */
  RK_E_NOMEM = -6,
  RK_E_HIP = -7,         /* a HIP runtime call failed; see rk_last_error */
  RK_E_NODEVICE = -8,    /* no usable gfx950 device */
  RK_E_TOO_MANY = -9,    /* n >= 2^32 - 1 (32-bit row ids); rk_classify_sharded: one rank's
                            Y range or gid range holds >= 2^30 records (30-bit pass counts) */
  RK_E_INTERNAL = -10,   /* a device-side consistency check failed */
  RK_E_PEER = -11,       /* rk_classify_sharded*: another rank of the comm failed; every
                            rank returns an error together (rk_last_error names the rank) */
} rk_status;

/* ---- classification (the hot path) ----------------------------------- */

typedef struct rk_ctx rk_ctx;

/* Fragments in FILE order, exactly the fields the hot path reads
 * (FragFile xStart/yStart/length/strand, structs.h:18-48). */
typedef struct {
  const uint64_t *x_start;
  const uint64_t *y_start;
  const uint64_t *length;
  const uint8_t *strand; /* 'f' = forward lists, anything else = reverse lists */
  uint64_t n;
} rk_frags_soa;

typedef struct {
  uint64_t len_x_hdr; /* raw "SeqX length" header value; +1 applied inside (FragmentsDatabase.cpp:62) */
  uint64_t len_y_hdr; /* raw "SeqY length" header value (FragmentsDatabase.cpp:65) */
  double len_ratio;   /* > 0 (commonFunctions.cpp:26) */
  double pos_ratio;   /* > 0 (commonFunctions.cpp:27) */
} rk_params;

typedef struct {
  /* All three arrays are in OUTPUT order (the order of the reference's CSV
   * rows, commonFunctions.cpp:126-128): entry k describes the k-th row written.
   * Caller-allocated with n entries; the first n_out are filled.  Rows of the
   * never-iterated last xStart/10 bucket (FragmentsDatabase.h:29-31) are not
   * written. */
  uint32_t *out_order; /* input row written k-th */
  uint32_t *gid;       /* its group id: the `block` column, creation order */
  uint8_t *repval;     /* its repeat flag: 0 singleton / 1 representative / 2 repeated */
  uint64_t n_out;      /* set by rk_classify*: rows written (= rows grouped) */
  uint64_t n_groups;   /* set by rk_classify*: groups created */
} rk_result;

/* Per-call counters of the last rk_classify* on a context. */
typedef struct {
  uint64_t n_in, n_proc, n_groups;
  uint32_t x_sweeps, y_sweeps, jump_rounds;
  uint64_t x_hits, y_hits;
  double device_ms; /* HIP-event time of the whole device pipeline */
  uint32_t pipeline; /* the pipeline that produced the result: 1 record, 2 generic */
  uint32_t record_fallback; /* why the record pipeline handed over: 0 it did not, 1 a row
                               does not pack into a record */
  double h2d_ms, d2h_ms;    /* rk_classify*: host wall time of the input upload and of the
                               result download (0 for the device entry points) */
  uint32_t wire;            /* rk_classify*: 1 when the rows crossed PCIe as 12-B wire
                               records (order + flag back, gids rebuilt on the host), 0
                               when as the SoA */
  uint32_t sweep_repeats;   /* record pipeline: ratio pairs whose queued sweeps left an axis
                               open, repeated with a readback per sweep (0 on the BASELINE
                               configs) */
  /* rk_classify*: NUMA nodes of the host side of the last upload (-1: unknown /
     not bound): the caller's input pages, the node the packing threads were
     bound to (RK_IO_NUMA=0: never bound), the pinned staging slots, the GPU */
  int32_t numa_input, numa_threads, numa_staging, numa_gpu;
} rk_stats;

int rk_create(rk_ctx **ctx, int device);
void rk_destroy(rk_ctx *ctx);
const char *rk_last_error(const rk_ctx *ctx);

/* Host buffers in and out (H2D, device pipeline, D2H); blocking. */
int rk_classify(rk_ctx *ctx, const rk_frags_soa *in, const rk_params *p, rk_result *out);

/* Device buffers in and out (hipMalloc'd); runs on the context's stream and
 * returns when the result is complete (n_out / n_groups are host values). */
int rk_classify_device(rk_ctx *ctx, const rk_frags_soa *in_dev, const rk_params *p,
                       rk_result *out_dev);

/* Several (len_ratio, pos_ratio) pairs over ONE fragment set -- the loop of
 * repkiller.cpp:60-72, which runs execWithParams (repkiller.cpp:80-97) once
 * per pair on the same FragmentsDatabase.  The ratio-independent work
 * (processing order, both occupancy axes, in-group sort keys) is done once;
 * p[i] / out[i] belong to pair i.  Every p[i] must carry the same
 * len_x_hdr / len_y_hdr (RK_E_ARG otherwise).  rk_get_stats reports the last
 * pair; phase profiling covers the shared part and the first pair. */
int rk_classify_pairs(rk_ctx *ctx, const rk_frags_soa *in, const rk_params *p, uint32_t npairs,
                      rk_result *out);
int rk_classify_device_pairs(rk_ctx *ctx, const rk_frags_soa *in_dev, const rk_params *p,
                             uint32_t npairs, rk_result *out_dev);

int rk_get_stats(const rk_ctx *ctx, rk_stats *st);

/* Which device pipeline rk_classify* uses on this context.  AUTO (default):
 * the record pipeline whenever every row packs into its 16-B record (length
 * < 2^24, yStart < 2^35) and there are fewer than 2^30 rows, else the
 * generic one; GENERIC: always the generic pipeline.
 * Both produce the same output. */
enum { RK_PIPELINE_AUTO = 0, RK_PIPELINE_GENERIC = 1 };
int rk_set_pipeline(rk_ctx *ctx, int pipeline);

/* ---- ONE fragment set sharded over several GPUs ----------------------
 *
 * The reference runs the whole path on one host thread per ratio pair
 * (repkiller.cpp:60-72 -> execWithParams :80-97).  rk_classify_sharded runs
 * the same path for ONE fragment set spread over P ranks, one rk_ctx per GPU
 * (one process or thread each), and produces exactly the output of
 * rk_classify on the concatenated input: the processing order is partitioned
 * by xStart/10 ranges (balanced by an all-reduced histogram), the X and Y
 * occupancy lists by centre-bucket ranges with halo exchanges, group roots are
 * resolved across ranks, and the in-group order by gid ranges
 * (DESIGN.md "Multi-GPU").  Collectives go through an rk_comm: RCCL over xGMI
 * for production, or host callbacks (e.g. torch.distributed gloo) for tests.
 * Every rank of the comm must call it with the same params.
 */
typedef struct rk_comm rk_comm;

#define RK_COMM_ID_BYTES 128 /* sizeof(ncclUniqueId) */

/* Host-callback collectives (buffers are HOST memory; return 0 on success). */
typedef struct {
  void *user;
  /* recv = concatenation over ranks of every rank's `bytes` bytes */
  int (*allgather)(void *user, const void *send, void *recv, uint64_t bytes);
  /* rank r's send block for rank q is send_bytes[q] bytes (blocks packed in
   * rank order); recv receives rank q's block for r, recv_bytes[q] bytes, packed
   * in rank order */
  int (*alltoallv)(void *user, const void *send, const uint64_t *send_bytes, void *recv,
                   const uint64_t *recv_bytes);
} rk_comm_host_ops;

int rk_comm_create_host(int rank, int size, const rk_comm_host_ops *ops, rk_comm **comm);
/* An in-process group of `size` comms (comms[r] for rank r), for one thread per
 * rank: exchanges are direct device copies between the ranks' buffers (peer
 * copies over xGMI when the ranks use different GPUs).  Destroy each with
 * rk_comm_destroy. */
int rk_comm_create_local(int size, rk_comm **comms);
/* RCCL communicator (librccl.so.1 is loaded on first use): rank 0 makes the
 * id, the caller distributes it (e.g. a torch.distributed broadcast), every
 * rank then creates its comm on its device. */
int rk_comm_rccl_id(uint8_t id[RK_COMM_ID_BYTES]);
int rk_comm_create_rccl(int rank, int size, int device, const uint8_t id[RK_COMM_ID_BYTES],
                        rk_comm **comm);
void rk_comm_destroy(rk_comm *comm);
/* A rank that cannot make its rk_classify_sharded* call (e.g. rk_create
 * failed) calls this instead, once: it takes part in the peers' first
 * collective with `status`, and every peer's call returns RK_E_PEER instead of
 * waiting for it. */
int rk_comm_abandon(rk_comm *comm, int status);
const char *rk_comm_last_error(const rk_comm *comm);

typedef struct {
  /* DEVICE arrays owned by the context (valid until its next call), in output
   * order: this rank's share of the global output, rows
   * [out_offset, out_offset + n_out) of what rk_classify writes. */
  const uint32_t *out_order; /* global input row (rank q's rows follow rank q-1's) */
  const uint32_t *gid;
  const uint8_t *repval;
  uint64_t n_out;
  uint64_t out_offset;
  uint64_t n_out_total; /* rows of the whole output */
  uint64_t n_groups;    /* groups of the whole set */
} rk_shard_result;

typedef struct {
  uint64_t n_in, n_total;    /* this rank's input rows / all ranks' */
  uint64_t n_slice;          /* processing-order entries this rank owns */
  uint64_t x_ghosts;         /* X lead-in entries received from earlier slices */
  uint64_t y_entries;        /* Y-range entries held (own + halo) */
  uint32_t x_rounds, y_rounds;   /* halo verification rounds */
  uint32_t x_reruns, y_reruns;   /* local re-resolutions with owner-fixed halos */
  uint32_t root_rounds;      /* cross-rank root resolution rounds */
  uint64_t bytes_sent;       /* payload bytes this rank sent */
  double ms_total, ms_ingress, ms_x, ms_y, ms_roots, ms_members; /* host wall */
  uint32_t generic_driver;   /* 1: the generic driver ran (a row outside the 16-B record
                                or a slice of >= 2^30 rows, or RK_SHARD_GENERIC=1) */
  uint32_t order_split;      /* 1: this rank's slice took the two-stage order sort
                                (coarse passes + per-segment LDS sort) */
  uint32_t gathers;          /* all-gathers of host metadata this call (agreement points
                                included) */
  uint32_t exchanges;        /* all-to-alls of device blocks this call */
  uint32_t host_syncs;       /* host waits for the device stream (readbacks) this call */
  uint32_t agree_skipped;    /* receive-buffer agreements skipped: every rank's buffer
                                was already large enough */
  uint32_t fast_path;        /* 1: the call started on the fast path (sizes agreed up front
                                through device-assembled messages, rk_shard_fast.h) */
  uint32_t fast_retry;       /* 1: the fast attempt found a halo disagreement or an axis
                                left open and the careful driver repeated the call */
  uint32_t fast_stages;      /* fast-path stages run without agreement points (bits:
                                1 axes, 2 parents + first roots round, 4 later rounds
                                + members) */
} rk_shard_stats;

/* in_dev: this rank's block of input rows (device SoA, FILE order); blocks are
 * consecutive in rank order.  lead_in: halo depth in 100-bp buckets beyond the
 * probed neighbour (< 0: default 2); any value gives the same output, deeper
 * halos only make re-resolution rounds rarer. */
int rk_classify_sharded(rk_ctx *ctx, rk_comm *comm, const rk_frags_soa *in_dev,
                        const rk_params *p, int32_t lead_in, rk_shard_result *out);
/* The same with this rank's rows in HOST memory (copied to the device first). */
int rk_classify_sharded_host(rk_ctx *ctx, rk_comm *comm, const rk_frags_soa *in_host,
                             const rk_params *p, int32_t lead_in, rk_shard_result *out);
int rk_get_shard_stats(const rk_ctx *ctx, rk_shard_stats *st);
/* Copy a rank's share (n_out rows) into caller buffers (host or device). */
int rk_shard_copy_result(rk_ctx *ctx, const rk_shard_result *res, uint32_t *out_order,
                         uint32_t *gid, uint8_t *repval);

/* The in-group ordering primitive on its own: libstdc++ 11 std::sort (the
 * exact permutation, ties included -- commonFunctions.cpp:158) of every
 * segment [seg_off[s], seg_off[s+1]) of `keys`, on the device.  perm[x] =
 * index (into keys) of the element that ends at position x.  Host buffers. */
int rk_std_sort_segments(rk_ctx *ctx, const uint64_t *keys, uint64_t n, const uint32_t *seg_off,
                         uint32_t nseg, uint32_t *perm);

/* Phase profiling: when enabled, HIP events are recorded on the context
 * stream at every phase boundary of rk_classify*; rk_get_phase_ms returns the
 * accumulated device milliseconds (and call counts) per phase. */
enum {
  RK_PH_PREP = 0,       /* xStart/10 keys, last-bucket drop, probe validation */
  RK_PH_ORDER = 1,      /* processing-order counting sort (FragmentsDatabase buckets) */
  RK_PH_GATHER = 2,     /* processing-order SoA, centres, sort keys */
  RK_PH_OCC_CSR = 3,    /* X and Y 100-bp occupancy CSRs */
  RK_PH_SWEEP_X = 4,    /* X-axis occupancy resolution */
  RK_PH_SWEEP_Y = 5,    /* Y-axis occupancy resolution */
  RK_PH_ROOTS = 6,      /* winner chains -> roots -> group ids */
  RK_PH_MEMBERS = 7,    /* group member CSR */
  RK_PH_GROUP_SORT = 8, /* libstdc++ introsort per group */
  RK_PH_EMIT = 9,       /* repeat flags + output order */
  RK_N_PHASES = 10
};
/* enable: 0 off; 1 phase events and every kernel launch timed; 2 + k: phase
 * events and only kernel k's launches (rk_kernel_name(k)) -- the others record
 * no events, so a timed run pays for few of them. */
int rk_set_profiling(rk_ctx *ctx, int enable);
int rk_get_phase_ms(const rk_ctx *ctx, double *ms /* [RK_N_PHASES] */,
                    uint32_t *calls /* nullable */);
int rk_reset_phases(rk_ctx *ctx);
/* Launch-level timing of the pipeline's kernels while profiling: for kernel
 * index `kernel` (0 .. rk_kernel_count()-1, named by rk_kernel_name), the
 * summed HIP-event milliseconds of its launches, their summed ALGORITHMIC
 * bytes (the minimum HBM traffic each launch's job needs) and the
 * number of launches since the last rk_reset_phases. */
int rk_get_kernel_timing(const rk_ctx *ctx, int kernel, double *total_ms, double *algo_bytes,
                         uint64_t *launches);
int rk_kernel_count(void);
const char *rk_kernel_name(int kernel);
const char *rk_phase_name(int phase);

/* ---- host ingress: FragmentsDatabase (FragmentsDatabase.cpp:17-101) ---- */

typedef struct rk_db rk_db;

/* Parse a GECKO-style CSV with the reference's acceptance rules.  Returns
 * RK_E_IO if unreadable, RK_E_COUNT if more Frag lines than the header total. */
int rk_db_load_csv(const char *path, rk_db **db);
void rk_db_free(rk_db *db);
/* A parsed database as a binary SoA cache file: the header
 * text and every column rk_db_load_csv produced, so a later run skips the
 * parse (FragmentsDatabase.cpp:17-100).  Loading a cache gives a database
 * whose classification and egress are byte-identical to the CSV's.
 * RK_E_IO: cannot open / read / write; RK_E_ARG: not a complete cache file. */
int rk_db_save_soa(const rk_db *db, const char *path);
int rk_db_load_soa(const char *path, rk_db **db);
/* Borrow the SoA view (valid until rk_db_free) and header values. */
int rk_db_view(const rk_db *db, rk_frags_soa *soa, uint64_t *len_x_hdr, uint64_t *len_y_hdr,
               uint64_t *total_hdr);

/* ---- host egress: save_all_frag_pairs + SaverQueue ------------------- */

/* Write the reference's output CSV (commonFunctions.cpp:101-146). */
int rk_db_write_csv(const rk_db *db, const char *path, const rk_result *res);

/* SaverQueue (SaverQueue.h:37-41): background writer thread.  add() takes
 * ownership of copies of the result arrays; on open failure the request is
 * written to represults-<k>.csv instead (SaverQueue.cpp:16-20). */
typedef struct rk_saver rk_saver;
int rk_saver_start(const rk_db *db, rk_saver **sq);
int rk_saver_add(rk_saver *sq, const char *path, const rk_result *res, uint64_t n);
int rk_saver_stop(rk_saver *sq); /* drains the queue, joins, frees */

/* ---- synthetic inputs --------------------------------- */

typedef struct {
  uint64_t n;          /* fragments */
  uint64_t genome_len; /* L: both sequences */
  uint64_t seed;
  double family_frac;  /* share of repeat-family fragments (0.8 default, 0.95 repeat-rich) */
  uint32_t copies_lo;  /* copies per family ~ U[lo, hi): 2,30 default; 100,600 repeat-rich */
  uint32_t copies_hi;
} rk_synth_params;

int rk_synth_generate(const rk_synth_params *p, uint64_t *x_start, uint64_t *y_start,
                      uint64_t *length, uint8_t *strand, uint64_t *ident /* nullable */);
int rk_synth_write_csv(const char *path, uint64_t n, const uint64_t *x_start,
                       const uint64_t *y_start, const uint64_t *length, const uint8_t *strand,
                       const uint64_t *ident /* nullable */, uint64_t len_x_hdr,
                       uint64_t len_y_hdr);

#ifdef __cplusplus
}
#endif
#endif
