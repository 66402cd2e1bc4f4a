// rk_groups.hip -- processing order, group resolution and in-group ordering.
//
//   prep_keys      FragmentsDatabase bucketing: key xStart/10, the last bucket
//                  (vsize-1) is never iterated (FragmentsDatabase.h:29-31) and
//                  xStart/10 >= vsize is out of bounds in the reference (:96-97);
//                  probe ranges of SequenceOcupationList are validated here.
//   gather_proc    processing-order SoA (rows gathered in the radix-sorted
//                  order): centres xStart+len/2 / yStart+len/2
//                  (commonFunctions.cpp:55,59,63,67), 100-bp bucket keys, and
//                  the sort key |yStart - diag_func[xStart/10]| where diag_func[b]
//                  is the yStart of the LAST fragment of bucket b
//                  (commonFunctions.cpp:161-177, `oh` never updated; :149-157).
//   make_parents / jump_round / assign_gid
//                  a fragment joins the group of its X winner, else of its Y
//                  winner, else opens a new group (commonFunctions.cpp:55-76);
//                  groups never merge, so group(i) = group(root of the winner
//                  chain); gid = rank of the root among new groups in processing
//                  order (creation order, :74 and :120,127).
//   (sort_groups    -> rk_groupsort.hip)
//   emit_result    repeat flag: singleton 0, first 1, rest 2 (:106-115).
#include "rk_internal.h"

namespace rk {
namespace {

#define GRID_STRIDE(i, n)                                                      \
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < (n);           \
       i += gridDim.x * blockDim.x)

// largest bucket index get_associated_group touches for centre c
__device__ __forceinline__ uint64_t probe_max_bucket(uint64_t c, uint64_t max_index) {
  uint64_t b = c / 100;
  if (c < max_index && (c + 1) / 100 > b) b = (c + 1) / 100;
  if (c < max_index - 1 && (c + 2) / 100 > b) b = (c + 2) / 100;
  return b;
}

__global__ void k_prep_keys(Frags f, uint64_t vsize, uint64_t max_x, uint64_t max_y,
                            uint32_t *pkey, ulonglong2 *rec, uint32_t *kept, uint32_t *err) {
  uint32_t mine = 0;
  bool wide = false;  // a length >= 2^31 (disables the 32-bit sweep)
  GRID_STRIDE(i, f.n) {
    const uint64_t x = f.x[i];
    wide |= f.len[i] >= 0x80000000ull;
    const uint64_t pk = x / 10;
    // pack the row once, coalesced, so the processing-order gather is one
    // 32-B read per row instead of four scattered reads (the sharded driver
    // packs its rows elsewhere: rec null)
    if (rec) {
      rec[2 * (size_t)i] = make_ulonglong2(x, f.y[i]);
      rec[2 * (size_t)i + 1] = make_ulonglong2(f.len[i], f.strand[i]);
    }
    uint32_t key = (uint32_t)(vsize - 1);  // the never-iterated last bucket sorts last
    if (pk >= vsize) {
      atomicOr(err, ERRB_UB_BUCKET);
    } else if (pk != vsize - 1) {
      const uint64_t h = f.len[i] / 2;
      if (probe_max_bucket(x + h, max_x) > max_x || probe_max_bucket(f.y[i] + h, max_y) > max_y)
        atomicOr(err, ERRB_UB_CENTER);
      key = (uint32_t)pk;
      ++mine;
    }
    pkey[i] = key;
  }
  // one atomic per block (grid <= 2048 blocks)
  __shared__ uint32_t part[4];
  for (int off = 32; off > 0; off >>= 1) mine += __shfl_xor(mine, off);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = mine;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t = part[0] + part[1] + part[2] + part[3];
    if (t) atomicAdd(kept, t);
  }
  // the ballot runs in every lane (inside `lane == 0 && ...` it would see lane 0 only)
  const uint64_t any_wide = __ballot(wide);
  if ((threadIdx.x & 63) == 0 && any_wide) atomicOr(err, ERRB_WIDE_LENGTH);
}

// Processing-order SoA and bucket keys (one 32-B record gather per row).
__global__ void k_gather_proc(Proc p, uint32_t m, uint32_t nbx, uint32_t nby) {
  GRID_STRIDE(k, m) {
    const uint32_t r = p.row[k];
    const ulonglong2 a = p.rec[2 * (size_t)r], b = p.rec[2 * (size_t)r + 1];
    const uint64_t x = a.x, y = a.y, L = b.x;
    const uint64_t xc = x + L / 2;
    const uint32_t s = (uint8_t)b.y == 'f' ? 0u : 1u;  // strand: the low byte
    p.ys[k] = y;
    p.xrec[k] = make_ulonglong2(xc, L);
    p.yrec[k] = make_ulonglong2(y + L / 2, L & 0xFFFFFFFFull);  // X result merged later
    if (p.ylenhi) p.ylenhi[k] = (uint32_t)(L >> 32);
    if (p.grow) p.grow[k] = (uint32_t)(b.y >> 32);
    p.keyx[k] = s * nbx + (uint32_t)(xc / 100);
    p.keyy[k] = s * nby + (uint32_t)((y + L / 2) / 100);
  }
}

// In-group sort key |yStart - diag_func[xStart/10]|: diag_func[b] is the yStart
// of the LAST fragment of processing bucket b, i.e. of the end of k's run of
// equal processing keys.  Run ends inside the wavefront come from a ballot and
// a shuffle; the run that crosses the wave's end (always the one holding lane
// 63) is followed by the whole wave, 64 keys per step.
__global__ void __launch_bounds__(256) k_sort_keys(Proc p, uint32_t m, uint32_t *wide) {
  const uint32_t lane = threadIdx.x & 63;
  bool wd = false;
  for (uint32_t base = (blockIdx.x * blockDim.x + threadIdx.x) & ~63u; base < m;
       base += gridDim.x * blockDim.x) {
    const uint32_t k = base + lane;
    const bool in = k < m;
    const uint32_t key = in ? p.pkey[k] : 0u;
    const uint64_t y = in ? p.ys[k] : 0ull;
    const bool end = in && (k + 1 == m || p.pkey[k + 1] != key);
    const uint64_t ends = __ballot(end) & ~((1ull << lane) - 1ull);
    const int src = ends ? __ffsll((unsigned long long)ends) - 1 : 63;
    uint64_t d = __shfl(y, src);
    if (__ballot(in && !ends)) {  // the last run continues past this wave
      const uint32_t klast = __shfl(key, 63);
      uint32_t e = 0;
      for (uint32_t b = base + 64;; b += 64) {
        const uint32_t q = b + lane;
        const uint64_t stop = __ballot(q >= m || p.pkey[q] != klast);
        if (stop) {
          e = b + __builtin_ctzll(stop) - 1;  // the run's last entry
          break;
        }
      }
      if (in && !ends) d = p.ys[e];
    }
    const uint64_t h = y > d ? y - d : d - y;
    if (in) p.hrec[k] = make_ulonglong2(h, p.row[k]);
    wd |= in && (h >> 32) != 0;
  }
  // one flag per wave, and only while unset: a 15-Gbp set has wide keys in
  // every wave, and one hot atomic address serialises (~90 per us)
  if (__ballot(wd) && lane == 0 && *(volatile uint32_t *)wide == 0) atomicOr(wide, 1u);
}

__device__ __forceinline__ uint8_t nbd_code(uint64_t c, uint64_t max_index) {
  const int d = neighbour_dir(c, max_index);
  return d < 0 ? 1 : d > 0 ? 2 : 0;
}

__global__ void k_csr_fill_x(Csr c, const ulonglong2 *xrec, uint32_t m, uint64_t max_index) {
  GRID_STRIDE(q, m) {
    const ulonglong2 r = xrec[c.ent[q]];
    if (c.cen) c.cen[q] = r.x, c.len[q] = r.y;  // the 64-bit kernels only
    c.pk[q] = make_uint2((uint32_t)r.x, (uint32_t)r.y);
    c.nbd[q] = nbd_code(r.x, max_index);
    c.state[q] = ST_UNKNOWN;
  }
}

// X hits sit in the Y list (commonFunctions.cpp:59); X misses query Y
__global__ void k_csr_fill_y(Csr c, const ulonglong2 *yrec, const uint32_t *ylenhi, uint32_t m,
                             uint64_t max_index) {
  GRID_STRIDE(q, m) {
    const size_t k = c.ent[q];
    const ulonglong2 a = yrec[k];
    if (c.cen) {  // the 64-bit kernels only
      c.cen[q] = a.x;
      c.len[q] = (a.y & 0xFFFFFFFFull) | (ylenhi ? (uint64_t)ylenhi[k] << 32 : 0ull);
    }
    c.pk[q] = make_uint2((uint32_t)a.x, (uint32_t)a.y);
    c.nbd[q] = nbd_code(a.x, max_index);
    c.state[q] = (uint32_t)(a.y >> 32) != NONE ? ST_ACTIVE : ST_UNKNOWN;
  }
}

__global__ void k_group_offsets_unaligned(const uint32_t *sgid, uint32_t m, uint32_t ngroups,
                                          uint32_t *goff) {
  GRID_STRIDE(q, m) {
    if (q == 0 || sgid[q] != sgid[q - 1]) goff[sgid[q]] = q;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) goff[ngroups] = m;
}
// the same with four positions per thread (one 16-B load; sgid 16-B aligned):
// a group starts where the gid differs from the previous position's
__global__ void __launch_bounds__(256) k_group_offsets(const uint32_t *sgid, uint32_t m,
                                                        uint32_t ngroups, uint32_t *goff) {
  const uint32_t nq = (m + 3) / 4;
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < nq; t += gridDim.x * blockDim.x) {
    const uint32_t q0 = t * 4;
    uint32_t g[4];
    if (q0 + 4 <= m) {
      const uint4 v = *reinterpret_cast<const uint4 *>(sgid + q0);
      g[0] = v.x, g[1] = v.y, g[2] = v.z, g[3] = v.w;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) g[j] = q0 + j < m ? sgid[q0 + j] : 0u;
    }
    uint32_t prev = q0 ? sgid[q0 - 1] : ~0u;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (q0 + j < m && g[j] != prev) goff[g[j]] = q0 + j;
      prev = g[j];
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) goff[ngroups] = m;
}

// Every thread follows its parent chain towards the root (up to 32 links per
// round) and stores what it reached; other threads compress the same chains
// concurrently, which only ever replaces a parent by one of its ancestors.
// Winner chains are short, so one round usually finishes; a chain longer than
// the step budget reports `changed` and the host runs another round.
__global__ void k_jump(Proc p, uint32_t m, uint32_t *changed, uint32_t *isnew, uint32_t *err,
                       const uint32_t *open) {
  if (open && (open[0] | open[1])) return;  // parents not final: the caller repeats the axes
  bool ch = false;
  GRID_STRIDE(k, m) {
    const uint32_t a0 = p.par[k];
    uint32_t a = a0;
    if (isnew && a > k) {  // first round: parents are always earlier
      atomicOr(err, ERRB_INTERNAL);
      a = k;
      p.par[k] = k;
    }
    if (isnew) isnew[k] = a == k;
    int step = 0;
    for (; step < 32; ++step) {
      const uint32_t b = p.par[a];
      if (b == a) break;
      a = b;
    }
    if (a != a0) p.par[k] = a;
    // a root stays a root (only non-roots' parents are rewritten), so a chain
    // that ended on one is final; 32 jumps without reaching one need a round more
    if (step == 32) ch = true;
  }
  if (ch) *changed = 1u;
}

// The first round again, except that an element whose chain is longer than
// the step budget is listed (list[(*count)++] = k) instead of flagging another
// round, and k_jump_rest follows only the listed chains: the sharded fast
// path compresses its slice without reading a flag back between rounds.
__global__ void k_jump_list(Proc p, uint32_t m, uint32_t *isnew, uint32_t *err, uint32_t *list,
                            uint32_t *count) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k - lane < m;
       k += gridDim.x * blockDim.x) {
    bool open = false;
    if (k < m) {
      const uint32_t a0 = p.par[k];
      uint32_t a = a0;
      if (a > k) {  // parents are always earlier
        atomicOr(err, ERRB_INTERNAL);
        a = k;
        p.par[k] = k;
      }
      isnew[k] = a == k;
      int step = 0;
      for (; step < 32; ++step) {
        const uint32_t b = p.par[a];
        if (b == a) break;
        a = b;
      }
      if (a != a0) p.par[k] = a;
      open = step == 32;
    }
    const uint64_t b = __ballot(open);
    if (b) {
      uint32_t at = 0;
      if (lane == 0) at = atomicAdd(count, (uint32_t)__popcll(b));
      at = (uint32_t)__shfl((int)at, 0);
      if (open) list[at + __popcll(b & ((1ull << lane) - 1ull))] = k;
    }
  }
}

// the listed chains to their roots (the other listed elements compress the
// same chains meanwhile); a chain still open after 4096 links (a crafted
// input) raises *changed
__global__ void k_jump_rest(Proc p, const uint32_t *list, const uint32_t *count,
                            uint32_t *changed) {
  const uint32_t n = *count;
  bool ch = false;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t k = list[i];
    uint32_t a = p.par[k];
    int step = 0;
    for (; step < 4096; ++step) {
      const uint32_t b = p.par[a];
      if (b == a) break;
      a = b;
    }
    p.par[k] = a;
    ch |= step == 4096;
  }
  if (ch) *changed = 1u;
}

__global__ void k_assign_gid(Proc p, uint32_t m, const uint32_t *newrank) {
  GRID_STRIDE(k, m) p.gid[k] = newrank[p.par[k]];
}

// one 16-B gather per member: sort key and file row; the tag is the member's
// slot, so the emit below reads the row back from inside its own group
__global__ void k_build_records(uint32_t *gmem, const ulonglong2 *hrec, uint32_t m,
                                uint64_t *key, uint32_t *tag) {
  GRID_STRIDE(t, m) {
    const ulonglong2 r = hrec[gmem[t]];
    key[t] = r.x;
    tag[t] = t;
    gmem[t] = (uint32_t)r.y;
  }
}

__global__ void k_emit(const uint32_t *otag, const uint32_t *sgid, const uint32_t *goff,
                       const uint32_t *mrow, uint32_t m, uint32_t *out_gid, uint8_t *out_rep,
                       uint32_t *out_order) {
  GRID_STRIDE(t, m) {
    const uint32_t g = sgid[t];
    const uint32_t o = otag[t];  // issued beside the bounds (unwritten for a singleton)
    const uint32_t b = goff[g], e = goff[g + 1];
    // a one-member group is not written by the group sort: its slot is itself
    out_order[t] = mrow[e - b == 1 ? t : o];
    out_gid[t] = g;
    out_rep[t] = e - b == 1 ? 0 : (t == b ? 1 : 2);
  }
}

}  // namespace

void prep_keys(const Frags &f, uint64_t vsize, uint64_t max_x, uint64_t max_y, uint32_t *pkey,
               ulonglong2 *rec, uint32_t *kept, uint32_t *err, hipStream_t st) {
  if (f.n)
  {
    kt_begin(st, KID_PREP);
    k_prep_keys<<<grid_for(f.n, 256, 2048), 256, 0, st>>>(f, vsize, max_x, max_y, pkey, rec, kept,
                                                           err);
    kt_end(st, KID_PREP, (rec ? 61.0 : 29.0) * f.n);  // x, y, len, strand in; key (+ 32-B record) out
  }
}
void gather_proc(const Frags &f, Proc p, uint32_t m, uint32_t nbx, uint32_t nby, hipStream_t st) {
  if (!m) return;
  (void)f;
  kt_begin(st, KID_GATHER);
  k_gather_proc<<<grid_for(m, 256), 256, 0, st>>>(p, m, nbx, nby);
  kt_end(st, KID_GATHER, 84.0 * m);  // row + record in; ys, xrec, yrec, keyx, keyy out
}
void sort_keys(Proc p, uint32_t m, uint32_t *wide, hipStream_t st) {
  if (!m) return;
  kt_begin(st, KID_SORT_KEYS);
  k_sort_keys<<<grid_for(m, 256), 256, 0, st>>>(p, m, wide);
  kt_end(st, KID_SORT_KEYS, 32.0 * m);  // key, yStart, row in; (sort key, row) out
}
void csr_fill_x(Csr c, const ulonglong2 *xrec, uint32_t m, uint64_t max_index, hipStream_t st) {
  if (!m) return;
  kt_begin(st, KID_CSR_FILL_X);
  k_csr_fill_x<<<grid_for(m, 256), 256, 0, st>>>(c, xrec, m, max_index);
  // id + record in; (centre, length,) packed record, neighbour code, state out
  kt_end(st, KID_CSR_FILL_X, (c.cen ? 46.0 : 30.0) * m);
}
void csr_fill_y(Csr c, const ulonglong2 *yrec, const uint32_t *ylenhi, uint32_t m,
                uint64_t max_index, hipStream_t st) {
  if (!m) return;
  kt_begin(st, KID_CSR_FILL_Y);
  k_csr_fill_y<<<grid_for(m, 256), 256, 0, st>>>(c, yrec, ylenhi, m, max_index);
  // id, Y record in; (centre, length,) packed record, neighbour code, state out
  kt_end(st, KID_CSR_FILL_Y, (c.cen ? 46.0 : 30.0) * m);
}
void group_offsets(const uint32_t *sgid, uint32_t m, uint32_t ngroups, uint32_t *goff,
                   hipStream_t st) {
  kt_begin(st, KID_GROUP_OFFSETS);
  if ((reinterpret_cast<uintptr_t>(sgid) & 15) == 0)
    k_group_offsets<<<grid_for((m + 3) / 4, 256, 16384), 256, 0, st>>>(sgid, m, ngroups, goff);
  else
    k_group_offsets_unaligned<<<grid_for(m, 256), 256, 0, st>>>(sgid, m, ngroups, goff);
  kt_end(st, KID_GROUP_OFFSETS, 4.0 * m + 4.0 * ngroups);
}
void jump_round(Proc p, uint32_t m, uint32_t *changed, uint32_t *isnew, uint32_t *err,
                hipStream_t st, const uint32_t *open) {
  if (!m) return;
  kt_begin(st, KID_JUMP);
  k_jump<<<grid_for(m, 256, (size_t)1 << 20), 256, 0, st>>>(p, m, changed, isnew, err, open);
  kt_end(st, KID_JUMP, (isnew ? 16.0 : 12.0) * m);  // parent, root, parent written (+ new flag)
}
void jump_listed(Proc p, uint32_t m, uint32_t *isnew, uint32_t *err, uint32_t *list,
                 uint32_t *count, uint32_t *changed, hipStream_t st) {
  if (!m) return;
  (void)hipMemsetAsync(count, 0, 4, st);
  kt_begin(st, KID_JUMP);
  k_jump_list<<<grid_for(m, 256, (size_t)1 << 20), 256, 0, st>>>(p, m, isnew, err, list, count);
  kt_end(st, KID_JUMP, 16.0 * m);
  kt_begin(st, KID_JUMP);
  k_jump_rest<<<1024, 256, 0, st>>>(p, list, count, changed);
  kt_end(st, KID_JUMP, 0.0);
}
void assign_gid(Proc p, uint32_t m, const uint32_t *newrank, hipStream_t st) {
  if (!m) return;
  kt_begin(st, KID_ASSIGN_GID);
  k_assign_gid<<<grid_for(m, 256), 256, 0, st>>>(p, m, newrank);
  kt_end(st, KID_ASSIGN_GID, 12.0 * m);  // root, root's rank in; gid out
}
void build_records(uint32_t *gmem, const ulonglong2 *hrec, uint32_t m, uint64_t *key,
                   uint32_t *tag, hipStream_t st) {
  if (!m) return;
  kt_begin(st, KID_BUILD_RECORDS);
  k_build_records<<<grid_for(m, 256), 256, 0, st>>>(gmem, hrec, m, key, tag);
  kt_end(st, KID_BUILD_RECORDS, 36.0 * m);  // member, (key, row) in; key, tag, row out
}
void emit_result(const uint32_t *otag, const uint32_t *sgid, const uint32_t *goff,
                 const uint32_t *mrow, uint32_t m, uint32_t *out_gid, uint8_t *out_rep,
                 uint32_t *out_order, hipStream_t st) {
  if (!m) return;
  kt_begin(st, KID_EMIT);
  k_emit<<<grid_for(m, 256), 256, 0, st>>>(otag, sgid, goff, mrow, m, out_gid, out_rep,
                                           out_order);
  kt_end(st, KID_EMIT, 29.0 * m);  // slot, gid, group bounds, row in; gid, flag, order out
}

}  // namespace rk
