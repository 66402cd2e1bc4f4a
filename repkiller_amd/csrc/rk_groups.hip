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
                            uint32_t *pkey, uint32_t *kept, uint32_t *err) {
  uint32_t mine = 0;
  GRID_STRIDE(i, f.n) {
    const uint64_t x = f.x[i];
    const uint64_t pk = x / 10;
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
}

// Processing-order SoA, bucket keys and the in-group sort key
// |yStart - diag_func[xStart/10]|: diag_func[b] is the yStart of the LAST
// fragment of processing bucket b, i.e. of the end of k's run of equal keys.
__global__ void k_gather_proc(Frags f, Proc p, uint32_t m, uint32_t nbx, uint32_t nby) {
  GRID_STRIDE(k, m) {
    const uint32_t r = p.row[k];
    const uint64_t L = f.len[r], x = f.x[r], y = f.y[r];
    const uint64_t xc = x + L / 2, yc = y + L / 2;
    const uint32_t s = f.strand[r] == 'f' ? 0u : 1u;
    const uint32_t key = p.pkey[k];
    uint32_t e = k;
    while (e + 1 < m && p.pkey[e + 1] == key) ++e;
    const uint64_t d = e == k ? y : f.y[p.row[e]];
    p.xrec[k] = make_ulonglong2(xc, L);
    p.yrec[k] = make_ulonglong2(yc, L);
    p.ha[k] = y > d ? y - d : d - y;
    p.keyx[k] = s * nbx + (uint32_t)(xc / 100);
    p.keyy[k] = s * nby + (uint32_t)(yc / 100);
  }
}

__global__ void k_csr_fill(Csr c, const ulonglong2 *rec, const uint8_t *xstate, bool for_y,
                           uint32_t m) {
  GRID_STRIDE(q, m) {
    const uint32_t k = c.ent[q];
    const ulonglong2 r = rec[k];
    c.cen[q] = r.x;
    c.len[q] = r.y;
    c.state[q] = for_y && xstate[k] == ST_HIT ? ST_ACTIVE : ST_UNKNOWN;
  }
}

__global__ void k_csr_scatter_back(Csr c, uint8_t *state, uint32_t *win, uint32_t m) {
  GRID_STRIDE(q, m) {
    const uint32_t k = c.ent[q];
    const uint8_t st = c.state[q];
    state[k] = st;
    if (st == ST_HIT) win[k] = c.win[q];
  }
}

__global__ void k_group_offsets(const uint32_t *sgid, uint32_t m, uint32_t ngroups,
                                uint32_t *goff) {
  GRID_STRIDE(q, m) {
    if (q == 0 || sgid[q] != sgid[q - 1]) goff[sgid[q]] = q;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) goff[ngroups] = m;
}

__global__ void k_make_parents(Proc p, uint32_t m, uint32_t *isnew, uint32_t *err) {
  GRID_STRIDE(k, m) {
    const uint8_t xs = p.xstate[k], ys = p.ystate[k];
    uint32_t par = k, nw = 0;
    if (xs == ST_HIT) par = p.xwin[k];
    else if (xs == ST_ACTIVE && ys == ST_HIT) par = p.ywin[k];
    else if (xs == ST_ACTIVE && ys == ST_ACTIVE) nw = 1;
    else atomicOr(err, ERRB_INTERNAL);
    if (par > k) {  // winners are always earlier; never let a bad id reach the gathers
      atomicOr(err, ERRB_INTERNAL);
      par = k;
    }
    p.par[k] = par;
    isnew[k] = nw;
  }
}

__global__ void k_jump(Proc p, uint32_t m, uint32_t *changed) {
  bool ch = false;
  GRID_STRIDE(k, m) {
    const uint32_t a = p.par[k];
    const uint32_t b = p.par[a];
    if (a != b) {
      p.par[k] = b;
      ch = true;
    }
  }
  if (ch) *changed = 1u;
}

__global__ void k_assign_gid(Proc p, uint32_t m, const uint32_t *newrank) {
  GRID_STRIDE(k, m) p.gid[k] = newrank[p.par[k]];
}

__global__ void k_build_records(const uint32_t *gmem, const uint64_t *ha, uint32_t m,
                                uint64_t *key, uint32_t *tag) {
  GRID_STRIDE(t, m) {
    const uint32_t k = gmem[t];
    key[t] = ha[k];
    tag[t] = k;
  }
}

__global__ void k_emit(const uint32_t *tag, const uint32_t *gid_proc, const uint32_t *goff,
                       const uint32_t *row, uint32_t m, uint32_t *out_gid, uint8_t *out_rep,
                       uint32_t *out_order) {
  GRID_STRIDE(t, m) {
    const uint32_t k = tag[t];
    const uint32_t g = gid_proc[k];
    const uint32_t b = goff[g], e = goff[g + 1];
    const uint32_t r = row[k];
    out_order[t] = r;
    out_gid[r] = g;
    out_rep[r] = e - b == 1 ? 0 : (t == b ? 1 : 2);
  }
}

}  // namespace

void prep_keys(const Frags &f, uint64_t vsize, uint64_t max_x, uint64_t max_y, uint32_t *pkey,
               uint32_t *kept, uint32_t *err, hipStream_t st) {
  if (f.n)
    k_prep_keys<<<grid_for(f.n, 256, 2048), 256, 0, st>>>(f, vsize, max_x, max_y, pkey, kept, err);
}
void gather_proc(const Frags &f, Proc p, uint32_t m, uint32_t nbx, uint32_t nby, hipStream_t st) {
  if (!m) return;
  k_gather_proc<<<grid_for(m, 256), 256, 0, st>>>(f, p, m, nbx, nby);
}
void csr_fill(Csr c, const ulonglong2 *rec, const uint8_t *xstate, bool for_y, uint32_t m,
              hipStream_t st) {
  if (m) k_csr_fill<<<grid_for(m, 256), 256, 0, st>>>(c, rec, xstate, for_y, m);
}
void csr_scatter_back(Csr c, uint8_t *state, uint32_t *win, uint32_t m, hipStream_t st) {
  if (m) k_csr_scatter_back<<<grid_for(m, 256), 256, 0, st>>>(c, state, win, m);
}
void group_offsets(const uint32_t *sgid, uint32_t m, uint32_t ngroups, uint32_t *goff,
                   hipStream_t st) {
  k_group_offsets<<<grid_for(m, 256), 256, 0, st>>>(sgid, m, ngroups, goff);
}
void make_parents(Proc p, uint32_t m, uint32_t *isnew, uint32_t *err, hipStream_t st) {
  if (m) k_make_parents<<<grid_for(m, 256), 256, 0, st>>>(p, m, isnew, err);
}
void jump_round(Proc p, uint32_t m, uint32_t *changed, hipStream_t st) {
  if (m) k_jump<<<grid_for(m, 256), 256, 0, st>>>(p, m, changed);
}
void assign_gid(Proc p, uint32_t m, const uint32_t *newrank, hipStream_t st) {
  if (m) k_assign_gid<<<grid_for(m, 256), 256, 0, st>>>(p, m, newrank);
}
void build_records(const uint32_t *gmem, const uint64_t *ha, uint32_t m, uint64_t *key,
                   uint32_t *tag, hipStream_t st) {
  if (m) k_build_records<<<grid_for(m, 256), 256, 0, st>>>(gmem, ha, m, key, tag);
}
void emit_result(const uint32_t *tag, const uint32_t *gid_proc, const uint32_t *goff,
                 const uint32_t *row, uint32_t m, uint32_t *out_gid, uint8_t *out_rep,
                 uint32_t *out_order, hipStream_t st) {
  if (m)
    k_emit<<<grid_for(m, 256), 256, 0, st>>>(tag, gid_proc, goff, row, m, out_gid, out_rep,
                                             out_order);
}
void fill_dropped(uint32_t n, uint32_t *out_gid, uint8_t *out_rep, hipStream_t st) {
  (void)hipMemsetAsync(out_gid, 0xFF, (size_t)n * sizeof(uint32_t), st);
  (void)hipMemsetAsync(out_rep, 0xFF, (size_t)n, st);
}

}  // namespace rk
