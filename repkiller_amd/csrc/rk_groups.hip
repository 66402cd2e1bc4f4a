// rk_groups.hip -- processing order, group resolution and in-group ordering.
//
//   prep_keys      FragmentsDatabase bucketing: key xStart/10, the last bucket
//                  (vsize-1) is never iterated (FragmentsDatabase.h:29-31) and
//                  xStart/10 >= vsize is out of bounds in the reference (:96-97);
//                  probe ranges of SequenceOcupationList are validated here.
//   gather_proc    processing-order SoA: centres xStart+len/2 / yStart+len/2
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
//   sort_groups    std::sort of every group with more than one member by that
//                  key (commonFunctions.cpp:158), the libstdc++ 11 introsort
//                  reproduced exactly (depth 2*lg n, median-of-3 pivot moved to
//                  first, unguarded Hoare partition, heapsort fallback, final
//                  insertion sort) -- ties make the permutation implementation-
//                  defined, and the repeat flag depends on which member ends first.
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
  // one atomic per wave
  for (int off = 32; off > 0; off >>= 1) mine += __shfl_xor(mine, off);
  if ((threadIdx.x & 63) == 0 && mine) atomicAdd(kept, mine);
}

__global__ void k_gather_proc(Frags f, Proc p, uint32_t m, uint32_t nbx, uint32_t nby) {
  GRID_STRIDE(k, m) {
    const uint32_t r = p.row[k];
    const uint64_t L = f.len[r], x = f.x[r], y = f.y[r];
    const uint64_t xc = x + L / 2, yc = y + L / 2;
    const uint32_t s = f.strand[r] == 'f' ? 0u : 1u;
    p.xc[k] = xc;
    p.yc[k] = yc;
    p.len[k] = L;
    p.keyx[k] = s * nbx + (uint32_t)(xc / 100);
    p.keyy[k] = s * nby + (uint32_t)(yc / 100);
  }
}

// In-group sort key |yStart - diag_func[xStart/10]|: diag_func[b] is the yStart
// of the LAST fragment of processing bucket b.  The thread at each run end of
// the sorted processing keys fills its whole run (each element written once).
__global__ void k_diag_keys(Proc p, uint32_t m) {
  GRID_STRIDE(k, m) {
    const uint32_t key = p.pkey[k];
    if (k + 1 < m && p.pkey[k + 1] == key) continue;
    const uint64_t d = p.yc[k] - p.len[k] / 2;  // yStart of the last fragment
    uint32_t j = k;
    for (;;) {
      const uint64_t y = p.yc[j] - p.len[j] / 2;
      p.ha[j] = y > d ? y - d : d - y;
      if (j == 0 || p.pkey[j - 1] != key) break;
      --j;
    }
  }
}

__global__ void k_csr_fill(Csr c, const uint64_t *cen, const uint64_t *len,
                           const uint8_t *xstate, bool for_y, uint32_t m) {
  GRID_STRIDE(q, m) {
    const uint32_t k = c.ent[q];
    c.cen[q] = cen[k];
    c.len[q] = len[k];
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

// ---- libstdc++ 11 std::sort, restated on (key, tag) arrays ----------------
struct Seq {
  uint64_t *key;
  uint32_t *tag;
  __device__ __forceinline__ void swap(long a, long b) const {
    uint64_t k = key[a];
    key[a] = key[b];
    key[b] = k;
    uint32_t t = tag[a];
    tag[a] = tag[b];
    tag[b] = t;
  }
};

// __adjust_heap + __push_heap (bits/stl_heap.h)
__device__ void adjust_heap(const Seq &s, long hole, long len, uint64_t vk, uint32_t vt) {
  const long top = hole;
  long child = hole;
  while (child < (len - 1) / 2) {
    child = 2 * (child + 1);
    if (s.key[child] < s.key[child - 1]) child--;
    s.key[hole] = s.key[child];
    s.tag[hole] = s.tag[child];
    hole = child;
  }
  if ((len & 1) == 0 && child == (len - 2) / 2) {
    child = 2 * (child + 1);
    s.key[hole] = s.key[child - 1];
    s.tag[hole] = s.tag[child - 1];
    hole = child - 1;
  }
  long parent = (hole - 1) / 2;
  while (hole > top && s.key[parent] < vk) {
    s.key[hole] = s.key[parent];
    s.tag[hole] = s.tag[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  s.key[hole] = vk;
  s.tag[hole] = vt;
}

// __partial_sort(first, last, last) == __make_heap + __sort_heap
__device__ void heap_sort(const Seq &s, long len) {
  if (len >= 2) {
    for (long parent = (len - 2) / 2;; --parent) {
      adjust_heap(s, parent, len, s.key[parent], s.tag[parent]);
      if (parent == 0) break;
    }
  }
  for (long last = len; last > 1;) {
    --last;
    const uint64_t vk = s.key[last];
    const uint32_t vt = s.tag[last];
    s.key[last] = s.key[0];
    s.tag[last] = s.tag[0];
    adjust_heap(s, 0, last, vk, vt);
  }
}

__device__ __forceinline__ void median_to_first(const Seq &s, long r, long a, long b, long c) {
  const uint64_t ka = s.key[a], kb = s.key[b], kc = s.key[c];
  long m;
  if (ka < kb) m = kb < kc ? b : (ka < kc ? c : a);
  else m = ka < kc ? a : (kb < kc ? c : b);
  s.swap(r, m);
}

__device__ __forceinline__ long unguarded_partition(const Seq &s, long first, long last,
                                                    uint64_t pivot) {
  for (;;) {
    while (s.key[first] < pivot) ++first;
    --last;
    while (pivot < s.key[last]) --last;
    if (!(first < last)) return first;
    s.swap(first, last);
    ++first;
  }
}

__device__ void std_sort(const Seq &s, long n) {
  if (n < 2) return;
  struct Frame {
    long first, last;
    int depth;
  };
  Frame stack[72];
  int sp = 0;
  stack[sp++] = {0, n, 2 * (63 - __builtin_clzll((unsigned long long)n))};
  while (sp) {
    Frame f = stack[--sp];
    long first = f.first, last = f.last;
    int depth = f.depth;
    while (last - first > 16) {  // __introsort_loop
      if (depth == 0) {
        heap_sort(Seq{s.key + first, s.tag + first}, last - first);
        break;
      }
      --depth;
      median_to_first(s, first, first + 1, first + (last - first) / 2, last - 1);
      const long cut = unguarded_partition(s, first + 1, last, s.key[first]);
      stack[sp++] = {cut, last, depth};
      last = cut;
    }
  }
  // __final_insertion_sort: a stable insertion pass (guarded for the first 16)
  for (long i = 1; i < n; ++i) {
    const uint64_t vk = s.key[i];
    const uint32_t vt = s.tag[i];
    long j = i;
    while (j > 0 && vk < s.key[j - 1]) {
      s.key[j] = s.key[j - 1];
      s.tag[j] = s.tag[j - 1];
      --j;
    }
    s.key[j] = vk;
    s.tag[j] = vt;
  }
}

__global__ void k_sort_groups(const uint32_t *goff, uint32_t ngroups, uint64_t *key,
                              uint32_t *tag) {
  GRID_STRIDE(g, ngroups) {
    const uint32_t b = goff[g], e = goff[g + 1];
    if (e - b > 1) std_sort(Seq{key + b, tag + b}, (long)(e - b));
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
  if (f.n) k_prep_keys<<<grid_for(f.n, 256), 256, 0, st>>>(f, vsize, max_x, max_y, pkey, kept, err);
}
void gather_proc(const Frags &f, Proc p, uint32_t m, uint32_t nbx, uint32_t nby, hipStream_t st) {
  if (!m) return;
  k_gather_proc<<<grid_for(m, 256), 256, 0, st>>>(f, p, m, nbx, nby);
  k_diag_keys<<<grid_for(m, 256), 256, 0, st>>>(p, m);
}
void csr_fill(Csr c, const uint64_t *cen, const uint64_t *len, const uint8_t *xstate, bool for_y,
              uint32_t m, hipStream_t st) {
  if (m) k_csr_fill<<<grid_for(m, 256), 256, 0, st>>>(c, cen, len, xstate, for_y, m);
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
void sort_groups(const uint32_t *goff, uint32_t ngroups, uint64_t *key, uint32_t *tag,
                 hipStream_t st) {
  if (ngroups) k_sort_groups<<<grid_for(ngroups, 64), 64, 0, st>>>(goff, ngroups, key, tag);
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
