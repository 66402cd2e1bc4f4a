// rk_groupsort.hip -- sort_groups (commonFunctions.cpp:148-159) on gfx950.
//
// The reference std::sort()s every group with more than one member by
// |yStart - diag_func[xStart/10]|.  std::sort is libstdc++'s unstable introsort
// and the keys have many ties, so the exact permutation -- which member is
// written first and gets repeat flag 1 -- depends on every median-of-three
// choice and every Hoare swap.  This file reproduces libstdc++ 11 exactly
// (bits/stl_algo.h __sort / __introsort_loop / __unguarded_partition_pivot /
// __final_insertion_sort, bits/stl_heap.h for the depth-limit heapsort),
// restated in oracle/rk_oracle.c and pinned against std::sort by
// tests/test_oracle.py.
//
// Parallel form:
//   * Hoare partition of [f,l) with pivot p at f: the left scan stops at
//     "L-stoppers" (key >= p, positions > f), the right scan at "R-stoppers"
//     (key <= p, the pivot itself included).  Because every swap only touches
//     positions the scans have already passed, the k-th swap exchanges the
//     k-th L-stopper (from the left) with the k-th R-stopper (from the right)
//     of the ORIGINAL segment, for every k < K where K is the first k with
//     Lpos[k] >= Rpos[k]; the returned cut is min(Lpos[K], Rpos[K-1]) (Lpos[0]
//     when K == 0).  A wavefront computes both lists with ballots, finds K and
//     does the K swaps in parallel.
//   * After the loop every leaf segment (<= 16) is mutually ordered with its
//     neighbours, so __final_insertion_sort == a stable sort inside each leaf:
//     every element's final slot is its stable rank inside its leaf.
//
// Tiers (chosen per group by size): 1..16 members -> one thread per member
// (insertion sort == stable rank); 17..64 -> one wavefront per group entirely
// in registers; 65..512 and 513..2048 -> one wavefront per group with the
// group staged in LDS (12 KB / 45 KB per wave); larger -> the same wavefront
// code on global memory.  Segments of <= 64 inside the larger tiers are
// finished in registers as well.
// In every tier the result goes to `otag` (member order, group-major).
#include "rk_internal.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace rk {
namespace {

constexpr int THRESH = 16;  // libstdc++ _S_threshold

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// global-memory tier: stores by one lane must be visible to the other lanes
__device__ __forceinline__ void wave_sync_global() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

template <bool GLOBAL>
__device__ __forceinline__ void sync_mem() {
  if (GLOBAL) wave_sync_global();
  else wave_sync();
}

// a group's working arrays: keys, tags, the stopper position lists and leaf
// marks; the LDS tiers keep 32-bit keys (when every key fits), 16-bit
// positions and 16-bit tags (positions inside the group: the output adds the
// group's base), the global tier 64-bit keys and 32-bit positions and tags
template <class KT_, class PT_, class TT_ = uint32_t>
struct ViewT {
  using key_t = KT_;
  using tag_t = TT_;
  KT_ *K;
  TT_ *T;
  PT_ *PL, *PR;  // stopper position lists (capacity n)
  uint8_t *B;    // 1 = leaf start, 2 = inside a heap-sorted segment
};
using GView = ViewT<uint64_t, uint32_t>;

template <class V>
__device__ __forceinline__ void vswap(const V &v, uint32_t a, uint32_t b) {
  const typename V::key_t k = v.K[a];
  v.K[a] = v.K[b];
  v.K[b] = k;
  const uint32_t t = v.T[a];
  v.T[a] = v.T[b];
  v.T[b] = t;
}

// __move_median_to_first(result=f, a=f+1, b=mid, c=l-1)
template <class V>
__device__ __forceinline__ void median_to_first(const V &v, uint32_t f, uint32_t l) {
  const uint32_t a = f + 1, b = f + (l - f) / 2, c = l - 1;
  const typename V::key_t ka = v.K[a], kb = v.K[b], kc = v.K[c];
  uint32_t m;
  if (ka < kb) m = kb < kc ? b : (ka < kc ? c : a);
  else m = ka < kc ? a : (kb < kc ? c : b);
  vswap(v, f, m);
}

// __adjust_heap + __push_heap on v.K/T[base ..)
template <class V>
__device__ void adjust_heap(const V &v, uint32_t base, long hole, long len,
                            typename V::key_t vk, uint32_t vt) {
  const long top = hole;
  long child = hole;
  typename V::key_t *K = v.K + base;
  typename V::tag_t *T = v.T + base;
  while (child < (len - 1) / 2) {
    child = 2 * (child + 1);
    if (K[child] < K[child - 1]) child--;
    K[hole] = K[child];
    T[hole] = T[child];
    hole = child;
  }
  if ((len & 1) == 0 && child == (len - 2) / 2) {
    child = 2 * (child + 1);
    K[hole] = K[child - 1];
    T[hole] = T[child - 1];
    hole = child - 1;
  }
  long parent = (hole - 1) / 2;
  while (hole > top && K[parent] < vk) {
    K[hole] = K[parent];
    T[hole] = T[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  K[hole] = vk;
  T[hole] = vt;
}

// __partial_sort(first, last, last): __make_heap + __sort_heap; marks B = 2
template <class V>
__device__ void heap_sort_segment(const V &v, uint32_t f, uint32_t l) {
  const long len = (long)(l - f);
  if (len >= 2) {
    for (long parent = (len - 2) / 2;; --parent) {
      adjust_heap(v, f, parent, len, v.K[f + parent], v.T[f + parent]);
      if (parent == 0) break;
    }
  }
  for (long last = len; last > 1;) {
    --last;
    const typename V::key_t vk = v.K[f + last];
    const uint32_t vt = v.T[f + last];
    v.K[f + last] = v.K[f];
    v.T[f + last] = v.T[f];
    adjust_heap(v, f, 0, last, vk, vt);
  }
  if (v.B)
    for (uint32_t x = f; x < l; ++x) v.B[x] = 2;
}

// ---------------------------------------------------------------------------
// __partial_sort(first, last, last) of a LARGE segment (its depth budget spent:
// a median-of-three killer, never ordinary data), one 256-thread block:
//  * __make_heap calls __adjust_heap for the parents (len-2)/2 down to 0; a
//    call touches only its own subtree and every deeper level comes first, so
//    the calls of one level run in parallel, level after level;
//  * __sort_heap by wavefront 0, the heap's top HLV levels kept in LDS.  A
//    pop's __adjust_heap descent (the larger child -- the right one unless
//    right < left --, down while the hole has two children, then a lone left
//    child) is found up to HR levels at a time: lanes load the 2^(HR+1) - 2
//    nodes below the hole (two per lane), each right child compares with its
//    left sibling (one xor shuffle), one ballot holds every direction and the
//    path follows in scalar steps.  __push_heap of the displaced value then
//    needs no loads: the path's keys descend, so the value rises past exactly
//    the path keys below it (a ballot count), and only the path positions
//    above its slot are written.
constexpr uint32_t HEAP_BLOCK_MIN = 2048;  // smaller exhausted segments: one thread
constexpr int HLV = 13;                    // heap levels in LDS
// k_heap_segments keeps the heap's top HLV levels in LDS: 2^13 x (8 + 4)
// B = 96 KB of static LDS, which needs gfx950's 160 KB per workgroup (64 KB
// on gfx942 / gfx90a)
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "rk_groupsort.hip: k_heap_segments needs gfx950 (160 KB of LDS per workgroup)"
#endif
constexpr uint32_t HTOP = (1u << HLV) - 1;
constexpr int HR = 6;                      // levels per descent round (126 nodes)
constexpr uint32_t HR_LAST = (1u << HR) - 2, HR_NODES = (2u << HR) - 2;  // 62, 126
static_assert(HR_NODES <= 128, "two logical nodes per lane");
constexpr int HRMAX = 6;                   // rounds per pop (heaps below 2^36 nodes)

// node x: LDS below HTOP, else the segment in global memory.  The LDS access
// is unconditional (slot HTOP of the LDS arrays is a dummy) and the global one
// conditional: `x < HTOP ? lk[x] : K[x]` compiled to a select of the two
// pointers and one FLAT access, which costs every LDS access a flat round trip
struct HeapMem {
  uint64_t *K;
  uint32_t *T;
  uint64_t *lk;  // HTOP + 1 entries
  uint32_t *lt;
  __device__ __forceinline__ uint64_t key(uint32_t x) const {
    uint64_t v = lk[x < HTOP ? x : HTOP];
    if (x >= HTOP) v = K[x];
    return v;
  }
  __device__ __forceinline__ uint32_t tag(uint32_t x) const {
    uint32_t v = lt[x < HTOP ? x : HTOP];
    if (x >= HTOP) v = T[x];
    return v;
  }
  __device__ __forceinline__ void put(uint32_t x, uint64_t k, uint32_t t) const {
    const uint32_t y = x < HTOP ? x : HTOP;
    lk[y] = k, lt[y] = t;
    if (x >= HTOP) K[x] = k, T[x] = t;
  }
};

// __sort_heap of [0, n) by one wavefront (lane = 0..63)
__device__ void wave_sort_heap(const HeapMem &h, uint32_t n, uint32_t lane) {
  for (uint32_t last = n - 1; last > 0; --last) {
    // __pop_heap: the root moves to `last`, the value there is re-inserted
    const uint64_t vk = h.key(last);
    const uint32_t vt = h.tag(last);
    const uint64_t rk = h.key(0);
    const uint32_t rt = h.tag(0);
    if (lane == 0) h.put(last, rk, rt);
    const uint32_t len = last;
    const uint32_t two_lim = (len - 1) / 2;  // hole x has two children iff x < two_lim
    // descent rounds: per round, the path's nodes among the loaded ones
    uint64_t pm0[HRMAX], pm1[HRMAX];  // path masks: logical node c in round r (c < 64 / >= 64)
    uint64_t k0[HRMAX], k1[HRMAX];    // keys of this lane's two logical nodes
    uint32_t t0[HRMAX], t1[HRMAX];
    uint32_t x0[HRMAX], x1[HRMAX];    // their heap positions
    uint32_t hole = 0;
    int rounds = 0;
    bool more = true;
#pragma unroll
    for (int r = 0; r < HRMAX; ++r) {
      pm0[r] = pm1[r] = 0;
      k0[r] = k1[r] = 0;
      t0[r] = t1[r] = 0;
      x0[r] = x1[r] = 0;
      if (!more) continue;
      ++rounds;
      // logical node c (0..125): depth d = log2(c + 2) below the hole, offset
      // o = c + 2 - 2^d: heap position (hole + 1) 2^d - 1 + o
      uint64_t kk[2];
      uint32_t tt[2], xx[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const uint32_t c = lane + 64 * s;
        const int d = 31 - __clz((int)(c + 2));
        const uint64_t pos = ((uint64_t)hole + 1) * (1ull << d) - 1 + (c + 2 - (1u << d));
        const bool in = c < HR_NODES && pos < len;
        xx[s] = in ? (uint32_t)pos : 0u;
        kk[s] = in ? h.key((uint32_t)pos) : 0ull;
        tt[s] = in ? h.tag((uint32_t)pos) : 0u;
      }
      // right children (odd c) against their left siblings: ties go right
      uint64_t dir[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const uint32_t lo = (uint32_t)kk[s], hi = (uint32_t)(kk[s] >> 32);
        const uint64_t sib = (uint64_t)(uint32_t)__shfl_xor((int)hi, 1) << 32 |
                             (uint32_t)__shfl_xor((int)lo, 1);
        dir[s] = __ballot((lane & 1) && !(kk[s] < sib));
      }
      // the walk (scalar): internal node J (0 = the hole, else logical node
      // J - 1) has children c = 2J, 2J + 1
      uint32_t J = 0, x = hole;
      more = false;
      for (;;) {
        if (x >= two_lim) {  // no second child: a lone left child ends the descent
          if ((len & 1) == 0 && x == (len - 2) / 2) {
            const uint32_t c = 2 * J;
            if (c < 64) pm0[r] |= 1ull << c;
            else pm1[r] |= 1ull << (c - 64);
          }
          break;
        }
        const uint32_t cr = 2 * J + 1;
        const bool right = ((cr < 64 ? dir[0] >> cr : dir[1] >> (cr - 64)) & 1ull) != 0;
        const uint32_t c = right ? cr : cr - 1;
        if (c < 64) pm0[r] |= 1ull << c;
        else pm1[r] |= 1ull << (c - 64);
        x = 2 * x + (right ? 2 : 1);
        if (c >= HR_LAST) {  // the round's last level: the next round starts below x
          hole = x;
          more = true;
          break;
        }
        J = c + 1;
      }
      k0[r] = kk[0], k1[r] = kk[1];
      t0[r] = tt[0], t1[r] = tt[1];
      x0[r] = xx[0], x1[r] = xx[1];
    }
    // __push_heap: the value rises past the path keys below it (a suffix)
    uint32_t D = 0, below = 0;
#pragma unroll
    for (int r = 0; r < HRMAX; ++r) {
      if (r >= rounds) break;
      D += __popcll(pm0[r]) + __popcll(pm1[r]);
      below += __popcll(__ballot(((pm0[r] >> lane) & 1) && k0[r] < vk)) +
               __popcll(__ballot(((pm1[r] >> lane) & 1) && k1[r] < vk));
    }
    const uint32_t j = D - below;  // the value's slot is path position j (0: the root)
    // path position p (1-based) of every path node: its key moves to its
    // parent when p <= j, and the value lands at position j
    uint32_t before = 0;
    const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int r = 0; r < HRMAX; ++r) {
      if (r >= rounds) break;
      const bool on0 = (pm0[r] >> lane) & 1, on1 = (pm1[r] >> lane) & 1;
      const uint32_t p0 = before + __popcll(pm0[r] & lt) + 1;
      const uint32_t p1 = before + __popcll(pm0[r]) + __popcll(pm1[r] & lt) + 1;
      if (on0 && p0 <= j) {
        h.put((x0[r] - 1) / 2, k0[r], t0[r]);
        if (p0 == j) h.put(x0[r], vk, vt);
      }
      if (on1 && p1 <= j) {
        h.put((x1[r] - 1) / 2, k1[r], t1[r]);
        if (p1 == j) h.put(x1[r], vk, vt);
      }
      before += __popcll(pm0[r]) + __popcll(pm1[r]);
    }
    if (j == 0 && lane == 0) h.put(0, vk, vt);
    // the next pop reads what this one wrote: one wavefront's LDS and global
    // accesses are performed in order, so a wavefront-scope fence (no wait
    // for the stores' completion) keeps the compiler from reordering them
    wave_sync();
  }
}

// __sort_heap of [0, n) when every key is equal -- the heap segment of a
// median-of-three killer is exactly that: the adversary leaves the members it
// never separated for the fallback.  No comparison is then true, so every
// pop's descent is the right spine 0, 2, 6, .., 2^(j+1) - 2 while the hole has
// two children (then the lone left child, `len` - 1, under the even-length
// rule) and the displaced value stays where the descent ends: the descent's
// slots shift up by one, the root leaves to `last`.  Spine slot j lives in
// lane j; the descent's slots 0..m form a ring from lane `head` (re-linearised
// by one shuffle when m shrinks, ~lg n times), so a pop is two lane reads and
// two lane selects.  Every other position is read once, in descending order,
// from two prefetched 64-position chunks.  Tags only: the keys are all equal.
__device__ void wave_sort_heap_equal(uint32_t *T, uint32_t n, uint32_t lane) {
  auto sp = [](uint32_t j) { return (2ull << j) - 2; };
  uint32_t s = lane < 32 && sp(lane) < n ? T[sp(lane)] : 0u;
  uint32_t L = n - 1, m = 0;
  while (sp(m) < (L - 1) / 2) ++m;
  uint32_t head = 0, pv = 0;
  bool pend = false;  // the previous pop left its value at position L
  // chunk [B - 63, B] holds L: the chunk's positions are in one register
  // (position B - lane), the next two chunks' in two more, and the pops'
  // outputs gather in ob (position B - lane), stored once per chunk -- a store
  // per pop would make every lane read wait for it.  The three registers take
  // turns (the loop below is unrolled by three), so a chunk's load lands in
  // its own register a whole chunk of pops before it is read
  int64_t B = L;
  auto ld = [&](int64_t q) { return T[q >= 0 ? q : 0]; };  // below 0: never read
  uint32_t ca = ld(B - lane), cb = ld(B - 64 - lane), cc = ld(B - 128 - lane), ob = 0;
  // the spine arrives before the loop: left pending, every lane read of it in
  // the loop would wait for all memory accesses in flight (the chunks' too)
  __builtin_amdgcn_s_waitcnt(0);
  auto chunk = [&](const uint32_t c0, const uint32_t c1) {  // pops L = B .. B - 63
    auto at = [&](int64_t q) {
      const int i = (int)(B - q);
      return (uint32_t)(i < 64 ? __builtin_amdgcn_readlane((int)c0, i)
                               : __builtin_amdgcn_readlane((int)c1, i - 64));
    };
    // A chunk with no event -- no shrink of the descent, no even-length rule,
    // no spine slot among its positions, no value left by the previous pop --
    // is a FIFO of delay m + 1: pop i outputs ring slot i (i <= m), else the
    // value pop i - m - 1 re-inserted (chunk lane i - m - 1), and leaves the
    // chunk's last m + 1 values as the ring.  Events come only near L = 2^k - 2
    // (a few chunks per heap level); the other chunks take three shuffles.
    const int64_t lo = B - 63;
    const int64_t shrink_at = m > 0 ? (int64_t)(2 * sp(m - 1) + 2) : -1;
    const int64_t special_at = (int64_t)(2 * sp(m) + 2);
    const int kb = 31 - __clz((int)(B + 2));
    const bool spine_in = ((1ll << kb) - 2) >= lo;
    if (lo >= 1 && !pend && shrink_at < lo && !(special_at >= lo && special_at <= B) && !spine_in) {
      const uint32_t mp1 = m + 1, hl = head + lane;
      const uint32_t from_s = (uint32_t)__shfl((int)s, (int)(hl < mp1 ? hl : hl - mp1));
      const uint32_t from_c = (uint32_t)__shfl((int)c0, (int)(lane - mp1) & 63);
      const uint32_t ring = (uint32_t)__shfl((int)c0, (int)(64 - mp1 + lane) & 63);
      ob = lane < mp1 ? from_s : from_c;
      s = lane < mp1 ? ring : s;
      head = 0;
      L -= 64;
    }
    for (; L > 0 && B - L < 64; --L) {
      while (m > 0 && sp(m - 1) >= (L - 1) / 2) {
        s = (uint32_t)__shfl((int)s, lane <= m ? (int)((head + lane) % (m + 1)) : (int)lane);
        head = 0;
        --m;
      }
      uint32_t v;
      if (pend) v = pv;
      else if (((L + 2) & (L + 1)) == 0)  // a spine slot below the descent
        v = (uint32_t)__builtin_amdgcn_readlane((int)s, 30 - __clz((int)(L + 2)));
      else v = at(L);
      const uint32_t root = (uint32_t)__builtin_amdgcn_readlane((int)s, (int)head);
      ob = lane == (uint32_t)(B - L) ? root : ob;
      const bool special = (L & 1) == 0 && sp(m) == (L - 2) / 2;
      const uint32_t bottom = special ? at(L - 1) : v;
      s = lane == head ? bottom : s;
      head = head == m ? 0 : head + 1;
      pend = special;
      pv = v;
    }
    if ((int64_t)lane < B - L) T[B - lane] = ob;  // positions B .. L + 1
    B -= 64;
  };
  for (;;) {
    chunk(ca, cb);
    if (L == 0) break;
    ca = ld(B - 128 - lane);
    chunk(cb, cc);
    if (L == 0) break;
    cb = ld(B - 128 - lane);
    chunk(cc, ca);
    if (L == 0) break;
    cc = ld(B - 128 - lane);
  }
  if (lane == 0) T[0] = (uint32_t)__builtin_amdgcn_readlane((int)s, (int)head);
}

// __make_heap of [0, n) of K/T (global memory) by one block: the calls of
// one heap level touch disjoint subtrees, deeper levels first
__device__ void block_make_heap(uint64_t *K, uint32_t *T, uint32_t n) {
  const uint32_t tid = threadIdx.x;
  if (n < 2) return;
  const uint32_t last_parent = (n - 2) / 2;
  for (int lv = 31 - __clz((int)(last_parent + 1)); lv >= 0; --lv) {
    const uint32_t a = (1u << lv) - 1;
    const uint32_t e = min((1u << (lv + 1)) - 2, last_parent);
    for (uint32_t x = a + tid; x <= e; x += blockDim.x)
      adjust_heap(GView{K, T, nullptr, nullptr, nullptr}, 0, x, n, K[x], T[x]);
    __syncthreads();
  }
}

// The whole __partial_sort of segment [0, n) of K/T (global memory) by one
// 256-thread block; its final tags go to out[0..n).
__device__ void block_heap_sort(uint64_t *K, uint32_t *T, uint32_t n, uint32_t *out, uint64_t *lk,
                                uint32_t *lt) {
  const uint32_t tid = threadIdx.x;
  if (n < 2) {
    for (uint32_t x = tid; x < n; x += blockDim.x) out[x] = T[x];
    __syncthreads();
    return;
  }
  int neq = 0;
  for (uint32_t x = tid; x < n; x += blockDim.x) neq |= K[x] != K[0];
  const bool equal = __syncthreads_or(neq) == 0;
  {
    block_make_heap(K, T, n);
    if (equal) {
      if (tid < 64) wave_sort_heap_equal(T, n, tid);
      __syncthreads();
      for (uint32_t x = tid; x < n; x += blockDim.x) out[x] = T[x];
      __syncthreads();
      return;
    }
    for (uint32_t x = tid; x < n && x < HTOP; x += blockDim.x) lk[x] = K[x], lt[x] = T[x];
    __syncthreads();
    if (tid < 64) wave_sort_heap(HeapMem{K, T, lk, lt}, n, tid);
    __syncthreads();
  }
  for (uint32_t x = tid; x < n; x += blockDim.x) out[x] = x < HTOP ? lt[x] : T[x];
  __syncthreads();
}

// cross-lane moves: pull from lane `src` (ds_bpermute) / push to lane `dst`
// (ds_permute; the destinations must form a permutation)
__device__ __forceinline__ uint32_t pull(int src, uint32_t v) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)v);
}
__device__ __forceinline__ uint64_t pull(int src, uint64_t v) {
  return (uint64_t)pull(src, (uint32_t)v) | (uint64_t)pull(src, (uint32_t)(v >> 32)) << 32;
}
__device__ __forceinline__ uint32_t push(int dst, uint32_t v) {
  return (uint32_t)__builtin_amdgcn_ds_permute(dst << 2, (int)v);
}
// popcount of the bits of m below this lane
__device__ __forceinline__ int below_count(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                        __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// __introsort_loop on segments of at most 64 elements, in registers (lane x
// holds one element).  Partitions of disjoint sub-segments are independent,
// so every sub-segment of one recursion level is partitioned at once (each
// keeps its own depth budget, as in the sequential recursion); each Hoare
// partition is the stopper matching of wave_partition done with ballots and
// lane permutes.  With L_k / R_k the k-th L-stopper from the left / R-stopper
// from the right of a segment:
//   * L_k < R_k  <=>  more than k R-stoppers lie above L_k, so the swap count
//     K is the rank of the first L-stopper without that property;
//   * the swap partners come from two compacted lists (lane j of LL / RL holds
//     the j-th L- / R-stopper of the whole wave; a segment's stoppers are a
//     contiguous slice of them), built with one ds_permute each;
//   * the cut min(R_{K-1}, L_K) (L_0 when K == 0) is the lowest lane that is
//     one of those two, one ballot.
// Each lane ends with its final segment [sf, sl) (lane indices) -- a leaf, or
// a heap-sorted range when `heaped`: a depth-exhausted sub-segment is written
// to memory (lane x at mpos), heap-sorted there by its first lane and read
// back.
template <bool GLOBAL, class KT, class V>
__device__ void reg_sort_core(const V &v, bool in, uint32_t mpos, int &sf, int &sl, int sd,
                              uint32_t lane, KT &k, uint32_t &t, bool &heaped) {
  const int x = (int)lane;
  heaped = false;
  for (;;) {
    bool active = in && !heaped && sl - sf > THRESH;
    const bool need_heap = active && sd == 0;
    if (__ballot(need_heap)) {  // rare: heap fallback in memory
      if (in) v.K[mpos] = (typename V::key_t)k, v.T[mpos] = t;
      sync_mem<GLOBAL>();
      if (need_heap && x == sf) heap_sort_segment(v, mpos, mpos + (sl - sf));
      sync_mem<GLOBAL>();
      if (in) k = (KT)v.K[mpos], t = v.T[mpos];
      heaped |= need_heap;
      active &= !need_heap;
    }
    if (!__ballot(active)) break;
    const int len = sl - sf;
    // __move_median_to_first(f, f+1, mid, l-1)
    const int a = active ? sf + 1 : x, b = active ? sf + len / 2 : x, c = active ? sl - 1 : x;
    const KT ka = pull(a, k), kb = pull(b, k), kc = pull(c, k);
    int med;
    if (ka < kb) med = kb < kc ? b : (ka < kc ? c : a);
    else med = ka < kc ? a : (kb < kc ? c : b);
    int src = x;
    if (active) src = x == sf ? med : (x == med ? sf : x);
    k = pull(src, k);
    t = pull(src, t);
    const KT p = pull(active ? sf : x, k);
    // stoppers of __unguarded_partition(f+1, l, f)
    const uint64_t segm = (sl >= 64 ? ~0ull : (1ull << sl) - 1ull) & ~((1ull << sf) - 1ull);
    const bool lf = active && x > sf && !(k < p);
    const bool rf = active && !(p < k);
    const uint64_t BL = __ballot(lf), BR = __ballot(rf);
    const uint64_t Ls = BL & segm, Rs = BR & segm;
    const int nL = __popcll(Ls), nR = __popcll(Rs);
    const int pL = below_count(BL), pR = below_count(BR);
    const uint64_t lowseg = (1ull << sf) - 1ull;
    const int offL = __popcll(BL & lowseg), offR = __popcll(BR & lowseg);
    const int rl = pL - offL;                          // rank from the left (L lanes)
    const int rr = nR - 1 - (pR - offR);               // rank from the right (R lanes)
    const int rabove = nR - (pR - offR) - (rf ? 1 : 0);  // R-stoppers above this lane
    const uint64_t stopm = __ballot(lf && rabove <= rl) & segm;
    const int lim = nL < nR ? nL : nR;
    const int K = stopm ? __popcll(Ls & ((1ull << __builtin_ctzll(stopm)) - 1ull)) : lim;
    // compacted stopper lists (stable partition of the lanes, one push each)
    const int nBL = __popcll(BL), nBR = __popcll(BR);
    const uint32_t LL = push(lf ? pL : nBL + (x - pL), (uint32_t)x);
    const uint32_t RL = push(rf ? pR : nBR + (x - pR), (uint32_t)x);
    const bool swl = lf && rl < K, swr = rf && rr < K;
    const int idx = swl ? offR + nR - 1 - rl : swr ? offL + rr : x;
    const uint32_t g = pull(idx, LL | RL << 8);
    const int s2 = swl ? (int)(g >> 8) : swr ? (int)(g & 0xff) : x;
    k = pull(s2, k);
    t = pull(s2, t);
    const uint64_t cm = __ballot((lf && rl == K) || (K > 0 && rf && rr == K - 1)) & segm;
    if (active) {
      const int cut = __builtin_ctzll(cm);
      if (x < cut) sl = cut;
      else sf = cut;
      --sd;
    }
  }
}

// Lane x of a batch holds one element of one of up to three small segments
// packed side by side (segment j in lanes [bl, bl + len), memory [bm, bm +
// len), depth budget d).  Keys below 2^32 in the whole batch run the core on
// 32-bit registers (half the shuffle traffic).  The final order -- stable
// leaf ranks, or heap-sorted ranges in place -- is written to out[] and the
// positions are marked B = 3.
template <bool GLOBAL, class KT, class V>
__device__ void reg_finish(const V &v, bool in, int bl, uint32_t bm, int len, int d,
                           uint32_t lane, uint64_t k64, uint32_t t, uint32_t *out,
                           uint32_t tbase) {
  const int x = (int)lane;
  KT k = in ? (KT)k64 : (KT)~(KT)0;
  int sf = in ? bl : x, sl = in ? bl + len : x + 1;
  bool heaped;
  const uint32_t mpos = bm + (uint32_t)(x - bl);
  reg_sort_core<GLOBAL, KT, V>(v, in, mpos, sf, sl, d, lane, k, t, heaped);
  // stable rank inside the leaf; the loop runs to the longest leaf of the wave
  uint32_t r = 0;
  const int my = in && !heaped ? sl - sf : 0;
  for (int j = 0; __ballot(j < my); ++j) {
    const int y = sf + j;
    const KT ky = pull(y < 64 ? y : 63, k);
    r += (j < my) && (ky < k || (ky == k && y < x));
  }
  if (in) {
    out[heaped ? mpos : bm + (uint32_t)(sf - bl) + r] = tbase + t;
    if (v.B) v.B[mpos] = 3;
  }
}

template <bool GLOBAL, class V>
__device__ void reg_batch(const V &v, bool in, int bl, uint32_t bm, int len, int d,
                          uint32_t lane, uint32_t *out, uint32_t tbase = 0) {
  const uint32_t mpos = bm + (uint32_t)((int)lane - bl);
  const uint64_t k = in ? (uint64_t)v.K[mpos] : ~0ull;
  // the group arrays' tags are positions (tag[x] == x, sort_groups_exact):
  // not read from memory; LDS views hold the moved tags
  const uint32_t t = in ? (GLOBAL ? mpos : v.T[mpos]) : 0u;
  if (sizeof(typename V::key_t) == 8 && __ballot(in && (k >> 32) != 0))
    reg_finish<GLOBAL, uint64_t, V>(v, in, bl, bm, len, d, lane, k, t, out, tbase);
  else
    reg_finish<GLOBAL, uint32_t, V>(v, in, bl, bm, len, d, lane, k, t, out, tbase);
}

// The lanes that sort one group: the whole wavefront (W = 64), or one half of
// it (W = 32: two groups per wavefront, each half with its own LDS slab and
// stack).  Halves diverge freely -- a ballot sees only the lanes still running
// that code -- so every mask is shifted down to the half's own lanes.  With
// two groups per instruction stream the fixed part of every partition (the
// median by one lane, the stopper search, the cut, the stack) and the
// segments of <= 32 members cost half the issue slots per group.
template <int W>
struct GLanes {
  uint32_t lane;  // [0, W)
  uint32_t base;  // this group's first lane in the wavefront (0 or 32)
  __device__ __forceinline__ uint64_t ballot(bool p) const {
    return W == 64 ? (uint64_t)__ballot(p) : ((uint64_t)__ballot(p) >> base) & 0xffffffffull;
  }
  __device__ __forceinline__ uint32_t bcast(uint32_t x) const {  // from lane 0 of the group
    return (uint32_t)__shfl((int)x, (int)base);
  }
};

// wavefront-parallel __unguarded_partition_pivot on [f, l); returns the cut
template <bool GLOBAL, class V, int W>
__device__ uint32_t wave_partition(const V &v, uint32_t f, uint32_t l, GLanes<W> L) {
  const uint32_t lane = L.lane;
  // __move_median_to_first by lane 0 with every read issued up front (the
  // three candidates and the first slot, then the median's tag); the pivot
  // (the median's key) reaches the other lanes by a lane read, not from memory
  typename V::key_t p = 0;
  if (lane == 0) {
    const uint32_t a = f + 1, b = f + (l - f) / 2, c = l - 1;
    const typename V::key_t ka = v.K[a], kb = v.K[b], kc = v.K[c], kf = v.K[f];
    const uint32_t tf = v.T[f];
    uint32_t m;
    typename V::key_t km;
    if (ka < kb) {
      if (kb < kc) m = b, km = kb;
      else if (ka < kc) m = c, km = kc;
      else m = a, km = ka;
    } else {
      if (ka < kc) m = a, km = ka;
      else if (kb < kc) m = c, km = kc;
      else m = b, km = kb;
    }
    const uint32_t tm = v.T[m];
    v.K[m] = kf;
    v.T[m] = tf;
    v.K[f] = km;
    v.T[f] = tm;
    p = km;
  }
  if (sizeof(p) == 8) {
    const uint64_t p64 = (uint64_t)p;
    p = (typename V::key_t)((uint64_t)L.bcast((uint32_t)p64) |
                            (uint64_t)L.bcast((uint32_t)(p64 >> 32)) << 32);
  } else {
    p = (typename V::key_t)L.bcast((uint32_t)p);
  }
  sync_mem<GLOBAL>();
  const uint64_t lt = (1ull << lane) - 1ull;
  uint32_t nL = 0, nR = 0;
  for (uint32_t c = f; c < l; c += W) {
    const uint32_t x = c + lane;
    const bool in = x < l;
    const typename V::key_t k = in ? v.K[x] : 0;
    const bool lf = in && x > f && !(k < p);
    const bool rf = in && !(p < k);
    const uint64_t bl = L.ballot(lf), br = L.ballot(rf);
    if (lf) v.PL[nL + __popcll(bl & lt)] = x;
    if (rf) v.PR[nR + __popcll(br & lt)] = x;
    nL += __popcll(bl);
    nR += __popcll(br);
  }
  sync_mem<GLOBAL>();
  // K = first k with Lpos[k] >= Rpos[k]; Rpos[k] = PR[nR-1-k] (k-th from the right)
  const uint32_t lim = nL < nR ? nL : nR;
  uint32_t K = lim;
  for (uint32_t c = 0; c < lim; c += W) {
    const uint32_t k = c + lane;
    const bool stop = k < lim && v.PL[k] >= v.PR[nR - 1 - k];
    const uint64_t b = L.ballot(stop);
    if (b) {
      K = c + (uint32_t)__ffsll((unsigned long long)b) - 1;
      break;
    }
  }
  for (uint32_t c = 0; c < K; c += W) {
    const uint32_t k = c + lane;
    if (k < K) vswap(v, v.PL[k], v.PR[nR - 1 - k]);
  }
  uint32_t cut;
  if (K == 0) {
    cut = v.PL[0];
  } else {
    cut = v.PR[nR - K];
    if (K < nL && v.PL[K] < cut) cut = v.PL[K];
  }
  sync_mem<GLOBAL>();
  return cut;
}

template <class KT>
__device__ __forceinline__ KT lane_key(KT k, uint32_t src) {  // (src wave-uniform)
  if (sizeof(KT) == 8) {
    const uint64_t v = (uint64_t)k;
    return (KT)((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)src) |
                (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)src)
                    << 32);
  }
  return (KT)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)k, (int)src);
}

// wave_partition on a segment of 17..64 elements, one per lane, in registers:
// the keys and tags are read once, the median moves by lane reads, the
// stoppers are two ballots, K is the rank of the first L-stopper with at most
// its rank of R-stoppers above it (wave_partition's stop test), the partners
// come from two lists compacted by lane permutes (reg_sort_core's form), and
// every element is written once at its slot -- two memory round trips where
// the list form (stopper lists written, read by the search, read again by the
// swaps, keys and tags read and written per swap, the cut read) takes ten.
template <bool GLOBAL, class V>
__device__ uint32_t wave_partition_small(const V &v, uint32_t f, uint32_t l, uint32_t lane) {
  using KT = typename V::key_t;
  const uint32_t len = l - f;
  const bool in = lane < len;
  const uint32_t x = f + (in ? lane : 0u);
  KT k = v.K[x];  // (lanes past the segment hold a copy of its first element, unused)
  uint32_t t = v.T[x];
  // __move_median_to_first(f, f + 1, f + len / 2, l - 1)
  const uint32_t la = 1, lb = len / 2, lc = len - 1;
  const KT ka = lane_key(k, la), kb = lane_key(k, lb), kc = lane_key(k, lc);
  uint32_t mi;
  if (ka < kb) mi = kb < kc ? lb : (ka < kc ? lc : la);
  else mi = ka < kc ? la : (kb < kc ? lc : lb);
  mi = (uint32_t)__builtin_amdgcn_readfirstlane((int)mi);
  const KT k0 = lane_key(k, 0u), p = lane_key(k, mi);
  const uint32_t t0 = (uint32_t)__builtin_amdgcn_readlane((int)t, 0),
                 tm = (uint32_t)__builtin_amdgcn_readlane((int)t, (int)mi);
  if (lane == 0) k = p, t = tm;
  else if (lane == mi) k = k0, t = t0;
  // stoppers of __unguarded_partition(f + 1, l, f)
  const bool lf = in && lane > 0 && !(k < p);
  const bool rf = in && !(p < k);
  const uint64_t BL = __ballot(lf), BR = __ballot(rf);
  const uint32_t nL = (uint32_t)__popcll(BL), nR = (uint32_t)__popcll(BR);
  const uint32_t pL = (uint32_t)below_count(BL), pR = (uint32_t)below_count(BR);
  const uint32_t ra = nR - pR - (rf ? 1u : 0u);  // R-stoppers above: its rank from the right
  const uint64_t SB = __ballot(lf && ra <= pL);
  const uint32_t lim = nL < nR ? nL : nR;
  const uint32_t K =
      SB ? (uint32_t)__popcll(BL & ((1ull << __builtin_ctzll(SB)) - 1ull)) : lim;
  // compacted stopper lists (lane j: the j-th L- / R-stopper), one permute each;
  // the k-th L-stopper and the k-th R-stopper from the right trade places, k < K
  const uint32_t LL = push((int)(lf ? pL : nL + (lane - pL)), lane);
  const uint32_t RL = push((int)(rf ? pR : nR + (lane - pR)), lane);
  const bool swl = lf && pL < K, swr = rf && ra < K;
  const uint32_t g = pull((int)(swl ? nR - 1u - pL : swr ? ra : lane), LL | RL << 8);
  const uint32_t src = swl ? g >> 8 : swr ? g & 0xffu : lane;
  k = pull((int)src, k);
  t = pull((int)src, t);
  if (in) {
    v.K[x] = k;
    v.T[x] = (typename V::tag_t)t;
  }
  // the cut min(L_K, R_{K-1}) (L_0 when K == 0): the lowest lane that is either
  const uint64_t cm = __ballot((lf && pL == K) || (K > 0 && rf && ra == K - 1u));
  const uint32_t cut = f + (uint32_t)__builtin_ctzll(cm);
  sync_mem<GLOBAL>();
  return cut;
}

struct Frame {
  uint32_t f, l;
  int d;
};

#ifdef RK_GS_PROF
// measurement build only: shader cycles per phase of the LDS tiers' sort
__device__ unsigned long long g_gs_prof[8];
#define GS_T(k) const uint64_t _g##k = __builtin_amdgcn_s_memtime()
#define GS_ADD(slot, v) do { if (lane == 0) atomicAdd(&g_gs_prof[slot], (unsigned long long)(v)); } while (0)
#else
#define GS_T(k)
#define GS_ADD(slot, v)
#endif

// the whole libstdc++ std::sort of one group [0, n) of view v, then stable
// leaf ranks written to out[0..n) (tags only)
template <bool GLOBAL, class V, int W = 64>
__device__ void wave_std_sort(const V &v, uint32_t n, uint32_t *out, Frame *stack,
                              Frame *smallq, Frame *heapq, GLanes<W> L, int d0,
                              uint32_t reg_max, uint32_t tbase = 0, bool small_part = true) {
  static_assert(W == 64 || W == 32, "a wavefront or a half");
  const uint32_t lane = L.lane;
  if (W != 64) reg_max = 0;  // register batches assume the whole wavefront
  GS_T(0);
#ifdef RK_GS_PROF
  uint64_t part_cyc = 0, nparts = 0;
#endif
  for (uint32_t x = lane; x < n; x += W) v.B[x] = 0;
  int sp = 0, nsmall = 0, nheap = 0;
  if (lane == 0) stack[0] = {0u, n, d0};
  sp = 1;
  sync_mem<GLOBAL>();
  while (sp) {
    Frame fr = stack[--sp];
    uint32_t f = fr.f, l = fr.l;
    int d = fr.d;
    bool final_leaf = true;
    while (l - f > THRESH) {
      if (d == 0) {  // heapsort fallback, done lane-parallel below
        if (lane == 0) heapq[nheap] = {f, l, 0};
        ++nheap;
        final_leaf = false;
        break;
      }
      if (l - f <= reg_max) {  // small: finished in registers (reg_batch)
        if (lane == 0) smallq[nsmall] = {f, l, d};
        ++nsmall;
        final_leaf = false;
        break;
      }
      --d;
#ifdef RK_GS_PROF
      const uint64_t _p0 = __builtin_amdgcn_s_memtime();
#endif
      // (segments of <= 64 in registers, RK_GS_SMALLPART=0: the list form)
      const uint32_t cut = W == 64 && small_part && l - f <= 64
                               ? wave_partition_small<GLOBAL, V>(v, f, l, lane)
                               : wave_partition<GLOBAL, V, W>(v, f, l, L);
#ifdef RK_GS_PROF
      part_cyc += __builtin_amdgcn_s_memtime() - _p0;
      ++nparts;
#endif
      if (lane == 0) stack[sp] = {cut, l, d};
      ++sp;
      l = cut;
    }
    if (final_leaf && lane == 0) v.B[f] = 1;
    sync_mem<GLOBAL>();
  }
  GS_T(1);
#ifdef RK_GS_PROF
  uint64_t nbatch = 0;
#endif
  // small segments, packed up to three per 64-lane batch
  for (int q0 = 0; W == 64 && q0 < nsmall;) {
#ifdef RK_GS_PROF
    ++nbatch;
#endif
    int tot = 0, q1 = q0;
    while (q1 < nsmall && tot + (int)(smallq[q1].l - smallq[q1].f) <= 64)
      tot += (int)(smallq[q1].l - smallq[q1].f), ++q1;
    int bl = 0, j = q0;
    while (j + 1 < q1 && (int)lane >= bl + (int)(smallq[j].l - smallq[j].f))
      bl += (int)(smallq[j].l - smallq[j].f), ++j;
    const Frame fr = smallq[j];
    reg_batch<GLOBAL, V>(v, (int)lane < tot, bl, fr.f, (int)(fr.l - fr.f), fr.d, lane, out,
                         tbase);
    q0 = q1;
  }
  sync_mem<GLOBAL>();
  GS_T(2);
  for (int q = (int)lane; q < nheap; q += W) heap_sort_segment(v, heapq[q].f, heapq[q].l);
  sync_mem<GLOBAL>();
  // __final_insertion_sort == stable sort inside every leaf (segments
  // finished in registers are already written, B == 3).  A leaf is a B == 1
  // start followed by B == 0 positions (at most 16); its bounds come from one
  // ballot over this chunk's B and one over the next chunk's, and the rank
  // reads are independent (one LDS round trip).
  uint32_t carry = 0;  // start of the leaf still open at the end of the previous chunk
  for (uint32_t c = 0; c < n; c += W) {
    const uint32_t x = c + lane;
    const uint8_t b = x < n ? v.B[x] : 1;
    const uint8_t bn = x + W < n ? v.B[x + W] : 1;
    const uint64_t bd = L.ballot(b != 0), bdn = L.ballot(bn != 0);
    const uint64_t upto = lane == 63 ? ~0ull : (2ull << lane) - 1ull;
    const uint64_t le = bd & upto, gt = bd & ~upto;
    const uint32_t s = le ? c + 63 - (uint32_t)__clzll(le) : carry;
    const uint32_t e = gt ? c + (uint32_t)__builtin_ctzll(gt)
                          : bdn ? c + W + (uint32_t)__builtin_ctzll(bdn) : c + 2 * W;
    if (bd) carry = c + 63 - (uint32_t)__clzll(bd);
    if (x < n && b != 3) {
      if (b == 2) {
        out[x] = tbase + v.T[x];
      } else {
        const typename V::key_t kx = v.K[x];
        uint32_t r = 0;
        typename V::key_t ky[THRESH];
#pragma unroll
        for (int j = 0; j < THRESH; ++j) ky[j] = v.K[s + j < e ? s + j : x];
        // the rank terms as bitwise ands: the short-circuit form compiled to a
        // branch per term (group-sort phase 1.19 -> 1.18 ms at cfg3)
#pragma unroll
        for (int j = 0; j < THRESH; ++j)
          r += (uint32_t)(s + j < e) &
               ((uint32_t)(ky[j] < kx) | ((uint32_t)(ky[j] == kx) & (uint32_t)(s + j < x)));
        out[s + r] = tbase + v.T[x];
      }
    }
  }
#ifdef RK_GS_PROF
  GS_T(3);
  if (!GLOBAL) {
    GS_ADD(0, _g1 - _g0 - part_cyc);  // init + stack walk outside the partitions
    GS_ADD(1, part_cyc);
    GS_ADD(2, _g2 - _g1);             // register batches
    GS_ADD(3, _g3 - _g2);             // heap + final insertion pass
    GS_ADD(4, nparts);
    GS_ADD(5, nbatch);
    GS_ADD(6, 1);
    GS_ADD(7, n);
  }
#endif
}

// The listed tiers' groups, tier-major in one array: tier u (1..6) owns
// list[off[(u-1)*nblk] .. off[u*nblk]) (off = exclusive scan of per-block
// tier counts, see k_tier_lists).  Kernels read their range on the device, so
// no host round trip sizes the launches.
struct TierLists {
  const uint32_t *list, *off;
  uint32_t nblk;
  __device__ __forceinline__ void range(int u, uint32_t &lo, uint32_t &hi) const {
    lo = off[(size_t)u * nblk];
    hi = off[(size_t)(u + 1) * nblk];
  }
};

// Register tiers: groups of 17..64 members in registers, no LDS -- PACK
// groups per wavefront (lanes [64/PACK * j, 64/PACK * (j+1)) hold group j of
// the wave's PACK consecutive list entries; reg_sort_core keeps every lane's
// own segment, so the groups never mix).  The introsort runs there and
// __final_insertion_sort is the stable rank inside each leaf (<= 16 lanes,
// by shuffles); heap-sorted ranges are already in order.
template <int PACK>
__global__ void __launch_bounds__(256) k_sort_groups_reg(TierLists tl, int tier,
                                                         const uint32_t *goff, uint64_t *key,
                                                         uint32_t *tag, uint32_t *otag) {
  constexpr int SPAN = 64 / PACK;
  const uint32_t lane = threadIdx.x & 63;
  const int j = (int)lane / SPAN;
  uint32_t lo, hi;
  tl.range(tier, lo, hi);
  const GView v{key, tag, nullptr, nullptr, nullptr};
  for (uint32_t w = lo + ((blockIdx.x * blockDim.x + threadIdx.x) >> 6) * PACK; w < hi;
       w += ((gridDim.x * blockDim.x) >> 6) * PACK) {
    const bool has = w + j < hi;
    const uint32_t g = has ? tl.list[w + j] : 0u;
    const uint32_t b = has ? goff[g] : 0u, n = has ? goff[g + 1] - b : 0u;
    const int bl = j * SPAN;
    reg_batch<true, GView>(v, (int)lane - bl < (int)n, bl, b, (int)n,
                           n ? 2 * (31 - __clz((int)n)) : 0, lane, otag);
  }
}

// LDS tier: one wavefront (block of 64) per group of up to `cap` members,
// staged in LDS with KT keys and 16-bit positions.  The explicit stack holds
// at most one frame per partition level: 2 * log2(cap) + 2.
__host__ __device__ constexpr uint32_t lds_stack(uint32_t cap) {
  return 2 * (31 - __builtin_clz(cap)) + 4;
}
// WPB independent wavefronts per block, each with its own LDS slab of `slab`
// bytes (a CU holds a bounded number of blocks, so one-wave blocks of the
// small caps leave it with few resident wavefronts)
// (W = 32: each half of a wavefront sorts its own group in its own slab)
template <class KT, int WPB, int W = 64>
__global__ void __launch_bounds__(64 * WPB)
__attribute__((amdgpu_waves_per_eu(W == 32 && sizeof(KT) == 4 ? 8 : 1))) k_sort_groups_lds(TierLists tl, int tier,
                                                              const uint32_t *goff,
                                                              const uint64_t *key,
                                                              const uint32_t *tag, uint32_t *otag,
                                                              uint32_t cap, uint32_t reg_max,
                                                              uint32_t slab, bool small_part) {
  extern __shared__ __align__(16) uint8_t smem_all[];
  constexpr uint32_t GPW = 64 / W;  // groups per wavefront
  // the wavefront index in a scalar register: every LDS base stays uniform
  // (per half when W = 32)
  const uint32_t wl = threadIdx.x & 63,
                 wv = WPB == 1 ? 0u : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t half = W == 64 ? 0u : wl / W;
  const GLanes<W> L{wl & (W - 1), half * W};
  const uint32_t lane = L.lane;
  uint8_t *smem = smem_all + ((size_t)wv * GPW + half) * slab;
  const uint32_t nfr = cap / (THRESH + 1) + 2;
  KT *K = reinterpret_cast<KT *>(smem);
  uint16_t *T = reinterpret_cast<uint16_t *>(K + cap);  // tags: positions in the group
  Frame *stack = reinterpret_cast<Frame *>(T + cap);
  Frame *smallq = stack + lds_stack(cap);
  Frame *heapq = reg_max ? smallq + nfr : smallq;  // (no register batches: no queue for them)
  uint16_t *PL = reinterpret_cast<uint16_t *>(heapq + nfr);
  uint16_t *PR = PL + cap;
  uint8_t *B = reinterpret_cast<uint8_t *>(PR + cap);
  const ViewT<KT, uint16_t, uint16_t> v{K, T, PL, PR, B};
  uint32_t lo, hi;
  tl.range(tier, lo, hi);
  for (uint32_t w = lo + (blockIdx.x * WPB + wv) * GPW + half; w < hi;
       w += gridDim.x * WPB * GPW) {
    const uint32_t g = tl.list[w];
    const uint32_t b = goff[g], n = goff[g + 1] - b;
    for (uint32_t x = lane; x < n; x += W) {
      K[x] = (KT)key[b + x];
      T[x] = (uint16_t)x;  // tags are positions (the output adds b)
    }
    wave_sync();
    wave_std_sort<false, ViewT<KT, uint16_t, uint16_t>, W>(v, n, otag + b, stack, smallq, heapq,
                                                           L, 2 * (31 - __clz((int)n)), reg_max,
                                                           b, small_part);
    wave_sync();
  }
}

// Groups above the largest LDS cap (repeat families: 10^4 - 10^6 members)
// run in two phases.
//
// Phase A, one 256-thread block per group: the introsort loop on the group's
// slice of global memory, but only segments of more than SPLIT_T members are
// partitioned here, each by the whole block -- stopper lists from one
// ballot pass (each wave compacts its quarter's stoppers into that quarter's
// slice; the k-th stopper is found through the four counts), K by a 256-ary
// search (the stop predicate Lpos[k] >= Rpos[k] is
// monotone in k), the K swaps in parallel.  A segment that reaches SPLIT_T
// members or less is final for this phase: its start gets bnd = 1 and
// head = length | depth << 16.  (A segment above SPLIT_T whose depth budget
// is spent is heap-sorted here by one thread -- libstdc++'s own fallback --
// and written out directly.)  Stopper lists of a segment [f, l) live in
// pl/pr[f, l), so final segments' heads are never overwritten.
//
// Phase B, one wavefront per final segment (found by scanning bnd over 64
// positions per step): the LDS introsort of the other tiers, started with the
// segment's remaining depth budget, writing the segment's final order.
// Together the two phases are the libstdc++ recursion exactly: sibling
// segments are independent, and every segment keeps its own depth budget.
#ifndef RK_SPLIT_T
#define RK_SPLIT_T 512
#endif
constexpr uint32_t SPLIT_T = RK_SPLIT_T;
constexpr int SPLIT_STACK = 72;  // one frame per level: 2 * log2(2^32) + slack

// One pass over the segment: each wave compacts the stoppers of its quarter
// into that quarter's own slice of PL / PR (a quarter holds at most as many
// stoppers as positions), and the k-th stopper of the whole segment is found
// through the four waves' counts -- the same lists as a counting pass followed
// by ranked writes, without reading the keys twice.
struct StopperMap {
  uint32_t off[5];  // stoppers before wave w's slice (off[4] = total)
  uint32_t at[4];   // wave w's slice start
  __device__ __forceinline__ uint32_t pos(const uint32_t *P, uint32_t k) const {
    const uint32_t w = (k >= off[1]) + (k >= off[2]) + (k >= off[3]);
    return P[at[w] + (k - off[w])];
  }
};

__device__ uint32_t block_partition(uint64_t *K, uint32_t *T, uint32_t *PL, uint32_t *PR,
                                    uint32_t f, uint32_t l, uint32_t *s_w) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) median_to_first(GView{K, T, nullptr, nullptr, nullptr}, f, l);
  __syncthreads();
  const uint64_t p = K[f];
  const uint32_t len = l - f;
  const uint32_t per = ((len + 3) / 4 + 255) & ~255u;  // a wave's share, 4 x 64 aligned
  const uint32_t a = f + wv * per < l ? f + wv * per : l;
  const uint32_t e = a + per < l ? a + per : l;
  const uint64_t lt = (1ull << lane) - 1ull;
  // the wave's stoppers, compacted into PL / PR [a, a + count)
  uint32_t cl = 0, cr = 0;
  for (uint32_t c = a; c < e; c += 256) {
    uint64_t k[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t x = c + 64 * u + lane;
      k[u] = x < e ? K[x] : 0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t x = c + 64 * u + lane;
      const bool lf = x < e && x > f && !(k[u] < p);
      const bool rf = x < e && !(p < k[u]);
      const uint64_t bl = __ballot(lf), br = __ballot(rf);
      if (lf) PL[a + cl + __popcll(bl & lt)] = x;
      if (rf) PR[a + cr + __popcll(br & lt)] = x;
      cl += __popcll(bl);
      cr += __popcll(br);
    }
  }
  if (lane == 0) s_w[wv] = cl, s_w[4 + wv] = cr;
  __syncthreads();
  StopperMap ML, MR;
  ML.off[0] = MR.off[0] = 0;
#pragma unroll
  for (uint32_t u = 0; u < 4; ++u) {
    ML.off[u + 1] = ML.off[u] + s_w[u];
    MR.off[u + 1] = MR.off[u] + s_w[4 + u];
    const uint32_t au = f + u * per;
    ML.at[u] = MR.at[u] = au < l ? au : l;
  }
  const uint32_t nL = ML.off[4], nR = MR.off[4];
  // K = first k < lim with PL[k] >= PR[nR-1-k] (lim if none), 256 probes a round
  const uint32_t lim = nL < nR ? nL : nR;
  uint32_t lo = 0, hi = lim;  // K in [lo, hi]
  while (lo < hi) {
    const uint32_t span = hi - lo;
    const uint32_t k = lo + (uint32_t)(((uint64_t)span * tid) / 256);
    const bool probe = tid == 0 || k != lo + (uint32_t)(((uint64_t)span * (tid - 1)) / 256);
    const bool stop = probe && ML.pos(PL, k) >= MR.pos(PR, nR - 1 - k);
    if (tid == 0) s_w[8] = 0xFFFFFFFFu;
    __syncthreads();
    if (stop) atomicMin(&s_w[8], k);
    __syncthreads();
    const uint32_t first = s_w[8];
    // the largest probed k below `first` (or below hi) is known false
    uint32_t nlo = lo;
    {
      const uint32_t bound = first == 0xFFFFFFFFu ? hi : first;
      // probes are increasing in tid: the false ones below bound
      const bool f_ok = probe && !stop && k < bound;
      if (tid == 0) s_w[9] = 0;
      __syncthreads();
      if (f_ok) atomicMax(&s_w[9], k + 1);
      __syncthreads();
      nlo = s_w[9] > lo ? s_w[9] : lo;
      hi = bound;
    }
    lo = nlo;
    __syncthreads();
  }
  const uint32_t Kc = lo;
  for (uint32_t k = tid; k < Kc; k += 256) {
    const uint32_t xa = ML.pos(PL, k), xb = MR.pos(PR, nR - 1 - k);
    const uint64_t ka = K[xa];
    K[xa] = K[xb];
    K[xb] = ka;
    const uint32_t ta = T[xa];
    T[xa] = T[xb];
    T[xb] = ta;
  }
  uint32_t cut;
  if (Kc == 0) {
    cut = ML.pos(PL, 0);
  } else {
    cut = MR.pos(PR, nR - Kc);
    if (Kc < nL) {
      const uint32_t c2 = ML.pos(PL, Kc);
      if (c2 < cut) cut = c2;
    }
  }
  __syncthreads();
  return cut;
}

// The same partition as a block-wide Hoare scan (round 6, the default; RK_SPLIT_Q=0
// keeps block_partition): the block runs libstdc++'s two cursors a chunk at a time.  The
// left cursor scans QP_C positions upward from f + 1, the right one QP_C
// downward from l - 1; each scan appends its stoppers -- position, key and
// tag, in scan order -- to a ring queue in LDS, and a round pairs the two
// queues' heads (the k-th left stopper with the k-th right one) up to the
// first pair that crosses, swapping the others straight from the queues.  A
// position is read once by each cursor at most and written only if swapped,
// with no stopper lists in memory: ~12 B read and ~6 B written per member and
// level against ~45 B for block_partition's list pass, probe search and
// gathered swaps (cfg5's phase A was bound by that traffic).
// Exactness: the pairs before the crossing Kc are the original lists' (a
// position swapped as R_j lies above every left stopper still to come before
// the crossing, and symmetrically), so the queues' first Kc entries do not
// depend on when a scan reads a swapped position; at index Kc the queues hold
// min(L[Kc], R[Kc-1]) or L[Kc] (left) and max(R[Kc], L[Kc-1]) or R[Kc]
// (right), which cross either way, and the cut is min(QL[Kc], R[Kc-1]) --
// where libstdc++'s left cursor stops on the modified array.
#ifndef RK_QP_PER
#define RK_QP_PER 1
#endif
constexpr int QP_PER = RK_QP_PER;        // positions per thread in a scanned chunk
constexpr uint32_t QP_C = 256 * QP_PER;  // a chunk (and the pairs per round at most)
constexpr uint32_t QP_CAP = 2 * QP_C;    // ring capacity (a power of 2)
constexpr uint32_t QP_M = QP_CAP - 1;
struct QPart {
  uint64_t lk[QP_CAP], rk[QP_CAP];
  uint32_t lp[QP_CAP], rp[QP_CAP], lt[QP_CAP], rt[QP_CAP];
  uint32_t cnt[2][QP_PER * 4];
  uint32_t cross[2];  // by round parity (see the end of a round)
};

__device__ uint32_t block_partition_q(uint64_t *K, uint32_t *T, uint32_t f, uint32_t l,
                                      QPart &q) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
  // __move_median_to_first(f, f + 1, mid, l - 1) folded into the first
  // chunks' round trip: every thread reads the three candidates and slot f,
  // picks the median m, and keeps its own copies of the two swapped slots
  // right (slot m holds K[f]'s key and tag, slot f the pivot's) whenever it
  // loads them; thread 0 writes the swap after the first barrier (before any
  // pair's swap can write slot m)
#ifndef RK_QP_FOLD
#define RK_QP_FOLD 1
#endif
  if (!RK_QP_FOLD) {  // (A/B: the median's swap first, by thread 0)
    if (tid == 0) median_to_first(GView{K, T, nullptr, nullptr, nullptr}, f, l);
    __syncthreads();
  }
  const uint32_t ca = f + 1, cb = f + (l - f) / 2, cc = l - 1;
  const uint64_t ka = K[ca], kb = K[cb], kc = K[cc], k0 = K[f];
  const uint32_t ta = T[ca], tb = T[cb], tc = T[cc], t0 = T[f];
  // cursors: the left scan's next position, the right scan's next end (its
  // next position is rpos - 1); queue heads / tails count entries ever
  // pushed / popped (slots modulo QP_CAP)
  uint32_t lpos = f + 1, rpos = l;
  uint32_t qlh = 0, qlt = 0, qrh = 0, qrt = 0;
  uint32_t lastR = 0;  // R[Kc - 1]: the last right stopper swapped
  uint64_t ak[QP_PER], bk[QP_PER];
  uint32_t at[QP_PER], bt[QP_PER];
  uint32_t m = 0xFFFFFFFFu, fp = 0xFFFFFFFFu;  // (no patch for the first loads)
  uint64_t p = 0;
  uint32_t tm = 0;
  auto load_left = [&]() {
#pragma unroll
    for (int u = 0; u < QP_PER; ++u) {
      const uint32_t x = lpos + 256 * u + tid;
      const bool ok = x < l;
      const uint64_t k = ok ? K[x] : 0;
      const uint32_t t = ok ? T[x] : 0;
      ak[u] = x == m ? k0 : k;
      at[u] = x == m ? t0 : t;
    }
  };
  auto load_right = [&]() {
#pragma unroll
    for (int u = 0; u < QP_PER; ++u) {
      const uint32_t o = 256 * u + tid;
      const bool ok = o < rpos - f;
      const uint32_t x = ok ? rpos - 1 - o : f;
      const uint64_t k = ok ? K[x] : 0;
      const uint32_t t = ok ? T[x] : 0;
      bk[u] = x == m ? k0 : (x == fp ? p : k);
      bt[u] = x == m ? t0 : (x == fp ? tm : t);
    }
  };
  load_left();
  load_right();
  if (!RK_QP_FOLD) m = f;
  else if (ka < kb) m = kb < kc ? cb : (ka < kc ? cc : ca);
  else m = ka < kc ? ca : (kb < kc ? cc : cb);
  p = m == f ? k0 : m == ca ? ka : (m == cb ? kb : kc);
  tm = m == f ? t0 : m == ca ? ta : (m == cb ? tb : tc);
  fp = f;
#pragma unroll
  for (int u = 0; u < QP_PER; ++u) {
    const uint32_t x = lpos + 256 * u + tid;
    if (x == m) ak[u] = k0, at[u] = t0;
    const uint32_t o = 256 * u + tid;
    const uint32_t y = o < rpos - f ? rpos - 1 - o : 0xFFFFFFFFu;
    if (y == m) bk[u] = k0, bt[u] = t0;
    if (y == f) bk[u] = p, bt[u] = tm;
  }
  bool first = true;
  uint32_t par = 0;
  uint32_t cut = 0;
  for (;;) {
    const bool addl = qlt - qlh < QP_C && lpos < l;
    const bool addr = qrt - qrh < QP_C && rpos > f;
    if (!addl && qlt == qlh) {  // left cursor past l: it stops on R[Kc - 1]
      cut = qrh ? lastR : (qrt > qrh ? q.rp[qrh & QP_M] : f + 1);
      break;
    }
    if (!addr && qrt == qrh) {  // (unreachable: f itself is a right stopper)
      cut = q.lp[qlh & QP_M];
      break;
    }
    uint64_t bl[QP_PER], br[QP_PER];
#pragma unroll
    for (int u = 0; u < QP_PER; ++u) {
      const bool okl = addl && lpos + 256 * u + tid < l;
      const bool okr = addr && 256 * u + tid < rpos - f;
      bl[u] = __ballot(okl && !(ak[u] < p));
      br[u] = __ballot(okr && !(p < bk[u]));
      if (lane == 0) q.cnt[0][u * 4 + wv] = __popcll(bl[u]), q.cnt[1][u * 4 + wv] = __popcll(br[u]);
    }
    if (tid == 0) q.cross[par] = 0xFFFFFFFFu;
    __syncthreads();
    if (first && tid == 0) {  // the median's swap (every candidate read by now)
      K[f] = p;
      T[f] = tm;
      K[m] = k0;
      T[m] = t0;
    }
    first = false;
    uint32_t nl = 0, nr = 0, ol[QP_PER], orr[QP_PER];
#pragma unroll
    for (int j = 0; j < QP_PER * 4; ++j) {
      const uint32_t cl = q.cnt[0][j], cr = q.cnt[1][j];
      if (j % 4 == (int)wv) ol[j / 4] = nl, orr[j / 4] = nr;
      nl += cl;
      nr += cr;
    }
#pragma unroll
    for (int u = 0; u < QP_PER; ++u) {
      if ((bl[u] >> lane) & 1ull) {
        const uint32_t s = (qlt + ol[u] + __popcll(bl[u] & lt)) & QP_M;
        q.lk[s] = ak[u];
        q.lt[s] = at[u];
        q.lp[s] = lpos + 256 * u + tid;
      }
      if ((br[u] >> lane) & 1ull) {
        const uint32_t s = (qrt + orr[u] + __popcll(br[u] & lt)) & QP_M;
        q.rk[s] = bk[u];
        q.rt[s] = bt[u];
        q.rp[s] = rpos - 1 - (256 * u + tid);
      }
    }
    if (addl) {
      qlt += nl;
      lpos += QP_C;
      if (lpos < l) load_left();
    }
    if (addr) {
      qrt += nr;
      rpos = rpos - f > QP_C ? rpos - QP_C : f;
      if (rpos > f) load_right();
    }
    __syncthreads();
    uint32_t m = qlt - qlh < qrt - qrh ? qlt - qlh : qrt - qrh;
    if (m > QP_C) m = QP_C;
    for (uint32_t i = tid; i < m; i += 256)
      if (q.lp[(qlh + i) & QP_M] >= q.rp[(qrh + i) & QP_M]) atomicMin(&q.cross[par], i);
    __syncthreads();
    const uint32_t cr = q.cross[par];
    const uint32_t kc = cr < m ? cr : m;
    for (uint32_t i = tid; i < kc; i += 256) {
      const uint32_t sl = (qlh + i) & QP_M, sr = (qrh + i) & QP_M;
      const uint32_t xl = q.lp[sl], xr = q.rp[sr];
      K[xl] = q.rk[sr];
      K[xr] = q.lk[sl];
      T[xl] = q.rt[sr];
      T[xr] = q.lt[sl];
    }
    if (kc) lastR = q.rp[(qrh + kc - 1) & QP_M];
    if (cr < m) {
      const uint32_t cl = q.lp[(qlh + kc) & QP_M];
      cut = qrh + kc ? (cl < lastR ? cl : lastR) : cl;
      break;
    }
    qlh += kc;
    qrh += kc;
    // no barrier here: the next round's appends (the only writes to the
    // queues' slots) follow its first barrier, which every wavefront reaches
    // only after this round's swaps; the crossing word alternates by parity,
    // so the next round's reset cannot meet a slow wavefront's read of it
    par ^= 1u;
  }
  __syncthreads();
  return cut;
}

// Depth-exhausted segments of at least HEAP_BLOCK_MIN members found by phase
// A, heap-sorted afterwards by k_heap_segments (one block each, its LDS holding
// the heap's top levels)
struct HeapSeg {
  uint32_t b, f, n, pad;
};
constexpr uint32_t HEAPQ_CAP = 512;

// The groups are claimed one at a time (claim[0..1], zeroed): first every
// group of at least `big` members, then the rest -- the largest jobs first, so
// no block is left with a large group at the end (a static round-robin
// share of ~18 groups per block left the launch waiting on its heaviest
// blocks).  big = 0: one dynamic pass in list order; claim null: the static
// round-robin.
// 8 wavefronts per SIMD (the queue partition's 53 VGPRs, 8 blocks of 17 KB of
// LDS per CU; the SGPRs above 96 spill to VGPR lanes) instead of the 7 its
// SGPRs allowed.  RK_SPLIT_WPE=0: the compiler's choice
#ifndef RK_SPLIT_WPE
#define RK_SPLIT_WPE 8
#endif
#if RK_SPLIT_WPE
#define RK_SPLIT_WPE_ATTR __attribute__((amdgpu_waves_per_eu(RK_SPLIT_WPE)))
#else
#define RK_SPLIT_WPE_ATTR
#endif
template <bool qpart>
__global__ void __launch_bounds__(256) RK_SPLIT_WPE_ATTR k_sort_groups_split(TierLists tl, int tier,
                                                           const uint32_t *goff, uint64_t *key,
                                                           uint32_t *tag, uint32_t *otag,
                                                           uint32_t *pl, uint32_t *pr,
                                                           uint8_t *bnd, uint32_t *heapq_n,
                                                           HeapSeg *heapq, uint32_t *claim,
                                                           uint32_t big) {
  __shared__ Frame stack[SPLIT_STACK];
  __shared__ uint32_t s_w[16];
  // the queues in dynamic LDS: reserved only when the queue partition runs
  extern __shared__ __attribute__((aligned(16))) uint8_t split_lds[];
  QPart &qp = *reinterpret_cast<QPart *>(split_lds);
  const uint32_t tid = threadIdx.x;
  uint32_t lo, hi;
  tl.range(tier, lo, hi);
  if (lo == hi) return;
  const int npass = claim ? (big ? 2 : 1) : 1;
  for (int pass = 0; pass < npass; ++pass)
  for (uint32_t w = lo + blockIdx.x;; w += gridDim.x) {
    if (claim) {
      if (tid == 0) s_w[11] = lo + atomicAdd(&claim[pass], 1u);
      __syncthreads();
      w = s_w[11];
      __syncthreads();  // (read by every thread before the next claim)
    }
    if (w >= hi) break;
    const uint32_t g = tl.list[w];
    const uint32_t b = goff[g], n = goff[g + 1] - b;
    if (claim && big && (n >= big) != (pass == 0)) continue;
    uint64_t *K = key + b;
    uint32_t *T = tag + b;
    // the tags (positions) written here: phase A moves them in memory, phase
    // B and the heap kernel read them back
    for (uint32_t x = tid; x < n; x += 256) T[x] = b + x;
    int sp = 1;
    if (tid == 0) stack[0] = {0u, n, 2 * (31 - __clz((int)n))};
    __syncthreads();
    while (sp) {
      const Frame fr = stack[--sp];
      __syncthreads();  // every thread has read the frame before it is reused
      uint32_t f = fr.f, l = fr.l;
      int d = fr.d;
      for (;;) {
        if (l - f <= SPLIT_T) {
          if (tid == 0) {
            bnd[b + f] = 1;
            pl[b + f] = (l - f) | (uint32_t)d << 16;
          }
          break;
        }
        if (d == 0) {  // __partial_sort fallback on a large segment
          if (l - f >= HEAP_BLOCK_MIN) {  // queued for k_heap_segments
            if (tid == 0) {
              const uint32_t i = atomicAdd(heapq_n, 1u);
              s_w[10] = i < HEAPQ_CAP;
              if (i < HEAPQ_CAP) heapq[i] = HeapSeg{b, f, l - f, 0u};
            }
            __syncthreads();
            const bool queued = s_w[10] != 0;
            __syncthreads();
            if (queued) break;
          }
          if (tid == 0) heap_sort_segment(GView{K, T, nullptr, nullptr, nullptr}, f, l);
          __syncthreads();
          for (uint32_t x = f + tid; x < l; x += 256) otag[b + x] = T[x];
          break;
        }
        --d;
        const uint32_t cut = qpart ? block_partition_q(K, T, f, l, qp)
                                   : block_partition(K, T, pl + b, pr + b, f, l, s_w);
        if (tid == 0) stack[sp] = {cut, l, d};
        ++sp;
        l = cut;
        __syncthreads();
      }
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(256) k_heap_segments(const uint32_t *heapq_n,
                                                       const HeapSeg *heapq, uint64_t *key,
                                                       uint32_t *tag, uint32_t *otag) {
  __shared__ uint64_t lk[HTOP + 1];
  __shared__ uint32_t lt[HTOP + 1];
  const uint32_t cnt = min(*heapq_n, HEAPQ_CAP);
  for (uint32_t s = blockIdx.x; s < cnt; s += gridDim.x) {
    const HeapSeg g = heapq[s];
    const size_t o = (size_t)g.b + g.f;
    block_heap_sort(key + o, tag + o, g.n, otag + o, lk, lt);
  }
}

// ---------------------------------------------------------------------------
// Heap segments with a few distinct keys (2..RANK_MAX): a median-of-three
// killer whose never-compared members carry a few values.  A pop's path
// depends on the keys alone, and a pop moves the tags along that path: the
// root's to `last`, the one at `last` to path slot j, path slots 1..j up one
// level each.  So instead of replaying the pops with the tags (one pop after
// another, ~2.7 us each: 285 ms for a 100K heap):
//  1. k_heap_prep: __make_heap (level-parallel), the segment's distinct keys
//     (one block-wide minimum per key) and every key's rank (one byte) --
//     or, with one key, the spine-ring path; with more than RANK_MAX, the
//     general pops;
//  2. k_heap_rank_pops: the pops on the ranks alone, one wavefront, the heap
//     in LDS as far as it fits (one byte per node: 160K nodes), the descent
//     found HR levels per round as in wave_sort_heap; each pop logs its
//     direction bits from the root (D levels) and the slot j where the
//     displaced value lands;
//  3. the (node, pop) pairs of every pop's written slots p_0..p_j, sorted by
//     node (stable: by pop within a node);
//  4. k_heap_trace: every output position independently, backwards through
//     the pops: the element at node y just before pop t was put there by the
//     last pop t' < t that wrote y -- from its slot i + 1 when y is its slot
//     i < j, from its `last` when y is its slot j --, or has been there since
//     __make_heap when no pop before t wrote y.
constexpr uint32_t RANK_MAX = 16;  // distinct keys of the rank path (one pass each)
enum : uint32_t { HM_EQUAL = 1, HM_RANK = 2, HM_GENERAL = 3 };

__global__ void __launch_bounds__(256) k_heap_prep(uint64_t *K, uint32_t *T, uint32_t n,
                                                  uint8_t *R, uint32_t *mode) {
  __shared__ unsigned long long vals[RANK_MAX];
  __shared__ unsigned long long s_min;
  __shared__ uint32_t s_found;
  const uint32_t tid = threadIdx.x;
  block_make_heap(K, T, n);
  // the distinct keys in ascending order, one block-wide minimum per round
  uint32_t D = 0;
  for (;;) {
    if (tid == 0) s_min = ~0ull, s_found = 0;
    __syncthreads();
    const unsigned long long prev = D ? vals[D - 1] : 0ull;
    unsigned long long mn = ~0ull;
    bool found = false;
    for (uint32_t x = tid; x < n; x += blockDim.x) {
      const unsigned long long k = K[x];
      if (D == 0 || k > prev) {
        found = true;
        mn = k < mn ? k : mn;
      }
    }
    if (found) {
      atomicMin(&s_min, mn);
      atomicOr(&s_found, 1u);
    }
    __syncthreads();
    if (!s_found) break;
    if (D == RANK_MAX) {  // too many distinct keys for the rank path
      ++D;
      break;
    }
    if (tid == 0) vals[D] = s_min;
    ++D;
    __syncthreads();
  }
  // (the rank pops' 32-bit positions: heaps below 2^23 nodes)
  const uint32_t md = D <= 1 ? HM_EQUAL : D <= RANK_MAX && n < (1u << 23) ? HM_RANK : HM_GENERAL;
  if (md == HM_RANK)
    for (uint32_t x = tid; x < n; x += blockDim.x) {
      const unsigned long long k = K[x];
      uint32_t r = 0;
      while (vals[r] != k) ++r;
      R[x + 1] = (uint8_t)r;  // (shifted: a node pair is one aligned 16-bit word)
    }
  if (tid == 0) mode[0] = md, mode[1] = D;  // (D exact up to RANK_MAX)
}

// the spine-ring path (one key) and the general pops (more than RANK_MAX keys)
// of a heap segment after k_heap_prep; each returns at once on the other modes
__global__ void __launch_bounds__(64) k_heap_equal(uint32_t *T, uint32_t n, uint32_t *out,
                                                  const uint32_t *mode) {
  if (*mode != HM_EQUAL) return;
  const uint32_t lane = threadIdx.x;
  wave_sort_heap_equal(T, n, lane);
  wave_sync_global();  // (this wavefront's stores before its loads)
  for (uint32_t x = lane; x < n; x += 64) out[x] = T[x];
}
__global__ void __launch_bounds__(256) k_heap_general(uint64_t *K, uint32_t *T, uint32_t n,
                                                     uint32_t *out, const uint32_t *mode) {
  __shared__ uint64_t lk[HTOP + 1];
  __shared__ uint32_t lt[HTOP + 1];
  if (*mode != HM_GENERAL) return;
  const uint32_t tid = threadIdx.x;
  for (uint32_t x = tid; x < n && x < HTOP; x += blockDim.x) lk[x] = K[x], lt[x] = T[x];
  __syncthreads();
  if (tid < 64) wave_sort_heap(HeapMem{K, T, lk, lt}, n, tid);
  __syncthreads();
  for (uint32_t x = tid; x < n; x += blockDim.x) out[x] = x < HTOP ? lt[x] : T[x];
}

typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint16_t lds_u16;

// k_heap_rank_pops: __sort_heap of [0, n) on the ranks alone by one
// wavefront; pop t = n - 1 - last logs its direction bits from the root
// (logb, the first level the highest of D bits) and D | j << 8 (logq).  The
// ranks come from k_heap_prep at R[x + 1]; nodes x < RT live in LDS at
// L[x + 1] (the whole heap when it fits, BIG = false; else the top ~159K
// nodes, RT odd, and the rest stays in R) -- shifted by one so that a node's
// two children 2y + 1, 2y + 2 are one aligned 16-bit word, read by one 16-bit
// load per pair (RT odd: no pair straddles the two arrays).  L[SENT],
// L[SENT + 1] hold a sentinel pair (1, 0) -- right < left, no "right"
// direction -- read in place of every pair whose right child is outside the
// heap, so a direction is one compare.  No static LDS: the array starts at
// LDS address 0 and constant offsets fold into the ds instructions.  32-bit
// positions (a round's (hole + 1) << 8 stays below 2^32 for heaps below 2^23
// nodes; the host routes larger ones to the general pops).  A lone wavefront
// pays every instruction in latency (~5-8 cycles each,
// `tools/mb/clockprobe.hip`), so the pop is cut to what it needs:
//  * a pop's descent is found 8 levels per round: lane l holds the child pairs
//    of the round's internal nodes J = l + 64 s, s < 4, numbered from 1 (J's
//    children are 2J, 2J + 1), one ballot per s holds every direction (ties go
//    right), and the round's direction bits are J - 2^Dr at its end;
//  * the first round's pairs (the heap's top 8 levels, fixed positions 2J - 1,
//    2J) stay in registers, re-read after each pop's stores;
//  * the walk takes all 8 steps as s_bitcmp1 (SCC = the direction bit) +
//    s_addc (J = 2J + SCC) and is cut afterwards to the levels that exist
//    without a test (descents onto the complete levels; the first k steps of
//    a walk are J >> (8 - k)); at most one step more, onto the incomplete last
//    level, is tested;
//  * __push_heap: lane i reads path node i (x_0 the root) at the position the
//    bits give, one ballot counts the path keys below the displaced value
//    (they form a suffix: the path's keys descend), and lane i moves its key to
//    x_{i-1} when 1 <= i <= j, the value landing at x_j; the log collects in
//    two registers, lane t % 64 holding pop t, 64 pops per store.
// The round-4 general pops (64-bit keys, tags moved along) took ~2.9 us per
// pop; the first rank version (64-bit positions, per-node LDS / global
// selection, path keys through a scratch) ~3 us, bound by instruction
// latency; this one ~0.5 us with the heap in LDS.
constexpr int RHR = 8;                          // levels per round
constexpr uint32_t RPAIRS = (1u << RHR) - 1;    // internal nodes of a round (255)
constexpr int RS = (int)((RPAIRS + 64) / 64);   // pairs per lane (4: J = 0 .. 255)
__device__ __forceinline__ uint32_t dir_bit(uint64_t d0, uint64_t d1, uint64_t d2, uint64_t d3,
                                            uint32_t J) {
  const uint64_t lo = J < 64 ? d0 : d1, hi = J < 192 ? d2 : d3;
  return (uint32_t)((J < 128 ? lo : hi) >> (J & 63)) & 1u;
}
template <bool BIG>
__global__ void __launch_bounds__(64) k_heap_rank_pops(uint8_t *R, uint32_t n, uint32_t RT,
                                                      uint32_t *logb, uint16_t *logq,
                                                      const uint32_t *mode) {
  extern __shared__ uint8_t lr[];
  if (*mode != HM_RANK) return;
  lds_u8 *L = (lds_u8 *)lr;
  const uint32_t lane = threadIdx.x;
  const uint32_t SENT = (RT + 2) & ~1u, DUMMY = SENT + 4;  // (a discarded store's slot)
  for (uint32_t x = lane; x < RT; x += 64) L[x + 1] = R[x + 1];
  if (lane == 0) L[0] = 0, L[RT + 1] = 0, L[SENT] = 1, L[SENT + 1] = 0;
  wave_sync();
  const auto key = [&](uint32_t x) {  // (wave-uniform x)
    return BIG && x >= RT ? (uint32_t)R[x + 1] : (uint32_t)L[x + 1];
  };
  // (lane 0's J = 0 is no node: its words and direction bit are never used)
  uint32_t Jv[RS], sh[RS], ad[RS], w1[RS];
#pragma unroll
  for (int s = 0; s < RS; ++s) {
    const uint32_t J = lane + 64 * s, d = 31 - __clz((int)(J | 1u));
    Jv[s] = J;
    sh[s] = d + 1;                         // left child of J below hole h:
    ad[s] = 2 * (J - (1u << d)) - 1u;      // ((h + 1) << (d + 1)) - 1 + 2 (J - 2^d)
  }
  const auto load_w1 = [&] {  // (positions <= 510 < RT)
#pragma unroll
    for (int s = 0; s < RS; ++s) w1[s] = *(const lds_u16 *)(L + 2 * Jv[s]);
  };
  load_w1();
  uint32_t lb = 0, lq = 0;
#ifdef RK_HEAP_PROF
  unsigned long long c_load = 0, c_walk = 0, c_push = 0, c_rounds = 0;
#define HP_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#else
#define HP_T(v)
#endif
  for (uint32_t last = n - 1; last > 0; --last) {
    const uint32_t vk = key(last);
    const uint32_t len = last;
    const uint32_t fl = 31 - __clz((int)(len + 1));  // levels 0 .. fl - 1 are complete
    uint32_t hole = 0, bits = 0, D = 0;
    for (bool first = true;; first = false) {
      HP_T(h0);
      uint32_t w[RS];
      if (first) {
#pragma unroll
        for (int s = 0; s < RS; ++s) w[s] = 2 * Jv[s] < len ? w1[s] : 1u;  // (1, 0): no direction
      } else {
        uint32_t lp[RS];
        bool glob[RS], anyg = false;
#pragma unroll
        for (int s = 0; s < RS; ++s) {
          const uint32_t l = ((hole + 1) << sh[s]) + ad[s];
          const bool pres = l + 1 < len;
          lp[s] = l + 1;
          glob[s] = BIG && pres && l >= RT;
          anyg |= glob[s];
          w[s] = *(const lds_u16 *)(L + (pres && !glob[s] ? l + 1 : SENT));
        }
        if (BIG && __builtin_amdgcn_ballot_w64(anyg)) {  // a round below the LDS levels
#pragma unroll
          for (int s = 0; s < RS; ++s)
            if (glob[s]) w[s] = *(const uint16_t *)(R + lp[s]);
        }
      }
      uint64_t dm[RS];
#pragma unroll
      for (int s = 0; s < RS; ++s) dm[s] = __builtin_amdgcn_ballot_w64((w[s] >> 8) >= (w[s] & 0xffu));  // ties go right
      HP_T(h1);
      D = __builtin_amdgcn_readfirstlane(D);
      hole = __builtin_amdgcn_readfirstlane(hole);
      bits = __builtin_amdgcn_readfirstlane(bits);
      const uint64_t d0 = dm[0], d1 = dm[1 % RS], d2 = dm[2 % RS], d3 = dm[3 % RS];
      uint32_t J8 = 1;
      uint64_t tmp;
      static_assert(RHR == 8 && RS == 4, "the walk below is written for 8 levels");
      asm volatile(
          "s_bitcmp1_b64 %[d0], %[J]\n\ts_addc_u32 %[J], %[J], %[J]\n\t"
          "s_bitcmp1_b64 %[d0], %[J]\n\ts_addc_u32 %[J], %[J], %[J]\n\t"
          "s_bitcmp1_b64 %[d0], %[J]\n\ts_addc_u32 %[J], %[J], %[J]\n\t"
          "s_bitcmp1_b64 %[d0], %[J]\n\ts_addc_u32 %[J], %[J], %[J]\n\t"
          "s_bitcmp1_b64 %[d0], %[J]\n\ts_addc_u32 %[J], %[J], %[J]\n\t"
          "s_bitcmp1_b64 %[d0], %[J]\n\ts_addc_u32 %[J], %[J], %[J]\n\t"
          "s_bitcmp1_b64 %[d1], %[J]\n\ts_addc_u32 %[J], %[J], %[J]\n\t"
          "s_cmpk_lt_u32 %[J], 0xc0\n\ts_cselect_b64 %[t], %[d2], %[d3]\n\t"
          "s_bitcmp1_b64 %[t], %[J]\n\ts_addc_u32 %[J], %[J], %[J]"
          : [J] "+s"(J8), [t] "=&s"(tmp)
          : [d0] "s"(d0), [d1] "s"(d1), [d2] "s"(d2), [d3] "s"(d3)
          : "scc");
      const uint32_t lim = fl >= D + 2 ? min((uint32_t)RHR, fl - 1 - D) : 0u;
      uint32_t J = J8 >> (RHR - lim), Dr = lim;
      uint32_t x = ((hole + 1) << Dr) - 1 + (J - (1u << Dr));
      bool more;
      if (Dr == RHR) {
        more = 2 * x + 1 < len;
      } else {
        const uint32_t two = 2 * x + 2;
        more = false;
        if (two <= len) {
          const uint32_t bt = two < len ? dir_bit(d0, d1, d2, d3, J) : 0u;  // (==: a lone left child)
          J = 2 * J + bt;
          x = two - 1 + bt;
          if (++Dr == RHR) more = 2 * x + 1 < len;
        }
      }
      bits = (Dr ? bits << Dr : bits) | (J - (1u << Dr));
      D += Dr;
      hole = x;
#ifdef RK_HEAP_PROF
      HP_T(h2);
      c_load += h1 - h0, c_walk += h2 - h1, ++c_rounds;
#endif
      if (!more) break;
    }
    HP_T(h4);
    // __push_heap
    const uint32_t i = lane;
    const bool on = i <= D;
    const uint32_t xi = (1u << i) - 1u + (on ? bits >> (D - i) : 0u);
    const bool gi = BIG && on && xi >= RT;
    uint32_t ki = on && !gi ? (uint32_t)L[xi + 1] : 0u;
    if (BIG && gi) ki = R[xi + 1];
    const uint32_t j = D - (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(on && i >= 1 && ki < vk));
    wave_sync();  // (every lane's read before any write; one wavefront's memory ops are in order)
    if (i >= 1 && i <= j) {
      const uint32_t y = (xi - 1) / 2;  // x_{i-1}
      if (!BIG || y < RT) L[y + 1] = (uint8_t)ki;
      else R[y + 1] = (uint8_t)ki;
    }
    if (i == j) {
      if (!BIG || xi < RT) L[xi + 1] = (uint8_t)vk;
      else R[xi + 1] = (uint8_t)vk;
    }
    const uint32_t t = n - 1 - last;
    if (lane == (t & 63)) lb = bits, lq = D | j << 8;
    if ((t & 63) == 63 || last == 1) {
      const uint32_t t0 = t & ~63u;
      if (t0 + lane <= t) logb[t0 + lane] = lb, logq[t0 + lane] = (uint16_t)lq;
    }
    wave_sync();
    load_w1();
#ifdef RK_HEAP_PROF
    HP_T(h5);
    c_push += h5 - h4;
#endif
  }
  (void)DUMMY;
#ifdef RK_HEAP_PROF
  if (lane == 0)
    printf("HEAPPROF n=%u cycles/pop: load %.0f walk %.0f push %.0f | rounds/pop %.2f\n", n,
           (double)c_load / (n - 1), (double)c_walk / (n - 1), (double)c_push / (n - 1),
           (double)c_rounds / (n - 1));
#endif
#undef HP_T
}

// k_heap_pipe_pops: the pops of k_heap_rank_pops, pipelined.  A rank pop is a
// top-down sift of the displaced value vk = R[last] from the root: the hole
// takes its larger child's key (the right one unless right < left; a lone
// left child below the last full level) while that key is >= vk, and vk lands
// where it stops.  __adjust_heap's descent to a leaf followed by __push_heap
// ends the same way: the path's keys descend and __push_heap lifts vk past
// exactly the path keys below it, so the nodes below the landing slot end
// unchanged.  A pop therefore writes one node per level, top down, and pop
// k + 1 can descend behind pop k: with pop k's hole two levels below pop
// k + 1's, every node pop k + 1 reads (its hole's two children) already holds
// pop k's write.  One wavefront carries up to ~depth / 2 pops, a lane each; a
// tick moves every pop one level (one LDS load of its children, its write as
// an and / or pair), and the next pop starts when
//  * the previous one started at least two ticks ago (two levels down), and
//  * no pop in flight can still write the new pop's `last` node (no hole is
//    that node or an ancestor of it), so vk is final when it is read.
// The log is the path's direction bits down to the landing level j (D = j in
// logq: the nodes below j are unchanged).  Ranks packed P bits per node (P =
// 1, 2, 4 for 2, <= 4, <= 16 distinct keys), node x at bit (x + 1) P, so the
// children pair 2x + 1, 2x + 2 is 2P aligned bits of one byte.  The whole heap
// lives in LDS (the host checks the size); a pop costs two ticks instead of
// its whole descent and push.
typedef __attribute__((address_space(3))) uint32_t lds_u32;
template <int P>
__device__ __forceinline__ void pipe_pops(lds_u8 *LB, lds_u32 *LW, uint32_t n, uint32_t HD,
                                          uint32_t *logb, uint16_t *logq, uint32_t lane) {
  constexpr uint32_t M = (1u << P) - 1u;
  const auto pair = [&](uint32_t bit) -> uint32_t {  // the 2P bits at `bit`
    if constexpr (P == 8) return *(const lds_u16 *)(LB + (bit >> 3));
    else return (uint32_t)LB[bit >> 3] >> (bit & 7);
  };
  const uint32_t npop = n - 1, PMAX = (HD + 1) * P;  // (a pair's bit stays below PMAX)
  // a lane's pop: B = hole + 1 -- a leading 1, then the path's direction bits
  // from the root (its level is B's bit length - 1; the hole's children 2B - 1,
  // 2B are the pair at bit 2B P; the next hole + 1 is 2B + direction) --, the
  // displaced key vk, the heap length len (0: an idle lane, B = HD + 1: its
  // writes go to the spare word) and the pop's index k
  uint32_t B = HD + 1, vk = 0, len = 0, k = 0;
  uint32_t knext = 0, ndone = 0;
  int since = 2;  // ticks since the last start (very negative: every pop started)
  uint64_t busy = 0;
  while (ndone < npop) {
    // the tick's loads first: every pop's children, the root's, the next `last`
    uint32_t w = pair(min(2 * B * P, PMAX));
    const uint32_t wroot = pair(2 * P);
    const uint32_t y = n - 1 - knext, bv = (y + 1) * P;  // the next pop's `last`
    const uint32_t v = ((uint32_t)LB[bv >> 3] >> (bv & 7)) & M;
    if (since >= 2) {
      // a pop in flight whose hole is y or an ancestor of it (B a binary prefix
      // of y + 1; never an idle lane's HD + 1) may still write y: y is a leaf of
      // its heap (else it might move a child's key up), so only its own
      // displaced key, which matters only when it is not v
      const uint32_t cy = __clz((int)(y + 1)), cb = __clz((int)B);
      const bool unsafe = (cb >= cy) & (((y + 1) >> (cb - cy)) == B) &
                          ((vk != v) | (2 * y + 1 < len));  // (no short cut: no branch)
      if (!__builtin_amdgcn_ballot_w64(unsafe)) {  // (fewer pops in flight than lanes)
        const uint32_t slot = (uint32_t)__builtin_ctzll(~busy);
        busy |= 1ull << slot;
        if (lane == slot) B = 1, vk = v, len = y, k = knext, w = wroot;
        since = ++knext < npop ? 0 : -(1 << 30);
      }
    }
    ++since;
    const uint32_t kl = w & M, kr = (w >> P) & M;
    const bool rt = (2 * B < len) & (kr >= kl);  // right child present and not smaller
    const uint32_t kc = rt ? kr : kl;
    const bool cont = (2 * B <= len) & (kc >= vk);  // (left child present)
    const uint32_t nv = cont ? kc : vk;
    if constexpr (P == 8) {
      LB[B] = (uint8_t)nv;
    } else {
      const uint32_t bh = B * P, sh = bh & 31;
      __hip_atomic_fetch_and(LW + (bh >> 5), ~(M << sh), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_or(LW + (bh >> 5), nv << sh, __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    const bool fin = (len != 0) & !cont;
    const uint64_t fm = __builtin_amdgcn_ballot_w64(fin);
    if (fm) {
      if (fin) logb[k] = B;  // (k_heap_log_split: the bits and the level)
      ndone += (uint32_t)__popcll(fm);
      busy &= ~fm;
    }
    B = cont ? 2 * B + (rt ? 1u : 0u) : fin ? HD + 1 : B;
    len = fin ? 0u : len;
  }
  (void)logq;
}
// The same pops for a heap too large for LDS: levels 0 .. L - 1 packed in LDS,
// the bottom level L (leaves only) in the global byte array R (node x at
// R[x + 1] = R[B]).  A leaf is read only as a child of a level L - 1 hole and
// written only as a pop's last write, so:
//  * when a pop's hole reaches level L - 2 (end of a tick) it loads its four
//    leaf descendants (one u32 at R[4B]); two ticks later, at level L - 1, two
//    of those bytes are its children pair -- the load had a whole tick (~390
//    cycles) against an L2 hit's ~200;
//  * the loads go to a slot by tick parity (the tick is written twice, loads
//    unconditional: a lane with nothing to load reads R[0]), so the wait
//    counts are fixed and a slot is consumed before the same-parity tick
//    reloads it;
//  * leaf writes (at most one a tick: one pop per level) go to R and to a
//    2-tick ring of (R index, key) in scalars, which patches the loaded bytes
//    of the one pop at level L - 1 (its load was issued before those writes);
//  * the next pop's `last` node, a leaf until the heap is down to L levels,
//    comes the same way (loaded by parity, patched by the ring).
// Every store is unconditional too (a lane with nothing to store writes R[0]
// or logb[npop]).
template <int P>
__device__ __forceinline__ void pipe_pops_tail(lds_u8 *LB, lds_u32 *LW, uint8_t *R, uint32_t n,
                                               uint32_t L, uint32_t HD, uint32_t *logb,
                                               uint32_t lane) {
  constexpr uint32_t M = (1u << P) - 1u;
  const auto pair = [&](uint32_t bit) -> uint32_t {
    if constexpr (P == 8) return *(const lds_u16 *)(LB + (bit >> 3));
    else return (uint32_t)LB[bit >> 3] >> (bit & 7);
  };
  const uint32_t npop = n - 1, PMAX = (HD + 1) * P;
  const uint32_t TOPB = 1u << L, HALF = TOPB >> 1, QTR = TOPB >> 2;  // B < TOPB: in LDS
  const uint32_t RMAX = n + 12;  // (R holds n + 16 bytes: a u32 at <= n + 12)
  uint32_t B = HD + 1, vk = 0, len = 0, k = 0;
  uint32_t knext = 0, ndone = 0;
  int since = 2;
  uint64_t busy = 0;
  // the leaf writes of the last two ticks (R index, key), newest first: a load
  // issued at the end of tick t and used at t + 2 misses t + 1's write (and
  // t's is kept too); older stores come before the load in the wave's order
  uint32_t rb0 = 0, rv0 = 0, rb1 = 0, rv1 = 0;
  const auto patch = [&](uint32_t at, uint32_t val) {  // (uniform operands: scalar)
    val = rb1 == at ? rv1 : val;
    return rb0 == at ? rv0 : val;
  };
  uint32_t pf0 = 0, pf1 = 0, vg0 = *(const uint32_t *)(R + (n & ~3u)), vg1 = vg0;  // (node n - 1)
  // a zero the compiler cannot see through: the `last` word's load stays a
  // vector load (a uniform one is moved to a scalar at once, waiting on it)
  uint32_t vzero;
  asm volatile("v_mov_b32 %0, 0" : "=v"(vzero));
  const auto tick = [&](uint32_t &pf, uint32_t &vg) {
    uint32_t w = pair(min(2 * B * P, PMAX));
    const uint32_t wroot = pair(2 * P);
    const uint32_t y = n - 1 - knext;
    if (since >= 2) {
      uint32_t v;
      if (y + 1 >= TOPB) {  // (its aligned word loaded)
        const uint32_t sv = (uint32_t)__builtin_amdgcn_readfirstlane((int)vg);
        v = patch(y + 1, (sv >> ((y + 1) & 3u) * 8) & 0xffu);
      } else {
        const uint32_t bv = (y + 1) * P;
        v = ((uint32_t)LB[bv >> 3] >> (bv & 7)) & M;
      }
      const uint32_t cy = __clz((int)(y + 1)), cb = __clz((int)B);
      // (len != 0: an idle lane's B = HD + 1 = TOPB is the first leaf's B)
      const bool unsafe = (len != 0) & (cb >= cy) & (((y + 1) >> (cb - cy)) == B) &
                          ((vk != v) | (2 * y + 1 < len));
      if (!__builtin_amdgcn_ballot_w64(unsafe)) {
        const uint32_t slot = (uint32_t)__builtin_ctzll(~busy);
        busy |= 1ull << slot;
        if (lane == slot) B = 1, vk = v, len = y, k = knext, w = wroot;
        since = ++knext < npop ? 0 : -(1 << 30);
      }
    }
    ++since;
    uint32_t kl = w & M, kr = (w >> P) & M;
    // a hole at level L - 1 takes its children from pf -- one lane at most
    // (pops are two levels apart): its bytes and their patch in scalars
    const uint64_t lpm = __builtin_amdgcn_ballot_w64((B >= HALF) & (B < TOPB));
    if (lpm) {
      const int li = (int)__builtin_ctzll(lpm);
      const uint32_t sb = (uint32_t)__builtin_amdgcn_readlane((int)B, li);
      const uint32_t sp = (uint32_t)__builtin_amdgcn_readlane((int)pf, li);
      const uint32_t sh = (sb & 1u) * 16u;  // B = 2 B' + direction since the load at B'
      const uint32_t gl = patch(2 * sb, (sp >> sh) & 0xffu);
      const uint32_t gr = patch(2 * sb + 1, (sp >> (sh + 8)) & 0xffu);
      kl = lane == (uint32_t)li ? gl : kl;
      kr = lane == (uint32_t)li ? gr : kr;
    }
    const bool rt = (2 * B < len) & (kr >= kl);
    const uint32_t kc = rt ? kr : kl;
    const bool cont = (2 * B <= len) & (kc >= vk);
    const uint32_t nv = cont ? kc : vk;
    const bool gw = (B >= TOPB) & (len != 0);  // a leaf hole: the pop's last write
    const uint32_t Bw = gw ? HD + 1 : B;       // (its LDS write to the spare word)
    if constexpr (P == 8) {
      LB[Bw] = (uint8_t)nv;
    } else {
      const uint32_t bh = Bw * P, sh = bh & 31;
      __hip_atomic_fetch_and(LW + (bh >> 5), ~(M << sh), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_or(LW + (bh >> 5), nv << sh, __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    R[gw ? B : 0u] = (uint8_t)nv;
    const uint64_t gm = __builtin_amdgcn_ballot_w64(gw);
    const int gi = gm ? (int)__builtin_ctzll(gm) : 0;
    const uint32_t gb = (uint32_t)__builtin_amdgcn_readlane((int)B, gi);
    const uint32_t gv = (uint32_t)__builtin_amdgcn_readlane((int)nv, gi);
    rb1 = rb0, rv1 = rv0;
    rb0 = gm ? gb : 0u, rv0 = gv;
    const bool fin = (len != 0) & !cont;
    const uint64_t fm = __builtin_amdgcn_ballot_w64(fin);
    logb[fin ? k : npop] = B;  // (k_heap_log_split: the bits and the level)
    ndone += (uint32_t)__popcll(fm);
    busy &= ~fm;
    B = cont ? 2 * B + (rt ? 1u : 0u) : fin ? HD + 1 : B;
    len = fin ? 0u : len;
    // the loads for two ticks on: leaf descendants, the next `last` leaf
    const uint32_t pa = ((B >= QTR) & (B < HALF) & (4 * B <= RMAX)) ? 4 * B : 0u;
    pf = *(const uint32_t *)(R + pa);
    const uint32_t y2 = n - 1 - knext;  // (a u32 load: no byte value carried over the loop)
    vg = *(const uint32_t *)(R + (((y2 + 1 >= TOPB ? y2 + 1 : 0u) & ~3u) + vzero));
  };
  while (ndone < npop) {
    tick(pf0, vg0);
    if (ndone >= npop) break;
    tick(pf1, vg1);
  }
}

// k_heap_pipe_pops logs B (a leading 1, then the j direction bits): logb, logq
// as k_heap_rank_pops writes them (D = j)
__global__ void k_heap_log_split(uint32_t *logb, uint16_t *logq, uint32_t npop,
                                 const uint32_t *mode) {
  if (mode[0] != HM_RANK) return;
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < npop; t += gridDim.x * blockDim.x) {
    const uint32_t b = logb[t], j = 31 - __clz((int)b);
    logb[t] = b ^ (1u << j);
    logq[t] = (uint16_t)(j | j << 8);
  }
}

// The LDS bytes of k_heap_pipe_pops: the heap's ranks P bits per node, node x
// at bit (x + 1) P (positions 0 .. n, whole words), and a spare word
__host__ __device__ constexpr uint32_t pipe_lds_bytes(uint32_t n, uint32_t P) {
  return ((n + 1) * P + 31) / 32 * 4 + 16;
}
// P: 8 when the heap fits in LDS a byte per node, else 1, 2, 4 for 2, <= 4,
// <= 16 distinct keys (the host checks that the packed heap fits)
// tailL > 0: only the levels above tailL in LDS (pipe_pops_tail)
__global__ void __launch_bounds__(256) k_heap_pipe_pops(uint8_t *R, uint32_t n, uint32_t P,
                                                       uint32_t tailL, uint32_t *logb,
                                                       uint16_t *logq, const uint32_t *mode) {
  extern __shared__ uint32_t lw[];
  if (mode[0] != HM_RANK) return;
  lds_u32 *LW = (lds_u32 *)lw;
  const uint32_t ntop = tailL ? (1u << tailL) - 1u : n;  // nodes in LDS
  const uint32_t per = 32 / P, nw = (pipe_lds_bytes(ntop, P) - 16) / 4;
  for (uint32_t q = threadIdx.x; q < nw; q += blockDim.x) {
    uint32_t v = 0;
    for (uint32_t i = 0; i < per; i += 4) {  // R holds n + 16 bytes
      const uint32_t p0 = q * per + i;
      const uint32_t r4 = p0 <= n ? *(const uint32_t *)(R + p0) : 0u;
#pragma unroll
      for (uint32_t b = 0; b < 4; ++b) {
        const uint32_t p = p0 + b;
        if (p >= 1 && p <= ntop) v |= ((r4 >> (8 * b)) & 0xffu) << ((i + b) * P);
      }
    }
    LW[q] = v;
  }
  if (threadIdx.x < 4) LW[nw + threadIdx.x] = 0;
  __syncthreads();
  if (threadIdx.x >= 64) return;
  lds_u8 *LB = (lds_u8 *)lw;
  const uint32_t HD = nw * per - 1;  // (HD + 1) P: the first spare word, nw
  if (tailL) {
    switch (P) {
      case 1: pipe_pops_tail<1>(LB, LW, R, n, tailL, HD, logb, threadIdx.x); break;
      case 2: pipe_pops_tail<2>(LB, LW, R, n, tailL, HD, logb, threadIdx.x); break;
      default: pipe_pops_tail<4>(LB, LW, R, n, tailL, HD, logb, threadIdx.x); break;
    }
    return;
  }
  switch (P) {
    case 1: pipe_pops<1>(LB, LW, n, HD, logb, logq, threadIdx.x); break;
    case 2: pipe_pops<2>(LB, LW, n, HD, logb, logq, threadIdx.x); break;
    case 4: pipe_pops<4>(LB, LW, n, HD, logb, logq, threadIdx.x); break;
    default: pipe_pops<8>(LB, LW, n, HD, logb, logq, threadIdx.x); break;
  }
}

__global__ void k_heap_pair_counts(const uint16_t *logq, uint32_t npop, uint32_t *cnt) {
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < npop + 1; t += gridDim.x * blockDim.x)
    cnt[t] = t < npop ? (uint32_t)(logq[t] >> 8) + 1u : 0u;
}
// the slots p_0..p_j pop t wrote: (node, pop) pairs at off[t]
__global__ void k_heap_pairs(const uint32_t *logb, const uint16_t *logq, const uint32_t *off,
                             uint32_t npop, uint32_t *key, uint32_t *val) {
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < npop; t += gridDim.x * blockDim.x) {
    const uint32_t b = logb[t], q = logq[t], D = q & 255u, j = q >> 8;
    uint32_t y = 0;
    const uint32_t o = off[t];
    for (uint32_t i = 0;; ++i) {
      key[o + i] = y;
      val[o + i] = t;
      if (i == j) break;
      y = 2 * y + 1 + ((b >> (D - 1 - i)) & 1u);
    }
  }
}
// first pair of every node y in [0, n] (the pairs sorted by node)
__global__ void k_heap_node_starts(const uint32_t *skey, uint32_t P, uint32_t n, uint32_t *noff) {
  for (uint32_t y = blockIdx.x * blockDim.x + threadIdx.x; y <= n; y += gridDim.x * blockDim.x) {
    uint32_t a = 0, b = P;
    while (a < b) {
      const uint32_t mid = a + (b - a) / 2;
      if (skey[mid] < y) a = mid + 1;
      else b = mid;
    }
    noff[y] = a;
  }
}
__global__ void k_heap_trace(const uint32_t *sval, const uint32_t *noff, const uint32_t *logb,
                             const uint16_t *logq, const uint32_t *T, uint32_t n, uint32_t *out) {
  for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < n; x += gridDim.x * blockDim.x) {
    uint32_t y = 0, t = n - 1 - x;  // position x is the root just before pop n - 1 - x
    for (;;) {
      const uint32_t lo = noff[y], hi = noff[y + 1];
      uint32_t a = lo, b = hi;  // the first of y's writers at or after t
      while (a < b) {
        const uint32_t mid = a + (b - a) / 2;
        if (sval[mid] < t) a = mid + 1;
        else b = mid;
      }
      if (a == lo) break;  // no pop before t wrote y
      const uint32_t tp = sval[a - 1];
      const uint32_t q = logq[tp], D = q & 255u, j = q >> 8;
      const uint32_t i = 31 - __clz(y + 1);  // y's depth: it is slot i of pop tp
      y = i < j ? 2 * y + 1 + ((logb[tp] >> (D - 1 - i)) & 1u) : n - 1 - tp;
      t = tp;
    }
    out[x] = T[y];
  }
}

// One stream-ordered allocation of the heap path; RK_HEAP_ALLOC_CAP (a test
// hook) fails every allocation above that many bytes, as HBM exhaustion would.
static hipError_t heap_alloc(void **p, size_t bytes, hipStream_t st) {
  static const size_t cap = [] {
    const char *e = getenv("RK_HEAP_ALLOC_CAP");
    return e ? (size_t)strtoull(e, nullptr, 10) : (size_t)0;
  }();
  *p = nullptr;
  if (cap && bytes > cap) return hipErrorOutOfMemory;
  return hipMallocAsync(p, bytes, st);
}
static int heap_status(hipError_t e) {
  return e == hipSuccess ? RK_OK : e == hipErrorOutOfMemory ? RK_E_NOMEM : RK_E_HIP;
}

// The queued heap segments (their number already read back), one after
// another: prep, then the path its keys take.  A rare path (only crafted
// inputs reach libstdc++'s depth limit on 2048+ members): its buffers are
// stream-ordered allocations of its own, and it waits for the device twice
// per rank-path segment to size them.  Returns RK_E_NOMEM when a buffer
// cannot be had (nothing is launched on a missing buffer; what was allocated
// is freed), RK_E_HIP on any other runtime failure.
static int heap_segments(const HeapSeg *dq, uint32_t nheap, uint64_t *key, uint32_t *tag,
                         uint32_t *otag, uint32_t *host_words, hipStream_t st) {
  std::vector<HeapSeg> q(nheap);
  hipError_t e = hipMemcpyAsync(q.data(), dq, nheap * sizeof(HeapSeg), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return RK_E_HIP;
  uint32_t nmax = 0;
  for (const HeapSeg &g : q) nmax = g.n > nmax ? g.n : nmax;
  constexpr uint32_t LDS_MAX = 160 * 1024 - 1024;
  static const bool attr = [] {
    (void)hipFuncSetAttribute((const void *)k_heap_rank_pops<false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_MAX);
    (void)hipFuncSetAttribute((const void *)k_heap_rank_pops<true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_MAX);
    (void)hipFuncSetAttribute((const void *)k_heap_pipe_pops,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_MAX);
    return true;
  }();
  (void)attr;
  // RK_HEAP_PIPE=0: the rank pops one after another (k_heap_rank_pops) only
  static const bool heap_pipe = [] {
    const char *s = getenv("RK_HEAP_PIPE");
    return !(s && s[0] == '0');
  }();
  // RK_HEAP_TAIL=0: no pipelined pops with the bottom level in global memory
  static const bool heap_tail = [] {
    const char *s = getenv("RK_HEAP_TAIL");
    return !(s && s[0] == '0');
  }();
  uint8_t *R = nullptr;
  uint32_t *logb = nullptr, *mode = nullptr, *cnt = nullptr, *off = nullptr, *ssb = nullptr;
  uint16_t *logq = nullptr;
  const size_t sscap = scan_blocks((size_t)nmax + 1) + 64;
  int rc = RK_OK;
  {
    void **bufs[7] = {(void **)&R, (void **)&logb, (void **)&logq, (void **)&mode, (void **)&cnt,
                      (void **)&off, (void **)&ssb};
    const size_t sizes[7] = {(size_t)nmax + 16, (size_t)nmax * 4 + 16, (size_t)nmax * 2 + 16, 16,
                             ((size_t)nmax + 1) * 4 + 16, ((size_t)nmax + 1) * 4 + 16, sscap * 4};
    for (int i = 0; i < 7 && !rc; ++i) rc = heap_status(heap_alloc(bufs[i], sizes[i], st));
  }
  for (size_t si = 0; si < q.size() && !rc; ++si) {
    const HeapSeg &g = q[si];
    const size_t o = (size_t)g.b + g.f;
    uint64_t *K = key + o;
    uint32_t *T = tag + o, *out = otag + o;
    const uint32_t n = g.n, RT = (LDS_MAX - 32) | 1u;  // (odd: no pair straddles)
    k_heap_prep<<<1, 256, 0, st>>>(K, T, n, R, mode);
    k_heap_equal<<<1, 64, 0, st>>>(T, n, out, mode);
    k_heap_general<<<1, 256, 0, st>>>(K, T, n, out, mode);
    e = hipMemcpyAsync(host_words, mode, 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if ((rc = heap_status(e))) break;
    if (host_words[0] != HM_RANK) continue;
    const uint32_t D = host_words[1];  // bits per node: a byte when the heap fits
    const uint32_t bpn = pipe_lds_bytes(n, 8) <= LDS_MAX ? 8u : D <= 2 ? 1u : D <= 4 ? 2u : 4u;
    // a heap too large: its levels above the bottom one in LDS, when they fit
    const uint32_t L = 31 - __builtin_clz(n), tailL =
        pipe_lds_bytes(n, bpn) > LDS_MAX && heap_tail && L >= 6 &&
                pipe_lds_bytes((1u << L) - 1u, bpn) <= LDS_MAX ? L : 0u;
    if (heap_pipe && (tailL || pipe_lds_bytes(n, bpn) <= LDS_MAX)) {  // the (packed) heap in LDS
      const uint32_t lds = pipe_lds_bytes(tailL ? (1u << L) - 1u : n, bpn);
      k_heap_pipe_pops<<<1, 256, lds, st>>>(R, n, bpn, tailL, logb, logq, mode);
      k_heap_log_split<<<grid_for(n, 256), 256, 0, st>>>(logb, logq, n - 1, mode);
    }
    else if (n + 16 <= LDS_MAX)  // the whole heap in LDS
      k_heap_rank_pops<false><<<1, 64, n + 16, st>>>(R, n, n, logb, logq, mode);
    else  // the top RT (odd) nodes in LDS
      k_heap_rank_pops<true><<<1, 64, RT + 16, st>>>(R, n, RT, logb, logq, mode);
    const uint32_t npop = n - 1;
    k_heap_pair_counts<<<grid_for(npop + 1, 256), 256, 0, st>>>(logq, npop, cnt);
    exclusive_scan_u32(cnt, off, (size_t)npop + 1, ScanScratch{ssb, sscap}, st);
    e = hipMemcpyAsync(host_words, off + npop, 4, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if ((rc = heap_status(e))) break;
    const uint32_t P = host_words[0];
    const size_t rw = radix_scratch_words(P);
    uint32_t *pk = nullptr, *pv = nullptr, *sk = nullptr, *sv = nullptr, *tk = nullptr,
             *tv = nullptr, *rs = nullptr, *noff = nullptr;
    for (uint32_t **b : {&pk, &pv, &sk, &sv, &tk, &tv})
      if (!rc) rc = heap_status(heap_alloc((void **)b, (size_t)P * 4 + 16, st));
    if (!rc) rc = heap_status(heap_alloc((void **)&rs, rw * 4, st));
    if (!rc) rc = heap_status(heap_alloc((void **)&noff, ((size_t)n + 2) * 4, st));
    if (!rc) {
      k_heap_pairs<<<grid_for(npop, 256), 256, 0, st>>>(logb, logq, off, npop, pk, pv);
      radix_sort_pairs(pk, pv, sk, sv, tk, tv, P, bit_length(n), rs, rw, st);
      k_heap_node_starts<<<grid_for(n + 1, 256), 256, 0, st>>>(sk, P, n, noff);
      k_heap_trace<<<grid_for(n, 256), 256, 0, st>>>(sv, noff, logb, logq, T, n, out);
    }
    for (uint32_t *b : {pk, pv, sk, sv, tk, tv, rs, noff})
      if (b) (void)hipFreeAsync(b, st);
  }
  for (void *b : {(void *)R, (void *)logb, (void *)logq, (void *)mode, (void *)cnt, (void *)off,
                  (void *)ssb})
    if (b) (void)hipFreeAsync(b, st);
  if (!rc && hipGetLastError() != hipSuccess) rc = RK_E_HIP;
  return rc;
}

// phase B: LDS layout of k_sort_groups_lds with a stack for any depth budget
__host__ __device__ constexpr size_t seg_lds_bytes(uint32_t cap, size_t key_bytes) {
  return (size_t)cap * (key_bytes + 4 + 2 + 2 + 1) +
         (SPLIT_STACK + 2 * (cap / (THRESH + 1) + 2)) * sizeof(Frame) + 16;
}
template <class KT, int WPB>
__global__ void __launch_bounds__(64 * WPB) k_sort_segments(TierLists tl, int tier, uint32_t m,
                                                            const uint8_t *bnd,
                                                            const uint32_t *head,
                                                            const uint64_t *key,
                                                            const uint32_t *tag, uint32_t *otag,
                                                            uint32_t reg_max, uint32_t slab,
                                                            const uint32_t *heapq_n,
                                                            uint32_t *heap_count, bool small_part) {
  // phase A's heap-segment count to the caller's word (read back with its own)
  if (heap_count && blockIdx.x == 0 && threadIdx.x == 0) *heap_count = *heapq_n;
  {
    uint32_t lo, hi;
    tl.range(tier, lo, hi);
    if (lo == hi) return;
  }
  extern __shared__ __align__(16) uint8_t smem_all[];
  constexpr uint32_t cap = SPLIT_T;
  // the wavefront index in a scalar register: every LDS base stays uniform
  const uint32_t lane = threadIdx.x & 63,
                 wv = WPB == 1 ? 0u : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t *smem = smem_all + (size_t)wv * slab;
  const uint32_t nfr = cap / (THRESH + 1) + 2;
  KT *K = reinterpret_cast<KT *>(smem);
  uint32_t *T = reinterpret_cast<uint32_t *>(K + cap);
  Frame *stack = reinterpret_cast<Frame *>(T + cap);
  Frame *smallq = stack + SPLIT_STACK;
  Frame *heapq = smallq + nfr;
  uint16_t *PL = reinterpret_cast<uint16_t *>(heapq + nfr);
  uint16_t *PR = PL + cap;
  uint8_t *B = reinterpret_cast<uint8_t *>(PR + cap);
  const ViewT<KT, uint16_t> v{K, T, PL, PR, B};
  for (uint32_t w0 = (blockIdx.x * WPB + wv) * 64; w0 < m; w0 += gridDim.x * WPB * 64) {
    uint64_t hb = __ballot(w0 + lane < m && bnd[w0 + lane] == 1);
    while (hb) {
      const uint32_t x = w0 + (uint32_t)__builtin_ctzll(hb);
      hb &= hb - 1;
      const uint32_t h = head[x], n = h & 0xFFFFu;
      for (uint32_t y = lane; y < n; y += 64) {
        K[y] = (KT)key[x + y];
        T[y] = tag[x + y];
      }
      wave_sync();
      wave_std_sort<false>(v, n, otag + x, stack, smallq, heapq, GLanes<64>{lane, 0u},
                           (int)(h >> 16), reg_max, 0u, small_part);
      wave_sync();
    }
  }
}

// Groups of 2..16 members (tier 0): __final_insertion_sort alone sorts them,
// so a member's final slot is its stable rank inside the group.  Sixteen
// lanes per group, four groups per wavefront: lane l loads member l (the
// group's members are contiguous), ranks itself against the other lanes of
// its segment by width-16 shuffles and writes its tag at its rank.
// Singletons are not listed and not written: emit_result takes a one-member
// group's slot as it is (tag[x] == x for every caller).
__global__ void __launch_bounds__(256) k_sort_small(TierLists tl, const uint32_t *goff,
                                                    const uint64_t *key, const uint32_t *tag,
                                                    uint32_t *otag) {
  uint32_t lo, hi;
  tl.range(0, lo, hi);
  const uint32_t l = threadIdx.x & 15;
  for (uint32_t w = lo + ((blockIdx.x * blockDim.x + threadIdx.x) >> 4); w - lo < hi - lo;
       w += (gridDim.x * blockDim.x) >> 4) {
    const uint32_t g = tl.list[w];
    const uint32_t b = goff[g], n = goff[g + 1] - b;
    const bool in = l < n;
    const uint64_t k = in ? key[b + l] : ~0ull;
    uint32_t r = 0;
#pragma unroll
    for (int j = 0; j < THRESH; ++j) {
      const uint64_t kj = __shfl(k, j, 16);
      r += (uint32_t)j < n && (kj < k || (kj == k && (uint32_t)j < l));
    }
    if (in) otag[b + r] = b + l;  // tags are positions
  }
}

// Tiers by group size (singletons: none): 0 = 2..16 members (k_sort_small), 1 =
// 17..32 (registers, two groups per wavefront), 2 = 33..64 (registers), 3..6
// = up to LDS_CAPS[t-3] (LDS), 7 = larger (global memory).  Small LDS caps
// keep many wavefronts resident per CU (a 65..128-member group needs ~3 KB of
// LDS, a 2048-member one ~30 KB).
constexpr int NTIER = GS_NTIER;
constexpr int NLDS = 4;
constexpr int TIER_LDS0 = 3;
static_assert(TIER_LDS0 + NLDS + 1 == NTIER, "tier layout");
struct Caps {
  uint32_t c[NLDS];
};
__host__ __device__ constexpr Caps lds_caps() { return Caps{{128, 256, 512, 2048}}; }

__device__ __forceinline__ int tier_of(uint32_t n) {
  constexpr Caps caps = lds_caps();
  if (n <= 1) return NTIER;  // a singleton: nothing to sort, nothing listed
  if (n <= (uint32_t)THRESH) return 0;
  if (n <= 32) return 1;
  if (n <= 64) return 2;
#pragma unroll
  for (int j = 0; j < NLDS; ++j)
    if (n <= caps.c[j]) return TIER_LDS0 + j;
  return NTIER - 1;
}

// Tier lists in two passes over the groups, TCH groups per block: count the
// listed tiers per block (and, for the timing accounts, their members), then
// -- after an exclusive scan of the tier-major block counts -- write every
// group at its tier's block offset + its rank in the block.
constexpr uint32_t TCH = 4096;
// (block 0 also zeroes the scan's end word bc[NTIER * nblk] and the three
// heap / claim counters of phase A: no clear launched for them)
__global__ void __launch_bounds__(256) k_tier_count(const uint32_t *goff, uint32_t ngroups,
                                                    uint32_t nblk, uint32_t *bc, uint32_t *bm,
                                                    uint32_t *heapq_n) {
  __shared__ uint32_t cnt[NTIER], mem[NTIER];
  if (blockIdx.x == 0 && threadIdx.x < 4) {
    if (threadIdx.x == 3) bc[(size_t)NTIER * nblk] = 0;
    else heapq_n[threadIdx.x] = 0;
  }
  if (threadIdx.x < NTIER) cnt[threadIdx.x] = mem[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t g0 = blockIdx.x * TCH, g1 = min(g0 + TCH, ngroups);
  uint32_t c[NTIER] = {}, mm[NTIER] = {};
  for (uint32_t g = g0 + threadIdx.x; g < g1; g += 256) {
    const uint32_t n = goff[g + 1] - goff[g];
    const int t = tier_of(n);
#pragma unroll
    for (int u = 0; u < NTIER; ++u) c[u] += t == u, mm[u] += t == u ? n : 0;
  }
#pragma unroll
  for (int u = 0; u < NTIER; ++u) {
    uint32_t v = c[u], x = mm[u];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off), x += __shfl_xor(x, off);
    if ((threadIdx.x & 63) == 0 && (v || x)) atomicAdd(&cnt[u], v), atomicAdd(&mem[u], x);
  }
  __syncthreads();
  if (threadIdx.x < NTIER) bc[(size_t)threadIdx.x * nblk + blockIdx.x] = cnt[threadIdx.x];
  if (bm && threadIdx.x < NTIER) bm[(size_t)threadIdx.x * nblk + blockIdx.x] = mem[threadIdx.x];
}

// (and, when the largest tier lists any group, bnd cleared for phase A: its
// segment starts, which phase B scans for over all m positions)
__global__ void __launch_bounds__(256) k_tier_lists(const uint32_t *goff, uint32_t ngroups,
                                                    uint32_t nblk, const uint32_t *off,
                                                    uint32_t *list, uint8_t *bnd, uint32_t m) {
  __shared__ uint32_t wc[4][NTIER];
  if (off[(size_t)(NTIER - 1) * nblk] != off[(size_t)NTIER * nblk]) {
    for (uint32_t x = (blockIdx.x * blockDim.x + threadIdx.x) * 16; x < m;
         x += gridDim.x * blockDim.x * 16) {
      if (x + 16 <= m) {
        *reinterpret_cast<uint4 *>(bnd + x) = make_uint4(0, 0, 0, 0);
      } else {
        for (uint32_t y = x; y < m; ++y) bnd[y] = 0;
      }
    }
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t run[NTIER];
#pragma unroll
  for (int u = 0; u < NTIER; ++u) run[u] = off[(size_t)u * nblk + blockIdx.x];
  const uint32_t g0 = blockIdx.x * TCH, g1 = min(g0 + TCH, ngroups);
  for (uint32_t c0 = g0; c0 < g1; c0 += 256) {
    const uint32_t g = c0 + threadIdx.x;
    const int t = g < g1 ? tier_of(goff[g + 1] - goff[g]) : 0;
    uint32_t rank = 0;
#pragma unroll
    for (int u = 0; u < NTIER; ++u) {
      const uint64_t b = __ballot(g < g1 && t == u);
      if (t == u) rank = __popcll(b & ((1ull << lane) - 1ull));
      if (lane == 0) wc[wv][u] = (uint32_t)__popcll(b);
    }
    __syncthreads();
    if (g < g1 && t < NTIER) {  // singletons are not listed
      uint32_t before = 0;
      for (int k = 0; k < wv; ++k) before += wc[k][t];
#pragma unroll
      for (int u = 0; u < NTIER; ++u)
        if (u == t) list[run[u] + before + rank] = g;
    }
#pragma unroll
    for (int u = 0; u < NTIER; ++u) run[u] += wc[0][u] + wc[1][u] + wc[2][u] + wc[3][u];
    __syncthreads();
  }
}

// keys, 16-bit tags, PL, PR, B, frames (the register-batch queue only when
// reg_max > 0: without it the 257..512 tier's slab is 6.3 KB, 25 resident
// wavefronts per CU instead of 23)
size_t lds_bytes(uint32_t cap, size_t key_bytes, uint32_t reg_max) {
  const uint32_t nfr = cap / (THRESH + 1) + 2;
  return (size_t)cap * (key_bytes + 2 + 2 + 2 + 1) +
         (lds_stack(cap) + (reg_max ? 2 : 1) * nfr) * sizeof(Frame) + 16;
}

}  // namespace

size_t groupsort_scratch_bytes(uint32_t n) {
  const size_t nblk = (size_t)n / TCH + 1;
  // pl, pr (stopper lists; segment heads); tier lists; bounds; block counts
  // (+ scan), block members
  return (size_t)n * 4 * 2 + ((size_t)n + 1) * 4 + (size_t)n + 128 +
         (nblk * NTIER + 1) * 4 * 2 + nblk * NTIER * 4 + 256 + 256 +
         (HEAPQ_CAP + 1) * sizeof(HeapSeg) + 64;
}

// the heap-segment queue inside sort_groups_exact's scratch (the layout below)
static HeapSeg *heap_queue(void *scratch, uint32_t m, uint32_t ngroups) {
  const uint32_t nblk = (ngroups + TCH - 1) / TCH;
  uint32_t *pl = reinterpret_cast<uint32_t *>(scratch);
  uint32_t *list = pl + 2 * (size_t)m;
  uint8_t *bnd = reinterpret_cast<uint8_t *>(
      (reinterpret_cast<uintptr_t>(list + ngroups + 1) + 15) & ~(uintptr_t)15);
  uint32_t *bc = reinterpret_cast<uint32_t *>(
      (reinterpret_cast<uintptr_t>(bnd + m) + 63) & ~(uintptr_t)63);
  uint32_t *bm = bc + 2 * ((size_t)NTIER * nblk + 1);
  return reinterpret_cast<HeapSeg *>(
      (reinterpret_cast<uintptr_t>(bm + (size_t)NTIER * nblk) + 63) & ~(uintptr_t)63);
}

// The heap segments of a sort_groups_exact call made with `heap_count`: their
// number was copied to heap_count, which the caller read back together with
// its own words; this sorts them (their tags into otag) afterwards.
int sort_groups_heap_deferred(uint32_t ngroups, uint32_t m, uint64_t *key, uint32_t *tag,
                              uint32_t *otag, void *scratch, uint32_t nheap,
                              uint32_t *host_words, hipStream_t st) {
  nheap = nheap < HEAPQ_CAP ? nheap : HEAPQ_CAP;
  if (!nheap) return RK_OK;
  return heap_segments(heap_queue(scratch, m, ngroups), nheap, key, tag, otag, host_words, st);
}

int sort_groups_exact(const uint32_t *gid_sorted, const uint32_t *goff, uint32_t ngroups,
                       uint32_t m, uint64_t *key, uint32_t *tag, uint32_t *otag, void *scratch,
                       ScanScratch ss, uint32_t *host_words, bool narrow_keys, hipStream_t st,
                       hipStream_t side, hipEvent_t ev_fork, hipEvent_t ev_join,
                       uint32_t *heap_count) {
  if (!m) {
    if (heap_count) (void)hipMemsetAsync(heap_count, 0, 4, st);
    return RK_OK;
  }
  int hrc = RK_OK;  // the heap segments' status (sorted here only without heap_count)
  constexpr int NL = NTIER;  // every tier is listed
  // groups of <= 64 members (k_sort_small, registers) run on `side`,
  // concurrently with the LDS tiers
  hipStream_t s2 = side ? side : st;
  constexpr Caps caps = lds_caps();
  const uint32_t nblk = (ngroups + TCH - 1) / TCH;
  uint32_t *pl = reinterpret_cast<uint32_t *>(scratch);
  uint32_t *pr = pl + m;
  uint32_t *list = pr + m;
  uint8_t *bnd = reinterpret_cast<uint8_t *>(
      (reinterpret_cast<uintptr_t>(list + ngroups + 1) + 15) & ~(uintptr_t)15);
  uint32_t *bc = reinterpret_cast<uint32_t *>(
      (reinterpret_cast<uintptr_t>(bnd + m) + 63) & ~(uintptr_t)63);
  uint32_t *boff = bc + (size_t)NL * nblk + 1;
  uint32_t *bm = boff + (size_t)NL * nblk + 1;
  HeapSeg *heapq = heap_queue(scratch, m, ngroups);  // (after bm's NL * nblk words)
  uint32_t *heapq_n = reinterpret_cast<uint32_t *>(heapq + HEAPQ_CAP);
  const bool timing = g_ktimer != nullptr;
  if (timing) {
    g_ktimer->tier_nblk = nblk;
    for (int u = 0; u < KernelTimer::TIERS; ++u) g_ktimer->tier_slot[u] = -1;
  }
  k_tier_count<<<nblk, 256, 0, st>>>(goff, ngroups, nblk, bc, timing ? bm : nullptr, heapq_n);
  exclusive_scan_u32(bc, boff, (size_t)NL * nblk + 1, ss, st);
  k_tier_lists<<<nblk, 256, 0, st>>>(goff, ngroups, nblk, boff, list, bnd, m);
  const TierLists tl{list, boff, nblk};
  // algorithmic bytes of every tier (timing only): each member's key read, its
  // tag (its position) written once at its final slot -- 12 B x the tier's members,
  // filled in from bm when the timings are collected
  if (timing && g_ktimer->only < 0) g_ktimer->tier_counts = bm;  // read back at collection
  auto tier_slot = [&](int u) {
    if (timing && g_ktimer->only < 0 && g_ktimer->n > 0) g_ktimer->tier_slot[u] = g_ktimer->n - 1;
  };
  // fixed grids: every kernel reads its list range on the device
  if (side) {
    (void)hipEventRecord(ev_fork, st);  // the tier lists are ready
    (void)hipStreamWaitEvent(s2, ev_fork, 0);
  }
  // segments of 17..reg_max members inside the LDS tiers would be finished in
  // registers (reg_batch); by default (0) the LDS partitions go down to the
  // leaves, which the vectorised final pass ranks -- LDS tiers 1.29 -> 1.25
  // ms at cfg3 (RK_GS_REGMAX=64 restores the register batches)
  static const uint32_t reg_max = [] {
    const char *e = getenv("RK_GS_REGMAX");
    return e ? (uint32_t)atoi(e) : 0u;
  }();
  // partitions of segments of <= 64 elements in registers
  // (wave_partition_small; RK_GS_SMALLPART=0: the stopper-list form)
  static const bool small_part = [] {
    const char *e = getenv("RK_GS_SMALLPART");
    return !(e && e[0] == '0');
  }();
  // the first `lds_side` LDS tiers also run on `side` (RK_GS_SIDE, measurements)
  static const int lds_side = [] {
    const char *e = getenv("RK_GS_SIDE");
    return e ? atoi(e) : 0;
  }();
  // the last `lds_big` LDS tiers (the largest groups: few, long wavefronts
  // that leave the device idle at the end of their own launch) run first on
  // `side`, under the smaller LDS tiers on `st` (RK_GS_BIG).  cfg3 group-sort
  // phase with 0 / 1 / 2 / 3 / 4 of them: 1.38-1.39 / 1.26 / 1.23-1.24 /
  // 1.40-1.41 / 1.57 ms
  static const int lds_big = [] {
    const char *e = getenv("RK_GS_BIG");
    const int b = e ? atoi(e) : 2;
    return b < 0 ? 0 : b > NLDS ? NLDS : b;
  }();
  // wavefronts per block of the LDS tiers up to 512 members (RK_GS_WPB: 1 or 4;
  // cfg3 group-sort phase 1.199-1.205 / 1.203-1.205 ms, neutral)
  static const int wpb = [] {
    const char *e = getenv("RK_GS_WPB");
    return e && atoi(e) == 4 ? 4 : 1;
  }();
  // LDS tiers up to `half_cap` members sort two groups per wavefront, one per
  // half (RK_GS_HALF: that cap; default 0 = whole wavefronts everywhere).
  // Measured at cfg3 with 256: LDS tiers 1.92-1.95 against 1.55 ms, group-sort
  // phase 1.28-1.29 against 1.14-1.18 ms -- slower, kept as an option
  static const uint32_t half_cap = [] {
    const char *e = getenv("RK_GS_HALF");
    return e ? (uint32_t)atoi(e) : 0u;
  }();
  auto launch_lds = [&](int j, hipStream_t sj) {
    const uint32_t cap = caps.c[j];
    // (more blocks than stay resident: a grid capped at the resident blocks, or
    // half of them, was slower -- group-sort phase 1.275 / 1.37 against 1.20 ms;
    // a larger one is faster, below)
    // x4 (RK_GS_WAVES_MUL): cfg3's group-sort phase 1.070 / 1.073 -> 1.027 /
    // 1.032 ms (x2: 1.032 / 1.037), the hardware balancing the static group
    // shares as wavefronts finish (`gpurun_out` r5gs)
    static const uint32_t gs_mul = [] {
      const char *e = getenv("RK_GS_WAVES_MUL");
      const int v = e ? atoi(e) : 4;
      return v > 0 ? (uint32_t)v : 1u;
    }();
    const uint32_t waves = (cap <= 256 ? 16384 : cap <= 512 ? 8192 : 2048) * gs_mul;
    const int wp = cap <= 512 ? wpb : 1;
    const size_t slab = (lds_bytes(cap, narrow_keys ? 4 : 8, reg_max) + 15) & ~(size_t)15;
    kt_begin(sj, KID_SORT_LDS);
    if (cap <= half_cap && 2 * slab <= 65536) {
      if (narrow_keys)
        k_sort_groups_lds<uint32_t, 1, 32><<<waves / 2, 64, 2 * slab, sj>>>(
            tl, TIER_LDS0 + j, goff, key, tag, otag, cap, 0u, (uint32_t)slab, small_part);
      else
        k_sort_groups_lds<uint64_t, 1, 32><<<waves / 2, 64, 2 * slab, sj>>>(
            tl, TIER_LDS0 + j, goff, key, tag, otag, cap, 0u, (uint32_t)slab, small_part);
    } else if (wp == 4) {
      if (narrow_keys)
        k_sort_groups_lds<uint32_t, 4><<<waves / 4, 256, 4 * slab, sj>>>(
            tl, TIER_LDS0 + j, goff, key, tag, otag, cap, reg_max, (uint32_t)slab, small_part);
      else
        k_sort_groups_lds<uint64_t, 4><<<waves / 4, 256, 4 * slab, sj>>>(
            tl, TIER_LDS0 + j, goff, key, tag, otag, cap, reg_max, (uint32_t)slab, small_part);
    } else {
      if (narrow_keys)
        k_sort_groups_lds<uint32_t, 1><<<waves, 64, slab, sj>>>(tl, TIER_LDS0 + j, goff, key, tag,
                                                                otag, cap, reg_max, (uint32_t)slab, small_part);
      else
        k_sort_groups_lds<uint64_t, 1><<<waves, 64, slab, sj>>>(tl, TIER_LDS0 + j, goff, key, tag,
                                                                otag, cap, reg_max, (uint32_t)slab, small_part);
    }
    kt_end(sj, KID_SORT_LDS, 0.0);
    tier_slot(TIER_LDS0 + j);
  };
  const int big0 = side ? NLDS - lds_big : NLDS;  // tiers [big0, NLDS) go first on side
  for (int j = NLDS - 1; j >= big0; --j) launch_lds(j, s2);
  // groups of 2..16 and 17..32 members: on `side` after its LDS tiers
  // (RK_GS_SMALL1=0, the default) or on `st` after the 33..64 tier (1).  With
  // 32-bit LDS tags the side stream's two large LDS tiers were the longer
  // chain and 1 was faster (group-sort phase 1.20 -> 1.13 ms); with 16-bit
  // tags (the 257..512 tier's slab 7.7 -> 6.7 KB: 24 resident wavefronts per
  // CU instead of 20) 0 is: 1.07-1.08 against 1.15 ms
  static const int small_main = [] {
    const char *e = getenv("RK_GS_SMALL1");
    return e ? atoi(e) : 0;
  }();
  auto launch_small = [&](hipStream_t sj) {
    kt_begin(sj, KID_SORT_SMALL);
    k_sort_small<<<2048, 256, 0, sj>>>(tl, goff, key, tag, otag);
    kt_end(sj, KID_SORT_SMALL, 0.0);  // bytes filled in from the tier sizes at collection
    tier_slot(0);
    kt_begin(sj, KID_SORT_REG);
    k_sort_groups_reg<2><<<4096, 256, 0, sj>>>(tl, 1, goff, key, tag, otag);
    kt_end(sj, KID_SORT_REG, 0.0);
    tier_slot(1);
  };
  if (!small_main || !side) launch_small(s2);
  // the 33..64-member tier on `st` after its LDS tiers (RK_GS_REG1=1, the
  // default) or on `side` (0): the two streams' kernel time is then ~1.06 /
  // ~1.0 ms instead of 0.94 / 1.12 (cfg3 kernel trace); group-sort phase
  // 1.23-1.24 -> 1.21 ms
  static const int reg1_main = [] {
    const char *e = getenv("RK_GS_REG1");
    return e ? atoi(e) : 1;
  }();
  auto launch_reg1 = [&](hipStream_t sj) {
    kt_begin(sj, KID_SORT_REG);
    k_sort_groups_reg<1><<<4096, 256, 0, sj>>>(tl, 2, goff, key, tag, otag);
    kt_end(sj, KID_SORT_REG, 0.0);
    tier_slot(2);
  };
  if (!reg1_main || !side) launch_reg1(s2);
  for (int pass = 0; pass < 2; ++pass) {
    if (pass == 1 && side) (void)hipEventRecord(ev_join, s2);
    for (int j = 0; j < big0; ++j) {
      if ((j < lds_side) != (pass == 0)) continue;
      launch_lds(j, pass == 0 ? s2 : st);
    }
  }
  if (reg1_main && side) launch_reg1(st);
  if (small_main && side) launch_small(st);
#ifdef RK_GS_PROF
  {
    unsigned long long h[8];
    (void)hipStreamSynchronize(st);
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_gs_prof), sizeof h);
    const double g = h[6] ? (double)h[6] : 1.0;
    fprintf(stderr, "GSPROF groups=%llu members/group %.1f cyc/group: stack %.0f partitions %.0f batches %.0f final %.0f | partitions/group %.2f batches/group %.2f\n",
            h[6], h[7] / g, h[0] / g, h[1] / g, h[2] / g, h[3] / g, h[4] / g, h[5] / g);
    void *p = nullptr;
    (void)hipGetSymbolAddress(&p, HIP_SYMBOL(g_gs_prof));
    (void)hipMemsetAsync(p, 0, sizeof h, st);
  }
#endif
  // phase A marks the final segments' starts in bnd (cleared first); both
  // kernels return at once when no group is that large
  // (bnd cleared by k_tier_lists, the heap count and the two claim counters by
  // k_tier_count)
  // RK_SPLIT_DYN=0: the static round-robin; RK_SPLIT_BIG: the first pass' size
  static const bool split_dyn = [] {
    const char *e = getenv("RK_SPLIT_DYN");
    return !(e && e[0] == '0');
  }();
  static const uint32_t split_big = [] {
    const char *e = getenv("RK_SPLIT_BIG");
    return e ? (uint32_t)atoi(e) : 65536u;
  }();
  // RK_SPLIT_GRID: blocks of phase A; RK_SPLIT_LDSPAD: LDS bytes reserved per
  // block beyond its own (fewer resident blocks: a larger L2 share each)
  static const uint32_t split_grid = [] {
    const char *e = getenv("RK_SPLIT_GRID");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? (uint32_t)v : 2048u;
  }();
  static const uint32_t split_pad = [] {
    const char *e = getenv("RK_SPLIT_LDSPAD");
    const int v = e ? atoi(e) : 0;
    return v > 0 && v <= 32768 ? (uint32_t)v : 0u;
  }();
  static const bool split_q = [] {
    const char *e = getenv("RK_SPLIT_Q");
    return !(e && e[0] == '0');
  }();
  kt_begin(st, KID_SORT_GLOBAL);
  {
    const uint32_t lds = split_pad + (split_q ? (uint32_t)sizeof(QPart) : 0u);
    auto kern = split_q ? k_sort_groups_split<true> : k_sort_groups_split<false>;
    kern<<<split_grid, 256, lds, st>>>(tl, NTIER - 1, goff, key, tag, otag, pl, pr, bnd, heapq_n,
                                       heapq, split_dyn ? heapq_n + 1 : nullptr, split_big);
  }
  kt_end(st, KID_SORT_GLOBAL, 0.0);
  tier_slot(NTIER - 1);
  // the heap segments (libstdc++'s depth-limit fallback on 2048+ members: a
  // median-of-three killer, never ordinary data): their number back to the
  // host, which sizes their buffers (RK_HEAP_RANK=0: every segment through
  // k_heap_segments, the one-block general / spine-ring pops)
  static const bool heap_rank = [] {
    const char *e = getenv("RK_HEAP_RANK");
    return !(e && e[0] == '0');
  }();
  kt_begin(st, KID_SORT_HEAP);
  if (heap_rank && heap_count) {
    // the caller reads the count back with its own words (k_sort_segments
    // copies it there)
  } else if (heap_rank) {
    (void)hipMemcpyAsync(host_words, heapq_n, 4, hipMemcpyDeviceToHost, st);
    (void)hipStreamSynchronize(st);
    const uint32_t nheap = host_words[0] < HEAPQ_CAP ? host_words[0] : HEAPQ_CAP;
    if (nheap) hrc = heap_segments(heapq, nheap, key, tag, otag, host_words, st);
  } else {
    k_heap_segments<<<64, 256, 0, st>>>(heapq_n, heapq, key, tag, otag);
  }
  kt_end(st, KID_SORT_HEAP, 0.0);
  kt_begin(st, KID_SORT_SEGS);
  {
    const size_t slab = (seg_lds_bytes(SPLIT_T, narrow_keys ? 4 : 8) + 15) & ~(size_t)15;
    if (wpb == 4) {
      if (narrow_keys)
        k_sort_segments<uint32_t, 4><<<2048, 256, 4 * slab, st>>>(
            tl, NTIER - 1, m, bnd, pl, key, tag, otag, reg_max, (uint32_t)slab, heapq_n,
            heap_rank ? heap_count : nullptr, small_part);
      else
        k_sort_segments<uint64_t, 4><<<2048, 256, 4 * slab, st>>>(
            tl, NTIER - 1, m, bnd, pl, key, tag, otag, reg_max, (uint32_t)slab, heapq_n,
            heap_rank ? heap_count : nullptr, small_part);
    } else {
      // Each wavefront scans a fixed 1/grid of the positions: a grid many
      // times the resident wavefronts (~19 per CU) lets the hardware balance
      // the segments' uneven work as wavefronts finish -- one wavefront per
      // 8192 members, 8192 .. 131072 (cfg5: 8192 -> 131072 wavefronts, phase
      // B 47.6 -> 38.5 ms; cfg3 has no phase B).  RK_SEG_WAVES: a fixed grid
      static const int seg_env = [] {
        const char *e = getenv("RK_SEG_WAVES");
        return e ? atoi(e) : 0;
      }();
      const int seg_waves =
          seg_env > 0 ? seg_env : (int)std::min(131072u, std::max(8192u, m / 8192));
      if (narrow_keys)
        k_sort_segments<uint32_t, 1><<<seg_waves, 64, slab, st>>>(
            tl, NTIER - 1, m, bnd, pl, key, tag, otag, reg_max, (uint32_t)slab, heapq_n,
            heap_rank ? heap_count : nullptr, small_part);
      else
        k_sort_segments<uint64_t, 1><<<seg_waves, 64, slab, st>>>(
            tl, NTIER - 1, m, bnd, pl, key, tag, otag, reg_max, (uint32_t)slab, heapq_n,
            heap_rank ? heap_count : nullptr, small_part);
    }
  }
  kt_end(st, KID_SORT_SEGS, 0.0);
  tier_slot(NTIER);
  if (side) (void)hipStreamWaitEvent(st, ev_join, 0);
  return hrc;
}

}  // namespace rk
