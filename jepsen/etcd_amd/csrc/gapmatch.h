// gapmatch.h — the gap tier's matching of gaps to optional ops (one wave,
// over compact per-gap / per-op arrays in LDS or a global-memory workspace),
// shared by the gap tier (gap_tier.hip) and the version-order tier's
// in-place decision of crash-light keys (check_kernel.hip).  The procedure
// and its exactness argument are in gap_tier.hip's header.
#pragma once
#include <climits>
#include <type_traits>

#include "kernels.h"
#include "records.h"
#include "wave.h"

namespace lcdev {
namespace {

constexpr int kAny = INT_MIN;      // no value required / not a CAS
constexpr int kNodeBudget = 4096;  // matching passes per decision
constexpr int kMaxCls = 64;        // class-indexed matching: at most one class per lane
constexpr int kClsMinOps = 128;    // ... used from this many optional ops on

enum { GD_VALID = 1, GD_INVALID = 0, GD_NA = -1, GD_BUDGET = -2, GD_SKIP = -3, GD_RETRY = -4 };

// Matching footprint of one decision in LDS: per gap a 16-byte record and 5
// ints, per op a 16-byte record and 7 ints, and the class table.
__host__ __device__ constexpr int match_lds_bytes(int G, int n_opt) {
  return 36 * G + 44 * n_opt + 16 * kMaxCls + 16;  // (+16: the table's alignment)
}

// ---------------------------------------------------------------------------
// The matching, over compact arrays.  Per gap gi a 16-byte record (deadline
// D: ops called at or after it cannot fill the gap; value requirement R;
// value before the gap B, kAny when the position before is a free gap;
// position P), the matched op and the DFS stack (gap, resume op, chosen op).
// Per optional op o a 16-byte record (call C, value V, expectation E = kAny
// for a write, pinned position OP = -1 for a crashed op), the matched gap
// and a visit stamp.  In LDS when L (tight, sized by G and n_opt), else in
// the workspace.
// Class-indexed matching (CM, below) adds per gap the head of its list of
// pinned optional ops, per op its class, its rank in the class and the next
// pinned op of its gap, and the ops grouped by class (CL) with their calls
// (CLc: a cursor's head op and call load together).
enum { aMG, aSG, aSR, aSO, aPH, aMO, aVis, aCls, aRank, aPN, aCL, aCLc };
constexpr int kGapInts = aMO;           // int arrays per gap
constexpr int kOpInts = aCLc + 1 - aMO;  // int arrays per op

// The LDS placement addresses the kernel's dynamic shared memory directly
// (lds_dyn + moff, never a pointer held in the struct): in the matching
// functions the compiler does not inline, a generic pointer loaded from the
// struct would turn every LDS access into a flat_* one.
extern __shared__ int4 lds_dyn[];

template <bool L>
struct Cmp {
  int32_t *ws;   // workspace base (HBM fallback)
  int G, n_opt;
  int cap;
  int moff;      // LDS: int4 offset of the region in lds_dyn
  // LDS: gap records [0, 16G), op records [16G, 16(G+n_opt)), then the
  // int arrays MG SG SR SO PH (G each), MO Vis Cls Rank PN CL (n_opt each),
  // then the class table (kMaxCls 16-byte entries).
  // HBM: Opt at array 10, gap records at 14, int arrays at 18..29, the class
  // table at 30 (class mode needs cap >= 4 * kMaxCls there).
  __device__ __forceinline__ int4 * gaps() const {
    if constexpr (L)
      return lds_dyn + moff;
    else
      return reinterpret_cast<int4 *>(ws + 14 * cap);
  }
  __device__ __forceinline__ int4 * ops() const {
    if constexpr (L)
      return lds_dyn + moff + G;
    else
      return reinterpret_cast<int4 *>(ws + 10 * cap);
  }
  __device__ __forceinline__ int &at(int a, int i) const {
    if constexpr (L) {
      int *b = reinterpret_cast<int *>(lds_dyn + moff + G + n_opt);
      return b[a < aMO ? a * G + i : kGapInts * G + (a - aMO) * n_opt + i];
    } else {
      return ws[(18 + a) * cap + i];
    }
  }
  // class table: x = value, y = expectation, z = first slot in CL, w = size
  __device__ __forceinline__ int4 * cls() const {
    if constexpr (L)
      return lds_dyn + moff + G + n_opt + (kGapInts * G + kOpInts * n_opt + 3) / 4;
    else
      return reinterpret_cast<int4 *>(ws + 30 * cap);
  }
};

// gap record: x = D, y = R, z = B, w = P;  op record: x = C, y = V, z = E, w = OP
// (bitwise, no short-circuit: the wave's loops stay uniform, see below)
__device__ __forceinline__ bool elig(const int4 gp, const int4 op) {
  return ((uint32_t)op.x < (uint32_t)gp.x) & ((op.w == -1) | (op.w == gp.w)) &
         ((gp.y == kAny) | (op.y == gp.y)) & ((op.z == kAny) | (gp.z == kAny) | (op.z == gp.z));
}

// The matching runs on one wave.  Its loops are written so the compiler
// keeps them uniform (SGPR counters, scalar branches): loop variables pass
// through readfirstlane (uni), and lane predicates are branch-free over
// clamped indices — a short-circuit `o < n && a[o] ...` makes the loop a
// divergent exec-mask loop and costs several times the instructions.

// Stores of the matching arrays must be visible to the wave's later loads
// from other lanes.  In LDS a wave's DS instructions execute in order, so a
// compiler barrier is enough; in the HBM fallback wait for the stores
// (same CU, so L1-coherent).
template <bool L>
__device__ __forceinline__ void match_fence() {
  if constexpr (L)
    __asm__ volatile("" ::: "memory");
  else
    wave_fence();
}

// One chunk of 64 ops from `base` against gap record gp: bit l of *hit = op
// base+l is eligible (and free / unvisited per `pred`); returns false when
// the chunk reaches the gap's deadline (ops are sorted by call: none later
// can be eligible).
template <bool L, class Pred>
__device__ __forceinline__ bool scan_chunk(const Cmp<L> &c, const int4 gp, int base, int n_opt,
                                           Pred pred, uint64_t *hit) {
  const int lane = threadIdx.x & (kWave - 1);
  const int o = base + lane, oc = min(o, n_opt - 1);
  const int4 op = c.ops()[oc];
  const bool in = o < n_opt;
  const bool before = in & ((uint32_t)op.x < (uint32_t)gp.x);
  const bool e = elig(gp, op);
  const bool ok = pred(oc);
  *hit = __ballot(before & e & ok);
  return __ballot(before) == ~0ull;  // every op of the chunk is before the deadline
}

#ifdef GAP_PROFILE
// matching counters of workgroups 0..3: first-fits, augments, augment steps,
// failed augments, nodes
__device__ unsigned long long g_mprof[4][8];
#define MPROF(i, v) \
  do { if (blockIdx.x < 4 && (threadIdx.x & 63) == 0) g_mprof[blockIdx.x][i] += (v); } while (0)
#else
#define MPROF(i, v) do { } while (0)
#endif

// First free op eligible for gap gi (or -1); *ff = first possibly-free op.
template <bool L>
__device__ int first_fit(const Cmp<L> &c, int gi, int n_opt, int *ff) {
  const int lane = threadIdx.x & (kWave - 1);
  const int4 gp = uni4(c.gaps()[gi]);
  int base = uni(*ff);
  auto free_op = [&](int oc) { return c.at(aMO, oc) == -1; };
  for (bool first = true; base < n_opt; base = uni(base + kWave), first = false) {
    if (first) {  // advance *ff past the matched prefix with the same chunk
      const int o = base + lane;
      const uint64_t fb = __ballot((o < n_opt) & free_op(min(o, n_opt - 1)));
      *ff = fb ? uni(base + first_lane(fb)) : uni(base + kWave);
    }
    uint64_t hit;
    const bool more = scan_chunk(c, gp, base, n_opt, free_op, &hit);
    if (hit) return uni(base + first_lane(hit));
    if (!more) break;
  }
  return -1;
}

// Depth-first augmenting path from the unmatched gap g0 (Kuhn).  Ops
// visited in this search carry `stamp`.  True iff g0 was matched.
template <bool L>
__device__ bool augment(const Cmp<L> &c, int g0, int n_opt, int stamp) {
  const int lane = threadIdx.x & (kWave - 1);
  int depth = 0, g = uni(g0), base = 0;
  auto unvisited = [&](int oc) { return c.at(aVis, oc) != stamp; };
  for (;;) {
    MPROF(2, 1);
    const int4 gp = uni4(c.gaps()[g]);
    int found = -1;
    for (; base < n_opt; base = uni(base + kWave)) {
      uint64_t hit;
      const bool more = scan_chunk(c, gp, base, n_opt, unvisited, &hit);
      if (hit) {
        found = uni(base + first_lane(hit));
        break;
      }
      if (!more) break;
    }
    if (found < 0) {  // dead end: back to the previous gap
      if (depth == 0) return false;
      depth--;
      g = uni(c.at(aSG, depth));
      base = uni(c.at(aSR, depth));
      continue;
    }
    c.at(aSG, depth) = g;
    c.at(aSR, depth) = found + 1;
    c.at(aSO, depth) = found;
    c.at(aVis, found) = stamp;
    const int m = uni(c.at(aMO, found));
    if (m == -1) {  // flip the path
      match_fence<L>();
      for (int d0 = 0; d0 <= depth; d0 += kWave) {
        const int d = d0 + lane;
        if (d <= depth) {
          const int gg = c.at(aSG, d), oo = c.at(aSO, d);
          c.at(aMG, gg) = oo;
          c.at(aMO, oo) = gg;
        }
      }
      match_fence<L>();
      return true;
    }
    depth++;
    g = m;
    base = 0;
  }
}

// ---------------------------------------------------------------------------
// Class-indexed matching (many optional ops).  The eligibility of an op for
// a gap depends only on its call (before the gap's deadline), its class
// (value, expectation) and, for the few optional ops pinned to a position
// (pending :ok mutations of a prefix), that position.  The unpinned ops of
// one class are kept in call order (CL), so for any gap the eligible ops of
// a class are a prefix of its list.  Lane k holds class k with two cursors:
//   f  the first free op of the class (first-fit),
//   p  the first op not yet visited by the current augmenting search
// (visits are always a prefix of each class list, because the search takes
// each class's ops in call order).  The first free (unvisited) eligible op
// in call order — what the chunked scans above find — is then the
// smallest-call head among the compatible classes plus the gap's pinned
// list: one ballot and a wave min per step instead of a scan over every op
// before the deadline.  The exploration order, hence the matching, equals
// the scans' exactly.
struct ClsSt {
  int K;                 // classes (uniform)
  int any_pin;           // some optional op is pinned to a position (uniform)
  int V, E, start, n;    // lane k: class k's value, expectation, CL slots
  int f, p;              // lane k: free / visit cursor
  int fo, po;            // lane k: the op at each cursor (-1 past the end) ...
  uint32_t fc, pc;       // ... and its call (kNever past the end)
};


// The op at slot i of this lane's class list and its call.
template <bool L>
__device__ __forceinline__ void cls_head(const Cmp<L> &c, const ClsSt &st, int i, int *o,
                                         uint32_t *call) {
  if (i < st.n) {
    *o = c.at(aCL, st.start + i);
    *call = (uint32_t)c.at(aCLc, st.start + i);
  } else {
    *o = -1;
    *call = kNever;
  }
}

// Build the class table, ranks, CL and the pinned lists (wave 0).  Returns
// the number of classes, or -1 when there are more than kMaxCls.
template <bool L>
__device__ int build_classes(const Cmp<L> &c, int G, int n_opt, ClsSt &st) {
  const int lane = threadIdx.x & (kWave - 1);
  const auto tab = c.cls();
  const auto ops = c.ops();
  int K = 0, cnt = 0;
  uint64_t any_pin = 0;
  for (int gi = lane; gi < G; gi += kWave) c.at(aPH, gi) = -1;
  for (int base = 0; base < n_opt; base = uni(base + kWave)) {
    const int o = base + lane, oc = min(o, n_opt - 1);
    const bool in = o < n_opt;
    const int4 op = ops[oc];
    const bool pinned = op.w != -1;
    any_pin |= __ballot(in & pinned);
    int cid = -1;
    for (int k = 0; k < K; k++) {
      const int4 t = uni4(tab[k]);
      cid = ((op.y == t.x) & (op.z == t.y)) ? k : cid;
    }
    if (pinned) cid = -1;
    for (uint64_t need = __ballot(in & !pinned & (cid == -1)); need;
         need = __ballot(in & !pinned & (cid == -1))) {
      if (K == kMaxCls) return -1;
      const int l = first_lane(need);
      const int V = __builtin_amdgcn_readlane(op.y, l), E = __builtin_amdgcn_readlane(op.z, l);
      if (lane == 0) tab[K] = make_int4(V, E, 0, 0);
      cid = (in & !pinned & (op.y == V) & (op.z == E)) ? K : cid;
      K = uni(K + 1);
    }
    match_fence<L>();
    // ranks within each class, in call order
    for (uint64_t todo = __ballot(in & (cid >= 0)); todo;) {
      const int k = uni(__builtin_amdgcn_readlane(cid, first_lane(todo)));
      const uint64_t m = __ballot(in & (cid == k));
      const int before = uni(__builtin_amdgcn_readlane(cnt, k));
      if (in & (cid == k)) c.at(aRank, o) = before + lanes_below(m);
      if (lane == k) cnt += __popcll(m);
      todo &= ~m;
    }
    if (in) c.at(aCls, o) = pinned ? -1 : cid;
  }
  // class slots: exclusive prefix of the counts over the lanes
  int incl = lane < K ? cnt : 0;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  st.K = K;
  st.any_pin = any_pin != 0;
  st.n = lane < K ? cnt : 0;
  st.start = incl - st.n;
  st.f = st.p = 0;
  if (lane < K) {
    const int4 t = tab[lane];
    st.V = t.x;
    st.E = t.y;
    tab[lane] = make_int4(t.x, t.y, st.start, st.n);
  } else {
    st.V = st.E = kAny;
  }
  match_fence<L>();
  // CL, and the pinned ops onto their gap's list (gaps are sorted by
  // position: binary search)
  const auto gaps = c.gaps();
  for (int base = 0; base < n_opt; base = uni(base + kWave)) {
    const int o = base + lane, oc = min(o, n_opt - 1);
    const int k = c.at(aCls, oc);
    const int kst = __shfl(st.start, max(k, 0));  // (every lane: bpermute from active lanes)
    if ((o < n_opt) & (k >= 0)) {
      const int slot = kst + c.at(aRank, o);
      c.at(aCL, slot) = o;
      c.at(aCLc, slot) = ops[o].x;
    }
    if (!st.any_pin) continue;
    const int pos = ops[oc].w;
    int gi = -1;
    if ((o < n_opt) & (pos != -1)) {
      int lo = 0, hi = G;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (gaps[mid].w < pos) lo = mid + 1; else hi = mid;
      }
      gi = (lo < G && gaps[lo].w == pos) ? lo : -1;
    }
    // one op at a time onto its gap's list (lists never race)
    for (uint64_t todo = __ballot(gi >= 0); todo; todo &= todo - 1) {
      const int l = first_lane(todo);
      const int g = uni(__builtin_amdgcn_readlane(gi, l)), q = uni(base + l);
      if (lane == 0) {
        c.at(aPN, q) = c.at(aPH, g);
        c.at(aPH, g) = q;
      }
      match_fence<L>();
    }
  }
  match_fence<L>();
  cls_head(c, st, 0, &st.fo, &st.fc);
  st.po = st.fo;
  st.pc = st.fc;
  return K;
}

__device__ __forceinline__ bool cls_compat(const ClsSt &st, const int4 gp) {
  const int lane = threadIdx.x & (kWave - 1);
  return (lane < st.K) & ((gp.y == kAny) | (st.V == gp.y)) &
         ((st.E == kAny) | (gp.z == kAny) | (st.E == gp.z));
}

// Preference key of this lane's free head for gap gp (kNever: not
// eligible): CAS classes before write classes, then the earliest call.  A
// write fits any value before the gap, a CAS only its expectation, so
// spending the CAS where it fits keeps the writes for the gaps only they
// can fill (C4: 93 -> 49 augmenting searches; the augmenting search itself
// takes ops in plain call order).  Any choice is exact: the matching's
// augmenting paths repair it.
__device__ __forceinline__ uint32_t cls_key(const ClsSt &st, const int4 gp, uint32_t head_call) {
  if (!(cls_compat(st, gp) & (head_call < (uint32_t)gp.x))) return kNever;
  return st.E == kAny ? (head_call | 0x80000000u) : head_call;
}

// First free eligible op for gap gi in call order (class heads and the gap's
// pinned list), or -1.  The caller matches it: its class's free cursor moves
// on at once.
template <bool L>
__device__ int first_fit_cls(const Cmp<L> &c, int gi, ClsSt &st) {
  const int lane = threadIdx.x & (kWave - 1);
  const int4 gp = uni4(c.gaps()[gi]);
  const auto ops = c.ops();
  // a head matched since (the end of an augmenting path): move on
  while (st.fo >= 0 && c.at(aMO, st.fo) != -1) {
    st.f++;
    cls_head(c, st, st.f, &st.fo, &st.fc);
  }
  uint32_t call = cls_key(st, gp, st.fc);
  int o = st.fo;
  if (st.any_pin) {
    for (int q = uni(c.at(aPH, gi)); q >= 0; q = uni(c.at(aPN, q))) {
      const int4 op = uni4(ops[q]);
      if (uni(c.at(aMO, q)) == -1 && elig(gp, op) && (uint32_t)op.x < call) {
        call = (uint32_t)op.x;  // lanes whose class head is later take it
        o = q;
      }
    }
  }
  const uint32_t best = wave_min_u32(call);
  if (best == kNever) return -1;
  const int wl = first_lane(__ballot(call == best));
  const int found = uni(__builtin_amdgcn_readlane(o, wl));
  if (lane == wl && found == st.fo) {
    st.f++;
    cls_head(c, st, st.f, &st.fo, &st.fc);
  }
  return found;
}

// Augmenting path from the unmatched gap g0 over the class cursors.
template <bool L>
__device__ bool augment_cls(const Cmp<L> &c, int g0, int stamp, ClsSt &st) {
  const int lane = threadIdx.x & (kWave - 1);
  const auto ops = c.ops();
  st.p = 0;
  cls_head(c, st, 0, &st.po, &st.pc);
  // free cursors past the ops matched since they last moved (nothing is
  // matched or freed during the search itself)
  while (st.fo >= 0 && c.at(aMO, st.fo) != -1) {
    st.f++;
    cls_head(c, st, st.f, &st.fo, &st.fc);
  }
  int depth = 0, g = uni(g0);
  for (;;) {
    MPROF(2, 1);
    const int4 gp = uni4(c.gaps()[g]);
    const bool compat = cls_compat(st, gp);
    // lookahead: a free eligible op ends the path here (Kuhn's search would
    // reach it only after exhausting the matched ops called before it)
    uint32_t fcall = cls_key(st, gp, st.fc);
    int fop = st.fo;
    if (st.any_pin) {
      for (int q = uni(c.at(aPH, g)); q >= 0; q = uni(c.at(aPN, q))) {
        const int4 op = uni4(ops[q]);
        if (uni(c.at(aMO, q)) == -1 && elig(gp, op) && (uint32_t)op.x < fcall) {
          fcall = (uint32_t)op.x;
          fop = q;
        }
      }
    }
    const uint32_t fbest = wave_min_u32(fcall);
    if (fbest != kNever) {
      const int free_op = uni(__builtin_amdgcn_readlane(fop, first_lane(__ballot(fcall == fbest))));
      c.at(aSG, depth) = g;
      c.at(aSO, depth) = free_op;
      match_fence<L>();
      for (int d0 = 0; d0 <= depth; d0 += kWave) {
        const int d = d0 + lane;
        if (d <= depth) {
          const int gg = c.at(aSG, d), oo = c.at(aSO, d);
          c.at(aMG, gg) = oo;
          c.at(aMO, oo) = gg;
        }
      }
      match_fence<L>();
      return true;
    }
    uint32_t call = (compat & (st.pc < (uint32_t)gp.x)) ? st.pc : kNever;
    int o = st.po;
    if (st.any_pin) {
      for (int q = uni(c.at(aPH, g)); q >= 0; q = uni(c.at(aPN, q))) {
        const int4 op = uni4(ops[q]);
        if (uni(c.at(aVis, q)) != stamp && elig(gp, op) && (uint32_t)op.x < call) {
          call = (uint32_t)op.x;
          o = q;
        }
      }
    }
    const uint32_t best = wave_min_u32(call);
    if (best == kNever) {  // dead end: back to the previous gap
      if (depth == 0) return false;
      depth--;
      g = uni(c.at(aSG, depth));
      continue;
    }
    const int wl = first_lane(__ballot(call == best));
    const int found = uni(__builtin_amdgcn_readlane(o, wl));
    const int head = uni(__builtin_amdgcn_readlane(st.po, wl));
    if (found != head) {
      c.at(aVis, found) = stamp;  // a pinned op
    } else if (lane == wl) {      // visited: the class's visit cursor moves past it
      st.p++;
      cls_head(c, st, st.p, &st.po, &st.pc);
    }
    c.at(aSG, depth) = g;
    c.at(aSO, depth) = found;
    const int m = uni(c.at(aMO, found));
    if (m == -1) {  // flip the path
      match_fence<L>();
      for (int d0 = 0; d0 <= depth; d0 += kWave) {
        const int d = d0 + lane;
        if (d <= depth) {
          const int gg = c.at(aSG, d), oo = c.at(aSO, d);
          c.at(aMG, gg) = oo;
          c.at(aMO, oo) = gg;
        }
      }
      match_fence<L>();
      return true;
    }
    depth++;
    g = m;
  }
}

// Fill every unmatched gap (first-fit, else an augmenting path).  False as
// soon as one cannot be filled: no matching covers all gaps (once no path
// leaves a gap, none ever will in Kuhn's algorithm).
template <bool L, bool CM>
__device__ bool fill(const Cmp<L> &c, int G, int n_opt, int *ff, int *stamp, ClsSt &st) {
  const int lane = threadIdx.x & (kWave - 1);
  for (int g0 = 0; g0 < G; g0 = uni(g0 + kWave)) {
    const int gl = g0 + lane;
    uint64_t todo = __ballot((gl < G) & (c.at(aMG, min(gl, G - 1)) == -1));
    while (todo) {
      const int gi = uni(g0 + first_lane(todo));
      todo &= todo - 1;
      int o;
      MPROF(0, 1);
      if constexpr (CM)
        o = first_fit_cls(c, gi, st);
      else
        o = first_fit(c, gi, n_opt, ff);
      if (o >= 0) {
        c.at(aMG, gi) = o;
        c.at(aMO, o) = gi;
        match_fence<L>();
        continue;
      }
      *stamp = uni(*stamp + 1);
      MPROF(1, 1);
      bool ok;
      if constexpr (CM)
        ok = augment_cls(c, gi, *stamp, st);
      else
        ok = augment(c, gi, n_opt, *stamp);
      if (!ok) {
        MPROF(3, 1);
        return false;
      }
    }
  }
  return true;
}

// Smallest value > last among the ops eligible for gap gi (INT_MAX if none).
template <bool L, bool CM>
__device__ int next_value(const Cmp<L> &c, int gi, int last, int n_opt, const ClsSt &st) {
  const int lane = threadIdx.x & (kWave - 1);
  const int4 gp = uni4(c.gaps()[gi]);
  const auto ops = c.ops();
  int best = INT_MAX;
  if constexpr (CM) {
    // a class has an eligible op iff its earliest op is called in time
    if (cls_compat(st, gp) & (st.n > 0) & (st.V > last)) {
      if ((uint32_t)c.at(aCLc, st.start) < (uint32_t)gp.x) best = st.V;
    }
    for (int q = uni(c.at(aPH, gi)); q >= 0; q = uni(c.at(aPN, q))) {
      const int4 op = uni4(ops[q]);
      if (elig(gp, op) && op.y > last) best = min(best, op.y);
    }
  } else {
    for (int base = 0; base < n_opt; base = uni(base + kWave)) {
      const int o = base + lane;
      const int4 op = ops[min(o, n_opt - 1)];
      const bool before = (o < n_opt) & ((uint32_t)op.x < (uint32_t)gp.x);
      const bool e = elig(gp, op);
      best = (before & e & (op.y > last)) ? min(best, op.y) : best;
      if (__ballot(before) != ~0ull) break;  // the deadline falls in this chunk
    }
  }
  return uni(wave_min_i32(best));
}

// Set gap gi's value requirement to v (kAny = free), with the value-before
// of the gap after it, and unmatch the pairs this makes ineligible.  *ff (or
// the class's free cursor) is lowered to any op freed.
template <bool L, bool CM>
__device__ void set_req(const Cmp<L> &c, int gi, int v, int G, int *ff, ClsSt &st) {
  const int lane = threadIdx.x & (kWave - 1);
  const auto gaps = c.gaps();
  reinterpret_cast<int *>(&gaps[gi])[1] = v;
  const bool next = gi + 1 < G && uni(gaps[gi + 1].w) == uni(gaps[gi].w) + 1;
  if (next) reinterpret_cast<int *>(&gaps[gi + 1])[2] = v;
  match_fence<L>();
  for (int k = 0; k < (next ? 2 : 1); k++) {
    const int g = gi + k;
    const int o = uni(c.at(aMG, g));
    if (o < 0) continue;
    if (!elig(uni4(gaps[g]), uni4(c.ops()[o]))) {
      c.at(aMG, g) = -1;
      c.at(aMO, o) = -1;
      if constexpr (CM) {
        const int k2 = uni(c.at(aCls, o));
        if (k2 >= 0 && lane == k2) {
          const int rk = c.at(aRank, o);
          if (rk < st.f) {
            st.f = rk;
            st.fo = o;
            st.fc = (uint32_t)c.ops()[o].x;
          }
        }
      } else {
        *ff = uni(min(*ff, o));
      }
      match_fence<L>();
    }
  }
}

// Decide the gap filling by matching plus depth-first branching on the
// values of free gaps that a matched CAS depends on.  Wave 0 only.  The
// branch stack (gap, value) lives in the skeleton's Claim / Req arrays,
// free once the compact arrays are built.
template <bool L, bool CM, class P>
__device__ int match_branch_m(const Cmp<L> &c, int G, int n_opt, P brPos, P brVal,
                              int64_t *nodes, ClsSt &st) {
  const int lane = threadIdx.x & (kWave - 1);
  const auto gaps = c.gaps();
  const auto ops = c.ops();
  int ff = 0, stamp = 0, depth = 0;
  for (int node = 0;; node++) {
    if (node >= kNodeBudget) return GD_BUDGET;
    (*nodes)++;
    if (fill<L, CM>(c, G, n_opt, &ff, &stamp, st)) {
      // the matching ignored CAS expectations after free gaps: check them
      int viol = INT_MAX;
      for (int g0 = 1; g0 < G; g0 = uni(g0 + kWave)) {
        const int gi = min(g0 + lane, G - 1);  // gaps gi-1, gi; gi-1 free if B = kAny
        const int e = ops[c.at(aMG, gi)].z, pv = ops[c.at(aMG, gi - 1)].y;
        const uint64_t b =
            __ballot((g0 + lane < G) & (gaps[gi].z == kAny) & (e != kAny) & (pv != e));
        if (b) {
          viol = uni(g0 + first_lane(b) - 1);
          break;
        }
      }
      if (viol == INT_MAX) return GD_VALID;
      // branch on the value of free gap `viol`
      const int v = next_value<L, CM>(c, viol, INT_MIN, n_opt, st);
      if (lane == 0) {
        brPos[depth] = viol;
        brVal[depth] = v;
      }
      depth++;
      set_req<L, CM>(c, viol, v, G, &ff, st);
      continue;
    }
    // no filling: next value of the deepest branch, else backtrack
    for (;;) {
      if (depth == 0) return GD_INVALID;
      const int gi = uni(brPos[depth - 1]), last = uni(brVal[depth - 1]);
      set_req<L, CM>(c, gi, kAny, G, &ff, st);
      const int v = next_value<L, CM>(c, gi, last, n_opt, st);
      if (v != INT_MAX) {
        if (lane == 0) brVal[depth - 1] = v;
        set_req<L, CM>(c, gi, v, G, &ff, st);
        break;
      }
      depth--;
    }
  }
}

// Class-indexed when there are many optional ops of few classes (and, in
// the HBM fallback, room for the class table); else the chunked scans.
template <bool L, class P>
__device__ int match_branch(const Cmp<L> &c, int G, int n_opt, P brPos, P brVal,
                            int64_t *nodes) {
  ClsSt st;
  st.K = 0;
  if (n_opt >= kClsMinOps && (L || c.cap >= 4 * kMaxCls) && build_classes(c, G, n_opt, st) >= 0)
    return match_branch_m<L, true>(c, G, n_opt, brPos, brVal, nodes, st);
  return match_branch_m<L, false>(c, G, n_opt, brPos, brVal, nodes, st);
}

}  // namespace
}  // namespace lcdev
