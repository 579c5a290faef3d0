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
constexpr int kNodeBudget = kGapNodeBudget;  // matching passes per decision
constexpr int kMaxCls = 64;        // class-indexed matching: at most one class per lane
constexpr int kClsMinOps = 128;    // ... used from this many optional ops on
#ifdef GAP_SINGLE_PUSH  // A/B: one violation branched on per matching
constexpr bool kGapMultiPush = false;
#else
constexpr bool kGapMultiPush = true;
#endif

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
  // class-indexed matching in LDS, when there is room (ClsSt::mgr): per op
  // a copy of the record of the gap it is matched to, after the class table
  __device__ __forceinline__ int4 * mgr() const { return cls() + kMaxCls; }
};

// LDS for the per-op copies of matched gap records (Cmp::mgr)
__host__ __device__ constexpr int match_mgr_bytes(int n_opt) { return 16 * n_opt; }

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
// matching counters of this workgroup: first-fits, augments, augment steps,
// failed augments, cycles (first-fit, augment, cursor steps, fill); LDS adds
// whose result is unused (no wait inside the timed sections)
__shared__ unsigned long long s_mprof[12];
#define MPROF(i, v) \
  do { if ((threadIdx.x & 63) == 0) atomicAdd(&s_mprof[i], (unsigned long long)(v)); } while (0)
// cycles of a section (s_memtime), and the wave-max of a per-lane loop count
#define MCLK0(t) const uint64_t t = __builtin_amdgcn_s_memtime()
#define MCLK1(t, i) MPROF(i, __builtin_amdgcn_s_memtime() - t)
#define MITER(i, n) MPROF(i, (unsigned long long)(-wave_min_i32(-(n))))
#else
#define MPROF(i, v) do { } while (0)
#define MCLK0(t) do { } while (0)
#define MCLK1(t, i) do { } while (0)
#define MITER(i, n) do { } while (0)
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
  int mgr = 0;           // (uniform) Cmp::mgr holds each matched op's gap record
  // lane k: matched ops of class k at or past its free cursor (every op
  // before the cursor is matched; an augmenting path or a branch's unmatch
  // leaves matched ops ahead of it).  While 0 the head is known free.
  int ma = 0;
  int stamp = 0;         // (uniform) visit stamp of the last augmenting search: never reused
  // (uniform) node budget of the expected-value-first search before the plain
  // rerun (GapJob::pref_budget: kGapPrefBudget; tests set a tiny one)
  int pref_budget = kGapPrefBudget;
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

// First free eligible op for gap gi (record gp) in call order (class heads
// and the gap's pinned list), or -1.  The caller matches it: its class's
// free cursor moves on at once.
template <bool L>
__device__ int first_fit_cls(const Cmp<L> &c, int gi, const int4 gp, ClsSt &st) {
  const int lane = threadIdx.x & (kWave - 1);
  const auto ops = c.ops();
  // move each free cursor past matched heads (only lanes with matched ops
  // ahead of the cursor look: no LDS round trip in the common case)
#ifdef GAP_PROFILE
  int adv = 0;
#endif
  while (st.ma > 0 && st.fo >= 0 && c.at(aMO, st.fo) != -1) {
    st.f++;
    st.ma--;
    cls_head(c, st, st.f, &st.fo, &st.fc);
#ifdef GAP_PROFILE
    adv++;
#endif
  }
#ifdef GAP_PROFILE
  MITER(6, adv);
#endif
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

// Match gap SG[d] to op SO[d] for d = 0..depth (an augmenting path found).
template <bool L>
__device__ __forceinline__ void flip_path(const Cmp<L> &c, int depth, int last, ClsSt &st) {
  const int lane = threadIdx.x & (kWave - 1);
  // the path's last op was free (so at or past its class's free cursor) and
  // is matched now; every other op on it stays matched
  if (lane == uni(c.at(aCls, last))) st.ma++;
  match_fence<L>();
  for (int d0 = 0; d0 <= depth; d0 += kWave) {
    const int d = d0 + lane;
    if (d <= depth) {
      const int gg = c.at(aSG, d), oo = c.at(aSO, d);
      c.at(aMG, gg) = oo;
      c.at(aMO, oo) = gg;
      if constexpr (L)
        if (st.mgr) c.mgr()[oo] = c.gaps()[gg];
    }
  }
  match_fence<L>();
}

// Augmenting path from the unmatched gap g0 (record gp0) over the class
// cursors.  Called right after first_fit_cls failed on g0, so every free
// cursor's head is free.  With st.mgr the op a step reaches
// brings the record of its gap along (one LDS round trip per step).
template <bool L>
__device__ bool augment_cls(const Cmp<L> &c, int g0, const int4 gp0, int stamp, ClsSt &st) {
  const int lane = threadIdx.x & (kWave - 1);
  const auto ops = c.ops();
  st.p = 0;
  cls_head(c, st, 0, &st.po, &st.pc);
  int depth = 0, g = uni(g0);
  int4 gp = gp0;
  for (;;) {
    MPROF(2, 1);
    const bool compat = cls_compat(st, gp);
    // lookahead: a free eligible op ends the path here (Kuhn's search would
    // reach it only after exhausting the matched ops called before it)
    uint32_t fcall = cls_key(st, gp, st.fc);
    int fop = st.fo;
    // else the first unvisited eligible op in call order
    uint32_t call = (compat & (st.pc < (uint32_t)gp.x)) ? st.pc : kNever;
    int o = st.po;
    if (st.any_pin) {
      for (int q = uni(c.at(aPH, g)); q >= 0; q = uni(c.at(aPN, q))) {
        const int4 op = uni4(ops[q]);
        const bool e = elig(gp, op);
        if (uni(c.at(aMO, q)) == -1 && e && (uint32_t)op.x < fcall) {
          fcall = (uint32_t)op.x;
          fop = q;
        }
        if (uni(c.at(aVis, q)) != stamp && e && (uint32_t)op.x < call) {
          call = (uint32_t)op.x;
          o = q;
        }
      }
    }
    const uint32_t fbest = wave_min_u32(fcall);
    const uint32_t best = wave_min_u32(call);
    if (fbest != kNever) {
      const int free_op = uni(__builtin_amdgcn_readlane(fop, first_lane(__ballot(fcall == fbest))));
      c.at(aSG, depth) = g;
      c.at(aSO, depth) = free_op;
      flip_path(c, depth, free_op, st);
      return true;
    }
    if (best == kNever) {  // dead end: back to the previous gap
      if (depth == 0) return false;
      depth--;
      g = uni(c.at(aSG, depth));
      gp = uni4(c.gaps()[g]);
      continue;
    }
    const int wl = first_lane(__ballot(call == best));
    const int found = uni(__builtin_amdgcn_readlane(o, wl));
    const int head = uni(__builtin_amdgcn_readlane(st.po, wl));
    // the op's match (and, with mgr, its gap's record) in flight together
    const int mo = c.at(aMO, found);
    int4 gpn = make_int4(0, 0, 0, 0);
    if constexpr (L)
      if (st.mgr) gpn = c.mgr()[found];
    if (found != head) {
      c.at(aVis, found) = stamp;  // a pinned op
    } else if (lane == wl) {      // visited: the class's visit cursor moves past it
      st.p++;
      cls_head(c, st, st.p, &st.po, &st.pc);
    }
    c.at(aSG, depth) = g;
    c.at(aSO, depth) = found;
    const int m = uni(mo);
    if (m == -1) {  // flip the path
      flip_path(c, depth, found, st);
      return true;
    }
    depth++;
    g = m;
    if (L && st.mgr)
      gp = uni4(gpn);
    else
      gp = uni4(c.gaps()[g]);
  }
}

// Augmenting path from the unmatched gap g0 by breadth-first search over the
// class cursors (the default; GAP_DFS_AUG selects augment_cls).  The depth-
// first search above visits one op per step, and each step is a chain of
// wave reductions and LDS round trips (≈1,000 cycles on C4); here a dequeued
// gap visits, in one lane-parallel loop, EVERY unvisited op it can reach —
// the prefix of each compatible class up to its deadline, all matched (a free
// one would have ended the search) — and queues their gaps.  Visits stay
// prefixes of each class list, so every op is visited at most once and every
// gap queued at most once, as in the depth-first search; the search fails
// iff no augmenting path leaves g0 (Kuhn).  Per gap the queue (aSR) and the
// gap it was reached from (aSG, indexed by gap); the path is flipped from its
// free end back to g0.
template <bool L>
__device__ bool augment_bfs_cls(const Cmp<L> &c, int g0, const int4 gp0, int stamp, ClsSt &st) {
  const int lane = threadIdx.x & (kWave - 1);
  const auto ops = c.ops();
  st.p = 0;
  cls_head(c, st, 0, &st.po, &st.pc);
  int po2;        // the op after the visit cursor's, and its call: a lane
  uint32_t pc2;   // visits two per round trip
  cls_head(c, st, 1, &po2, &pc2);
  if (lane == 0) c.at(aSR, 0) = g0;
  match_fence<L>();
  int qh = 0, qt = 1;
  while (qh < qt) {
    MPROF(2, 1);
    const int g = uni(c.at(aSR, qh));
    qh = uni(qh + 1);
    const int4 gp = g == g0 ? gp0 : uni4(c.gaps()[g]);
    // a free eligible op ends the path here (class heads, then pinned ops)
    uint32_t fcall = cls_key(st, gp, st.fc);
    int fop = st.fo;
    if (st.any_pin) {
      for (int q = uni(c.at(aPH, g)); q >= 0; q = uni(c.at(aPN, q))) {
        const int4 op = uni4(ops[q]);
        if (!elig(gp, op)) continue;
        const int mq = uni(c.at(aMO, q));
        if (mq == -1) {
          if ((uint32_t)op.x < fcall) {
            fcall = (uint32_t)op.x;
            fop = q;
          }
        } else if (uni(c.at(aVis, q)) != stamp) {  // a pinned matched op: visit it
          if (lane == 0) {
            c.at(aVis, q) = stamp;
            c.at(aSR, qt) = mq;
            c.at(aSG, mq) = g;
          }
          qt = uni(qt + 1);
        }
      }
    }
    const uint32_t fbest = wave_min_u32(fcall);
    if (fbest != kNever) {
      int o = uni(__builtin_amdgcn_readlane(fop, first_lane(__ballot(fcall == fbest))));
      if (lane == uni(c.at(aCls, o))) st.ma++;  // matched now, at or past its class's free cursor
      match_fence<L>();
      for (int gg = g;;) {  // flip: each gap of the path takes the op that reached its successor
        const int o_old = uni(c.at(aMG, gg));
        const int par = uni(c.at(aSG, gg));
        if (lane == 0) {
          c.at(aMG, gg) = o;
          c.at(aMO, o) = gg;
          if constexpr (L)
            if (st.mgr) c.mgr()[o] = c.gaps()[gg];
        }
        match_fence<L>();
        if (gg == g0) break;
        o = o_old;
        gg = par;
      }
      return true;
    }
    // visit every unvisited op of the compatible classes called before the
    // deadline (all matched: no free one is eligible), queueing their gaps
    const bool compat = cls_compat(st, gp);
    MCLK0(tv);
    for (;;) {
      const bool a1 = compat & (st.pc < (uint32_t)gp.x);
      const bool a2 = a1 & (pc2 < (uint32_t)gp.x);
      const uint64_t m1 = __ballot(a1), m2 = __ballot(a2);
      if (!m1) break;
      MPROF(8, 1);
      MPROF(11, __popcll(m1) + __popcll(m2));
      if (a1) {
        // the visited ops' gaps and the next two heads in flight together
        // (the head loads are issued before the stores that wait for the gaps)
        const int mo1 = c.at(aMO, st.po);
        const int mo2 = a2 ? c.at(aMO, po2) : 0;
        st.p += a2 ? 2 : 1;
        cls_head(c, st, st.p, &st.po, &st.pc);
        cls_head(c, st, st.p + 1, &po2, &pc2);
        c.at(aSR, qt + lanes_below(m1)) = mo1;
        c.at(aSG, mo1) = g;
        if (a2) {
          c.at(aSR, qt + __popcll(m1) + lanes_below(m2)) = mo2;
          c.at(aSG, mo2) = g;
        }
      }
      qt = uni(qt + __popcll(m1) + __popcll(m2));
    }
    MCLK1(tv, 9);
    match_fence<L>();
  }
  return false;
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
    // CM: the next gap's record is loaded while this one is filled
    int4 gpv = make_int4(0, 0, 0, 0);
    if (CM && todo) gpv = c.gaps()[uni(g0 + first_lane(todo))];
    while (todo) {
      const int gi = uni(g0 + first_lane(todo));
      todo &= todo - 1;
      int4 gp = make_int4(0, 0, 0, 0);
      if constexpr (CM) {
        gp = uni4(gpv);
        if (todo) gpv = c.gaps()[uni(g0 + first_lane(todo))];
      }
      int o;
      MPROF(0, 1);
      MCLK0(tf);
      if constexpr (CM)
        o = first_fit_cls(c, gi, gp, st);
      else
        o = first_fit(c, gi, n_opt, ff);
      MCLK1(tf, 4);
      if (o >= 0) {
        c.at(aMG, gi) = o;
        c.at(aMO, o) = gi;
        if constexpr (CM && L)
          if (st.mgr && lane == 0) c.mgr()[o] = gp;
        match_fence<L>();
        continue;
      }
      *stamp = uni(*stamp + 1);
      MPROF(1, 1);
      bool ok;
      MCLK0(ta);
      if constexpr (CM) {
#ifdef GAP_DFS_AUG
        ok = augment_cls(c, gi, gp, *stamp, st);
#else
        ok = augment_bfs_cls(c, gi, gp, *stamp, st);
#endif
      } else {
        ok = augment(c, gi, n_opt, *stamp);
      }
      MCLK1(ta, 5);
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
    const int4 gr = uni4(gaps[g]);
    if constexpr (CM && L)
      if (st.mgr && lane == 0) c.mgr()[o] = gr;  // (stale if unmatched below: unread then)
    if (!elig(gr, uni4(c.ops()[o]))) {
      c.at(aMG, g) = -1;
      c.at(aMO, o) = -1;
      if constexpr (CM) {
        const int k2 = uni(c.at(aCls, o));
        if (k2 >= 0 && lane == k2) {
          const int rk = c.at(aRank, o);
          if (rk < st.f) {  // the ops between it and the old cursor stay matched
            st.ma += st.f - 1 - rk;
            st.f = rk;
            st.fo = o;
            st.fc = (uint32_t)c.ops()[o].x;
          } else {
            st.ma--;
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
// branch stack (gap, value, first value) lives in skeleton arrays that are
// free once the compact arrays are built.
//
// A branch on free gap g (the CAS matched after it expects e, which the op
// matched at g does not write) tries e first, when some op eligible for g
// writes e: that one value repairs the violation, and the matching then
// usually needs no further branch (C4: 65 -> 4 matchings).  Then the other
// values in increasing order, e skipped.  Every value is tried once, so the
// search is exactly as complete as the plain ascending order.  PREF false:
// ascending order only (brFst unused; the crash-light pass, whose keys
// rarely branch, keeps its register budget).
template <bool L, bool CM, bool PREF, class P>
__device__ int match_branch_m(const Cmp<L> &c, int G, int n_opt, P brPos, P brVal, P brFst,
                              int64_t *nodes, ClsSt &st) {
  const int lane = threadIdx.x & (kWave - 1);
  const auto gaps = c.gaps();
  const auto ops = c.ops();
  int ff = 0, depth = 0;
  int &stamp = st.stamp;  // (a rerun after the budget keeps counting: stale visits never match)
  for (int node = 0;; node++) {
    if (node >= (PREF ? st.pref_budget : kNodeBudget)) {
      // PREF: back to the gaps' own requirements (every branch gap was free),
      // so the caller can rerun with the plain order
      if (PREF)
        for (; depth > 0; depth--) set_req<L, CM>(c, uni(brPos[depth - 1]), kAny, G, &ff, st);
      return GD_BUDGET;
    }
    (*nodes)++;
    MCLK0(tn);
    const bool filled = fill<L, CM>(c, G, n_opt, &ff, &stamp, st);
    MCLK1(tn, 7);
#ifdef GAP_ONE_FILL  // dev timing build: every decision ends after its first fill (verdicts meaningless)
    return filled ? GD_VALID : GD_INVALID;
#endif
    if (filled) {
      // the matching ignored CAS expectations after free gaps: check them.
      // PREF: every violation whose expected value some eligible op writes
      // is branched on at once, the expected value first (a run of levels
      // of the same depth-first search, each level a gap of its own, pushed
      // without a fill between: a failing fill prunes the deepest); else
      // the first violation, ascending.
      int pushed = 0, viol0 = INT_MAX;
      for (int g0 = 1; g0 < G; g0 = uni(g0 + kWave)) {
        const int gi = min(g0 + lane, G - 1);  // gaps gi-1, gi; gi-1 free if B = kAny
        // (a push earlier in this scan may have unmatched a gap: such a pair
        // is no violation of this matching)
        const int mg = c.at(aMG, gi), mg1 = c.at(aMG, gi - 1);
        const int e = ops[max(mg, 0)].z, pv = ops[max(mg1, 0)].y;
        uint64_t b = __ballot((g0 + lane < G) & (mg >= 0) & (mg1 >= 0) & (gaps[gi].z == kAny) &
                              (e != kAny) & (pv != e));
        if (b && viol0 == INT_MAX) viol0 = uni(g0 + first_lane(b) - 1);
        if (!PREF) {
          if (viol0 != INT_MAX) break;  // the first violation only
          continue;
        }
        for (; b; b &= b - 1) {
          const int viol = uni(g0 + first_lane(b) - 1);
          if (!kGapMultiPush && viol != viol0) break;
          const int want = uni(__builtin_amdgcn_readlane(e, first_lane(b)));
          if (uni(gaps[viol + 1].z) != kAny) continue;  // fixed by a push just made
          if (next_value<L, CM>(c, viol, want - 1, n_opt, st) != want) continue;
          if (lane == 0) {
            brPos[depth] = viol;
            brVal[depth] = want;
            brFst[depth] = want;
          }
          depth++;
          pushed++;
          set_req<L, CM>(c, viol, want, G, &ff, st);
        }
        if (viol0 != INT_MAX && !kGapMultiPush) break;
      }
      if (viol0 == INT_MAX) return GD_VALID;
      if (!pushed) {  // branch on the first violation, ascending
        const int v = next_value<L, CM>(c, viol0, INT_MIN, n_opt, st);
        if (lane == 0) {
          brPos[depth] = viol0;
          brVal[depth] = v;
          if (PREF) brFst[depth] = kAny;
        }
        depth++;
        set_req<L, CM>(c, viol0, v, G, &ff, st);
      }
      continue;
    }
    // no filling: next value of the deepest branch, else backtrack
    for (;;) {
      if (depth == 0) return GD_INVALID;
      const int gi = uni(brPos[depth - 1]), last = uni(brVal[depth - 1]);
      const int fst = PREF ? uni(brFst[depth - 1]) : kAny;
      set_req<L, CM>(c, gi, kAny, G, &ff, st);
      // after the first value: ascending from the smallest, the first skipped
      int v = next_value<L, CM>(c, gi, fst != kAny && last == fst ? INT_MIN : last, n_opt, st);
      if (fst != kAny && v == fst) v = next_value<L, CM>(c, gi, v, n_opt, st);
      if (PREF && v != INT_MAX) {
        // relaxation first: with gi free and only the levels above fixed, is
        // there a filling at all?  If not, no value of gi (and nothing deeper)
        // can give one: pop the level instead of trying each value.  (A run of
        // levels pushed at once makes blind backtracking exponential.)
        if (node + 1 >= st.pref_budget) break;  // (the loop's budget exit unwinds the stack)
        node++;
        (*nodes)++;
        if (!fill<L, CM>(c, G, n_opt, &ff, &stamp, st)) {
          depth--;
          continue;
        }
      }
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
__device__ int match_branch(const Cmp<L> &c, int G, int n_opt, P brPos, P brVal, P brFst,
                            int64_t *nodes, bool mgr_room, int pref_budget) {
  ClsSt st;
  st.K = 0;
  st.pref_budget = pref_budget;
  if (n_opt >= kClsMinOps && (L || c.cap >= 4 * kMaxCls) && build_classes(c, G, n_opt, st) >= 0) {
    st.mgr = L && mgr_room;
    const int r = match_branch_m<L, true, true>(c, G, n_opt, brPos, brVal, brFst, nodes, st);
    // the expected-value-first order ran out of nodes: the plain order (round 2's
    // search) gets a budget of its own, so no key is left to the JIT tier that
    // it decided
    return r != GD_BUDGET ? r
                          : match_branch_m<L, true, false>(c, G, n_opt, brPos, brVal, brFst, nodes, st);
  }
  const int r = match_branch_m<L, false, true>(c, G, n_opt, brPos, brVal, brFst, nodes, st);
  return r != GD_BUDGET ? r
                        : match_branch_m<L, false, false>(c, G, n_opt, brPos, brVal, brFst, nodes, st);
}

}  // namespace
}  // namespace lcdev
