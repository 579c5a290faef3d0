// gap_tier.hip — exact decision for version-pinned keys that also hold
// crashed (:info) writes/CAS: the ":info blow-up" keys (SURVEY.md §7,
// BASELINE configs[3]) on which every frontier search — knossos's, the JIT
// tier's — grows exponentially.
//
// Model (register.clj:59-96).  In any linearization the k-th mutation (a
// write or a successful CAS) takes the register from version V0+k-1 to V0+k.
// An :ok mutation claiming version v is therefore PINNED to position
// p = v-V0-1, a read claiming version v sits between positions v-V0-1 and
// v-V0, and the only freedom left is which optional ops (crashed mutations;
// in a history prefix also the pending :ok mutations, each pinned to its own
// position) fill the positions no required mutation holds — the GAPS.
// Positions past the last one a required op needs are never filled: an
// optional op may always be left out.
//
// With one linearization point t_k per position, the key is linearizable iff
// a filling exists with
//     L_k < t_k < U_k,  L_k = max(call(m_k), calls of reads of version V0+k)
//                       U_k = min(ret(m_k),  rets of reads of version V0+k+1)
// whose values chain (CAS expectations register.clj:77, read claims
// register.clj:90-94).  Points exist iff max(L_0..L_k) < U_k for every k,
// i.e. iff L_j < Uh_j = min(U_j, U_j+1, ...) for every j: the time
// constraint splits into fixed checks on pinned positions plus one DEADLINE
// per gap, call(op filling gap j) < Uh_j.  What remains is a bipartite
// MATCHING of gaps to optional ops (deadline + value eligibility), coupled
// only where a gap's value is free (no read claims it, no pinned CAS follows)
// and the next gap takes a CAS, whose expectation then fixes it.  Those
// couplings are resolved by depth-first branching on the free value, with
// the matching as the bound (tests/gapmatch_ref.py restates this procedure;
// tests check it against the oracle's searches).
//
// For an invalid key, the canonical counterexample (the :ok op whose return
// empties knossos's JIT frontier) is the first return event r whose prefix
// is not linearizable; linearizability is prefix-closed, so r is found by
// bisection over r, each probe one decision on the prefix (ops called after
// r dropped, ops returning after r pending = optional).
//
// One 256-thread workgroup makes one decision (a key's whole history, or one
// prefix of it): the record scan, the suffix-min scan and the gap/optional-op
// compaction are spread over the workgroup, with O(n) int32 arrays per
// workgroup in HBM/L2.  The matching itself is serial in the gaps, so wave 0
// runs it alone, barrier-free, over compact per-gap / per-op arrays staged in
// LDS (HBM fallback when they do not fit): first-fit over the free ops
// (ballot over 64 ops at a time, ops sorted by call so the deadline cuts the
// scan), then a depth-first augmenting path per gap first-fit cannot fill
// (Kuhn's algorithm; visit stamps instead of clears).  Branch nodes are warm
// started: fixing a free gap's value only unmatches the pairs it makes
// ineligible.  The counterexample search is a multisection: P workgroups
// probe P prefixes of each open interval per round (GapJob, kernels.h), so a
// single hot key (BASELINE configs[3]) spreads over the whole GPU.  Keys it
// cannot decide (an :ok mutation without a version, a read [nil x], malformed
// records, the branch budget) go on to the JIT tier.
#include <algorithm>
#include <climits>
#include <type_traits>

#include "kernels.h"
#include "records.h"

namespace lcdev {
namespace {

constexpr int kGapThreads = 256;
constexpr int kGapWaves = kGapThreads / kWave;
constexpr int kAny = INT_MIN;      // no value required / not a CAS
constexpr int kNodeBudget = 4096;  // matching passes per decision
constexpr int kGapArrays = 31;     // 32-bit arrays of `cap` entries per workgroup
constexpr int kMaxCls = 64;        // class-indexed matching: at most one class per lane
constexpr int kClsMinOps = 128;    // ... used from this many optional ops on

enum { GD_VALID = 1, GD_INVALID = 0, GD_NA = -1, GD_BUDGET = -2, GD_SKIP = -3, GD_RETRY = -4 };
enum { F_NA = 1, F_INVALID = 2 };

// Matching footprint of one decision in LDS: per gap a 16-byte record and 5
// ints, per op a 16-byte record and 6 ints, and the class table.
__host__ __device__ constexpr int match_lds_bytes(int G, int n_opt) {
  return 36 * G + 44 * n_opt + 16 * kMaxCls + 16;  // (+16: the table's alignment)
}

extern __shared__ int4 lds_dyn[];

// Per-workgroup workspace: kGapArrays arrays of `cap` 32-bit entries (cap a
// multiple of 4, so the 16-byte record regions stay aligned).
//   0 A  1 B  2 Uh  3 Pin  4 Val  5 PinExp  6 Claim  7 Req  8 OptRec  9 Gap
//   10..13 Opt: the optional ops as 16-byte records (call, value, exp, pos)
//   14..17 gap records, 18..29 the matching's scalar arrays, 30 its class
//   table — the HBM homes of the matching when it does not fit in LDS;
//   during gap_setup 18..23 also hold the ballot masks and prefix counts of
//   the compactions.
// A key short enough (kSkelLdsBytes per record with its matching) keeps the
// whole skeleton in LDS instead: arrays 0..13, the masks at 14..15 and the
// prefix counts at 16, followed by the matching's LDS region.  Then the
// setup's barriers wait for LDS stores only, not for HBM write acks.
constexpr int kSkelArrays = 17;
constexpr int kSkelLdsBytes = 4 * kSkelArrays;  // per record; the matching follows it
constexpr int kMatchReserve = 8 << 10;           // LDS kept for the matching after a skeleton

// Skeleton arrays are addressed through pointers typed by placement: LDS
// (address space 3) when SL, global otherwise, so the setup compiles to ds_*
// / global_* instructions rather than flat ones (a flat access waits on both
// the LDS and the vector-memory counters, and flat atomics to LDS are slow).
template <bool SL, class X>
using WsP = std::conditional_t<SL, __attribute__((address_space(3))) X *, X *>;

template <bool SL>
struct GapWs {
  int32_t *base;   // HBM workspace base (the matching's HBM homes; unused when SL)
  int64_t cap;
  int moff;        // int4 offset of the matching's LDS region in lds_dyn (SL)
  WsP<SL, uint32_t> A, B, Uh;
  WsP<SL, int> Pin, Val, PinExp, Claim, Req, Gap;
  WsP<SL, int> OptRec;     // record index of each optional op (witnesses)
  WsP<SL, int4> Opt;
  WsP<SL, uint64_t> Mask;  // compaction ballots
  WsP<SL, int> Pre;        // compaction prefix counts
};

struct GapSh {
  int flag, maxpos, maxread, n_opt, n_gap;
  int res;
  uint32_t maxret;
  int wtot[kGapWaves];
  uint32_t wtotu[kGapWaves];
#ifdef GAP_PROFILE
  uint64_t prof[12];
#endif
};

// SL: the skeleton at the start of lds_dyn (cap entries per array); else the
// workgroup's HBM workspace at base.
template <bool SL>
__device__ __forceinline__ GapWs<SL> gap_ws(int32_t *base, int64_t cap) {
  GapWs<SL> w;
  int32_t *b = SL ? reinterpret_cast<int32_t *>(lds_dyn) : base;
  w.base = base;
  w.cap = cap;
  w.moff = SL ? (int)(kSkelArrays * cap / 4) : 0;
  auto P = [&](int a) { return (WsP<SL, int>)(b + a * cap); };
  w.A = (WsP<SL, uint32_t>)P(0);
  w.B = (WsP<SL, uint32_t>)P(1);
  w.Uh = (WsP<SL, uint32_t>)P(2);
  w.Pin = P(3);
  w.Val = P(4);
  w.PinExp = P(5);
  w.Claim = P(6);
  w.Req = P(7);
  w.Gap = P(9);
  w.OptRec = P(8);
  w.Opt = (WsP<SL, int4>)P(10);
  w.Mask = (WsP<SL, uint64_t>)P(SL ? 14 : 18);
  w.Pre = P(SL ? 16 : 20);
  return w;
}

// int4's members take a generic `this`: 16-byte skeleton records go through
// a cast (folded back to the pointer's address space after inlining)
template <class P>
__device__ __forceinline__ int4 ws_ld4(P p) {
  return *(const int4 *)p;
}
template <class P>
__device__ __forceinline__ void ws_st4(P p, int4 v) {
  *(int4 *)p = v;
}
template <class P>
__device__ __forceinline__ void ws_max(P p, uint32_t v) {
  atomicMax((uint32_t *)p, v);
}
template <class P>
__device__ __forceinline__ void ws_min(P p, uint32_t v) {
  atomicMin((uint32_t *)p, v);
}

// Exclusive prefix sum over the workgroup; *total = the sum of all v.
template <int T>
__device__ __forceinline__ int block_excl_sum(int v, GapSh &sh, int *total) {
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  int incl = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == kWave - 1) sh.wtot[w] = incl;
  __syncthreads();
  int pre = 0, tot = 0;
#pragma unroll
  for (int j = 0; j < (T / kWave); j++) {
    if (j < w) pre += sh.wtot[j];
    tot += sh.wtot[j];
  }
  __syncthreads();
  *total = tot;
  return pre + incl - v;
}

// Exclusive suffix minimum over the workgroup (threads above this one).
template <int T>
__device__ __forceinline__ uint32_t block_suffix_min_excl(uint32_t v, GapSh &sh) {
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  uint32_t incl = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_down((int)incl, o);
    if (lane + o < kWave) incl = incl < y ? incl : y;
  }
  if (lane == 0) sh.wtotu[w] = incl;
  __syncthreads();
  uint32_t post = kNever;
#pragma unroll
  for (int j = 0; j < (T / kWave); j++)
    if (j > w) post = post < sh.wtotu[j] ? post : sh.wtotu[j];
  uint32_t excl = (uint32_t)__shfl_down((int)incl, 1);
  if (lane == kWave - 1) excl = kNever;
  __syncthreads();
  return post < excl ? post : excl;
}

__device__ __forceinline__ int wave_min_i32(int v) {
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) v = min(v, __shfl_xor(v, o));
  return v;
}

__device__ __forceinline__ int first_lane(uint64_t b) { return (int)__builtin_ctzll(b); }

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ int4 uni4(int4 v) {
  return make_int4(uni(v.x), uni(v.y), uni(v.z), uni(v.w));
}

__device__ __forceinline__ int lanes_below(uint64_t m) {
  const int lane = threadIdx.x & (kWave - 1);
  return __popcll(m & ((1ull << lane) - 1));
}

// Makes this wave's earlier stores to the matching arrays visible to all of
// its lanes (LDS: lgkmcnt; HBM fallback: vmcnt, same CU so L1-coherent).
__device__ __forceinline__ void wave_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

// Stable compaction, phase 2: word-level exclusive prefix of the ballot
// masks Mask[0..nw) into Pre[0..nw); returns the total.  Two barriers.
template <int T, bool SL>
__device__ int mask_prefix(const GapWs<SL> &w, int nw, GapSh &sh) {
  const int tid = threadIdx.x;
  const int per = (nw + T - 1) / T;
  const int k0 = min(tid * per, nw), k1 = min(k0 + per, nw);
  int loc = 0;
  for (int k = k0; k < k1; k++) loc += __popcll(w.Mask[k]);
  int tot;
  int run = block_excl_sum<T>(loc, sh, &tot);
  for (int k = k0; k < k1; k++) {
    w.Pre[k] = run;
    run += __popcll(w.Mask[k]);
  }
  __syncthreads();
  return tot;
}

struct GapKey {
  const lc_op *kops;
  int n;
  int64_t base;  // call index of the key's first record
  int V0, init;
  GapSh *sh;
};

// One record of the prefix at `cut`, classified.
enum { K_NONE, K_READ, K_PIN, K_OPT };
struct Cls {
  int kind;   // K_*
  int k;      // K_READ: version index; K_PIN: position
  int val;    // K_READ: claimed value (-1 none); K_PIN: value written
  int exp;    // K_PIN: CAS expectation (kAny for a write)
  uint32_t call, ret;
  int4 op;    // K_OPT: the optional op's record (call, value, exp, pos)
};

// Branch-free: every condition is computed and the outcome selected, so a
// wave runs one straight-line path per record instead of a divergent branch
// tree (which cost ~2,000 instructions per chunk with exec-mask bookkeeping).
// Past the end (r >= n) the record is K_NONE.
__device__ __forceinline__ Cls classify(const GapKey &g, const Raw &raw, int64_t prev_call,
                                        int r, uint32_t cut, int *flag, uint32_t *maxret) {
  const int n = g.n;
  const Rec d = decode(raw, g.base);
  const bool in = r < n;
  const bool malformed = in & (d.bad | (d.f > LC_F_CAS) | ((r > 0) & (prev_call >= raw.c.x)) |
                               (raw.c.x < 0));
  const bool live = in & !malformed & (d.call <= cut);
  const uint32_t ret = d.ret > cut ? kNever : d.ret;  // pending at the cut
  const bool crashed = ret == kNever;
  const bool isread = d.f == LC_F_READ;
  // reads: crashed or [nil nil] never constrain; [nil x] is the JIT tier's
  const bool rd_uncon = crashed | ((d.ver == -1) & (d.val == -1));
  const bool rd_na = !rd_uncon & (d.ver == -1);
  const int kr = d.ver - g.V0;
  const bool rd_bad = !rd_uncon & !rd_na & ((kr < 0) | (kr > n));
  // mutations: crashed ones are optional (unless never placeable); an :ok
  // one without a version is the JIT tier's; one past the key is invalid
  const int pos = d.ver - g.V0 - 1;
  const bool pos_out = (pos < 0) | (pos >= n);
  const bool mu_na = !crashed & (d.ver == -1);
  const bool mu_bad = !crashed & !mu_na & pos_out;
  const bool is_read = live & isread & !rd_uncon & !rd_na & !rd_bad;
  const bool is_pin = live & !isread & !crashed & !mu_na & !mu_bad;
  const bool is_opt = live & !isread & crashed & ((d.ver == -1) | !pos_out);
  const bool na = malformed | (live & (isread ? rd_na : mu_na));
  const bool inv = live & (isread ? rd_bad : mu_bad);
  *flag |= (na ? F_NA : 0) | (inv ? F_INVALID : 0);
  *maxret = (live & !crashed) ? max(*maxret, ret) : *maxret;
  Cls c;
  c.kind = is_read ? K_READ : is_pin ? K_PIN : is_opt ? K_OPT : K_NONE;
  c.k = is_read ? kr : pos;
  c.val = d.val;
  c.exp = d.f == LC_F_CAS ? d.exp : kAny;
  c.call = d.call;
  c.ret = ret;
  c.op = make_int4((int)d.call, d.val, c.exp, d.ver == -1 ? -1 : pos);
  return c;
}

constexpr int kSetupBatch = 4;  // record chunks whose loads are in flight together

// Build the skeleton of the key's prefix at `cut` (key-relative event index;
// kNever = the whole history).  Returns GD_VALID when the skeleton is
// consistent (then sh.n_gap / sh.n_opt / sh.maxret are set), else
// GD_INVALID / GD_NA.  Two passes over the records, each issuing the loads
// of kSetupBatch chunks at once: pass 1 folds bounds with fire-and-forget
// atomics and claims positions / read values with plain owner stores; pass 2
// checks the owners (two mutations on one version, two values claimed for
// one version) and appends the optional ops.  Optional ops and gaps are
// compacted stably through per-wave ballot words: no barrier per chunk.
template <int T, bool SL>
__device__ int gap_setup(const GapKey &g, const GapWs<SL> &w, uint32_t cut) {
  const int tid = threadIdx.x, n = g.n, wv = tid / kWave, lane = tid & (kWave - 1);
  GapSh &sh = *g.sh;
  // Every wave must be done reading the previous decision's shared words
  // (sh.flag on its early-return paths, sh.maxret) before thread 0 resets
  // them: decisions follow each other without a barrier in the bisection.
  __syncthreads();
  for (int k = tid; k <= n; k += T) {
    w.A[k] = 0;  // max call + 1 of what must precede t_k; 0 = nothing
    w.B[k] = kNever;
    w.Pin[k] = -1;
    w.Claim[k] = kAny;
  }
  if (tid == 0) {
    sh.flag = 0;
    sh.maxpos = -1;
    sh.maxread = -1;
    sh.maxret = 0;
    sh.n_opt = 0;
    sh.n_gap = 0;
  }
  __syncthreads();
#ifdef GAP_PROFILE
  if (tid == 0) sh.prof[0] = wall_clock64();
#endif
  int flag = 0, maxpos = -1, maxread = -1;
  uint32_t maxret = 0;
  const int nch = (n + T - 1) / T;
  // A key of at most kSetupBatch chunks is loaded once: pass 2 reuses the
  // registers (one load round trip per decision instead of two).
  const bool resident = nch <= kSetupBatch;
  Raw raw[kSetupBatch];
  int64_t pc[kSetupBatch];
  for (int pass = 1; pass <= 2; pass++) {
    for (int c0 = 0; c0 < nch; c0 += kSetupBatch) {
      if (pass == 1 || !resident) {
#pragma unroll
        for (int b = 0; b < kSetupBatch; b++) {
          const int r = (c0 + b) * T + tid;
          raw[b] = load_raw(g.kops, r, n);
          pc[b] = (r > 0 && r < n) ? g.kops[r - 1].call : -1;
        }
      }
#ifdef GAP_PROFILE
      if (pass == 1 && c0 == 0) {
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (tid == 0) sh.prof[7] = wall_clock64();
      }
#endif
#pragma unroll
      for (int b = 0; b < kSetupBatch; b++) {
        const int ch = c0 + b, r = ch * T + tid;
        if (ch >= nch) break;
        const Cls c = classify(g, raw[b], pc[b], r, cut, &flag, &maxret);
        const bool rd = c.kind == K_READ, pin = c.kind == K_PIN;
        const bool claim = rd & (c.val != -1);
        if (pass == 1) {
          maxread = rd ? max(maxread, c.k) : maxread;
          maxpos = pin ? max(maxpos, c.k) : maxpos;
          if (rd | pin) ws_max(&w.A[c.k], c.call + 1);
          if (pin | (rd & (c.k > 0))) ws_min(&w.B[pin ? c.k : c.k - 1], c.ret);
          if (claim) w.Claim[c.k] = c.val;
          if (pin) {
            w.Pin[c.k] = r;
            w.Val[c.k] = c.val;
            w.PinExp[c.k] = c.exp;
          }
          const uint64_t m = __ballot(c.kind == K_OPT);
          if (lane == 0) w.Mask[ch * (T / kWave) + wv] = m;
        } else {
          // two values claimed for one version / two mutations on one version
          if (claim) flag |= w.Claim[c.k] != c.val ? F_INVALID : 0;
          if (pin) flag |= w.Pin[c.k] != r ? F_INVALID : 0;
          const int wi = ch * (T / kWave) + wv;
          if (c.kind == K_OPT) {
            const uint64_t m = w.Mask[wi];
            const int o = w.Pre[wi] + lanes_below(m);
            ws_st4(&w.Opt[o], c.op);
            w.OptRec[o] = r;
          }
        }
#ifdef GAP_PROFILE
        if (pass == 1 && tid == 0) sh.prof[8 + b] = wall_clock64();
#endif
      }
    }
    if (pass == 1) {
      if (flag) atomicOr(&sh.flag, flag);
      if (maxpos >= 0) atomicMax(&sh.maxpos, maxpos);
      if (maxread >= 0) atomicMax(&sh.maxread, maxread);
      if (maxret) atomicMax(&sh.maxret, maxret);
      __syncthreads();
#ifdef GAP_PROFILE
    if (tid == 0) sh.prof[1] = wall_clock64();
#endif
      if (sh.flag & (F_NA | F_INVALID)) return (sh.flag & F_NA) ? GD_NA : GD_INVALID;
      sh.n_opt = mask_prefix<T, SL>(w, nch * (T / kWave), sh);  // same value in every thread
#ifdef GAP_PROFILE
    if (tid == 0) sh.prof[2] = wall_clock64();
#endif
      flag = 0;
    }
  }
  if (flag) atomicOr(&sh.flag, flag);
  __syncthreads();
#ifdef GAP_PROFILE
    if (tid == 0) sh.prof[3] = wall_clock64();
#endif
  if (sh.flag & F_INVALID) return GD_INVALID;
  const int n_opt = sh.n_opt;
  const int M = max(sh.maxpos + 1, sh.maxread);
  // Uh[k] = min(B[k..M-1]): chunked suffix-min scan
  const int per = (M + T - 1) / T;
  const int k0 = min(tid * per, M), k1 = min(k0 + per, M);
  uint32_t loc = kNever;
  for (int k = k0; k < k1; k++) loc = min(loc, w.B[k]);
  uint32_t run = block_suffix_min_excl<T>(loc, sh);
  for (int k = k1 - 1; k >= k0; k--) {
    run = min(run, w.B[k]);
    w.Uh[k] = run;
  }
  __syncthreads();
#ifdef GAP_PROFILE
    if (tid == 0) sh.prof[4] = wall_clock64();
#endif
  // fixed checks: pinned / read-only lower bounds below the deadline, and
  // the value chain around pinned positions; the requirement on each gap;
  // one ballot word of gap positions per wave chunk
  flag = 0;
  if (tid == 0) {
    if (w.Claim[0] != kAny && w.Claim[0] != g.init) flag |= F_INVALID;
    if (M > 0 && w.Pin[0] != -1 && w.PinExp[0] != kAny && w.PinExp[0] != g.init)
      flag |= F_INVALID;
  }
  const int mch = (M + T - 1) / T;
  for (int ch = 0; ch < mch; ch++) {
    const int k = ch * T + tid;
    bool gap = false;
    if (k < M) {
      const uint32_t lo = w.A[k];
      if (lo != 0 && lo - 1 >= w.Uh[k]) flag |= F_INVALID;
      int rq = w.Claim[k + 1];
      if (k + 1 < M && w.Pin[k + 1] != -1 && w.PinExp[k + 1] != kAny) {
        if (rq != kAny && rq != w.PinExp[k + 1]) flag |= F_INVALID;
        rq = w.PinExp[k + 1];
      }
      if (w.Pin[k] != -1) {
        if (rq != kAny && rq != w.Val[k]) flag |= F_INVALID;
      } else {
        w.Req[k] = rq;
        gap = true;
      }
    }
    const uint64_t m = __ballot(gap);
    if (lane == 0) w.Mask[ch * (T / kWave) + wv] = m;
  }
  if (flag) atomicOr(&sh.flag, flag);
  __syncthreads();
#ifdef GAP_PROFILE
    if (tid == 0) sh.prof[5] = wall_clock64();
#endif
  if (sh.flag & F_INVALID) return GD_INVALID;
  const int G = mask_prefix<T, SL>(w, mch * (T / kWave), sh);
#ifdef GAP_PROFILE
    if (tid == 0) sh.prof[6] = wall_clock64();
#endif
  for (int ch = 0; ch < mch; ch++) {
    const int wi = ch * (T / kWave) + wv;
    const uint64_t m = w.Mask[wi];
    if ((m >> lane) & 1) w.Gap[w.Pre[wi] + lanes_below(m)] = ch * T + tid;
  }
  if (tid == 0) {
    sh.n_opt = n_opt;
    sh.n_gap = G;
  }
  __syncthreads();
  return GD_VALID;
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
  __device__ __forceinline__ int4 *gaps() const {
    if constexpr (L)
      return lds_dyn + moff;
    else
      return reinterpret_cast<int4 *>(ws + 14 * cap);
  }
  __device__ __forceinline__ int4 *ops() const {
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
  __device__ __forceinline__ int4 *cls() const {
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

// Minimum over the wave (wave-uniform): DPP butterfly within rows of 16
// (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror), then the
// four row results by readlane — no LDS round trips (a shfl_xor butterfly
// costs six).
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x141, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x140, 0xF, 0xF, false));
  return min(min((uint32_t)__builtin_amdgcn_readlane((int)v, 0),
                 (uint32_t)__builtin_amdgcn_readlane((int)v, 16)),
             min((uint32_t)__builtin_amdgcn_readlane((int)v, 32),
                 (uint32_t)__builtin_amdgcn_readlane((int)v, 48)));
}

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
  int4 *tab = c.cls();
  const int4 *ops = c.ops();
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
  const int4 *gaps = c.gaps();
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
  const int4 *ops = c.ops();
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
  const int4 *ops = c.ops();
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
  const int4 *ops = c.ops();
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
  int4 *gaps = c.gaps();
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
  const int4 *gaps = c.gaps(), *ops = c.ops();
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

// The linearization a valid decision found (lc_aux witness): every record of
// the key -1, then each pinned position's record and each gap's matched op
// their position.  The matched pairs come from the matching's arrays (gap
// gi -> op aMG[gi] -> record OptRec[op]); with no gaps only the pins.
template <int T, bool SL, class C>
__device__ void gap_witness(const GapKey &g, const GapWs<SL> &w, const C *c, int G,
                            int32_t *__restrict__ wk) {
  const int tid = threadIdx.x;
  for (int r = tid; r < g.n; r += T) wk[r] = -1;
  __syncthreads();  // the -1 stores before the positions (same addresses)
  for (int k = tid; k <= g.n; k += T) {
    const int r = w.Pin[k];
    if (r != -1) wk[r] = k;
  }
  if (c)
    for (int gi = tid; gi < G; gi += T) wk[w.OptRec[c->at(aMG, gi)]] = c->gaps()[gi].w;
  __syncthreads();
}

// Decide the prefix at `cut`.  *nodes accumulates matching passes.  With wk
// (this key's witness records), a valid decision also writes its
// linearization (gap_witness).
template <int T, bool SL>
__device__ int gap_decide(const GapKey &g, const GapWs<SL> &w, uint32_t cut, int lds_bytes,
                          int64_t *nodes, int *n_gaps, int32_t *wk) {
  const int tid = threadIdx.x;
  GapSh &sh = *g.sh;
#ifdef GAP_PROFILE
  const uint64_t t0 = wall_clock64();
#endif
  const int st = gap_setup<T, SL>(g, w, cut);
  if (st != GD_VALID) return st;
#ifdef GAP_PROFILE
  const uint64_t t1 = wall_clock64();
#endif
  const int G = sh.n_gap, n_opt = sh.n_opt;
  *n_gaps = G;
  if (G == 0) {
    if (wk) gap_witness<T, SL, Cmp<true>>(g, w, nullptr, 0, wk);
    return GD_VALID;
  }
  if (G > n_opt) return GD_INVALID;
  const bool in_lds = 16 * w.moff + match_lds_bytes(G, n_opt) <= lds_bytes;
  // skeleton in LDS but no room left for this matching: the caller redoes the
  // decision with the skeleton in HBM (the whole LDS then holds the matching)
  if (SL && !in_lds) return GD_RETRY;
  Cmp<true> cl;
  Cmp<false> cg;
  cl.ws = cg.ws = w.base;
  cl.G = cg.G = G;
  cl.n_opt = cg.n_opt = n_opt;
  cl.cap = cg.cap = (int)w.cap;
  cl.moff = cg.moff = w.moff;
  // compact per-gap / per-op arrays, then the matching on wave 0; each
  // placement instantiated apart so every access keeps its address space
  auto compact = [&](const auto &c) {
    int4 *gaps = c.gaps();
    for (int gi = tid; gi < G; gi += T) {
      const int pos = w.Gap[gi];
      const int before =
          pos == 0 ? g.init : (w.Pin[pos - 1] != -1 ? w.Val[pos - 1] : w.Req[pos - 1]);
      gaps[gi] = make_int4((int)w.Uh[pos], w.Req[pos], before, pos);
      c.at(aMG, gi) = -1;
    }
    for (int o = tid; o < n_opt; o += T) {
      if (in_lds) c.ops()[o] = ws_ld4(&w.Opt[o]);
      c.at(aMO, o) = -1;
      c.at(aVis, o) = 0;
    }
  };
  if (SL || in_lds)
    compact(cl);
  else
    compact(cg);
  __syncthreads();
#ifdef GAP_PROFILE
  const uint64_t t2 = wall_clock64();
#endif
  if (tid < kWave) {
    int r;
    if (SL || in_lds)
      r = match_branch(cl, G, n_opt, w.Claim, w.Req, nodes);
    else
      r = match_branch(cg, G, n_opt, w.Claim, w.Req, nodes);
    if (tid == 0) sh.res = r;
  }
  __syncthreads();
  const int r = sh.res;
  __syncthreads();
  if (wk && r == GD_VALID) {
    if (SL || in_lds)
      gap_witness<T, SL>(g, w, &cl, G, wk);
    else
      gap_witness<T, SL>(g, w, &cg, G, wk);
  }
#ifdef GAP_PROFILE
  if (tid == 0 && blockIdx.x < 2) {
    printf("  matching wg %d: first-fits %llu augments %llu steps %llu failed %llu\n",
           (int)blockIdx.x, g_mprof[blockIdx.x][0], g_mprof[blockIdx.x][1],
           g_mprof[blockIdx.x][2], g_mprof[blockIdx.x][3]);
    for (int i = 0; i < 8; i++) g_mprof[blockIdx.x][i] = 0;
  }
  if (tid == 0 && blockIdx.x < 2)
    printf("gap_decide wg %d cut %u n %d G %d n_opt %d lds %d nodes %ld: setup %lu [clr %lu p1 %lu (ld %lu c %lu %lu %lu %lu) pre %lu p2 %lu smin %lu chk %lu gcmp %lu] compact %lu match %lu (x10ns)\n",
           (int)blockIdx.x, cut, g.n, G, n_opt, (int)in_lds, (long)*nodes, (unsigned long)(t1 - t0),
           (unsigned long)(sh.prof[0] - t0), (unsigned long)(sh.prof[1] - sh.prof[0]),
           (unsigned long)(sh.prof[7] - sh.prof[0]), (unsigned long)(sh.prof[8] - sh.prof[7]),
           (unsigned long)(sh.prof[9] - sh.prof[8]), (unsigned long)(sh.prof[10] - sh.prof[9]),
           (unsigned long)(sh.prof[11] - sh.prof[10]),
           (unsigned long)(sh.prof[2] - sh.prof[1]), (unsigned long)(sh.prof[3] - sh.prof[2]),
           (unsigned long)(sh.prof[4] - sh.prof[3]), (unsigned long)(sh.prof[5] - sh.prof[4]),
           (unsigned long)(t1 - sh.prof[5]),
           (unsigned long)(t2 - t1), (unsigned long)(wall_clock64() - t2));
#endif
  return r;
}

template <int T>
__device__ __forceinline__ int64_t key_fail_op(const GapKey &g, uint32_t at, GapSh &sh) {
  // the record whose return is event `at` (key-relative)
  if (threadIdx.x == 0) sh.res = INT_MAX;
  __syncthreads();
  for (int r = threadIdx.x; r < g.n; r += T)
    if (g.kops[r].ret == g.base + (int64_t)at) atomicMin(&sh.res, r);
  __syncthreads();
  const int r = sh.res;
  __syncthreads();
  return r == INT_MAX ? -1 : r;
}

// Probe j of P on the interval [lo, hi]: the candidates are lo..hi-1 (hi is
// known to fail).  Returns kNever when probe j has nothing to test.
__host__ __device__ __forceinline__ uint32_t probe_cut(uint32_t lo, uint32_t hi, int j, int P) {
  if (lo >= hi) return kNever;
  const uint64_t len = (uint64_t)(hi - lo);
  if (len <= (uint64_t)P) return (uint64_t)j < len ? lo + (uint32_t)j : kNever;
  return lo + (uint32_t)((uint64_t)(j + 1) * len / (uint64_t)(P + 1));
}

template <int T>
__global__ __launch_bounds__(T) void gap_tier_kernel(
    const lc_op *__restrict__ ops, const int64_t *__restrict__ key_off,
    const int32_t *__restrict__ keys, const KParams p, lc_key_result *__restrict__ out,
    int32_t *__restrict__ ws, const int64_t cap, int32_t *__restrict__ pass_keys,
    KStatus *__restrict__ status, const GapJob job) {
  __shared__ GapSh sh;
  const int64_t key_base = key_off[0];
  GapKey g;
  int32_t *const ws_hbm = ws + (size_t)blockIdx.x * kGapArrays * cap;
  g.sh = &sh;
  g.V0 = p.init_ver;
  g.init = p.init_val;
  for (int t = blockIdx.x; t < job.n_tasks; t += gridDim.x) {
    int ci = -1;  // counterexample index (probe / bisect)
    int64_t key;
    if (job.mode == kGapFull) {
      key = keys[t];
    } else {
      ci = t / job.P;
      key = job.cex_key[ci];
    }
    const int64_t beg = key_off[key], end = key_off[key + 1];
    if (end - beg <= 0 || end - beg + 2 > cap) {  // cannot happen past kGapFull
      if (threadIdx.x == 0 && job.mode == kGapFull)
        pass_keys[atomicAdd(&status->n_jit2, 1)] = (int32_t)key;
      continue;
    }
    g.kops = ops + (beg - key_base);
    g.n = (int)(end - beg);
    g.base = g.kops[0].call;
    // the skeleton goes to LDS when it fits with room for a small matching
    const int64_t capk = (end - beg + 2 + 3) & ~int64_t(3);
    const bool skel_lds = kSkelLdsBytes * capk + kMatchReserve <= job.lds_bytes;
    const GapWs<true> ws_l = gap_ws<true>(ws_hbm, capk);
    const GapWs<false> ws_g = gap_ws<false>(ws_hbm, cap);
    int64_t nodes = 0, wnodes = 0;
    int G = 0, G_full = 0;
    // this key's witness records (lc_aux), when witnesses are wanted
    int32_t *const kwit = job.wit ? job.wit + (beg - key_base) : nullptr;
    // One decision (full / probe / witness), or a bisection of decisions,
    // then with witnesses one more decision on the prefix before the failing
    // return.  One call site per skeleton placement keeps the kernel's code
    // and register budget in check.
    uint32_t lo = 0, hi = 0, cut = kNever;
    bool bis = false;    // bisecting a counterexample in this workgroup
    bool wpass = false;  // the decision that writes an invalid key's witness
    int32_t *wk = job.mode == kGapFull ? kwit : nullptr;
    if (job.mode == kGapProbe)
      cut = job.cex_state[ci] ? kNever
                              : probe_cut(job.cex_lo[ci], job.cex_hi[ci], t - ci * job.P, job.P);
    if (job.mode == kGapWitness) {  // a counterexample the multisection closed
      cut = (job.cex_state[ci] == 1 && job.cex_lo[ci] > 0) ? job.cex_lo[ci] - 1 : kNever;
      wk = kwit;
    }
    int res = GD_SKIP, wres = GD_SKIP;
    if (job.mode == kGapFull || cut != kNever) {
      for (;;) {
        int64_t *const nd = wpass || job.mode == kGapWitness ? &wnodes : &nodes;
        res = GD_RETRY;
        if (skel_lds) res = gap_decide<T, true>(g, ws_l, cut, job.lds_bytes, nd, &G, wk);
        // skeleton in HBM; or rare: a matching larger than the LDS left
        if (res == GD_RETRY) res = gap_decide<T, false>(g, ws_g, cut, job.lds_bytes, nd, &G, wk);
        if (wpass) {
          wres = res;
          res = GD_INVALID;
          break;
        }
        if (!bis) {
          if (job.mode != kGapFull || !job.bisect || res != GD_INVALID) break;
          bis = true;  // counterexample: the first return whose prefix fails
          wk = nullptr;
          G_full = G;
          lo = 0;
          hi = sh.maxret;
        } else if (res == GD_INVALID) {
          hi = cut;
        } else if (res == GD_VALID) {
          lo = cut + 1;
        } else {
          break;  // not decidable on a prefix: leave it to the JIT tier
        }
        if (lo >= hi) {
          res = GD_INVALID;
          if (!kwit || lo == 0) break;
          wpass = true;  // the prefix just before the failing return, with its witness
          wk = kwit;
          cut = lo - 1;
          continue;
        }
        cut = lo + (hi - lo) / 2;
      }
    }
    if (bis) {
      int64_t fail_op = -1;
      if (res == GD_INVALID) {
        fail_op = key_fail_op<T>(g, lo, sh);
        if (fail_op < 0) res = GD_NA;  // not a return: cannot happen
      }
      if (threadIdx.x == 0) {
        if (res == GD_INVALID) {
          out[key] = lc_key_result{LC_INVALID, LC_REASON_NONLINEARIZABLE, fail_op,
                                   g.base + (int64_t)lo, nodes, G_full};
          if (kwit) job.wkind[key] = wres == GD_VALID ? LC_WITNESS_PREFIX : LC_WITNESS_NONE;
        } else {
          pass_keys[atomicAdd(&status->n_jit2, 1)] = (int32_t)key;
        }
      }
    } else if (job.mode == kGapFull) {
      if (threadIdx.x == 0) {
        if (res == GD_VALID) {
          out[key] = lc_key_result{LC_VALID, LC_REASON_NONE, -1, -1, nodes, G};
          if (kwit) job.wkind[key] = LC_WITNESS_FULL;
        } else if (res == GD_INVALID) {
          const int i = atomicAdd(&status->n_cex, 1);
          job.cex_key[i] = (int32_t)key;
          job.cex_lo[i] = 0;
          job.cex_hi[i] = sh.maxret;
          job.cex_gaps[i] = G;
          job.cex_state[i] = 0;
          job.cex_nodes[i] = nodes;
          atomicMax(&status->max_lds, match_lds_bytes(G, sh.n_opt));
        } else {
          pass_keys[atomicAdd(&status->n_jit2, 1)] = (int32_t)key;
        }
      }
    } else if (job.mode == kGapWitness) {
      if (threadIdx.x == 0 && cut != kNever)
        job.wkind[key] = res == GD_VALID ? LC_WITNESS_PREFIX : LC_WITNESS_NONE;
    } else {  // kGapProbe
      if (threadIdx.x == 0) {
        job.probe[t] = res;
        if (nodes) atomicAdd((unsigned long long *)&job.cex_nodes[ci], (unsigned long long)nodes);
      }
    }
    __syncthreads();
  }
}

// One wave per counterexample interval: shrink [lo, hi] by the probes'
// verdicts; close it (result written) when lo == hi.
__global__ __launch_bounds__(kWave) void gap_narrow_kernel(
    const lc_op *__restrict__ ops, const int64_t *__restrict__ key_off, const int32_t n_cex,
    lc_key_result *__restrict__ out, int32_t *__restrict__ pass_keys,
    KStatus *__restrict__ status, const GapJob job) {
  const int ci = blockIdx.x, lane = threadIdx.x;
  if (ci >= n_cex || job.cex_state[ci]) return;
  const uint32_t lo = job.cex_lo[ci], hi = job.cex_hi[ci];
  uint32_t min_bad = hi;  // smallest failing cut
  uint32_t good_hi = lo;  // largest linearizable cut + 1
  bool na = false;
  for (int j = lane; j < job.P; j += kWave) {
    const uint32_t cut = probe_cut(lo, hi, j, job.P);
    if (cut == kNever) continue;
    const int r = job.probe[(int64_t)ci * job.P + j];
    if (r == GD_INVALID)
      min_bad = min(min_bad, cut);
    else if (r == GD_VALID)
      good_hi = max(good_hi, cut + 1);
    else
      na = true;
  }
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    min_bad = min(min_bad, (uint32_t)__shfl_xor((int)min_bad, o));
    good_hi = max(good_hi, (uint32_t)__shfl_xor((int)good_hi, o));
    na = na | (bool)__shfl_xor((int)na, o);
  }
  const int64_t key = job.cex_key[ci];
  const int64_t beg = key_off[key], end = key_off[key + 1];
  const lc_op *kops = ops + (beg - key_off[0]);
  // prefix-closed: every linearizable cut lies below every failing one
  // (give_up: the rounds did not converge; cannot happen with P >= 2 probes
  // per interval, but the JIT tier decides the key rather than the call fail)
  if (na || good_hi > min_bad || (job.give_up && good_hi < min_bad)) {
    if (lane == 0) {
      job.cex_state[ci] = 2;
      pass_keys[atomicAdd(&status->n_jit2, 1)] = (int32_t)key;
    }
    return;
  }
  if (good_hi < min_bad) {
    if (lane == 0) {
      job.cex_lo[ci] = good_hi;
      job.cex_hi[ci] = min_bad;
      atomicAdd(&status->n_open, 1);
    }
    return;
  }
  // closed: the first failing return is event `min_bad`
  const int64_t base = kops[0].call, at = base + (int64_t)min_bad;
  int fo = INT_MAX;
  for (int r = lane; r < (int)(end - beg); r += kWave)
    if (kops[r].ret == at) fo = min(fo, r);
  fo = wave_min_i32(fo);
  if (lane == 0) {
    job.cex_state[ci] = fo == INT_MAX ? 2 : 1;
    job.cex_lo[ci] = job.cex_hi[ci] = min_bad;
    if (fo == INT_MAX)
      pass_keys[atomicAdd(&status->n_jit2, 1)] = (int32_t)key;
    else
      out[key] = lc_key_result{LC_INVALID, LC_REASON_NONLINEARIZABLE, fo, at, job.cex_nodes[ci],
                               job.cex_gaps[ci]};
  }
}

}  // namespace

size_t gap_tier_ws_bytes(int n_wg, int64_t cap) {
  return (size_t)n_wg * kGapArrays * (size_t)cap * sizeof(int32_t);
}

template <int T>
hipError_t launch_gap_tier_t(const lc_op *d_ops, const int64_t *d_key_off, const int32_t *d_keys,
                             const KParams &p, lc_key_result *d_out, int32_t *d_ws, int n_wg,
                             int64_t cap, int32_t *d_pass_keys, KStatus *d_status,
                             const GapJob &job, hipStream_t stream) {
  if (job.lds_bytes > (64 << 10)) {  // beyond the default dynamic-LDS limit (gfx950: 160 KB per CU)
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(gap_tier_kernel<T>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             job.lds_bytes);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(gap_tier_kernel<T>, dim3((unsigned)n_wg), dim3(T), (unsigned)job.lds_bytes,
                     stream, d_ops, d_key_off, d_keys, p, d_out, d_ws, cap, d_pass_keys, d_status,
                     job);
  return hipGetLastError();
}

hipError_t launch_gap_tier(const lc_op *d_ops, const int64_t *d_key_off, const int32_t *d_keys,
                           const KParams &p, lc_key_result *d_out, int32_t *d_ws, int n_wg,
                           int64_t cap, int32_t *d_pass_keys, KStatus *d_status,
                           const GapJob &job, hipStream_t stream) {
  if (job.n_tasks <= 0) return hipSuccess;
  return job.threads == kWave
             ? launch_gap_tier_t<kWave>(d_ops, d_key_off, d_keys, p, d_out, d_ws, n_wg, cap,
                                        d_pass_keys, d_status, job, stream)
             : launch_gap_tier_t<kGapThreads>(d_ops, d_key_off, d_keys, p, d_out, d_ws, n_wg, cap,
                                              d_pass_keys, d_status, job, stream);
}

hipError_t launch_gap_narrow(const lc_op *d_ops, const int64_t *d_key_off, int32_t n_cex,
                             lc_key_result *d_out, int32_t *d_pass_keys, KStatus *d_status,
                             const GapJob &job, hipStream_t stream) {
  if (n_cex <= 0) return hipSuccess;
  hipLaunchKernelGGL(gap_narrow_kernel, dim3((unsigned)n_cex), dim3(kWave), 0, stream, d_ops,
                     d_key_off, n_cex, d_out, d_pass_keys, d_status, job);
  return hipGetLastError();
}

}  // namespace lcdev
