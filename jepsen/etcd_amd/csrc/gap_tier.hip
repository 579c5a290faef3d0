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
#include <atomic>
#include <climits>
#include <type_traits>

#include "gapmatch.h"
#include "kernels.h"
#include "records.h"
#include "wave.h"

namespace lcdev {
namespace {

constexpr int kGapThreads = 256;
// a few long keys' full decisions (GapJob::threads = 512): twice the waves
// for the setup's record passes and scans; the matching stays on wave 0
constexpr int kGapWideThreads = 512;
constexpr int kGapWaves = kGapWideThreads / kWave;  // (per-wave slots of the shared words)
constexpr int kGapArrays = 31;     // 32-bit arrays of `cap` entries per workgroup

enum { F_NA = 1, F_INVALID = 2 };



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
// (address space 3) when SL, global (1) otherwise, so the setup compiles to
// ds_* / global_* instructions rather than flat ones (a flat access waits on
// both the LDS and the vector-memory counters, and flat atomics to LDS are
// slow).  (Round 4: the HBM placement was generic — flat — until then.)
template <bool SL, class X>
using WsP = std::conditional_t<SL, __attribute__((address_space(3))) X *,
                               __attribute__((address_space(1))) X *>;

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

// load_raw (records.h) through a global-address-space pointer: global_*
// loads where the generic pointer of a non-inlined function gave flat ones
__device__ __forceinline__ Raw load_raw_g(const __attribute__((address_space(1))) lc_op *o, int i,
                                          int n) {
  Raw r;
  if (i < n) {
    const __attribute__((address_space(1))) long long *q =
        reinterpret_cast<const __attribute__((address_space(1))) long long *>(o + i);
    r.a = make_longlong2(q[0], q[1]);
    r.b = make_longlong2(q[2], q[3]);
    r.c = make_longlong2(q[4], q[5]);
  } else {
    r.a = make_longlong2(0, -1);
    r.b = make_longlong2(-1, -1);
    r.c = make_longlong2(-1, -1);  // call = ret = -1 marks "past the end"
  }
  return r;
}

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
  const int incl = wave_prefix_sum(v, lane);
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
  uint32_t incl;
  const uint32_t excl = wave_suffix_min_excl(v, lane, kNever, &incl);
  if (lane == 0) sh.wtotu[w] = incl;
  __syncthreads();
  uint32_t post = kNever;
#pragma unroll
  for (int j = 0; j < (T / kWave); j++)
    if (j > w) post = post < sh.wtotu[j] ? post : sh.wtotu[j];
  __syncthreads();
  return post < excl ? post : excl;
}

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

using GOp = const __attribute__((address_space(1))) lc_op;  // records in global memory

struct GapKey {
  GOp *kops;
  int n;
  int64_t base;  // call index of the key's first record
  int V0, init;
  int pref_budget;  // GapJob::pref_budget
};

// The workgroup's shared words, at namespace scope so every access is a ds_*
// instruction (through a pointer carried in GapKey they were flat ones).
__shared__ GapSh s_gsh;

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
  GapSh &sh = s_gsh;
  // Every wave must be done reading the previous decision's shared words
  // (sh.flag on its early-return paths, sh.maxret) before thread 0 resets
  // them: decisions follow each other without a barrier in the bisection.
  __syncthreads();
  for (int k = tid; k <= n; k += T) {
    w.A[k] = 0;  // max call + 1 of what must precede t_k; 0 = nothing
    w.B[k] = kNever;
    w.Pin[k] = -1;
    w.Claim[k] = kAny;
#ifdef GAP_SETUP_TOUCH  // A/B: also touch the arrays pass 1 writes first
    w.Val[k] = 0;
    w.PinExp[k] = kAny;
#endif
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
#if GAP_STOP_AT == 1  // dev timing builds (with GAP_STOP_SETUP): end the setup early
  return GD_VALID;
#endif
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
          raw[b] = load_raw_g(g.kops, r, n);
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
#if GAP_STOP_AT == 2
      return GD_VALID;
#endif
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
#if GAP_STOP_AT == 3
  return GD_VALID;
#endif
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
__device__ int gap_decide(const GapKey &g_arg, const GapWs<SL> &w_arg, uint32_t cut, int lds_bytes,
                          int64_t *nodes, int *n_gaps, int32_t *wk) {
  const int tid = threadIdx.x;
  GapSh &sh = s_gsh;
  // local copies: through the caller's references every field was reloaded
  // from the caller's stack after each store the compiler could not rule out
  // aliasing it (this function is not inlined)
  const GapKey g = g_arg;
  const GapWs<SL> w = w_arg;
#ifdef GAP_PROFILE
#ifdef GAP_WARM  // dev: a first setup pass whose result is dropped (cold-code cost)
  const uint64_t tw = wall_clock64();
  (void)gap_setup<T, SL>(g, w, cut);
  __syncthreads();
  if (tid == 0 && blockIdx.x < 2) printf("warm setup %lu (x10ns)\n", (unsigned long)(wall_clock64() - tw));
#endif
  const uint64_t t0 = wall_clock64();
  if (tid < 12) s_mprof[tid] = 0;
#endif
  const int st = gap_setup<T, SL>(g, w, cut);
  if (st != GD_VALID) return st;
#ifdef GAP_STOP_SETUP  // dev timing build: every decision ends after its setup (verdicts meaningless)
  return GD_VALID;
#endif
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
  // room for the class-indexed matching's copies of matched gap records
  const bool mgr_room = in_lds && 16 * w.moff + match_lds_bytes(G, n_opt) + match_mgr_bytes(n_opt) <= lds_bytes;
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
      r = match_branch(cl, G, n_opt, w.Claim, w.Req, w.PinExp, nodes, mgr_room, g.pref_budget);
    else
      r = match_branch(cg, G, n_opt, w.Claim, w.Req, w.PinExp, nodes, false, g.pref_budget);
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
    printf("  matching wg %d: first-fits %llu augments %llu steps %llu failed %llu | cycles: first-fit %llu augment %llu fill %llu; cursor steps %llu; bfs visit iters %llu cycles %llu ops %llu\n",
           (int)blockIdx.x, s_mprof[0], s_mprof[1], s_mprof[2], s_mprof[3], s_mprof[4],
           s_mprof[5], s_mprof[7], s_mprof[6], s_mprof[8], s_mprof[9], s_mprof[11]);
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
  GapSh &sh = s_gsh;
  const int64_t key_base = key_off[0];
  GapKey g;
  int32_t *const ws_hbm = ws + (size_t)blockIdx.x * kGapArrays * cap;
  g.V0 = p.init_ver;
  g.init = p.init_val;
  g.pref_budget = job.pref_budget;
  const int32_t n_tasks = job.n_tasks_dev ? min(job.n_tasks, *job.n_tasks_dev) : job.n_tasks;
  for (int t = blockIdx.x; t < n_tasks; t += gridDim.x) {
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
    g.kops = (GOp *)(ops + (beg - key_base));
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

constexpr int kMaxGapDevices = 64;

template <int T>
hipError_t launch_gap_tier_t(const lc_op *d_ops, const int64_t *d_key_off, const int32_t *d_keys,
                             const KParams &p, lc_key_result *d_out, int32_t *d_ws, int n_wg,
                             int64_t cap, int32_t *d_pass_keys, KStatus *d_status,
                             const GapJob &job, hipStream_t stream) {
  if (job.lds_bytes > (64 << 10)) {  // beyond the default dynamic-LDS limit (gfx950: 160 KB per CU)
    // once per device and kernel at the largest size asked for (a runtime
    // call on the launch path of every decision otherwise)
    static std::atomic<int> granted[kMaxGapDevices];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxGapDevices ||
        granted[dev].load(std::memory_order_relaxed) < job.lds_bytes) {
      const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(gap_tier_kernel<T>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               job.lds_bytes);
      if (e != hipSuccess) return e;
      if (dev >= 0 && dev < kMaxGapDevices) {
        int cur = granted[dev].load(std::memory_order_relaxed);
        while (cur < job.lds_bytes && !granted[dev].compare_exchange_weak(cur, job.lds_bytes)) {
        }
      }
    }
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
  if (job.threads == kWave)
    return launch_gap_tier_t<kWave>(d_ops, d_key_off, d_keys, p, d_out, d_ws, n_wg, cap,
                                    d_pass_keys, d_status, job, stream);
  if (job.threads == kGapWideThreads)
    return launch_gap_tier_t<kGapWideThreads>(d_ops, d_key_off, d_keys, p, d_out, d_ws, n_wg, cap,
                                              d_pass_keys, d_status, job, stream);
  return launch_gap_tier_t<kGapThreads>(d_ops, d_key_off, d_keys, p, d_out, d_ws, n_wg, cap,
                                        d_pass_keys, d_status, job, stream);
}

int gap_tier_resident(int lds_bytes, int threads) {
  const void *fn = threads == kGapWideThreads
                       ? reinterpret_cast<const void *>(gap_tier_kernel<kGapWideThreads>)
                       : reinterpret_cast<const void *>(gap_tier_kernel<kGapThreads>);
  if (lds_bytes > (64 << 10) &&
      hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes) != hipSuccess)
    return 0;
  int per_cu = 0, dev = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, threads, (size_t)lds_bytes) !=
          hipSuccess ||
      hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  return per_cu * cus;
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
