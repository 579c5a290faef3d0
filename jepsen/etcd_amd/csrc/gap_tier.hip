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
// One 256-thread workgroup decides one key: the record scan, the suffix-min
// scan, gap/optional-op compaction and every matching pass (greedy, then a
// level-synchronous BFS per augmenting path over all (frontier gap, op)
// pairs) are spread over the workgroup; the workspace (O(n) int32 arrays) is
// per workgroup in HBM/L2.  Keys it cannot decide (an :ok mutation without a
// version, a read [nil x], malformed records, the branch budget) go on to the
// JIT tier.
#include <algorithm>
#include <climits>

#include "kernels.h"
#include "records.h"

namespace lcdev {
namespace {

constexpr int kGapThreads = 256;
constexpr int kAny = INT_MIN;  // no value required / not a CAS
constexpr int kNodeBudget = 4096;  // matching passes per decision
constexpr int kGapArrays = 21;     // 32-bit arrays in GapWs

enum { GD_VALID = 1, GD_INVALID = 0, GD_NA = -1, GD_BUDGET = -2 };
enum { F_NA = 1, F_INVALID = 2 };

// Per-workgroup workspace: kGapArrays arrays of `cap` 32-bit entries.
struct GapWs {
  uint32_t *A, *B, *Uh, *OptCall;
  int *Pin, *Val, *PinExp, *Claim, *Req, *GI, *Gap, *OptVal, *OptExp, *OptPos;
  int *MatchOp, *MatchGap, *Par, *Fr0, *Fr1, *StPos, *StVal;
};

struct GapSh {
  int flag, maxpos, maxread, n_opt, n_gap, total;
  int found, n_next, viol, cand;
  uint32_t maxret;
  int wtot[kGapThreads / kWave];
  uint32_t wtotu[kGapThreads / kWave];
};

__device__ __forceinline__ GapWs gap_ws(int32_t *base, int64_t cap) {
  GapWs w;
  int32_t *p = base;
  auto nxt = [&]() {
    int32_t *q = p;
    p += cap;
    return q;
  };
  w.A = (uint32_t *)nxt();
  w.B = (uint32_t *)nxt();
  w.Uh = (uint32_t *)nxt();
  w.OptCall = (uint32_t *)nxt();
  w.Pin = nxt();
  w.Val = nxt();
  w.PinExp = nxt();
  w.Claim = nxt();
  w.Req = nxt();
  w.GI = nxt();
  w.Gap = nxt();
  w.OptVal = nxt();
  w.OptExp = nxt();
  w.OptPos = nxt();
  w.MatchOp = nxt();
  w.MatchGap = nxt();
  w.Par = nxt();
  w.Fr0 = nxt();
  w.Fr1 = nxt();
  w.StPos = nxt();
  w.StVal = nxt();
  return w;
}

// Exclusive prefix sum over the workgroup; *total = the sum of all v.
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
  for (int j = 0; j < kGapThreads / kWave; j++) {
    if (j < w) pre += sh.wtot[j];
    tot += sh.wtot[j];
  }
  __syncthreads();
  *total = tot;
  return pre + incl - v;
}

// Exclusive suffix minimum over the workgroup (threads above this one).
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
  for (int j = 0; j < kGapThreads / kWave; j++)
    if (j > w) post = post < sh.wtotu[j] ? post : sh.wtotu[j];
  uint32_t excl = (uint32_t)__shfl_down((int)incl, 1);
  if (lane == kWave - 1) excl = kNever;
  __syncthreads();
  return post < excl ? post : excl;
}

struct GapKey {
  const lc_op *kops;
  int n;
  int64_t base;  // call index of the key's first record
  int V0, init;
  GapWs ws;
  GapSh *sh;
};

__device__ __forceinline__ int value_before(const GapKey &g, int pos) {
  if (pos == 0) return g.init;
  return g.ws.Pin[pos - 1] != -1 ? g.ws.Val[pos - 1] : g.ws.Req[pos - 1];
}

// May optional op o fill gap gi under the current value requirements?
__device__ __forceinline__ bool eligible(const GapKey &g, int gi, int o) {
  const int pos = g.ws.Gap[gi];
  if (g.ws.OptCall[o] >= g.ws.Uh[pos]) return false;  // deadline
  const int opos = g.ws.OptPos[o];
  if (opos != -1 && opos != pos) return false;  // pending :ok op: its own version only
  const int rq = g.ws.Req[pos];
  if (rq != kAny && g.ws.OptVal[o] != rq) return false;
  const int e = g.ws.OptExp[o];
  if (e == kAny) return true;  // a write
  const int b = value_before(g, pos);
  return b == kAny || e == b;  // kAny: the gap before is free (checked later)
}

// Build the skeleton of the key's prefix at `cut` (key-relative event index;
// kNever = the whole history).  Returns GD_VALID when the skeleton is
// consistent (then sh.n_gap / sh.n_opt / sh.maxret are set), else
// GD_INVALID / GD_NA.
__device__ int gap_setup(const GapKey &g, uint32_t cut) {
  const int tid = threadIdx.x, n = g.n;
  GapSh &sh = *g.sh;
  const GapWs &w = g.ws;
  for (int k = tid; k <= n; k += kGapThreads) {
    w.A[k] = 0;  // max call + 1 of what must precede t_k; 0 = nothing
    w.B[k] = kNever;
    w.Pin[k] = -1;
    w.Claim[k] = kAny;
  }
  if (tid == 0) {
    sh.flag = 0;
    sh.maxpos = -1;
    sh.maxread = -1;
    sh.n_opt = 0;
    sh.maxret = 0;
  }
  __syncthreads();
  int flag = 0, maxpos = -1, maxread = -1;
  uint32_t maxret = 0;
  for (int r0 = 0; r0 < n; r0 += kGapThreads) {
    const int r = r0 + tid;
    bool opt = false;
    uint32_t ocall = 0;
    int oval = 0, oexp = 0, opos = 0;
    if (r < n) {
      const Raw raw = load_raw(g.kops, r, n);
      const Rec d = decode(raw, g.base);
      const bool unsorted = r > 0 && g.kops[r - 1].call >= raw.c.x;
      if (d.bad || d.f > LC_F_CAS || unsorted || raw.c.x < 0) {
        flag |= F_NA;  // the JIT tier reports malformed / unknown :f
      } else if (d.call <= cut) {
        const uint32_t ret = d.ret > cut ? kNever : d.ret;  // pending at the cut
        if (ret != kNever) maxret = max(maxret, ret);
        if (d.f == LC_F_READ) {
          if (ret == kNever || (d.ver == -1 && d.val == -1)) {
            // an optional or [nil nil] read never constrains
          } else if (d.ver == -1) {
            flag |= F_NA;  // read [nil x]: its version is free
          } else {
            const int k = d.ver - g.V0;
            if (k < 0 || k > n) {
              flag |= F_INVALID;
            } else {
              maxread = max(maxread, k);
              atomicMax(&w.A[k], d.call + 1);
              if (k > 0) atomicMin(&w.B[k - 1], ret);
              if (d.val != -1) {
                const int prev = atomicCAS(&w.Claim[k], kAny, d.val);
                if (prev != kAny && prev != d.val) flag |= F_INVALID;
              }
            }
          }
        } else if (ret == kNever) {
          const int pos = d.ver == -1 ? -1 : d.ver - g.V0 - 1;
          if (d.ver == -1 || (pos >= 0 && pos < n)) {  // else never placeable
            opt = true;
            ocall = d.call;
            oval = d.val;
            oexp = d.f == LC_F_CAS ? d.exp : kAny;
            opos = pos;
          }
        } else if (d.ver == -1) {
          flag |= F_NA;  // :ok mutation without a version: order not pinned
        } else {
          const int pos = d.ver - g.V0 - 1;
          if (pos < 0 || pos >= n || atomicCAS(&w.Pin[pos], -1, r) != -1) {
            flag |= F_INVALID;  // impossible version, or two mutations claim one
          } else {
            atomicMax(&w.A[pos], d.call + 1);
            atomicMin(&w.B[pos], ret);
            w.Val[pos] = d.val;
            w.PinExp[pos] = d.f == LC_F_CAS ? d.exp : kAny;
            maxpos = max(maxpos, pos);
          }
        }
      }
    }
    // stable append of the optional ops (record order)
    int tot;
    const int at = block_excl_sum(opt ? 1 : 0, sh, &tot);
    if (opt) {
      const int i = sh.n_opt + at;
      w.OptCall[i] = ocall;
      w.OptVal[i] = oval;
      w.OptExp[i] = oexp;
      w.OptPos[i] = opos;
    }
    __syncthreads();
    if (tid == 0) sh.n_opt += tot;
  }
  if (flag) atomicOr(&sh.flag, flag);
  if (maxpos >= 0) atomicMax(&sh.maxpos, maxpos);
  if (maxread >= 0) atomicMax(&sh.maxread, maxread);
  if (maxret) atomicMax(&sh.maxret, maxret);
  __syncthreads();
  if (sh.flag & F_NA) return GD_NA;
  if (sh.flag & F_INVALID) return GD_INVALID;
  const int M = max(sh.maxpos + 1, sh.maxread);
  // Uh[k] = min(B[k..M-1]): chunked suffix-min scan
  const int per = (M + kGapThreads - 1) / kGapThreads;
  const int k0 = min(tid * per, M), k1 = min(k0 + per, M);
  uint32_t loc = kNever;
  for (int k = k0; k < k1; k++) loc = min(loc, w.B[k]);
  uint32_t run = block_suffix_min_excl(loc, sh);
  for (int k = k1 - 1; k >= k0; k--) {
    run = min(run, w.B[k]);
    w.Uh[k] = run;
  }
  __syncthreads();
  // fixed checks: pinned / read-only lower bounds below the deadline, and
  // the value chain around pinned positions; the requirement on each gap
  flag = 0;
  if (tid == 0) {
    if (w.Claim[0] != kAny && w.Claim[0] != g.init) flag |= F_INVALID;
    if (M > 0 && w.Pin[0] != -1 && w.PinExp[0] != kAny && w.PinExp[0] != g.init)
      flag |= F_INVALID;
  }
  for (int k = tid; k < M; k += kGapThreads) {
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
    }
  }
  // stable compaction of the gap positions
  if (tid == 0) sh.n_gap = 0;
  __syncthreads();
  for (int c0 = 0; c0 < M; c0 += kGapThreads) {
    const int k = c0 + tid;
    const bool gap = k < M && w.Pin[k] == -1;
    int tot;
    const int at = block_excl_sum(gap ? 1 : 0, sh, &tot);
    if (gap) {
      w.Gap[sh.n_gap + at] = k;
      w.GI[k] = sh.n_gap + at;
    }
    __syncthreads();
    if (tid == 0) sh.n_gap += tot;
  }
  if (flag) atomicOr(&sh.flag, flag);
  __syncthreads();
  return (sh.flag & F_INVALID) ? GD_INVALID : GD_VALID;
}

// Maximum matching of the gaps; true iff every gap is filled.
__device__ bool gap_match(const GapKey &g, int G, int n_opt) {
  const int tid = threadIdx.x;
  GapSh &sh = *g.sh;
  const GapWs &w = g.ws;
  for (int o = tid; o < n_opt; o += kGapThreads) w.MatchOp[o] = -1;
  for (int i = tid; i < G; i += kGapThreads) w.MatchGap[i] = -1;
  __syncthreads();
  for (int gi = 0; gi < G; gi++) {
    // greedy: the first free eligible op
    if (tid == 0) sh.cand = INT_MAX;
    __syncthreads();
    for (int o = tid; o < n_opt; o += kGapThreads)
      if (w.MatchOp[o] == -1 && eligible(g, gi, o)) atomicMin(&sh.cand, o);
    __syncthreads();
    const int c = sh.cand;
    __syncthreads();
    if (c != INT_MAX) {
      if (tid == 0) {
        w.MatchOp[c] = gi;
        w.MatchGap[gi] = c;
      }
      __syncthreads();
      continue;
    }
    // augmenting path: level-synchronous BFS over (frontier gap, op) pairs
    for (int o = tid; o < n_opt; o += kGapThreads) w.Par[o] = -1;
    if (tid == 0) {
      w.Fr0[0] = gi;
      sh.found = INT_MAX;
    }
    int nf = 1;
    int *fr = w.Fr0, *fn = w.Fr1;
    __syncthreads();
    for (;;) {
      if (tid == 0) sh.n_next = 0;
      __syncthreads();
      const int64_t total = (int64_t)nf * n_opt;
      for (int64_t idx = tid; idx < total; idx += kGapThreads) {
        const int f = fr[idx / n_opt], o = (int)(idx % n_opt);
        if (eligible(g, f, o) && atomicCAS(&w.Par[o], -1, f) == -1) {
          const int m = w.MatchOp[o];
          if (m == -1)
            atomicMin(&sh.found, o);
          else
            fn[atomicAdd(&sh.n_next, 1)] = m;
        }
      }
      __syncthreads();
      nf = sh.n_next;
      const int found = sh.found;
      __syncthreads();
      if (found != INT_MAX || nf == 0) break;
      int *t = fr;
      fr = fn;
      fn = t;
    }
    const int found = sh.found;
    if (found == INT_MAX) return false;  // Hall's condition fails at gi
    if (tid == 0) {
      int o = found;
      for (;;) {
        const int gg = w.Par[o];
        const int prev = w.MatchGap[gg];
        w.MatchGap[gg] = o;
        w.MatchOp[o] = gg;
        if (gg == gi) break;
        o = prev;
      }
    }
    __syncthreads();
  }
  return true;
}

// Smallest value > last among the ops eligible for the gap at position pos
// (INT_MAX if none).
__device__ int next_value(const GapKey &g, int pos, int last, int n_opt) {
  GapSh &sh = *g.sh;
  if (threadIdx.x == 0) sh.cand = INT_MAX;
  __syncthreads();
  const int gi = g.ws.GI[pos];
  for (int o = threadIdx.x; o < n_opt; o += kGapThreads) {
    const int v = g.ws.OptVal[o];
    if (v > last && eligible(g, gi, o)) atomicMin(&sh.cand, v);
  }
  __syncthreads();
  const int c = sh.cand;
  __syncthreads();
  return c;
}

// Decide the prefix at `cut`.  *nodes accumulates matching passes.
__device__ int gap_decide(const GapKey &g, uint32_t cut, int64_t *nodes, int *n_gaps) {
  const int tid = threadIdx.x;
  GapSh &sh = *g.sh;
  const GapWs &w = g.ws;
  const int st = gap_setup(g, cut);
  if (st != GD_VALID) return st;
  const int G = sh.n_gap, n_opt = sh.n_opt;
  *n_gaps = G;
  if (G == 0) return GD_VALID;
  if (G > n_opt) return GD_INVALID;
  int depth = 0;
  for (int node = 0;; node++) {
    if (node >= kNodeBudget) return GD_BUDGET;
    (*nodes)++;
    if (gap_match(g, G, n_opt)) {
      // the matching ignored CAS expectations after free gaps: check them
      if (tid == 0) sh.viol = INT_MAX;
      __syncthreads();
      for (int gi = tid; gi < G; gi += kGapThreads) {
        const int pos = w.Gap[gi];
        if (pos == 0 || w.Pin[pos - 1] != -1 || w.Req[pos - 1] != kAny) continue;
        const int e = w.OptExp[w.MatchGap[gi]];
        if (e != kAny && w.OptVal[w.MatchGap[w.GI[pos - 1]]] != e) atomicMin(&sh.viol, pos - 1);
      }
      __syncthreads();
      const int viol = sh.viol;
      __syncthreads();
      if (viol == INT_MAX) return GD_VALID;
      // branch on the value of the free gap at position viol
      const int v = next_value(g, viol, INT_MIN, n_opt);
      if (tid == 0) {
        w.StPos[depth] = viol;
        w.StVal[depth] = v;
        w.Req[viol] = v;
      }
      depth++;
      __syncthreads();
      continue;
    }
    // no filling: next value of the deepest branch, else backtrack
    for (;;) {
      if (depth == 0) return GD_INVALID;
      const int pos = w.StPos[depth - 1], last = w.StVal[depth - 1];
      __syncthreads();
      if (tid == 0) w.Req[pos] = kAny;
      __syncthreads();
      const int v = next_value(g, pos, last, n_opt);
      if (v != INT_MAX) {
        if (tid == 0) {
          w.StVal[depth - 1] = v;
          w.Req[pos] = v;
        }
        __syncthreads();
        break;
      }
      depth--;
    }
  }
}

__global__ __launch_bounds__(kGapThreads) void gap_tier_kernel(
    const lc_op *__restrict__ ops, const int64_t *__restrict__ key_off,
    const int32_t *__restrict__ keys, const int32_t n_list, const KParams p,
    lc_key_result *__restrict__ out, int32_t *__restrict__ ws, const int64_t cap,
    int32_t *__restrict__ pass_keys, KStatus *__restrict__ status) {
  __shared__ GapSh sh;
  const int64_t key_base = key_off[0];
  GapKey g;
  g.ws = gap_ws(ws + (size_t)blockIdx.x * kGapArrays * cap, cap);
  g.sh = &sh;
  g.V0 = p.init_ver;
  g.init = p.init_val;
  for (int li = blockIdx.x; li < n_list; li += gridDim.x) {
    const int64_t key = keys[li];
    const int64_t beg = key_off[key], end = key_off[key + 1];
    int res = GD_NA;
    int64_t nodes = 0, fail_op = -1, fail_end = -1;
    int G = 0;
    if (end - beg > 0 && end - beg + 2 <= cap) {
      g.kops = ops + (beg - key_base);
      g.n = (int)(end - beg);
      g.base = g.kops[0].call;
      res = gap_decide(g, kNever, &nodes, &G);
      if (res == GD_INVALID) {
        // bisection for the first return whose prefix is not linearizable
        uint32_t lo = 0, hi = sh.maxret;
        __syncthreads();
        int g2 = 0;
        while (lo < hi && res == GD_INVALID) {
          const uint32_t mid = lo + (hi - lo) / 2;
          const int r = gap_decide(g, mid, &nodes, &g2);
          if (r == GD_INVALID)
            hi = mid;
          else if (r == GD_VALID)
            lo = mid + 1;
          else
            res = r;  // not decidable on a prefix: leave it to the JIT tier
        }
        if (res == GD_INVALID) {
          if (threadIdx.x == 0) sh.cand = INT_MAX;
          __syncthreads();
          for (int r = threadIdx.x; r < g.n; r += kGapThreads)
            if (g.kops[r].ret == g.base + (int64_t)lo) atomicMin(&sh.cand, r);
          __syncthreads();
          if (sh.cand == INT_MAX) res = GD_NA;  // not a return: cannot happen
          fail_op = sh.cand;
          fail_end = g.base + (int64_t)lo;
          __syncthreads();
        }
      }
    }
    if (threadIdx.x == 0) {
      if (res == GD_VALID)
        out[key] = lc_key_result{LC_VALID, LC_REASON_NONE, -1, -1, nodes, G};
      else if (res == GD_INVALID)
        out[key] = lc_key_result{LC_INVALID, LC_REASON_NONLINEARIZABLE, fail_op, fail_end,
                                 nodes, G};
      else
        pass_keys[atomicAdd(&status->n_jit2, 1)] = (int32_t)key;
    }
    __syncthreads();
  }
}

}  // namespace

size_t gap_tier_ws_bytes(int n_wg, int64_t cap) {
  return (size_t)n_wg * kGapArrays * (size_t)cap * sizeof(int32_t);
}

hipError_t launch_gap_tier(const lc_op *d_ops, const int64_t *d_key_off, const int32_t *d_keys,
                           int32_t n_list, const KParams &p, lc_key_result *d_out,
                           int32_t *d_ws, int n_wg, int64_t cap, int32_t *d_pass_keys,
                           KStatus *d_status, hipStream_t stream) {
  if (n_list <= 0) return hipSuccess;
  hipLaunchKernelGGL(gap_tier_kernel, dim3((unsigned)n_wg), dim3(kGapThreads), 0, stream,
                     d_ops, d_key_off, d_keys, n_list, p, d_out, d_ws, cap, d_pass_keys,
                     d_status);
  return hipGetLastError();
}

}  // namespace lcdev
