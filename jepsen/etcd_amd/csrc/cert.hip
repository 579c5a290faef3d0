// cert.hip — infeasibility certificates for invalid keys (lc_aux
// certificate / certificate_set, include/lincheck.h, ABI 3).
//
// An invalid key's PREFIX witness shows that the history prefix just before
// its failing return is linearizable; the certificate written here names
// facts that rule out every linearization of the prefix AT the failing
// return, so the pair certifies the fail op as the first failure (prefix
// closure).  oracle/cert.c checks the facts from the records alone.
//
// The facts are those of the version order (register.clj:60-96): a mutation
// claiming version v holds position v-V0-1 in every linearization, a read of
// version v reads the value written at v-V0-1, a CAS expects the value
// before it, and real time orders the points.  In the prefix P at the
// failing return, in order of the search:
//   UNREACH  a required op claims a version P cannot reach;
//   DUP      two required mutations claim one version;
//   CLAIMS   two required reads of one version read different values;
//   PAIR     a required CAS / read against the required mutation before it;
//   ORDER    the version order puts a's point before b's, yet b returned
//            before a was called (L_j > Uh_j, the gap tier's fixed check);
//   HALL     a needed position no required op holds that no op of P can
//            hold (its candidates: mutations of P pinned to it or to none,
//            called before its deadline, writing the value its successors
//            need, expecting the value before it where P fixes that);
//   PAIR     two needed positions whose only candidates disagree on the
//            value between them (a CAS expecting another value);
//   HALL     the needed open positions together outnumber their candidates.
// The first five are the gap tier's fixed checks (gap_tier.hip,
// gap_setup); the last three its matching's infeasibility at the root.  A
// failure that only the matching's branching finds (a free value chosen
// wrong) gets no certificate (LC_CERT_NONE) — none has been seen at a
// failing prefix of the test batches, where the returning op itself
// completes a fixed contradiction (tests/test_cert.py restates this search
// in tests/cert_ref.py and checks it on the oracle's own failing prefixes).
//
// One 256-thread workgroup per key of the call (those not invalid leave at
// once); its arrays live in a workspace of kCertSlots int32 per (record + 2)
// of the batch.  Run when the caller asks for certificates and some key can
// be invalid (a call whose version-order pass decided every key has none:
// lincheck.cpp, run_certificates); the drop-ins ask for them on every call
// (dropin_leg in bench.py times it on C5).
#include <algorithm>
#include <climits>

#include "kernels.h"
#include "records.h"
#include "wave.h"

namespace lcdev {
namespace {

constexpr int kCertThreads = 256;
// Workspace per (record + 2) of the batch, in int32 slots: seven int32
// arrays, two uint64 arrays (two slots each) and the candidate list (int4,
// four slots); the stride is a multiple of 4 so the wide arrays stay aligned.
constexpr int kCertSlots = 7 + 2 * 2 + 4;
constexpr int kFree = INT_MIN;  // no value fixed

struct CertSh {
  int n_mut, m_need, n_gap, n_cand;
  unsigned long long best;  // a stage's lowest (a+1, b+1) pair found
  int pos;                  // a stage's lowest position found
  int rb;                   // PAIR: the lowest consumer
  int n_u;                  // HALL: unpinned candidates listed
  unsigned long long wmin[kCertThreads / kWave];
  int cnt[kCertThreads];    // HALL: per-thread candidate counts, then their prefix
};

__device__ __forceinline__ void cert_write(int32_t *c, int kind, int a, int b, int x) {
  c[0] = kind;
  c[1] = a;
  c[2] = b;
  c[3] = x;
}

__device__ __forceinline__ unsigned long long shfl_down64(unsigned long long v, int o) {
  const uint32_t lo = (uint32_t)__shfl_down((int)(uint32_t)v, o);
  const uint32_t hi = (uint32_t)__shfl_down((int)(uint32_t)(v >> 32), o);
  return ((unsigned long long)hi << 32) | lo;
}

__global__ __launch_bounds__(kCertThreads) void cert_kernel(
    const lc_op *__restrict__ ops, const int64_t *__restrict__ key_off, const KParams p,
    const lc_key_result *__restrict__ res, int32_t *__restrict__ ws, int64_t ws_stride,
    int32_t *__restrict__ cert, int32_t *__restrict__ cset) {
  __shared__ CertSh sh;
  const int64_t key = blockIdx.x;
  const int tid = threadIdx.x;
  int32_t *c = cert + 4 * key;
  if (res[key].verdict != LC_INVALID) {
    if (tid == 0) cert_write(c, LC_CERT_NONE, -1, -1, 0);
    return;
  }
  const int64_t beg = key_off[key], end = key_off[key + 1];
  const int64_t rb = beg - key_off[0];
  const int n = (int)(end - beg);
  const lc_op *kops = ops + rb;
  int32_t *ks = cset + rb;
  const int64_t base = n > 0 ? kops[0].call : 0;
  const int64_t cut64 = res[key].fail_prefix_end - base;
  const uint32_t cut = cut64 < 0 ? 0u : cut64 >= (int64_t)kNever ? kNever - 1 : (uint32_t)cut64;
  const int V0 = p.init_ver, init = p.init_val;
  // this key's arrays, positions / records 0..n+1 (ws_stride slots per int32 array)
  const int64_t off = rb + 2 * key;
  int *held_rec = ws + off;                  // lowest required mutation pinned at k
  int *held_cnt = ws + ws_stride + off;      // how many; for an open position: its one candidate
  int *claim_rec = ws + 2 * ws_stride + off; // lowest required read of version V0+k with a value
  int *cnt = ws + 3 * ws_stride + off;       // open positions: candidate count
  int *mark = ws + 4 * ws_stride + off;      // records: a candidate of some open position
  int *pin_head = ws + 5 * ws_stride + off;  // positions: pending :ok mutations pinned there (list)
  int *pin_next = ws + 6 * ws_stride + off;  // records: the next of that list
  // bounds with the record that sets them: (call + 1) << 32 | r, max; ret << 32 | r, min
  unsigned long long *lo64 = reinterpret_cast<unsigned long long *>(ws + 7 * ws_stride) + off;
  unsigned long long *uh64 = reinterpret_cast<unsigned long long *>(ws + 9 * ws_stride) + off;
  int4 *ulist = reinterpret_cast<int4 *>(ws + 11 * ws_stride) + off;  // HALL: unpinned candidates
  constexpr unsigned long long kUhNone = ((unsigned long long)kNever << 32) | 0xFFFFFFFFull;
  for (int k = tid; k <= n + 1; k += kCertThreads) {
    held_rec[k] = INT_MAX;
    held_cnt[k] = 0;
    claim_rec[k] = INT_MAX;
    cnt[k] = -1;
    mark[k] = 0;
    pin_head[k] = -1;
    lo64[k] = 0;
    uh64[k] = kUhNone;
  }
  if (tid == 0) {
    sh.n_mut = sh.m_need = sh.n_gap = sh.n_cand = sh.n_u = 0;
    sh.best = ~0ull;
    sh.pos = sh.rb = INT_MAX;
    cert_write(c, LC_CERT_NONE, -1, -1, 0);
  }
  __syncthreads();
  auto rec = [&](int r) { return decode(load_raw(kops, r, n), base); };
  auto in_p = [&](const Rec &d) { return d.call <= cut; };
  auto req = [&](const Rec &d) { return d.call <= cut && d.ret <= cut; };
  auto is_mut = [](const Rec &d) { return d.f == LC_F_WRITE || d.f == LC_F_CAS; };
  auto found = [&](int a, int b) {
    atomicMin(&sh.best, ((unsigned long long)(uint32_t)(a + 1) << 32) | (uint32_t)(b + 1));
  };
  // a stage's lowest find, written as `kind`; uniform across the workgroup
  auto emit = [&](int kind) {
    const unsigned long long bst = sh.best;
    if (bst == ~0ull) return false;
    if (tid == 0) cert_write(c, kind, (int)(bst >> 32) - 1, (int)(uint32_t)bst - 1, 0);
    return true;
  };
  // mutations in P
  int nm = 0;
  for (int r = tid; r < n; r += kCertThreads) {
    const Rec d = rec(r);
    nm += in_p(d) && is_mut(d);
  }
  atomicAdd(&sh.n_mut, nm);
  __syncthreads();
  const int n_mut = sh.n_mut;
  // UNREACH; and the positions held, the claims, the bounds of the required ops
  int need = 0;
  for (int r = tid; r < n; r += kCertThreads) {
    const Rec d = rec(r);
    if (!req(d) || d.ver == -1 || d.bad) continue;
    const unsigned long long lo = ((unsigned long long)(d.call + 1) << 32) | (uint32_t)r;
    const unsigned long long hi = ((unsigned long long)d.ret << 32) | (uint32_t)r;
    if (is_mut(d)) {
      const int pos = d.ver - V0 - 1;
      if (pos < 0 || pos + 1 > n_mut) {
        found(r, -1);
        continue;
      }
      atomicAdd(&held_cnt[pos], 1);
      atomicMin(&held_rec[pos], r);
      atomicMax(&lo64[pos], lo);
      atomicMin(&uh64[pos], hi);
      need = max(need, pos + 1);
    } else if (d.f == LC_F_READ) {
      const int k = d.ver - V0;
      if (k < 0 || k > n_mut || (k == 0 && d.val != -1 && d.val != init)) {
        found(r, -1);
        continue;
      }
      if (d.val != -1) atomicMin(&claim_rec[k], r);
      atomicMax(&lo64[k], lo);
      if (k > 0) atomicMin(&uh64[k - 1], hi);
      need = max(need, k);
    }
  }
  atomicMax(&sh.m_need, need);
  __syncthreads();
  if (emit(LC_CERT_UNREACH)) return;
  const int M = sh.m_need;
  // DUP
  for (int r = tid; r < n; r += kCertThreads) {
    const Rec d = rec(r);
    if (!req(d) || !is_mut(d) || d.ver == -1 || d.bad) continue;
    const int pos = d.ver - V0 - 1;
    if (held_cnt[pos] > 1 && held_rec[pos] != r) found(held_rec[pos], r);
  }
  __syncthreads();
  if (emit(LC_CERT_DUP)) return;
  // CLAIMS
  for (int r = tid; r < n; r += kCertThreads) {
    const Rec d = rec(r);
    if (!req(d) || d.f != LC_F_READ || d.ver == -1 || d.val == -1 || d.bad) continue;
    const int o = claim_rec[d.ver - V0];
    if (o != r && (int)kops[o].value != d.val) found(o, r);
  }
  __syncthreads();
  if (emit(LC_CERT_CLAIMS)) return;
  // PAIR against a required holder: the lowest consumer position q
  for (int r = tid; r < n; r += kCertThreads) {
    const Rec d = rec(r);
    if (!req(d) || d.ver == -1 || d.bad) continue;
    int q = -1, want = 0;
    if (d.f == LC_F_CAS) q = d.ver - V0 - 1, want = d.exp;
    else if (d.f == LC_F_READ && d.val != -1) q = d.ver - V0, want = d.val;
    if ((q == 0 && d.f == LC_F_CAS && want != init) ||
        (q >= 1 && held_rec[q - 1] != INT_MAX && (int)kops[held_rec[q - 1]].value != want))
      atomicMin(&sh.pos, q);
  }
  __syncthreads();
  if (sh.pos != INT_MAX) {
    const int q = sh.pos;
    for (int r = tid; r < n; r += kCertThreads) {  // its lowest consumer
      const Rec d = rec(r);
      if (!req(d) || d.ver == -1 || d.bad) continue;
      int want;
      if (d.f == LC_F_CAS && d.ver - V0 - 1 == q) want = d.exp;
      else if (d.f == LC_F_READ && d.val != -1 && d.ver - V0 == q) want = d.val;
      else continue;
      const int have = q == 0 ? init : (int)kops[held_rec[q - 1]].value;
      if (want != have) atomicMin(&sh.rb, r);
    }
    __syncthreads();
    if (tid == 0) cert_write(c, LC_CERT_PAIR, q == 0 ? -1 : held_rec[q - 1], sh.rb, q);
    return;
  }
  // ORDER: the suffix minimum of the upper bounds, then a lower bound above
  // it; each bound carries the record that sets it (a record
  // found by matching timestamps could be an unrelated op's)
  const int L = M + 1;  // indices 0..M (reads of the last version bound index M from below)
  {
    const int per = (L + kCertThreads - 1) / kCertThreads;
    const int k0 = min(tid * per, L), k1 = min(k0 + per, L);
    unsigned long long loc = kUhNone;
    for (int k = k0; k < k1; k++) loc = min(loc, uh64[k]);
    const int lane = tid & (kWave - 1), wv = tid / kWave;
    unsigned long long incl = loc;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const unsigned long long y = shfl_down64(incl, o);
      if (lane + o < kWave) incl = min(incl, y);
    }
    if (lane == 0) sh.wmin[wv] = incl;
    unsigned long long run = shfl_down64(incl, 1);
    if (lane == kWave - 1) run = kUhNone;
    __syncthreads();
    for (int j = wv + 1; j < kCertThreads / kWave; j++) run = min(run, sh.wmin[j]);
    for (int k = k1 - 1; k >= k0; k--) {
      run = min(run, uh64[k]);
      uh64[k] = run;
    }
  }
  __syncthreads();
  for (int k = tid; k < L; k += kCertThreads) {
    const uint32_t lo = (uint32_t)(lo64[k] >> 32);  // call + 1, 0: none
    if (lo != 0 && lo - 1 > (uint32_t)(uh64[k] >> 32)) atomicMin(&sh.pos, k);
  }
  __syncthreads();
  if (sh.pos != INT_MAX) {
    // a: the op whose call is the lower bound, b: the op whose return is the
    // upper bound
    const int j = sh.pos;
    if (tid == 0)
      cert_write(c, LC_CERT_ORDER, (int)(uint32_t)lo64[j], (int)(uint32_t)uh64[j], 0);
    return;
  }
  // The open positions (needed, held by no required op) and their
  // candidates: the mutations of P without a version, listed once in call
  // order (each thread takes a contiguous run of records, their counts
  // prefix-summed), and the pending :ok mutations pinned to the position
  // (linked per position).  An open position scans the list only up to its
  // deadline: O(open positions x candidates called before it) instead of a
  // pass over every record per position.
  {
    const int per = (n + kCertThreads - 1) / kCertThreads;
    const int r0 = min(tid * per, n), r1 = min(r0 + per, n);
    int u = 0;
    for (int r = r0; r < r1; r++) {
      const Rec d = rec(r);
      if (!in_p(d) || !is_mut(d) || d.bad) continue;
      if (d.ver == -1) {
        u++;
      } else if (!req(d)) {
        const int g = d.ver - V0 - 1;
        if (g >= 0 && g <= n) pin_next[r] = atomicExch(&pin_head[g], r);
      }
    }
    sh.cnt[tid] = u;
    __syncthreads();
    if (tid == 0) {
      int acc = 0;
      for (int t = 0; t < kCertThreads; t++) {
        const int x = sh.cnt[t];
        sh.cnt[t] = acc;
        acc += x;
      }
      sh.n_u = acc;
    }
    __syncthreads();
    int at = sh.cnt[tid];
    for (int r = r0; r < r1; r++) {
      const Rec d = rec(r);
      if (in_p(d) && is_mut(d) && !d.bad && d.ver == -1)
        ulist[at++] = make_int4((int)d.call, d.val, d.f == LC_F_CAS ? d.exp : kFree, r);
    }
  }
  __syncthreads();
  const int n_u = sh.n_u;
  int n_gap = 0;
  for (int g = tid; g < M; g += kCertThreads) {
    if (held_rec[g] != INT_MAX) continue;
    n_gap++;
    // what its holder must write; what a CAS holding it must expect
    int want = kFree, before = kFree;
    bool clash = false;
    if (held_rec[g + 1] != INT_MAX && kops[held_rec[g + 1]].f == LC_F_CAS)
      want = (int)kops[held_rec[g + 1]].expected;
    if (claim_rec[g + 1] != INT_MAX) {
      const int v = (int)kops[claim_rec[g + 1]].value;
      clash = want != kFree && want != v;
      want = v;
    }
    if (g == 0) before = init;
    else if (held_rec[g - 1] != INT_MAX) before = (int)kops[held_rec[g - 1]].value;
    else if (claim_rec[g] != INT_MAX) before = (int)kops[claim_rec[g]].value;
    const uint32_t dl = (uint32_t)(uh64[g] >> 32);
    int k = 0, one = -1;
    if (!clash) {
      for (int j = 0; j < n_u; j++) {
        const int4 e = ulist[j];
        if ((uint32_t)e.x >= dl) break;  // (call order)
        if (e.z != kFree && before != kFree && e.z != before) continue;
        if (want != kFree && e.y != want) continue;
        k++;
        one = e.w;
        mark[e.w] = 1;
      }
      for (int x = pin_head[g]; x >= 0; x = pin_next[x]) {
        const Rec d = rec(x);
        if (d.call >= dl) continue;
        if (d.f == LC_F_CAS && before != kFree && d.exp != before) continue;
        if (want != kFree && d.val != want) continue;
        k++;
        one = x;
        mark[x] = 1;
      }
    }
    cnt[g] = k;
    held_cnt[g] = one;
    if (k == 0) atomicMin(&sh.pos, g);
  }
  atomicAdd(&sh.n_gap, n_gap);
  __syncthreads();
  if (sh.pos != INT_MAX) {
    if (tid == 0) {
      ks[0] = sh.pos;
      cert_write(c, LC_CERT_HALL, -1, -1, 1);
    }
    return;
  }
  // two open positions whose only candidates disagree on the value between
  // them (or a required holder before an open one)
  for (int q = 1 + tid; q < M; q += kCertThreads) {
    if (cnt[q] != 1 || kops[held_cnt[q]].f != LC_F_CAS) continue;
    const int a = held_rec[q - 1] != INT_MAX ? held_rec[q - 1] : cnt[q - 1] == 1 ? held_cnt[q - 1] : -1;
    if (a >= 0 && kops[a].value != kops[held_cnt[q]].expected) atomicMin(&sh.pos, q);
  }
  __syncthreads();
  if (sh.pos != INT_MAX) {
    if (tid == 0) {
      const int q = sh.pos;
      cert_write(c, LC_CERT_PAIR,
                 held_rec[q - 1] != INT_MAX ? held_rec[q - 1] : held_cnt[q - 1], held_cnt[q], q);
    }
    return;
  }
  // Hall's condition over every open position
  int u = 0;
  for (int x = tid; x < n; x += kCertThreads) u += mark[x] != 0;
  atomicAdd(&sh.n_cand, u);
  __syncthreads();
  if (sh.n_gap > sh.n_cand) {
    if (tid == 0) {
      int i = 0;
      for (int g = 0; g < M; g++)
        if (held_rec[g] == INT_MAX) ks[i++] = g;
      cert_write(c, LC_CERT_HALL, -1, -1, i);
    }
    return;
  }
  // Infeasibility only a search finds: a PROOF — its case splits; the
  // forced choices between them and the empty positions that close each
  // case are re-derived by the checker's propagation (tests/cert_ref.py
  // prove, oracle/cert.c proof_ok) — searched by wave 0 (the other waves
  // are done).
  if (tid >= kWave) return;
  // the arrays free by now: the open positions' list (cnt), the assumed
  // holder per position (held_cnt), the assumed ops (mark), the log of
  // assumed positions and the case-split frames (lo64's slots)
  int *glist = cnt, *asg = held_cnt, *used = mark;
  int *logp = reinterpret_cast<int *>(lo64);
  int4 *frames = reinterpret_cast<int4 *>(logp + ((n + 2 + 3) & ~3));
  const int n_frames = (n + 2) / 4;
  int ng = 0;  // the open positions, in order
  for (int g = 0; g < M; g++)
    if (held_rec[g] == INT_MAX) {
      if (tid == 0) glist[ng] = g;
      ng++;
    }
  for (int k = tid; k <= n + 1; k += kWave) {
    asg[k] = -1;
    used[k] = 0;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  if (ng < 1 || n > 0x7FFF || M > 0x7FFF) return;
  // candidates of open position g under the assumptions: their count and
  // the lowest record index above `after` (one lane, sequential)
  long long work = 0;
  auto cands = [&](int g, int after, int *first) -> int {
    int want = kFree, before = kFree;
    if (held_rec[g + 1] != INT_MAX && kops[held_rec[g + 1]].f == LC_F_CAS)
      want = (int)kops[held_rec[g + 1]].expected;
    if (claim_rec[g + 1] != INT_MAX) {
      const int v = (int)kops[claim_rec[g + 1]].value;
      if (want != kFree && want != v) return 0;
      want = v;
    }
    if (g + 1 < M && asg[g + 1] >= 0 && kops[asg[g + 1]].f == LC_F_CAS) {
      const int v = (int)kops[asg[g + 1]].expected;
      if (want != kFree && want != v) return 0;
      want = v;
    }
    if (g == 0) before = init;
    else if (held_rec[g - 1] != INT_MAX) before = (int)kops[held_rec[g - 1]].value;
    else if (claim_rec[g] != INT_MAX) before = (int)kops[claim_rec[g]].value;
    else if (asg[g - 1] >= 0) before = (int)kops[asg[g - 1]].value;
    const uint32_t dl = (uint32_t)(uh64[g] >> 32);
    int k = 0, lo = INT_MAX;
    for (int j = 0; j < n_u; j++) {
      const int4 e = ulist[j];
      if ((uint32_t)e.x >= dl) break;
      work++;
      if (used[e.w] || e.w <= after) continue;
      if (e.z != kFree && before != kFree && e.z != before) continue;
      if (want != kFree && e.y != want) continue;
      k++;
      lo = min(lo, e.w);
    }
    for (int x = pin_head[g]; x >= 0; x = pin_next[x]) {
      work++;
      if (used[x] || x <= after) continue;
      const lc_op &y = kops[x];
      if ((uint32_t)(y.call - base) >= dl) continue;
      if (y.f == LC_F_CAS && before != kFree && (int)y.expected != before) continue;
      if (want != kFree && (int)y.value != want) continue;
      k++;
      lo = min(lo, x);
    }
    *first = lo;
    return k;
  };
  auto token = [](int kind, int a, int b) { return (int32_t)(((uint32_t)kind << 30) | ((uint32_t)a << 15) | (uint32_t)b); };
  auto assign = [&](int g, int x, int &nlog) {  // (lane 0 writes; all lanes keep the counts)
    if (tid == 0) {
      asg[g] = x;
      used[x] = 1;
      logp[nlog] = g;
    }
    nlog++;
  };
  auto sync = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  };
  constexpr int kNodes = 2048;                       // as tests/cert_ref.py PROOF_NODES
  constexpr long long kWork = 1ll << 22;             // candidate checks per lane
  // frames of the open case splits: (position, cases << 16 | case index,
  // log length before the split's own assumption, the op assumed in the
  // current case)
  int T = 0, nlog = 0, sp = 0, nodes = 0;
  bool ok = false;
  for (;;) {
    // at the current assumptions: an open position with no candidate (the
    // lowest), else one with one (the lowest), else the fewest
    if (++nodes > kNodes) break;
    int best_e = INT_MAX, best_f = INT_MAX, best_fx = -1, best_b = INT_MAX, best_bk = INT_MAX;
    int any = 0;
    for (int i = tid; i < ng; i += kWave) {
      const int g = glist[i];
      if (asg[g] >= 0) continue;
      any = 1;
      int f;
      const int k = cands(g, -1, &f);
      if (k == 0) best_e = min(best_e, g);
      else if (k == 1 && g < best_f) best_f = g, best_fx = f;
      else if (k < best_bk || (k == best_bk && g < best_b)) best_bk = k, best_b = g;
    }
    if (__ballot(work > kWork)) break;
    if (!__ballot(any)) break;  // every open position held: no contradiction here
    const int e = wave_min_i32(best_e);
    if (e != INT_MAX) {
      // this case is closed (the checker re-derives that: no token): back to
      // the innermost split with a case left
      bool resumed = false;
      while (sp > 0) {
        const int4 fr = frames[sp - 1];
        // undo the assumptions made inside the case, then the case's own
        while (nlog > fr.z) {
          nlog--;
          if (tid == 0) {
            const int g = logp[nlog];
            used[asg[g]] = 0;
            asg[g] = -1;
          }
        }
        sync();
        const int k = fr.y >> 16, i = fr.y & 0xFFFF;
        if (i + 1 < k) {
          // the next case: the lowest candidate above the one just closed
          int x = INT_MAX;
          if (tid == 0) cands(fr.x, fr.w, &x);
          x = uni(x);
          if (x == INT_MAX) break;  // (cannot happen: the split counted its cases)
          if (tid == 0) frames[sp - 1] = make_int4(fr.x, (k << 16) | (i + 1), fr.z, x);
          assign(fr.x, x, nlog);
          sync();
          resumed = true;
          break;
        }
        sp--;  // every case of this split closed: the case around it is too
      }
      if (resumed) continue;
      ok = sp == 0;
      break;
    }
    const int f = wave_min_i32(best_f);
    if (f != INT_MAX) {
      // forced (the checker re-derives it: no token)
      const int x = uni(__shfl(best_fx, __builtin_ctzll(__ballot(best_f == f))));
      assign(f, x, nlog);
      sync();
      continue;
    }
    // a case split at the position with the fewest candidates (the lowest
    // position among equals), its first case the lowest candidate
    const int bk = wave_min_i32(best_bk);
    const int b = wave_min_i32(best_bk == bk ? best_b : INT_MAX);
    if (sp >= n_frames || bk > 0x7FFF || T >= n) break;
    int x = INT_MAX;
    if (tid == 0) cands(b, -1, &x);
    x = uni(x);
    if (tid == 0) {
      ks[T] = token(2, b, bk);
      frames[sp] = make_int4(b, bk << 16, nlog, x);
    }
    T++;
    sp++;
    assign(b, x, nlog);
    sync();
  }
  if (ok && tid == 0) cert_write(c, LC_CERT_PROOF, -1, -1, T);
}

__global__ __launch_bounds__(256) void cert_none_kernel(int32_t *__restrict__ cert, int64_t n_keys) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n_keys; k += stride)
    reinterpret_cast<int4 *>(cert)[k] = make_int4(LC_CERT_NONE, -1, -1, 0);
}

}  // namespace

hipError_t launch_cert_none(int32_t *d_cert, int64_t n_keys, hipStream_t stream) {
  if (n_keys <= 0) return hipSuccess;
  const int64_t wgs = std::min<int64_t>((n_keys + 255) / 256, 1024);
  hipLaunchKernelGGL(cert_none_kernel, dim3((unsigned)wgs), dim3(256), 0, stream, d_cert, n_keys);
  return hipGetLastError();
}

// (the stride, records + 2 per key, rounded up to a multiple of 4)
static int64_t cert_stride(int64_t n_records, int64_t n_keys) {
  return (n_records + 2 * n_keys + 2 + 3) & ~int64_t(3);
}

size_t cert_ws_bytes(int64_t n_records, int64_t n_keys) {
  return sizeof(int32_t) * (size_t)kCertSlots * (size_t)cert_stride(n_records, n_keys);
}

hipError_t launch_certificates(const lc_op *d_ops, const int64_t *d_key_off, int64_t n_keys,
                               int64_t n_records, const KParams &p, const lc_key_result *d_out,
                               int32_t *d_ws, int32_t *d_cert, int32_t *d_cset,
                               hipStream_t stream) {
  if (n_keys <= 0) return hipSuccess;
  const int64_t stride = cert_stride(n_records, n_keys);
  hipLaunchKernelGGL(cert_kernel, dim3((unsigned)n_keys), dim3(kCertThreads), 0, stream, d_ops,
                     d_key_off, p, d_out, d_ws, stride, d_cert, d_cset);
  return hipGetLastError();
}

}  // namespace lcdev
