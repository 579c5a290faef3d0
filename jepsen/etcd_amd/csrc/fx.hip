// fx.hip — frontier exchange: one oversized key's JIT frontier search over a
// whole GPU, and over several ranks by hash ownership (include/lincheck_fx.h,
// DESIGN.md §7).
//
// The search is knossos.linear's (the JIT linearization behind
// checker/linearizable, register.clj:110-111) with the exact reductions the
// other tiers use (eager read closure, deadline order, retirement), restated
// by oracle.c's check_key_jit under JITC; this file keeps its structure:
// events in history order; a call takes a window slot (the lowest free one);
// an :ok return of x expands every configuration lacking x until x is
// linearized (level-synchronous here, oracle.c:416-463), the configurations
// that linearized x become the frontier, and ops linearized in every
// configuration retire (oracle.c:479-511).  The model step is
// register.clj:60-96 in precondition form (records.h):
//     legal(ver, val) <=> (((ver ^ nv) & nvm) | ((val ^ nl) & nlm)) == 0.
//
// Device layout (per rank):
//   F, R lists      16-B configurations (mask over the 64 window slots,
//                   int32 version, int32 value id); F is the frontier, R the
//                   configurations that linearized x (the next frontier)
//   V levels        three lists of the same entries: level k of the
//                   expansion is list k % 3 (one launch reads level k and
//                   appends level k + 1)
//   R and V tables  open-addressed dedup sets.  Compact (the usual case): one
//                   64-bit word per entry, (mask, value id), claimed by one
//                   atomicCAS and reset to EMPTY per return.  Wide: a 16-B key
//                   plus an 8-B tag (epoch << 32 | fingerprint; fingerprint 0
//                   = being written), epoch bumped per return
//   candidate regions (partitioned mode) one per owner rank
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../../include/lincheck_fx.h"
#include "rccl_dl.h"

// RCCL, loaded on first use.  librccl is part of ROCm; a host without it
// keeps every single-GPU path (only lc_fx_open_devices / lc_fx_open_rccl
// need it).
const RcclApi &rccl_api() {
  static RcclApi api;
  static std::once_flag once;
  std::call_once(once, [] {
    void *h = nullptr;
    for (const char *name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
      if ((h = dlopen(name, RTLD_NOW | RTLD_GLOBAL))) break;
    if (!h) {
      api.err = std::string("cannot load librccl: ") + dlerror();
      return;
    }
    bool all = true;
    auto get = [&](auto &fp, const char *sym) {
      fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, sym));
      if (!fp) {
        all = false;
        api.err += std::string(api.err.empty() ? "librccl lacks " : ", ") + sym;
      }
    };
    get(api.GetUniqueId, "ncclGetUniqueId");
    get(api.CommInitAll, "ncclCommInitAll");
    get(api.CommInitRank, "ncclCommInitRank");
    get(api.CommDestroy, "ncclCommDestroy");
    get(api.CommAbort, "ncclCommAbort");
    get(api.GroupStart, "ncclGroupStart");
    get(api.GroupEnd, "ncclGroupEnd");
    get(api.Send, "ncclSend");
    get(api.Recv, "ncclRecv");
    get(api.AllReduce, "ncclAllReduce");
    get(api.AllToAll, "ncclAllToAll");
    get(api.GetErrorString, "ncclGetErrorString");
    api.ok = all;
  });
  return api;
}

namespace {

constexpr int kW = 64;
constexpr int32_t kFieldMax = 0x7FFFFFFE;
// Table probes per insert before the return is redone with a 4x larger table
// prefix.  Linear probing at the <= 25 % load the prefix is sized for keeps
// chains short; a prefix that turns out too small (a return much larger than
// the last) is caught after a bounded chain instead of probing a nearly full
// table for thousands of steps per insert (measured: 43 such levels were 40 %
// of the oversized key's expand time at 4,096).
constexpr int kMaxProbe = 128;
constexpr int kMaxSpin = 1 << 22;      // loop iterations per insert, busy waits included
#ifndef FX_EXPAND_WG
#define FX_EXPAND_WG 512
#endif
// expand grid (most), 4 waves per workgroup: a level reaches a quarter of
// the chip's wave slots; fewer, busier workgroups gather more successors per
// insert round and pay the window load and the flush once for more configs
// (oversized key: 2,048 -> 512 workgroups, 0.13 -> 0.095 s)
constexpr int kExpandWG = FX_EXPAND_WG;
constexpr int kFlatWG = 1024;          // thread-per-configuration kernels
// replicated returns run whole in one workgroup while the frontier, the last
// return's work and every level stay this small
constexpr int64_t kSmallF = 256;
constexpr int64_t kSmallWork = 2048;
constexpr unsigned long long kSmallLevel = 1024;

struct Cfg {
  uint64_t mask;
  uint32_t ver;
  uint32_t val;
};
static_assert(sizeof(Cfg) == 16, "16-byte configuration");

struct Slot {
  int32_t nv, nvm, nl, nlm;  // precondition
  int32_t value;             // effect of a write/CAS: the new value
  int32_t cls;               // counted class lane: kClsLane | width << 8 | field shift; else 0
  uint64_t before;           // deadline order: same-class slots to linearize first
  uint64_t zob;              // Zobrist word of the op (0 for reads); class lane: members available
};

// Counted classes: crashed writes/CAS with equal (f, value,
// expected, version) are interchangeable (their completion never arrived,
// so their version stays nil — register.clj:64,71), and deadline order
// linearizes them in call order, after every pending :ok member of the class.
// So a configuration needs only how many of a class it has linearized, not
// one window slot per crashed op: the class is a bit field of the mask (a
// count, relative to the members every configuration has linearized, which
// retire) and a lane of its own, the top lanes (kClsLane0 and up).  A key's
// crashed ops then cost log2(count) bits per class instead of one slot each,
// which lifts the 64-slot window for crash-heavy keys without versions.
constexpr int32_t kClsLane = 1 << 30;
constexpr int kMaxCls = 16;
constexpr int kClsLane0 = 64 - kMaxCls;
__host__ __device__ inline int cls_shift(int32_t c) { return c & 0xFF; }
__host__ __device__ inline int cls_width(int32_t c) { return (c >> 8) & 0xFF; }
__host__ __device__ inline uint64_t cls_get(uint64_t mask, int32_t c) {
  return (mask >> cls_shift(c)) & ((1ULL << cls_width(c)) - 1);
}

struct Win {
  uint64_t occ;    // occupied slots
  uint64_t reads;  // slots holding reads (never candidates: closed eagerly)
  uint64_t xbit;   // slot of the returning op
  uint64_t kzob;   // Zobrist words of every retired mutation, xor-ed
  // One rank: the frontier's updates since the last return, applied to each
  // configuration as the split reads it instead of by launches of their own:
  // the ops retired then (clear), then the reads called since (closure).
  uint64_t fclear, fclose;
  int32_t rank, n_ranks;
  uint64_t fsub;   // one rank: class members retired since the last return (fields to subtract)
  // ownership with counted classes (several ranks): the mask's slot bits, and
  // per class the members retired (a field counts the members linearized
  // beyond them), so the owner hashes a class by its absolute count
  uint64_t slot_bits;
  int32_t n_cls, pad_;
  uint32_t cbase[kMaxCls];
  Slot s[kW];
};

__device__ inline bool legal(const Slot &s, uint32_t ver, uint32_t val);

__device__ inline void fix_f(Cfg &c, const Win &w) {
  c.mask &= ~w.fclear;
  c.mask -= w.fsub;  // (every configuration holds at least the retired count in each field)
  for (uint64_t pr = w.fclose; pr;) {
    const int b = __builtin_ctzll(pr);
    pr &= pr - 1;
    if (legal(w.s[b], c.ver, c.val)) c.mask |= 1ULL << b;
  }
}

// The explored counter is added to by every workgroup of every level: one
// same-address atomic each serialised; 64 shards on lines of their own, in
// Ctr so that the host's copy of Ctr after a batch carries them (sync_ctr
// sums them).
constexpr int kExpShards = 64;
constexpr int kExpStride = 16;  // u64 per shard: 128 B

// The same holds for every counter a level's workgroups all touch: on a
// multi-XCD chip a device-scope atomic is executed past the XCD's L2, and
// atomics on one 128-B line queue behind one another.  So the two list
// reservations (R, the next level's V) sit on lines of their own, and the
// retirement AND is sharded like `exp` (the host ANDs the shards: sync_ctr).
constexpr int kAndShards = 16;

struct Ctr {
  unsigned long long nV;        // V entries of the levels expanded so far
  unsigned long long kcur;      // fx_small_return_kernel: the first level it left unexpanded
  unsigned long long explored;  // successors generated (cumulative)
  unsigned long long levels;    // non-empty levels (cumulative)
  unsigned long long andmask;   // AND of R's masks (host: the AND of `andm`, sync_ctr)
  unsigned long long overflow;  // a list ran out of room (the budget)
  unsigned long long nsel;      // filter output
  unsigned long long tfull;     // a table probe ran too long: redo the return with a larger table
  alignas(128) unsigned long long nR;      // R list size (reserved per workgroup)
  alignas(128) unsigned long long cnt[3];  // V levels, triple-buffered: level k is list k % 3
  alignas(128) unsigned long long cand[64];  // partitioned: candidates per owner rank
  unsigned long long cmin[kMaxCls];  // counted classes: the smallest field over R (retirement)
  alignas(128) unsigned long long andm[kAndShards * kExpStride];  // AND of R's masks, sharded
  alignas(128) unsigned long long exp[kExpShards * kExpStride];  // explored, sharded
};

// What the host reads of Ctr after a batch (sync_ctr): the counters, the
// shards already summed / ANDed, written by fx_report_kernel into host-mapped
// memory with `seq` last, so that the host spins on one word instead of a
// device-to-host copy and a stream synchronisation (≈3 µs of copy on the
// device plus the host's wake-up, per batch).
struct Rep {
  unsigned long long nV, kcur, explored, levels, andmask, overflow, nsel, tfull, nR;
  unsigned long long cnt[3];
  unsigned long long cand[64];
  unsigned long long cmin[kMaxCls];
  alignas(64) unsigned int seq;
};

// One wave: lane i sums explored shard i (64 of them), ANDs AND shard i (16),
// copies owner count i and class minimum i; lane 0 the scalars; then a
// system-scope release and `seq`.
__global__ __launch_bounds__(64) void fx_report_kernel(const Ctr *__restrict__ c, Rep *r, unsigned int seq);

__device__ inline void and_into(Ctr *ctr, unsigned long long a) {
  atomicAnd(&ctr->andm[(blockIdx.x % kAndShards) * kExpStride], a);
}

__host__ __device__ inline uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

__device__ inline uint64_t cfg_hash(const Cfg &c) {
  return mix64(c.mask ^ mix64(((uint64_t)c.ver << 32) | c.val));
}

__device__ inline bool legal(const Slot &s, uint32_t ver, uint32_t val) {
  return ((((int32_t)ver ^ s.nv) & s.nvm) | (((int32_t)val ^ s.nl) & s.nlm)) == 0;
}

// Owner rank: a Zobrist hash over the mutations the configuration has
// linearized, retired ones included (kzob), and its state.  Retirement clears
// a bit in every configuration and folds the op's word into kzob, so owners
// never move; reads carry no word, so read closure never moves them either.
// A counted class enters by its absolute member count (retired members plus
// its field): retirement shrinks the field and grows cbase together, so it
// moves no owner either.
__device__ inline uint32_t owner_of(const Cfg &c, const Win &w) {
  uint64_t z = w.kzob, m = c.mask & w.slot_bits;
  while (m) {
    const int b = __builtin_ctzll(m);
    m &= m - 1;
    z ^= w.s[b].zob;
  }
  for (int k = 0; k < w.n_cls; k++) {
    const uint64_t cnt = cls_get(c.mask, w.s[kClsLane0 + k].cls) + w.cbase[k];
    if (cnt) z ^= mix64(((uint64_t)(k + 1) << 56) ^ cnt);
  }
  z ^= mix64(((uint64_t)c.ver << 32) | c.val);
  return (uint32_t)(mix64(z) % (uint64_t)w.n_ranks);
}

// Insert into an open-addressed table.  1: new, 0: present, -1: no room.
// The winner of a stale tag writes the key and publishes the tag inside the
// loop body (not after a divergent loop exit), so a lane of the same wave
// spinning on the busy tag sees it on its next iteration.
__device__ int tab_insert(unsigned long long *tags, Cfg *keys, uint64_t tmask, uint32_t epoch,
                          const Cfg &c) {
  const uint64_t h = cfg_hash(c);
  const uint32_t fp = (uint32_t)(h >> 32) | 1u;
  const unsigned long long busy = (unsigned long long)epoch << 32;
  const unsigned long long pub = busy | fp;
  uint64_t i = h & tmask;
  int res = -1, probes = 0;
  bool done = false;
  for (int it = 0; !done && it < kMaxSpin; it++) {
    unsigned long long t = __hip_atomic_load(&tags[i], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    if ((uint32_t)(t >> 32) != epoch) {
      unsigned long long expct = t;
      if (__hip_atomic_compare_exchange_strong(&tags[i], &expct, busy, __ATOMIC_ACQ_REL,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        keys[i] = c;
        __hip_atomic_store(&tags[i], pub, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        res = 1;
        done = true;
      }
    } else if ((uint32_t)t == fp) {
      const Cfg k = keys[i];
      if (k.mask == c.mask && k.ver == c.ver && k.val == c.val) {
        res = 0;
        done = true;
      } else {
        i = (i + 1) & tmask;
        done = ++probes >= kMaxProbe;
      }
    } else if ((uint32_t)t != 0) {
      i = (i + 1) & tmask;
      done = ++probes >= kMaxProbe;
    }
    // (uint32_t)t == 0: being written by another lane; read it again
  }
  return res;
}

struct Tabs {
  unsigned long long *tagR, *tagV;
  Cfg *keyR, *keyV;
  Cfg *listR;
  // V levels: three lists of list_cap entries at vbase; a launch reads its
  // level from vsrc and appends the next one to vdst, counted in *vcnt
  Cfg *vbase, *vsrc, *vdst;
  unsigned long long *vcnt;
  uint64_t tmask;
  unsigned long long list_cap;
  int compact;  // one-word keys (ctab_insert) instead of tag + 16-B key
  int cshift;   // compact: the value id's bit offset in the word (64 - value bits)
  unsigned long long *exp;  // Ctr::exp
};

__device__ inline unsigned long long wave_sum_shards(unsigned long long *exp) {
  unsigned long long v =
      __hip_atomic_load(&exp[__lane_id() * kExpStride], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t lo = __shfl_xor((uint32_t)v, off), hi = __shfl_xor((uint32_t)(v >> 32), off);
    v += ((unsigned long long)hi << 32) | lo;
  }
  return v;
}

// Compact tables.  Within one return every configuration has linearized the
// retired mutations plus those its mask names, so its version is
// V0 + (retired mutations) + popcount(mask & mutation slots): a function of
// the mask.  The state reduces to the value, which the host interns per key
// to a dense id.  With v bits for the value ids (6 to 20, as the key needs:
// the all-ones id is never used) and every occupied slot below 64 - v,
// (mask, value id) packs into one 64-bit word (Tabs::cshift = 64 - v), and
// a table entry is that word: insertion is one device-scope atomicCAS per
// probe (EMPTY -> word; the value returned says new, present, or occupied by
// another word), with no key payload, tag or fence.  Tables are reset to
// EMPTY (all ones) before each return.
constexpr unsigned long long kEmpty = ~0ULL;

__device__ inline int ctab_insert(unsigned long long *tab, uint64_t tmask, const Cfg &c, int cshift,
                                  uint64_t start = ~0ULL) {
  const unsigned long long word = c.mask | ((unsigned long long)c.val << cshift);
  uint64_t i = (start == ~0ULL ? mix64(word) : start) & tmask;
  for (int probes = 0; probes < kMaxProbe; probes++) {
    const unsigned long long old = atomicCAS(&tab[i], kEmpty, word);
    if (old == kEmpty) return 1;
    if (old == word) return 0;
    i = (i + 1) & tmask;
  }
  return -1;
}

__device__ inline int any_insert(const Tabs &t, bool toR, uint32_t epoch, const Cfg &c) {
  if (t.compact) return ctab_insert(toR ? t.tagR : t.tagV, t.tmask, c, t.cshift);
  return tab_insert(toR ? t.tagR : t.tagV, toR ? t.keyR : t.keyV, t.tmask, epoch, c);
}

__device__ inline unsigned long long wave_and(unsigned long long v) {
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t lo = __shfl_xor((uint32_t)v, off), hi = __shfl_xor((uint32_t)(v >> 32), off);
    v &= ((unsigned long long)hi << 32) | lo;
  }
  return v;
}

__device__ inline unsigned long long wave_sum(unsigned long long v) {
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t lo = __shfl_xor((uint32_t)v, off), hi = __shfl_xor((uint32_t)(v >> 32), off);
    v += ((unsigned long long)hi << 32) | lo;
  }
  return v;
}

static_assert(kExpShards == 64 && kAndShards <= 64 && kMaxCls <= 64, "one lane per shard");

__global__ __launch_bounds__(64) void fx_report_kernel(const Ctr *__restrict__ c, Rep *r, unsigned int seq) {
  const int i = threadIdx.x;
  const unsigned long long e = wave_sum(c->exp[i * kExpStride]);
  const unsigned long long q = wave_sum(c->exp[i * kExpStride + 1]);
  const unsigned long long a = wave_and(i < kAndShards ? c->andm[i * kExpStride] : ~0ULL);
  r->cand[i] = c->cand[i];
  if (i < kMaxCls) r->cmin[i] = c->cmin[i];
  if (i < 3) r->cnt[i] = c->cnt[i];
  if (i == 0) {
    r->nV = c->nV + q;
    r->kcur = c->kcur;
    r->explored = e;
    r->levels = c->levels;
    r->andmask = a;
    r->overflow = c->overflow;
    r->nsel = c->nsel;
    r->tfull = c->tfull;
    r->nR = c->nR;
  }
  __syncthreads();
  if (i == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __hip_atomic_store(&r->seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Wave-aggregated append of the lanes in `take` (each with its own c).
__device__ inline void wave_append(bool take, const Cfg &c, Cfg *list, unsigned long long *count,
                                   unsigned long long cap, unsigned long long *overflow) {
  const uint64_t m = __ballot(take);
  if (!m) return;
  const int lane = __lane_id();
  const int leader = __builtin_ctzll(m);
  unsigned long long base = 0;
  if (lane == leader) base = atomicAdd(count, (unsigned long long)__popcll(m));
  base = __shfl(base, leader);
  if (take) {
    const unsigned long long pos = base + __popcll(m & ((1ULL << lane) - 1));
    if (pos < cap) list[pos] = c;
    else atomicOr(overflow, 1ULL);
  }
}

// Insert successors (or split frontier configurations): those that
// linearized x (xbit) go to R with x's bit cleared, the others to V.  `rand`
// (per lane) takes the AND of the masks this lane appended to R.
__device__ inline void insert_rv(bool have, Cfg c, uint64_t xbit, const Tabs &t, uint32_t epoch,
                                 Ctr *ctr, uint64_t &rand) {
  bool toR = have && (c.mask & xbit);
  if (toR) c.mask &= ~xbit;
  int r = -1;
  if (have) r = any_insert(t, toR, epoch, c);
  if (have && r < 0) atomicOr(&ctr->tfull, 1ULL);
  if (r == 1 && toR) rand &= c.mask;
  wave_append(r == 1 && toR, c, t.listR, &ctr->nR, t.list_cap, &ctr->overflow);
  wave_append(r == 1 && !toR, c, t.vdst, t.vcnt, t.list_cap, &ctr->overflow);
}

// Counters of a return about to start: R and V empty, explored at `explored`
// (the shards), levels from 0.
__device__ inline void ctr_start(Ctr *ctr, unsigned long long explored) {
  for (int i = 0; i < kExpShards; i++) {
    ctr->exp[i * kExpStride] = i ? 0 : explored;
    ctr->exp[i * kExpStride + 1] = 0;  // second-hop configurations (nV's part kept here)
  }
  ctr->nR = ctr->nV = ctr->kcur = 0;
  ctr->cnt[0] = ctr->cnt[1] = ctr->cnt[2] = 0;
  ctr->levels = 0;
  for (int i = 0; i < kAndShards; i++) ctr->andm[i * kExpStride] = ~0ULL;
  ctr->nsel = 0;
  ctr->tfull = 0;
  ctr->explored = explored;
  for (int i = 0; i < 64; i++) ctr->cand[i] = 0;
  for (int i = 0; i < kMaxCls; i++) ctr->cmin[i] = ~0ULL;
}

// Split F into R and V: the configurations that linearized the returning op
// to R (its bit cleared), the others to V level 0.
__device__ inline void split_into_rv(const Cfg *__restrict__ in, int64_t n, const Win &win, Tabs t,
                                     uint32_t epoch, Ctr *ctr) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const uint64_t xbit = win.xbit;
  const bool fix = win.fclear | win.fclose | win.fsub;
  uint64_t rand = ~0ULL;
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x; b < n; b += stride) {
    const int64_t i = b + threadIdx.x;
    const bool have = i < n;
    Cfg c{};
    if (have) c = in[i];
    if (have && fix) fix_f(c, win);
    insert_rv(have, c, xbit, t, epoch, ctr, rand);
  }
  // the R entries' AND, one atomic per workgroup (ctr->andmask holds the
  // AND of R as it grows: the replicated levels add theirs in wg_flush)
  __shared__ unsigned long long s_and[4];
  rand = wave_and(rand);
  if (__lane_id() == 0) s_and[threadIdx.x / kW] = rand;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long a = s_and[0] & s_and[1] & s_and[2] & s_and[3];
    if (a != ~0ULL) and_into(ctr, a);
  }
}

__global__ __launch_bounds__(256) void fx_insert_kernel(const Cfg *__restrict__ in, int64_t n,
                                                        const Win *__restrict__ win, Tabs t,
                                                        uint32_t epoch, Ctr *ctr) {
  split_into_rv(in, n, *win, t, epoch, ctr);
}

// One rank's split at the start of a return by the grid: the window travels
// as the argument (with `dwin` the first workgroup stores it for the levels
// that follow), and the launch also prepares the NEXT return — the other
// parity's counters, its one-word tables (`prep_words` entries) to EMPTY —
// so that return needs no reset launch of its own (fx_reset_kernel: ≈4 µs of
// each return on the oversized key).
__global__ __launch_bounds__(256) void fx_split_kernel(const Cfg *__restrict__ in, int64_t n,
                                                       const Win win, Win *dwin, Tabs t,
                                                       uint32_t epoch, Ctr *ctr, Ctr *prep_ctr,
                                                       unsigned long long *prep_tR,
                                                       unsigned long long *prep_tV,
                                                       int64_t prep_words) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if (dwin && blockIdx.x == 0) {
    const uint32_t *src = reinterpret_cast<const uint32_t *>(&win);
    uint32_t *dst = reinterpret_cast<uint32_t *>(dwin);
    for (int i = threadIdx.x; i < (int)(sizeof(Win) / 4); i += blockDim.x) dst[i] = src[i];
  }
  if (prep_ctr) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < prep_words; i += stride) {
      prep_tR[i] = kEmpty;
      prep_tV[i] = kEmpty;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) ctr_start(prep_ctr, 0);
  }
  split_into_rv(in, n, win, t, epoch, ctr);
}


// One level of the expansion: every wave takes configurations of V[lo, hi)
// one at a time, lane t tests window slot t (pending, not a read, its
// deadline-order predecessors linearized, legal), builds the successor with
// its eager read closure, and either inserts it (replicated mode) or appends
// it to its owner's candidate region (partitioned mode: cand_cap != 0).
// Per-wave LDS staging of new list entries (replicated mode): one atomic per
// flush of up to kStage entries instead of one per configuration expanded —
// the list counters are the only same-address atomics of a level.
constexpr int kStage = 128;
constexpr int kHop2 = 64;  // most successors a wave expands itself in a level launch
struct Stage {
  Cfg r[kStage];
  Cfg v[kStage];
  Cfg s[64];  // successors gathered from several configurations, inserted together
  Cfg q[2][kHop2];  // new successors this wave expands in the same launch (later hops)
};

__device__ inline void stage_flush(Cfg *buf, int &n, Cfg *list, unsigned long long *count,
                                   unsigned long long cap, unsigned long long *overflow) {
  if (!n) return;
  __builtin_amdgcn_wave_barrier();
  const int lane = __lane_id();
  unsigned long long base = 0;
  if (lane == 0) base = atomicAdd(count, (unsigned long long)n);
  base = __shfl(base, 0);
  for (int j = lane; j < n; j += kW) {
    if (base + j < cap) list[base + j] = buf[j];
    else atomicOr(overflow, 1ULL);
  }
  __builtin_amdgcn_wave_barrier();
  n = 0;
}

__device__ inline void stage_put(bool isnew, bool toR, const Cfg &c, Stage *stg, int &nr, int &nv,
                                 const Tabs &t, Ctr *ctr) {
  const uint64_t below = (1ULL << __lane_id()) - 1;
  const uint64_t mR = __ballot(isnew && toR), mV = __ballot(isnew && !toR);
  if (isnew && toR) stg->r[nr + __popcll(mR & below)] = c;
  if (isnew && !toR) stg->v[nv + __popcll(mV & below)] = c;
  nr += __popcll(mR);
  nv += __popcll(mV);
  if (nr > kStage - kW) stage_flush(stg->r, nr, t.listR, &ctr->nR, t.list_cap, &ctr->overflow);
  if (nv > kStage - kW) stage_flush(stg->v, nv, t.vdst, t.vcnt, t.list_cap, &ctr->overflow);
}

// End of a level: the workgroup's waves reserve their staged entries with one
// atomic per list for the whole workgroup (the list counters and the
// explored shards are the level's only same-address atomics), then each wave
// writes its own.  Every wave of the workgroup must call it.
struct WgFlush {
  int n[4][2];
  int nq[4];
  unsigned long long base[2];
  unsigned long long explored[4];
  unsigned long long andm[4];
};

__device__ inline void wg_flush(WgFlush *wf, Stage *stg, int nr, int nv, int nq,
                                unsigned long long explored, uint64_t rand, const Tabs &t, Ctr *ctr) {
  const int w = threadIdx.x / kW, lane = __lane_id();
  rand = wave_and(rand);
  if (lane == 0) {
    wf->n[w][0] = nr;
    wf->n[w][1] = nv;
    wf->nq[w] = nq;
    wf->explored[w] = explored;
    wf->andm[w] = rand;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = blockDim.x / kW;
    unsigned long long tr = 0, tv = 0, te = 0, ta = ~0ULL, tq = 0;
    for (int k = 0; k < nw; k++) {
      tr += wf->n[k][0];
      tv += wf->n[k][1];
      tq += wf->nq[k];
      te += wf->explored[k];
      ta &= wf->andm[k];
    }
    if (ta != ~0ULL) and_into(ctr, ta);
    wf->base[0] = tr ? atomicAdd(&ctr->nR, tr) : 0;
    wf->base[1] = tv ? atomicAdd(t.vcnt, tv) : 0;
    if (te) atomicAdd(&t.exp[(blockIdx.x % kExpShards) * kExpStride], te);
    if (tq) atomicAdd(&t.exp[(blockIdx.x % kExpShards) * kExpStride + 1], tq);
  }
  __syncthreads();
  unsigned long long br = wf->base[0], bv = wf->base[1];
  for (int k = 0; k < w; k++) {
    br += wf->n[k][0];
    bv += wf->n[k][1];
  }
  for (int j = lane; j < nr; j += kW) {
    if (br + j < t.list_cap) t.listR[br + j] = stg->r[j];
    else atomicOr(&ctr->overflow, 1ULL);
  }
  for (int j = lane; j < nv; j += kW) {
    if (bv + j < t.list_cap) t.vdst[bv + j] = stg->v[j];
    else atomicOr(&ctr->overflow, 1ULL);
  }
}

// One level of the expansion: every wave takes configurations of V[lo, hi)
// (two at a time in replicated mode, their table probes in flight
// together), lane t tests window slot t (pending, not a read, its
// deadline-order predecessors linearized, legal), builds the successor with
// its eager read closure, and either inserts it (replicated mode) or appends
// it to its owner's candidate region (partitioned mode: cand_cap != 0).
// Read closure: the reads a successor's state makes legal are, for reads
// without a version, fixed by the value this lane's op writes (rv_me, once
// per launch); only reads that name a version are tested per successor.
// Later hops (replicated mode, `hops` > 0): up to `hop2` of the new
// successors a wave finds that stay in V are expanded by that wave in the
// same launch instead of going to the next level's list, and up to `hop2` of
// theirs, `hops` times, so a launch covers up to 1 + `hops` levels of the
// search.  A configuration is still expanded exactly
// once (the one whose insert found it new does it, whenever), so the
// configurations explored and the frontiers are those of one level per
// launch; the levels' lists are then work queues whose entries may differ in
// depth.
__device__ inline void expand_range(const Win &w, const Tabs &t, uint32_t epoch, Ctr *ctr,
                                    int64_t lo, int64_t hi, int64_t wave, int64_t nwaves,
                                    Cfg *cbuf, unsigned long long cand_cap, Stage *stg,
                                    WgFlush *wf, int hop2 = 0, int hops = 0, bool from_f = false) {
  const int lane = __lane_id();
  int nr = 0, nv = 0;  // staged entries (wave-uniform)
  int nq = 0;          // configurations kept for the next hop, in stg->q[qb] (wave-uniform)
  int qb = 0;
  int nkept = 0;       // configurations the later hops expanded
  const Slot me = w.s[lane];
  const uint64_t bit = 1ULL << lane;
  const uint64_t muts = w.occ & ~w.reads;
  const uint64_t reads = w.occ & w.reads;
  const bool is_mut = (muts & bit) != 0;
  uint64_t rv_me = 0, vreads = 0;
  for (uint64_t pr = reads; pr;) {
    const int b = __builtin_ctzll(pr);
    pr &= pr - 1;
    const Slot &r = w.s[b];
    if (r.nvm) vreads |= 1ULL << b;
    else if (!r.nlm || r.nl == me.value) rv_me |= 1ULL << b;
  }
  const bool is_cls = me.cls != 0;
  auto succ = [&](const Cfg &c, bool &cand, Cfg &s) {
    // a slot's op not yet linearized; or a class with a member left
    const bool avail = is_cls ? cls_get(c.mask, me.cls) < me.zob : is_mut && !(c.mask & bit);
    cand = avail && !(me.before & ~c.mask) && legal(me, c.ver, c.val);
    s = c;
    if (cand) {
      s.mask = (is_cls ? s.mask + (1ULL << cls_shift(me.cls)) : s.mask | bit) | rv_me;
      s.ver = c.ver + 1;
      s.val = (uint32_t)me.value;
      uint64_t pr = vreads & ~s.mask;
      while (pr) {
        const int b = __builtin_ctzll(pr);
        pr &= pr - 1;
        if (legal(w.s[b], s.ver, s.val)) s.mask |= 1ULL << b;
      }
    }
  };
  unsigned long long explored = 0;
  uint64_t rand = ~0ULL;  // AND of the masks this lane put in R
  if (!cand_cap) {
    // A wave takes a run of `chunk` configurations (one load per lane), lane t
    // tests slot t of each in turn, and the successors are gathered in LDS
    // until 64 are pending; then every lane inserts one, so a probe round trip
    // serves up to 64 successors of several configurations.  The run length
    // spreads the level over every wave first (chunk = 1 on small levels).
    const uint64_t below = (1ULL << lane) - 1;
    const int64_t n = hi - lo;
    const int64_t chunk = std::min<int64_t>(kW, std::max<int64_t>(1, (n + nwaves - 1) / nwaves));
    int ns = 0;
    int room = hops ? hop2 : 0;  // places left for the next hop
    auto insert_stash = [&]() {
      __builtin_amdgcn_wave_barrier();
      const bool have = lane < ns;
      Cfg sc{};
      if (have) sc = stg->s[lane];
      __builtin_amdgcn_wave_barrier();
      const bool toR = have && (sc.mask & w.xbit);
      if (toR) sc.mask &= ~w.xbit;
      int x = -2;
      if (have) x = any_insert(t, toR, epoch, sc);
      if (x == -1) atomicOr(&ctr->tfull, 1ULL);
      if (x == 1 && toR) rand &= sc.mask;
      bool keep = false;
      if (room) {
        const uint64_t mk = __ballot(x == 1 && !toR);
        const int r = __popcll(mk & below);
        keep = x == 1 && !toR && r < room;
        if (keep) stg->q[qb][nq + r] = sc;
        const int took = min(__popcll(mk), room);
        nq += took;
        room -= took;
      }
      stage_put(x == 1 && !keep, toR, sc, stg, nr, nv, t, ctr);
      ns = 0;
    };
    auto expand_one = [&](const Cfg &c) {
      bool cand;
      Cfg sc;
      succ(c, cand, sc);
      const uint64_t m = __ballot(cand);
      const int k = __popcll(m);
      explored += k;
      if (ns + k > kW) insert_stash();
      if (cand) stg->s[ns + __popcll(m & below)] = sc;
      ns += k;
    };
    for (int64_t base = lo + wave * chunk; base < hi; base += nwaves * chunk) {
      const int cnt = (int)std::min<int64_t>(chunk, hi - base);
      Cfg mine{};
      if (lane < cnt) mine = t.vsrc[base + lane];
      if (from_f) {
        // the frontier itself (fx_split_expand_kernel): each configuration,
        // with the updates since the last return, is inserted as a successor
        // would be — to R if it linearized the returning op, else to V, where
        // a new one is kept and expanded below like any kept successor
        if (lane < cnt) {
          fix_f(mine, w);
          stg->s[lane] = mine;
        }
        ns = cnt;
        insert_stash();
        continue;
      }
      for (int j = 0; j < cnt; j++) {
        Cfg c;
        c.mask = ((uint64_t)__shfl((uint32_t)(mine.mask >> 32), j) << 32) |
                 __shfl((uint32_t)mine.mask, j);
        c.ver = __shfl(mine.ver, j);
        c.val = __shfl(mine.val, j);
        expand_one(c);
      }
    }
    if (ns) insert_stash();
    for (int h = 1; h <= hops && nq; h++) {
      // hop h + 1: the kept configurations (their new successors kept again
      // while hops are left, else to the lists)
      const int n = nq, cur = qb;
      nkept += n;
      qb ^= 1;
      nq = 0;
      room = h < hops ? hop2 : 0;
      __builtin_amdgcn_wave_barrier();
      for (int j = 0; j < n; j++) {
        const Cfg c = stg->q[cur][j];
        expand_one(c);
      }
      if (ns) insert_stash();
    }
  } else {
    for (int64_t i = lo + wave; i < hi; i += nwaves) {
      const Cfg c = t.vsrc[i];
      bool cand;
      Cfg s;
      succ(c, cand, s);
      explored += __popcll(__ballot(cand));
      // append to the owner's region; one atomic per distinct owner in the wave
      const uint32_t own = cand ? owner_of(s, w) : 0xFFFFFFFFu;
      uint64_t pend = __ballot(cand);
      while (pend) {
        const uint32_t o = __shfl(own, __builtin_ctzll(pend));
        const bool mine = cand && own == o;
        const uint64_t m = __ballot(mine);
        pend &= ~m;
        wave_append(mine, s, cbuf + (size_t)o * cand_cap, &ctr->cand[o], cand_cap, &ctr->overflow);
      }
    }
  }
  wg_flush(wf, stg, nr, nv, nkept, explored, rand, t, ctr);
}

__device__ inline void load_win(Win &w, const Win *gwin) {
  const uint32_t *src = reinterpret_cast<const uint32_t *>(gwin);
  uint32_t *dst = reinterpret_cast<uint32_t *>(&w);
  for (int i = threadIdx.x; i < (int)(sizeof(Win) / 4); i += blockDim.x) dst[i] = src[i];
}

// A level over the grid: level k whole (lo_arg < 0: replicated mode; its
// size is ctr->cnt[k % 3], fixed while it runs, since this launch appends to
// level k + 1 and only zeroes the count of level k + 2, whose list level k - 1
// held) or [lo_arg, hi_arg) of it (partitioned mode: the host keeps the
// books).  No level-marking launch sits between two levels.  Workgroups past
// the level's end leave before staging the window, so the speculative
// launches of the replicated mode cost little when empty.
__global__ __launch_bounds__(256) void fx_expand_kernel(const Win *__restrict__ gwin, Tabs t,
                                                        uint32_t epoch, Ctr *ctr, int64_t k,
                                                        int64_t lo_arg, int64_t hi_arg, Cfg *cbuf,
                                                        unsigned long long cand_cap, int hop2,
                                                        int hops) {
  // The prologue's loads go out together — the level's size, the table-full
  // flag and this thread's words of the window — one round trip to memory
  // before the first configuration instead of three in a row (a level's
  // launch is a chain of dependent round trips: DESIGN.md §7).
  constexpr int kWinWords = (int)(sizeof(Win) / 4);
  constexpr int kWinPer = (kWinWords + 255) / 256;
  uint32_t wv[kWinPer];
  const uint32_t *wsrc = reinterpret_cast<const uint32_t *>(gwin);
#pragma unroll
  for (int j = 0; j < kWinPer; j++) {
    const int i = (int)threadIdx.x + j * 256;
    wv[j] = i < kWinWords ? wsrc[i] : 0u;
  }
  const int64_t cnt = lo_arg < 0 ? (int64_t)ctr->cnt[k % 3] : 0;
  const unsigned long long tfull = ctr->tfull;
  int64_t lo, hi;
  if (lo_arg < 0) {
    lo = 0;
    hi = cnt;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      ctr->cnt[(k + 2) % 3] = 0;
      if (hi) {
        ctr->levels++;
        ctr->nV += (unsigned long long)hi;
      }
    }
  } else {
    lo = lo_arg;
    hi = hi_arg;
  }
  if (lo + (int64_t)blockIdx.x * (blockDim.x / kW) >= hi) return;
  if (tfull) return;  // this attempt will be redone with a larger table
  __shared__ Win w;
  __shared__ Stage stg[4];
  __shared__ WgFlush wf;
  {
    uint32_t *dst = reinterpret_cast<uint32_t *>(&w);
#pragma unroll
    for (int j = 0; j < kWinPer; j++) {
      const int i = (int)threadIdx.x + j * 256;
      if (i < kWinWords) dst[i] = wv[j];
    }
  }
  __syncthreads();
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kW;
  const int64_t nwaves = (int64_t)gridDim.x * blockDim.x / kW;
  expand_range(w, t, epoch, ctr, lo, hi, wave, nwaves, cbuf, cand_cap, &stg[threadIdx.x / kW], &wf,
               hop2, hops);
}


// A return's split and its first levels in one launch (one rank): the
// frontier F, with the updates since the last return applied, goes to R (it
// linearized the returning op) or V (dedup tables as the split's); a new V
// configuration is kept and expanded in the same launch up to `hops` levels
// deep (expand_range's later hops), and what does not fit goes to V level 0,
// which the batch's level launches take on.  Like fx_split_kernel it stores
// the window for the level launches (dwin) and prepares the next return's
// counters and tables (prep_*): one launch instead of the split and the
// return's first level launch, and no list round trip for the configurations
// it expands itself.
__global__ __launch_bounds__(256) void fx_split_expand_kernel(const Cfg *__restrict__ F, int64_t nF,
                                                              const Win win, Win *dwin, Tabs t,
                                                              uint32_t epoch, Ctr *ctr, Ctr *prep_ctr,
                                                              unsigned long long *prep_tR,
                                                              unsigned long long *prep_tV,
                                                              int64_t prep_words, int hop2, int hops) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if (dwin && blockIdx.x == 0) {
    const uint32_t *src = reinterpret_cast<const uint32_t *>(&win);
    uint32_t *dst = reinterpret_cast<uint32_t *>(dwin);
    for (int i = threadIdx.x; i < (int)(sizeof(Win) / 4); i += blockDim.x) dst[i] = src[i];
  }
  if (prep_ctr) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < prep_words; i += stride) {
      prep_tR[i] = kEmpty;
      prep_tV[i] = kEmpty;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) ctr_start(prep_ctr, 0);
  }
  if ((int64_t)blockIdx.x * (blockDim.x / kW) >= nF) return;  // (workgroup-uniform)
  __shared__ Win w;
  __shared__ Stage stg[4];
  __shared__ WgFlush wf;
  {
    const uint32_t *src = reinterpret_cast<const uint32_t *>(&win);
    uint32_t *dst = reinterpret_cast<uint32_t *>(&w);
    for (int i = threadIdx.x; i < (int)(sizeof(Win) / 4); i += blockDim.x) dst[i] = src[i];
  }
  __syncthreads();
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kW;
  const int64_t nwaves = (int64_t)gridDim.x * blockDim.x / kW;
  Tabs tf = t;
  tf.vsrc = const_cast<Cfg *>(F);
  expand_range(w, tf, epoch, ctr, 0, nF, wave, nwaves, nullptr, 0, &stg[threadIdx.x / kW], &wf, hop2,
               hops, true);
}

// Counted classes: the smallest field of each class over list[lo, hi) (this
// thread strided by `step`), into ctr->cmin (retirement of the members every
// configuration has linearized).  Only when the window has class lanes.
__device__ inline void cls_min_over(const Win &w, const Cfg *list, int64_t lo, int64_t hi,
                                    int64_t step, Ctr *ctr) {
  for (int k = 0; k < kMaxCls; k++) {
    const int32_t cl = w.s[kClsLane0 + k].cls;
    if (!cl) continue;
    uint32_t m = 0xFFFFFFFFu;
    for (int64_t i = lo; i < hi; i += step) m = min(m, (uint32_t)cls_get(list[i].mask, cl));
    for (int off = 32; off > 0; off >>= 1) m = min(m, (uint32_t)__shfl_xor((int)m, off));
    if (__lane_id() == 0 && m != 0xFFFFFFFFu) atomicMin(&ctr->cmin[k], (unsigned long long)m);
  }
}

__global__ __launch_bounds__(256) void fx_cmin_kernel(const Cfg *__restrict__ list,
                                                      const unsigned long long *n,
                                                      const Win *__restrict__ gwin, Ctr *ctr) {
  __shared__ Win w;
  load_win(w, gwin);
  __syncthreads();
  cls_min_over(w, list, (int64_t)blockIdx.x * blockDim.x + threadIdx.x, (int64_t)*n,
               (int64_t)gridDim.x * blockDim.x, ctr);
}

// A whole return in one workgroup while the frontier is small (replicated
// mode): split F, then levels separated by barriers, then the AND for
// retirement — one launch instead of one per level.  A level larger than
// `cutoff` is left to the grid: ctr->kcur names it, with the same books the
// grid's launches keep.
__global__ __launch_bounds__(256) void fx_small_return_kernel(const Cfg *__restrict__ F, int64_t nF,
                                                              const Win *__restrict__ gwin, Tabs t,
                                                              uint32_t epoch, Ctr *ctr,
                                                              unsigned long long cutoff) {
  __shared__ Win w;
  __shared__ Stage stg[4];
  __shared__ WgFlush wf;
  __shared__ long long s_n;
  load_win(w, gwin);
  __syncthreads();
  for (int64_t b = 0; b < nF; b += blockDim.x) {
    const int64_t i = b + threadIdx.x;
    const bool have = i < nF;
    Cfg c{};
    if (have) c = F[i];
    uint64_t rand = ~0ULL;  // the full AND over R below covers these
    if (have) fix_f(c, w);
    insert_rv(have, c, w.xbit, t, epoch, ctr, rand);
  }
  const int64_t wave = threadIdx.x / kW;
  const int64_t nwaves = blockDim.x / kW;
  for (int64_t k = 0;; k++) {
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned long long n =
          __hip_atomic_load(&ctr->cnt[k % 3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const bool full =
          __hip_atomic_load(&ctr->tfull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
      if (n && n <= cutoff && !full) {
        ctr->cnt[(k + 2) % 3] = 0;
        ctr->levels++;
        ctr->nV += n;
        s_n = (long long)n;
      } else {
        ctr->kcur = (unsigned long long)k;
        s_n = 0;
      }
    }
    __syncthreads();
    if (!s_n) break;
    Tabs tk = t;
    tk.vsrc = t.vbase + (size_t)(k % 3) * t.list_cap;
    tk.vdst = t.vbase + (size_t)((k + 1) % 3) * t.list_cap;
    tk.vcnt = &ctr->cnt[(k + 1) % 3];
    expand_range(w, tk, epoch, ctr, 0, s_n, wave, nwaves, nullptr, 0, &stg[threadIdx.x / kW], &wf);
  }
  // retirement AND over R (meaningful when the return finished here)
  const int64_t nR =
      (int64_t)__hip_atomic_load(&ctr->nR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned long long a = ~0ULL;
  for (int64_t i = threadIdx.x; i < nR; i += blockDim.x) a &= t.listR[i].mask;
  a = wave_and(a);
  if (__lane_id() == 0 && a != ~0ULL) and_into(ctr, a);
  cls_min_over(w, t.listR, threadIdx.x, nR, blockDim.x, ctr);
  __syncthreads();
  if (threadIdx.x < kW) {
    const unsigned long long e = wave_sum_shards(t.exp);
    if (threadIdx.x == 0) ctr->explored = e;
  }
}


// AND of the masks of list[0 .. *n) into ctr->andmask (retirement).
__global__ __launch_bounds__(256) void fx_and_kernel(const Cfg *__restrict__ list,
                                                     const unsigned long long *n, Ctr *ctr,
                                                     unsigned long long *exp) {
  if (blockIdx.x == 0 && threadIdx.x < kW) {
    const unsigned long long e = wave_sum_shards(exp);
    if (threadIdx.x == 0) ctr->explored = e;
  }
  const int64_t cnt = (int64_t)*n;
  unsigned long long a = ~0ULL;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cnt;
       i += (int64_t)gridDim.x * blockDim.x)
    a &= list[i].mask;
  a = wave_and(a);
  if (__lane_id() == 0 && a != ~0ULL) and_into(ctr, a);
}

__global__ __launch_bounds__(256) void fx_clear_kernel(Cfg *list, int64_t n, uint64_t bits) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    list[i].mask &= ~bits;
}

// Several ranks: retired class members leave every configuration's field at
// once (fields are disjoint and each holds at least the retired count, so one
// subtraction of the packed word borrows across no field).
__global__ __launch_bounds__(256) void fx_sub_kernel(Cfg *list, int64_t n, uint64_t sub) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    list[i].mask -= sub;
}

// A read is called: linearize it at once wherever it is legal (closure).
__global__ __launch_bounds__(256) void fx_close_read_kernel(Cfg *list, int64_t n, uint64_t bit,
                                                            Slot s) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    Cfg c = list[i];
    if (legal(s, c.ver, c.val)) list[i].mask = c.mask | bit;
  }
}

// Keep the configurations this rank owns (replicated -> partitioned).
__global__ __launch_bounds__(256) void fx_filter_kernel(const Cfg *__restrict__ in, int64_t n,
                                                        const Win *__restrict__ gwin, Cfg *out,
                                                        unsigned long long cap, Ctr *ctr) {
  __shared__ Win w;
  load_win(w, gwin);
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x; b < n; b += stride) {
    const int64_t i = b + threadIdx.x;
    Cfg c{};
    bool keep = false;
    if (i < n) {
      c = in[i];
      keep = owner_of(c, w) == (uint32_t)w.rank;
    }
    wave_append(keep, c, out, &ctr->nsel, cap, &ctr->overflow);
  }
}

// Start (or redo) a return: empty R and V, explored back to its value
// before the return.
// ... and, with `words` > 0, fill the first `words` entries of both tables
// with `fill` (the one-word tables' EMPTY): one launch where three were.
__global__ __launch_bounds__(256) void fx_reset_kernel(Ctr *ctr, unsigned long long explored,
                                                       unsigned long long *exp,
                                                       unsigned long long *tagR,
                                                       unsigned long long *tagV, int64_t words,
                                                       unsigned long long fill, Win *dwin,
                                                       const Win win, int put_win) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if (put_win && blockIdx.x == 0) {  // the window travels as the argument: no copy of its own
    const uint32_t *src = reinterpret_cast<const uint32_t *>(&win);
    uint32_t *dst = reinterpret_cast<uint32_t *>(dwin);
    for (int i = threadIdx.x; i < (int)(sizeof(Win) / 4); i += blockDim.x) dst[i] = src[i];
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += stride) {
    tagR[i] = fill;
    tagV[i] = fill;
  }
  if (blockIdx.x || threadIdx.x) return;
  (void)exp;
  ctr_start(ctr, explored);
}

// ------------------------------------------------------------ the queue path
//
// One rank, one-word tables (the usual case): a return is ONE launch, with
// no level structure.  The order in which configurations are expanded does
// not change what a return computes — R (the configurations that linearized
// x), the configurations explored (every V configuration is expanded exactly
// once, by whoever wins its table insert) and the AND over R are functions of
// the frontier and the window alone — so instead of level-synchronous BFS
// (one launch or one grid barrier per level, ~4.6 per return on the oversized
// key, each waiting for the level's slowest wave), the V configurations go
// through one device-wide work queue:
//
//   * every wave first splits its share of F (insert into R / V), then
//     claims runs of queue entries (one atomicAdd on qhead), expands each
//     (lane = window slot), inserts the successors 64 per probe round, and
//     appends the new V ones to the queue (one atomicAdd on qtail per flush);
//   * a queue entry is the configuration's one-word table key, written and
//     read by atomic exchange, which is performed where every CU's atomics
//     are (so no cache of any XCD can hold a stale copy, and no fence is
//     needed); the reader exchanges in EMPTY, so a consumed queue is empty
//     again for the next launch;
//   * termination: total = |F| + qtail counts an item before it exists (at
//     its reservation) and `done` after it is finished (after its successors
//     are reserved), so done <= total always; done read before qtail and
//     equal to |F| + qtail means nothing is left anywhere;
//   * each configuration's version is a function of its mask (vbase +
//     popcount(mask & mutation slots)), so the word is all a queue entry
//     needs;
//   * two table sets and two counter blocks alternate between launches: a
//     launch clears the other set's dirty prefix and zeroes the other
//     counters for the next launch, so a return needs no reset launch;
//   * each workgroup reports (explored, AND of the R entries it appended,
//     the R and V entries it reserved, table-full / overflow flags) to
//     host-mapped memory; the host sums them after one stream sync.  (R
//     entries are flushed after the wave's last item, so no counter read in
//     the kernel can be final for R.)
struct QCtr {
  unsigned long long qtail;  // V entries reserved (the queue's length)
  unsigned long long p0[15];
  unsigned long long qhead;  // V entries claimed
  unsigned long long p1[15];
  unsigned long long done;   // items finished: F entries split + V entries expanded
  unsigned long long p2[15];
  unsigned long long nR;     // R entries reserved
  unsigned long long p3[15];
};
static_assert(sizeof(QCtr) == 512, "one 128-B line per counter");

struct QRep {
  unsigned long long explored;
  unsigned long long andmask;
  unsigned long long flags;  // kQTfull | kQOverflow
  unsigned long long nR, nV; // R and V entries this workgroup reserved (the lists' lengths are the sums)
  unsigned long long tm[8];  // LC_FXQ_TIME: wave-cycles by phase (split, claim, take, drain, insert, flush, wait)
  unsigned long long pad[3];
};
constexpr unsigned long long kQTfull = 1, kQOverflow = 2;
constexpr int kQMaxWG = 512;

struct QArgs {
  const Cfg *F;
  long long nF;
  unsigned long long *Q;  // V queue: one-word keys, EMPTY when free
  Cfg *listR;
  unsigned long long cap;  // capacity of Q and of listR
  unsigned long long *tabR, *tabV;
  uint64_t tmask;
  int cshift;
  uint32_t vbase;  // version of a configuration: vbase + popcount(mask & mutation slots)
  QCtr *ctr;       // this launch's counters (zero on entry)
  QCtr *ctr_next;  // zeroed here for the next launch
  unsigned long long *clrR, *clrV;  // the other table set, whose first clr_words entries ...
  long long clr_words;              // ... are cleared here for the next launch
  QRep *rep;                        // host-mapped, one per workgroup
  int min_claim;                    // smallest run of queue entries a wave claims
  int local;                        // V entries a wave keeps on its own stack (<= kLoc - 64)
  int qatomic;                      // queue entries by atomic exchange (A/B)
  int max_g;
};

// Read a counter where its atomics are performed.  Not an atomic load: the
// compiler turns an idempotent read-modify-write (fetch_add 0) into
// `global_load ... sc1`, which an XCD's L2 may serve from a stale line — a
// stale qtail makes the termination test fire early (configurations lost).
// A returning atomic add of 0, in asm, is a real read-modify-write.
__device__ inline unsigned long long q_read(unsigned long long *p) {
  unsigned long long v;
  asm volatile("global_atomic_add_x2 %0, %1, %2, off sc0\n\ts_waitcnt vmcnt(0)"
               : "=v"(v)
               : "v"(p), "v"(0ULL)
               : "memory");
  return v;
}

// A cheap look at a counter: an agent-scope atomic load (`global_load ...
// sc1`), served by the XCD's L2 and possibly behind — never above — the
// counter (the counters only grow).  Idle waves poll with it, so that they
// do not queue their reads behind the busy waves' claims and reservations
// at the one place the counter's atomics are performed; anything a decision
// rests on is then confirmed with q_read.
__device__ inline unsigned long long q_peek(unsigned long long *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Finished when every item that exists is done: done read before qtail, and
// done <= |F| + qtail always.  Looked at cheaply first; confirmed by real
// reads (or every `every`-th look, so stale peeks cannot hold it off).
__device__ inline bool q_finished(QCtr *ctr, unsigned long long nF, int look, int every) {
  const unsigned long long d = q_peek(&ctr->done);
  const unsigned long long t = q_peek(&ctr->qtail);
  if (d != nF + t && (look % every) != every - 1) return false;
  const unsigned long long d2 = q_read(&ctr->done);
  const unsigned long long t2 = q_read(&ctr->qtail);
  return d2 == nF + t2;
}

// Queue entries.  A producer writes its entry with one 8-byte write-through
// (sc1) store; the consumer polls it with sc1 loads until it is not EMPTY,
// then stores EMPTY back (the queue is empty again for the next launch).
// Every 8th poll of an entry that has not arrived is a read-modify-write
// (compare EMPTY -> EMPTY: changes nothing, returns the entry where the
// atomics are performed), so a stale cached line cannot hold a consumer off.
// qatomic (LC_FXQ_ATOMIC=1, A/B): atomic exchange both ways instead.
__device__ inline void q_put(unsigned long long *e, unsigned long long w, int qatomic) {
  if (qatomic) (void)atomicExch(e, w);
  else __hip_atomic_store(e, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ inline unsigned long long q_take(unsigned long long *e, bool rmw) {
  unsigned long long w;
  if (rmw) w = atomicCAS(e, kEmpty, kEmpty);
  else w = __hip_atomic_load(e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (w != kEmpty) __hip_atomic_store(e, kEmpty, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return w;
}

__device__ inline void q_sleep(int n) {
  for (int i = 0; i < n; i++) __builtin_amdgcn_s_sleep(8);
}

constexpr int kLoc = 256;
struct QStage {
  Cfg s[64];                     // successors gathered, inserted together
  Cfg r[kStage];                 // new R entries
  unsigned long long v[kStage];  // new V entries to spill to the queue (one-word keys)
  unsigned long long loc[kLoc];  // the wave's own stack of V entries to expand
};

__global__ __launch_bounds__(256) void fx_return_kernel(const QArgs a, const Win warg) {
  __shared__ Win w;
  __shared__ QStage stg_all[4];
  __shared__ unsigned long long red_e[4], red_a[4], red_f[4], red_r[4], red_v[4], red_t[4][8];
  // the other table set and counters, for the next launch (plain stores: the
  // launch boundary publishes them)
  {
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < a.clr_words; i += stride) {
      a.clrR[i] = kEmpty;
      a.clrV[i] = kEmpty;
    }
    if (blockIdx.x == 0 && threadIdx.x < 4) {
      unsigned long long *z = &a.ctr_next->qtail + 16 * threadIdx.x;
      *z = 0;
    }
  }
  load_win(w, &warg);
  __syncthreads();
  const int lane = __lane_id(), wid = threadIdx.x / kW;
  QStage *stg = &stg_all[wid];
  const long long wave = (long long)blockIdx.x * (blockDim.x / kW) + wid;
  const long long nwaves = (long long)gridDim.x * (blockDim.x / kW);
  const uint64_t below = (1ULL << lane) - 1;
  const Slot me = w.s[lane];
  const uint64_t bit = 1ULL << lane;
  const uint64_t muts = w.occ & ~w.reads;
  const uint64_t reads = w.occ & w.reads;
  const bool is_mut = (muts & bit) != 0;
  const uint64_t lowmask = (1ULL << a.cshift) - 1;
  uint64_t rv_me = 0, vreads = 0;
  for (uint64_t pr = reads; pr;) {
    const int b = __builtin_ctzll(pr);
    pr &= pr - 1;
    const Slot &r = w.s[b];
    if (r.nvm) vreads |= 1ULL << b;
    else if (!r.nlm || r.nl == me.value) rv_me |= 1ULL << b;
  }
  int ns = 0, nr = 0, nv = 0, nl = 0;  // stash / R stage / V spill stage / local stack (wave-uniform)
  unsigned long long explored = 0, andm = ~0ULL, flags = 0;
  unsigned long long cnt_r = 0, cnt_v = 0;  // entries this wave reserved (wave-uniform)
  unsigned long long tm[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define QT0(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define QT1(v, i) tm[i] += __builtin_amdgcn_s_memtime() - v

  auto flush_r = [&]() {
    if (!nr) return;
    QT0(tf);
    __builtin_amdgcn_wave_barrier();
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(&a.ctr->nR, (unsigned long long)nr);
    base = __shfl(base, 0);
    cnt_r += nr;
    for (int j = lane; j < nr; j += kW) {
      if (base + j < a.cap) a.listR[base + j] = stg->r[j];
      else flags |= kQOverflow;
    }
    __builtin_amdgcn_wave_barrier();
    nr = 0;
    QT1(tf, 5);
  };
  auto flush_v = [&]() {
    if (!nv) return;
    QT0(tf);
    __builtin_amdgcn_wave_barrier();
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(&a.ctr->qtail, (unsigned long long)nv);
    base = __shfl(base, 0);
    cnt_v += nv;
    for (int j = lane; j < nv; j += kW) {
      if (base + j < a.cap) q_put(&a.Q[base + j], stg->v[j], a.qatomic);
      else flags |= kQOverflow;
    }
    __builtin_amdgcn_wave_barrier();
    nv = 0;
    QT1(tf, 5);
  };
  // insert one configuration per lane (have): R when it linearized x (x's
  // bit cleared), else V; the new ones are staged
  auto insert_put = [&](bool have, Cfg c) {
    QT0(ti);
    const bool toR = have && (c.mask & w.xbit);
    if (toR) c.mask &= ~w.xbit;
    int r = -2;
    if (have) r = ctab_insert(toR ? a.tabR : a.tabV, a.tmask, c, a.cshift);
    if (r == -1) flags |= kQTfull;
    QT1(ti, 4);
    const bool nR = r == 1 && toR, nV = r == 1 && !toR;
    const uint64_t mR = __ballot(nR), mV = __ballot(nV);
    if (nR) {
      stg->r[nr + __popcll(mR & below)] = c;
      andm &= c.mask;
    }
    // new V: the wave's own stack first, up to a.local entries; the excess
    // spills to the queue
    const int kv = __popcll(mV), room = max(0, a.local - nl), rk = __popcll(mV & below);
    const unsigned long long word = c.mask | ((unsigned long long)c.val << a.cshift);
    if (nV && rk < room) stg->loc[nl + rk] = word;
    else if (nV) stg->v[nv + rk - room] = word;
    const int kl = min(kv, room);
    nl += kl;
    nr += __popcll(mR);
    nv += kv - kl;
    if (nr > kStage - kW) flush_r();
    if (nv > kStage - kW) flush_v();
  };
  auto insert_stash = [&]() {
    __builtin_amdgcn_wave_barrier();
    const bool have = lane < ns;
    Cfg sc{};
    if (have) sc = stg->s[lane];
    __builtin_amdgcn_wave_barrier();
    insert_put(have, sc);
    ns = 0;
  };
  // expand one configuration (wave-uniform c): lane t tests slot t
  auto expand = [&](const Cfg &c) {
    const bool cand = is_mut && !(c.mask & bit) && !(me.before & ~c.mask) && legal(me, c.ver, c.val);
    Cfg s = c;
    if (cand) {
      s.mask |= bit | rv_me;
      s.ver = c.ver + 1;
      s.val = (uint32_t)me.value;
      uint64_t pr = vreads & ~s.mask;
      while (pr) {
        const int b = __builtin_ctzll(pr);
        pr &= pr - 1;
        if (legal(w.s[b], s.ver, s.val)) s.mask |= 1ULL << b;
      }
    }
    const uint64_t m = __ballot(cand);
    const int k = __popcll(m);
    explored += k;
    if (ns + k > kW) insert_stash();
    if (cand) stg->s[ns + __popcll(m & below)] = s;
    ns += k;
  };

  // Work-first: a wave finishes what it finds.  New V configurations go to
  // the wave's own LDS stack (up to a.local of them) and are expanded by the
  // wave itself; only the excess spills to the device-wide queue, where idle
  // waves claim it.  So the hot queue counters are touched per spilled batch
  // and per claim, not per configuration.  Termination accounting is per
  // GLOBAL item (an F entry, or a queue entry): it counts as done once its
  // local subtree is finished and the wave's spills are reserved.
  unsigned long long g = 0;  // global items taken whose local subtrees are not finished
  auto drain_local = [&]() {
    for (;;) {
      if (nl == 0) {
        if (ns) {  // pending successors may still push local work
          insert_stash();
          continue;
        }
        break;
      }
      const int k = min(nl, kW);
      unsigned long long word = 0;
      if (lane < k) word = stg->loc[nl - k + lane];
      __builtin_amdgcn_wave_barrier();
      nl -= k;
      for (int j = 0; j < k; j++) {
        const unsigned long long wj =
            ((unsigned long long)__shfl((uint32_t)(word >> 32), j) << 32) | __shfl((uint32_t)word, j);
        Cfg c;
        c.mask = wj & lowmask;
        c.val = (uint32_t)(wj >> a.cshift);
        c.ver = a.vbase + (uint32_t)__popcll(c.mask & muts);
        expand(c);
      }
    }
    flush_v();  // spills reserved before the items are counted done
    if (g && lane == 0) atomicAdd(&a.ctr->done, g);
    g = 0;
  };

  // 1. F: a wave takes 64 entries at a time, splits them, and finishes
  // their local subtrees
  QT0(tsplit);
  for (long long b = wave * kW; b < a.nF; b += nwaves * kW) {
    const int cnt = (int)min((long long)kW, a.nF - b);
    Cfg c{};
    if (lane < cnt) {
      c = a.F[b + lane];
      fix_f(c, w);
    }
    insert_put(lane < cnt, c);
    g += (unsigned long long)cnt;
    drain_local();
  }

  QT1(tsplit, 0);
  // 2. the queue: claim runs of spilled entries, finish each one's subtree
  uint64_t pending = 0;  // lanes holding a claimed entry not yet read
  unsigned long long my_idx = 0, t_seen = 0;
  int idle = 0, waits = 0;
  const unsigned long long nF = (unsigned long long)a.nF;
  for (;;) {
    if (!pending) {
      QT0(tc);
      unsigned long long h = 0, t = 0;
      if (lane == 0) {
        t = q_peek(&a.ctr->qtail);
        h = q_peek(&a.ctr->qhead);
      }
      h = __shfl(h, 0);
      t = __shfl(t, 0);
      t_seen = max(t_seen, t);
      if (h < t) {
        const unsigned long long c = min(
            64ULL, max((unsigned long long)a.min_claim,
                       (t - h + (unsigned long long)nwaves - 1) / (unsigned long long)nwaves));
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(&a.ctr->qhead, c);
        base = __shfl(base, 0);
        pending = c == 64 ? ~0ULL : ((1ULL << c) - 1);
        my_idx = base + lane;
        idle = 0;
        QT1(tc, 1);
      } else {
        // nothing to claim: finished when every item that exists is done
        // (done read before qtail; done <= |F| + qtail always)
        int fin = 0;
        if (lane == 0) fin = q_finished(a.ctr, nF, idle, 16);
        if (__shfl(fin, 0)) {
          QT1(tc, 1);
          break;
        }
        q_sleep(idle < 6 ? 1 << idle : 64);
        idle++;
        QT1(tc, 1);
        continue;
      }
    }
    // read the claimed entries that have arrived (an entry reserved beyond
    // the capacity is never written: it is done as soon as it exists)
    const bool mine = (pending >> lane) & 1;
    const bool beyond = my_idx >= a.cap;
    const bool dead = mine && beyond && my_idx < t_seen;
    unsigned long long word = kEmpty;
    QT0(tt);
    if (mine && !beyond) word = q_take(&a.Q[my_idx], a.qatomic || (waits & 7) == 7);
    const bool got = mine && !beyond && word != kEmpty;
    const uint64_t mgot = __ballot(got), mdead = __ballot(dead);
    pending &= ~(mgot | mdead);
    g += (unsigned long long)__popcll(mgot | mdead);
    if (got) stg->loc[__popcll(mgot & below)] = word;  // the local stack is empty here
    nl = __popcll(mgot);
    QT1(tt, 2);
    if (g) {
      QT0(td);
      drain_local();
      QT1(td, 3);
    }
    if (pending && !mgot) {
      QT0(tw);
      // claimed entries not written yet (their producer is mid-flush), or
      // beyond the queue's final length: wait, or finish with everyone
      int end = 0;
      unsigned long long t2 = 0;
      if (lane == 0) {
        end = q_finished(a.ctr, nF, waits, 16);
        t2 = q_peek(&a.ctr->qtail);
      }
      if (__shfl(end, 0)) break;
      t_seen = max(t_seen, __shfl(t2, 0));
      waits++;
      q_sleep(1);
      QT1(tw, 6);
    }
  }
  flush_r();
  // 3. report: this workgroup's explored, R AND, flags
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t lo = __shfl_xor((uint32_t)andm, off), hi = __shfl_xor((uint32_t)(andm >> 32), off);
    andm &= ((unsigned long long)hi << 32) | lo;
    flags |= ((unsigned long long)__shfl_xor((uint32_t)(flags >> 32), off) << 32) |
             __shfl_xor((uint32_t)flags, off);
  }
  if (lane == 0) {
    red_e[wid] = explored;
    red_a[wid] = andm;
    red_f[wid] = flags;
    red_r[wid] = cnt_r;
    red_v[wid] = cnt_v;
    for (int i = 0; i < 8; i++) red_t[wid][i] = tm[i];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    QRep r{};
    r.andmask = ~0ULL;
    for (int k = 0; k < (int)(blockDim.x / kW); k++) {
      r.explored += red_e[k];
      r.andmask &= red_a[k];
      r.flags |= red_f[k];
      r.nR += red_r[k];
      r.nV += red_v[k];
      for (int i = 0; i < 8; i++) r.tm[i] += red_t[k][i];
    }
    a.rep[blockIdx.x] = r;
  }
}

// ------------------------------------------------------------ host side

uint64_t splitmix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}

int32_t clamp_ver(int64_t v) { return (v < -1 || v > kFieldMax) ? kFieldMax : (int32_t)v; }

// In-process transport: k ranks as threads on one device.
struct Hub {
  int P;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool aborted = false;
  std::vector<int64_t> counts;            // P x P
  std::vector<const char *> sendp;
  std::vector<const int64_t *> sendc;
  std::vector<int64_t> red;               // P x n
  explicit Hub(int p) : P(p), counts((size_t)p * p), sendp(p), sendc(p) {}
  int barrier() {
    std::unique_lock<std::mutex> g(mu);
    if (aborted) return -ECANCELED;
    const uint64_t my = gen;
    if (++arrived == P) {
      arrived = 0;
      gen++;
      cv.notify_all();
    } else {
      cv.wait(g, [&] { return gen != my || aborted; });
    }
    return aborted ? -ECANCELED : 0;
  }
  void abort() {
    std::lock_guard<std::mutex> g(mu);
    aborted = true;
    cv.notify_all();
  }
};

struct HubRank {
  Hub *hub;
  int rank;
};

int hub_exchange_counts(void *u, const int64_t *send, int64_t *recv) {
  HubRank *r = static_cast<HubRank *>(u);
  Hub *h = r->hub;
  for (int j = 0; j < h->P; j++) h->counts[(size_t)r->rank * h->P + j] = send[j];
  int e = h->barrier();
  if (e) return e;
  for (int j = 0; j < h->P; j++) recv[j] = h->counts[(size_t)j * h->P + r->rank];
  return h->barrier();
}

int hub_alltoallv(void *u, const void *d_send, const int64_t *send_counts, void *d_recv,
                  const int64_t *recv_counts, int64_t bytes) {
  HubRank *r = static_cast<HubRank *>(u);
  Hub *h = r->hub;
  h->sendp[r->rank] = static_cast<const char *>(d_send);
  h->sendc[r->rank] = send_counts;
  int e = h->barrier();
  if (e) return e;
  char *dst = static_cast<char *>(d_recv);
  for (int j = 0; j < h->P; j++) {
    int64_t off = 0;
    for (int k = 0; k < r->rank; k++) off += h->sendc[j][k];
    const int64_t cnt = h->sendc[j][r->rank];
    if (cnt != recv_counts[j]) {
      h->abort();
      return -EPROTO;
    }
    if (cnt && hipMemcpy(dst, h->sendp[j] + off * bytes, (size_t)(cnt * bytes),
                         hipMemcpyDeviceToDevice) != hipSuccess) {
      h->abort();
      return -EIO;
    }
    dst += cnt * bytes;
  }
  // a device-to-device hipMemcpy may return before the copy has run: the
  // engine reads d_recv on its own stream next
  if (hipStreamSynchronize(nullptr) != hipSuccess) {
    h->abort();
    return -EIO;
  }
  return h->barrier();
}

int hub_allreduce(void *u, int64_t *vals, int32_t n, int32_t op) {
  HubRank *r = static_cast<HubRank *>(u);
  Hub *h = r->hub;
  {
    std::lock_guard<std::mutex> g(h->mu);
    if (h->red.size() < (size_t)h->P * n) h->red.resize((size_t)h->P * n);
  }
  int e = h->barrier();
  if (e) return e;
  std::memcpy(&h->red[(size_t)r->rank * n], vals, sizeof(int64_t) * n);
  e = h->barrier();
  if (e) return e;
  for (int i = 0; i < n; i++) {
    int64_t a = h->red[i];
    for (int j = 1; j < h->P; j++) {
      const int64_t b = h->red[(size_t)j * n + i];
      a = op == LC_FX_MAX ? std::max(a, b) : a + b;
    }
    vals[i] = a;
  }
  return h->barrier();
}

#define FX_TRY(expr)                                                          \
  do {                                                                        \
    hipError_t e_ = (expr);                                                   \
    if (e_ != hipSuccess) {                                                   \
      err = std::string(#expr) + ": " + hipGetErrorString(e_);                \
      return -EIO;                                                            \
    }                                                                         \
  } while (0)

#define FX_COLL(expr)                                                         \
  do {                                                                        \
    int e_ = (expr);                                                          \
    if (e_ != 0) {                                                            \
      err = std::string("collective failed: ") + #expr + " -> " + std::to_string(e_); \
      return e_ < 0 ? e_ : -EIO;                                              \
    }                                                                         \
  } while (0)

#define NC_TRY(expr)                                                          \
  do {                                                                        \
    ncclResult_t r_ = (expr);                                                 \
    if (r_ != ncclSuccess) {                                                  \
      err = std::string(#expr) + ": " + nc->api->GetErrorString(r_);          \
      return -EIO;                                                            \
    }                                                                         \
  } while (0)

// A rank's RCCL communicator (lc_fx_open_devices / lc_fx_open_rccl), with a
// small device + pinned host scratch for the count exchange and the
// reductions.
struct Nccl {
  const RcclApi *api = nullptr;
  ncclComm_t comm = nullptr;
  int64_t *d = nullptr;  // kScr int64: [0, 64) send counts / values, [64, 128) received
  int64_t *h = nullptr;
  bool aborted = false;  // ncclCommAbort freed the communicator
  static constexpr int kScr = 192;
};

struct Rank {
  int dev = 0;
  int rank = 0, P = 1;
  lc_fx_transport tr{};
  Nccl *nc = nullptr;       // collectives over RCCL instead of tr
  bool xself = false;       // LC_FX_FLAG_EXCHANGE_SELF: own candidates go through the exchange too
  // the search runs the multi-rank protocol (ownership, exchange, reductions):
  // several ranks, or one rank exchanging with itself
  bool multi() const { return P > 1 || xself; }
  int64_t part_above = 65536, repl_below = 16384;
  int table_log2 = 0;
  bool force_wide = false;  // LC_FX_FLAG_WIDE_TABLES (tests)
  int cur_cshift = 58;      // this key's compact-word split (tabs())
  hipStream_t st = nullptr;
  std::string err;
  lc_fx_stats stats{};

  // device state
  Cfg *F = nullptr, *Rl = nullptr, *Vl = nullptr, *tmp = nullptr;
  unsigned long long list_cap = 0;
  unsigned long long *tagR = nullptr, *tagV = nullptr;
  Cfg *keyR = nullptr, *keyV = nullptr;
  uint64_t tmask = 0;
  Win *dWin = nullptr, *hWin = nullptr;
  Ctr *dCtr = nullptr, *hCtr = nullptr;
  Rep *hRep = nullptr, *dRep = nullptr;  // host-mapped (sync_ctr)
  unsigned int rep_seq = 0;
  bool copy_sync = false;  // LC_FX_COPY_SYNC=1 (A/B): the copy and stream synchronisation instead
  // LC_FX_HOSTPROF (dev): host time between counter reports (launching, the
  // host's books) against time spinning for them, per check
  bool hostprof = false;
  double hp_host = 0, hp_wait = 0, hp_split = 0, hp_expand = 0;
  long long hp_syncs = 0, hp_nsplit = 0, hp_nexpand = 0;
  std::chrono::steady_clock::time_point hp_mark;
  // Returns alternate between two sets of counters and (one-word mode) two
  // tables, so that a return can prepare the next one's (fx_split_kernel):
  // dCtr = dCtrBase + par, the one-word tables of parity 1 are tagR2 / tagV2.
  Ctr *dCtrBase = nullptr;
  unsigned long long *tagR2 = nullptr, *tagV2 = nullptr;
  int par = 0;
  uint64_t dirtyC[2] = {0, 0};     // one-word tables: entries past this are EMPTY
  bool prepped[2] = {false, false};  // counters reset and tables all EMPTY
  unsigned long long exp_off = 0;  // added to the device's explored (prepared counters start at 0)
  unsigned long long *dExp = nullptr;  // explored shards
  Cfg *cand = nullptr;
  unsigned long long cand_cap = 0;  // per owner region
  Cfg *sendb = nullptr, *recvb = nullptr;
  size_t send_cap = 0, recv_cap = 0;
  uint32_t epoch = 0;
  // queue path (fx_return_kernel): queue, two table sets, two counter blocks,
  // host-mapped per-workgroup reports
  bool qpath = false;  // LC_FX_QUEUE=1: the one-launch-per-return queue path (dev A/B)
  int qdbg_g = 0, qmax_g = kQMaxWG, qmin_claim = 1;
  bool qdbg_time = false;  // LC_FXQ_TIME: host-side launch / sync split on stderr
  double qt_launch = 0, qt_sync = 0, qt_ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int64_t qt_n = 0;
  int64_t qper_wg = 256;
  int qlocal = 64, qatomic = 0;
  bool qdbg_hostclear = false;
  unsigned long long *qQ = nullptr;
  unsigned long long *qtab[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
  QCtr *qctr = nullptr;
  QRep *qrep = nullptr, *qrep_dev = nullptr;
  int qpar = 0;
  long long qdirty[2] = {0, 0};

  ~Rank() { release(); }

  void release() {
    for (void *p : {(void *)F, (void *)Rl, (void *)Vl, (void *)tmp, (void *)tagR, (void *)tagV,
                    (void *)tagR2, (void *)tagV2, (void *)keyR, (void *)keyV, (void *)dWin,
                    (void *)dCtrBase, (void *)cand, (void *)sendb, (void *)recvb})
      if (p) (void)hipFree(p);
    F = Rl = Vl = tmp = keyR = keyV = cand = sendb = recvb = nullptr;
    tagR = tagV = tagR2 = tagV2 = nullptr;
    dWin = nullptr;
    dCtr = dCtrBase = nullptr;
    dExp = nullptr;
    for (void *p : {(void *)qQ, (void *)qtab[0][0], (void *)qtab[0][1], (void *)qtab[1][0],
                    (void *)qtab[1][1], (void *)qctr})
      if (p) (void)hipFree(p);
    qQ = nullptr;
    qtab[0][0] = qtab[0][1] = qtab[1][0] = qtab[1][1] = nullptr;
    qctr = nullptr;
    if (qrep) (void)hipHostFree(qrep);
    qrep = qrep_dev = nullptr;
    if (hWin) (void)hipHostFree(hWin);
    if (hCtr) (void)hipHostFree(hCtr);
    if (hRep) (void)hipHostFree(hRep);
    hWin = nullptr;
    hCtr = nullptr;
    hRep = dRep = nullptr;
    list_cap = 0;
    if (nc) {
      if (nc->d) (void)hipFree(nc->d);
      if (nc->h) (void)hipHostFree(nc->h);
      if (nc->comm && !nc->aborted) (void)nc->api->CommDestroy(nc->comm);
      delete nc;
      nc = nullptr;
    }
    if (st) (void)hipStreamDestroy(st);
    st = nullptr;
  }

  // ---- collectives: the caller's callbacks / the in-process hub (tr), or
  // RCCL on this rank's stream (nc).  Every rank calls them in one order.
  int coll_counts(const int64_t *send, int64_t *recv) {
    if (!nc) return tr.exchange_counts(tr.user, send, recv);
    FX_TRY(hipMemcpyAsync(nc->d, send, sizeof(int64_t) * P, hipMemcpyHostToDevice, st));
    NC_TRY(nc->api->AllToAll(nc->d, nc->d + 64, 1, ncclInt64, nc->comm, st));
    FX_TRY(hipMemcpyAsync(nc->h, nc->d + 64, sizeof(int64_t) * P, hipMemcpyDeviceToHost, st));
    FX_TRY(hipStreamSynchronize(st));
    std::memcpy(recv, nc->h, sizeof(int64_t) * P);
    return 0;
  }

  // Grouped point-to-point sends and receives on the engine's stream: no host
  // synchronisation (the inserts that read d_recv follow on the same stream).
  int nc_a2av(const char *const *src, const int64_t *sc, char *d_recv, const int64_t *rc,
              int64_t bytes) {
    NC_TRY(nc->api->GroupStart());
    int64_t roff = 0;
    for (int j = 0; j < P; j++) {
      if (sc[j]) {
        const ncclResult_t r = nc->api->Send(src[j], (size_t)(sc[j] * bytes / 8), ncclUint64, j,
                                             nc->comm, st);
        if (r != ncclSuccess) {
          (void)nc->api->GroupEnd();
          err = std::string("ncclSend: ") + nc->api->GetErrorString(r);
          return -EIO;
        }
      }
      if (rc[j]) {
        const ncclResult_t r = nc->api->Recv(d_recv + roff * bytes, (size_t)(rc[j] * bytes / 8),
                                             ncclUint64, j, nc->comm, st);
        if (r != ncclSuccess) {
          (void)nc->api->GroupEnd();
          err = std::string("ncclRecv: ") + nc->api->GetErrorString(r);
          return -EIO;
        }
      }
      roff += rc[j];
    }
    NC_TRY(nc->api->GroupEnd());
    return 0;
  }

  int coll_a2av(const void *d_send, const int64_t *sc, void *d_recv, const int64_t *rc,
                int64_t bytes) {
    if (!nc) return tr.alltoallv(tr.user, d_send, sc, d_recv, rc, bytes);
    std::vector<const char *> src(P);
    int64_t off = 0;
    for (int j = 0; j < P; j++) {
      src[j] = static_cast<const char *>(d_send) + off * bytes;
      off += sc[j];
    }
    return nc_a2av(src.data(), sc, static_cast<char *>(d_recv), rc, bytes);
  }

  int coll_allreduce(int64_t *vals, int n, int op) {
    if (!nc) return tr.allreduce(tr.user, vals, n, op);
    if (n > Nccl::kScr) {
      err = "allreduce: too many values";
      return -EINVAL;
    }
    FX_TRY(hipMemcpyAsync(nc->d, vals, sizeof(int64_t) * n, hipMemcpyHostToDevice, st));
    NC_TRY(nc->api->AllReduce(nc->d, nc->d, (size_t)n, ncclInt64, op == LC_FX_MAX ? ncclMax : ncclSum,
                              nc->comm, st));
    FX_TRY(hipMemcpyAsync(nc->h, nc->d, sizeof(int64_t) * n, hipMemcpyDeviceToHost, st));
    FX_TRY(hipStreamSynchronize(st));
    std::memcpy(vals, nc->h, sizeof(int64_t) * n);
    return 0;
  }

  int open() {
    FX_TRY(hipSetDevice(dev));
    FX_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    FX_TRY(hipMalloc(&dWin, sizeof(Win)));
    FX_TRY(hipMalloc(&dCtrBase, 2 * sizeof(Ctr)));
    FX_TRY(hipMemset(dCtrBase, 0, 2 * sizeof(Ctr)));
    dCtr = dCtrBase;
    dExp = &dCtr->exp[0];  // device address, not dereferenced here
    FX_TRY(hipHostMalloc(&hWin, sizeof(Win), hipHostMallocDefault));
    FX_TRY(hipHostMalloc(&hCtr, sizeof(Ctr), hipHostMallocDefault));
    FX_TRY(hipHostMalloc(&hRep, sizeof(Rep), hipHostMallocMapped | hipHostMallocCoherent));
    FX_TRY(hipHostGetDevicePointer(reinterpret_cast<void **>(&dRep), hRep, 0));
    std::memset(hRep, 0, sizeof(Rep));
    rep_seq = 0;
    copy_sync = getenv("LC_FX_COPY_SYNC") && getenv("LC_FX_COPY_SYNC")[0] == '1';
    hostprof = getenv("LC_FX_HOSTPROF") != nullptr;
    std::memset(hWin, 0, sizeof(Win));
    if (const char *q = getenv("LC_FX_QUEUE")) qpath = q[0] == '1';
    if (const char *q = getenv("LC_FXQ_G")) qdbg_g = atoi(q);
    qdbg_time = getenv("LC_FXQ_TIME") != nullptr;
    if (const char *q = getenv("LC_FXQ_MAXG")) qmax_g = std::max(1, std::min(kQMaxWG, atoi(q)));
    if (const char *q = getenv("LC_FXQ_MINCLAIM")) qmin_claim = std::max(1, std::min(64, atoi(q)));
    if (const char *q = getenv("LC_FXQ_PERWG")) qper_wg = std::max(1, atoi(q));
    if (const char *q = getenv("LC_FXQ_LOCAL")) qlocal = std::max(0, std::min(kLoc - 64, atoi(q)));
    if (const char *q = getenv("LC_FXQ_ATOMIC")) qatomic = q[0] == '1';
    if (const char *q = getenv("LC_FXQ_HOSTCLEAR")) qdbg_hostclear = q[0] == '1';
    FX_TRY(hipMalloc(&qctr, 2 * sizeof(QCtr)));
    FX_TRY(hipMemset(qctr, 0, 2 * sizeof(QCtr)));
    FX_TRY(hipHostMalloc(&qrep, kQMaxWG * sizeof(QRep), hipHostMallocMapped | hipHostMallocCoherent));
    FX_TRY(hipHostGetDevicePointer(reinterpret_cast<void **>(&qrep_dev), qrep, 0));
    if (nc) {
      FX_TRY(hipMalloc(&nc->d, sizeof(int64_t) * Nccl::kScr));
      FX_TRY(hipHostMalloc(&nc->h, sizeof(int64_t) * Nccl::kScr, hipHostMallocDefault));
    }
    return 0;
  }

  // Lists and tables for a budget of `budget` configurations.
  int reserve(int64_t budget) {
    if (const char *f = getenv("LC_FX_FAIL_RESERVE"); f && f[0] == '1') {
      err = "list allocation failed (injected: LC_FX_FAIL_RESERVE)";  // test hook
      return -ENOMEM;
    }
    unsigned long long need = (unsigned long long)budget + 1;
    int lg = table_log2;
    if (lg <= 0) {
      lg = 10;
      while ((1ULL << lg) < 2 * need) lg++;
    }
    const uint64_t tcap = 1ULL << lg;
    if (list_cap >= need && tmask + 1 == tcap) return 0;
    for (void *p : {(void *)F, (void *)Rl, (void *)Vl, (void *)tmp, (void *)tagR, (void *)tagV,
                    (void *)tagR2, (void *)tagV2, (void *)keyR, (void *)keyV})
      if (p) (void)hipFree(p);
    FX_TRY(hipMalloc(&F, need * sizeof(Cfg)));
    FX_TRY(hipMalloc(&Rl, need * sizeof(Cfg)));
    FX_TRY(hipMalloc(&Vl, 3 * need * sizeof(Cfg)));  // three V levels
    FX_TRY(hipMalloc(&tmp, need * sizeof(Cfg)));
    FX_TRY(hipMalloc(&tagR, tcap * 8));
    FX_TRY(hipMalloc(&tagV, tcap * 8));
    FX_TRY(hipMalloc(&keyR, tcap * sizeof(Cfg)));
    FX_TRY(hipMalloc(&keyV, tcap * sizeof(Cfg)));
    FX_TRY(hipMemsetAsync(tagR, 0, tcap * 8, st));
    FX_TRY(hipMemsetAsync(tagV, 0, tcap * 8, st));
    if (!multi()) {  // (several ranks reset every return: fx_reset_kernel)
      FX_TRY(hipMalloc(&tagR2, tcap * 8));
      FX_TRY(hipMalloc(&tagV2, tcap * 8));
      FX_TRY(hipMemsetAsync(tagR2, 0xFF, tcap * 8, st));  // EMPTY
      FX_TRY(hipMemsetAsync(tagV2, 0xFF, tcap * 8, st));
    }
    dirtyC[0] = tcap;  // zeroed: epoch tags, not EMPTY
    dirtyC[1] = 0;
    prepped[0] = prepped[1] = false;
    for (void *p : {(void *)qQ, (void *)qtab[0][0], (void *)qtab[0][1], (void *)qtab[1][0],
                    (void *)qtab[1][1]})
      if (p) (void)hipFree(p);
    qQ = nullptr;
    qtab[0][0] = qtab[0][1] = qtab[1][0] = qtab[1][1] = nullptr;
    if (qpath) {
      FX_TRY(hipMalloc(&qQ, need * 8));
      FX_TRY(hipMemsetAsync(qQ, 0xFF, need * 8, st));
      for (int sI = 0; sI < 2; sI++)
        for (int t = 0; t < 2; t++) {
          FX_TRY(hipMalloc(&qtab[sI][t], tcap * 8));
          FX_TRY(hipMemsetAsync(qtab[sI][t], 0xFF, tcap * 8, st));
        }
      qdirty[0] = qdirty[1] = 0;
    }
    list_cap = need;
    tmask = tcap - 1;
    epoch = 0;
    if (multi() && !cand) {
      cand_cap = 1ULL << 21;  // per owner: a chunk of cand_cap / 64 configurations
      FX_TRY(hipMalloc(&cand, (size_t)P * cand_cap * sizeof(Cfg)));
    }
    return 0;
  }

  int ensure_buf(Cfg **p, size_t *cap, size_t n) {
    if (*cap >= n && *p) return 0;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    size_t c = std::max<size_t>(n, 1 << 16);
    FX_TRY(hipMalloc(p, c * sizeof(Cfg)));
    *cap = c;
    return 0;
  }

  // k: the V level a launch reads (it appends level k + 1); k < 0: appends level 0
  Tabs tabs(int lg, int compact, int64_t k) const {
    Tabs t;
    t.compact = compact;
    t.cshift = cur_cshift;
    t.tagR = compact && par ? tagR2 : tagR;
    t.tagV = compact && par ? tagV2 : tagV;
    t.keyR = keyR;
    t.keyV = keyV;
    t.listR = Rl;
    t.vbase = Vl;
    const int64_t src = k < 0 ? 2 : k % 3, dst = k < 0 ? 0 : (k + 1) % 3;
    t.vsrc = Vl + (size_t)src * list_cap;
    t.vdst = Vl + (size_t)dst * list_cap;
    t.vcnt = &dCtr->cnt[dst];
    t.tmask = std::min<uint64_t>(tmask, (1ULL << lg) - 1);
    t.list_cap = list_cap;
    t.exp = dExp;
    return t;
  }

  // Ctr to the host; its explored is the sum of the shards.
  // The report kernel writes the counters to host-mapped memory, `seq` last;
  // the host spins on it (checking the stream every 1,024 rounds, so that an
  // error ends the wait; past 20 ms it synchronises the stream instead).
  int sync_ctr() {
    if (!copy_sync) {
      const unsigned int s = ++rep_seq;
      fx_report_kernel<<<1, 64, 0, st>>>(dCtr, dRep, s);
      FX_TRY(hipGetLastError());
      const auto t0 = std::chrono::steady_clock::now();
      if (hostprof) {
        hp_host += std::chrono::duration<double, std::micro>(t0 - hp_mark).count();
        hp_syncs++;
      }
      for (uint32_t i = 1; __atomic_load_n(&hRep->seq, __ATOMIC_ACQUIRE) != s; i++) {
        if (i & 1023) continue;
        const hipError_t q = hipStreamQuery(st);
        if (q != hipSuccess && q != hipErrorNotReady) FX_TRY(q);
        if (q == hipSuccess && __atomic_load_n(&hRep->seq, __ATOMIC_ACQUIRE) != s) {
          err = "counter report lost";
          return -EIO;
        }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20))
          FX_TRY(hipStreamSynchronize(st));
      }
      const Rep &r = *hRep;
      hCtr->nV = r.nV;
      hCtr->kcur = r.kcur;
      hCtr->explored = r.explored + exp_off;
      hCtr->levels = r.levels;
      hCtr->andmask = r.andmask;
      hCtr->overflow = r.overflow;
      hCtr->nsel = r.nsel;
      hCtr->tfull = r.tfull;
      hCtr->nR = r.nR;
      for (int i = 0; i < 3; i++) hCtr->cnt[i] = r.cnt[i];
      for (int i = 0; i < 64; i++) hCtr->cand[i] = r.cand[i];
      for (int i = 0; i < kMaxCls; i++) hCtr->cmin[i] = r.cmin[i];
      if (hostprof) {
        hp_mark = std::chrono::steady_clock::now();
        hp_wait += std::chrono::duration<double, std::micro>(hp_mark - t0).count();
      }
      return 0;
    }
    FX_TRY(hipMemcpyAsync(hCtr, dCtr, sizeof(Ctr), hipMemcpyDeviceToHost, st));
    FX_TRY(hipStreamSynchronize(st));
    unsigned long long e = 0;
    for (int i = 0; i < kExpShards; i++) {
      e += hCtr->exp[i * kExpStride];
      hCtr->nV += hCtr->exp[i * kExpStride + 1];
    }
    hCtr->explored = e + exp_off;
    unsigned long long a = ~0ULL;
    for (int i = 0; i < kAndShards; i++) a &= hCtr->andm[i * kExpStride];
    hCtr->andmask = a;
    return 0;
  }

  static int grid_for(int64_t n) {
    return (int)std::max<int64_t>(1, std::min<int64_t>(kFlatWG, (n + 255) / 256));
  }

  // Send `n` configurations at `src` (device) to every rank as a group, or
  // count-first all-to-all of the per-owner candidate regions.
  int gather_all(int64_t nF, int64_t *nOut) {
    std::vector<int64_t> sc(P, nF), rc(P, 0);
    if (int e = ensure_buf(&sendb, &send_cap, (size_t)std::max<int64_t>(nF * P, 1))) return e;
    for (int j = 0; j < P; j++)
      if (nF)
        FX_TRY(hipMemcpyAsync(sendb + (size_t)j * nF, F, nF * sizeof(Cfg), hipMemcpyDeviceToDevice, st));
    FX_TRY(hipStreamSynchronize(st));
    FX_COLL(coll_counts(sc.data(), rc.data()));
    int64_t tot = 0;
    for (int j = 0; j < P; j++) tot += rc[j];
    if ((unsigned long long)tot > list_cap) {
      err = "gathered frontier exceeds the list capacity";
      return -ENOMEM;
    }
    FX_COLL(coll_a2av(sendb, sc.data(), F, rc.data(), sizeof(Cfg)));
    *nOut = tot;
    stats.gathers++;
    return 0;
  }

  // One partitioned level chunk: candidates of V[a, b) to their owners.
  // Over RCCL the per-owner counts the expand kernel left in dCtr->cand are
  // exchanged on the device (one all-to-all of P words, read back with the
  // counters in one copy), and each owner's region is sent straight from
  // where the kernel wrote it (grouped ncclSend / ncclRecv, no packing, no
  // host synchronisation before the inserts that follow on the stream).
  int part_chunk(int64_t a, int64_t b, const Tabs &tb) {
    FX_TRY(hipMemsetAsync(dCtr->cand, 0, sizeof(unsigned long long) * P, st));
    if (b > a) {
      const int g = (int)std::max<int64_t>(1, std::min<int64_t>(kExpandWG, (b - a + 3) / 4));
      fx_expand_kernel<<<g, 256, 0, st>>>(dWin, tb, epoch, dCtr, 0, a, b, cand, cand_cap, 0, 0);
      FX_TRY(hipGetLastError());
    }
    std::vector<int64_t> sc(P), rc(P);
    if (nc) {
      static_assert(sizeof(unsigned long long) == sizeof(int64_t), "count words");
      NC_TRY(nc->api->AllToAll(dCtr->cand, nc->d + 64, 1, ncclInt64, nc->comm, st));
      FX_TRY(hipMemcpyAsync(nc->h + 64, nc->d + 64, sizeof(int64_t) * P, hipMemcpyDeviceToHost, st));
    }
    if (int e = sync_ctr()) return e;
    int64_t tot_send = 0, tot = 0;
    for (int j = 0; j < P; j++) {
      const bool peer = j != rank || xself;  // own candidates are inserted directly
      sc[j] = peer ? (int64_t)std::min<unsigned long long>(hCtr->cand[j], cand_cap) : 0;
      // (a sender clamps an overflowing region to cand_cap and raises the
      // overflow flag, which makes the level :unknown on every rank)
      if (nc) rc[j] = peer ? std::min<int64_t>(nc->h[64 + j], (int64_t)cand_cap) : 0;
      tot_send += sc[j];  // (its own only with LC_FX_FLAG_EXCHANGE_SELF)
    }
    const int64_t self =
        xself ? 0 : (int64_t)std::min<unsigned long long>(hCtr->cand[rank], cand_cap);
    if (self) {
      fx_insert_kernel<<<grid_for(self), 256, 0, st>>>(cand + (size_t)rank * cand_cap, self, dWin,
                                                      tb, epoch, dCtr);
      FX_TRY(hipGetLastError());
    }
    if (nc) {
      for (int j = 0; j < P; j++) tot += rc[j];
      if (int e = ensure_buf(&recvb, &recv_cap, (size_t)std::max<int64_t>(tot, 1))) return e;
      std::vector<const char *> src(P);
      for (int j = 0; j < P; j++)
        src[j] = reinterpret_cast<const char *>(cand + (size_t)j * cand_cap);
      FX_COLL(nc_a2av(src.data(), sc.data(), reinterpret_cast<char *>(recvb), rc.data(),
                      sizeof(Cfg)));
    } else {
      int64_t n_send = 0;
      for (int j = 0; j < P; j++) n_send += sc[j];
      if (int e = ensure_buf(&sendb, &send_cap, (size_t)std::max<int64_t>(n_send, 1))) return e;
      int64_t off = 0;
      for (int j = 0; j < P; j++) {
        if (sc[j])
          FX_TRY(hipMemcpyAsync(sendb + off, cand + (size_t)j * cand_cap, sc[j] * sizeof(Cfg),
                                hipMemcpyDeviceToDevice, st));
        off += sc[j];
      }
      FX_TRY(hipStreamSynchronize(st));
      FX_COLL(coll_counts(sc.data(), rc.data()));
      for (int j = 0; j < P; j++) tot += rc[j];
      if (int e = ensure_buf(&recvb, &recv_cap, (size_t)std::max<int64_t>(tot, 1))) return e;
      FX_COLL(coll_a2av(sendb, sc.data(), recvb, rc.data(), sizeof(Cfg)));
    }
    stats.sent_configs += tot_send;
    if (tot) {
      fx_insert_kernel<<<grid_for(tot), 256, 0, st>>>(recvb, tot, dWin, tb, epoch, dCtr);
      FX_TRY(hipGetLastError());
    }
    return 0;
  }

  int check(const lc_op *o, int64_t n, const lc_opts *opts, lc_key_result *res);

  // lc_fx_frontier: stop at the return of record stop_op and copy out up to
  // dump_max configurations of the frontier that return would expand
  int64_t stop_op = -1;
  lc_fx_config *dump = nullptr;
  int32_t dump_max = 0, dump_n = 0;
};

bool same_class(const lc_op &a, const lc_op &b) {
  return a.f == b.f && a.value == b.value && a.expected == b.expected && a.version == b.version;
}

struct Ev {
  int64_t idx;
  int32_t is_ret;
  int32_t op;
};

void result_init(lc_key_result *r) {
  r->verdict = LC_VALID;
  r->reason = LC_REASON_NONE;
  r->fail_op = -1;
  r->fail_prefix_end = -1;
  r->configs_explored = 0;
  r->max_frontier = 0;
}

void result_unknown(lc_key_result *r, int reason) {
  r->verdict = LC_UNKNOWN;
  r->reason = reason;
  r->fail_op = -1;
  r->fail_prefix_end = -1;
}

int Rank::check(const lc_op *o, int64_t n, const lc_opts *opts_in, lc_key_result *res) {
  const auto t0 = std::chrono::steady_clock::now();
  hp_mark = t0;
  std::memset(&stats, 0, sizeof(stats));
  lc_opts opts;
  if (opts_in) {
    opts = *opts_in;
  } else {
    opts.init_version = 0;
    opts.init_value = LC_NIL;
    opts.max_configs_per_key = 0;
    opts.time_budget_ms = 0;
    opts.flags = 0;
  }
  if (opts.init_version < 0 || opts.init_version > kFieldMax || opts.init_value < -1 ||
      opts.init_value > kFieldMax) {
    err = "lc_opts: init_version/init_value out of int32 range";
    return -EINVAL;
  }
  result_init(res);
  if (n == 0) return 0;
  // Per-key validity (lc_check's rules): malformed -> :unknown reason 4,
  // an unknown :f -> reason 5 (register.clj:63 throws).
  for (int64_t i = 0; i < n; i++) {
    const lc_op &a = o[i];
    if (a.call < 0 || a.ret <= a.call || (i > 0 && a.call <= o[i - 1].call) || a.value < -1 ||
        a.value > kFieldMax || a.expected < -1 || a.expected > kFieldMax) {
      result_unknown(res, LC_REASON_MALFORMED);
      return 0;
    }
  }
  for (int64_t i = 0; i < n; i++)
    if (o[i].f != LC_F_READ && o[i].f != LC_F_WRITE && o[i].f != LC_F_CAS) {
      result_unknown(res, LC_REASON_UNKNOWN_F);
      return 0;
    }
  const int64_t budget = opts.max_configs_per_key > 0 ? opts.max_configs_per_key : (int64_t)1 << 24;
  if (int e = reserve(budget)) return e;

  std::vector<Ev> ev;
  ev.reserve((size_t)(2 * n));
  for (int64_t i = 0; i < n; i++) {
    ev.push_back({o[i].call, 0, (int32_t)i});
    if (o[i].ret != LC_INF) ev.push_back({o[i].ret, 1, (int32_t)i});
  }
  std::sort(ev.begin(), ev.end(), [](const Ev &a, const Ev &b) {
    if (a.idx != b.idx) return a.idx < b.idx;
    if (a.is_ret != b.is_ret) return a.is_ret < b.is_ret;
    return a.op < b.op;
  });

  std::vector<int32_t> slot_of((size_t)n, -1);
  int32_t slot_op[kW];
  uint64_t before[kW] = {0};
  uint64_t occ = 0, reads = 0, kzob = 0;
  uint64_t fclear = 0, fclose = 0;  // one rank: F's pending retirement / read closures
  Win &w = *hWin;
  std::memset(&w, 0, sizeof(Win));
  w.rank = rank;
  w.n_ranks = P;

  // Values are interned per key to dense ids (nil first): the model only
  // compares them for equality (register.clj:77,92), and the compact tables
  // pack the id beside the mask.
  std::unordered_map<int64_t, int32_t> vids;
  auto vid = [&](int64_t v) {
    auto it = vids.find(v);
    if (it != vids.end()) return it->second;
    const int32_t k = (int32_t)vids.size();
    vids.emplace(v, k);
    return k;
  };
  vid(LC_NIL);
  vid(opts.init_value);
  for (int64_t i = 0; i < n; i++) {
    if (o[i].f != LC_F_READ || o[i].value != LC_NIL) vid(o[i].value);
    if (o[i].f == LC_F_CAS) vid(o[i].expected);
  }
  const int64_t n_vals = (int64_t)vids.size();
  int vbits = 6;  // value-id bits of the compact word: ids 0 .. n_vals - 1, all-ones unused
  while ((1LL << vbits) - 1 < n_vals) vbits++;
  const int cshift = 64 - vbits;  // < 44 (over 2^20 - 1 values): 16-byte keys
  cur_cshift = cshift;

  // F = {(init state, nothing linearized)}
  Cfg init{0, (uint32_t)opts.init_version, (uint32_t)vid(opts.init_value)};
  FX_TRY(hipMemcpyAsync(F, &init, sizeof(Cfg), hipMemcpyHostToDevice, st));
  FX_TRY(hipMemsetAsync(dCtrBase, 0, 2 * sizeof(Ctr), st));
  FX_TRY(hipStreamSynchronize(st));
  par = 0;
  dCtr = dCtrBase;
  dExp = &dCtr->exp[0];
  prepped[0] = prepped[1] = false;
  exp_off = 0;
  int64_t levels_total = 0;  // levels expanded (each return's counters count from 0)
  int64_t nF = 1, nFglobal = 1;
  bool part = false;
  int64_t max_frontier = 1;
  int64_t explored_repl = 0, explored_part = 0;
  unsigned long long explored_seen = 0;
  int spec_levels = 4;
  int64_t levels_seen = 0, last_work = 0, work_hi = 0;
  bool tags_dirty = true;
  const int tlog_full = __builtin_ctzll(tmask + 1);
  int tlog = 12;
  const bool timed = opts.time_budget_ms > 0;
  bool decided = false;
  const bool debug = getenv("LC_FX_DEBUG") != nullptr;
  const int64_t tmul = getenv("LC_FX_TABLE_MUL") ? std::max(1, atoi(getenv("LC_FX_TABLE_MUL"))) : 4;
  const int64_t spad = getenv("LC_FX_SPEC_PAD") ? atoi(getenv("LC_FX_SPEC_PAD")) : 1;
  // second-hop places per wave of a level launch (LC_FX_HOP2, 0..kHop2)
  const int hop2 = getenv("LC_FX_HOP2") ? std::max(0, std::min(kHop2, atoi(getenv("LC_FX_HOP2")))) : 32;
  // later hops per level launch (LC_FX_HOPS; 0: one level per launch)
  const int hops = hop2 ? (getenv("LC_FX_HOPS") ? std::max(0, std::min(16, atoi(getenv("LC_FX_HOPS")))) : 8) : 0;
  // the split and the first levels in one launch (one rank; LC_FX_MERGE=0:
  // fx_split_kernel, then the level launches)
  const bool merge_on = !multi() && hops > 0 && !(getenv("LC_FX_MERGE") && getenv("LC_FX_MERGE")[0] == '0');
  const int64_t mpad = getenv("LC_FX_MERGE_PAD") ? std::max(0, atoi(getenv("LC_FX_MERGE_PAD"))) : 0;
  // A/B switch (dev): LC_FX_PREP=0 resets every return by a launch of its own
  const bool allow_prep = !(getenv("LC_FX_PREP") && getenv("LC_FX_PREP")[0] == '0');
  // queue path: the version every configuration of a return has before the
  // mutation slots its mask names (the initial one plus every mutation that
  // left the window linearized: returned, or retired)
  uint32_t vbase = (uint32_t)opts.init_version;

  auto slot_pre = [&](const lc_op &a, Slot &s) {
    const int32_t ver = clamp_ver(a.version);
    const int32_t vchk = ver != -1 ? -1 : 0;
    if (a.f == LC_F_READ) {
      s.nv = ver;
      s.nvm = vchk;
      s.nl = a.value != LC_NIL ? vid(a.value) : 0;
      s.nlm = a.value != LC_NIL ? -1 : 0;
      s.value = 0;
    } else {
      s.nv = ver - 1;
      s.nvm = vchk;
      s.nl = a.f == LC_F_CAS ? vid(a.expected) : 0;
      s.nlm = a.f == LC_F_CAS ? -1 : 0;
      s.value = vid(a.value);
    }
  };

  // Counted classes (see kClsLane): crashed writes/CAS grouped by
  // (f, value, expected, version), each class a field wide enough for all of
  // its members in the key, placed just below the value-id bits; the slots
  // keep the bits below the fields.  LC_FX_CLASSES=0: one slot per crashed op.
  std::vector<int32_t> cls_of((size_t)n, -1);
  std::vector<std::vector<int32_t>> cls_members;  // call order
  int64_t cls_called[kMaxCls] = {0}, cls_base[kMaxCls] = {0};
  int slot_max = kW;  // slots are bits [0, slot_max)
  uint64_t fsub = 0;  // one rank: class members retired since the last return
  // (several ranks apply retirement at once: fx_clear_kernel / fx_sub_kernel)
  {
    const char *ce = getenv("LC_FX_CLASSES");
    const bool want = !(ce && ce[0] == '0');
    std::vector<int32_t> rep;
    for (int64_t i = 0; want && i < n; i++) {
      if (o[i].ret != LC_INF || o[i].f == LC_F_READ) continue;
      int c = 0;
      while (c < (int)rep.size() && !same_class(o[rep[c]], o[i])) c++;
      if (c == (int)rep.size()) {
        if (c == kMaxCls) break;  // too many classes: slots as before
        rep.push_back((int32_t)i);
        cls_members.emplace_back();
      }
      cls_members[c].push_back((int32_t)i);
    }
    int sumw = 0;
    for (auto &m : cls_members) sumw += 64 - __builtin_clzll((unsigned long long)m.size());
    const int top = cshift >= 44 ? cshift : kW;
    const bool fits = !rep.empty() && (int)rep.size() <= kMaxCls &&
                      (int64_t)rep.size() == (int64_t)cls_members.size() && sumw + 8 <= top;
    bool complete = true;  // every crashed mutation found its class
    for (int64_t i = 0; i < n && fits; i++)
      if (o[i].ret == LC_INF && o[i].f != LC_F_READ) {
        bool in = false;
        for (auto &r : rep) in |= same_class(o[r], o[i]);
        complete &= in;
      }
    if (fits && complete) {
      int shift = top - sumw;
      slot_max = std::min(shift, kClsLane0);
      for (int c = 0; c < (int)rep.size(); c++) {
        const int width = 64 - __builtin_clzll((unsigned long long)cls_members[c].size());
        for (int32_t m : cls_members[c]) cls_of[m] = c;
        Slot &cl = w.s[kClsLane0 + c];
        std::memset(&cl, 0, sizeof(Slot));
        slot_pre(o[rep[c]], cl);
        cl.cls = kClsLane | (width << 8) | shift;
        cl.zob = 0;  // members available (called, not retired)
        shift += width;
      }
    } else {
      cls_members.clear();
    }
  }
  const int n_cls = (int)cls_members.size();

  for (size_t e = 0; e < ev.size() && !decided; e++) {
    const int32_t x = ev[e].op;
    const lc_op &ox = o[x];
    if (!ev[e].is_ret) {
      // trivial reads (crashed, or [nil nil]) never constrain: no slot
      if (ox.f == LC_F_READ && (ox.ret == LC_INF || (ox.version == LC_NIL && ox.value == LC_NIL)))
        continue;
      if (cls_of[x] >= 0) {  // a crashed write/CAS: one more member of its class
        const int c = cls_of[x];
        cls_called[c]++;
        w.s[kClsLane0 + c].zob = (uint64_t)(cls_called[c] - cls_base[c]);
        continue;
      }
      if (occ == ~0ULL || __builtin_ctzll(~occ) >= slot_max) {
        result_unknown(res, LC_REASON_WINDOW_OVERFLOW);
        decided = true;
        break;
      }
      const int s = __builtin_ctzll(~occ);
      const uint64_t sb = 1ULL << s;
      occ |= sb;
      slot_of[x] = s;
      slot_op[s] = x;
      before[s] = 0;
      Slot &sl = w.s[s];
      std::memset(&sl, 0, sizeof(Slot));
      slot_pre(ox, sl);
      if (ox.f == LC_F_READ) {
        reads |= sb;
        sl.zob = 0;
        // closure: the new read is linearized wherever it is legal now (one
        // rank: by the next split, as it reads the frontier)
        if (!multi()) {
          fclose |= sb;
        } else if (nF) {
          fx_close_read_kernel<<<grid_for(nF), 256, 0, st>>>(F, nF, sb, sl);
          FX_TRY(hipGetLastError());
        }
      } else {
        reads &= ~sb;
        sl.zob = splitmix(0xF0F0ULL + (uint64_t)x) | 1;
        for (int u = 0; u < kW; u++) {
          if (u == s || !((occ >> u) & 1) || ((reads >> u) & 1)) continue;
          if (!same_class(o[slot_op[u]], ox)) continue;
          if (o[slot_op[u]].ret <= ox.ret) before[s] |= 1ULL << u;
          else before[u] |= sb;
        }
        // a counted class's crashed members wait for its pending :ok members
        for (int c = 0; c < n_cls; c++)
          if (same_class(o[cls_members[c][0]], ox)) before[kClsLane0 + c] |= sb;
      }
      continue;
    }
    if (slot_of[x] < 0) continue;  // trivial read, or retired
    if (x == stop_op) {
      // lc_fx_frontier: the frontier this return would expand, with the
      // updates the next split would apply (retirements, reads called since)
      const int64_t k = std::min<int64_t>(nF, dump_max);
      std::vector<Cfg> hc((size_t)k);
      if (k) FX_TRY(hipMemcpy(hc.data(), F, sizeof(Cfg) * (size_t)k, hipMemcpyDeviceToHost));
      std::vector<int64_t> val_of(vids.size());
      for (const auto &kv : vids) val_of[(size_t)kv.second] = kv.first;
      for (int64_t i = 0; i < k; i++) {
        Cfg c = hc[(size_t)i];
        c.mask &= ~fclear;
        for (uint64_t pr = fclose; pr;) {
          const int b = __builtin_ctzll(pr);
          pr &= pr - 1;
          const Slot &r = w.s[b];
          if (((((int32_t)c.ver ^ r.nv) & r.nvm) | (((int32_t)c.val ^ r.nl) & r.nlm)) == 0)
            c.mask |= 1ULL << b;
        }
        lc_fx_config &d = dump[i];
        d.version = (int64_t)c.ver;
        d.value = val_of[c.val];
        d.n_pending = 0;
        for (uint64_t pend = occ & ~c.mask; pend;) {
          const int b = __builtin_ctzll(pend);
          pend &= pend - 1;
          d.pending[d.n_pending++] = slot_op[b];
        }
        c.mask -= fsub;  // (class members retired since the last split)
        for (int cc = 0; cc < n_cls; cc++) {  // a class's members past this configuration's count
          const int64_t lin = cls_base[cc] + (int64_t)cls_get(c.mask, w.s[kClsLane0 + cc].cls);
          for (int64_t j = lin; j < cls_called[cc] && d.n_pending < 64; j++)
            d.pending[d.n_pending++] = cls_members[cc][(size_t)j];
        }
        std::sort(d.pending, d.pending + d.n_pending);
      }
      dump_n = (int32_t)k;
      res->verdict = LC_UNKNOWN;
      res->reason = LC_REASON_NONE;
      decided = true;
      break;
    }
    const int sx = slot_of[x];
    const uint64_t xb = 1ULL << sx;
    // the window as the device sees it during this return
    w.occ = occ;
    w.reads = reads;
    w.xbit = xb;
    w.kzob = kzob;
    for (int u = 0; u < kW; u++) w.s[u].before = before[u];
    w.fclear = fclear;
    w.fclose = fclose;
    w.fsub = fsub;
    fclear = fclose = fsub = 0;
    w.slot_bits = n_cls ? (1ULL << slot_max) - 1 : ~0ULL;
    w.n_cls = n_cls;
    for (int c = 0; c < n_cls; c++) w.cbase[c] = (uint32_t)cls_base[c];
    if (multi()) FX_TRY(hipMemcpyAsync(dWin, &w, sizeof(Win), hipMemcpyHostToDevice, st));
    // mode switches (several ranks only)
    if (multi() && !part && nFglobal > part_above) {
      FX_TRY(hipMemsetAsync(&dCtr->nsel, 0, sizeof(unsigned long long), st));
      fx_filter_kernel<<<grid_for(nF), 256, 0, st>>>(F, nF, dWin, tmp, list_cap, dCtr);
      FX_TRY(hipGetLastError());
      if (int er = sync_ctr()) return er;
      std::swap(F, tmp);
      nF = (int64_t)hCtr->nsel;
      part = true;
    } else if (multi() && part && nFglobal < repl_below) {
      int64_t tot = 0;
      if (int er = gather_all(nF, &tot)) return er;
      nF = tot;
      part = false;
    }
    stats.returns++;
    const int compact = !force_wide && (occ >> cshift) == 0 && cshift >= 44;
    if (!compact) stats.wide_returns++;
    int64_t nRg = 0;   // global size of R after this return
    bool over = false, timeout = false;
    // Dedup tables: a power-of-two prefix sized from the work this return is
    // likely to hold (the frontier, and the last return's R + V), so small
    // returns probe lines that stay in L2; a probe chain that runs too long
    // (tfull) redoes the return with a 4x larger prefix.
    {
      // the prefix follows the recent peak (decaying), not only the last return
    work_hi = std::max<int64_t>(last_work, work_hi - work_hi / 8);
    const int64_t guess = std::max<int64_t>(std::max<int64_t>(nF, last_work), work_hi / 2) * tmul;
      tlog = 12;
      while (tlog < tlog_full && (1LL << tlog) < guess) tlog++;
    }
    dCtr = dCtrBase + par;
    dExp = &dCtr->exp[0];
    // the replicated return by the grid (not one workgroup, not the queue path)
    const bool grid_ret = !part && !(qpath && !multi() && compact && !n_cls) &&
                          !(nF <= kSmallF && last_work <= kSmallWork);
    for (int attempt = 0;; attempt++) {
      const Tabs tb = tabs(tlog, compact, -1);  // the split appends V level 0
      epoch++;
      if (compact) {
        tags_dirty = true;  // one-word tables start EMPTY: the reset fills this attempt's prefix
      } else {
        dirtyC[0] = tmask + 1;  // tagR / tagV hold epoch tags
        if (tags_dirty) {
          // back to epoch tags after compact returns: no stale word may look live
          FX_TRY(hipMemsetAsync(tagR, 0, (tmask + 1) * 8, st));
          FX_TRY(hipMemsetAsync(tagV, 0, (tmask + 1) * 8, st));
          tags_dirty = false;
        }
      }
      // the previous return prepared this one's counters and tables (one
      // rank, one-word tables, first attempt): no reset launch
      const bool use_prep = attempt == 0 && compact && grid_ret && prepped[par] && !multi();
      prepped[par] = false;
      levels_seen = 0;  // (the reset and the preparation count levels from 0)
      if (use_prep) {
        exp_off = explored_seen;
      } else {
        exp_off = 0;
        const int64_t words = compact ? (int64_t)1 << tlog : 0;
        fx_reset_kernel<<<grid_for(words), 256, 0, st>>>(dCtr, explored_seen, dExp, tb.tagR, tb.tagV,
                                                          words, kEmpty, dWin, w, !multi());
        FX_TRY(hipGetLastError());
      }
      if (compact) dirtyC[par] = std::max<uint64_t>(dirtyC[par], 1ULL << tlog);
      bool tfull = false;
      if (qpath && !multi() && compact && !n_cls) {
        // one launch per attempt (fx_return_kernel): split, queue, report
        int G = (int)std::min<int64_t>(
            qmax_g, std::max<int64_t>(1, (std::max(nF, last_work) + qper_wg - 1) / qper_wg));
        if (qdbg_g > 0) G = qdbg_g;  // LC_FXQ_G (debug)
        QArgs qa;
        qa.F = F;
        qa.nF = nF;
        qa.Q = qQ;
        qa.listR = Rl;
        qa.cap = list_cap;
        qa.tabR = qtab[qpar][0];
        qa.tabV = qtab[qpar][1];
        qa.tmask = std::min<uint64_t>(tmask, (1ULL << tlog) - 1);
        qa.cshift = cshift;
        qa.vbase = vbase;
        qa.ctr = qctr + qpar;
        qa.ctr_next = qctr + (qpar ^ 1);
        qa.clrR = qtab[qpar ^ 1][0];
        qa.clrV = qtab[qpar ^ 1][1];
        qa.clr_words = qdirty[qpar ^ 1];
        qa.rep = qrep_dev;
        qa.min_claim = qmin_claim;
        qa.local = qlocal;
        qa.qatomic = qatomic;
        qa.max_g = 0;
        if (qdbg_hostclear) {  // LC_FXQ_HOSTCLEAR (debug): tables cleared by the host instead
          FX_TRY(hipMemsetAsync(qa.tabR, 0xFF, (qa.tmask + 1) * 8, st));
          FX_TRY(hipMemsetAsync(qa.tabV, 0xFF, (qa.tmask + 1) * 8, st));
          qa.clr_words = 0;
        }
        const auto tq0 = std::chrono::steady_clock::now();
        fx_return_kernel<<<G, 256, 0, st>>>(qa, w);
        FX_TRY(hipGetLastError());
        qdirty[qpar ^ 1] = 0;
        qdirty[qpar] = (long long)qa.tmask + 1;
        qpar ^= 1;
        const auto tq1 = std::chrono::steady_clock::now();
        FX_TRY(hipStreamSynchronize(st));
        if (qdbg_time) {
          const auto tq2 = std::chrono::steady_clock::now();
          qt_launch += std::chrono::duration<double, std::micro>(tq1 - tq0).count();
          qt_sync += std::chrono::duration<double, std::micro>(tq2 - tq1).count();
          qt_n++;
        }
        unsigned long long q_expl = 0, q_and = ~0ULL, q_flags = 0;
        int64_t q_nR = 0, q_nV = 0;
        for (int g = 0; g < G; g++) {
          if (qdbg_time)
            for (int i = 0; i < 8; i++) qt_ph[i] += (double)qrep[g].tm[i];
          q_expl += qrep[g].explored;
          q_and &= qrep[g].andmask;
          q_flags |= qrep[g].flags;
          q_nR += (int64_t)qrep[g].nR;
          q_nV += (int64_t)qrep[g].nV;
        }
        const bool q_tfull = (q_flags & kQTfull) != 0;
        if (q_tfull && tlog < tlog_full) {
          tlog = std::min(tlog + 2, tlog_full);
          stats.redos++;
          continue;
        }
        over = q_tfull || (q_flags & kQOverflow) || q_nR + q_nV > budget;
        explored_repl += (int64_t)q_expl;
        explored_seen += q_expl;  // the level path's counters start from it
        hCtr->nR = (unsigned long long)q_nR;
        hCtr->andmask = q_and;
        nRg = q_nR;
        last_work = q_nR + q_nV;
        if (timed) timeout = std::chrono::duration<double, std::milli>(
                                 std::chrono::steady_clock::now() - t0).count() > (double)opts.time_budget_ms;
        break;
      }
      if (!part) {
        // replicated: a small return runs whole in one workgroup; otherwise
        // (or for what it leaves) speculative batches of levels over the
        // grid, one sync per batch
        const bool small = nF <= kSmallF && last_work <= kSmallWork;
        const bool merge = merge_on && !small;
        int64_t k = 0;  // the next V level to expand
        bool done = false;
        if (small) {
          fx_small_return_kernel<<<1, 256, 0, st>>>(F, nF, dWin, tb, epoch, dCtr, kSmallLevel);
          FX_TRY(hipGetLastError());
          if (int er = sync_ctr()) return er;
          k = (int64_t)hCtr->kcur;
          done = hCtr->tfull || hCtr->overflow || hCtr->cnt[k % 3] == 0;
        } else if (nF) {
          // one rank, one-word tables: the split also prepares the next
          // return (the other parity's counters, its tables to EMPTY)
          const int q = par ^ 1;
          const bool prep = !multi() && compact && allow_prep;
          const int64_t pw = prep ? (int64_t)dirtyC[q] : 0;
          const auto ts0 = std::chrono::steady_clock::now();
          if (merge) {
            // one rank: the split and the return's first levels in one launch
            const int gm = (int)std::max<int64_t>(16, std::min<int64_t>(kExpandWG, (std::max(nF, last_work) + 3) / 4));
            fx_split_expand_kernel<<<std::max(gm, grid_for(pw)), 256, 0, st>>>(
                F, nF, w, use_prep ? dWin : nullptr, tb, epoch, dCtr, prep ? dCtrBase + q : nullptr,
                q ? tagR2 : tagR, q ? tagV2 : tagV, pw, hop2, hops);
          } else {
            fx_split_kernel<<<std::max(grid_for(nF), grid_for(pw)), 256, 0, st>>>(
                F, nF, w, use_prep ? dWin : nullptr, tb, epoch, dCtr, prep ? dCtrBase + q : nullptr,
                q ? tagR2 : tagR, q ? tagV2 : tagV, pw);
          }
          FX_TRY(hipGetLastError());
          if (hostprof) {
            hp_split += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - ts0).count();
            hp_nsplit++;
          }
          if (prep) {
            dirtyC[q] = 0;
            prepped[q] = true;
          }
        }
        const int g = (int)std::max<int64_t>(16, std::min<int64_t>(kExpandWG, (std::max(nF, last_work) + 3) / 4));
        // the merged launch may have expanded the whole return: its first
        // batch may launch no level (spec_levels 0, then the count of V level 0)
        if (!merge || small || !nF) spec_levels = std::max(spec_levels, 1);
        for (int batch = 0; !done; batch++) {
          // ctr->andmask is the AND of R as it grows (the insert and every
          // level add theirs): no pass over R unless counted classes need
          // their minima, which that pass recomputes whole
          if (n_cls && (small || batch)) {  // the reset set them for a first batch
            FX_TRY(hipMemsetAsync(dCtr->andm, 0xFF, sizeof(dCtr->andm), st));
            FX_TRY(hipMemsetAsync(dCtr->cmin, 0xFF, sizeof(dCtr->cmin), st));
          }
          const auto te0 = std::chrono::steady_clock::now();
          for (int l = 0; l < spec_levels; l++, k++)
            fx_expand_kernel<<<g, 256, 0, st>>>(dWin, tabs(tlog, compact, k), epoch, dCtr, k, -1, -1,
                                                nullptr, 0, hop2, hops);
          if (hostprof) {
            hp_expand += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - te0).count();
            hp_nexpand += spec_levels;
          }
          if (n_cls) {
            const int ga = grid_for((int64_t)std::max(nF, last_work));
            fx_and_kernel<<<ga, 256, 0, st>>>(Rl, &dCtr->nR, dCtr, dExp);
            fx_cmin_kernel<<<ga, 256, 0, st>>>(Rl, &dCtr->nR, dWin, dCtr);
          }
          FX_TRY(hipGetLastError());
          if (int er = sync_ctr()) return er;
          if (hCtr->tfull || hCtr->overflow ||
              (int64_t)(hCtr->nR + hCtr->nV + hCtr->cnt[k % 3]) > budget)
            break;
          if (hCtr->cnt[k % 3] == 0) break;  // the last level found nothing new
          spec_levels = std::min(std::max(1, spec_levels * 2), 64);
        }
        // levels this attempt expanded (a redone attempt's count too)
        const int64_t used = (int64_t)hCtr->levels - levels_seen;
        levels_seen = (int64_t)hCtr->levels;
        levels_total += used;
        const bool my_tfull = hCtr->tfull != 0;
        const bool my_redo = my_tfull && tlog < tlog_full;
        const bool my_over = my_tfull || hCtr->overflow ||
                             (int64_t)(hCtr->nR + hCtr->nV + hCtr->cnt[k % 3]) > budget;
        if (multi()) {
          // A probe chain's length depends on the order of the atomic inserts,
          // so ranks expanding the same replicated frontier may disagree on
          // tfull: agree, so that every rank takes the same branch (and makes
          // the same collectives) next.  Full at full size anywhere: :unknown.
          int64_t v[3] = {my_redo ? 1 : 0, my_tfull && !my_redo ? 1 : 0, my_over ? 1 : 0};
          FX_COLL(coll_allreduce(v, 3, LC_FX_SUM));
          if (!v[1] && v[0]) {
            if (my_redo) tlog = std::min(tlog + 2, tlog_full);
            stats.redos++;
            continue;
          }
          over = v[1] || v[2];
        } else {
          if (my_redo) {
            tlog = std::min(tlog + 2, tlog_full);
            stats.redos++;
            continue;
          }
          over = my_over;
        }
        // next return: as many speculative levels as this one needed, plus one
        // (merged launches: plus LC_FX_MERGE_PAD, default 0: none when the merged
        // launch finished the last return)
        spec_levels = merge_on ? (int)std::min<int64_t>(64, used + mpad)
                               : (int)std::max<int64_t>(spad > 0 ? 2 : 1, std::min<int64_t>(64, used + spad));
        const unsigned long long ex = hCtr->explored;
        explored_repl += (int64_t)(ex - explored_seen);
        explored_seen = ex;
        nRg = (int64_t)hCtr->nR;
        last_work = (int64_t)(hCtr->nR + hCtr->nV);
        if (timed) timeout = std::chrono::duration<double, std::milli>(
                                 std::chrono::steady_clock::now() - t0).count() > (double)opts.time_budget_ms;
        if (multi() && timed) {
          int64_t v[1] = {timeout ? 1 : 0};
          FX_COLL(coll_allreduce(v, 1, LC_FX_SUM));
          timeout = v[0] > 0;
        }
        break;
      }
      // partitioned: every level is chunks of (expand, exchange, insert)
      if (attempt == 0) stats.part_returns++;
      if (nF) {
        fx_insert_kernel<<<grid_for(nF), 256, 0, st>>>(F, nF, dWin, tb, epoch, dCtr);
        FX_TRY(hipGetLastError());
      }
      if (int er = sync_ctr()) return er;
      // level k: V list k % 3, n_k entries here; its successors become level
      // k + 1, whose count the host zeroes before the level starts
      int64_t k = 0, n_k = (int64_t)hCtr->cnt[0], v_done = 0, pos = 0;
      const int64_t chunk = (int64_t)(cand_cap / kW);
      FX_TRY(hipMemsetAsync(&dCtr->cnt[1], 0, sizeof(unsigned long long), st));
      for (;;) {
        const int64_t a = pos, b = std::min(n_k, pos + chunk);
        pos = b;
        if (int er = part_chunk(a, b, tabs(tlog, compact, k))) return er;
        if (int er = sync_ctr()) return er;
        if (timed) timeout = std::chrono::duration<double, std::milli>(
                                 std::chrono::steady_clock::now() - t0).count() > (double)opts.time_budget_ms;
        const int64_t n_next = (int64_t)hCtr->cnt[(k + 1) % 3];
        int64_t v[6] = {pos < n_k ? 1 : 0, n_next,
                        (int64_t)hCtr->nR + v_done + n_k + n_next, (int64_t)hCtr->overflow ? 1 : 0,
                        timeout ? 1 : 0, (int64_t)hCtr->tfull ? 1 : 0};
        FX_COLL(coll_allreduce(v, 6, LC_FX_SUM));
        if (v[5]) {  // some rank's table is too small: every rank redoes the return
          tfull = true;
          break;
        }
        if (v[3] || v[2] > budget) {
          over = true;
          break;
        }
        if (v[4]) {
          timeout = true;
          break;
        }
        if (v[0]) continue;  // some rank has more of this level
        stats.part_levels++;
        v_done += n_k;
        if (v[1] == 0) break;  // no rank found anything new
        k++;
        n_k = n_next;
        pos = 0;
        FX_TRY(hipMemsetAsync(&dCtr->cnt[(k + 1) % 3], 0, sizeof(unsigned long long), st));
      }
      const int64_t part_v = v_done;  // V entries of this return on this rank
      if (tfull) {
        // "full at full size" must be judged on the table this attempt used,
        // before it grows: a table grown to full size here has not been tried
        const bool at_full = tlog >= tlog_full;
        if (hCtr->tfull && !at_full) tlog = std::min(tlog + 2, tlog_full);
        int64_t v[1] = {hCtr->tfull && at_full ? 1 : 0};  // full size and still full
        FX_COLL(coll_allreduce(v, 1, LC_FX_SUM));
        if (!v[0]) {
          stats.redos++;
          continue;
        }
        over = true;
      }
      if (!over && !timeout) {
        fx_and_kernel<<<grid_for(nF), 256, 0, st>>>(Rl, &dCtr->nR, dCtr, dExp);
        if (n_cls) fx_cmin_kernel<<<grid_for(nF), 256, 0, st>>>(Rl, &dCtr->nR, dWin, dCtr);
        FX_TRY(hipGetLastError());
      }
      if (int er = sync_ctr()) return er;
      explored_part += (int64_t)(hCtr->explored - explored_seen);
      explored_seen = hCtr->explored;
      last_work = (int64_t)hCtr->nR + part_v;
      // global |R| and the global AND (bit b set everywhere <=> no rank lacks it)
      int64_t v[1 + kW];
      v[0] = (int64_t)hCtr->nR;
      for (int b = 0; b < kW; b++) v[1 + b] = ((hCtr->andmask >> b) & 1) ? 0 : 1;
      FX_COLL(coll_allreduce(v, 1 + kW, LC_FX_SUM));
      nRg = v[0];
      unsigned long long gand = 0;
      for (int b = 0; b < kW; b++)
        if (!v[1 + b]) gand |= 1ULL << b;
      hCtr->andmask = gand;
      if (n_cls && !over && !timeout) {
        // each class's smallest field over every rank's R: max of the negated
        // local minima (a rank with R empty contributes nothing)
        int64_t m[kMaxCls];
        for (int c = 0; c < n_cls; c++)
          m[c] = hCtr->cmin[c] == ~0ULL ? INT64_MIN : -(int64_t)hCtr->cmin[c];
        FX_COLL(coll_allreduce(m, n_cls, LC_FX_MAX));
        for (int c = 0; c < n_cls; c++)
          hCtr->cmin[c] = m[c] == INT64_MIN ? ~0ULL : (unsigned long long)(-m[c]);
      }
      break;
    }
    if (!multi()) par ^= 1;  // the next return takes the other counters and tables
    if (over) {
      result_unknown(res, LC_REASON_CONFIG_BUDGET);
      decided = true;
      break;
    }
    if (timeout) {
      result_unknown(res, LC_REASON_TIME_BUDGET);
      decided = true;
      break;
    }
    // F := R
    std::swap(F, Rl);
    nF = (int64_t)hCtr->nR;
    nFglobal = nRg;
    stats.max_local_frontier = std::max<int64_t>(stats.max_local_frontier, nF);
    if (!((reads >> sx) & 1)) vbase++;  // x, linearized in every configuration now
    occ &= ~xb;
    reads &= ~xb;
    kzob ^= w.s[sx].zob;
    for (int u = 0; u < kW; u++) before[u] &= ~xb;
    max_frontier = std::max(max_frontier, nFglobal);
    if (nFglobal == 0) {
      res->verdict = LC_INVALID;
      res->reason = LC_REASON_NONLINEARIZABLE;
      res->fail_op = x;
      res->fail_prefix_end = ox.ret;
      decided = true;
      break;
    }
    // LC_FX_DEBUG: the retirement AND kept incrementally (the insert and
    // every level AND the masks they put into R, one atomic per workgroup)
    // must equal the AND of R recomputed whole: a bit set that some
    // configuration lacks would retire an op not linearized everywhere
    if (debug && !multi() && nF) {
      std::vector<Cfg> hR((size_t)nF);
      FX_TRY(hipMemcpy(hR.data(), F, sizeof(Cfg) * (size_t)nF, hipMemcpyDeviceToHost));
      unsigned long long whole = ~0ULL;
      for (const Cfg &cf : hR) whole &= cf.mask;
      if (whole != hCtr->andmask) {
        err = "LC_FX_DEBUG: incremental retirement AND " + std::to_string(hCtr->andmask) +
              " != AND of R " + std::to_string(whole) + " at the return of record " +
              std::to_string(x);
        return -EIO;
      }
      fprintf(stderr, "fx and-check ok x=%d nR=%lld\n", (int)x, (long long)nF);
    }
    // retirement: ops linearized in every configuration free their slots
    const uint64_t all = occ & hCtr->andmask;
    if (debug)
      fprintf(stderr, "fx r%d ret x=%d slot=%d part=%d nF=%lld nFg=%lld nV=%llu expl=%llu and=%llx occ=%llx\n",
              rank, x, sx, (int)part, (long long)nF, (long long)nFglobal, hCtr->nV, hCtr->explored,
              hCtr->andmask, (unsigned long long)occ);
    if (all) {
      if (!multi()) {
        fclear |= all;  // applied by the next split
      } else if (nF) {
        fx_clear_kernel<<<grid_for(nF), 256, 0, st>>>(F, nF, all);
        FX_TRY(hipGetLastError());
      }
      for (int u = 0; u < kW; u++) {
        if (!((all >> u) & 1)) continue;
        slot_of[slot_op[u]] = -1;  // its return (if any) is now a no-op
        kzob ^= w.s[u].zob;
        if (!((reads >> u) & 1)) vbase++;
      }
      occ &= ~all;
      reads &= ~all;
      for (int u = 0; u < kW; u++) before[u] &= ~all;
    }
    // counted classes: members every configuration has linearized retire
    // (the fields shrink by as many: one rank lazily, at the next split —
    // fsub; several ranks now, as cbase grows with them for owner_of)
    uint64_t sub = 0;
    for (int c = 0; c < n_cls; c++) {
      const unsigned long long m = hCtr->cmin[c];
      if (m == 0 || m == ~0ULL) continue;
      Slot &cl = w.s[kClsLane0 + c];
      cls_base[c] += (int64_t)m;
      cl.zob -= m;
      sub += (uint64_t)m << cls_shift(cl.cls);
      vbase += (uint32_t)m;
    }
    if (sub && !multi()) {
      fsub += sub;
    } else if (sub && nF) {
      fx_sub_kernel<<<grid_for(nF), 256, 0, st>>>(F, nF, sub);
      FX_TRY(hipGetLastError());
    }
  }
  // every rank reports the same totals
  int64_t tot_part = explored_part;
  if (multi()) {
    int64_t v[1] = {explored_part};
    FX_COLL(coll_allreduce(v, 1, LC_FX_SUM));
    tot_part = v[0];
  }
  res->configs_explored = 1 + explored_repl + tot_part;
  res->max_frontier = max_frontier;
  FX_TRY(hipStreamSynchronize(st));
  stats.levels = levels_total + stats.part_levels;
  stats.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (hostprof) {
    fprintf(stderr, "fx hostprof: total %.2f ms, reports %lld, host between reports %.2f ms, waiting %.2f ms; "
            "split launches %lld %.2f ms, expand launches %lld %.2f ms\n",
            stats.total_ms, hp_syncs, hp_host * 1e-3, hp_wait * 1e-3, hp_nsplit, hp_split * 1e-3, hp_nexpand,
            hp_expand * 1e-3);
    hp_host = hp_wait = hp_split = hp_expand = 0;
    hp_syncs = hp_nsplit = hp_nexpand = 0;
  }
  if (qdbg_time) {
    fprintf(stderr, "fxq: returns %lld redos %lld launches %lld launch us %.1f sync us %.1f total ms %.2f\n",
            (long long)stats.returns, (long long)stats.redos, (long long)qt_n, qt_launch, qt_sync,
            stats.total_ms);
    fprintf(stderr, "fxq phases (G wave-cycles): split %.2f claim %.2f take %.2f drain %.2f [insert %.2f flush %.2f] wait %.2f\n",
            qt_ph[0] * 1e-9, qt_ph[1] * 1e-9, qt_ph[2] * 1e-9, qt_ph[3] * 1e-9, qt_ph[4] * 1e-9,
            qt_ph[5] * 1e-9, qt_ph[6] * 1e-9);
    for (double &v : qt_ph) v = 0;
    qt_launch = qt_sync = 0;
    qt_n = 0;
  }
  return 0;
}

}  // namespace

struct lc_fx {
  lc_fx_params params{};
  bool threads = false;         // several ranks of this process, one host thread each
  std::atomic<bool> broken{false};  // its RCCL communicators were aborted (failure, lc_fx_abort)
  std::mutex abort_mu;
  std::vector<Rank *> ranks;    // threads: all of them; else this process's one rank
  std::unique_ptr<Hub> hub;     // in-process transport (virtual ranks)
  std::vector<HubRank> hub_ranks;
  std::string err;
  lc_fx_stats stats{};
};

namespace {

void configure(Rank *r, const lc_fx_params *params) {
  if (params->part_above >= 0) r->part_above = params->part_above;
  r->repl_below = params->repl_below >= 0 ? params->repl_below : r->part_above / 4;
  r->table_log2 = (int)params->table_log2;
  r->force_wide = (params->flags & LC_FX_FLAG_WIDE_TABLES) != 0;
  r->xself = (params->flags & LC_FX_FLAG_EXCHANGE_SELF) != 0;
}

// Abort every RCCL communicator of the engine (once): collectives waiting on
// a rank that failed or hangs return, and the engine is unusable after.
void abort_comms(lc_fx *fx) {
  std::lock_guard<std::mutex> g(fx->abort_mu);
  for (Rank *r : fx->ranks)
    if (r->nc && r->nc->comm && !r->nc->aborted) {
      (void)r->nc->api->CommAbort(r->nc->comm);
      r->nc->aborted = true;
    }
  fx->broken = true;
}

int open_ranks(lc_fx *fx) {
  for (Rank *r : fx->ranks)
    if (int e = r->open()) {
      fx->err = r->err;
      return e;
    }
  return 0;
}

}  // namespace

extern "C" {

int lc_fx_open(const lc_fx_params *params, const lc_fx_transport *transport, lc_fx **out) {
  if (!params || !out) return -EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return -ENODEV;
  if (params->device < 0 || params->device >= ndev) return -ENODEV;
  int P = 1;
  if (transport) {
    if (transport->n_ranks < 1 || transport->n_ranks > 64 || transport->rank < 0 ||
        transport->rank >= transport->n_ranks || !transport->exchange_counts ||
        !transport->alltoallv || !transport->allreduce)
      return -EINVAL;
    P = transport->n_ranks;
  } else {
    P = std::max(1, params->virtual_ranks);
    if (P > 64) return -EINVAL;
  }
  lc_fx *fx = new lc_fx();
  fx->params = *params;
  if (!transport) {
    fx->threads = P > 1;
    fx->hub.reset(new Hub(P));
    fx->hub_ranks.resize(P);
  }
  const int nr = transport ? 1 : P;
  for (int i = 0; i < nr; i++) {
    Rank *r = new Rank();
    r->dev = params->device;
    r->P = P;
    if (transport) {
      r->tr = *transport;
      r->rank = transport->rank;
    } else {
      r->rank = i;
      fx->hub_ranks[i] = HubRank{fx->hub.get(), i};
      r->tr.user = &fx->hub_ranks[i];
      r->tr.rank = i;
      r->tr.n_ranks = P;
      r->tr.exchange_counts = hub_exchange_counts;
      r->tr.alltoallv = hub_alltoallv;
      r->tr.allreduce = hub_allreduce;
    }
    configure(r, params);
    fx->ranks.push_back(r);
  }
  if (int e = open_ranks(fx)) {
    lc_fx_close(fx);
    return e;
  }
  *out = fx;
  return 0;
}

int lc_fx_open_devices(const lc_fx_params *params, const int32_t *devices, int32_t n_devices,
                       lc_fx **out) {
  if (!params || !out || !devices || n_devices < 1 || n_devices > 64) return -EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return -ENODEV;
  for (int i = 0; i < n_devices; i++)
    if (devices[i] < 0 || devices[i] >= ndev) return -ENODEV;
  const RcclApi &api = rccl_api();
  if (!api.ok) return -ENOSYS;
  std::vector<ncclComm_t> comms((size_t)n_devices, nullptr);
  std::vector<int> devlist(devices, devices + n_devices);
  const ncclResult_t nr = api.CommInitAll(comms.data(), n_devices, devlist.data());
  if (nr != ncclSuccess) return nr == ncclInvalidUsage || nr == ncclInvalidArgument ? -EINVAL : -EIO;
  lc_fx *fx = new lc_fx();
  fx->params = *params;
  fx->threads = n_devices > 1;
  for (int i = 0; i < n_devices; i++) {
    Rank *r = new Rank();
    r->dev = devices[i];
    r->P = n_devices;
    r->rank = i;
    r->nc = new Nccl();
    r->nc->api = &api;
    r->nc->comm = comms[(size_t)i];
    configure(r, params);
    fx->ranks.push_back(r);
  }
  if (int e = open_ranks(fx)) {
    lc_fx_close(fx);
    return e;
  }
  *out = fx;
  return 0;
}

int lc_fx_rccl_unique_id(uint8_t *id) {
  if (!id) return -EINVAL;
  const RcclApi &api = rccl_api();
  if (!api.ok) return -ENOSYS;
  ncclUniqueId u;
  if (api.GetUniqueId(&u) != ncclSuccess) return -EIO;
  static_assert(sizeof(u) == LC_FX_RCCL_ID_BYTES, "ncclUniqueId size");
  std::memcpy(id, &u, sizeof u);
  return 0;
}

int lc_fx_open_rccl(const lc_fx_params *params, const uint8_t *id, int32_t rank, int32_t n_ranks,
                    lc_fx **out) {
  if (!params || !out || !id || n_ranks < 1 || n_ranks > 64 || rank < 0 || rank >= n_ranks)
    return -EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return -ENODEV;
  if (params->device < 0 || params->device >= ndev) return -ENODEV;
  const RcclApi &api = rccl_api();
  if (!api.ok) return -ENOSYS;
  if (hipSetDevice(params->device) != hipSuccess) return -EIO;
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof u);
  ncclComm_t comm = nullptr;
  if (api.CommInitRank(&comm, n_ranks, u, rank) != ncclSuccess) return -EIO;
  lc_fx *fx = new lc_fx();
  fx->params = *params;
  Rank *r = new Rank();
  r->dev = params->device;
  r->P = n_ranks;
  r->rank = rank;
  r->nc = new Nccl();
  r->nc->api = &api;
  r->nc->comm = comm;
  configure(r, params);
  fx->ranks.push_back(r);
  if (int e = open_ranks(fx)) {
    lc_fx_close(fx);
    return e;
  }
  *out = fx;
  return 0;
}

int lc_fx_check(lc_fx *fx, const lc_op *ops, int64_t n, const lc_opts *opts, lc_key_result *out) {
  if (!fx || !out || n < 0 || (n > 0 && !ops)) return -EINVAL;
  if (fx->broken) {
    fx->err = "the engine's RCCL communicators were aborted after an earlier failure";
    return -EIO;
  }
  if (!fx->threads) {
    Rank *r = fx->ranks[0];
    (void)hipSetDevice(r->dev);
    const int e = r->check(ops, n, opts, out);
    fx->stats = r->stats;
    if (e) fx->err = r->err;
    return e;
  }
  const int P = (int)fx->ranks.size();
  if (fx->hub) {
    std::lock_guard<std::mutex> g(fx->abort_mu);
    fx->hub.reset(new Hub(P));
    for (int i = 0; i < P; i++) fx->hub_ranks[i].hub = fx->hub.get();
  }
  std::vector<lc_key_result> res(P);
  std::vector<int> rc(P, 0);
  std::vector<std::thread> th;
  for (int i = 0; i < P; i++)
    th.emplace_back([&, i] {
      (void)hipSetDevice(fx->ranks[i]->dev);
      rc[i] = fx->ranks[i]->check(ops, n, opts, &res[i]);
      if (!rc[i]) return;
      if (fx->hub) {
        std::lock_guard<std::mutex> g(fx->abort_mu);
        fx->hub->abort();
      } else {
        // the other ranks may be waiting in a collective that will never
        // complete: abort every communicator (RCCL's kernels then exit)
        abort_comms(fx);
      }
    });
  for (auto &t : th) t.join();
  for (int i = 0; i < P; i++)
    if (rc[i] && rc[i] != -ECANCELED) {
      fx->err = fx->ranks[i]->err;
      return rc[i];
    }
  for (int i = 0; i < P; i++)
    if (rc[i]) {
      fx->err = fx->ranks[i]->err;
      return rc[i];
    }
  for (int i = 1; i < P; i++)
    if (std::memcmp(&res[i], &res[0], sizeof(lc_key_result)) != 0) {
      fx->err = "ranks disagree on the result";
      return -EPROTO;
    }
  *out = res[0];
  fx->stats = fx->ranks[0]->stats;
  return 0;
}

void lc_fx_abort(lc_fx *fx) {
  if (!fx) return;
  {
    std::lock_guard<std::mutex> g(fx->abort_mu);
    if (fx->hub) fx->hub->abort();
  }
  bool rccl = false;
  for (Rank *r : fx->ranks) rccl |= r->nc != nullptr;
  if (rccl) abort_comms(fx);
}

int lc_fx_frontier(lc_fx *fx, const lc_op *ops, int64_t n, const lc_opts *opts, int64_t stop_op,
                   lc_fx_config *out, int32_t max, int32_t *n_out) {
  if (!fx || !n_out || n < 0 || (n > 0 && !ops) || max < 0 || (max > 0 && !out)) return -EINVAL;
  *n_out = 0;
  if (fx->threads || fx->ranks[0]->multi()) {
    fx->err = "lc_fx_frontier: a one-rank engine only (the frontier is partitioned otherwise)";
    return -EINVAL;
  }
  if (stop_op < 0 || stop_op >= n || ops[stop_op].ret == LC_INF) {
    fx->err = "lc_fx_frontier: stop_op must be an op of the key that returns";
    return -EINVAL;
  }
  Rank *r = fx->ranks[0];
  (void)hipSetDevice(r->dev);
  r->stop_op = stop_op;
  r->dump = out;
  r->dump_max = max;
  r->dump_n = 0;
  lc_key_result res;
  const int e = r->check(ops, n, opts, &res);
  r->stop_op = -1;
  r->dump = nullptr;
  if (e) {
    fx->err = r->err;
    return e;
  }
  *n_out = r->dump_n;
  return 0;
}

int lc_fx_last_stats(lc_fx *fx, lc_fx_stats *out) {
  if (!fx || !out) return -EINVAL;
  *out = fx->stats;
  return 0;
}

const char *lc_fx_last_error(lc_fx *fx) { return fx ? fx->err.c_str() : "null lc_fx"; }

void lc_fx_close(lc_fx *fx) {
  if (!fx) return;
  for (Rank *r : fx->ranks) {
    (void)hipSetDevice(r->dev);
    delete r;
  }
  delete fx;
}

}  // extern "C"
