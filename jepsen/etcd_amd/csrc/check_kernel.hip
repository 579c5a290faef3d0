// check_kernel.hip — batched per-key linearizability search for the
// VersionedRegister model on CDNA4 (gfx950).
//
// Reference semantics: the model step is
//   /root/reference/src/jepsen/etcd/register.clj:59-96
// and the search replaces knossos's JIT-linear analyzer invoked through
// (checker/linearizable {:model (->VersionedRegister 0 nil)}) at
// register.clj:110-111, once per independent key (register.clj:108).
//
// Mapping to the hardware:
//  * one wavefront owns one key; a 256-thread workgroup runs 4 independent keys;
//  * LANE t = WINDOW SLOT t: the record of the t-th open call (called, not yet
//    returned, or crashed) lives in lane t's VGPRs, so "which pending ops may
//    the model step next from state s" is ONE vector compare + __ballot over
//    all 64 open calls (wave-level candidate compaction);
//  * a configuration (linearized-slot bitmask, (version, value)) is 16 bytes and
//    wave-uniform.  While the frontier holds ONE configuration (the common case:
//    :ok mutations are pinned by version, register.clj:64-75) it lives in SGPRs
//    and a return's expansion is a chain walk of ballots; a larger frontier
//    lives in LDS (3 regions x kLdsCap configs per wave), and a key that
//    outgrows LDS is re-run from HBM hash tables (hbm_tier_kernel);
//  * the key's records are streamed from HBM 64 at a time (one 48-byte record
//    per lane, double-buffered), and read out by v_readlane as calls happen;
//  * the next event is min(next call, min over open slots of ret): a 64-lane
//    DPP min to an SGPR, so no per-key event sort is ever built.
//
// Search (Lowe's just-in-time linearization, as knossos.linear) with one exact,
// model-specific reduction — EAGER READ CLOSURE: a read (a no-op on the state,
// register.clj:84-96) that is pending and legal in a configuration is
// linearized immediately.  (s, L+{r}) dominates (s, L): any continuation of the
// latter linearizes r at some state where it is legal, and deleting that step
// leaves every other step unchanged.  So the frontier is empty at exactly the
// same returns as knossos's, verdicts and counterexample prefixes are
// unchanged, and the 2^k subsets of concurrent reads never materialise.
#include <algorithm>
#include <atomic>
#include <climits>
#include <type_traits>

#include "../../../include/lincheck_fx.h"
#include "kernels.h"
#include "records.h"
#include "wave.h"
#include "gapmatch.h"

namespace lcdev {
namespace {

#ifdef LC_FG_PROF  // dev only: per-phase clocks of the fused pass, summed over keys
__device__ unsigned long long g_fgp[8];
__device__ unsigned int g_fgdone;
#define FGP_T(i) uint64_t fgp_t##i = __builtin_amdgcn_s_memtime()
#define FGP_ADD(i, a, b) if (threadIdx.x == 0) atomicAdd(&g_fgp[i], (unsigned long long)(fgp_t##b - fgp_t##a))
#else
#define FGP_T(i)
#define FGP_ADD(i, a, b)
#endif

#ifdef LC_FAST_PROF  // dev only: per-phase clocks of fast_tier_kernel (thread 0), summed over keys
__device__ unsigned long long g_fp[8];
__device__ unsigned int g_fpdone;
#define FP_T(i) const uint64_t fp_t##i = __builtin_amdgcn_s_memtime()
#else
#define FP_T(i)
#endif

#ifdef LC_COOP_PROF
// Dev only (tools/build_variants.sh NAME -DLC_COOP_PROF): wave 0's shader
// clocks per cooperative workgroup, by phase of its returns (see
// CoopProf); launch_hbm_coop prints them after the launch
constexpr int kCpN = 30;
__device__ unsigned long long g_cp[4096][2][kCpN];  // waves 0 and 1
#define CP_NOW() __builtin_amdgcn_s_memtime()
#endif
#ifdef HBM_PROFILE
// Dev only (tools/build_variants.sh NAME -DHBM_PROFILE): per cooperative
// return, by log2 of its larger set: returns, device ticks (100 MHz), LDS-
// mode returns, configurations explored; printed by the last workgroup.
__device__ unsigned long long g_hhist[20][4];
// per workgroup: ticks in LDS-mode returns, in HBM-mode returns (incl. failed LDS attempts), whole keys
__device__ unsigned long long g_hwg[4096][3];
__device__ unsigned int g_hdone;
#endif

struct Cfg {
  uint64_t mask;  // bit t: the op in window slot t is linearized
  uint64_t sv;    // (uint32 version << 32) | uint32 value-id (NIL = 0xFFFFFFFF)
};

__device__ __forceinline__ uint64_t pack_sv(int32_t ver, int32_t val) {
  return ((uint64_t)(uint32_t)ver << 32) | (uint32_t)val;
}
__device__ __forceinline__ int32_t sv_ver(uint64_t sv) { return (int32_t)(sv >> 32); }
__device__ __forceinline__ int32_t sv_val(uint64_t sv) { return (int32_t)(uint32_t)sv; }

__device__ __forceinline__ int rl32(int v, int l) {
  return __builtin_amdgcn_readlane(v, l);
}
__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}
// Bitwise AND of a 64-bit value over the 64 lanes (wave-uniform result).
__device__ __forceinline__ uint32_t wave_and_u32(uint32_t v) {
  v &= (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false);
  v &= (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false);
  v &= (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x141, 0xF, 0xF, false);
  v &= (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x140, 0xF, 0xF, false);
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) &
         (uint32_t)__builtin_amdgcn_readlane((int)v, 16) &
         (uint32_t)__builtin_amdgcn_readlane((int)v, 32) &
         (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}
__device__ __forceinline__ uint64_t wave_and_u64(uint64_t v) {
  return ((uint64_t)wave_and_u32((uint32_t)(v >> 32)) << 32) | wave_and_u32((uint32_t)v);
}

__device__ __forceinline__ bool pre_ok(int nv, int nvm, int nl, int nlm, int ver, int val) {
  return (((ver ^ nv) & nvm) | ((val ^ nl) & nlm)) == 0;
}

struct KeyOut {
  int verdict, reason;
  int64_t fail_op, fail_end, explored, max_frontier;
};

// ---------------------------------------------------------------- stores
// A Store holds three configuration regions (roles rotate: frontier F,
// results R, worklist/visited W) and deduplicating insertion into the R and W
// roles.  All member functions are called by the whole wave with uniform
// arguments unless named *_lane.

enum { ROLE_R = 0, ROLE_W = 1 };

struct LdsStore {
  Cfg *base;  // 3 regions of cap configurations, contiguous
  static constexpr int cap = kLdsCap;
  __device__ __forceinline__ Cfg *reg(int r) const { return base + r * cap; }
  __device__ __forceinline__ Cfg get(int r, int j) const { return reg(r)[j]; }
  __device__ __forceinline__ void set_mask_lane(int r, int j, uint64_t m) {
    reg(r)[j].mask = m;
  }
  __device__ __forceinline__ void begin_return() {}
  // Lane-parallel insertion of configurations known to be distinct.
  __device__ __forceinline__ void add_unique_lane(int, int r, int j, const Cfg &c) {
    reg(r)[j] = c;
  }
  // Returns 1 inserted, 0 duplicate, -1 full.
  __device__ __forceinline__ int insert(int, int r, int &n, uint64_t m,
                                        uint64_t sv, int lane) {
    const Cfg *R = reg(r);
    for (int j0 = 0; j0 < n; j0 += kWave) {
      const int j = j0 + lane;
      bool eq = false;
      if (j < n) {
        const Cfg c = R[j];
        eq = (c.mask == m) & (c.sv == sv);
      }
      if (__ballot(eq)) return 0;
    }
    if (n >= cap) return -1;
    if (lane == 0) reg(r)[n] = Cfg{m, sv};
    n++;
    return 1;
  }
};

// HBM store: regions are global arrays of `cap` configurations; R and W each
// have an open-addressed table of 2*cap entries in 8-entry (128-byte) buckets,
// valid when their epoch tag equals the current return's epoch, so a table is
// "cleared" by bumping the epoch.  One wave owns one workspace.  Probing is
// linear from the start of the hashed bucket, whole buckets at a time.
// Per-return copy of the window's slots in LDS for the cooperative tier's
// worker waves (each loads slot `lane` into registers and tests slots with
// ballots / v_readlane, see legal_by_state).
struct SlotLds {
  int4 pre[kWave];      // (nv, nvm, nl, nlm)
  int val[kWave];
  uint64_t pbit[kWave];
};

// Cooperative HBM tier: the waves of one workgroup expand one key's
// frontier together.  Wave 0 runs the event loop (check_key); at a return on
// the general path it publishes the expansion here and every wave runs
// coop_expand (level-synchronous BFS: a level's worklist range is fixed,
// batches of 64 are claimed with an LDS counter, appends are reserved with
// LDS atomics, barriers between levels).
enum { kCoopExpand = 0, kCoopExit = 1 };
constexpr int kVTab = 16;  // (LDS: four 4-wave workgroups per CU leave ~170 bytes each)
constexpr uint32_t kBusy = 0x80000000u;  // table tag: claimed, configuration being written
struct CoopShared {
  int cmd;
  int rF, rR, rW, nF;
  uint64_t bs, muts, reads, ordered;  // ordered: slots with class predecessors (pbit)
  uint32_t epoch, tmask;
  union {  // set sizes; a round's appends to both reserve with one atomic
    struct { int nR, nW; };
    unsigned long long nRW;
  };
  int head, lo, hi, go, status;
  unsigned long long qword;  // LDS work queue: claimed head (low), expanding waves (high)
  int lds;  // this attempt keeps its tables and sets in LDS (CoopTab)
  uint32_t lepoch;  // its LDS epoch (8 bits)
  int kw;           // LDS mode: W's versions are kw + popc(mask & muts) (set by the split)
  int lclear;       // the LDS epoch wrapped: clear the tags first
  unsigned long long explored;
  long long budget;
  uint64_t fclear, fclose;  // F's pending updates (CoopStore), applied by the split
  unsigned long long rand;  // AND of R's masks (every wave ANDs in what it adds)
  SlotLds slots;
  // the slots legal at value id v - 1 whatever the version, for v < kVTab
  // (used when no pending slot constrains the version: version-less models)
  uint64_t vlegal[kVTab];
  int vt;  // vlegal holds this return's slots (no pending slot constrains the version)
};

struct HbmStore {
  static constexpr int kLT = 0;  // no LDS tables (CoopStore has them)
  CoopShared *coop = nullptr;  // set in the cooperative kernel
  int nwaves = 1;
  Cfg *base;      // 3 regions of cap configurations, contiguous
  Cfg *tabs;      // 2 tables (roles R, W) of 2*cap entries
  uint32_t *tags; // 2 tag arrays of 2*cap
  int cap;         // configurations per region
  uint32_t tmask;  // table entries - 1 (power of two, >= 7), this return's size
  uint32_t tmask_full;  // the workspace's table size - 1 (2 * cap entries)
  int hint = 0;    // largest R / W set of this key's returns so far
  uint32_t epoch;
#ifdef LC_COOP_PROF
  // [0] start barrier [1] split [2] split barrier [3] queue [4] end barrier
  // (LDS-mode returns), [5] LDS-mode returns, [6] all cooperative returns'
  // clocks, [7] whole keys, [8] cooperative returns, [9] HBM-mode ones,
  // [10] keys; LDS-mode queue phase: [11] batches [12] successor rounds
  // [13] queue-empty sleeps [14] clocks claiming [15] clocks waiting for
  // ready flags [16] clocks computing candidates [17] clocks in rounds;
  // event loop: [18] clocks in calls [19] in single-configuration returns
  // [20] after cooperative returns [21] calls [22] single returns;
  // ts: this return's marks
  uint64_t cp[30] = {0};
  uint64_t ts[6];
#endif
  // Table size of a return (adaptive, round 2).  The sets of one return are
  // usually far smaller than the workspace's capacity, and a table sized for
  // the capacity spreads them over 512 KB per role: every probe missed L2
  // and the Infinity Cache (~2 GB of tables over 1,000 keys).  A return
  // starts with 4x the larger of its frontier and the key's largest set so
  // far (at least `floor` entries); a role that fills past `lim` aborts the
  // return, which is redone with a 4x table (the expansion is deterministic
  // up to order, so R, the explored count and the verdict are unchanged).
  __device__ __forceinline__ uint32_t pick_tmask(int nF, uint32_t floor) const {
    const uint32_t need = (uint32_t)max(4 * max(nF, hint), (int)floor);
    uint32_t t = 8;
    while (t < need && t <= tmask_full) t <<= 1;
    return min(t - 1, tmask_full);
  }
  __device__ __forceinline__ uint32_t grow_tmask() const {
    return min(((tmask + 1) << 2) - 1, tmask_full);
  }
  // Entries a role may hold before the return aborts: half the table less
  // one round of inserts of every wave (each wave checks after its round),
  // so a probe always finds a free entry; the full table holds `cap`.
  __device__ __forceinline__ int lim(int nwaves) const {
    return tmask == tmask_full ? cap : min(cap, (int)((tmask + 1) / 2) - kWave * nwaves);
  }
  __device__ __forceinline__ Cfg *reg(int r) const { return base + (size_t)r * cap; }
  __device__ __forceinline__ Cfg *tab(int role) const { return tabs + (size_t)role * (tmask + 1); }
  __device__ __forceinline__ uint32_t *tag(int role) const { return tags + (size_t)role * (tmask + 1); }
  __device__ __forceinline__ Cfg get(int r, int j) const { return reg(r)[j]; }
  __device__ __forceinline__ void set_mask_lane(int r, int j, uint64_t m) {
    reg(r)[j].mask = m;
  }
  __device__ __forceinline__ void begin_return() { epoch++; }
  __device__ __forceinline__ static uint32_t hash(uint64_t m, uint64_t sv) {
    uint64_t h = m * 0x9E3779B97F4A7C15ULL ^ (sv + 0x632BE59BD9B4E019ULL);
    h ^= h >> 29;
    h *= 0xBF58476D1CE4E5B9ULL;
    h ^= h >> 32;
    return (uint32_t)h;
  }
  // Lane-parallel: each active lane inserts its own distinct config into the
  // role's table, claiming the first free entry at or after its bucket start
  // with atomicCAS (lanes of one wave may race for one bucket), and stores it
  // at region index j.
  __device__ __forceinline__ void add_unique_lane(int role, int r, int j,
                                                  const Cfg &c) {
    reg(r)[j] = c;
    uint32_t h = (hash(c.mask, c.sv) & tmask) & ~7u;
    for (;;) {
      const uint32_t old = tag(role)[h];
      if (old != epoch) {
        if (atomicCAS(&tag(role)[h], old, epoch) == old) {
          tab(role)[h] = c;
          return;
        }
        continue;
      }
      h = (h + 1) & tmask;
    }
  }
  // Lane-parallel dedup insert: every lane with `want` inserts its own c
  // into table `role`, probing linearly from its bucket start (as
  // add_unique_lane and insert do).  In lock-step rounds: read the entry's
  // tag; a stale tag is claimed with atomicCAS (one lane of a racing set
  // wins and writes the configuration), a live one is compared.  A lane
  // that lost a race re-reads the same entry next round, after the winner's
  // store has been fenced, so equal configurations inserted together are
  // kept once.  Returns 1 (inserted), 0 (already there), per lane.
  // (role may differ per lane: the R and W inserts of a round run together,
  // so a round costs one chain of dependent table round trips, not two)
  __device__ __forceinline__ int insert_lanes(int role, const Cfg &c, bool want) {
    uint32_t h = (hash(c.mask, c.sv) & tmask) & ~7u;
    int res = 0;
    bool pend = want;
    while (__ballot(pend)) {
      if (pend) {
        const uint32_t old = tag(role)[h];
        if (old != epoch) {
          if (atomicCAS(&tag(role)[h], old, epoch) == old) {
            tab(role)[h] = c;
            res = 1;
            pend = false;
          }
        } else {
          const Cfg e = tab(role)[h];
          if (e.mask == c.mask && e.sv == c.sv)
            pend = false;  // already there
          else
            h = (h + 1) & tmask;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    }
    return res;
  }
  // Cross-wave variants (cooperative tier): a claimed entry is tagged
  // epoch|kBusy until its configuration is stored, then released as epoch;
  // a lane that meets a busy entry retries it next round.
  __device__ __forceinline__ void claim_unique_lane(int role, int r, int j, const Cfg &c) {
    reg(r)[j] = c;
    uint32_t h = (hash(c.mask, c.sv) & tmask) & ~7u;
    for (;;) {
      const uint32_t old = __hip_atomic_load(&tag(role)[h], __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_WORKGROUP);
      if ((old & ~kBusy) != epoch) {
        if (atomicCAS(&tag(role)[h], old, epoch | kBusy) == old) {
          tab(role)[h] = c;
          __hip_atomic_store(&tag(role)[h], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          return;
        }
        continue;
      }
      h = (h + 1) & tmask;
    }
  }
  __device__ __forceinline__ int insert_lanes_coop(int role, const Cfg &c, bool want) {  // (role per lane)
    uint32_t h = (hash(c.mask, c.sv) & tmask) & ~7u;
    int res = 0;
    bool pend = want;
    while (__ballot(pend)) {
      if (pend) {
        const uint32_t t = __hip_atomic_load(&tag(role)[h], __ATOMIC_ACQUIRE,
                                             __HIP_MEMORY_SCOPE_WORKGROUP);
        if (t == epoch) {
          const Cfg e = tab(role)[h];
          if (e.mask == c.mask && e.sv == c.sv)
            pend = false;  // already there
          else
            h = (h + 1) & tmask;
        } else if (t != (epoch | kBusy)) {  // stale: claim it
          if (atomicCAS(&tag(role)[h], t, epoch | kBusy) == t) {
            tab(role)[h] = c;
            __hip_atomic_store(&tag(role)[h], epoch, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
            res = 1;
            pend = false;
          }
        }  // busy: being written by another lane, retry
      }
    }
    return res;
  }
  // Wave-uniform dedup insert: probe one 128-byte bucket (8 lanes x 16 B)
  // per step.
  __device__ __forceinline__ int insert(int role, int r, int &n, uint64_t m,
                                        uint64_t sv, int lane) {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    uint32_t b = (hash(m, sv) & tmask) & ~7u;
    const int sub = lane & 7;
    for (uint32_t probes = 0; probes <= tmask; probes += 8) {
      bool live = false, eq = false;
      if (lane < 8) {
        live = tag(role)[b + sub] == epoch;
        if (live) {
          const Cfg c = tab(role)[b + sub];
          eq = (c.mask == m) & (c.sv == sv);
        }
      }
      if (__ballot(eq)) return 0;
      const uint64_t free_m = __ballot(lane < 8 && !live);
      if (free_m) {
        if (n >= cap) return -1;
        const int slot = __builtin_ctzll(free_m);
        if (lane == slot) {
          tag(role)[b + slot] = epoch;
          tab(role)[b + slot] = Cfg{m, sv};
        }
        if (lane == 0) reg(r)[n] = Cfg{m, sv};
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        n++;
        return 1;
      }
      b = (b + 8) & tmask;
    }
    return -1;
  }
};

// LDS tables of the cooperative tier (round 2).  Most returns of a key on
// the HBM tiers have small R / W sets (model leg: 75 configurations on
// average) but many BFS levels, and each level's inserts are a chain of
// dependent table round trips: in HBM (tag load, CAS, entry store, release)
// one probe took ~1.4 us.  A return whose frontier fits runs its expansion
// with both tables and both sets in LDS (R is also appended to the global
// region the event loop reads); one whose sets outgrow the pool is redone with
// the HBM tables (status -3, as for the adaptive HBM size), so R, the
// explored count and the verdict do not depend on it.
// Round 6: both roles share one table and one pool of set entries — R
// takes pool slots from the bottom, W from the top — so a return fits while
// nR + nW fits the pool, whatever its split (the returns that outgrew the
// per-role sets had one set just past the limit and the other far below).
// A table entry is 4 bytes, (epoch << 16) | (role << 15) | index into the
// role's set; the pool holds 12-byte configurations plus a 1-byte ready flag
// (CoopTab): 1,688 in a 4-wave workgroup's 40 KB (four per CU), 3,456 in an
// 8- or 16-wave one's 80 KB.
#ifndef LC_LEPOCH_MASK
#define LC_LEPOCH_MASK 0xFFu  // (8 bits: wrdy; a dev build with 0x3 wraps every 3 returns)
#endif
constexpr uint32_t kLepochMask = LC_LEPOCH_MASK;
constexpr int kSpinMax = 1 << 22;       // queue waits (s_sleep 1 each) before giving up
constexpr uint32_t kIdxBusy = 0xFFFFu;  // claimed, index not yet published
constexpr uint32_t kIdxOvf = 0xFFFEu;   // claimed past the pool (the return is redone)
template <int LT>
struct CoopTab {
  // pool entries: 13 B each (below), the table (2 * LT entries) at <= 42 %
  // load: 1,688 in 38 KB (4-wave: 40 fewer than the load allows, for scr),
  // 3,456 in 78 KB (8- and 16-wave)
  static constexpr int kPool = LT * 27 / 32 - (LT < 4096 ? 40 : 0);
  static constexpr int kScrWaves = LT < 4096 ? 4 : 16;
  static_assert(kPool < 0x7FFE, "set index must fit 15 bits");
  uint32_t tag[2 * LT];     // (epoch << 16) | (role << 15) | index
  // R and W of this return as (linearized set, value): within one return and
  // role the version follows from the set (every configuration has freed the
  // same mutation slots), so it is not stored; W's is kw + popc(mask & muts).
  // R's index i is pool slot i, W's is kPool - 1 - i
  uint64_t smask[kPool];
  int32_t sval[kPool];
  uint8_t wrdy[kPool];      // W entry i written (its epoch): the work queue's readiness
  // per wave, a round's successors: (source lane << 6) | slot (coop_expand)
  uint16_t scr[kScrWaves][kWave];
};
template <int LT>
__device__ __forceinline__ int pool_slot(int role, int ix) {
  return role == ROLE_R ? ix : CoopTab<LT>::kPool - 1 - ix;
}
// a configuration's table position: R and W probe apart
__device__ __forceinline__ uint32_t pool_hash(const Cfg &c, int role) {
  return HbmStore::hash(c.mask, c.sv ^ ((uint64_t)role << 63));
}
template <int LT>
__device__ __forceinline__ CoopTab<LT> &coop_tab() {
  __shared__ CoopTab<LT> t;
  return t;
}
template <int LT>
struct CoopStore : HbmStore {
  static constexpr int kLT = LT;
  int last = 0;           // the previous return's larger set
  int lsum = 0;           // and its nR + nW
  uint32_t lepoch = 0;    // LDS table epoch (8 bits; 0 is never current)
  // The frontier's masks in the global region are brought up to date by the
  // next return's split, not by wave 0 as the events come (round 6): slots
  // retired since the last return (cleared from every configuration, before)
  // and reads called since (each linearized where legal); and the AND of
  // the last return's R, kept by the waves as they fill it
  uint64_t fclear = 0, fclose = 0, rand = ~0ull;
  // lane v < kVTab: the slots legal at value id v - 1 whatever the version
  // (kept as slots are taken, check_key; published as C.vlegal)
  uint64_t vleg = 0;
};
// (check_key: the cooperative stores defer their frontier updates)
template <class S, class = void>
struct DeferF {
  static constexpr bool value = false;
};
template <class S>
struct DeferF<S, std::void_t<decltype(S::kLT)>> {
  static constexpr bool value = S::kLT > 0;
};

// Wave priority of wave 0 (s_setprio): the event loop between returns is
// each key's serial path, so it issues ahead of other workgroups' expansion
// waves on its SIMD (model_leg 9.22 -> 8.88 ms; raising the expansion
// waves' too, or dropping wave 0's during its share of the expansion,
// measured slower: profiles/r06/model_prio_ab.txt)
#ifndef LC_COOP_PRIO
#define LC_COOP_PRIO 3
#endif
// Sleep of a wave whose work queue is empty while others expand, or whose
// claimed entries are not yet written (s_sleep units of 64 clocks)
#ifndef LC_COOP_SLEEP
#define LC_COOP_SLEEP 1
#endif
// LDS-only fences: the tables are workgroup-private, so publishing an entry
// waits for LDS (lgkmcnt) only, not for the wave's global R appends.
__device__ __forceinline__ void lds_release() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
}
__device__ __forceinline__ void lds_acquire() {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
__device__ __forceinline__ void lds_barrier() {
  lds_release();
  __builtin_amdgcn_s_barrier();
  lds_acquire();
}
__device__ __forceinline__ uint32_t lds_tag_load(uint32_t *p) {
  const uint32_t t = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  lds_acquire();
  return t;
}
__device__ __forceinline__ void lds_tag_publish(uint32_t *p, uint32_t v) {
  lds_release();
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Lane-parallel dedup insert into the LDS tables (each lane its own role):
// a stale entry is claimed as (epoch, kIdxBusy) with CAS; the lanes that won
// this round reserve their set indices together (one packed atomic on
// C.nRW), store the configuration (R also to the global region rR) and
// publish (epoch, index).  A busy entry is re-read next round; its owner
// publishes within the round it claimed it, so no wave waits on another
// wave's unfinished loop.  A lane that probed LT/4 entries, or whose index
// is past the pool, sets ovf.  Returns 1 (inserted) or 0 (already there).
template <int LT>
__device__ __forceinline__ int lds_insert_lanes(CoopTab<LT> &T, CoopShared &C, HbmStore &st,
                                                int rR, int role, const Cfg &c, bool want,
                                                uint32_t eb, bool &ovf, int lane) {
  constexpr int P = CoopTab<LT>::kPool;
  constexpr uint32_t TM = 2 * LT - 1;
  const uint32_t rbit = (uint32_t)role << 15;
  uint32_t h = pool_hash(c, role) & TM;
  int res = 0, probes = 0;
  bool pend = want;
  while (__ballot(pend)) {
    bool won = false;
    if (pend) {
      const uint32_t t = lds_tag_load(&T.tag[h]);
      if ((t & 0xFFFF0000u) == eb) {
        const uint32_t lo = t & 0xFFFFu;
        if (lo < kIdxOvf) {
          // (mask, value) decide: the version follows from the mask (CoopTab)
          const int sl = pool_slot<LT>(role, (int)(lo & 0x7FFFu));
          if ((lo & 0x8000u) == rbit && T.smask[sl] == c.mask && T.sval[sl] == sv_val(c.sv)) {
            pend = false;  // already there
          } else {
            h = (h + 1) & TM;
            if (++probes >= LT / 2) {
              ovf = true;
              pend = false;
            }
          }
        } else if (lo == kIdxOvf) {
          ovf = true;
          pend = false;
        }  // kIdxBusy: re-read next round
      } else {
        won = atomicCAS(&T.tag[h], t, eb | kIdxBusy) == t;
      }
    }
    const uint64_t wR = __ballot(won && role == ROLE_R), wW = __ballot(won && role == ROLE_W);
    if (wR | wW) {
      unsigned long long a = 0;
      if (lane == 0)
        a = atomicAdd(&C.nRW, (unsigned long long)__popcll(wR) | ((unsigned long long)__popcll(wW) << 32));
      const int aR = uni((int)a), aW = uni((int)(a >> 32));
      // R's slots [0, nR) and W's [P - nW, P) stay apart while nR + nW fits:
      // every reservation checks the totals including all earlier ones
      const bool fits = aR + __popcll(wR) + aW + __popcll(wW) <= P;
      if (won) {
        const int ix = role == ROLE_R ? aR + lanes_below(wR) : aW + lanes_below(wW);
        uint32_t pub = eb | kIdxOvf;
        if (fits) {
          const int sl = pool_slot<LT>(role, ix);
          T.smask[sl] = c.mask;
          T.sval[sl] = sv_val(c.sv);
          if (role == ROLE_R) st.reg(rR)[ix] = c;
          pub = eb | rbit | (uint32_t)ix;
        } else {
          ovf = true;
        }
        lds_tag_publish(&T.tag[h], pub);
        if (fits && role == ROLE_W)  // queue readiness, after the release above
          __hip_atomic_store(&T.wrdy[ix], (uint8_t)(eb >> 16), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        res = 1;
        pend = false;
      }
    }
  }
  return res;
}
// Claim an entry for a configuration known distinct whose set index ix is
// already reserved (the split of F); its set entry is stored by the caller.
template <int LT>
__device__ __forceinline__ void lds_claim_lane(CoopTab<LT> &T, int role, const Cfg &c, int ix,
                                               uint32_t eb, bool &ovf) {
  constexpr uint32_t TM = 2 * LT - 1;
  uint32_t h = pool_hash(c, role) & TM;
  lds_release();  // the set entry before its tag
  for (int probes = 0; probes < LT / 2;) {
    const uint32_t t = lds_tag_load(&T.tag[h]);
    if ((t & 0xFFFF0000u) != eb) {
      if (atomicCAS(&T.tag[h], t, eb | ((uint32_t)role << 15) | (uint32_t)ix) == t) return;
      continue;  // lost the race for this entry: re-read it
    }
    h = (h + 1) & TM;
    probes++;
  }
  ovf = true;
}

// ------------------------------------------------------------ the search

// Per-lane record of the window slot this lane holds (valid when the lane's
// bit is set in `occ`).  Slot kinds are uniform 64-bit masks (occ, rdm =
// reads, crashed); the per-lane fields are the precondition, the value a
// mutation writes, the class fields, the return index and the op index.
//   pbit  for a write/CAS: the pending slots of its class (equal f, value,
//         expected, version) with an earlier deadline (return index;
//         crashed = never, ties by call order).  Equal ops have equal
//         preconditions and effects, so linearizing the earliest-deadline
//         one first dominates (an exchange argument: oracle.c,
//         ORACLE_FLAG_DEADLINE_ORDER; crashed ops alone is the round-1
//         CRASH_SYMMETRY): a slot is a candidate only when its pbit slots
//         are linearized.  Checked against the faithful search in tests/.
struct Slot {
  int nv, nvm, nl, nlm;   // precondition
  int val;                // value written (mutations)
  int f, exp, ver;        // class fields
  int idx;                // op index within the key
  uint32_t ret;           // kNever: free or crashed (never returns)
  uint64_t pbit;
};

struct Masks {
  uint64_t occ;      // occupied slots
  uint64_t rdm;      // slots holding reads
  uint64_t crashed;  // slots holding crashed writes/CAS
};

__device__ __forceinline__ uint64_t legal_ballot(const Slot &sl, int ver, int val) {
  return __ballot(pre_ok(sl.nv, sl.nvm, sl.nl, sl.nlm, ver, val));
}

// Mutations that may step configuration (cm, state): legal, pending, and — for
// crashed ops — first of their class among the unlinearized ones.
__device__ __forceinline__ uint64_t mutation_candidates(const Slot &sl, const Masks &mk,
                                                        uint64_t cm, int ver, int val) {
  uint64_t cand = legal_ballot(sl, ver, val) & mk.occ & ~mk.rdm & ~cm;
  cand &= __ballot((sl.pbit & ~cm) == 0);  // deadline order within a class
  return cand;
}
// Eager read closure at a successor state: pending reads legal there.
__device__ __forceinline__ uint64_t read_closure(const Slot &sl, const Masks &mk,
                                                 uint64_t nm, int ver, int val) {
  return legal_ballot(sl, ver, val) & mk.occ & mk.rdm & ~nm;
}

// Retire slots rb: ops linearized in every configuration are finished (a
// crashed op has no return; an :ok op's return would keep every configuration
// unchanged), so their slots are freed and their returns never become events.
// Exact (oracle ORACLE_FLAG_RETIRE, checked against the faithful search).
__device__ __forceinline__ void retire(Slot &sl, Masks &mk, uint64_t rb, int lane) {
  mk.occ &= ~rb;
  mk.rdm &= ~rb;
  mk.crashed &= ~rb;
  if ((rb >> lane) & 1) sl.ret = kNever;
  sl.pbit &= ~rb;
}

// Expand the frontier held in region rF (nF configurations) for the return
// of the op in slot s.  Returns the new frontier size (in region rR), or -1
// (LDS/HBM sets full) / -2 (configuration budget).
template <class Store>
__device__ __forceinline__ int general_return(Store &st, const Slot &sl, const Masks &mk,
                                              int s, int rF, int rR, int rW, int nF,
                                              const KParams &p, KeyOut &o, int lane) {
  const uint64_t bs = 1ull << s;
  st.begin_return();
  int nR = 0, nW = 0;
  // Split F: configs that already linearized x go to R (x's bit dropped),
  // the others to the worklist W.  Ballot + lanes_below compaction.
  for (int j0 = 0; j0 < nF; j0 += kWave) {
    const int j = j0 + lane;
    const bool v = j < nF;
    Cfg c{0, 0};
    if (v) c = st.get(rF, j);
    const bool has = v && (c.mask & bs);
    const bool lacks = v && !(c.mask & bs);
    const uint64_t mh = __ballot(has), ml = __ballot(lacks);
    if (has) st.add_unique_lane(ROLE_R, rR, nR + lanes_below(mh), Cfg{c.mask & ~bs, c.sv});
    if (lacks) st.add_unique_lane(ROLE_W, rW, nW + lanes_below(ml), c);
    nR += __popcll(mh);
    nW += __popcll(ml);
  }
  // Expand W breadth-first until x is linearized in each branch.
  for (int head = 0; head < nW; head++) {
    const Cfg c = st.get(rW, head);
    const uint64_t cm = rfl64(c.mask), csv = rfl64(c.sv);
    const int cver = sv_ver(csv), cval = sv_val(csv);
    uint64_t cand = mutation_candidates(sl, mk, cm, cver, cval);
    while (cand) {
      const int t = __builtin_ctzll(cand);
      cand &= cand - 1;
      const int nver = cver + 1;
      const int nval = rl32(sl.val, t);
      uint64_t nm = cm | (1ull << t);
      nm |= read_closure(sl, mk, nm, nver, nval);
      o.explored++;
      const uint64_t nsv = pack_sv(nver, nval);
      const int r = (nm & bs) ? st.insert(ROLE_R, rR, nR, nm & ~bs, nsv, lane)
                              : st.insert(ROLE_W, rW, nW, nm, nsv, lane);
      if (r < 0) return -1;
      if (o.explored > p.budget) return -2;
    }
  }
  return nR;
}


__device__ __forceinline__ void coop_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Per lane, the slots (lane t holds slot t's precondition in spre) legal in
// the lane's state (ver, val): one ballot per distinct state among the
// lanes, which share few states (a batch's configurations differ mostly in
// which ops they linearized), instead of a test per slot and lane.
__device__ __forceinline__ uint64_t legal_by_state(const int4 &spre, int ver, int val, bool act) {
  uint64_t legal = 0;
  bool todo = act;
  for (uint64_t pend = __ballot(todo); pend; pend = __ballot(todo)) {
    const int l = __builtin_ctzll(pend);
    const int sver = rl32(ver, l), sval = rl32(val, l);
    const uint64_t m = __ballot(pre_ok(spre.x, spre.y, spre.z, spre.w, sver, sval));
    if (todo && ver == sver && val == sval) {
      legal = m;
      todo = false;
    }
  }
  return legal;
}

// One wave's share of a cooperative expansion (every wave of the workgroup
// calls it; the parameters are in C).  Barrier count is uniform: one after
// the split, two per BFS level.
template <int LT>
__device__ void coop_expand(HbmStore &st, CoopShared &C, int lane, int wave) {
  const int nw = st.nwaves;
#ifdef LC_COOP_PROF
  st.ts[1] = CP_NOW();
#endif
  st.epoch = C.epoch;
  st.tmask = C.tmask;
  CoopTab<LT> &T = coop_tab<LT>();
  const bool lds = C.lds;  // uniform over the workgroup
  constexpr int P = CoopTab<LT>::kPool;
  const int lim = lds ? P : st.lim(nw);
  const uint32_t eb = C.lepoch << 16;  // LDS tables' epoch
  bool ovf = false;
  if (lds && C.lclear) {  // the 8-bit LDS epoch wrapped: clear the tags and flags
    for (int i = wave * kWave + lane; i < 2 * LT; i += nw * kWave) T.tag[i] = 0;
    for (int i = wave * kWave + lane; i < P; i += nw * kWave) T.wrdy[i] = 0;
    lds_barrier();
  }
  const uint64_t bs = C.bs, ordered = C.ordered;
  const uint64_t muts = rfl64(C.muts), reads = rfl64(C.reads);  // scalar loops below
  const int rF = C.rF, rR = C.rR, rW = C.rW, nF = C.nF;
  const SlotLds &L = C.slots;
  // Lane t holds slot t's precondition, value and class bit: the candidate
  // and read-closure loops run over slots uniformly and read them with
  // v_readlane (no dependent LDS load per slot and lane).
  const int4 spre = L.pre[lane];
  const int sval = L.val[lane];
  const uint64_t spbit = L.pbit[lane];
  const bool vt = C.vt;  // (coop_return: C.vlegal)
  // split F into R (x linearized, its bit dropped) and W, after F's pending
  // updates: retired slots cleared, then reads called since linearized where
  // legal (a freed slot a new read took: both, in that order)
  const uint64_t fclear = C.fclear, fclose = C.fclose;
  uint64_t rand = ~0ull;  // AND of the masks this wave adds to R
  auto flush_rand = [&]() {
    const uint64_t r = wave_and_u64(rand);
    if (r != ~0ull && lane == 0)
      __hip_atomic_fetch_and(&C.rand, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    rand = ~0ull;
  };
  for (int j0 = wave * kWave; j0 < nF; j0 += nw * kWave) {
    const int j = j0 + lane;
    const bool v = j < nF;
    Cfg c{0, 0};
    if (v) c = st.get(rF, j);
    c.mask &= ~fclear;
    if (fclose) {
      const int fver = sv_ver(c.sv), fval = sv_val(c.sv);
      if (vt && !__ballot(v && (uint32_t)(fval + 1) >= (uint32_t)kVTab))
        c.mask |= v ? C.vlegal[fval + 1] & fclose : 0;
      else
        c.mask |= legal_by_state(spre, fver, fval, v) & fclose;
    }
    if (lds && j == 0) C.kw = sv_ver(c.sv) - __popcll(c.mask & muts);  // (any F config gives it)
    const bool has = v && (c.mask & bs);
    if (has) rand &= c.mask & ~bs;
    const bool lacks = v && !(c.mask & bs);
    const uint64_t mh = __ballot(has), ml = __ballot(lacks);
    int bR = 0, bW = 0;
    if (lane == 0) {
      bR = mh ? atomicAdd(&C.nR, __popcll(mh)) : 0;
      bW = ml ? atomicAdd(&C.nW, __popcll(ml)) : 0;
    }
    bR = __builtin_amdgcn_readfirstlane(bR);
    bW = __builtin_amdgcn_readfirstlane(bW);
    if (lds) {  // nF <= the pool: nR + nW = nF fits
      if (has) {
        const Cfg rc{c.mask & ~bs, c.sv};
        const int ix = bR + lanes_below(mh);
        st.reg(rR)[ix] = rc;
        T.smask[ix] = rc.mask;
        T.sval[ix] = sv_val(rc.sv);
        lds_claim_lane(T, ROLE_R, rc, ix, eb, ovf);
      }
      if (lacks) {
        const int ix = bW + lanes_below(ml);
        T.smask[P - 1 - ix] = c.mask;
        T.sval[P - 1 - ix] = sv_val(c.sv);
        lds_claim_lane(T, ROLE_W, c, ix, eb, ovf);  // (releases the entry first)
        __hip_atomic_store(&T.wrdy[ix], (uint8_t)(eb >> 16), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    } else {
      if (has) st.claim_unique_lane(ROLE_R, rR, bR + lanes_below(mh), Cfg{c.mask & ~bs, c.sv});
      if (lacks) st.claim_unique_lane(ROLE_W, rW, bW + lanes_below(ml), c);
    }
  }
  if (__ballot(ovf) && lane == 0) atomicMin(&C.status, -3);
  flush_rand();  // (before the split's barrier)
#ifdef LC_COOP_PROF
  st.ts[2] = CP_NOW();
#endif
  if (lds) {
    // LDS: W is a work queue.  The split's claims must all be in the tables
    // before any successor is deduplicated against them: one barrier.
    lds_barrier();
  } else {
    // HBM: level-synchronous.  Level bounds and the go flag are written by
    // wave 0 between two barriers, while no wave appends, so every wave
    // reads the same values.
    coop_barrier();
    if (wave == 0 && lane == 0) {
      C.lo = 0;
      C.hi = C.nW;
      C.head = 0;
      C.go = C.hi > 0 && C.status == 0;
    }
    coop_barrier();
  }
#ifdef LC_COOP_PROF
  st.ts[3] = CP_NOW();
#endif
  const uint32_t ep16 = eb >> 16;
  const int kw = lds ? C.kw : 0;  // (written in the split, before the barrier above)
  for (;;) {
    int lo = 0, hi = 0;
    if (!lds) {
      if (!C.go) break;
      lo = C.lo;
      hi = C.hi;
    }
    for (;;) {  // batches of up to 64 W configurations
      int b = 0, k = 0;
#ifdef LC_COOP_PROF
      const uint64_t qc0 = CP_NOW();
      int qsp = 0;
#endif
      if (lds) {
        // Queue claim: (head, active) packed in one word, so a wave that
        // finds the queue empty leaves only when no wave is expanding (a
        // wave that still expands re-reads the queue after its appends).
        if (lane == 0) {
          for (int spin = 0;; spin++) {
            if (spin == kSpinMax) atomicMin(&C.status, -3);  // safety net: redone in HBM
            if (__hip_atomic_load(&C.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
              k = -1;
              break;
            }
            const unsigned long long q =
                __hip_atomic_load(&C.qword, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const int h = (int)(uint32_t)q;
            const int n = min(__hip_atomic_load(&C.nW, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP), P);
            if (h < n) {
              const int kk = min(kWave, n - h);
              if (atomicCAS(&C.qword, q, q + (unsigned long long)kk + (1ull << 32)) == q) {
                b = h;
                k = kk;
                break;
              }
              continue;
            }
            if ((q >> 32) == 0) {  // nothing queued, nobody expanding
              k = -1;
              break;
            }
#ifdef LC_COOP_PROF
            qsp++;
#endif
            __builtin_amdgcn_s_sleep(LC_COOP_SLEEP);
          }
        }
        k = uni(k);
        b = uni(b);
#ifdef LC_COOP_PROF
        st.cp[13] += (uint64_t)uni(qsp);
        st.cp[14] += CP_NOW() - qc0;
#endif
        if (k < 0) break;
      } else {
        if (lane == 0) b = atomicAdd(&C.head, kWave);
        b = uni(b) + lo;
        if (b >= hi || __hip_atomic_load(&C.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
          break;
        k = min(kWave, hi - b);
      }
      const int j = b + lane;
      const bool act = lane < k;
      Cfg c;
      if (lds) {
        // entries reserved by a wave still in its round: wait for their flag
        // (an entry reserved past the pool never gets one: its wave sets the
        // status, and the return is redone)
        if (act)
          for (int spin = 0; __hip_atomic_load(&T.wrdy[j], __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP) != (uint8_t)ep16; spin++) {
            if (spin == kSpinMax ||  // (safety net: a writer is always mid-round)
                __hip_atomic_load(&C.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
              ovf = true;
              break;
            }
            __builtin_amdgcn_s_sleep(LC_COOP_SLEEP);
          }
        if (__ballot(ovf)) {
          if (lane == 0) {
            atomicMin(&C.status, -3);
            atomicAdd(&C.qword, ~0ull << 32);
          }
          break;
        }
#ifdef LC_COOP_PROF
        st.cp[15] += CP_NOW() - qc0;
#endif
        lds_acquire();
        const int jj = P - 1 - (act ? j : b);
        c.mask = T.smask[jj];
        c.sv = pack_sv(kw + __popcll(c.mask & muts), T.sval[jj]);
      } else {
        c = st.get(rW, act ? j : b);
      }
      const int cver = sv_ver(c.sv), cval = sv_val(c.sv);
      uint64_t cand;
      if (vt && !__ballot(act && (uint32_t)(cval + 1) >= (uint32_t)kVTab))
        cand = act ? C.vlegal[cval + 1] & muts & ~c.mask : 0;  // by value (versions free)
      else
        cand = legal_by_state(spre, cver, cval, act) & muts & ~c.mask;
      // an op only if its class predecessors (deadline order) are linearized
      for (uint64_t m = muts & ordered; m; m &= m - 1) {
        const int t = __builtin_ctzll(m);
        if (rl64(spbit, t) & ~c.mask) cand &= ~(1ull << t);
      }
#ifdef LC_COOP_PROF
      const uint64_t qc2 = CP_NOW();
      if (lds) {
        st.cp[11]++;
        st.cp[16] += qc2 - qc0;
      }
#endif
      // The batch's successors, one per lane and round: lane j of a round
      // takes the successor at position r0 + j of the batch's list (source
      // lanes in order, each its candidates by slot), so a round is full
      // unless it is the last, whatever the spread of candidates per lane
      const int ncand = __popcll(cand);
      const int incl = wave_prefix_sum(ncand, lane);
      const int total = __builtin_amdgcn_readlane(incl, kWave - 1);
      const unsigned long long exw = (unsigned long long)total;  // (one atomic per batch)
      uint16_t *scr = T.scr[wave];
      for (int r0 = 0; r0 < total; r0 += kWave) {
#ifdef LC_COOP_PROF
        if (lds) st.cp[12]++;
#endif
        {
          uint64_t cc = cand;
          for (int i = incl - ncand; cc && i < r0 + kWave; i++, cc &= cc - 1)
            if (i >= r0) scr[i - r0] = (uint16_t)((lane << 6) | __builtin_ctzll(cc));
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
        const bool has = r0 + lane < total;
        const int e = has ? (int)scr[lane] : 0;
        const int src = has ? e >> 6 : lane, t = e & 63;
        const uint64_t cm = ((uint64_t)(uint32_t)__shfl((int)(c.mask >> 32), src) << 32) |
                            (uint32_t)__shfl((int)(uint32_t)c.mask, src);
        const int nver = __shfl(cver, src) + 1, nval = __shfl(sval, t);
        uint64_t nm = cm | (1ull << t);
        // eager read closure
        if (vt && !__ballot(has && (uint32_t)(nval + 1) >= (uint32_t)kVTab))
          nm |= has ? C.vlegal[nval + 1] & reads : 0;
        else
          nm |= legal_by_state(spre, nver, nval, has) & reads;
        const bool toR = (nm & bs) != 0;
        const Cfg nc{toR ? nm & ~bs : nm, pack_sv(nver, nval)};
        if (lds) {  // inserts, set indices and appends in one pass
          if (lds_insert_lanes(T, C, st, rR, toR ? ROLE_R : ROLE_W, nc, has, eb, ovf, lane) && toR)
            rand &= nc.mask;
          if (__ballot(ovf)) {
            if (lane == 0) atomicMin(&C.status, -3);
            break;
          }
          continue;
        }
        const int ins = st.insert_lanes_coop(toR ? ROLE_R : ROLE_W, nc, has);
        const bool insR = ins && toR, insW = ins && !toR;
        const uint64_t bR = __ballot(insR), bW = __ballot(insW);
        unsigned long long aRW = 0;
        if (lane == 0 && (bR | bW))
          aRW = atomicAdd(&C.nRW, (unsigned long long)__popcll(bR) |
                                      ((unsigned long long)__popcll(bW) << 32));
        const int aR = uni((int)aRW), aW = uni((int)(aRW >> 32));
        const bool fullR = aR + __popcll(bR) > lim, fullW = aW + __popcll(bW) > lim;
        const bool full = fullR || fullW;
        if (insR && !fullR) {
          st.reg(rR)[aR + lanes_below(bR)] = nc;
          rand &= nc.mask;
        }
        if (insW && !fullW) st.reg(rW)[aW + lanes_below(bW)] = nc;
        // -3: this return's tables are too small (redone larger / in HBM);
        // -1: the workspace is full (next tier)
        if (full) {
          if (lane == 0) atomicMin(&C.status, lim < st.cap ? -3 : -1);
          break;
        }
      }
#ifdef LC_COOP_PROF
      if (lds) st.cp[17] += CP_NOW() - qc2;
#endif
      if (lane == 0 && exw) {
        const unsigned long long ex = atomicAdd(&C.explored, exw) + exw;
        if ((long long)ex > C.budget && C.status == 0) atomicMin(&C.status, -2);
      }
      if (lds && lane == 0) atomicAdd(&C.qword, ~0ull << 32);  // active - 1, after the appends
    }
    if (lds) break;
    flush_rand();
    coop_barrier();  // the level's appends are done
    if (wave == 0 && lane == 0) {
      C.lo = hi;
      C.hi = C.nW;
      C.head = 0;
      C.go = C.lo < C.hi && C.status == 0;
    }
    coop_barrier();
  }
#ifdef LC_COOP_PROF
  st.ts[4] = CP_NOW();
#endif
  if (lds) flush_rand();
  if (lds) coop_barrier();  // the global R appends, for wave 0 and the next split
#ifdef LC_COOP_PROF
  st.ts[5] = CP_NOW();
#endif
}

// Wave 0's side of a cooperative return: publish, expand with the others.
template <int LT>
__device__ int coop_return(CoopStore<LT> &st, const Slot &sl, const Masks &mk, int s, int rF, int rR,
                           int rW, int nF, const KParams &p, KeyOut &o, int lane) {
  CoopShared &C = *st.coop;
#ifdef LC_COOP_PROF
  const uint64_t ce0 = CP_NOW();
#endif
  C.slots.pre[lane] = make_int4(sl.nv, sl.nvm, sl.nl, sl.nlm);
  C.slots.val[lane] = sl.val;
  C.slots.pbit[lane] = sl.pbit;
  const uint64_t ordered = __ballot(sl.pbit != 0);  // (a ballot: outside the lane-0 block)
  // Legality by value id when no pending slot constrains the version (every
  // occupied slot's version mask nvm is 0: version-less models): lane v
  // kept the slots legal at value id v - 1 as they were taken (st.vleg)
  const bool vt = (__ballot(sl.nvm != 0) & mk.occ) == 0;
  if (vt && lane < kVTab) C.vlegal[lane] = st.vleg;
  // LDS tables first when this frontier fits the pool and the previous
  // return's sets did not far outgrow it
  constexpr int kPool = CoopTab<LT>::kPool;
  bool lds = nF <= kPool && st.lsum <= 2 * kPool;
  const uint32_t floor = max(1024u, 256u * (uint32_t)st.nwaves);
  if (!lds) st.tmask = st.pick_tmask(nF, floor);
#ifdef HBM_PROFILE
  const uint64_t tr0 = wall_clock64();
#endif
#ifdef LC_COOP_PROF
  const uint64_t cr0 = CP_NOW();
  st.cp[23] += cr0 - ce0;
#endif
  for (;;) {
    st.begin_return();  // a fresh epoch per attempt: the aborted one's entries are stale
    int lclear = 0;
    if (lds) {
      st.lepoch = (st.lepoch + 1) & kLepochMask;
      if (st.lepoch == 0) {
        st.lepoch = 1;
        lclear = 1;
      }
    }
    if (lane == 0) {
      C.cmd = kCoopExpand;
      C.rF = rF;
      C.rR = rR;
      C.rW = rW;
      C.nF = nF;
      C.bs = 1ull << s;
      C.muts = mk.occ & ~mk.rdm;
      C.reads = mk.occ & mk.rdm;
      C.ordered = ordered;
      C.epoch = st.epoch;
      C.tmask = st.tmask;
      C.lds = lds;
      C.qword = 0;
      C.lclear = lclear;
      C.lepoch = st.lepoch;
      C.nR = 0;
      C.nW = 0;
      C.status = 0;
      C.explored = (unsigned long long)o.explored;
      C.budget = (long long)p.budget;
      C.fclear = st.fclear;
      C.fclose = st.fclose;
      C.rand = ~0ull;
      C.vt = vt;
    }
#ifdef LC_COOP_PROF
    st.ts[0] = CP_NOW();
#endif
    coop_barrier();  // the workers' start barrier
    coop_expand<LT>(st, C, lane, 0);
#ifdef LC_COOP_PROF
    if (lds && C.status == 0) {
      for (int q = 0; q < 5; q++) st.cp[q] += st.ts[q + 1] - st.ts[q];
      st.cp[5]++;
    }
    if (lds && C.status == -3) st.cp[25] += CP_NOW() - st.ts[0];
    if (!lds) {
      st.cp[26]++;
      st.cp[27] += CP_NOW() - st.ts[0];
      st.cp[28] += (uint64_t)max(C.nR, C.nW);
    }
#endif
    if (C.status != -3) break;
    if (lds) {
      lds = false;
      st.tmask = st.pick_tmask(max(nF, kPool / 2), floor);
    } else {
      st.tmask = st.grow_tmask();
    }
  }
#ifdef HBM_PROFILE
  if (lane == 0 && C.status == 0) {
    const int mx = max(C.nR, C.nW);
    const int bkt = min(19, 32 - __builtin_clz((unsigned)max(mx, 1)));
    atomicAdd(&g_hhist[bkt][0], 1ull);
    atomicAdd(&g_hhist[bkt][1], (unsigned long long)(wall_clock64() - tr0));
    atomicAdd(&g_hhist[bkt][2], (unsigned long long)lds);
    atomicAdd(&g_hhist[bkt][3], (unsigned long long)(C.explored - (unsigned long long)o.explored));
  }
  if (lane == 0 && blockIdx.x < 4096) {
    g_hwg[blockIdx.x][lds ? 0 : 1] += wall_clock64() - tr0;
  }
#endif
#ifdef LC_COOP_PROF
  st.cp[6] += CP_NOW() - cr0;
  st.cp[8]++;
  if (!lds) st.cp[9]++;
#endif
  if (C.status < 0) return C.status;
  o.explored = (int64_t)C.explored;
  st.last = max(C.nR, C.nW);
  st.lsum = C.nR + C.nW;
  st.fclear = st.fclose = 0;  // applied by this return's split
  st.rand = C.rand;
  if (!lds) st.hint = max(st.hint, st.last);
  return C.nR;
}

// HBM tier: the same expansion as general_return, lane-parallel.  The
// worklist W is taken 64 configurations at a time, one per lane; each lane
// tests every pending mutation against its own configuration (slots staged
// in LDS), emits one successor per round with its eager read closure, and
// the round's successors are deduplicated into the R / W tables together
// (insert_lanes) and appended to the regions by ballot prefix.  Every W
// configuration is still expanded exactly once, so R, the explored count and
// the verdicts equal the serial expansion's; only the order differs.
__device__ __forceinline__ int general_return_par_try(HbmStore &st, const Slot &sl,
                                                      const Masks &mk, int s, int rF, int rR,
                                                      int rW, int nF, const KParams &p, KeyOut &o,
                                                      int lane);
template <class S>
__device__ __forceinline__ int general_return_par(S &st, const Slot &sl, const Masks &mk,
                                                  int s, int rF, int rR, int rW, int nF,
                                                  const KParams &p, KeyOut &o, int lane) {
  if constexpr (S::kLT > 0) return coop_return<S::kLT>(st, sl, mk, s, rF, rR, rW, nF, p, o, lane);
  st.tmask = st.pick_tmask(nF, 1024u);
  const int64_t explored0 = o.explored;
  for (;;) {
    const int r = general_return_par_try(st, sl, mk, s, rF, rR, rW, nF, p, o, lane);
    if (r != -3) return r;
    o.explored = explored0;
    st.tmask = st.grow_tmask();
  }
}

// One attempt of general_return_par with this return's table size: -3 when
// a role outgrows it (the caller redoes the return with a larger table).
__device__ __forceinline__ int general_return_par_try(HbmStore &st, const Slot &sl,
                                                      const Masks &mk, int s, int rF, int rR,
                                                      int rW, int nF, const KParams &p, KeyOut &o,
                                                      int lane) {
  const uint64_t bs = 1ull << s;
  st.begin_return();
  const int lim = st.lim(1);
  int nR = 0, nW = 0;
  for (int j0 = 0; j0 < nF; j0 += kWave) {  // split F into R and W, as serially
    const int j = j0 + lane;
    const bool v = j < nF;
    Cfg c{0, 0};
    if (v) c = st.get(rF, j);
    const bool has = v && (c.mask & bs);
    const bool lacks = v && !(c.mask & bs);
    const uint64_t mh = __ballot(has), ml = __ballot(lacks);
    if (has) st.add_unique_lane(ROLE_R, rR, nR + lanes_below(mh), Cfg{c.mask & ~bs, c.sv});
    if (lacks) st.add_unique_lane(ROLE_W, rW, nW + lanes_below(ml), c);
    nR += __popcll(mh);
    nW += __popcll(ml);
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  const uint64_t muts = mk.occ & ~mk.rdm, reads = mk.occ & mk.rdm;
  const int4 spre = make_int4(sl.nv, sl.nvm, sl.nl, sl.nlm);  // lane t: slot t
  const uint64_t ordered = __ballot(sl.pbit != 0);
  for (int head = 0; head < nW;) {
    const int j = head + lane;
    const bool act = j < nW;  // this batch: W[head, min(head + 64, nW)) as of now
    const int taken = min(kWave, nW - head);
    const Cfg c = st.get(rW, act ? j : head);
    const int cver = sv_ver(c.sv), cval = sv_val(c.sv);
    // candidates: legal pending mutations; a crashed one only if it is the
    // earliest unlinearized member of its class
    uint64_t cand = legal_by_state(spre, cver, cval, act) & muts & ~c.mask;
    for (uint64_t m = muts & ordered; m; m &= m - 1) {
      const int t = __builtin_ctzll(m);
      if (rl64(sl.pbit, t) & ~c.mask) cand &= ~(1ull << t);
    }
    for (;;) {
      const bool has = cand != 0;
      const uint64_t hb = __ballot(has);
      if (!hb) break;
      const int t = has ? __builtin_ctzll(cand) : 0;
      cand &= cand - 1;
      const int nver = cver + 1, nval = __shfl(sl.val, t);
      uint64_t nm = c.mask | (1ull << t);
      nm |= legal_by_state(spre, nver, nval, has) & reads;  // eager read closure
      const bool toR = (nm & bs) != 0;
      const Cfg nc{toR ? nm & ~bs : nm, pack_sv(nver, nval)};
      o.explored += __popcll(hb);
      // dedup into R or W, both roles in one round of inserts
      const int ins = st.insert_lanes(toR ? ROLE_R : ROLE_W, nc, has);
      const bool insR = ins && toR, insW = ins && !toR;
      const uint64_t bR = __ballot(insR), bW = __ballot(insW);
      if (nR + __popcll(bR) > lim || nW + __popcll(bW) > lim) return lim < st.cap ? -3 : -1;
      if (insR) st.reg(rR)[nR + lanes_below(bR)] = nc;
      if (insW) st.reg(rW)[nW + lanes_below(bW)] = nc;
      nR += __popcll(bR);
      nW += __popcll(bW);
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      if (o.explored > p.budget) return -2;
    }
    head += taken;  // entries appended meanwhile are taken by a later batch
  }
  st.hint = max(st.hint, max(nR, nW));
  return nR;
}

// Per-chunk uniform masks over the 64 records of the current chunk.
struct ChunkMasks {
  uint64_t special;    // malformed or unknown :f
  uint64_t isread;     // reads
  uint64_t skip;       // reads that never constrain: crashed, or [nil nil]
  uint64_t legal_now;  // reads legal in the lone configuration (single mode)
};

__device__ __forceinline__ ChunkMasks chunk_masks(const Rec &r, uint64_t fsv) {
  ChunkMasks m;
  m.special = __ballot(r.bad || r.f > LC_F_CAS);
  m.isread = __ballot(r.f == LC_F_READ);
  m.skip = __ballot(r.f == LC_F_READ && (r.ret == kNever || (r.ver == -1 && r.val == -1)));
  m.legal_now = m.isread & __ballot(pre_ok(r.nv, r.nvm, r.nl, r.nlm, sv_ver(fsv), sv_val(fsv)));
  return m;
}

// Calls must strictly increase within a key: compare each record with its
// predecessor (lane-1, or the previous chunk's last call for lane 0).
__device__ __forceinline__ void check_order(Rec &r, uint32_t &last_call, int lane) {
  const uint32_t prev = (uint32_t)wave_shr1((int)r.call, 0);
  const bool first_key_rec = lane == 0 && last_call == kNever;
  const uint32_t p = lane == 0 ? last_call : prev;
  if (r.call != kNever && !first_key_rec && r.call <= p) r.bad = 1;
  const uint32_t l = (uint32_t)__builtin_amdgcn_readlane((int)r.call, kWave - 1);
  if (l != kNever) last_call = l;
}

// lc_check_frontiers (knossos :configs): the search of check_key<.., true>
// stops at the :ok return of record `stop` (key-relative return stop_ret) and
// writes up to `max` configurations of the frontier that return expands; n
// = configurations written, 0 when the op's return was a no-op (it had been
// retired), -1 when the search ended before (an earlier failure, an
// overflow, the budget).  Wave-uniform.
struct DumpReq {
  int stop;
  uint32_t stop_ret;
  lc_fx_config *out;
  int max;
  int n;
};

// The frontier just before a return: the lone configuration (every occupied
// slot pending in it), or region rF's first min(nF, max) configurations;
// one lane per configuration writes its state and its pending ops (slots
// occupied and not linearized in it), sorted by record index.
template <class Store>
__device__ void dump_frontier(const Store &st, const Slot &sl, const Masks &mk, bool single,
                              uint64_t fsv, int rF, int nF, DumpReq &dr, int lane) {
  const int m = single ? 1 : min(nF, dr.max);
  for (int j0 = 0; j0 < m; j0 += kWave) {
    const int j = j0 + lane;
    const bool act = j < m;
    uint64_t lin = 0, sv = fsv;
    if (!single && act) {
      const Cfg c = st.get(rF, j);
      lin = c.mask;
      sv = c.sv;
    }
    const uint64_t pend = mk.occ & ~lin;
    lc_fx_config *c = dr.out + (act ? j : 0);
    int np = 0;
    for (int t = 0; t < kWave; t++) {
      if (!((mk.occ >> t) & 1)) continue;  // (uniform)
      const int idx = rl32(sl.idx, t);
      if (act && ((pend >> t) & 1)) c->pending[np++] = idx;
    }
    if (act) {
      for (int a = 1; a < np; a++) {  // insertion sort, <= 64 entries
        const int64_t v = c->pending[a];
        int b = a - 1;
        while (b >= 0 && c->pending[b] > v) {
          c->pending[b + 1] = c->pending[b];
          b--;
        }
        c->pending[b + 1] = v;
      }
      c->version = sv_ver(sv);
      c->value = sv_val(sv);
      c->n_pending = np;
    }
  }
  dr.n = m;
}

#ifdef LC_COOP_PROF
#define EL_PROF(stmt)                                  \
  do {                                                 \
    if constexpr (DeferF<Store>::value) { stmt; }      \
  } while (0)
#else
#define EL_PROF(stmt) \
  do {                \
  } while (0)
#endif
template <class Store, bool kDump = false>
__device__ void check_key(const lc_op *__restrict__ kops, const int n,
                          const KParams &p, Store &st, KeyOut &o,
                          const int lane, DumpReq *dreq = nullptr) {
  o.verdict = LC_VALID;
  o.reason = LC_REASON_NONE;
  o.fail_op = -1;
  o.fail_end = -1;
  o.explored = 1;
  o.max_frontier = 1;
  if (n <= 0) return;

  // Frontier: either ONE configuration in SGPRs (single; after retirement its
  // linearized set is always empty, so it is just the state fsv and every
  // occupied slot is pending in it), or nF configurations in region rF.
  bool single = true;
  uint64_t fsv = pack_sv(p.init_ver, p.init_val);
  int rF = 0, rR = 1, rW = 2, nF = 1;

  Slot sl{0, 0, 0, 0, -1, 0, -1, -1, -1, kNever, 0ull};
  Masks mk{0, 0, 0};

  const int64_t base_idx = kops[0].call;  // scalar load (key is wave-uniform)
  const uint64_t t0 = p.time_ticks ? wall_clock64() : 0;
  uint32_t last_call = kNever;
  Rec cur = decode(load_raw(kops, lane, n), base_idx);
  check_order(cur, last_call, lane);
  ChunkMasks cmk = chunk_masks(cur, fsv);
  Raw nxt = load_raw(kops, kWave + lane, n);
  int base = 0, i = 0;

#ifdef LC_COOP_PROF
  uint64_t el0 = 0;
#endif
  for (;;) {
    EL_PROF(el0 = CP_NOW());
    const uint32_t ncall = (i < n) ? (uint32_t)rl32((int)cur.call, i - base) : kNever;
    // Returns due before the next call: one ballot; the DPP min only when
    // several are due at once.
    const uint64_t due = __ballot(sl.ret < ncall);
    if (due == 0) {
      if constexpr (kDump) {
        if (ncall > dreq->stop_ret) {  // (i >= n included) its return came and went:
          dreq->n = 0;                 // the op had been retired
          return;
        }
      }
      if (i >= n) break;  // no calls left, no pending returns
      // ------------------------------------------------------- call of op i
      const int li = i - base;
      const uint64_t bit = 1ull << li;
      if (cmk.special & bit) {
        o.verdict = LC_UNKNOWN;
        // register.clj:63: condp without a default clause throws
        o.reason = rl32(cur.bad, li) ? LC_REASON_MALFORMED : LC_REASON_UNKNOWN_F;
        return;
      }
      // Reads that never constrain, and (lone configuration) reads legal
      // right now — eager closure + retirement — take no slot at all.
      const bool done = (cmk.isread & bit) &&
                        ((cmk.skip & bit) || (single && (cmk.legal_now & bit)));
      if (!done) {
        if (mk.occ == ~0ull) {
          o.verdict = LC_UNKNOWN;
          o.reason = LC_REASON_WINDOW_OVERFLOW;
          return;
        }
        const int s = __builtin_ctzll(~mk.occ);
        const uint64_t bs = 1ull << s;
        const int f = rl32(cur.f, li), val = rl32(cur.val, li);
        const int ex = rl32(cur.exp, li), ver = rl32(cur.ver, li);
        const int nv = rl32(cur.nv, li), nvm = rl32(cur.nvm, li);
        const int nl = rl32(cur.nl, li), nlm = rl32(cur.nlm, li);
        const uint32_t ret = (uint32_t)rl32((int)cur.ret, li);
        uint64_t pbit = 0;
        if (f != LC_F_READ) {
          // Deadline order (oracle ORACLE_FLAG_DEADLINE_ORDER): within a
          // class of equal writes/CAS (f, value, expected, version), an op
          // may be linearized only after the pending members with earlier
          // deadlines (return index; crashed = never, ties by call order).
          const uint64_t cls = __ballot(sl.f == f && sl.val == val && sl.exp == ex && sl.ver == ver) &
                               mk.occ & ~mk.rdm;
          pbit = cls & __ballot(sl.ret <= ret);  // before s (equal: both crashed, called first)
          if (((cls & ~pbit) >> lane) & 1) sl.pbit |= bs;  // the later ones wait for s
          if (ret == kNever) mk.crashed |= bs;
        }
        if constexpr (DeferF<Store>::value) {  // (coop_return's value table)
          const bool ok = (((lane - 1) ^ nl) & nlm) == 0;
          st.vleg = ok ? st.vleg | bs : st.vleg & ~bs;
        }
        if (lane == s) {
          sl.nv = nv;
          sl.nvm = nvm;
          sl.nl = nl;
          sl.nlm = nlm;
          sl.val = val;
          sl.f = f;
          sl.exp = ex;
          sl.ver = ver;
          sl.idx = i;
          sl.ret = ret;
          sl.pbit = pbit;
        }
        mk.occ |= bs;
        if (f == LC_F_READ) {
          mk.rdm |= bs;
          if constexpr (DeferF<Store>::value) {
            if (!single) st.fclose |= bs;  // (by the next split)
          } else if (!single) {  // eager read closure at the call, per configuration
            for (int j = lane; j < nF; j += kWave) {
              const Cfg c = st.get(rF, j);
              if (pre_ok(nv, nvm, nl, nlm, sv_ver(c.sv), sv_val(c.sv)))
                st.set_mask_lane(rF, j, c.mask | bs);
            }
          }
        }
      }
      i++;
      if (i - base == kWave) {
        base += kWave;
        cur = decode(nxt, base_idx);
        check_order(cur, last_call, lane);
        cmk = chunk_masks(cur, fsv);
        nxt = load_raw(kops, base + kWave + lane, n);
      }
      EL_PROF(st.cp[18] += CP_NOW() - el0; st.cp[21]++);
      continue;
    }

    // ----------------------------------------------------- return of x
    int s;
    if ((due & (due - 1)) == 0) {
      s = __builtin_ctzll(due);
    } else {
      const bool mine = (due >> lane) & 1;
      const uint32_t m = wave_min_u32(mine ? sl.ret : kNever);
      s = __builtin_ctzll(__ballot(mine && sl.ret == m));
    }
    const uint64_t bs = 1ull << s;
    const int x_idx = rl32(sl.idx, s);
    const uint32_t nret = (uint32_t)rl32((int)sl.ret, s);
    if constexpr (kDump) {
      if (nret > dreq->stop_ret) {
        dreq->n = 0;
        return;
      }
      if (x_idx == dreq->stop) {
        dump_frontier(st, sl, mk, single, fsv, rF, nF, *dreq, lane);
        return;
      }
    }
    bool empty = false;
#ifdef LC_COOP_PROF
    const bool was_single = single;
#endif
    if (single) {
      // x is pending (a linearized op would have been retired).  Chain walk:
      // while exactly one mutation can step the lone configuration, the JIT
      // expansion is a path (versions strictly increase, so no configuration
      // repeats) and stays in SGPRs.
      const int64_t explored0 = o.explored;
      uint64_t cm = 0, csv = fsv;
      bool branch = false;
      for (;;) {
        const int cver = sv_ver(csv), cval = sv_val(csv);
        const uint64_t cand = mutation_candidates(sl, mk, cm, cver, cval);
        if (cand == 0) {
          empty = true;
          break;
        }
        if (cand & (cand - 1)) {
          branch = true;
          break;
        }
        const int t = __builtin_ctzll(cand);
        const int nver = cver + 1;
        const int nval = rl32(sl.val, t);
        uint64_t nm = cm | (1ull << t);
        nm |= read_closure(sl, mk, nm, nver, nval);
        o.explored++;
        if (o.explored > p.budget) {
          o.verdict = LC_UNKNOWN;
          o.reason = LC_REASON_CONFIG_BUDGET;
          return;
        }
        cm = nm;
        csv = pack_sv(nver, nval);
        if (nm & bs) break;
      }
      if (branch) {
        // Several successors: redo this return on the general path from the
        // lone configuration.
        o.explored = explored0;
        single = false;
        rF = 0;
        rR = 1;
        rW = 2;
        nF = 1;
        if (lane == 0) st.reg(rF)[0] = Cfg{0ull, fsv};
      } else if (!empty) {
        fsv = csv;
        retire(sl, mk, cm, lane);  // x included
        cmk.legal_now = cmk.isread &
                        __ballot(pre_ok(cur.nv, cur.nvm, cur.nl, cur.nlm, sv_ver(fsv), sv_val(fsv)));
      }
    }
    EL_PROF(if (was_single) { st.cp[19] += CP_NOW() - el0; st.cp[22]++; });
    if (!single) {
      // the time budget is checked where time goes: returns on the general
      // (multi-configuration) path
      if (p.time_ticks && wall_clock64() - t0 > p.time_ticks) {
        o.verdict = LC_UNKNOWN;
        o.reason = LC_REASON_TIME_BUDGET;
        return;
      }
      int r;
      EL_PROF(st.cp[24] += CP_NOW() - el0);
      if constexpr (std::is_base_of<HbmStore, Store>::value)
        r = general_return_par(st, sl, mk, s, rF, rR, rW, nF, p, o, lane);
      else
        r = general_return(st, sl, mk, s, rF, rR, rW, nF, p, o, lane);
      if (r < 0) {
        o.verdict = LC_UNKNOWN;
        o.reason = r == -1 ? LC_REASON_FRONTIER_LDS : LC_REASON_CONFIG_BUDGET;
        return;
      }
#ifdef LC_COOP_PROF
      const uint64_t pr0 = CP_NOW();
#endif
      const int t = rF;
      rF = rR;
      rR = t;
      nF = r;
      if (nF > o.max_frontier) o.max_frontier = nF;
      empty = nF == 0;
      if (!empty) {
        retire(sl, mk, bs, lane);  // x returned
        uint64_t rb;
        if constexpr (DeferF<Store>::value) {
          rb = mk.occ & st.rand;  // (the AND the return's waves kept)
          if (rb) {
            retire(sl, mk, rb, lane);
            st.fclear |= rb;  // (by the next split)
          }
        } else {
          uint64_t acc = ~0ull;
          for (int j = lane; j < nF; j += kWave) acc &= st.get(rF, j).mask;
          rb = mk.occ & wave_and_u64(acc);
          if (rb) {
            retire(sl, mk, rb, lane);
            for (int j = lane; j < nF; j += kWave)
              st.set_mask_lane(rF, j, st.get(rF, j).mask & ~rb);
          }
        }
        if (nF == 1) {  // back to the register-resident frontier (mask now empty)
          fsv = rfl64(st.get(rF, 0).sv);
          if constexpr (DeferF<Store>::value) st.fclear = st.fclose = 0;
          single = true;
          cmk.legal_now = cmk.isread &
                          __ballot(pre_ok(cur.nv, cur.nvm, cur.nl, cur.nlm, sv_ver(fsv), sv_val(fsv)));
        }
      }
      EL_PROF(st.cp[20] += CP_NOW() - pr0);
    }
    if (empty) {
      o.verdict = LC_INVALID;
      o.reason = LC_REASON_NONLINEARIZABLE;
      o.fail_op = x_idx;
      o.fail_end = base_idx + (int64_t)nret;
      return;
    }
  }
}

__device__ __forceinline__ void write_result(lc_key_result *r, const KeyOut &o) {
  r->verdict = o.verdict;
  r->reason = o.reason;
  r->fail_op = o.fail_op;
  r->fail_prefix_end = o.fail_end;
  r->configs_explored = o.explored;
  r->max_frontier = o.max_frontier;
}

__global__ __launch_bounds__(kWave *kWavesPerWG) void lds_tier_kernel(
    const lc_op *__restrict__ ops, const int64_t *__restrict__ key_off,
    const int32_t *__restrict__ keys, const int64_t n_keys, const KParams p,
    lc_key_result *__restrict__ out, int32_t *__restrict__ ovf_keys,
    KStatus *__restrict__ status) {
  const int64_t key_base = key_off[0];  // ops points at key_off[0]'s record
  __shared__ Cfg lds[kWavesPerWG][3][kLdsCap];
  const int lane = threadIdx.x & (kWave - 1);
  // wave-uniform by construction; readfirstlane lets the compiler use scalar
  // loads for key_off and keeps vector-memory waits off the event loop
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int64_t item = (int64_t)blockIdx.x * kWavesPerWG + wid;
  if (item >= n_keys) return;
  const int64_t key = keys ? keys[item] : item;
  const int64_t beg = key_off[key], end = key_off[key + 1];
  KeyOut o;
  if (end < beg || end - beg > 0x7FFFFFFF) {
    o = KeyOut{LC_UNKNOWN, LC_REASON_MALFORMED, -1, -1, 0, 0};
  } else {
    LdsStore st{&lds[wid][0][0]};
    check_key(ops + (beg - key_base), (int)(end - beg), p, st, o, lane);
  }
  if (lane == 0) {
    write_result(&out[key], o);
    if (o.reason == LC_REASON_MALFORMED) atomicAdd(&status->malformed, 1);
    if (o.reason == LC_REASON_FRONTIER_LDS) {
      const int pos = atomicAdd(&status->n_overflow, 1);
      ovf_keys[pos] = (int32_t)key;
    }
  }
}

// lc_check_frontiers: one wavefront per key runs the LDS tier's search up to
// the :ok return of record stop_op[key] and writes the frontier that return
// expands (knossos's :configs for an invalid key whose stop_op is its fail
// op) to out[key * max ...]; n_out[key] as DumpReq::n.
// One key's search up to the :ok return of its record stop (DumpReq); the
// count written, or -1.
template <class Store>
__device__ int dump_key(const lc_op *__restrict__ ops, const int64_t *__restrict__ key_off,
                        int64_t key, int64_t stop, const KParams &p, Store &st,
                        lc_fx_config *out, int max, int lane) {
  const int64_t beg = key_off[key], end = key_off[key + 1];
  DumpReq dr{(int)stop, kNever, out, max, -1};
  if (end > beg && end - beg <= 0x7FFFFFFF && stop >= 0 && stop < end - beg) {
    const lc_op *kops = ops + (beg - key_off[0]);
    const int64_t b0 = kops[0].call, r = kops[stop].ret;
    if (r != kInf && r - b0 >= 0 && r - b0 < (int64_t)kNever) {  // (an :ok op's return)
      dr.stop_ret = (uint32_t)(r - b0);
      KeyOut o;
      check_key<Store, true>(kops, (int)(end - beg), p, st, o, lane, &dr);
    }
  }
  return dr.n;
}

// lc_check_frontiers: one wavefront per key runs the LDS tier's search up to
// the :ok return of record stop_op[key] and writes the frontier that return
// expands (knossos's :configs for an invalid key whose stop_op is its fail
// op) to out[key * max ...]; n_out[key] as DumpReq::n.  A key whose search
// outgrows the LDS regions (-1) is listed in retry (count *n_retry) for
// frontier_dump_hbm_kernel.
__global__ __launch_bounds__(kWave *kWavesPerWG) void frontier_dump_kernel(
    const lc_op *__restrict__ ops, const int64_t *__restrict__ key_off,
    const int64_t *__restrict__ stop_op, const int64_t n_keys, const KParams p,
    lc_fx_config *__restrict__ out, const int max, int32_t *__restrict__ n_out,
    int32_t *__restrict__ retry, int32_t *__restrict__ n_retry) {
  __shared__ Cfg lds[kWavesPerWG][3][kLdsCap];
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int64_t key = (int64_t)blockIdx.x * kWavesPerWG + wid;
  if (key >= n_keys) return;
  LdsStore st{&lds[wid][0][0]};
  const int n = dump_key(ops, key_off, key, stop_op[key], p, st, out + key * max, max, lane);
  if (lane == 0) {
    n_out[key] = n;
    if (n < 0) retry[atomicAdd(n_retry, 1)] = (int32_t)key;
  }
}

// ==================================================================
// Version-order fast tier (every key first).
//
// For a key whose :ok writes/CAS all carry a version and which has no crashed
// writes/CAS, the model pins the mutation order: the op with version v is the
// (v - init_version)-th mutation (register.clj:64-75).  Linearizability then
// reduces to (SURVEY.md §7 "version pinning"; exact, checked against the
// oracle's searches in tests/):
//   * versions init+1 .. init+M each held by exactly one mutation;
//   * each CAS's expected value equals the value before it (register.clj:77);
//   * each read [v x] sees version v and, when x is non-nil, the value at v;
//   * increasing linearization points t_1 < ... < t_M exist with
//       L_k < t_k < U_k,  L_k = max(call(m_k), calls of reads of version k-1),
//                         U_k = min(ret(m_k),  rets of reads of version k),
//     i.e. max(L_1..L_k) < U_k for every k (a prefix-max scan).
// Reads place themselves between t_v and t_{v+1}; crashed or [nil nil] reads
// never constrain.  One 256-thread workgroup decides one key from LDS tables
// filled by LDS atomics; keys it cannot decide (crashed mutations, nil
// versions, a read [nil x], more than kFastMax records, malformed records) or
// finds invalid are handed to the JIT search, which also names the canonical
// counterexample.
#ifndef LC_FAST_DEV
#define LC_FAST_DEV 0  // dev timing switches (tools/build_variants.sh); 0 in the product
#endif
// The version-order and fused kernels: one workgroup per key (0), or
// persistent workgroups that issue the next key's loads while deciding a key
// from LDS (1, fast_run; more VGPRs per thread, measured slower: DESIGN.md).
#ifndef LC_PIPE
#define LC_PIPE 0
#endif
// The version-order tier's pass 1: the case analysis the fused and
// crash-light passes run (1), or a branch-free form (0, A/B: 952 -> 723
// instructions and 52 -> 10 branches per wave, but 61 -> 76 VGPRs in
// fast_tier_kernel and 17 spilled in the resident grid's 80: C2's kernel
// unchanged, the resident 1,250-key request 15.1 -> 21.3 us;
// profiles/r06/pass_ab.txt)
#ifndef LC_FAST_P1_BRANCHY
#define LC_FAST_P1_BRANCHY 1
#endif
// The resident grid's decision: the version-order tier's two record passes
// (1), or value claims as LDS compare-and-swaps in the one pass (0, as the
// fused pass)
#ifndef LC_RES_TWO_PASS
#define LC_RES_TWO_PASS 1
#endif
// The other workgroups' polls of workgroup 0's copy: s_sleep between polls,
// and one word per poll (1) or every word (0)
#ifndef LC_RES_SLEEP
#define LC_RES_SLEEP 4
#endif
#ifndef LC_RES_POLL1
#define LC_RES_POLL1 0
#endif
constexpr int kFastThreads = 256;
constexpr int kFastWaves = kFastThreads / kWave;
constexpr int kFastMax = kFastMaxRecords;
constexpr int kPer = kFastMax / kFastThreads;  // records per thread

__device__ __forceinline__ uint32_t umax(uint32_t a, uint32_t b) { return a > b ? a : b; }

// Inclusive max-scan inside each 16-lane row: four DPP row_shr steps (lanes
// shifted in from outside the row read 0, the identity).
__device__ __forceinline__ uint32_t row_max_scan(uint32_t v) {
  v = umax(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false));
  v = umax(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false));
  v = umax(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false));
  v = umax(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false));
  return v;
}

// Maximum of v over the wave (wave-uniform): the DPP butterfly of
// wave_min_u32 with max.
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = umax(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false));
  v = umax(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false));
  v = umax(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x141, 0xF, 0xF, false));
  v = umax(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x140, 0xF, 0xF, false));
  return umax(umax((uint32_t)__builtin_amdgcn_readlane((int)v, 0),
                   (uint32_t)__builtin_amdgcn_readlane((int)v, 16)),
              umax((uint32_t)__builtin_amdgcn_readlane((int)v, 32),
                   (uint32_t)__builtin_amdgcn_readlane((int)v, 48)));
}

// A key's result: a plain store, or (WT, the resident grid) write-through
// eight-byte stores (sc1) that leave no line behind in this XCD's L2, so a
// reader on any XCD sees them once the storing lane's stores have drained.
typedef __attribute__((address_space(1))) uint64_t gu64_t;
typedef __attribute__((address_space(1))) int64_t gi64_t;
typedef __attribute__((address_space(1))) uint32_t gu32_t;
template <bool WT>
__device__ __forceinline__ void put_result(lc_key_result *o, const lc_key_result &r) {
  if constexpr (WT) {
    static_assert(sizeof(lc_key_result) == 40, "five words");
    uint64_t w[5];
    __builtin_memcpy(w, &r, sizeof(w));
    gu64_t *g = (gu64_t *)o;
#pragma unroll
    for (int i = 0; i < 5; i++) __hip_atomic_store(g + i, w[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    *o = r;
  }
}

// Hand key over to the JIT tier (thread 0 only); tell the host there is work.
// Hand key over (thread 0 only): a plain store of its flag (1: gap tier;
// 2: jit-only — an :ok mutation without a version, a read [nil x],
// malformed records).  The host is told there is work by one store to host
// memory: a store over PCIe per handoff costs ~50 ns each (10k handed-over
// keys: 0.11 -> 0.67 ms), so a workgroup stores only if the device-side
// any_handoff word still reads 0 (a few racing stores at most).
__device__ __forceinline__ void fast_tier_handoff(int64_t key, int32_t *flags, KStatus *status,
                                                  int32_t *h_handoff, bool jit_only, int *raised) {
  flags[key] = jit_only ? 2 : 1;
  // once per workgroup (the persistent kernels decide many keys each): the
  // device-side word is read with every load in flight drained first
  if (*raised) return;
  *raised = 1;
  if (__hip_atomic_load(&status->any_handoff, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
    __hip_atomic_store(&status->any_handoff, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(h_handoff, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    // wait until the host can see it: the host reads the flag after an
    // event created without a system-scope fence (lincheck.cpp), so the
    // writer, not the event, makes the store visible before the kernel ends
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
  }
}

// 14.5 KB of LDS per workgroup (7 workgroups per CU at 72 VGPRs).
// Index k of A/B is mutation position k (version V0+k+1):
//   A[k] = max(call(m_k), calls of reads of version V0+k) + 1     (= L_k + 1)
//   B[k] = min(ret(m_k),  rets of reads of version V0+k+1)        (= U_k)
// Both are single LDS atomics per record.  Val[k] is the value the state at
// version V0+k+1 must hold, claimed with one LDS compare-and-swap from kAny
// by every record that fixes it — the mutation placed at k (its value), the
// reads of that version and a CAS pinned right after it (their values and
// expectations): two different claims fail the key whatever order they land
// in, so the value checks need no second pass over the records.  Own[k] is
// the key-relative record index of the mutation placed at k (a plain store;
// two mutations on one version leave a position unheld below the count of
// placed ones, which the decision checks).  Per-wave summaries (counts,
// flags, extents, verdicts) go to per-wave slots, so there are no
// same-address atomics and no slots to clear.
struct FastLds {
  uint32_t A[kFastMax + 4], B[kFastMax];  // 16-byte aligned rows (timing check)
  int Val[kFastMax + 4];       // kAny: nothing claimed (cleared with A/B)
  uint16_t Own[kFastMax + 4];  // 0xFFFF: no mutation placed (cleared with A/B)
  uint32_t wsum[kFastWaves];  // per wave: mutations placed | kSum* flags
  uint32_t wext[kFastWaves];  // per wave: max(last placed position + 1, highest read version)
  uint32_t wbad[kFastWaves];  // per wave: 1 if a hole or timing condition failed
  int wg[4 * kFastWaves];     // crash-light path: per-wave words (below)
  // calls of each wave's first and last record per chunk: the order check
  // across wave boundaries (lane 0's predecessor is another wave's lane 63)
  uint32_t first_call[kPer][kFastWaves], last_call[kPer][kFastWaves];
  int64_t base;  // the key's first call (thread 0 publishes it at the LDS init)
  int raised;    // this workgroup has raised the handoff flag (thread 0 only)
};

// Pass 1's per-wave flags (FastLds::wsum, above the count of placed
// mutations).  Any of the first five makes the key ineligible for the version
// order; only kSumInel alone (crashed writes/CAS without a version) leaves it
// to the crash-light decision.  kSumVbad: a value claim failed (the version
// order finds the key invalid; the crash-light decision hands it over).
constexpr uint32_t kSumInel = 1u << 16;    // crashed write/CAS, or an :ok one without a version
constexpr uint32_t kSumBad = 1u << 17;     // a version no state reaches
constexpr uint32_t kSumJit = 1u << 18;     // jit-only (malformed, unknown :f, [nil x] read, ...)
constexpr uint32_t kSumGiveup = 1u << 19;  // a crashed write/CAS carrying a version
constexpr uint32_t kSumOvf = 1u << 20;     // more crashed writes/CAS in a wave than its stash holds
constexpr uint32_t kSumElig = 0x1Fu << 16;
constexpr uint32_t kSumVbad = 1u << 21;

// One thread's records of one key, as loaded (decoded only once they land).
struct FastRecs {
  Raw w[kPer];
};

// Issue every load of this thread's records without waiting: up to 4 x 48 B
// per thread, 48 KB per workgroup in flight.  Vector loads only: a scalar
// load in flight holds up every LDS wait (lgkmcnt) of the key the persistent
// kernels decide meanwhile, so the order check takes lane 0's predecessor
// from LDS (FastLds::last_call) and the key's first call arrives the same way.
__device__ __forceinline__ void fast_issue(const lc_op *__restrict__ kops, int n, int tid,
                                           FastRecs &b) {
#pragma unroll
  for (int u = 0; u < kPer; u++) {
    const int r = tid + u * kFastThreads;
    if (r < n) {
      const longlong2 *q = reinterpret_cast<const longlong2 *>(kops + r);
      b.w[u].a = q[0];
      b.w[u].b = q[1];
      b.w[u].c = q[2];
    } else {
      // (defined either way: the persistent kernels' registers then carry no
      // value of the key before across the loads)
      b.w[u].a = b.w[u].b = b.w[u].c = make_longlong2(0, 0);
    }
  }
}

// The same records as lc_op32 (ABI 4): one thread's 24-byte records as
// loaded — (f, value), (expected, version), (call, ret) — widened to the
// 48-byte form only as pass 1 reads each (rec_raw), so the registers in
// flight are half the 48-byte path's.  rec_raw widens exactly as
// widen32_kernel does (the key's base re-added, LC_INF32 -> kInf), so every
// decision equals the one on widened records.
struct Raw32 {
  int2 a, b, c;
};
struct FastRecs32 {
  Raw32 w[kPer];
};

__device__ __forceinline__ void fast_issue(const lc_op32 *__restrict__ kops, int n, int tid,
                                           FastRecs32 &b) {
#pragma unroll
  for (int u = 0; u < kPer; u++) {
    const int r = tid + u * kFastThreads;
    if (r < n) {
      const int2 *q = reinterpret_cast<const int2 *>(kops + r);
      b.w[u].a = q[0];
      b.w[u].b = q[1];
      b.w[u].c = q[2];
    } else {
      b.w[u].a = b.w[u].b = b.w[u].c = make_int2(0, 0);
    }
  }
}

__device__ __forceinline__ const Raw &rec_raw(const FastRecs &b, int u, int64_t) { return b.w[u]; }
__device__ __forceinline__ Raw rec_raw(const FastRecs32 &b, int u, int64_t kbase) {
  const Raw32 &q = b.w[u];
  Raw r;
  r.a = make_longlong2((int64_t)q.a.x, (int64_t)q.a.y);
  r.b = make_longlong2((int64_t)q.b.x, (int64_t)q.b.y);
  const uint32_t call = (uint32_t)q.c.x, ret = (uint32_t)q.c.y;
  r.c = make_longlong2(kbase + (int64_t)call, ret == LC_INF32 ? kInf : kbase + (int64_t)ret);
  return r;
}
// the key's first call (decode's base), a scalar load beside the records'
__device__ __forceinline__ int64_t first_call(const lc_op *__restrict__ k, int64_t) { return k[0].call; }
__device__ __forceinline__ int64_t first_call(const lc_op32 *__restrict__ k, int64_t kbase) {
  return kbase + (int64_t)k[0].call;
}

// Timing condition max(A[0..k]) - 1 < B[k] for every position k < M (A holds
// L + 1).  Thread t owns positions 4t..4t+3 (16-byte LDS reads).  The max
// over earlier positions is: a DPP row scan, the row totals (v_readlane), and
// for waves w > 0 the max of A over the earlier waves' positions, which the
// wave reads itself (3 x 16 B per lane at most) instead of waiting at a
// barrier for the other waves' totals.  Returns true if a position fails.
__device__ __forceinline__ bool timing_fails(const FastLds &s, int M, int tid) {
  const int lane = tid & (kWave - 1), w = tid / kWave, row = lane >> 4;
  const int k0 = 4 * tid;
  uint4 a = make_uint4(0, 0, 0, 0), b = make_uint4(kNever, kNever, kNever, kNever);
  if (k0 < M) {
    a = reinterpret_cast<const uint4 *>(s.A)[tid];
    b = reinterpret_cast<const uint4 *>(s.B)[tid];
  }
  // positions >= M do not exist: neutral values
  if (k0 + 1 >= M) a.y = 0, b.y = kNever;
  if (k0 + 2 >= M) a.z = 0, b.z = kNever;
  if (k0 + 3 >= M) a.w = 0, b.w = kNever;
  // max of A over the positions of earlier waves (4 * kWave per wave)
  uint32_t ew = 0;
#pragma unroll
  for (int j = 0; j < kFastWaves - 1; j++) {
    const int kj = 4 * (j * kWave + lane);
    if (j < w && kj < M) {
      uint4 e = reinterpret_cast<const uint4 *>(s.A)[j * kWave + lane];
      if (kj + 1 >= M) e.y = 0;
      if (kj + 2 >= M) e.z = 0;
      if (kj + 3 >= M) e.w = 0;
      ew = umax(ew, umax(umax(e.x, e.y), umax(e.z, e.w)));
    }
  }
  const uint32_t pre = w ? wave_max_u32(ew) : 0u;
  const uint32_t p1 = umax(a.x, a.y), p2 = umax(p1, a.z), p3 = umax(p2, a.w);
  const uint32_t rs = row_max_scan(p3);
  uint32_t ex = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)rs, 0x111, 0xF, 0xF, false);
  const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)rs, 15);
  const uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)rs, 31);
  const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)rs, 47);
  const uint32_t r01 = umax(r0, r1);
  ex = umax(umax(ex, pre), row == 0 ? 0u : row == 1 ? r0 : row == 2 ? r01 : umax(r01, r2));
  // need max call < U, i.e. prefix max of A (= call + 1) <= B
  return ((int)(umax(ex, a.x) > b.x) | (int)(umax(ex, p1) > b.y) |
          (int)(umax(ex, p2) > b.z) | (int)(umax(ex, p3) > b.w)) != 0;
}

// ---------------------------------------------------------------------------
// Crash-light keys decided in place.  A key whose only obstacle to the
// version order is a few crashed writes/CAS (a partition nemesis leaves a
// few percent of them, bench.py's crash_leg) is the gap tier's case, but its
// records are already in registers and its pinned positions already folded
// into A / B / Val / Own: the workgroup finishes the gap tier's decision
// here (gap_tier.hip, same procedure and same matching, gapmatch.h) instead
// of handing the key over for a second record pass.
//   * unheld positions below M = max(last pinned position + 1, last read
//     version) are the gaps; Val of a gap holds its value requirement,
//     claimed with atomicCAS by the reads of the version it writes and by a
//     pinned CAS right after it (two different claims: invalid);
//   * timing is the version order's own check over A / B (gap positions
//     carry the read bounds), and a gap's deadline is min(B[k..M-1]);
//   * the optional ops (crashed writes/CAS) and the gaps are compacted in
//     call / position order into dynamic LDS and wave 0 runs the gap
//     tier's matching over them.
// A valid key is decided here (and its witness completed: the matched ops'
// positions); anything else — invalid (the gap tier bisects for the fail
// op), more than kFgMaxGaps gaps or kFgMaxOps optional ops, a crashed op
// that carries a version, the branch budget — is handed over as before.
#ifndef LC_FG_MAXGAPS
#define LC_FG_MAXGAPS 48
#endif
#ifndef LC_FG_MAXOPS
#define LC_FG_MAXOPS 96
#endif
constexpr int kFgMaxGaps = LC_FG_MAXGAPS;
constexpr int kFgMaxOps = LC_FG_MAXOPS;
// dynamic LDS: the matching region at its largest (gapmatch.h layout without
// the class table: 16 B + 5 ints per gap, 16 B + 7 ints per op), then the
// optional ops' record indices and the branch stack (gap, value)
constexpr int kFgMatchBytes = 36 * kFgMaxGaps + 44 * kFgMaxOps;
constexpr int kFgLdsBytes = kFgMatchBytes + 4 * kFgMaxOps + 8 * kFgMaxGaps;
// Pass 1 stashes each wave's optional ops — (call, value, expectation or
// kAny, record index), in record order — at the matching region's end, up to
// kFgStash per wave (more: the key is handed over); the decision moves them
// into place.  Inside the region, so the LDS per workgroup (and 7 per CU)
// stays as it was.
constexpr int kFgStash = 32;
constexpr int kFgStashOff = kFgMatchBytes - 16 * kFgStash * 4;
static_assert(kFgStashOff >= 0 && kFgStashOff % 16 == 0, "stash inside the matching region");

// Exclusive suffix minimum over the workgroup's threads (those above this
// one), with the wave totals through s.wg[8..11]; one barrier.
__device__ __forceinline__ uint32_t fg_suffix_min_excl(uint32_t v, FastLds &s, int tid) {
  const int lane = tid & (kWave - 1), w = __builtin_amdgcn_readfirstlane(tid / kWave);
  uint32_t incl;
  uint32_t excl = wave_suffix_min_excl(v, lane, kNever, &incl);
  if (lane == 0) s.wg[8 + w] = (int)incl;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kFastWaves; j++)
    if (j > w) excl = umin(excl, (uint32_t)s.wg[8 + j]);
  return excl;
}

// Exclusive prefix sum over the workgroup's threads, wave totals through
// s.wg[12..15]; *total = the sum.  Shares the caller's next barrier: the
// caller reads the result only after one.
__device__ __forceinline__ int fg_prefix_wave(int v, FastLds &s, int tid) {
  const int lane = tid & (kWave - 1), w = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int incl = wave_prefix_sum(v, lane);
  if (lane == kWave - 1) s.wg[12 + w] = incl;
  return incl - v;
}

// Returns true when the key was decided valid here; false: hand it over.
// Works from LDS alone: pass 1 (fast_key) already claimed the values, took
// the extents and stashed the optional ops (kFgStash per wave, in record
// order), so the records' registers are free for the next key's loads
// (the persistent version-order / fused kernels) while this runs.
// NM: mutations placed by pass 1 over the workgroup.
__device__ __forceinline__ bool fast_gap(int64_t key, int n, int NM, const KParams &p, FastLds &s,
                         lc_key_result *__restrict__ out, int32_t *__restrict__ wit,
                         int32_t *__restrict__ kind, int tid) {
  FGP_T(17);
  const int lane = tid & (kWave - 1), w = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int init = p.init_val;
  // a value claim failed: invalid (the gap tier names the fail op)
  {
    const uint4 ws = *reinterpret_cast<const uint4 *>(s.wsum);
    if ((ws.x | ws.y | ws.z | ws.w) & kSumVbad) return false;
  }
  // extent M: past the last placed position and the highest read version
  int M;
  {
    const uint4 we = *reinterpret_cast<const uint4 *>(s.wext);
    M = (int)umax(umax(we.x, we.y), umax(we.z, we.w));
  }
  // optional-op slots: chunk-major, then wave, then lane (= record order)
  int n_opt = 0;
#pragma unroll
  for (int u = 0; u < kPer; u++)
#pragma unroll
    for (int j = 0; j < kFastWaves; j++) n_opt += reinterpret_cast<const uint8_t *>(&s.wg[4 + j])[u];
  if (n_opt > kFgMaxOps) return false;
  // this wave's stashed ops (one per lane) leave LDS before the compaction
  // below can overwrite the stash (it lies at the matching region's end)
  const uint32_t mycnt = (uint32_t)s.wg[4 + w];
  const int mytot = (int)((mycnt & 0xFF) + ((mycnt >> 8) & 0xFF) + ((mycnt >> 16) & 0xFF) + (mycnt >> 24));
  int4 mine = make_int4(0, 0, 0, 0);
  FGP_T(13);
  if (lane < mytot)
    mine = reinterpret_cast<const int4 *>(reinterpret_cast<const char *>(lds_dyn) + kFgStashOff)[w * kFgStash + lane];
  // deadlines: Uh[k] = min(B[k..M-1]) for this thread's positions 4t..4t+3
  uint32_t bmin = kNever;
  int gapc = 0;
  {
    const uint4 b4 = reinterpret_cast<const uint4 *>(s.B)[tid];
    const uint2 own2 = reinterpret_cast<const uint2 *>(s.Own)[tid];
    const uint32_t bb[4] = {b4.x, b4.y, b4.z, b4.w};
    const uint32_t oo[4] = {own2.x & 0xFFFF, own2.x >> 16, own2.y & 0xFFFF, own2.y >> 16};
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int k = 4 * tid + j;
      bmin = umin(bmin, k < M ? bb[j] : kNever);
      gapc += (k < M) && oo[j] == 0xFFFF;
    }
  }
  FGP_T(14);
  const int gpre = fg_prefix_wave(gapc, s, tid);
  FGP_T(15);
  const uint32_t after = fg_suffix_min_excl(bmin, s, tid);
  FGP_T(10);
  // (the barrier inside fg_suffix_min_excl also publishes s.wg[12..15])
  int G = 0, gbase = gpre;
#pragma unroll
  for (int j = 0; j < kFastWaves; j++) {
    G += s.wg[12 + j];
    if (j < w) gbase += s.wg[12 + j];
  }
  // the timing verdict, gathered per wave (s.wbad is free on this path)
  const bool tbad = __ballot(timing_fails(s, M, tid)) != 0;
  if (lane == 0) s.wbad[w] = tbad;
  if (G > kFgMaxGaps) return false;
  // every placed mutation sits below M: M - G held positions for NM of them,
  // fewer when two share a version (invalid)
  if (M - G != NM) return false;
  // compact gaps and optional ops into the matching region (lds_dyn)
  Cmp<true> c;
  c.ws = nullptr;
  c.G = G;
  c.n_opt = n_opt;
  c.cap = 0;
  c.moff = 0;
  int *opt_rec = reinterpret_cast<int *>(lds_dyn) + kFgMatchBytes / 4;
  int *brPos = opt_rec + kFgMaxOps, *brVal = brPos + kFgMaxGaps;
  if (gapc) {
    // this thread's positions high to low: the suffix minimum runs down
    uint32_t uh = after;
    int gi = gbase + gapc;
    const uint4 b4 = reinterpret_cast<const uint4 *>(s.B)[tid];
    const uint2 own2 = reinterpret_cast<const uint2 *>(s.Own)[tid];
    const int4 v4 = reinterpret_cast<const int4 *>(s.Val)[tid];
    const int vprev = tid == 0 ? init : s.Val[4 * tid - 1];
    const uint32_t bb[4] = {b4.x, b4.y, b4.z, b4.w};
    const uint32_t oo[4] = {own2.x & 0xFFFF, own2.x >> 16, own2.y & 0xFFFF, own2.y >> 16};
    const int vv[5] = {vprev, v4.x, v4.y, v4.z, v4.w};
#pragma unroll
    for (int j = 3; j >= 0; j--) {
      const int k = 4 * tid + j;
      uh = umin(uh, k < M ? bb[j] : kNever);
      if ((k < M) && oo[j] == 0xFFFF) {
        gi--;
        c.gaps()[gi] = make_int4((int)uh, vv[j + 1], vv[j], k);
        c.at(aMG, gi) = -1;
      }
    }
  }
  if (lane < mytot) {
    // stash item `lane` of this wave: chunk u where the wave's running count
    // passes it; its slot = ops of earlier chunks + earlier waves' ops of u
    int lo = 0, o = 0;
#pragma unroll
    for (int u = 0; u < kPer; u++) {
      const int cu = (int)((mycnt >> (8 * u)) & 0xFF);
      int before = 0, tot = 0;
#pragma unroll
      for (int j = 0; j < kFastWaves; j++) {
        const int cnt = reinterpret_cast<const uint8_t *>(&s.wg[4 + j])[u];
        before += j < w ? cnt : 0;
        tot += cnt;
      }
      if (lane >= lo && lane < lo + cu) o += before + (lane - lo);
      else if (lane >= lo + cu) o += tot;
      lo += cu;
    }
    c.ops()[o] = make_int4(mine.x, mine.y, mine.z, -1);
    c.at(aMO, o) = -1;
    c.at(aVis, o) = 0;
    opt_rec[o] = mine.w;
  }
  __syncthreads();
  FGP_T(11);
  {
    const uint4 tb = *reinterpret_cast<const uint4 *>(s.wbad);
    if (tb.x | tb.y | tb.z | tb.w) return false;
  }
  if (G > n_opt) return false;  // invalid: the gap tier names the fail op
#ifdef LC_FG_NOMATCH  // dev timing only: everything but the matching
  if (tid == 0) out[key] = lc_key_result{LC_VALID, LC_REASON_NONE, -1, -1, 0, G};
  return true;
#endif
  int res = GD_VALID;
  int64_t nodes = 0;
  if (G > 0 && w == 0) {
    ClsSt cst;  // (generic matching: at most kFgMaxOps < kClsMinOps optional ops)
    cst.K = 0;
    res = match_branch_m<true, false, false>(c, G, n_opt, brPos, brVal, brVal, &nodes, cst);
    if (lane == 0) s.wg[0] = res;
    if (res == GD_VALID && wit)
      for (int gi = lane; gi < G; gi += kWave) wit[opt_rec[c.at(aMG, gi)]] = c.gaps()[gi].w;
  }
  __syncthreads();
  FGP_T(12);
  FGP_ADD(3, 10, 11);
  FGP_ADD(4, 11, 12);
  FGP_ADD(5, 17, 13);
  FGP_ADD(6, 13, 14);
  if (G > 0) res = s.wg[0];
  if (res != GD_VALID) return false;
  if (tid == 0) {
    out[key] = lc_key_result{LC_VALID, LC_REASON_NONE, -1, -1, nodes, G};
    if (kind) kind[key] = LC_WITNESS_FULL;
  }
  FGP_T(16);
  FGP_ADD(7, 12, 16);
  return true;
}

// ---------------------------------------------------------------------------
// First failure of an invalid version-pinned key, in O(n) (round 4).
//
// A key the version order decides invalid needs its canonical fail op: the
// first :ok return r whose history prefix is not linearizable (knossos.linear
// empties its frontier there).  The gap tier found it by bisection over
// prefixes — nine dependent decisions for a 200-op key.  For a key with no
// crashed ops the prefix's choices collapse, and r follows from one pass.
//
// The prefix at return r: ops called before r; those returned by r are
// required, the others pending (optional, no return bound).  A pending read
// is left out.  Position p (version V0+p+1) is *needed* once a required op
// needs it — a mutation at p' >= p, or a read of version V0+k with k > p —
// from N(p) = min{ret(o) : need(o) > p} on (need = pos+1 for a mutation, k
// for a read; a suffix minimum over positions).  A needed position is held
// by the required mutation on it if there is one, else by a pending one.
// With one mutation per position the set S(r) of ops in the linearization is
// forced: m_p enters at N(p) (its own return at the latest), a read at its
// return; extra pending mutations only add constraints, so S(r) is minimal,
// and it grows with r.  The version-order conditions on S(r) are a
// conjunction whose terms, once present and false, stay false (L only grows,
// U only falls as pending ops return), so r* = the earliest time any term is
// present and false:
//   * hole: p needed before its mutation is called (or p has none): N(p);
//   * CAS at p against the value at p-1, once both are in: N(p) (N rises
//     with p);
//   * read [V0+k x] against the value at k-1: its return;
//   * timing: an op a with call(a) > ret(b) for some b whose U bound sits at
//     or after a's L bound (Uh = the suffix minimum of B, with final
//     returns: b returned before a was called, so b is in): a's entry time
//     (N(p) for m_p, the return for a read);
//   * a version no state reaches (below V0, or more positions than records):
//     the op's return.
// Two mutations on one version (a lost CAS shapes exactly that): m*, the
// one returning first, holds the position; the other enters only as the
// second required op of it, a violation at its return.  The rule, using m*,
// is then exact unless at r* the position is needed with m* still pending
// and another of its mutations already called — a real choice: the key is
// handed over (the gap tier bisects), which is rare (tests/test_oracle.py:
// `test_first_failure_rule_matches_search` restates the rule in
// tests/fastpath_ref.py and checks it against knossos.linear's fail op on
// thousands of keys, dup-version keys included; it declines ~2 %).  Prefix
// closure makes r* the first failure: every earlier prefix is linearizable
// by S(r) itself (the witness written here, certified independently by
// oracle/witness.c in the GPU tests).
//
// Runs where the version order's tables are already in LDS and the records
// in registers (crash-light pass / fused pass), so it costs one more pass
// over registers and five barriers.  LDS: A is reused for the earliest
// return of each position's mutations, B becomes its suffix minimum Uh, the
// dynamic region holds N, Own/Val are rewritten by m*.  Returns true when the
// key was decided (result and, if wanted, its PREFIX witness written).
__device__ __forceinline__ void suffix_min2_excl(uint32_t &a, uint32_t &b, FastLds &s) {
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  uint32_t ia, ib;
  uint32_t ea = wave_suffix_min_excl(a, lane, kNever, &ia);
  uint32_t eb = wave_suffix_min_excl(b, lane, kNever, &ib);
  if (lane == 0) s.wg[8 + w] = (int)ia, s.wg[12 + w] = (int)ib;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kFastWaves; j++)
    if (j > w) ea = umin(ea, (uint32_t)s.wg[8 + j]), eb = umin(eb, (uint32_t)s.wg[12 + j]);
  a = ea;
  b = eb;
}

__device__ bool first_failure(int64_t key, int n, const lc_op *__restrict__ kops, const FastRecs &b,
                              const KParams &p, FastLds &s, lc_key_result *__restrict__ out,
                              int32_t *__restrict__ wit, int32_t *__restrict__ kind) {
  const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
  const int64_t base_idx = kops[0].call;
  const int V0 = p.init_ver, init = p.init_val;
  uint32_t *MR = s.A;                                  // earliest return of each position's mutations
  uint32_t *NR = reinterpret_cast<uint32_t *>(lds_dyn);  // ops' returns by need, then N(p)
  if (4 * tid < n) reinterpret_cast<uint4 *>(MR)[tid] = make_uint4(kNever, kNever, kNever, kNever);
  if (4 * tid <= n + 1) reinterpret_cast<uint4 *>(NR)[tid] = make_uint4(kNever, kNever, kNever, kNever);
  __syncthreads();
  uint32_t t = kNever;  // this thread's earliest violation
  // step 1: each position's earliest-returning mutation; returns by need
#pragma unroll
  for (int u = 0; u < kPer; u++) {
    const int r = tid + u * kFastThreads;
    if (r >= n) continue;
    const Rec d = decode(b.w[u], base_idx);
    if (d.f != LC_F_READ) {
      const int pos = d.ver - V0 - 1;
      if (pos < 0 || pos >= n) {
        t = umin(t, d.ret);  // no state reaches this version
      } else {
        atomicMin(&MR[pos], d.ret);
        atomicMin(&NR[pos + 1], d.ret);
      }
    } else if (d.ret != kNever && d.ver != -1) {
      const int k = d.ver - V0;
      if (k < 0 || k > n) t = umin(t, d.ret);
      else if (k > 0) atomicMin(&NR[k], d.ret);
    }
  }
  __syncthreads();
  // step 2: m* claims its position; suffix minima N(p) and Uh(p) in place
#pragma unroll
  for (int u = 0; u < kPer; u++) {
    const int r = tid + u * kFastThreads;
    if (r >= n) continue;
    const Rec d = decode(b.w[u], base_idx);
    const int pos = d.ver - V0 - 1;
    if (d.f != LC_F_READ && pos >= 0 && pos < n) {
      if (d.ret == MR[pos]) {
        s.Own[pos] = (uint16_t)r;
        s.Val[pos] = d.val;
      } else {
        t = umin(t, d.ret);  // a second mutation of the version becomes required
      }
    }
  }
  uint4 nr4 = make_uint4(kNever, kNever, kNever, kNever), b4 = nr4;
  if (4 * tid <= n + 1) nr4 = reinterpret_cast<const uint4 *>(NR)[tid];
  if (4 * tid <= n) b4 = reinterpret_cast<const uint4 *>(s.B)[tid];
  uint32_t na = umin(umin(nr4.x, nr4.y), umin(nr4.z, nr4.w));
  uint32_t ba = umin(umin(b4.x, b4.y), umin(b4.z, b4.w));
  suffix_min2_excl(na, ba, s);  // (its barrier also orders step 2's stores)
  if (4 * tid <= n + 1) {
    // N(p) = min NR[p+1 ..]; Uh(p) = min B[p ..]
    const uint32_t n3 = na, n2 = umin(n3, nr4.w), n1 = umin(n2, nr4.z), n0 = umin(n1, nr4.y);
    reinterpret_cast<uint4 *>(NR)[tid] = make_uint4(n0, n1, n2, n3);
  }
  if (4 * tid <= n) {
    const uint32_t u3 = umin(ba, b4.w), u2 = umin(u3, b4.z), u1 = umin(u2, b4.y), u0 = umin(u1, b4.x);
    reinterpret_cast<uint4 *>(s.B)[tid] = make_uint4(u0, u1, u2, u3);
  }
  __syncthreads();
  // step 3: every term's activation time
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int q = 4 * tid + j;
    if (q < n && s.Own[q] == 0xFFFF) t = umin(t, NR[q]);  // needed, never held
  }
#pragma unroll
  for (int u = 0; u < kPer; u++) {
    const int r = tid + u * kFastThreads;
    if (r >= n) continue;
    const Rec d = decode(b.w[u], base_idx);
    if (d.f != LC_F_READ) {
      const int pos = d.ver - V0 - 1;
      if (pos < 0 || pos >= n || s.Own[pos] != r) continue;
      const uint32_t np = NR[pos];
      bool v = d.call > np;  // needed before it was called
      if (d.f == LC_F_CAS) {
        if (pos == 0) v |= d.exp != init;
        else if (s.Own[pos - 1] != 0xFFFF) v |= d.exp != s.Val[pos - 1];
      }
      v |= d.call >= s.B[pos];  // called after an op bounding it from above returned
      if (v) t = umin(t, np);
    } else if (d.ret != kNever && d.ver != -1) {
      const int k = d.ver - V0;
      if (k < 0 || k > n) continue;
      bool v = false;
      if (d.val != -1) {
        if (k == 0) v = d.val != init;
        else if (s.Own[k - 1] != 0xFFFF) v = d.val != s.Val[k - 1];
      }
      if (k < n) v |= d.call >= s.B[k];
      if (v) t = umin(t, d.ret);
    }
  }
  const uint32_t wt = wave_min_u32(t);
  if (lane == 0) s.wg[w] = (int)wt;
  __syncthreads();
  const uint4 tw = *reinterpret_cast<const uint4 *>(s.wg);
  const uint32_t T = umin(umin(tw.x, tw.y), umin(tw.z, tw.w));
  if (T == kNever) return false;  // (cannot happen for an invalid key: hand it over)
  // step 4: a real choice at T (declined), and the op returning at T
  int amb = 0, fo = 0;
#pragma unroll
  for (int u = 0; u < kPer; u++) {
    const int r = tid + u * kFastThreads;
    if (r >= n) continue;
    const Rec d = decode(b.w[u], base_idx);
    if (d.ret == T) fo = r + 1;
    const int pos = d.ver - V0 - 1;
    if (d.f != LC_F_READ && pos >= 0 && pos < n && s.Own[pos] != r)
      amb |= (d.call < T) & (NR[pos] <= T) & (T < MR[pos]);
  }
  const uint32_t wfo = wave_max_u32((uint32_t)fo);
  const bool wamb = __ballot(amb) != 0;
  if (lane == 0) s.wg[4 + w] = (int)(wfo | (wamb ? 0x80000000u : 0u));
  __syncthreads();
  const int4 fw = *reinterpret_cast<const int4 *>(&s.wg[4]);
  if ((fw.x | fw.y | fw.z | fw.w) < 0) return false;  // ambiguous: the gap tier bisects
  const int fail = max(max(fw.x, fw.y), max(fw.z, fw.w)) - 1;
  if (fail < 0) return false;
  if (wit) {
    // the prefix just before T: m* of every position needed by then
#pragma unroll
    for (int u = 0; u < kPer; u++) {
      const int r = tid + u * kFastThreads;
      if (r >= n) continue;
      const Rec d = decode(b.w[u], base_idx);
      const int pos = d.ver - V0 - 1;
      const bool in = d.f != LC_F_READ && pos >= 0 && pos < n && s.Own[pos] == r && NR[pos] < T;
      wit[r] = in ? pos : -1;
    }
  }
  if (tid == 0) {
    out[key] = lc_key_result{LC_INVALID, LC_REASON_NONLINEARIZABLE, fail,
                             base_idx + (int64_t)T, 0, 1};
    if (kind) kind[key] = LC_WITNESS_PREFIX;
  }
  return true;
}

// Where a key the workgroup does not decide goes: the version-order tier
// flags it for the handoff compaction; the crash-light pass (LIGHT, over the
// compacted list) appends it to the gap tier's list.  wit / kind: lc_aux.
struct FastSinks {
  int32_t *flags;
  KStatus *status;
  int32_t *h_handoff;
  int32_t *pass;
  int32_t *wit;
  int32_t *kind;
};

// Who runs fast_key: the version-order tier over every key; the crash-light
// pass over the keys that tier handed to the gap tier; or both in one pass
// (FUSED: the version order, and for a key whose only obstacle is crashed
// writes/CAS the crash-light decision, over every key — for batches where
// most keys carry crashed ops, which would otherwise be read twice).
enum { kModeFast = 0, kModeLight = 1, kModeFused = 2 };

template <int MODE>
__device__ __forceinline__ void fast_pass_on(int64_t key, const FastSinks &o, int *raised,
                                             bool jit_only = false) {
  if constexpr (MODE == kModeLight) {
    o.pass[atomicAdd(&o.status->n_gap2, 1)] = (int32_t)key;  // few: invalid / large keys
  } else {
    // fused: status->n_light counts the keys the gap procedure takes, here
    // or in the crash-light decision (fast_key)
    if constexpr (MODE == kModeFused)
      if (!jit_only) atomicAdd(light_shard(o.status, key), 1);
    fast_tier_handoff(key, o.flags, o.status, o.h_handoff, jit_only, raised);
  }
}


// Decide one key (records in b when 0 < n64 <= kFastMax) or hand it over.
// Three barriers: after the LDS init, after pass 1, before thread 0 reads
// the per-wave verdicts.  Pass 1 is the only pass over the records (value
// claims are LDS compare-and-swaps, FastLds), so once it is done the
// records' registers are free: `next()` — called once by every thread, there
// or at once for a key with nothing to decide — lets the persistent kernels
// issue the next key's loads into them while this key is decided from LDS.
// The crash-light pass (kModeLight) keeps the records for first_failure.
// RES: the resident grid (below) — the key's first call comes through LDS
// (thread 0 holds record 0) instead of a load that may be served from a
// cache filled in an earlier request, and results are written through.
template <int MODE, typename Next, class Op = lc_op, class Recs = FastRecs, bool RES = false>
__device__ __forceinline__ void fast_key(int64_t key, int64_t n64, const Op *__restrict__ kops,
                                         int64_t kbase, const Recs &b, const KParams &p, FastLds &s,
                                         lc_key_result *__restrict__ out, const FastSinks &o,
                                         int32_t *__restrict__ wit, Next &&next) {
  // the thread index, opaque to the compiler: in the persistent kernels'
  // loop everything derived from it (LDS addresses, lane masks) would
  // otherwise be hoisted out and held in VGPRs across every key
  int tid = threadIdx.x;
  if constexpr (LC_PIPE || RES) asm volatile("" : "+v"(tid));
  const int lane = tid & (kWave - 1), w = __builtin_amdgcn_readfirstlane(tid / kWave);
  if (n64 <= 0 || n64 > kFastMax) {
    next();
    if (tid == 0) {
      if (n64 == 0)
        put_result<RES>(out + key, lc_key_result{LC_VALID, LC_REASON_NONE, -1, -1, 0, 0});
      else
        fast_pass_on<MODE>(key, o, &s.raised);
    }
    return;
  }
  const int n = (int)n64;
  FGP_T(0);
  FP_T(0);
#if LC_FAST_DEV == 2  // dev timing only: loads, no decision
  {
    int64_t x = 0;
#pragma unroll
    for (int u = 0; u < kPer; u++)
      x ^= b.w[u].a.x ^ b.w[u].a.y ^ b.w[u].b.x ^ b.w[u].b.y ^ b.w[u].c.x ^ b.w[u].c.y;
    next();
    if (x == 0x123456789) out[key].configs_explored = x;
    if (tid == 0) out[key] = lc_key_result{LC_VALID, LC_REASON_NONE, -1, -1, 0, 1};
    return;
  }
#endif
  // thread t clears positions 4t..4t+3 of A, B, Own and Val (one 16-byte
  // store each, 8 for Own); A[kFastMax] (reads of the version after the last
  // possible mutation) by thread 0, which also publishes the key's first call
  if (4 * tid <= n) {
    reinterpret_cast<uint4 *>(s.A)[tid] = make_uint4(0, 0, 0, 0);  // nothing constrains t_k from below
    reinterpret_cast<uint4 *>(s.B)[tid] = make_uint4(kNever, kNever, kNever, kNever);
    reinterpret_cast<uint2 *>(s.Own)[tid] = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
    if (MODE != kModeFast || LC_PIPE || (RES && !LC_RES_TWO_PASS))  // (claimed values start unclaimed)
      reinterpret_cast<int4 *>(s.Val)[tid] = make_int4(kAny, kAny, kAny, kAny);
  }
  int64_t base_idx;
  if constexpr (LC_PIPE || RES) {
    if (tid == 0) {
      s.A[kFastMax] = 0;
      s.base = rec_raw(b, 0, kbase).c.x;
    }
    __syncthreads();
    base_idx = s.base;
  } else {
    if (tid == 0) s.A[kFastMax] = 0;
    base_idx = first_call(kops, kbase);  // (a scalar load, beside the records')
    __syncthreads();
  }
  FGP_T(1);
  FP_T(1);
  const int V0 = p.init_ver, init = p.init_val;
  int inel = 0, bad = 0, nmut = 0, jit_only = 0, giveup = 0, vbad = 0;
  int ext = 0;  // past the last placed position and the highest read version
  int nopt = 0;        // this wave's optional ops so far (wave-uniform)
  uint32_t optc = 0;   // per chunk, one byte each
  int4 *stash = reinterpret_cast<int4 *>(reinterpret_cast<char *>(lds_dyn) + kFgStashOff) +
                w * kFgStash;
  // The version-order tier (one workgroup per key) keeps its records in
  // registers through the decision: it stores each placed mutation's value
  // and checks the claims in a second pass over the registers (measured ~2 %
  // faster on C2 than the compare-and-swaps); the fused and light passes
  // claim in pass 1 and free the records.
  constexpr bool kTwoPass = MODE == kModeFast && !LC_PIPE && !(RES && !LC_RES_TWO_PASS);
  auto claim = [&](int k, int v) {  // value v required at version V0+k+1 (k >= 0)
    if constexpr (!kTwoPass) {
      const int old = atomicCAS(&s.Val[k], kAny, v);
      vbad |= (old != kAny) & (old != v);
    }
  };
  // pass 1: place mutations, fold read intervals into A / B, claim values,
  // stash crashed writes/CAS
  if constexpr (MODE == kModeFast && kTwoPass && !LC_FAST_P1_BRANCHY) {
    // The version-order tier's pass 1, branch-free (the same placements,
    // bounds and flags as the case analysis below, which the fused and
    // crash-light passes keep): every record issues its two LDS atomics and
    // two stores, a record that places nothing aimed at a no-op — max with
    // 0, min with kNever, stores into the arrays' spare slot kFastMax + 1 —
    // so the wave runs one straight line per record instead of ~13 masked
    // branches
    constexpr int kSpare = kFastMax + 1;
#pragma unroll
    for (int u = 0; u < kPer; u++) {
      const int r = tid + u * kFastThreads;
      auto &&bw = rec_raw(b, u, kbase);
      const Rec d = decode(bw, base_idx);
      const uint32_t prev = (uint32_t)wave_shr1((int)d.call, 0);
      // (a chunk's first call is read only when its first record is live,
      // its last call only when the next chunk's first is)
      if (lane == 0) s.first_call[u][w] = d.call;
      if (lane == kWave - 1) s.last_call[u][w] = d.call;
      const bool live = r < n;
      const bool brec = live & (d.bad | (d.f > LC_F_CAS) | ((lane > 0) & (prev >= d.call)));
      const bool ok = live & !brec;
      const bool is_read = d.f == LC_F_READ;
      // reads: a returned read other than [nil nil] constrains; [nil x] is
      // the JIT tier's; a version index outside [0, n] no state reaches
      const bool rd = ok & is_read & (d.ret != kNever) & !((d.ver == -1) & (d.val == -1));
      const bool rd_nil = rd & (d.ver == -1);
      const int k = d.ver - V0;
      const bool rd_v = rd & (d.ver != -1);
      const bool rd_bad = rd_v & ((k < 0) | (k > n));
      const bool rd_ok = rd_v & !rd_bad;
      // mutations: crashed or version-less ones are not pinned
      const bool mu = ok & !is_read;
      const bool mu_crash = mu & (d.ret == kNever), mu_nover = mu & (d.ver == -1);
      const int pos = d.ver - V0 - 1;
      const bool mu_v = mu & !mu_crash & !mu_nover;
      const bool mu_bad = mu_v & ((pos < 0) | (pos >= n));
      const bool mu_ok = mu_v & !mu_bad;
      atomicMax(&s.A[rd_ok ? k : mu_ok ? pos : kSpare], (rd_ok | mu_ok) ? d.call + 1 : 0u);
      atomicMin(&s.B[rd_ok && k > 0 ? k - 1 : mu_ok ? pos : 0],
                ((rd_ok & (k > 0)) | mu_ok) ? d.ret : kNever);
      const int ps = mu_ok ? pos : kSpare;
      s.Own[ps] = (uint16_t)r;
      s.Val[ps] = d.val;
      // the claims on the initial value (the others: pass 2)
      vbad |= (int)((mu_ok & (d.f == LC_F_CAS) & (pos == 0) & (d.exp != init)) |
                    (rd_ok & (k == 0) & (d.val != -1) & (d.val != init)));
      inel |= (int)(brec | rd_nil | mu_crash | mu_nover);
      jit_only |= (int)(brec | rd_nil | (mu_nover & !mu_crash));
      giveup |= (int)(mu_crash & (d.ver != -1));
      bad |= (int)(rd_bad | mu_bad);
      nmut += __popcll(__ballot(mu_ok));
    }
  } else
#pragma unroll
  for (int u = 0; u < kPer; u++) {
    const int r = tid + u * kFastThreads;
    auto &&bw = rec_raw(b, u, kbase);

    bool placed = false;
    // crashed writes/CAS without a version (a malformed one among them
    // reserves a slot too: its key goes to the JIT tier, the stash unread)
    uint64_t m = 0;
    if constexpr (MODE != kModeFast)
      m = __ballot(r < n && (bw.a.x == LC_F_WRITE || bw.a.x == LC_F_CAS) && bw.c.y == kInf &&
                   bw.b.y == -1);
    if (r < n) {
      const Rec d = decode(bw, base_idx);
      // calls in order: the previous record's is lane-1's of the same u
      // (lane 0's predecessor is checked after the barrier, from last_call).
      // Key-relative 32-bit calls: exact when neither record is malformed,
      // and a malformed one sends the key to the JIT tier anyway
      const uint32_t prev = (uint32_t)wave_shr1((int)d.call, 0);
      if (lane == 0) s.first_call[u][w] = d.call;
      if (lane == kWave - 1) s.last_call[u][w] = d.call;
      if (d.bad || d.f > LC_F_CAS || (lane > 0 && prev >= d.call)) {
        inel = jit_only = 1;  // the JIT tier reports malformed / unknown :f
      } else if (d.f == LC_F_READ) {
        if (d.ret != kNever && !(d.ver == -1 && d.val == -1)) {  // else never constrains
          if (d.ver == -1) {
            inel = jit_only = 1;  // read [nil x]: its version is free
          } else {
            const int k = d.ver - V0;
            if (k < 0 || k > n) {
              bad = 1;
            } else {
              atomicMax(&s.A[k], d.call + 1);
              if constexpr (MODE != kModeFast) ext = max(ext, k);
              if (k > 0) atomicMin(&s.B[k - 1], d.ret);
              if (d.val != -1) {
                if (k == 0) vbad |= d.val != init;
                else claim(k - 1, d.val);
              }
            }
          }
        }
      } else if (d.ret == kNever || d.ver == -1) {
        inel = 1;  // crashed (the gap tier's case), or no version: order not pinned
        if (d.ret != kNever) jit_only = 1;
        else if (d.ver != -1) giveup = 1;  // a crashed op pinned to a version: the gap tier's
        else if constexpr (MODE != kModeFast) {
          const int slot = nopt + lanes_below(m);
          if (slot < kFgStash) stash[slot] = make_int4((int)d.call, d.val, d.f == LC_F_CAS ? d.exp : kAny, r);
        }
      } else {
        const int pos = d.ver - V0 - 1;
        if (pos < 0 || pos >= n) {
          bad = 1;
        } else {
          atomicMax(&s.A[pos], d.call + 1);
          atomicMin(&s.B[pos], d.ret);
          s.Own[pos] = (uint16_t)r;
          if constexpr (kTwoPass) s.Val[pos] = d.val;
          else claim(pos, d.val);
          if constexpr (MODE != kModeFast) ext = max(ext, pos + 1);
          if (d.f == LC_F_CAS) {
            if (pos == 0) vbad |= d.exp != init;
            else claim(pos - 1, d.exp);
          }
          placed = true;
        }
      }
    }
    nmut += __popcll(__ballot(placed));
    if constexpr (MODE != kModeFast) {
      const int c = __popcll(m);
      nopt += c;
      optc |= (uint32_t)c << (8 * u);
    }
  }
  // the records are consumed: their registers take the next key's loads
  if constexpr (MODE != kModeLight) next();
  // (ballots outside the lane-0 branch: they must see every lane)
  uint32_t fl = 0;
  if (__ballot(inel | bad | vbad)) {  // a clean valid key skips the rest
    fl = (__ballot(inel) ? kSumInel : 0u) | (__ballot(bad) ? kSumBad : 0u) |
         (__ballot(jit_only) ? kSumJit : 0u) | (__ballot(giveup) ? kSumGiveup : 0u) |
         (__ballot(vbad) ? kSumVbad : 0u) | (nopt > kFgStash ? kSumOvf : 0u);
  }
  // extents (the crash-light decision's M; the version order checks its
  // tail from the tables instead)
  uint32_t wext = 0;
  if constexpr (MODE != kModeFast) wext = wave_max_u32((uint32_t)ext);
  if (lane == 0) {
    s.wsum[w] = (uint32_t)nmut | fl;
    if constexpr (MODE != kModeFast) {
      s.wext[w] = wext;
      s.wg[4 + w] = (int)optc;
    }
  }
  __syncthreads();
  FGP_T(2);
  FP_T(2);
  uint32_t wor;
  int M;
  {
    const uint4 ws = *reinterpret_cast<const uint4 *>(s.wsum);
    wor = ws.x | ws.y | ws.z | ws.w;
    // M = mutations placed
    M = (int)((ws.x & 0xFFFF) + (ws.y & 0xFFFF) + (ws.z & 0xFFFF) + (ws.w & 0xFFFF));
  }
  {
    // the order check across wave boundaries: lane j < 16 takes the first
    // record of (chunk j / 4, wave j % 4) against its predecessor's call
    const int j = lane & 15, ju = j >> 2, jw = j & 3;
    const int r0 = jw * kWave + ju * kFastThreads;
    bool ob = false;
    if (lane < 16 && r0 > 0 && r0 < n) {
      const uint32_t pc = jw > 0 ? s.last_call[ju][jw - 1] : s.last_call[ju - 1][kFastWaves - 1];
      ob = pc >= s.first_call[ju][jw];
    }
    if (__ballot(ob)) wor |= kSumInel | kSumJit;
  }
  FGP_T(4);
#ifdef LC_FG_STOP1  // dev timing only: the fused pass stops after pass 1
  if (MODE == kModeFused) {
    if (tid == 0) out[key] = lc_key_result{LC_VALID, LC_REASON_NONE, -1, -1, 0, 1};
    return;
  }
#endif
  if (wor & kSumElig) {  // ineligible or a version out of range: hand over
    // crash-light pass: crashed writes/CAS are the only obstacle
    if constexpr (MODE != kModeFast)
      if ((wor & kSumElig) == kSumInel && fast_gap(key, n, M, p, s, out, wit, o.kind, tid)) {
        if (MODE == kModeFused && tid == 0) atomicAdd(light_shard(o.status, key), 1);
#ifdef LC_FG_PROF
        if (MODE == kModeFused) {
          FGP_T(3);
          FGP_ADD(0, 0, 1);
          FGP_ADD(1, 1, 2);
          FGP_ADD(2, 2, 3);
        }
#endif
        return;
      }
    if (tid == 0) fast_pass_on<MODE>(key, o, &s.raised, (wor & kSumJit) != 0);
    return;
  }
  if constexpr (MODE == kModeLight) {
    // eligible here too: the version order found it invalid; name its first
    // failure in place (declined: the gap tier bisects)
    if (!first_failure(key, n, kops, b, p, s, out, wit, o.kind) && tid == 0)
      fast_pass_on<MODE>(key, o, &s.raised);
    return;
  }
  // the version order: positions 0..M-1 each held once (none below M
  // unheld, none at or above M held), no read of a version past M (A[k] of
  // k > M untouched: a read of version k, or a mutation at k, would have
  // raised it), every claim agreed (pass 1), and the timing condition
  const bool uni_bad = (wor & kSumVbad) != 0;
  int hole = 0;
  if constexpr (kTwoPass) {
    // pass 2: positions, duplicates, CAS expectations and read claims
    // against the placed values.  Pass 1 raised no flag, so every record is
    // well formed, every mutation versioned, returned and placed at a
    // position in [0, n), every read's version index in [0, n].  Branch-free:
    // all eight LDS reads of a thread's four records issue together (a
    // branch per record made them eight dependent round trips, ~3,000 cycles
    // of a lone key's decision), then the checks.
    int own[kPer], before[kPer];
#pragma unroll
    for (int u = 0; u < kPer; u++) {
      auto &&bw = rec_raw(b, u, kbase);
      const int f = (int)bw.a.x, ver = (int)bw.b.y;
      // mutation: Own[pos], Val[pos - 1]; read: Val[k - 1]  (k = ver - V0)
      const int i2 = (f == LC_F_READ ? ver - V0 : ver - V0 - 1) - 1;
      const int i1 = min(max(ver - V0 - 1, 0), kFastMax - 1);
      own[u] = s.Own[i1];
      before[u] = s.Val[min(max(i2, 0), kFastMax - 1)];
    }
#pragma unroll
    for (int u = 0; u < kPer; u++) {
      const int r = tid + u * kFastThreads;
      auto &&bw = rec_raw(b, u, kbase);
      const int f = (int)bw.a.x, val = (int)bw.a.y, exp = (int)bw.b.x;
      const int ver = (int)bw.b.y;
      const bool live = r < n, is_read = f == LC_F_READ;
      const int pos = ver - V0 - 1, k = ver - V0;
      const int bv = (is_read ? k : pos) == 0 ? init : before[u];
      // a gap below the last version, a version held twice, or a CAS whose
      // expectation is not the value before it
      const bool mbad = (pos >= M) | (own[u] != r) | ((f == LC_F_CAS) & (exp != bv));
      // a version no mutation wrote, or a value that is not the one there
      const bool rbad = (k > M) | ((val != -1) & (val != bv));
      const bool rchk = is_read & (ver != -1) & (bw.c.y != kInf);
      hole |= (int)(live & ((!is_read & mbad) | (rchk & rbad)));
    }
  } else if (4 * tid <= n) {
    const uint2 own2 = reinterpret_cast<const uint2 *>(s.Own)[tid];
    const uint4 a4 = reinterpret_cast<const uint4 *>(s.A)[tid];
    const uint32_t oo[4] = {own2.x & 0xFFFF, own2.x >> 16, own2.y & 0xFFFF, own2.y >> 16};
    const uint32_t aa[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int k = 4 * tid + j;
      if (k < M) hole |= oo[j] == 0xFFFF;
      else if (k < n) hole |= (oo[j] != 0xFFFF) | ((k > M) & (aa[j] != 0));
      else if (k == n) hole |= (k > M) & (aa[j] != 0);
    }
  }
  FP_T(3);
  if (timing_fails(s, M, tid)) hole = 1;
  const uint32_t wbad = __ballot(hole) ? 1u : 0u;
  if (lane == 0) s.wbad[w] = wbad;
  __syncthreads();
  FP_T(4);
  // (the fused pass hands invalid keys over: the first-failure rule there
  // costs 5 VGPRs, 72 -> 77, and a wave per SIMD on crash-heavy batches)
  if (tid == 0) {
    const uint4 wb = *reinterpret_cast<const uint4 *>(s.wbad);
    if (!uni_bad && !(wb.x | wb.y | wb.z | wb.w))
      put_result<RES>(out + key, lc_key_result{LC_VALID, LC_REASON_NONE, -1, -1, 0, 1});
    else
      fast_pass_on<MODE>(key, o, &s.raised);
#ifdef LC_FAST_PROF
    if (MODE == kModeFast) {
      atomicAdd(&g_fp[1], (unsigned long long)(fp_t1 - fp_t0));  // records landed + LDS init
      atomicAdd(&g_fp[2], (unsigned long long)(fp_t2 - fp_t1));  // pass 1 (placement, bounds)
      atomicAdd(&g_fp[3], (unsigned long long)(fp_t3 - fp_t2));  // order check, pass 2 (claims)
      atomicAdd(&g_fp[4], (unsigned long long)(fp_t4 - fp_t3));  // timing scan + barrier
      atomicAdd(&g_fp[5], (unsigned long long)(__builtin_amdgcn_s_memtime() - fp_t4));  // result
    }
#endif
  }
}

// The version-order and fused kernels: persistent workgroups (as many as
// are resident, lincheck.cpp sizes the grid), each deciding keys blockIdx.x,
// + gridDim.x, ... .  A key's loads are issued while the key before it is
// decided from LDS (fast_key's next()): one register set, the records in
// flight during the decision instead of the decision and the loads taking
// turns.  The next key's offsets come one key ahead, by vector loads (two
// lanes) for the same reason as fast_issue's.
template <int MODE>
__device__ __forceinline__ void fast_run(const lc_op *__restrict__ ops,
                                         const int64_t *__restrict__ key_off, int64_t n_keys,
                                         const KParams &p, FastLds &s,
                                         lc_key_result *__restrict__ out, const FastSinks &o) {
  const int tid = threadIdx.x, lane = tid & (kWave - 1);
  const int64_t off0 = key_off[0];
  int64_t key = blockIdx.x;
  if (key >= n_keys) return;
  if (tid == 0) s.raised = 0;
  int64_t beg = key_off[key], end = key_off[key + 1];
  FastRecs r;
  if (end - beg > 0 && end - beg <= kFastMax) fast_issue(ops + (beg - off0), (int)(end - beg), tid, r);
  // the next key's offsets (lanes 0 and 1)
  int64_t nx = key + gridDim.x;
  int64_t offv = 0;
  if (nx < n_keys && lane < 2) offv = key_off[nx + lane];
  for (;;) {
    int64_t nbeg = 0, nend = 0;
    const int64_t nx2 = nx + gridDim.x;
    auto next = [&]() {
      nbeg = __shfl(offv, 0);
      nend = __shfl(offv, 1);
      const int64_t nn = nx < n_keys ? nend - nbeg : 0;
      fast_issue(ops + (nbeg - off0), nn > 0 && nn <= kFastMax ? (int)nn : 0, tid, r);
      if (nx2 < n_keys && lane < 2) offv = key_off[nx2 + lane];
    };
    fast_key<MODE>(key, end - beg, ops + (beg - off0), 0, r, p, s, out, o,
                   o.wit ? o.wit + (beg - off0) : nullptr, next);
    if (nx >= n_keys) break;
    key = nx;
    beg = nbeg;
    end = nend;
    nx = nx2;
  }
}

template <int MODE>
__device__ __forceinline__ void fast_one(const lc_op *__restrict__ ops,
                                         const int64_t *__restrict__ key_off, int64_t key,
                                         const KParams &p, FastLds &s,
                                         lc_key_result *__restrict__ out, const FastSinks &o) {
#ifdef LC_FAST_PROF
  const uint64_t fp_e = __builtin_amdgcn_s_memtime();
#endif
  const int64_t beg = key_off[key], end = key_off[key + 1];
  const lc_op *kops = ops + (beg - key_off[0]);
#ifdef LC_FAST_PROF
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (MODE == kModeFast && threadIdx.x == 0)
    atomicAdd(&g_fp[0], (unsigned long long)(__builtin_amdgcn_s_memtime() - fp_e));  // offsets
#endif
  FastRecs r;
  if (end - beg > 0 && end - beg <= kFastMax) fast_issue(kops, (int)(end - beg), threadIdx.x, r);
  if (threadIdx.x == 0) s.raised = 0;
  fast_key<MODE>(key, end - beg, kops, 0, r, p, s, out, o,
                 o.wit ? o.wit + (beg - key_off[0]) : nullptr, [] {});
}

// fast_one over lc_op32 records (the native 24-byte pass, kernels *32 below)
template <int MODE>
__device__ __forceinline__ void fast_one32(const lc_op32 *__restrict__ ops,
                                           const int64_t *__restrict__ key_off,
                                           const int64_t *__restrict__ key_base, int64_t key,
                                           const KParams &p, FastLds &s,
                                           lc_key_result *__restrict__ out, const FastSinks &o) {
  static_assert(!LC_PIPE, "the 24-byte pass reads its base per key, not from LDS (LC_PIPE)");
  const int64_t beg = key_off[key], end = key_off[key + 1];
  const lc_op32 *kops = ops + (beg - key_off[0]);
  const int64_t kbase = key_base ? key_base[key] : 0;
  FastRecs32 r;
  if (end - beg > 0 && end - beg <= kFastMax) fast_issue(kops, (int)(end - beg), threadIdx.x, r);
  if (threadIdx.x == 0) s.raised = 0;
  fast_key<MODE>(key, end - beg, kops, kbase, r, p, s, out, o,
                 o.wit ? o.wit + (beg - key_off[0]) : nullptr, [] {});
}

// launch_done_signal (kernels.h): the follower of a pass launch.
__global__ void done_signal_kernel(uint32_t *h_done, uint32_t seq) {
  if (threadIdx.x == 0) __hip_atomic_store(h_done, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(kFastThreads) void fast_tier_kernel(
    const lc_op *__restrict__ ops, const int64_t *__restrict__ key_off, int64_t n_keys,
    const KParams p, lc_key_result *__restrict__ out,
    int32_t *__restrict__ flags, KStatus *__restrict__ status,
    int32_t *__restrict__ h_handoff) {
  __shared__ FastLds s;
  const FastSinks o{flags, status, h_handoff, nullptr, nullptr, nullptr};
#if LC_PIPE
  fast_run<kModeFast>(ops, key_off, n_keys, p, s, out, o);
#else
  fast_one<kModeFast>(ops, key_off, blockIdx.x, p, s, out, o);
#endif
#ifdef LC_FAST_PROF
  if (threadIdx.x == 0 && atomicAdd(&g_fpdone, 1u) == gridDim.x - 1) {
    printf("fastprof keys %u offsets %llu land+init %llu pass1 %llu order+pass2 %llu timing %llu result %llu\n",
           gridDim.x, g_fp[0], g_fp[1], g_fp[2], g_fp[3], g_fp[4], g_fp[5]);
    for (int i = 0; i < 8; i++) g_fp[i] = 0;
    g_fpdone = 0;
  }
#endif
}

// The version-order tier over lc_op32 records (lc_check32 / lc_check_device32
// without lc_aux outputs): the same decision on half the bytes; a key it
// hands over is decided by the later tiers on the records widened then.
__global__ __launch_bounds__(kFastThreads) void fast_tier32_kernel(
    const lc_op32 *__restrict__ ops, const int64_t *__restrict__ key_off,
    const int64_t *__restrict__ key_base, int64_t n_keys, const KParams p,
    lc_key_result *__restrict__ out, int32_t *__restrict__ flags, KStatus *__restrict__ status,
    int32_t *__restrict__ h_handoff) {
  __shared__ FastLds s;
  const FastSinks o{flags, status, h_handoff, nullptr, nullptr, nullptr};
  if ((int64_t)blockIdx.x < n_keys) fast_one32<kModeFast>(ops, key_off, key_base, blockIdx.x, p, s, out, o);
}

// ---------------------------------------------------------------------------
// Resident grid (kernels.h, launch_fast_resident).  A C3 shard's step (1,250
// keys, ~12 us of kernel) paid ~10 us for its launch and the follower
// kernel's completion signal; a grid that stays resident between calls pays
// neither.  Memory protocol (MI355X_MICROARCH.md, inter-workgroup
// visibility): the request is copied to device memory by write-through
// stores, drained, then its number stored; every other workgroup polls that
// one word with relaxed L1-bypassing loads and reads the request with such
// loads; the records, offsets and first calls are also read L1-bypassing
// (another kernel or a copy may have rewritten them since the last request,
// while this CU's L1 still holds lines of them); results go out write-through
// and each workgroup's storing lane drains its stores before it adds to the
// arrival counter.

// sc1 loads of this thread's records through a buffer descriptor whose range
// check reads zeros past the key's end (the zero fill fast_issue does)
__device__ __forceinline__ int64_t rfl64(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int64_t ld_wt(const int64_t *p) {
  return __hip_atomic_load((gi64_t *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void fast_issue_wt(const lc_op *kops, int n, int tid, FastRecs &b) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  void *base = reinterpret_cast<void *>(rfl64(reinterpret_cast<int64_t>(kops)));
  const int bytes = __builtin_amdgcn_readfirstlane(n * (int)sizeof(lc_op));
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, bytes, 0x00020000);
#pragma unroll
  for (int u = 0; u < kPer; u++) {
    const int off = (tid + u * kFastThreads) * (int)sizeof(lc_op);
    const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16);
    const u32x4 y = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, 16);
    const u32x4 z = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 32, 0, 16);
    __builtin_memcpy(&b.w[u].a, &x, 16);
    __builtin_memcpy(&b.w[u].b, &y, 16);
    __builtin_memcpy(&b.w[u].c, &z, 16);
  }
}

// Key blockIdx.x of a request (rq: its words in LDS, read at use so nothing
// of the request stays live across the request loop), as fast_one decides it
__device__ __forceinline__ void fast_one_res(const uint64_t *rq, int64_t key, FastLds &s) {
  auto w = [&](int i) { return rfl64((int64_t)res_val(rq[i])); };
  const lc_op *ops = reinterpret_cast<const lc_op *>(w(0));
  const int64_t *key_off = reinterpret_cast<const int64_t *>(w(1));
  lc_key_result *out = reinterpret_cast<lc_key_result *>(w(3));
  const FastSinks o{reinterpret_cast<int32_t *>(w(4)), reinterpret_cast<KStatus *>(w(5)),
                    reinterpret_cast<int32_t *>(w(6)), nullptr, nullptr, nullptr};
  KParams p;
  p.init_ver = (int32_t)(uint32_t)w(7);
  p.init_val = (int32_t)(uint32_t)w(8);
  p.budget = 0;      // (the version-order tier reads neither)
  p.time_ticks = 0;
  const int64_t off0 = rfl64(ld_wt(key_off));
  const int64_t beg = rfl64(ld_wt(key_off + key)), end = rfl64(ld_wt(key_off + key + 1));
  const lc_op *kops = ops + (beg - off0);
  const int64_t n = end - beg;
  // (the thread index opaque, so the record offsets are not hoisted out of
  // the request loop and held in VGPRs between requests)
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  FastRecs rr;
  fast_issue_wt(kops, n > 0 && n <= kFastMax ? (int)n : 0, tid, rr);
  if (tid == 0) s.raised = 0;
  auto nop = [] {};
  fast_key<kModeFast, decltype(nop) &, lc_op, FastRecs, true>(key, n, kops, 0, rr, p, s, out, o,
                                                             nullptr, nop);
}

// every wait of the grid is bounded by a poll count too (a clock that did
// not advance could not keep a wave alive) and the workgroups other than 0
// by a wall-clock bound of their own
constexpr uint32_t kResPollCap0 = 1u << 20;   // workgroup 0 (one PCIe read per poll)
constexpr uint32_t kResPollCap = 1u << 22;    // the others (L2 reads)
constexpr uint64_t kResStrayTicks = 20000000; // 200 ms of the 100 MHz clock

// (6 waves per SIMD: at most 80 VGPRs and 104 SGPRs, six workgroups per CU,
// 1,536 on the chip; left alone the request loop takes 84 VGPRs, and 7 per
// CU spills)
__global__ __launch_bounds__(kFastThreads, 6) void fast_resident_kernel(ResHost *h, ResDev *dv,
                                                                        uint64_t idle_ticks) {
  __shared__ FastLds s;
  __shared__ uint64_t rq[kResWords];
  const int tid = threadIdx.x;
  const uint32_t G = gridDim.x;
  const uint32_t nshard = min((uint32_t)kResShards, G), shard = blockIdx.x % nshard;
  const uint32_t per = G / nshard + (shard < G % nshard ? 1u : 0u);
  const bool first = blockIdx.x == 0;
  gu64_t *const src = first ? (gu64_t *)h->req : (gu64_t *)dv->req;
  uint32_t seq = 0;
  uint64_t idle_from = wall_clock64();
  for (;;) {
    if (tid < kWave) {
      // wave 0 takes request seq + 1: every word tagged with its number
      // (workgroup 0 from host memory, the others from its copy)
      const uint32_t want = (seq + 1) & 0xFFFFu;
      const uint64_t t0 = wall_clock64();
      uint64_t w = 0;
      bool leave = false;
      for (uint32_t polls = 0;; polls++) {
        if (!first && LC_RES_POLL1) {
          // one word per poll (the others only once it carries the number):
          // 1,249 pollers beside the record stream
          const uint64_t w0 = __hip_atomic_load(src + kResWords - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((uint32_t)(__builtin_amdgcn_readfirstlane((int)(uint32_t)(w0 >> 32)) >> 16) != want) {
            const uint64_t now = wall_clock64();
            if (now - t0 > kResStrayTicks || polls >= kResPollCap) {
              leave = true;
              break;
            }
            __builtin_amdgcn_s_sleep(LC_RES_SLEEP);
            continue;
          }
        }
        if (tid < kResWords)
          w = first ? __hip_atomic_load(src + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                    : __hip_atomic_load(src + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__all(tid >= kResWords || (uint32_t)(w >> 48) == want)) break;
        const uint64_t now = wall_clock64();
        if (first ? (now - idle_from > idle_ticks || polls >= kResPollCap0)
                  : (now - t0 > kResStrayTicks || polls >= kResPollCap)) {
          leave = true;
          break;
        }
        if (first) __builtin_amdgcn_s_sleep(1);
        else __builtin_amdgcn_s_sleep(LC_RES_SLEEP);
      }
      if (leave) {
        // workgroup 0 on its idle bound: says so, and hands the others an
        // exit request; the others on their stray bound just go
        if (first && tid == 0)
          __hip_atomic_store((gu32_t *)&h->exited, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        w = res_word(tid == 2 ? (uint64_t)kResExitKeys : 0u, want);
      } else if (first && tid == 0) {
        __hip_atomic_store((gu64_t *)&h->t0, (uint64_t)wall_clock64(), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      }
      if (tid < kResWords) {
        if (first)
          __hip_atomic_store((gu64_t *)dv->req + tid, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        rq[tid] = w;
      }
    }
    __syncthreads();
    seq++;
    const int64_t n_keys = rfl64((int64_t)res_val(rq[2]));
    if (n_keys == kResExitKeys) return;
    // one key per workgroup (the host launches at least n_keys workgroups;
    // a loop over keys blockIdx.x, + G, ... needs 22 more SGPRs than the
    // wave has and spills)
    if ((int64_t)blockIdx.x < n_keys) fast_one_res(rq, blockIdx.x, s);
    // (every key's LDS reads done before the next request's; rq rewritten
    // only after this barrier)
    __syncthreads();
    if (tid == 0) {
      // thread 0 made every global store of this workgroup (results,
      // handoff flags and words, workgroup 0's detection time): drained
      // before it arrives
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint32_t v = __hip_atomic_fetch_add((gu32_t *)&dv->ticket[shard * 32], 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT) + 1;
      if (v % per == 0) {  // this shard's last arrival of this request
        const uint32_t t = __hip_atomic_fetch_add((gu32_t *)&dv->top, 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT) + 1;
        if (t % nshard == 0)  // the request's last arrival
          __hip_atomic_store((gu64_t *)&h->done, (uint64_t)seq << 32 | (uint32_t)wall_clock64(),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    idle_from = wall_clock64();
  }
}

// Crash-light pass over the keys the version-order tier handed to the gap
// tier (status->n_jit of them, written by the compaction launched just
// before: no host round trip in between).  Same decision as the version-
// order tier plus the in-place gap decision; what it cannot decide goes to
// `pass` (status->n_gap2) for the gap tier.
// 4 waves per SIMD (at most 128 VGPRs): left alone the compiler takes 138
// (3 waves); 4 has no VGPR spills and decides bench.py's crash_leg in
// 0.24 ms against 0.29 ms (5 and 6 waves spill: 0.33 / 0.36 ms).
#ifndef LC_LIGHT_WPE
#define LC_LIGHT_WPE 4
#endif
#define LC_LIGHT_ATTR __attribute__((amdgpu_waves_per_eu(LC_LIGHT_WPE, 8)))
__global__ __launch_bounds__(kFastThreads) LC_LIGHT_ATTR void gap_light_kernel(
    const lc_op *__restrict__ ops, const int64_t *__restrict__ key_off,
    const int32_t *__restrict__ keys, const KParams p, lc_key_result *__restrict__ out,
    const FastSinks o) {
  __shared__ FastLds s;
  const int32_t n_list = __hip_atomic_load(&o.status->n_jit, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
  // one key per workgroup: the grid is sized for every key of the call, and
  // workgroups past the list's length (on the device) leave at once.  (A
  // grid-stride loop over the list kept the next iteration's state live: 128
  // VGPRs with SGPR spills, 4 waves per SIMD; one key each, 72 and 7.)
  const int t = blockIdx.x;
  if (t >= n_list) return;
  fast_one<kModeLight>(ops, key_off, keys[t], p, s, out, o);
}

// The version-order tier and the crash-light decision in one pass over every
// key (kModeFused), persistent as the version-order tier; keys it does not
// decide are flagged for the same handoff compaction.  The crash-light
// register budget — the host picks this kernel only for batches where most
// keys carry crashed ops (lincheck.cpp).
#ifndef LC_FUSED_WPE
#define LC_FUSED_WPE LC_LIGHT_WPE
#endif
__global__ __launch_bounds__(kFastThreads) __attribute__((amdgpu_waves_per_eu(LC_FUSED_WPE, 8))) void fused_tier_kernel(
    const lc_op *__restrict__ ops, const int64_t *__restrict__ key_off, int64_t n_keys,
    const KParams p, lc_key_result *__restrict__ out, const FastSinks o) {
  __shared__ FastLds s;
#if LC_PIPE
  fast_run<kModeFused>(ops, key_off, n_keys, p, s, out, o);
#else
  fast_one<kModeFused>(ops, key_off, blockIdx.x, p, s, out, o);
#endif
#ifdef LC_FG_PROF
  if (threadIdx.x == 0 && atomicAdd(&g_fgdone, 1u) == gridDim.x - 1) {
    printf("fgprof keys-wg %u entry->init %llu init->pass1 %llu pass1->light %llu scans %llu match %llu "
           "entry->stash %llu stash+deadlines %llu after-match %llu\n",
           gridDim.x, g_fgp[0], g_fgp[1], g_fgp[2], g_fgp[3], g_fgp[4], g_fgp[5], g_fgp[6], g_fgp[7]);
    for (int i = 0; i < 8; i++) g_fgp[i] = 0;
    g_fgdone = 0;
  }
#endif
}

// The fused pass over lc_op32 records (as fast_tier32_kernel)
__global__ __launch_bounds__(kFastThreads) __attribute__((amdgpu_waves_per_eu(LC_FUSED_WPE, 8))) void fused_tier32_kernel(
    const lc_op32 *__restrict__ ops, const int64_t *__restrict__ key_off,
    const int64_t *__restrict__ key_base, int64_t n_keys, const KParams p,
    lc_key_result *__restrict__ out, const FastSinks o) {
  __shared__ FastLds s;
  if ((int64_t)blockIdx.x < n_keys) fast_one32<kModeFused>(ops, key_off, key_base, blockIdx.x, p, s, out, o);
}

// Workspace layout per wave: 3 regions of cap Cfg, 2 tables of 2*cap Cfg,
// 2 tag arrays of 2*cap uint32.
__host__ __device__ inline size_t hbm_wave_bytes(int64_t cap) {
  return (size_t)cap * 16 * 3 + (size_t)cap * 2 * 16 * 2 + (size_t)cap * 2 * 4 * 2;
}

// The workspace's tag arrays (4 * cap entries) start stale for every epoch:
// each workgroup zeroes its own at launch (an eighth of its workspace; a host
// memset of the whole workspace, or a strided one of the tags, took 0.35 ms
// per launch on model_leg).  Epochs then start at 1.
__device__ __forceinline__ void hbm_zero_tags(uint32_t *tags, int64_t cap) {
  uint4 *t = reinterpret_cast<uint4 *>(tags);  // 4 * cap entries = cap uint4
  for (int64_t i = threadIdx.x; i < cap; i += blockDim.x) t[i] = make_uint4(0, 0, 0, 0);
  __syncthreads();  // (workgroup-scope: the stores are visible to every wave)
}

__global__ __launch_bounds__(kWave) void hbm_tier_kernel(
    const lc_op *__restrict__ ops, const int64_t *__restrict__ key_off,
    const int32_t *__restrict__ keys, const int32_t n_list,
    const KParams p, lc_key_result *__restrict__ out, char *__restrict__ ws,
    const int64_t cap, int32_t *__restrict__ ovf_out, int32_t *__restrict__ n_ovf_out,
    int32_t *__restrict__ n_malformed, int32_t *__restrict__ next, const int last_tier) {
  const int lane = threadIdx.x;
  char *w = ws + (size_t)blockIdx.x * hbm_wave_bytes(cap);
  HbmStore st;
  st.base = reinterpret_cast<Cfg *>(w);
  st.tabs = st.base + 3 * cap;
  st.tags = reinterpret_cast<uint32_t *>(st.tabs + 4 * cap);
  st.cap = (int)cap;
  st.tmask = st.tmask_full = (uint32_t)(2 * cap - 1);
  hbm_zero_tags(st.tags, cap);
  st.epoch = 0;  // epochs start at 1
  const int64_t key_base = key_off[0];
  for (;;) {  // list entries claimed one at a time (next: zero at launch)
    int li = 0;
    if (lane == 0) li = atomicAdd(next, 1);
    li = uni(li);
    if (li >= n_list) break;
    const int64_t key = keys[li];
    const int64_t beg = key_off[key], end = key_off[key + 1];
    KeyOut o;
    st.hint = 0;  // table-size hint: per key
    check_key(ops + (beg - key_base), (int)(end - beg), p, st, o, lane);
    if (o.reason == LC_REASON_FRONTIER_LDS) {
      if (last_tier) {
        o.reason = LC_REASON_CONFIG_BUDGET;  // largest sets full: give up
      } else if (lane == 0) {
        ovf_out[atomicAdd(n_ovf_out, 1)] = (int32_t)key;  // next, larger tier
      }
    }
    if (lane == 0) {
      if (o.reason == LC_REASON_MALFORMED) atomicAdd(n_malformed, 1);
      write_result(&out[key], o);
    }
  }
}

// The same over HBM tables (the one-wave HBM tier's store, workspace of
// hbm_wave_bytes(cap) per wave), for the listed keys, claimed one at a time.
__global__ __launch_bounds__(kWave) void frontier_dump_hbm_kernel(
    const lc_op *__restrict__ ops, const int64_t *__restrict__ key_off,
    const int64_t *__restrict__ stop_op, const int32_t *__restrict__ keys, const int32_t n_list,
    const KParams p, char *__restrict__ ws, const int64_t cap, lc_fx_config *__restrict__ out,
    const int max, int32_t *__restrict__ n_out, int32_t *__restrict__ next) {
  const int lane = threadIdx.x;
  char *w = ws + (size_t)blockIdx.x * hbm_wave_bytes(cap);
  HbmStore st;
  st.base = reinterpret_cast<Cfg *>(w);
  st.tabs = st.base + 3 * cap;
  st.tags = reinterpret_cast<uint32_t *>(st.tabs + 4 * cap);
  st.cap = (int)cap;
  st.tmask = st.tmask_full = (uint32_t)(2 * cap - 1);
  hbm_zero_tags(st.tags, cap);
  st.epoch = 0;
  for (;;) {
    int li = 0;
    if (lane == 0) li = atomicAdd(next, 1);
    li = uni(li);
    if (li >= n_list) break;
    const int64_t key = keys[li];
    st.hint = 0;
    const int n = dump_key(ops, key_off, key, stop_op[key], p, st, out + key * max, max, lane);
    if (lane == 0) n_out[key] = n;
  }
}

// launch_status_settle (kernels.h): one workgroup.
__global__ __launch_bounds__(256) void status_settle_kernel(KStatus *__restrict__ status,
                                                            int32_t *__restrict__ h_light) {
  const int tid = threadIdx.x;
  int v = tid < kLightShards ? status->n_light_sh[tid * kLightStride] : 0;
  if (tid < kWave) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (tid == 0) {
      __hip_atomic_store(h_light, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
    }
  }
  __syncthreads();
  uint32_t *w = reinterpret_cast<uint32_t *>(status);
  for (int i = tid; i < (int)(sizeof(KStatus) / 4); i += 256) w[i] = 0;
}

// Build the handoff lists from the fast tier's per-key flags (and clear
// them): one list reservation (atomicAdd) and one max per workgroup chunk.
constexpr int kCompactThreads = 256;
__global__ __launch_bounds__(kCompactThreads) void handoff_compact_kernel(
    int32_t *__restrict__ flags, const int64_t *__restrict__ key_off, const int64_t n_keys,
    const int route_direct, int32_t *__restrict__ jit_keys, int32_t *__restrict__ direct_keys,
    KStatus *__restrict__ status, int32_t *__restrict__ witness_kind) {
  __shared__ int wg[kCompactThreads / kWave], wd[kCompactThreads / kWave];
  __shared__ int base_g, base_d;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
  int32_t maxlen = 0;
  for (int64_t k0 = (int64_t)blockIdx.x * kCompactThreads; k0 < n_keys;
       k0 += (int64_t)gridDim.x * kCompactThreads) {
    const int64_t k = k0 + tid;
    int f = 0;
    if (k < n_keys) {
      f = flags[k];
      if (f) {
        flags[k] = 0;
        if (witness_kind) witness_kind[k] = LC_WITNESS_NONE;
      }
    }
    const bool dir = f == 2 && route_direct;
    const bool gap = f != 0 && !dir;
    if (gap) {
      const int64_t n = key_off[k + 1] - key_off[k];
      maxlen = max(maxlen, (int32_t)(n > INT_MAX ? INT_MAX : n));
    }
    const uint64_t bg = __ballot(gap), bd = __ballot(dir);
    if (lane == 0) {
      wg[w] = __popcll(bg);
      wd[w] = __popcll(bd);
    }
    __syncthreads();
    if (tid == 0) {
      int tg = 0, td = 0;
      for (int j = 0; j < kCompactThreads / kWave; j++) {
        tg += wg[j];
        td += wd[j];
      }
      base_g = tg ? atomicAdd(&status->n_jit, tg) : 0;
      base_d = td ? atomicAdd(&status->n_jit2, td) : 0;
    }
    __syncthreads();
    int pg = base_g, pd = base_d;
    for (int j = 0; j < w; j++) {
      pg += wg[j];
      pd += wd[j];
    }
    const uint64_t below = (1ull << lane) - 1;
    if (gap) jit_keys[pg + __popcll(bg & below)] = (int32_t)k;
    if (dir) direct_keys[pd + __popcll(bd & below)] = (int32_t)k;
    __syncthreads();
  }
  // max over the workgroup, one atomic
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) maxlen = max(maxlen, __shfl_xor(maxlen, o));
  if (lane == 0) wg[w] = maxlen;
  __syncthreads();
  if (tid == 0) {
    int m = 0;
    for (int j = 0; j < kCompactThreads / kWave; j++) m = max(m, wg[j]);
    if (m) atomicMax(&status->max_len, m);
  }
}

// Cooperative HBM tier: one workgroup of NW waves per key (few, large keys:
// the higher-capacity tiers).  Wave 0 runs the event loop; waves 1..NW-1
// serve its expansions until told to exit.
template <int NW>
__global__ __launch_bounds__(NW * kWave) __attribute__((amdgpu_waves_per_eu(4))) void hbm_coop_kernel(
    const lc_op *__restrict__ ops, const int64_t *__restrict__ key_off,
    const int32_t *__restrict__ keys, const int32_t n_list,
    const KParams p, lc_key_result *__restrict__ out, char *__restrict__ ws,
    const int64_t cap, int32_t *__restrict__ ovf_out, int32_t *__restrict__ n_ovf_out,
    int32_t *__restrict__ n_malformed, int32_t *__restrict__ next, const int last_tier) {
  __shared__ CoopShared C;
  constexpr int LT = NW >= 8 ? 4096 : 2048;  // LDS table: 2 * LT entries (both roles)
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  {  // LDS tags and W flags start stale (epochs start at 1)
    for (int i = threadIdx.x; i < 2 * LT; i += NW * kWave) coop_tab<LT>().tag[i] = 0;
    for (int i = threadIdx.x; i < CoopTab<LT>::kPool; i += NW * kWave) coop_tab<LT>().wrdy[i] = 0;
    __syncthreads();
  }
  char *w = ws + (size_t)blockIdx.x * hbm_wave_bytes(cap);
  CoopStore<LT> st;
  st.coop = &C;
  st.nwaves = NW;
  st.base = reinterpret_cast<Cfg *>(w);
  st.tabs = st.base + 3 * cap;
  st.tags = reinterpret_cast<uint32_t *>(st.tabs + 4 * cap);
  st.cap = (int)cap;
  st.tmask = st.tmask_full = (uint32_t)(2 * cap - 1);
  hbm_zero_tags(st.tags, cap);
  st.epoch = 0;  // epochs start at 1
  if (wave == 0) {
    if (LC_COOP_PRIO) __builtin_amdgcn_s_setprio(LC_COOP_PRIO);  // (LC_COOP_PRIO above)
    const int64_t key_base = key_off[0];
    for (;;) {  // list entries claimed one at a time (next: zero at launch)
      int li = 0;
      if (lane == 0) li = atomicAdd(next, 1);
      li = uni(li);
      if (li >= n_list) break;
      const int64_t key = keys[li];
      const int64_t beg = key_off[key], end = key_off[key + 1];
      KeyOut o;
      st.hint = 0;  // table-size hints: per key
      st.last = st.lsum = 0;
      st.vleg = 0;
      st.fclear = st.fclose = 0;
#ifdef HBM_PROFILE
      const uint64_t tk0 = wall_clock64();
#endif
#ifdef LC_COOP_PROF
      const uint64_t ck0 = CP_NOW();
#endif
      check_key(ops + (beg - key_base), (int)(end - beg), p, st, o, lane);
#ifdef LC_COOP_PROF
      st.cp[7] += CP_NOW() - ck0;
      st.cp[10]++;
#endif
#ifdef HBM_PROFILE
      if (lane == 0 && blockIdx.x < 4096) g_hwg[blockIdx.x][2] += wall_clock64() - tk0;
#endif
      if (o.reason == LC_REASON_FRONTIER_LDS) {
        if (last_tier)
          o.reason = LC_REASON_CONFIG_BUDGET;
        else if (lane == 0)
          ovf_out[atomicAdd(n_ovf_out, 1)] = (int32_t)key;
      }
      if (lane == 0) {
        if (o.reason == LC_REASON_MALFORMED) atomicAdd(n_malformed, 1);
        write_result(&out[key], o);
      }
    }
    if (lane == 0) C.cmd = kCoopExit;
#ifdef LC_COOP_PROF
    if (lane == 0 && blockIdx.x < 4096)
      for (int q = 0; q < kCpN; q++) g_cp[blockIdx.x][0][q] = st.cp[q];
#endif
#ifdef HBM_PROFILE
    __threadfence();
    if (lane == 0 && atomicAdd(&g_hdone, 1u) == gridDim.x - 1)
      for (int b = 0; b < 20; b++)
        if (g_hhist[b][0])
          printf("set<2^%d: returns %llu ticks %llu lds %llu configs %llu\n", b, g_hhist[b][0],
                 g_hhist[b][1], g_hhist[b][2], g_hhist[b][3]);
    if (lane == 0 && g_hdone == gridDim.x) {
      unsigned long long sum = 0;
      for (unsigned i = 0; i < gridDim.x && i < 4096; i++) sum += g_hwg[i][2];
      printf("workgroups %u mean key ticks %llu\n", gridDim.x, sum / gridDim.x);
      for (int t = 0; t < 6; t++) {
        unsigned best = 0;
        for (unsigned i = 0; i < gridDim.x && i < 4096; i++)
          if (g_hwg[i][2] > g_hwg[best][2]) best = i;
        printf("  slow wg %u: key %llu lds-returns %llu hbm-returns %llu\n", best, g_hwg[best][2],
               g_hwg[best][0], g_hwg[best][1]);
        g_hwg[best][2] = 0;
      }
    }
#endif
    coop_barrier();
  } else {
    for (;;) {
      coop_barrier();
      if (C.cmd == kCoopExit) break;
      coop_expand<LT>(st, C, lane, wave);
    }
#ifdef LC_COOP_PROF
    if (wave == 1 && lane == 0 && blockIdx.x < 4096)
      for (int q = 0; q < kCpN; q++) g_cp[blockIdx.x][1][q] = st.cp[q];
#endif
  }
}

// Version-order witnesses (lc_aux): a record's pinned mutation position, or
// -1.  Grid-stride over the records, then over the keys for their kind.
__global__ __launch_bounds__(256) void witness_init_kernel(
    const lc_op *__restrict__ ops, const int64_t *__restrict__ key_off, const int64_t n_keys,
    const int64_t n_records, const int32_t V0, const int fast_on, int32_t *__restrict__ wit,
    int32_t *__restrict__ kind) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n_records; r += stride) {
    const lc_op o = ops[r];
    // a version no state reaches (outside (V0, kFieldMax): decode saturates
    // the ones beyond int32 to kFieldMax) pins nothing, whatever its width
    // (lc_pack32 narrows such versions to kFieldMax)
    const bool pinned = (o.f == LC_F_WRITE || o.f == LC_F_CAS) && o.ret != kInf &&
                        o.version > (int64_t)V0 && o.version < kFieldMax;
    wit[r] = pinned ? (int32_t)(o.version - V0 - 1) : -1;
  }
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n_keys; k += stride)
    kind[k] = fast_on ? LC_WITNESS_FULL : LC_WITNESS_NONE;
}

// 24-byte records (lc_op32, ABI 4) into the 48-byte form every tier reads,
// with the key's base added back to call / ret, so the tiers see exactly the
// records lc_check would have been given (include/lincheck.h).  One
// workgroup per key (grid.x = keys, grid.y splits long keys); 8-byte loads
// (three per record), 16-byte stores (three per record).  HBM-bound:
// 24 B read + 48 B written per record.
__global__ __launch_bounds__(256) void widen32_kernel(const int2 *__restrict__ in,
                                                      const int64_t *__restrict__ key_off,
                                                      const int64_t *__restrict__ key_base,
                                                      longlong2 *__restrict__ out) {
  const int64_t k = blockIdx.x;
  const int64_t off0 = key_off[0];
  const int64_t b = key_off[k] - off0, e = key_off[k + 1] - off0;
  const int64_t base = key_base ? key_base[k] : 0;
  const int64_t step = (int64_t)blockDim.x * gridDim.y;
  for (int64_t r = b + (int64_t)blockIdx.y * blockDim.x + threadIdx.x; r < e; r += step) {
    const int2 fv = in[3 * r], ev = in[3 * r + 1], cr = in[3 * r + 2];
    const uint32_t call = (uint32_t)cr.x, ret = (uint32_t)cr.y;
    out[3 * r] = make_longlong2((int64_t)fv.x, (int64_t)fv.y);
    out[3 * r + 1] = make_longlong2((int64_t)ev.x, (int64_t)ev.y);
    out[3 * r + 2] = make_longlong2(base + (int64_t)call,
                                    ret == LC_INF32 ? kInf : base + (int64_t)ret);
  }
}

// lc_op16 records (include/lincheck.h, round 6) into lc_op records: one
// 16-byte load and three 16-byte stores per record
__global__ __launch_bounds__(256) void widen16_kernel(const uint4 *__restrict__ in,
                                                      const int64_t *__restrict__ key_off,
                                                      const int64_t *__restrict__ key_base,
                                                      longlong2 *__restrict__ out) {
  const int64_t k = blockIdx.x;
  const int64_t off0 = key_off[0];
  const int64_t b = key_off[k] - off0, e = key_off[k + 1] - off0;
  const int64_t base = key_base ? key_base[k] : 0;
  const int64_t step = (int64_t)blockDim.x * gridDim.y;
  for (int64_t r = b + (int64_t)blockIdx.y * blockDim.x + threadIdx.x; r < e; r += step) {
    const uint4 q = in[r];
    const uint32_t v = (q.x >> 15) & 0x7FFFu, x = q.x & 0x7FFFu;
    const int64_t value = v == 0x7FFFu ? -2 : (int64_t)v - 1;
    const int64_t expected = x == 0x7FFFu ? -2 : (int64_t)x - 1;
    out[3 * r] = make_longlong2((int64_t)(q.x >> 30), value);
    out[3 * r + 1] = make_longlong2(expected, (int64_t)(int32_t)q.y);
    out[3 * r + 2] = make_longlong2(base + (int64_t)q.z, q.w == LC_INF32 ? kInf : base + (int64_t)q.w);
  }
}

}  // namespace

hipError_t launch_widen16(const lc_op16 *d_in, const int64_t *d_key_off, const int64_t *d_key_base,
                          int64_t n_keys, int64_t max_len, lc_op *d_out, hipStream_t stream) {
  if (n_keys <= 0) return hipSuccess;
  if (n_keys > INT32_MAX) return hipErrorInvalidValue;
  const unsigned gy = (unsigned)std::min<int64_t>(64, std::max<int64_t>(1, (max_len + 1023) / 1024));
  hipLaunchKernelGGL(widen16_kernel, dim3((unsigned)n_keys, gy), dim3(256), 0, stream,
                     reinterpret_cast<const uint4 *>(d_in), d_key_off, d_key_base,
                     reinterpret_cast<longlong2 *>(d_out));
  return hipGetLastError();
}

hipError_t launch_frontier_dump(const lc_op *d_ops, const int64_t *d_key_off, const int64_t *d_stop,
                                int64_t n_keys, const KParams &p, lc_fx_config *d_out, int max,
                                int32_t *d_n_out, int32_t *d_retry, int32_t *d_n_retry,
                                hipStream_t stream) {
  if (n_keys <= 0) return hipSuccess;
  const int64_t wgs = (n_keys + kWavesPerWG - 1) / kWavesPerWG;
  hipLaunchKernelGGL(frontier_dump_kernel, dim3((unsigned)wgs), dim3(kWave * kWavesPerWG), 0, stream,
                     d_ops, d_key_off, d_stop, n_keys, p, d_out, max, d_n_out, d_retry, d_n_retry);
  return hipGetLastError();
}

hipError_t launch_frontier_dump_hbm(const lc_op *d_ops, const int64_t *d_key_off,
                                    const int64_t *d_stop, const int32_t *d_keys, int32_t n_list,
                                    const KParams &p, void *d_ws, int n_waves, int64_t cap,
                                    lc_fx_config *d_out, int max, int32_t *d_n_out, int32_t *d_next,
                                    hipStream_t stream) {
  if (n_list <= 0) return hipSuccess;
  hipLaunchKernelGGL(frontier_dump_hbm_kernel, dim3((unsigned)n_waves), dim3(kWave), 0, stream, d_ops,
                     d_key_off, d_stop, d_keys, n_list, p, static_cast<char *>(d_ws), cap, d_out, max,
                     d_n_out, d_next);
  return hipGetLastError();
}

hipError_t launch_widen32(const lc_op32 *d_in, const int64_t *d_key_off, const int64_t *d_key_base,
                          int64_t n_keys, int64_t max_len, lc_op *d_out, hipStream_t stream) {
  if (n_keys <= 0) return hipSuccess;
  if (n_keys > INT32_MAX) return hipErrorInvalidValue;
  // keys longer than 1,024 records get more workgroups (C4's 5,000-op key)
  const unsigned gy = (unsigned)std::min<int64_t>(64, std::max<int64_t>(1, (max_len + 1023) / 1024));
  hipLaunchKernelGGL(widen32_kernel, dim3((unsigned)n_keys, gy), dim3(256), 0, stream,
                     reinterpret_cast<const int2 *>(d_in), d_key_off, d_key_base,
                     reinterpret_cast<longlong2 *>(d_out));
  return hipGetLastError();
}

hipError_t launch_fast_resident(ResHost *h_res, ResDev *d_res, int64_t grid, uint64_t idle_ticks,
                                hipStream_t stream) {
  if (grid <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(fast_resident_kernel, dim3((unsigned)grid), dim3(kFastThreads), 0, stream, h_res,
                     d_res, idle_ticks);
  return hipGetLastError();
}

hipError_t launch_done_signal(uint32_t *h_done, uint32_t seq, hipStream_t stream) {
  hipLaunchKernelGGL(done_signal_kernel, dim3(1), dim3(64), 0, stream, h_done, seq);
  return hipGetLastError();
}

hipError_t launch_status_settle(KStatus *d_status, int32_t *h_light, hipStream_t stream) {
  hipLaunchKernelGGL(status_settle_kernel, dim3(1), dim3(256), 0, stream, d_status, h_light);
  return hipGetLastError();
}

hipError_t launch_handoff_compact(int32_t *d_flags, const int64_t *d_key_off, int64_t n_keys,
                                  int route_direct, int32_t *d_jit_keys, int32_t *d_direct_keys,
                                  KStatus *d_status, int32_t *d_witness_kind, hipStream_t stream) {
  if (n_keys <= 0) return hipSuccess;
  const int64_t wgs = std::min<int64_t>((n_keys + kCompactThreads - 1) / kCompactThreads, 1024);
  hipLaunchKernelGGL(handoff_compact_kernel, dim3((unsigned)wgs), dim3(kCompactThreads), 0, stream,
                     d_flags, d_key_off, n_keys, route_direct, d_jit_keys, d_direct_keys, d_status,
                     d_witness_kind);
  return hipGetLastError();
}

hipError_t launch_witness_init(const lc_op *d_ops, const int64_t *d_key_off, int64_t n_keys,
                               int64_t n_records, const KParams &p, int fast_on,
                               int32_t *d_witness, int32_t *d_witness_kind, hipStream_t stream) {
  if (n_keys <= 0) return hipSuccess;
  const int64_t work = std::max(n_records, n_keys);
  const int64_t wgs = std::max<int64_t>(1, std::min<int64_t>((work + 255) / 256, 8192));
  hipLaunchKernelGGL(witness_init_kernel, dim3((unsigned)wgs), dim3(256), 0, stream, d_ops,
                     d_key_off, n_keys, n_records, p.init_ver, fast_on, d_witness, d_witness_kind);
  return hipGetLastError();
}

// Resident workgroups of a persistent kernel on the current device (its
// grid): occupancy per CU x CUs, cached per device and kernel.
template <typename K>
static int64_t resident_wgs(K kernel, int which, size_t dyn_lds) {
  static std::atomic<int> cache[64][3];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  int c = cache[dev][which].load(std::memory_order_relaxed);
  if (c == 0) {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kFastThreads, dyn_lds) !=
            hipSuccess || per_cu < 1)
      per_cu = 1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus < 1)
      cus = 1;
    c = per_cu * cus;
    cache[dev][which].store(c, std::memory_order_relaxed);
  }
  return c;
}

// (at most 6 per CU whatever the occupancy query says: the SGPR count admits
// no more, and a workgroup that cannot become resident would never run)
int64_t fast_resident_capacity() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
    return 0;
  return std::min<int64_t>(resident_wgs(fast_resident_kernel, 2, 0), 6 * (int64_t)cus);
}

hipError_t launch_fast_tier(const lc_op *d_ops, const int64_t *d_key_off,
                            int64_t n_keys, const KParams &p,
                            lc_key_result *d_out, int32_t *d_flags,
                            KStatus *d_status, int32_t *h_handoff, hipStream_t stream) {
  if (n_keys <= 0) return hipSuccess;
  const int64_t wgs = LC_PIPE ? std::min(n_keys, resident_wgs(fast_tier_kernel, 0, 0)) : n_keys;
  hipLaunchKernelGGL(fast_tier_kernel, dim3((unsigned)wgs), dim3(kFastThreads), 0,
                     stream, d_ops, d_key_off, n_keys, p, d_out, d_flags, d_status, h_handoff);
  return hipGetLastError();
}

hipError_t launch_fused_tier(const lc_op *d_ops, const int64_t *d_key_off, int64_t n_keys,
                             const KParams &p, lc_key_result *d_out, int32_t *d_flags,
                             KStatus *d_status, int32_t *h_handoff, int32_t *d_witness,
                             int32_t *d_witness_kind, hipStream_t stream) {
  if (n_keys <= 0) return hipSuccess;
  const FastSinks o{d_flags, d_status, h_handoff, nullptr, d_witness, d_witness_kind};
  const int64_t wgs =
      LC_PIPE ? std::min(n_keys, resident_wgs(fused_tier_kernel, 1, kFgLdsBytes)) : n_keys;
  hipLaunchKernelGGL(fused_tier_kernel, dim3((unsigned)wgs), dim3(kFastThreads),
                     (unsigned)kFgLdsBytes, stream, d_ops, d_key_off, n_keys, p, d_out, o);
  return hipGetLastError();
}

hipError_t launch_fast_tier32(const lc_op32 *d_ops, const int64_t *d_key_off, const int64_t *d_key_base,
                              int64_t n_keys, const KParams &p, lc_key_result *d_out, int32_t *d_flags,
                              KStatus *d_status, int32_t *h_handoff, hipStream_t stream) {
  if (n_keys <= 0) return hipSuccess;
  hipLaunchKernelGGL(fast_tier32_kernel, dim3((unsigned)n_keys), dim3(kFastThreads), 0, stream, d_ops,
                     d_key_off, d_key_base, n_keys, p, d_out, d_flags, d_status, h_handoff);
  return hipGetLastError();
}

hipError_t launch_fused_tier32(const lc_op32 *d_ops, const int64_t *d_key_off, const int64_t *d_key_base,
                               int64_t n_keys, const KParams &p, lc_key_result *d_out, int32_t *d_flags,
                               KStatus *d_status, int32_t *h_handoff, hipStream_t stream) {
  if (n_keys <= 0) return hipSuccess;
  const FastSinks o{d_flags, d_status, h_handoff, nullptr, nullptr, nullptr};
  hipLaunchKernelGGL(fused_tier32_kernel, dim3((unsigned)n_keys), dim3(kFastThreads),
                     (unsigned)kFgLdsBytes, stream, d_ops, d_key_off, d_key_base, n_keys, p, d_out, o);
  return hipGetLastError();
}

hipError_t launch_gap_light(const lc_op *d_ops, const int64_t *d_key_off, const int32_t *d_keys,
                            int64_t max_keys, const KParams &p, lc_key_result *d_out,
                            int32_t *d_pass, KStatus *d_status, int32_t *d_witness,
                            int32_t *d_witness_kind, hipStream_t stream) {
  if (max_keys <= 0) return hipSuccess;
  const FastSinks o{nullptr, d_status, nullptr, d_pass, d_witness, d_witness_kind};
  // one workgroup per possible list entry (the list's length is on the
  // device); the ones past its end return at once
  const int64_t wgs = max_keys;
  hipLaunchKernelGGL(gap_light_kernel, dim3((unsigned)wgs), dim3(kFastThreads),
                     (unsigned)kFgLdsBytes, stream, d_ops, d_key_off, d_keys, p, d_out, o);
  return hipGetLastError();
}

hipError_t launch_lds_tier(const lc_op *d_ops, const int64_t *d_key_off,
                           const int32_t *d_keys, int64_t n_keys,
                           const KParams &p, lc_key_result *d_out, int32_t *d_ovf_keys,
                           KStatus *d_status, hipStream_t stream) {
  if (n_keys <= 0) return hipSuccess;
  const int64_t blocks = (n_keys + kWavesPerWG - 1) / kWavesPerWG;
  hipLaunchKernelGGL(lds_tier_kernel, dim3((unsigned)blocks),
                     dim3(kWave * kWavesPerWG), 0, stream, d_ops, d_key_off,
                     d_keys, n_keys, p, d_out, d_ovf_keys, d_status);
  return hipGetLastError();
}

size_t hbm_tier_ws_bytes(int n_waves, int64_t cap) {
  return hbm_wave_bytes(cap) * (size_t)n_waves;
}


hipError_t launch_hbm_coop(const lc_op *d_ops, const int64_t *d_key_off, const int32_t *d_keys,
                           int32_t n_list, const KParams &p, lc_key_result *d_out, void *d_ws,
                           int n_wg, int64_t cap, int32_t *d_ovf_out, int32_t *d_n_ovf_out,
                           int32_t *d_malformed, int32_t *d_next, int last_tier,
                           int waves_per_key, hipStream_t stream) {
  if (n_list <= 0) return hipSuccess;
  if (waves_per_key == 8)  // (A/B: LC_HBM_COOP=8)
    hipLaunchKernelGGL(hbm_coop_kernel<8>, dim3((unsigned)n_wg), dim3(8 * kWave), 0, stream,
                       d_ops, d_key_off, d_keys, n_list, p, d_out, static_cast<char *>(d_ws), cap,
                       d_ovf_out, d_n_ovf_out, d_malformed, d_next, last_tier);
  else if (waves_per_key >= 16)
    hipLaunchKernelGGL(hbm_coop_kernel<16>, dim3((unsigned)n_wg), dim3(16 * kWave), 0, stream,
                       d_ops, d_key_off, d_keys, n_list, p, d_out, static_cast<char *>(d_ws), cap,
                       d_ovf_out, d_n_ovf_out, d_malformed, d_next, last_tier);
  else
    hipLaunchKernelGGL(hbm_coop_kernel<4>, dim3((unsigned)n_wg), dim3(4 * kWave), 0, stream,
                       d_ops, d_key_off, d_keys, n_list, p, d_out, static_cast<char *>(d_ws), cap,
                       d_ovf_out, d_n_ovf_out, d_malformed, d_next, last_tier);
#ifdef LC_COOP_PROF
  {
    static unsigned long long h[4096][2][kCpN];
    const int nw = std::min(n_wg, 4096);
    void *sym = nullptr;
    if (hipStreamSynchronize(stream) == hipSuccess && hipGetSymbolAddress(&sym, HIP_SYMBOL(g_cp)) == hipSuccess &&
        hipMemcpy(h, sym, sizeof(h[0]) * nw, hipMemcpyDeviceToHost) == hipSuccess) {
      for (int wv = 0; wv < 2; wv++) {
        double sum[kCpN] = {0};
        int slow = 0;
        for (int w = 0; w < nw; w++) {
          for (int q = 0; q < kCpN; q++) sum[q] += (double)h[w][wv][q];
          if (h[w][0][7] > h[slow][0][7]) slow = w;
        }
        auto line = [&](const char *who, const double *v, double div, double rets) {
          const double r = std::max(1.0, rets), bt = std::max(1.0, v[11]);
          fprintf(stderr,
                  "coopprof wave %d %s: key clocks %.0f, coop returns %.0f (%.0f HBM-mode) taking %.0f; LDS-mode "
                  "returns %.0f: start-barrier %.0f split %.0f split-barrier %.0f queue %.0f end-barrier %.0f "
                  "(clocks each); per return: batches %.2f rounds %.2f sleeps %.1f; per batch clocks: claim %.0f "
                  "ready %.0f cand %.0f rounds %.0f\n",
                  wv, who, v[7] / div, v[8] / div, v[9] / div, v[6] / div, v[5] / div, v[0] / r, v[1] / r,
                  v[2] / r, v[3] / r, v[4] / r, v[11] / r, v[12] / r, v[13] / r, v[14] / bt, v[15] / bt,
                  v[16] / bt, v[17] / bt);
        };
        double rets = 0;
        for (int w = 0; w < nw; w++) rets += (double)h[w][0][5];
        line("mean per workgroup", sum, std::max(1, nw), rets);
        if (wv == 0)
          fprintf(stderr, "coopprof event loop per workgroup: calls %.0f taking %.0f, single returns %.0f taking "
                  "%.0f, after cooperative returns %.0f; before them: event loop %.0f, coop_return's "
                  "publish %.0f\n", sum[21] / nw, sum[18] / nw, sum[22] / nw,
                  sum[19] / nw, sum[20] / nw, sum[24] / nw, sum[23] / nw);
        if (wv == 0)
          fprintf(stderr, "coopprof HBM mode: failed LDS attempts' clocks %.0f per workgroup (slowest %.0f); HBM "
                  "attempts %.2f (slowest %.0f) taking %.0f (slowest %.0f), mean larger set %.0f\n",
                  sum[25] / nw, (double)h[slow][0][25], sum[26] / nw, (double)h[slow][0][26], sum[27] / nw,
                  (double)h[slow][0][27], sum[28] / std::max(1.0, sum[26]));
        double sl[kCpN];
        for (int q = 0; q < kCpN; q++) sl[q] = (double)h[slow][wv][q];
        line("slowest workgroup", sl, 1.0, (double)h[slow][0][5]);
      }
      (void)hipMemset(sym, 0, sizeof(h[0]) * nw);
    }
  }
#endif
  return hipGetLastError();
}

hipError_t launch_hbm_tier(const lc_op *d_ops, const int64_t *d_key_off,
                           const int32_t *d_keys,
                           int32_t n_list, const KParams &p, lc_key_result *d_out,
                           void *d_ws, int n_waves, int64_t cap,
                           int32_t *d_ovf_out, int32_t *d_n_ovf_out, int32_t *d_malformed,
                           int32_t *d_next, int last_tier, hipStream_t stream) {
  if (n_list <= 0) return hipSuccess;
  hipLaunchKernelGGL(hbm_tier_kernel, dim3((unsigned)n_waves), dim3(kWave), 0,
                     stream, d_ops, d_key_off, d_keys, n_list, p,
                     d_out, static_cast<char *>(d_ws), cap, d_ovf_out, d_n_ovf_out, d_malformed,
                     d_next, last_tier);
  return hipGetLastError();
}

}  // namespace lcdev
