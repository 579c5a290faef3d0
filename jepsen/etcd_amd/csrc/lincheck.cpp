// lincheck.cpp — host runtime behind include/lincheck.h.
//
// Replaces, as one unit, the checker built at
//   /root/reference/src/jepsen/etcd/register.clj:108-112
// (independent/checker over checker/linearizable with VersionedRegister).
// jepsen.independent checks keys concurrently on a bounded JVM thread pool;
// here all keys of a call go to the GPUs in one batch: contiguous,
// cost-balanced key ranges per device (one host thread + one HIP stream per
// device).  Per device: the version-order tier over every key (one launch,
// one sync when it decides them all), then the JIT-search tier over the keys
// it hands over, then HBM-tier re-runs of the few keys whose frontier outgrew
// LDS.  No collective is needed: keys are independent and results land in
// the caller's array.  There is no CPU fallback: without a usable GPU lc_open
// fails with -ENODEV.
#include <errno.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/lincheck.h"
#include "../../../include/lincheck_fx.h"
#include "kernels.h"

#ifndef LC_BUILD_ID
#define LC_BUILD_ID "unknown"
#endif

namespace {

constexpr int64_t kDefaultBudget = 1 << 24;   // configurations per key
// HBM tiers: (configurations per set, concurrent keys).  Workspace per key
// is ~128 B per configuration of capacity (3 regions + 2 hash tables).
// Each tier's workspace is <= 4 GiB; the first has the most waves (the
// lane-parallel expansion is latency-bound per wave).
// Timing events.  LC_EVENT_FLAGS (dev A/B): hipEventDisableSystemFence skips
// the event's own system-scope fence (cache writeback + invalidate) when it
// is recorded; kernel completion already releases the kernel's writes to
// device memory, and the one host-visible word the host reads after such an
// event (h_handoff) is made visible by its writer with a system-scope fence
// (fast_tier_handoff, check_kernel.hip).
#ifndef LC_EVENT_FLAGS
#define LC_EVENT_FLAGS hipEventDisableSystemFence
#endif
constexpr unsigned kEventFlags = LC_EVENT_FLAGS;
constexpr int kHbmTiers = 3;
constexpr size_t kFxEngines = 4;  // LC_FLAG_WHOLE_GPU: oversized keys searched at once
constexpr int64_t kHbmCap[kHbmTiers] = {1 << 14, 1 << 18, 1 << 21};
constexpr int kHbmWaves[kHbmTiers] = {2048, 128, 16};
// HBM tier lists up to these sizes get a workgroup of 16 (4) wavefronts per
// key; longer lists a wavefront per key.  Measured (tools/hbm_probe.py,
// DESIGN.md §4): 16 wins on 512 crash-heavy keys (4.9 s vs 13.1 s with 4,
// 40 s with 1), 4 on 1000-2000 version-less keys (71 vs 113 vs 119 ms),
// 1 on 10,000 (331 vs 355 ms with 4).
// 8-wave workgroups (two per CU) up to 512 keys, 4-wave ones beyond: version-
// less 1,000-op keys at concurrency 20 (tools/coop8_ab.py), HBM tier ms:
//   keys        64    256    400    512    700   1000
//   4 waves   11.6   11.8   12.0   12.1   12.7   13.5
//   8 waves    9.1    9.1    9.2    9.4   15.3   18.0
//   16 waves   9.0    9.1   14.6   16.4   21.6   30.0
constexpr int kHbmCoop8MaxKeys = 512;
constexpr int kHbmCoop16Resident = 256;   // 16-wave workgroups resident: one per CU
constexpr int kHbmCoop4Resident = 1024;   // 4-wave workgroups: four per CU (LDS tables)
constexpr int kJitDirectMaxKeys = 1024;  // 4 cooperative workgroups per CU x 256 CUs
// Gap tier: at most this many workgroups, and this much workspace (each
// workgroup needs 92 B per record of the longest key handed over).  Dynamic
// LDS for the matching arrays: up to kGapLdsFull per workgroup for whole-key
// decisions (occupancy), up to kGapLdsProbe for counterexample probes.
constexpr int kGapMaxWG = 1024;
constexpr size_t kGapWsBytes = size_t(1) << 30;
constexpr int kGapLdsFull = 48 << 10;
// few keys (at most this many workgroups): occupancy does not matter, so a
// whole-key decision may hold a large matching in LDS (gfx950: 160 KB per CU)
constexpr int kGapLdsFew = 128 << 10;
constexpr int64_t kGapFewKeys = 512;
constexpr int64_t kGapSkelLdsMax = 78 << 10;  // two such workgroups per CU (160 KB)
// (two 256-thread workgroups per CU either way: the kernel's 240 VGPRs)
constexpr int kGapLdsProbe = 72 << 10;
constexpr int kGapMaxRounds = 64;
constexpr int kGapProbeMinLen = 1024;
#ifndef LC_GAP_WAVE_MAX_LEN
#define LC_GAP_WAVE_MAX_LEN 256
#endif
constexpr int kGapWaveMaxLen = LC_GAP_WAVE_MAX_LEN;  // keys up to this long: one-wave gap-tier workgroups
constexpr int64_t kGapWaveMinKeys = 1024;             // ... when there are more of them than this
constexpr int64_t kGapWideMaxKeys = 64;    // at most this many keys for the gap tier ...
constexpr int kGapWideMinLen = 2048;        // ... the longest of them this long: 512-thread workgroups

struct Dev {
  int id = -1;
  hipStream_t stream = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr, e2 = nullptr;
  void *d_ops = nullptr;
  size_t ops_cap = 0;
  int64_t *d_off = nullptr;
  size_t off_cap = 0;
  lc_key_result *d_out = nullptr;
  size_t out_cap = 0;
  int32_t *d_ovf = nullptr;
  size_t ovf_cap = 0;
  int32_t *d_ovf2 = nullptr;
  size_t ovf2_cap = 0;
  int32_t *d_jit = nullptr;
  size_t jit_cap = 0;
  int32_t *d_flags = nullptr;          // per key: handed over by the fast tier (zero between calls)
  size_t flags_cap = 0;
  int32_t *d_jit2 = nullptr;           // keys the gap tier passes on
  size_t jit2_cap = 0;
  int32_t *d_gap2 = nullptr;           // keys the crash-light pass leaves to the gap tier
  size_t gap2_cap = 0;
  hipEvent_t el = nullptr;             // after the crash-light pass
  int32_t *d_gws = nullptr;            // gap-tier workspace
  size_t gws_cap = 0;
  char *d_cex = nullptr;               // gap-tier counterexample intervals + probes
  size_t cex_cap = 0;
  hipEvent_t eg = nullptr;
  double gap_ms = 0;
  int64_t n_gap = 0;
  hipEvent_t ef = nullptr;
  double fast_ms = 0, jit_ms = 0;
  int64_t n_jit = 0;
  lcdev::KStatus *d_status = nullptr;   // all-zero between calls
  lcdev::KStatus *h_status = nullptr;   // pinned: D2H copies of d_status
  int32_t *h_handoff = nullptr;         // host-coherent: [0] fast tier handed keys over, [1] a fused
                                        // pass's crash-light key count (status_settle_kernel)
  int32_t *h_handoff_dev = nullptr;     // its device address
  bool status_dirty = true;             // d_status may be non-zero
  // the handoff flags may be non-zero (the fast tier raised some and no
  // compaction, which clears them, followed)
  bool flags_dirty = true;
  // A fused call that handed nothing over copies its status without waiting
  // for it (the counts only choose the next call's pass and fill this call's
  // n_gap_keys): the next call, or lc_last_stats, settles it (settle_status).
  hipEvent_t es = nullptr;
  bool st_pending = false;
  int64_t st_keys = 0;
  void *d_ws = nullptr;
  size_t ws_cap = 0;
  int32_t *d_wit = nullptr;            // lc_check_ex: device copies of the lc_aux outputs
  size_t wit_cap = 0;
  int32_t *d_kind = nullptr;
  size_t kind_cap = 0;
  int32_t *d_cert = nullptr;           // lc_aux certificates (4 per key), their position sets
  size_t cert_cap = 0;
  int32_t *d_cset = nullptr;
  size_t cset_cap = 0;
  int32_t *d_cws = nullptr;            // certificate workspace
  size_t cws_cap = 0;
  double kernel_ms = 0, hbm_ms = 0;
  int64_t n_hbm = 0;
  int malformed = 0;
  bool use_fused = false;  // the next call takes the fused version-order + crash-light pass
  hipEvent_t eh0 = nullptr, eh1 = nullptr;  // around lc_check's host-to-device copies
  lc_device_stats last{};                   // this device's share of the last lc_check
  // lc_check's host-to-device pipeline: the copy stream, one event per chunk
  // (its records landed), the 24-byte staging records of lc_check32 /
  // lc_check_device32 and the keys' bases
  // (two copy streams, chunks alternating: two DMA engines read host memory
  // at once; measured 52-53 GB/s with one, 57 GB/s with two on one GPU)
  hipStream_t cst = nullptr, cst2 = nullptr;
  std::vector<hipEvent_t> cev;
  void *d_ops32 = nullptr;
  size_t ops32_cap = 0;
  int64_t *d_base = nullptr;
  size_t base_cap = 0;
  // some key of the last run_device call may be LC_INVALID (a key was handed
  // over past the version-order tier, which decides valid keys only): the
  // certificate pass runs only then
  bool maybe_invalid = true;
  double t_start = 0, t_end = 0;            // lc_call_profile: this thread's span (ms since the call began)
  // The version-order / fused pass's follower signal (kernels.h
  // launch_done_signal): a host-mapped word the host spins on instead of
  // waiting for an event; the pass's HIP-event time is read later
  // (timing_pending)
  uint32_t *h_done = nullptr, *h_done_dev = nullptr;
  uint32_t seq = 0;
  bool timing_pending = false;
  // the resident version-order grid (kernels.h launch_fast_resident), on its
  // own stream; res_grid: workgroups of the live grid (0: none)
  lcdev::ResHost *res_h = nullptr, *res_h_dev = nullptr;
  lcdev::ResDev *res_d = nullptr;
  hipStream_t rst = nullptr;
  int64_t res_grid = 0;
  uint32_t res_seq = 0;
  int res_khz = 0;          // the device's wall-clock rate
  int64_t res_idle_us = 50; // LC_RESIDENT_IDLE_US (read at each grid launch)
  int64_t res_cap = -1;     // lcdev::fast_resident_capacity() (once)
  bool res_broken = false;  // a request the grid did not complete: launches only from then on
  // this device's share of lc_last_totals: written only by the device's own
  // thread during a call (check_host runs one per device), summed by
  // lc_last_totals after the threads are joined
  lc_totals tot{};
  // lc_check's small calls from pageable memory: inputs and outputs pass
  // through this pinned buffer (kStageMax)
  char *h_stage = nullptr;
  size_t stage_cap = 0;
};

}  // namespace

struct lc_ctx {
  std::vector<Dev> devs;
  // LC_FLAG_WHOLE_GPU: frontier-exchange engines, opened on first use —
  // single-GPU ones (engine, device) and one over every GPU of the context
  std::vector<std::pair<lc_fx *, int>> fxs;
  lc_fx *fx_all = nullptr;
  bool fx_all_failed = false;
  std::string err;
  std::mutex err_mu;
  lc_stats stats{};
  // lc_host_register: caller buffers page-locked for this context's devices
  std::vector<std::pair<const char *, uint64_t>> pinned;
  std::mutex pin_mu;
  lc_call_profile prof{};  // lc_last_call_profile
};

namespace {

void set_err(lc_ctx *c, const std::string &s) {
  std::lock_guard<std::mutex> g(c->err_mu);
  c->err = s;
}

#define HIP_TRY(ctx, expr)                                                   \
  do {                                                                       \
    hipError_t e_ = (expr);                                                  \
    if (e_ != hipSuccess) {                                                  \
      set_err(ctx, std::string(#expr) + ": " + hipGetErrorString(e_));       \
      return -EIO;                                                           \
    }                                                                        \
  } while (0)

template <class T>
int ensure(lc_ctx *c, T **p, size_t *cap, size_t need) {
  if (*cap >= need && *p) return 0;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  size_t n = std::max<size_t>(need, 256);
  hipError_t e = hipMalloc(reinterpret_cast<void **>(p), n);
  if (e != hipSuccess) {
    set_err(c, std::string("hipMalloc: ") + hipGetErrorString(e));
    return -ENOMEM;
  }
  *cap = n;
  return 0;
}

int opts_to_params(lc_ctx *c, const lc_opts *o, lcdev::KParams *p) {
  lc_opts d;
  lc_default_opts(&d);
  if (!o) o = &d;
  if (o->init_version < 0 || o->init_version > 0x7FFFFFFE ||
      o->init_value < -1 || o->init_value > 0x7FFFFFFE) {
    set_err(c, "lc_opts: init_version/init_value out of int32 range");
    return -EINVAL;
  }
  p->init_ver = (int32_t)o->init_version;
  p->init_val = (int32_t)o->init_value;
  p->budget = o->max_configs_per_key > 0 ? o->max_configs_per_key : kDefaultBudget;
  p->time_ticks = 0;
  if (o->time_budget_ms > 0) {
    // device wall clock (s_memrealtime) rate, kHz = ticks per ms
    int dev = 0, khz = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0)
      khz = 100000;
    p->time_ticks = (uint64_t)o->time_budget_ms * (uint64_t)khz;
  }
  return 0;
}

// Is [p, p + n) inside a buffer registered with lc_host_register?
bool is_pinned(lc_ctx *c, const void *p, size_t n) {
  std::lock_guard<std::mutex> g(c->pin_mu);
  const char *q = static_cast<const char *>(p);
  for (const auto &pr : c->pinned)
    if (q >= pr.first && q + n <= pr.first + pr.second) return true;
  return false;
}

// lc_check's host-to-device pipeline on one device: the device's key range
// cut into chunks of about kChunkBytes of records.  run_device calls
// issue(i), which enqueues chunk i's record copy on the copy stream and
// records ready[i]; the compute stream waits for that event, widens 24-byte
// records (lc_check32), and runs the version-order (or fused) pass over the
// chunk's keys while the copy engine moves the next chunk.  (A pageable copy
// may block the issuing thread until it has landed; issuing each chunk's
// copy right before its kernels keeps the overlap either way.)
struct Chunks {
  int n = 0;
  std::vector<int64_t> k;   // key boundaries, n + 1, local to the device's range
  std::vector<int64_t> r;   // record offsets of those keys from the range's first record
  std::function<int(int)> issue;
  const hipEvent_t *ready = nullptr;
  const lc_op32 *d_ops32 = nullptr;  // staging records to widen into d_ops (null: 48-byte copies)
  const lc_op16 *d_ops16 = nullptr;  // (lc_check16) the same for 16-byte records
  const int64_t *d_base = nullptr;   // key bases for the widening (null: 0)
  int64_t max_len = 0;               // longest key (records)
};
// Chunks of kChunkBytes, the last ones halving down to kChunkTail: the
// compute stream's tail after the last copy is one small chunk's widening and
// version-order pass.  (Measured on C2's 240 MB of 24-byte records: 10
// chunks of 24 MB 4.66 ms per call, 0.12 ms of it after the last copy; 29
// chunks of 8 MB 5.2 ms — each pageable copy has a fixed cost.)
constexpr size_t kChunkBytes = size_t(24) << 20;
constexpr size_t kChunkTail = size_t(2) << 20;
constexpr int kMaxChunks = 48;
// A call whose pageable inputs and outputs fit in kStageMax bytes copies them
// through the device's pinned staging buffer (a memcpy on the host, then a
// DMA from pinned memory): the runtime's pageable path costs tens of
// microseconds per copy, which small calls (C1, C4) pay in full.  At a few
// MB the runtime's path is the faster one again (a 4.8 MB input staged:
// 0.07-0.15 ms slower, profiles/r05/stage_ab.txt).
// LC_STAGE=0 (A/B): the pageable copies.
constexpr size_t kStageMax = size_t(2) << 20;
bool stage_off() {
  const char *e = getenv("LC_STAGE");
  return e && e[0] == '0';
}
// The device's staging buffer (kStageMax bytes, allocated on first use), or
// null with the context's error set.
char *stage_buf(lc_ctx *c, Dev &d) {
  if (!d.h_stage) {
    if (hipHostMalloc(reinterpret_cast<void **>(&d.h_stage), kStageMax, 0) != hipSuccess) {
      d.h_stage = nullptr;
      set_err(c, "hipHostMalloc (staging) failed");
      return nullptr;
    }
    d.stage_cap = kStageMax;
  }
  return d.h_stage;
}

// Device-side lc_aux outputs of one run_device call (null: not wanted).
struct WitOut {
  int32_t *wit = nullptr;   // per record, indexed like d_ops
  int32_t *kind = nullptr;  // per key
  int32_t *cert = nullptr;  // per key, 4 int32 (infeasibility certificates)
  int32_t *cset = nullptr;  // per record (HALL position sets)
  int64_t n_records = 0;
  // (not an output) the shard's key offsets in host memory when the caller
  // has them (lc_check_ex): the gap tier may then be launched early
  const int64_t *h_off = nullptr;
  // (not an output) lc_check's chunked copies, or null: the records are in place
  const Chunks *chunks = nullptr;
  // (not an output) the first pass over lc_op32 records (lc_check32 /
  // lc_check_device32 without lc_aux outputs): ops32 and the keys' bases
  // (null: 0), indexed like d_ops / d_off; `widen` fills the 48-byte records
  // the later tiers read (and names them) once a key is handed over
  const lc_op32 *ops32 = nullptr;
  const int64_t *base32 = nullptr;
  std::function<int(const lc_op **)> widen;
};

// A gap-tier full-decision launch: its sizes and job (run_device).
struct GapPlan {
  int64_t gap_cap = 0;     // workspace entries per array per workgroup
  size_t gap_per_wg = 0;
  int wg_cap = 0, full_wg = 0;
  bool wide_wg = false, no_lds = false;
  size_t nk = 0;           // counterexample slots (the cex arrays' stride)
  lcdev::GapJob job{};
};

// Infeasibility certificates for the invalid keys of a run_device call
// (cert.hip), after every tier has decided.
int run_certificates(lc_ctx *c, Dev &d, const lc_op *d_ops, const int64_t *d_off, int64_t n_keys,
                     const lcdev::KParams &p, const lc_key_result *d_out, hipStream_t st,
                     const WitOut &wo) {
  if (!wo.cert || !wo.cset || n_keys <= 0) return 0;
  if (!d.maybe_invalid) {
    // every key was decided by the version-order tier, which decides valid
    // keys only: no certificate to find, every key LC_CERT_NONE
    HIP_TRY(c, lcdev::launch_cert_none(wo.cert, n_keys, st));
    return 0;
  }
  if (int rc = ensure(c, reinterpret_cast<char **>(&d.d_cws), &d.cws_cap,
                      lcdev::cert_ws_bytes(wo.n_records, n_keys)))
    return rc;
  HIP_TRY(c, lcdev::launch_certificates(d_ops, d_off, n_keys, wo.n_records, p, d_out, d.d_cws,
                                        wo.cert, wo.cset, st));
  HIP_TRY(c, hipStreamSynchronize(st));
  return 0;
}

// A fused call's lazily copied status (Dev::st_pending): choose the next
// call's pass from it and return the keys the crash-light decision took (the
// call's n_gap), or -1 when nothing was pending.
int64_t settle_status(Dev &d) {
  if (!d.st_pending) return -1;
  d.st_pending = false;
  if (hipEventSynchronize(d.es) != hipSuccess) return 0;
  const int32_t n_light = __atomic_load_n(d.h_handoff + 1, __ATOMIC_ACQUIRE);  // (status_settle_kernel)
  d.use_fused = 4 * (int64_t)n_light > d.st_keys;
  return n_light;
}

// A call that returned on the completion signal: its pass's HIP-event time,
// read once the kernel has retired (now, if it has not yet), into the
// device's statistics and the context's totals.  Before the events are
// recorded again, and by lc_last_stats / lc_last_totals.
void settle_timing(lc_ctx *c, Dev &d) {
  if (!d.timing_pending) return;
  d.timing_pending = false;
  float ms = 0;
  if (hipEventSynchronize(d.ef) == hipSuccess && hipEventElapsedTime(&ms, d.e0, d.ef) == hipSuccess) {
    d.fast_ms = ms;
    d.kernel_ms = ms;
    d.tot.timed_calls++;
    d.tot.fast_kernel_ms += ms;
    d.tot.kernel_ms += ms;
  }
}

// LC_NATIVE32=0 (A/B): 24-byte records are widened before the first pass, as
// in the first ABI-4 build, instead of decided as they are
bool native32_off() {
  const char *e = getenv("LC_NATIVE32");
  return e && e[0] == '0';
}

// Wait for the pass's follower signal (seq in *h_done): spin, checking the
// stream every 1,024 rounds; past 2 ms (or once the stream is idle, which
// cannot happen before the word) synchronise the stream instead.  Returns 0,
// or -EIO on a stream error.
int wait_done(lc_ctx *c, Dev &d, uint32_t seq, hipStream_t st) {
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t i = 1;; i++) {
    if (__atomic_load_n(d.h_done, __ATOMIC_ACQUIRE) == seq) return 0;
    if ((i & 1023) == 0) {
      const hipError_t q = hipStreamQuery(st);
      if (q == hipSuccess) return 0;
      if (q != hipErrorNotReady) {
        set_err(c, std::string("fast tier: ") + hipGetErrorString(q));
        return -EIO;
      }
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) {
        HIP_TRY(c, hipStreamSynchronize(st));
        return 0;
      }
    }
  }
}

// ---- Resident version-order grid (kernels.h, launch_fast_resident) ----
// lc_check_device on a batch of at most one key per resident workgroup
// (C3's 1,250-key shard) is served by a grid that stays on the GPU between
// calls: the call writes the request and rings, the grid decides it and
// signals, and back-to-back calls pay neither a launch nor the follower
// kernel.  The grid leaves after LC_RESIDENT_IDLE_US (default 50) without a
// request, before any other work of this library runs on the device, and at
// lc_close.  LC_RESIDENT=0 turns it off (every call launches).
bool resident_off() {
  const char *e = getenv("LC_RESIDENT");
  return e && e[0] == '0';
}

// Write request number d.res_seq + 1 (every word tagged with it).
void res_ring(Dev &d, const uint64_t (&v)[lcdev::kResWords]) {
  const uint32_t seq = ++d.res_seq;
  for (int i = 0; i < lcdev::kResWords; i++)
    __atomic_store_n(&d.res_h->req[i], lcdev::res_word(v[i], seq), __ATOMIC_RELEASE);
}

// Stop the grid (if one is live) and wait for it to leave.
int res_stop(lc_ctx *c, Dev &d) {
  if (!d.res_grid) return 0;
  uint64_t v[lcdev::kResWords] = {};
  v[2] = (uint64_t)lcdev::kResExitKeys;
  res_ring(d, v);
  d.res_grid = 0;
  HIP_TRY(c, hipStreamSynchronize(d.rst));
  return 0;
}

// One request: returns 0 with every key decided or flagged for the later
// tiers (d.h_handoff as after fast_tier_kernel), its device time in
// *dev_ms; 1 when the grid could not serve it (the caller launches
// instead); or a negative error.
int res_request(lc_ctx *c, Dev &d, const lc_op *d_ops, const int64_t *d_off, int64_t n_keys,
                const lcdev::KParams &p, lc_key_result *d_out, hipStream_t st, double *dev_ms) {
  if (!d.res_h) {
    if (hipHostMalloc(reinterpret_cast<void **>(&d.res_h), sizeof(lcdev::ResHost),
                      hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer(reinterpret_cast<void **>(&d.res_h_dev), d.res_h, 0) != hipSuccess ||
        hipMalloc(reinterpret_cast<void **>(&d.res_d), sizeof(lcdev::ResDev)) != hipSuccess ||
        hipStreamCreateWithFlags(&d.rst, hipStreamNonBlocking) != hipSuccess ||
        hipDeviceGetAttribute(&d.res_khz, hipDeviceAttributeWallClockRate, d.id) != hipSuccess ||
        d.res_khz <= 0) {
      d.res_broken = true;
      return 1;
    }
    std::memset(static_cast<void *>(d.res_h), 0, sizeof(lcdev::ResHost));
  }
  // the inputs (and this call's memsets) are ready once the caller's stream is
  if (hipStreamQuery(st) != hipSuccess) HIP_TRY(c, hipStreamSynchronize(st));
  lcdev::ResHost *h = d.res_h;
  const uint64_t v[lcdev::kResWords] = {
      (uint64_t)d_ops, (uint64_t)d_off, (uint64_t)n_keys, (uint64_t)d_out, (uint64_t)d.d_flags,
      (uint64_t)d.d_status, (uint64_t)d.h_handoff_dev, (uint64_t)(uint32_t)p.init_ver,
      (uint64_t)(uint32_t)p.init_val};
  for (int attempt = 0; attempt < 3; attempt++) {
    // a grid that left on its idle bound has finished (its stream drained)
    // before a new one starts; a grid too small for this batch is stopped
    if (d.res_grid && (__atomic_load_n(&h->exited, __ATOMIC_ACQUIRE) || d.res_grid < n_keys))
      if (int e = res_stop(c, d)) return e;
    if (!d.res_grid) {
      // a new grid: numbering from 0 (no word tagged 1 yet), counters zero
      for (int i = 0; i < 16; i++) __atomic_store_n(&h->req[i], 0, __ATOMIC_RELAXED);
      __atomic_store_n(&h->exited, 0u, __ATOMIC_RELAXED);
      __atomic_store_n(&h->done, 0, __ATOMIC_RELEASE);
      d.res_seq = 0;
      const char *ie = getenv("LC_RESIDENT_IDLE_US");  // (read at each launch)
      d.res_idle_us = ie ? std::max<int64_t>(1, atoll(ie)) : 50;
      HIP_TRY(c, hipMemsetAsync(d.res_d, 0, sizeof(lcdev::ResDev), d.rst));
      HIP_TRY(c, lcdev::launch_fast_resident(d.res_h_dev, d.res_d, n_keys,
                                             (uint64_t)d.res_idle_us * (uint64_t)d.res_khz / 1000u,
                                             d.rst));
      d.res_grid = n_keys;
    }
    res_ring(d, v);
    const uint32_t seq = d.res_seq;
    // wait for the completion; every 1,024 rounds check that the grid has
    // not left (idle bound before the request: serve it from a new grid)
    // and bound the wait (a request is at most ~0.1 ms of device work)
    const auto t0 = std::chrono::steady_clock::now();
    bool left = false;
    for (uint32_t i = 1;; i++) {
      const uint64_t dn = __atomic_load_n(&h->done, __ATOMIC_ACQUIRE);
      if ((uint32_t)(dn >> 32) == seq) {
        const uint32_t a = (uint32_t)__atomic_load_n(&h->t0, __ATOMIC_RELAXED);
        *dev_ms = (double)(uint32_t)((uint32_t)dn - a) / (double)d.res_khz;
        return 0;
      }
      if ((i & 1023) == 0) {
        if (__atomic_load_n(&h->exited, __ATOMIC_ACQUIRE)) {
          left = true;
          break;
        }
        const hipError_t q = hipStreamQuery(d.rst);
        if (q != hipSuccess && q != hipErrorNotReady) {
          set_err(c, std::string("resident grid: ") + hipGetErrorString(q));
          d.res_grid = 0;
          d.res_broken = true;
          return -EIO;
        }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(500)) break;
      }
    }
    if (int e = res_stop(c, d)) return e;
    if (!left) break;  // not served in 500 ms: launches from now on
    // (the grid left before it saw the request: the host was away longer
    // than the idle bound) — again, from a new grid
  }
  d.res_broken = true;
  return 1;
}

// Run the tiers for n_keys keys whose device arrays are in place.
int run_device(lc_ctx *c, Dev &d, const lc_op *d_ops, const int64_t *d_off,
               int64_t n_keys, const lcdev::KParams &p,
               lc_key_result *d_out, hipStream_t st, int64_t flags,
               const WitOut &wo = WitOut()) {
  (void)settle_status(d);  // before use_fused or h_status is read
  settle_timing(c, d);     // before e0 / ef are recorded again
  d.tot.calls++;
  d.kernel_ms = d.hbm_ms = d.fast_ms = d.jit_ms = d.gap_ms = 0;
  d.n_hbm = d.n_jit = d.n_gap = 0;
  d.malformed = 0;
  if (n_keys <= 0) return 0;
  if (n_keys > INT32_MAX) {
    set_err(c, "lc_check: more than 2^31-1 keys in one call");
    return -EINVAL;
  }
  int rc = ensure(c, &d.d_ovf, &d.ovf_cap, sizeof(int32_t) * (size_t)n_keys);
  if (!rc) rc = ensure(c, &d.d_ovf2, &d.ovf2_cap, sizeof(int32_t) * (size_t)n_keys);
  if (!rc) rc = ensure(c, &d.d_jit, &d.jit_cap, sizeof(int32_t) * (size_t)n_keys);
  if (!rc) rc = ensure(c, &d.d_jit2, &d.jit2_cap, sizeof(int32_t) * (size_t)n_keys);
  if (!rc) rc = ensure(c, &d.d_gap2, &d.gap2_cap, sizeof(int32_t) * (size_t)n_keys);
  const bool flags_new = d.flags_cap < sizeof(int32_t) * (size_t)n_keys || !d.d_flags;
  if (!rc) rc = ensure(c, &d.d_flags, &d.flags_cap, sizeof(int32_t) * (size_t)n_keys);
  if (rc) return rc;
  if (flags_new || d.flags_dirty)  // the flags are all-zero between calls that completed
    HIP_TRY(c, hipMemsetAsync(d.d_flags, 0, d.flags_cap, st));
  d.flags_dirty = false;
  // With the gap tier on, the fast tier sends keys it can only pass on (no
  // version on an :ok mutation, a read [nil x], malformed) straight to the
  // JIT list d_jit2, which the gap tier then appends to.
  const bool gap_on = !(flags & (LC_FLAG_NO_FAST_PATH | LC_FLAG_NO_GAP_TIER));
  int64_t n_direct = 0;
  // d_status is zero on entry (the fast tier re-zeroes it; later tiers are
  // followed by a memset).  Until this call ends cleanly, assume it is not.
  if (d.status_dirty)
    HIP_TRY(c, hipMemsetAsync(d.d_status, 0, sizeof(lcdev::KStatus), st));
  d.status_dirty = true;
  float ms = 0;
  // the gap tier's full-decision launch for keys up to max_len records long,
  // nj of them at most (buffers ensured)
  auto gap_plan = [&](int64_t max_len, int64_t nj, GapPlan &g) -> int {
    g.gap_cap = (max_len + 2 + 3) & ~int64_t(3);  // 16-B records
    g.gap_per_wg = lcdev::gap_tier_ws_bytes(1, g.gap_cap);
    if (g.gap_per_wg > kGapWsBytes) return 0;  // (the caller checks)
    g.wg_cap = (int)std::min<int64_t>(
        (int64_t)kGapMaxWG, std::max<int64_t>(1, (int64_t)(kGapWsBytes / g.gap_per_wg)));
    // many short keys: one-wave workgroups, four times as many decisions in
    // flight (10k 200-op keys: 0.78 -> 0.45 ms); few keys are latency-bound
    // and decide faster with 256 threads each (94 keys: 0.19 vs 0.145 ms)
    const bool wave_wg = max_len <= kGapWaveMaxLen && nj > kGapWaveMinKeys;
    g.full_wg = (int)std::min<int64_t>(nj, wave_wg ? 4 * (int64_t)g.wg_cap : g.wg_cap);
    int rc2 = ensure(c, reinterpret_cast<char **>(&d.d_gws), &d.gws_cap,
                     lcdev::gap_tier_ws_bytes(g.full_wg, g.gap_cap));
    // counterexample intervals: key, lo, hi, gaps, state (int32), nodes
    // (int64) per invalid key, and one int32 per probe workgroup
    g.nk = (size_t)nj;
    if (!rc2) rc2 = ensure(c, &d.d_cex, &d.cex_cap, g.nk * (5 * 4 + 8) + 4 * (size_t)g.wg_cap + 64);
    if (rc2) return rc2;
    lcdev::GapJob &job = g.job;
    job = lcdev::GapJob{};
    // LC_GAP_PREF_BUDGET (tests): a tiny budget sends every branching decision
    // through the plain-order rerun
    const char *pb_env = getenv("LC_GAP_PREF_BUDGET");
    job.pref_budget = pb_env ? std::max(1, atoi(pb_env)) : lcdev::kGapPrefBudget;
    const size_t nk = g.nk;
    job.cex_nodes = reinterpret_cast<int64_t *>(d.d_cex);
    job.cex_key = reinterpret_cast<int32_t *>(d.d_cex + 8 * nk);
    job.cex_lo = reinterpret_cast<uint32_t *>(job.cex_key + nk);
    job.cex_hi = job.cex_lo + nk;
    job.cex_gaps = reinterpret_cast<int32_t *>(job.cex_hi + nk);
    job.cex_state = job.cex_gaps + nk;
    job.probe = job.cex_state + nk;
    job.mode = lcdev::kGapFull;
    job.n_tasks = (int32_t)nj;
    const bool wants_wit = wo.wit && wo.kind;
    job.wit = wants_wit ? wo.wit : nullptr;
    job.wkind = wants_wit ? wo.kind : nullptr;
    // short keys: one-wave workgroups (barriers nearly free, 4x the decisions
    // in flight); longer keys: 256 threads share each decision's setup; a
    // few long keys (C4): 512, whose extra waves halve the setup's record
    // passes (the matching is one wave either way)
    const char *wide_env = getenv("LC_GAP_WIDE");  // A/B: 0 keeps 256
    g.wide_wg = !(wide_env && wide_env[0] == '0') && nj <= kGapWideMaxKeys &&
                max_len >= kGapWideMinLen;
    job.threads = wave_wg ? 64 : g.wide_wg ? 512 : 256;
    // Bisect counterexamples in place unless the keys are long and few
    // enough for multisection rounds to pay (each round costs two launches
    // and a sync; a probe of a short key costs less than that).
    job.bisect = max_len < kGapProbeMinLen || 2 * nj > g.wg_cap;
    // LDS per workgroup: the longest key's skeleton (68 B per record) plus
    // 8 KB for its matching when that stays within kGapSkelLdsMax (two
    // workgroups per CU); else room for the matching alone (80 B per record
    // plus its class table at worst), up to kGapLdsFull, or kGapLdsFew when
    // there are few keys
    const int64_t skel = 68 * g.gap_cap + (8 << 10);
    const int64_t match_cap = nj <= kGapFewKeys ? kGapLdsFew : kGapLdsFull;
    job.lds_bytes = (int)(skel <= kGapSkelLdsMax ? skel
                                                 : std::min<int64_t>(match_cap, 80 * g.gap_cap + 1040));
    // LC_GAP_LDS=0 (tests): keep every matching in the HBM workspace
    const char *lds_env = getenv("LC_GAP_LDS");
    g.no_lds = lds_env && lds_env[0] == '0';
    if (g.no_lds) job.lds_bytes = 0;
    return 0;
  };
  GapPlan early;              // the gap tier launched early (below), if it was
  bool early_launched = false;
  bool light = false;  // the crash-light pass ran (its time is in gap_ms)
  bool fused = false;  // the version-order and crash-light decisions ran as one pass
  int64_t n_jit = n_keys;
  const int32_t *jit_list = nullptr;
  const bool want_wit = wo.wit && wo.kind;
  const bool fast_on = !(flags & LC_FLAG_NO_FAST_PATH);
  d.maybe_invalid = true;
  if (fast_on) {
    // Crash-heavy batches (most keys carry crashed writes/CAS: every key goes
    // on to the crash-light decision) take the fused pass, which reads each
    // key's records once for both decisions; others the version-order tier,
    // whose smaller register budget keeps 7 workgroups per CU.  Chosen from
    // the previous call on this device (LC_FUSED=0/1 forces it).
    const char *fenv = getenv("LC_FUSED");
    fused = gap_on && (fenv ? fenv[0] == '1' : d.use_fused);
    // Only when some workgroup raised h_handoff is the count copied back.
    __atomic_store_n(d.h_handoff, 0, __ATOMIC_RELEASE);
    d.flags_dirty = true;  // until the handoff (if any) is compacted
  }
  // keys [k0, k0 + nk), records from r0 (relative to d_ops): the witness
  // initialisation (the version order is the witness of every key the fast
  // tier decides) and tier 0, the version-order decision (or the fused
  // pass); the keys it cannot decide are flagged for the later tiers
  // A call with one pass launch (no chunks) returns on the pass's follower
  // signal (kernels.h launch_done_signal) instead of an event wait; with
  // LC_FLAG_NO_TIMING it records no events around the pass either.
  const bool signal = !wo.chunks && fast_on && n_keys > 0;
  bool timing = !signal || !(flags & LC_FLAG_NO_TIMING);
  // the resident grid serves lc_check_device's plain version-order pass on
  // a batch of at most one key per resident workgroup (res_request); any
  // other call on this device first stops a live grid
  if (d.res_cap < 0) d.res_cap = lcdev::fast_resident_capacity();
  const bool resident = signal && !fused && !want_wit && !wo.ops32 && !d.res_broken &&
                        n_keys <= d.res_cap && !resident_off();
  int res_rc = 1;  // 0: the grid decided the pass
  double res_ms = 0;
  if (resident) {
    res_rc = res_request(c, d, d_ops, d_off, n_keys, p, d_out, st, &res_ms);
    if (res_rc < 0) return res_rc;
    if (res_rc == 1) {
      // not served (the grid may have decided part of it): launch instead,
      // from the state the pass starts from
      HIP_TRY(c, hipMemsetAsync(d.d_status, 0, sizeof(lcdev::KStatus), st));
      HIP_TRY(c, hipMemsetAsync(d.d_flags, 0, d.flags_cap, st));
      __atomic_store_n(d.h_handoff, 0, __ATOMIC_RELEASE);
    } else {
      timing = true;  // (the grid's device clock: free)
    }
  } else if (d.res_grid) {
    if (int e = res_stop(c, d)) return e;
  }
  auto first_pass = [&](int64_t k0, int64_t nk, int64_t r0, int64_t nrec) -> int {
    const int64_t *off = d_off + k0;
    if (wo.ops32) {  // the native 24-byte pass (no lc_aux outputs)
      const int64_t *base = wo.base32 ? wo.base32 + k0 : nullptr;
      if (fused)
        HIP_TRY(c, lcdev::launch_fused_tier32(wo.ops32 + r0, off, base, nk, p, d_out + k0,
                                              d.d_flags + k0, d.d_status, d.h_handoff_dev, st));
      else
        HIP_TRY(c, lcdev::launch_fast_tier32(wo.ops32 + r0, off, base, nk, p, d_out + k0,
                                             d.d_flags + k0, d.d_status, d.h_handoff_dev, st));
      return 0;
    }
    const lc_op *o = d_ops + r0;
    int32_t *wit = want_wit ? wo.wit + r0 : nullptr;
    int32_t *kind = want_wit ? wo.kind + k0 : nullptr;
    if (want_wit)
      HIP_TRY(c, lcdev::launch_witness_init(o, off, nk, nrec, p, fast_on, wit, kind, st));
    if (!fast_on) return 0;
    if (fused)
      HIP_TRY(c, lcdev::launch_fused_tier(o, off, nk, p, d_out + k0, d.d_flags + k0, d.d_status,
                                          d.h_handoff_dev, wit, kind, st));
    else
      HIP_TRY(c, lcdev::launch_fast_tier(o, off, nk, p, d_out + k0, d.d_flags + k0, d.d_status,
                                         d.h_handoff_dev, st));
    return 0;
  };
  if (res_rc == 0) {
    // (decided by the resident grid)
  } else if (timing) {
    HIP_TRY(c, hipEventRecord(d.e0, st));
  }
  if (res_rc == 0) {
  } else if (const Chunks *ch = wo.chunks) {
    // lc_check's pipeline: chunk i's copy is issued, the compute stream
    // waits for it, widens it (24-byte records) and decides its keys while
    // the copy engine moves chunk i + 1
    for (int i = 0; i < ch->n; i++) {
      if (int e = ch->issue(i)) return e;
      HIP_TRY(c, hipStreamWaitEvent(st, ch->ready[i], 0));
      const int64_t k0 = ch->k[i], nk = ch->k[i + 1] - k0;
      const int64_t r0 = ch->r[i], nrec = ch->r[i + 1] - r0;
      if (nk <= 0) continue;
      if (ch->d_ops32 && !wo.ops32)
        HIP_TRY(c, lcdev::launch_widen32(ch->d_ops32 + r0, d_off + k0,
                                         ch->d_base ? ch->d_base + k0 : nullptr, nk, ch->max_len,
                                         const_cast<lc_op *>(d_ops) + r0, st));
      if (ch->d_ops16)
        HIP_TRY(c, lcdev::launch_widen16(ch->d_ops16 + r0, d_off + k0,
                                         ch->d_base ? ch->d_base + k0 : nullptr, nk, ch->max_len,
                                         const_cast<lc_op *>(d_ops) + r0, st));
      if (int e = first_pass(k0, nk, r0, nrec)) return e;
    }
  } else if (int e = first_pass(0, n_keys, 0, wo.n_records)) {
    return e;
  }
  if (fast_on) {
    if (res_rc == 0) {
      // (completed already)
    } else if (timing) {
      HIP_TRY(c, hipEventRecord(d.ef, st));
    }
    if (res_rc == 0) {
    } else if (signal) {
      HIP_TRY(c, lcdev::launch_done_signal(d.h_done_dev, ++d.seq, st));
      if (int e = wait_done(c, d, d.seq, st)) return e;
    } else {
      HIP_TRY(c, hipEventSynchronize(d.ef));
    }
    n_jit = 0;
    jit_list = d.d_jit;
    const bool handed = __atomic_load_n(d.h_handoff, __ATOMIC_ACQUIRE) != 0;
    if (res_rc == 0) {
      d.fast_ms = res_ms;
      if (handed) {
        // the grid's exit publishes the flags and the status words to the
        // later tiers (and frees its CUs); their times are measured from here
        if (int e = res_stop(c, d)) return e;
        HIP_TRY(c, hipEventRecord(d.e0, st));
        HIP_TRY(c, hipEventRecord(d.ef, st));
      }
    } else if (signal && !handed) {
      // every key decided: the pass's event time (if any) is read later
      d.timing_pending = timing;
    } else {
      if (!timing) {
        // the later tiers' times are measured from here (the pass untimed)
        HIP_TRY(c, hipEventRecord(d.e0, st));
        HIP_TRY(c, hipEventRecord(d.ef, st));
      }
      HIP_TRY(c, hipEventSynchronize(d.ef));
      HIP_TRY(c, hipEventElapsedTime(&ms, d.e0, d.ef));
      d.fast_ms = ms;
    }
    if (!handed) {
      d.flags_dirty = false;  // no key raised its flag
      // the version-order tier and the fused pass decide valid keys only
      // (they hand invalid ones on for their counterexamples)
      d.maybe_invalid = false;
    }
    if (fused && !handed) {
      // every key decided in the one pass: were most of them crash-light?
      // (the answer picks the next call's pass; copied now, read later)
      // (one launch: the count to mapped host memory, d_status zeroed behind
      // it now — while the host returns — not at the start of the next call)
      HIP_TRY(c, lcdev::launch_status_settle(d.d_status, d.h_handoff_dev + 1, st));
      HIP_TRY(c, hipEventRecord(d.es, st));
      d.st_pending = true;
      d.st_keys = n_keys;
      d.status_dirty = false;
    }
    if (handed) {
      // the native 24-byte pass: the later tiers read 48-byte records
      if (wo.widen)
        if (int e = wo.widen(&d_ops)) return e;
      HIP_TRY(c, lcdev::launch_handoff_compact(d.d_flags, d_off, n_keys, gap_on ? 1 : 0, d.d_jit,
                                               d.d_jit2, d.d_status, want_wit ? wo.kind : nullptr,
                                               st));
      d.flags_dirty = false;  // the compaction clears every flag it reads
      // the crash-light pass reads the list and its length from the device:
      // no host round trip between the compaction and it.  After the fused
      // pass too: the keys it hands over are invalid or beyond the in-place
      // decision, and the light pass names an invalid version-pinned key's
      // first failure (check_kernel.hip, first_failure), so every path gives
      // the same results
      if (gap_on) {
        HIP_TRY(c, lcdev::launch_gap_light(d_ops, d_off, d.d_jit, n_keys, p, d_out, d.d_gap2,
                                           d.d_status, want_wit ? wo.wit : nullptr,
                                           want_wit ? wo.kind : nullptr, st));
        HIP_TRY(c, hipEventRecord(d.el, st));
        // Launched early: a few keys, one longer than the light pass holds
        // (kFastMaxRecords: it goes on to the gap tier proper) and the
        // shard's offsets in host memory — the full decisions start right
        // behind the light pass, sized from those offsets, their count read
        // on the device (GapJob::n_tasks_dev), instead of after a host round
        // trip for the status.  Same decisions, same results.
        if (wo.h_off && n_keys <= kGapWideMaxKeys) {
          int64_t ml = 0;
          for (int64_t k = 0; k < n_keys; k++) ml = std::max<int64_t>(ml, wo.h_off[k + 1] - wo.h_off[k]);
          const char *ee = getenv("LC_GAP_EARLY");  // A/B: 0 waits for the status
          if (ml > lcdev::kFastMaxRecords && !(ee && ee[0] == '0')) {
            if (int e = gap_plan(ml, n_keys, early)) return e;
            if (early.gap_per_wg <= kGapWsBytes) {
              early.job.n_tasks_dev = &d.d_status->n_gap2;
              HIP_TRY(c, lcdev::launch_gap_tier(d_ops, d_off, d.d_gap2, p, d_out, d.d_gws,
                                                early.full_wg, early.gap_cap, d.d_jit2, d.d_status,
                                                early.job, st));
              HIP_TRY(c, hipEventRecord(d.eg, st));
              early_launched = true;
            }
          }
        }
      }
      HIP_TRY(c, hipMemcpyAsync(d.h_status, d.d_status, sizeof(lcdev::KStatus),
                                hipMemcpyDeviceToHost, st));
      HIP_TRY(c, hipStreamSynchronize(st));
      n_direct = d.h_status->n_jit2;
      if (fused) lcdev::light_count(*d.h_status);
      if (gap_on) {
        // fused: were most keys crash-light?  Else: most keys handed to the
        // gap tier: the next call fuses the passes
        d.use_fused = fused ? 4 * (int64_t)d.h_status->n_light > n_keys
                            : 2 * (int64_t)d.h_status->n_jit > n_keys;
        light = true;
        HIP_TRY(c, hipEventElapsedTime(&ms, d.ef, d.el));
        d.gap_ms = ms;
        d.n_gap = fused ? d.h_status->n_light : d.h_status->n_jit;
        n_jit = d.h_status->n_gap2;  // what the gap tier proper still has to decide
        jit_list = d.d_gap2;
      } else {
        n_jit = d.h_status->n_jit;
      }
    }
  } else {
    HIP_TRY(c, hipEventRecord(d.ef, st));
  }
  if (n_jit == 0 && n_direct == 0) {
    d.kernel_ms = d.fast_ms + d.gap_ms;
    if (!d.timing_pending && timing) {
      d.tot.timed_calls++;
      d.tot.fast_kernel_ms += d.fast_ms;
      d.tot.kernel_ms += d.kernel_ms;
    }
    // after a handoff d_status is not zero: cleared behind this call's work
    // (the host has read it), not in front of the next call's
    if (light) HIP_TRY(c, hipMemsetAsync(d.d_status, 0, sizeof(lcdev::KStatus), st));
    d.status_dirty = false;
    return 0;
  }
  hipEvent_t before_jit = light ? d.el : d.ef;
  const int64_t gap_cap = ((int64_t)d.h_status->max_len + 2 + 3) & ~int64_t(3);  // 16-B records
  const size_t gap_per_wg = lcdev::gap_tier_ws_bytes(1, gap_cap);
  if (gap_on && (n_jit == 0 || gap_per_wg > kGapWsBytes)) {
    // no gap-tier pass: its queue (if any) joins the direct keys for the JIT
    if (n_jit > 0)
      HIP_TRY(c, hipMemcpyAsync(d.d_jit2 + n_direct, jit_list, sizeof(int32_t) * (size_t)n_jit,
                                hipMemcpyDeviceToDevice, st));
    n_jit += n_direct;
    jit_list = d.d_jit2;
  } else if (gap_on) {
    // tier 1: gap matching for version-pinned keys (crashed writes/CAS, long
    // keys, invalid keys); what it cannot decide goes on to the JIT search
    GapPlan g;
    if (early_launched) {
      g = early;  // launched behind the light pass; the status read since includes it
    } else {
      if (int e = gap_plan(d.h_status->max_len, n_jit, g)) return e;
      HIP_TRY(c, lcdev::launch_gap_tier(d_ops, d_off, jit_list, p, d_out, d.d_gws, g.full_wg,
                                        g.gap_cap, d.d_jit2, d.d_status, g.job, st));
      HIP_TRY(c, hipMemcpyAsync(d.h_status, d.d_status, sizeof(lcdev::KStatus),
                                hipMemcpyDeviceToHost, st));
      HIP_TRY(c, hipStreamSynchronize(st));
    }
    lcdev::GapJob &job = g.job;
    job.n_tasks_dev = nullptr;
    const int wg_cap = g.wg_cap;
    const bool wide_wg = g.wide_wg, no_lds = g.no_lds;
    const int32_t n_cex = d.h_status->n_cex;
    if (n_cex > 0) {
      // counterexamples of long keys: P probes per interval per round, over
      // the whole GPU
      job.mode = lcdev::kGapProbe;
      // the probes of a few long keys: 512-thread workgroups as for their full
      // decisions (half as many probes per round; C4's interval still closes in
      // two rounds)
      const char *wp_env = getenv("LC_GAP_WIDE_PROBE");  // A/B: 0 keeps 256
      job.threads = wide_wg && !(wp_env && wp_env[0] == '0') ? 512 : 256;
      job.lds_bytes = no_lds ? 0 : kGapLdsProbe;
      // as many probes as run at once: a round's time is its slowest batch
      // of resident workgroups, and a second batch doubles it for a few
      // more cuts (C4 invalid: 1,024 probes = two batches of 512 resident)
      const int resident = lcdev::gap_tier_resident(job.lds_bytes, job.threads);
      job.P = (resident / n_cex >= 2 ? std::min(resident, wg_cap) : wg_cap) / n_cex;
      job.n_tasks = n_cex * job.P;
      rc = ensure(c, reinterpret_cast<char **>(&d.d_gws), &d.gws_cap,
                  lcdev::gap_tier_ws_bytes(job.n_tasks, gap_cap));
      if (rc) return rc;
      for (int round = 0;; round++) {
        if (round == kGapMaxRounds) {
          // cannot happen (each round cuts an interval by P + 1 >= 3); the
          // JIT tier decides whatever is still open rather than the call fail
          job.give_up = 1;
          HIP_TRY(c, lcdev::launch_gap_narrow(d_ops, d_off, n_cex, d_out, d.d_jit2, d.d_status,
                                              job, st));
          break;
        }
        HIP_TRY(c, hipMemsetAsync(&d.d_status->n_open, 0, sizeof(int32_t), st));
        HIP_TRY(c, lcdev::launch_gap_tier(d_ops, d_off, nullptr, p, d_out, d.d_gws, job.n_tasks,
                                          gap_cap, d.d_jit2, d.d_status, job, st));
        HIP_TRY(c, lcdev::launch_gap_narrow(d_ops, d_off, n_cex, d_out, d.d_jit2, d.d_status,
                                            job, st));
        HIP_TRY(c, hipMemcpyAsync(d.h_status, d.d_status, sizeof(lcdev::KStatus),
                                  hipMemcpyDeviceToHost, st));
        HIP_TRY(c, hipStreamSynchronize(st));
        if (d.h_status->n_open == 0) break;
      }
      if (want_wit) {
        // the witness of each closed counterexample's last linearizable prefix
        job.mode = lcdev::kGapWitness;
        job.P = 1;
        job.n_tasks = n_cex;
        HIP_TRY(c, lcdev::launch_gap_tier(d_ops, d_off, nullptr, p, d_out, d.d_gws,
                                          std::min<int>(n_cex, wg_cap), gap_cap, d.d_jit2,
                                          d.d_status, job, st));
      }
    }
    if (!early_launched || n_cex > 0) {  // (launched early and done: the status is current)
      HIP_TRY(c, hipEventRecord(d.eg, st));
      HIP_TRY(c, hipMemcpyAsync(d.h_status, d.d_status, sizeof(lcdev::KStatus),
                                hipMemcpyDeviceToHost, st));
      HIP_TRY(c, hipStreamSynchronize(st));
    }
    HIP_TRY(c, hipEventElapsedTime(&ms, d.ef, d.eg));
    d.gap_ms = ms;
    if (!light && !fused) d.n_gap = n_jit;
    n_jit = d.h_status->n_jit2;
    jit_list = d.d_jit2;
    before_jit = d.eg;
  }
  d.n_jit = n_jit;
  // Few keys for the frontier search (at most kJitDirectMaxKeys: one 4-wave
  // workgroup per key, all resident at once) go straight to the cooperative
  // tier, whose LDS tables serve small frontiers and whose hash tables keep
  // large ones; the LDS tier's one-wave-per-key pass would be redone for
  // every key that outgrows it.  Measured (tools/jit_direct_ab.py, version-
  // less batches): 1,000 x 1,000 at concurrency 20 19.4 -> 15.0 ms,
  // 1,000 x 200 2.4 -> 1.8 ms, 64 x 1,000 10.1 -> 6.5 ms; but 4,000 x 100
  // 1.0 -> 3.0 ms, where the LDS tier's four keys per workgroup win.
  // LC_JIT_DIRECT=0 (A/B) keeps the LDS tier first.
  const char *direct_env = getenv("LC_JIT_DIRECT");
  // (not with LC_FLAG_NO_FAST_PATH, whose JIT list is implicit: every key)
  const bool direct = !(direct_env && direct_env[0] == '0') && n_jit > 0 && jit_list &&
                      n_jit <= kJitDirectMaxKeys && !(flags & LC_FLAG_NO_HBM_RETRY);
  if (direct) {
    HIP_TRY(c, hipMemcpyAsync(d.d_ovf, jit_list, sizeof(int32_t) * (size_t)n_jit,
                              hipMemcpyDeviceToDevice, st));
    HIP_TRY(c, hipEventElapsedTime(&ms, d.e0, before_jit));
    d.kernel_ms = ms;
  } else if (n_jit == 0) {
    HIP_TRY(c, hipEventElapsedTime(&ms, d.e0, before_jit));
    d.kernel_ms = ms;
  } else {
    // tier 2: JIT search with the frontier in SGPRs / LDS
    HIP_TRY(c, lcdev::launch_lds_tier(d_ops, d_off, jit_list, n_jit, p, d_out,
                                      d.d_ovf, d.d_status, st));
    HIP_TRY(c, hipEventRecord(d.e1, st));
    HIP_TRY(c, hipMemcpyAsync(d.h_status, d.d_status, sizeof(lcdev::KStatus),
                              hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipStreamSynchronize(st));
    HIP_TRY(c, hipEventElapsedTime(&ms, before_jit, d.e1));
    d.jit_ms = ms;
    HIP_TRY(c, hipEventElapsedTime(&ms, d.e0, d.e1));
    d.kernel_ms = ms;
  }
  d.malformed = d.h_status->malformed;
  const int32_t n_ovf = direct ? (int32_t)n_jit : d.h_status->n_overflow;
  d.n_hbm = n_ovf;
  if (n_ovf > 0 && !(flags & LC_FLAG_NO_HBM_RETRY)) {
    int32_t n_list = n_ovf;
    int32_t *list = d.d_ovf, *next = d.d_ovf2;
    HIP_TRY(c, hipEventRecord(d.e1, st));
    // LC_HBM_COOP (test/A-B knob): 0 one wavefront per key throughout,
    // 4 / 16 a workgroup of that many wavefronts per key throughout; default:
    // 8 for at most 512 keys (two workgroups per CU), else 4.  (Round 1 used
    // one wavefront per key beyond 4,096 keys; with the LDS tables the
    // 4-wave workgroups win there too: version-less 10,000 x 1,000 at
    // concurrency 20, HBM tier 128 -> 98 ms, tools/hbm_width_large.py.)
    const char *coop_env = getenv("LC_HBM_COOP");
    const int coop_mode = coop_env ? atoi(coop_env) : 1;
    for (int tier = 0; tier < kHbmTiers && n_list > 0; tier++) {
      int wpk = coop_mode == 1 ? (n_list <= kHbmCoop8MaxKeys ? 8 : 4) : coop_mode;
      const bool coop = wpk == 4 || wpk == 8 || wpk == 16;
      // workgroups: at most the resident ones (keys are claimed dynamically)
      const int resident = wpk == 16 ? kHbmCoop16Resident : wpk == 8 ? 512
                           : wpk == 4 ? kHbmCoop4Resident : kHbmWaves[tier];
      const int waves = std::min<int>(std::min(kHbmWaves[tier], resident), n_list);
      const size_t ws = lcdev::hbm_tier_ws_bytes(waves, kHbmCap[tier]);
      rc = ensure(c, reinterpret_cast<char **>(&d.d_ws), &d.ws_cap, ws);
      if (rc) return rc;
      HIP_TRY(c, hipMemsetAsync(&d.d_status->n_overflow2, 0, sizeof(int32_t), st));
      HIP_TRY(c, hipMemsetAsync(&d.d_status->hbm_next, 0, sizeof(int32_t), st));
      const int last = tier == kHbmTiers - 1;
      if (coop)
        HIP_TRY(c, lcdev::launch_hbm_coop(d_ops, d_off, list, n_list, p, d_out, d.d_ws, waves,
                                          kHbmCap[tier], next, &d.d_status->n_overflow2,
                                          &d.d_status->malformed, &d.d_status->hbm_next, last,
                                          wpk, st));
      else
        HIP_TRY(c, lcdev::launch_hbm_tier(d_ops, d_off, list, n_list, p,
                                          d_out, d.d_ws, waves, kHbmCap[tier], next,
                                          &d.d_status->n_overflow2, &d.d_status->malformed,
                                          &d.d_status->hbm_next, last, st));
      HIP_TRY(c, hipMemcpyAsync(d.h_status, d.d_status, sizeof(lcdev::KStatus),
                                hipMemcpyDeviceToHost, st));
      HIP_TRY(c, hipStreamSynchronize(st));
      n_list = tier < kHbmTiers - 1 ? d.h_status->n_overflow2 : 0;
      std::swap(list, next);
    }
    HIP_TRY(c, hipEventRecord(d.e2, st));
    HIP_TRY(c, hipStreamSynchronize(st));
    HIP_TRY(c, hipEventElapsedTime(&ms, d.e1, d.e2));
    d.hbm_ms = ms;
    d.malformed = d.h_status->malformed;  // (keys sent straight here report it)
  }
  HIP_TRY(c, hipMemsetAsync(d.d_status, 0, sizeof(lcdev::KStatus), st));
  HIP_TRY(c, hipStreamSynchronize(st));
  d.status_dirty = false;
  if (timing) {
    d.tot.timed_calls++;
    d.tot.fast_kernel_ms += d.fast_ms;
  }
  d.tot.kernel_ms += d.kernel_ms + d.hbm_ms;
  return 0;
}


// LC_FLAG_WHOLE_GPU: keys the tiers left :unknown at the configuration
// budget (one workgroup's HBM sets were not enough) are searched again by the
// frontier exchange (include/lincheck_fx.h), whose budget bounds each
// return's configuration sets, as the oracle's does; its result replaces the
// tiers' (verdict, fail op, explored, frontier).  fetch(k, records) and
// store(k, result) move a key between the caller's memory (host or device)
// and the engine.
//
// * Fewer such keys than the context has GPUs: each key's search spans every
//   GPU of the context — one rank per GPU over RCCL (lc_fx_open_devices),
//   the frontier partitioned by hash owner while it is large.
//   Device contexts that share one GPU (LC_VIRTUAL_DEVICES) run their ranks
//   in process instead (RCCL refuses two ranks on one device).
// * Otherwise keys are independent (register.clj:108): up to kFxEngines
//   single-GPU engines per GPU search different keys at once (one key's
//   levels are latency-bound, so concurrent searches fill a GPU the way one
//   cannot), as many as the GPU's free memory holds.
//
// Keys left :unknown because more than LC_MAX_WINDOW ops were open at once
// (crashed writes/CAS pile up in the tiers' windows) are searched again too,
// the same way: there the crashed ops of a key are counted per class instead
// of holding a window slot each (fx.hip, "Counted classes"; owner_of hashes a
// class by its absolute count, so the multi-GPU engine partitions them too).
//
// A failure of the re-search (an allocation, say) is this key's alone: it
// keeps the tiers' :unknown, the error text goes to lc_last_error, and the
// call still succeeds — as jepsen.independent loses only the key whose check
// throws.
int whole_gpu(lc_ctx *c, const std::vector<int64_t> &todo, const lc_opts *opts,
              const std::function<int(int64_t, std::vector<lc_op> &)> &fetch,
              const std::function<int(int64_t, const lc_key_result &)> &store) {
  if (todo.empty()) return 0;
  std::vector<int> ids;  // the context's distinct GPUs
  for (const Dev &d : c->devs)
    if (std::find(ids.begin(), ids.end(), d.id) == ids.end()) ids.push_back(d.id);
  const int nranks = (int)c->devs.size();
  std::atomic<int> failed{0};
  auto note = [&](int64_t k, const std::string &what) {
    failed++;
    set_err(c, "LC_FLAG_WHOLE_GPU: key " + std::to_string(k) + " kept :unknown: " + what);
  };
  if (nranks > 1 && todo.size() < (size_t)nranks) {
    if (!c->fx_all && !c->fx_all_failed) {
      lc_fx_params fp{};
      fp.part_above = -1;
      fp.repl_below = -1;
      int e;
      if ((int)ids.size() == nranks) {
        e = lc_fx_open_devices(&fp, ids.data(), (int32_t)ids.size(), &c->fx_all);
      } else {
        fp.device = ids[0];
        fp.virtual_ranks = nranks;
        e = lc_fx_open(&fp, nullptr, &c->fx_all);
      }
      if (e) {
        c->fx_all = nullptr;
        c->fx_all_failed = true;  // (e.g. no librccl) the single-GPU engines below take over
        set_err(c, "LC_FLAG_WHOLE_GPU: multi-GPU frontier exchange unavailable (" +
                       std::to_string(e) + "); searching keys one GPU each");
      }
    }
    if (c->fx_all) {
      std::vector<lc_op> recs;
      for (int64_t k : todo) {
        if (int x = fetch(k, recs)) return x;
        lc_key_result r;
        if (int x = lc_fx_check(c->fx_all, recs.data(), (int64_t)recs.size(), opts, &r)) {
          note(k, std::string("lc_fx_check: ") + lc_fx_last_error(c->fx_all) + " (" +
                      std::to_string(x) + ")");
          continue;
        }
        if (int x = store(k, r)) return x;
      }
      return 0;
    }
  }
  // key-parallel: engines per GPU, bounded by its free memory (lists and
  // tables take up to ~352 B per configuration of the budget, two one-word table sets included)
  const int64_t budget = opts && opts->max_configs_per_key > 0 ? opts->max_configs_per_key
                                                                : kDefaultBudget;
  const double per_engine = 352.0 * (double)(budget + 1) + (64 << 20);
  for (int id : ids) {
    int have = 0;
    for (const auto &e : c->fxs) have += e.second == id;
    size_t fr = 0, tot = 0;
    (void)hipSetDevice(id);
    int want = (int)kFxEngines;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess)
      want = (int)std::max<double>(1.0, std::min<double>(want, 0.8 * (double)fr / per_engine + have));
    const int per_dev = (int)std::min<size_t>((size_t)want, (todo.size() + ids.size() - 1) / ids.size());
    for (; have < per_dev; have++) {
      lc_fx_params fp{};
      fp.device = id;
      fp.virtual_ranks = 1;
      fp.part_above = -1;
      fp.repl_below = -1;
      lc_fx *f = nullptr;
      if (int e = lc_fx_open(&fp, nullptr, &f)) {
        set_err(c, "LC_FLAG_WHOLE_GPU: lc_fx_open failed (" + std::to_string(e) + ")");
        break;
      }
      c->fxs.emplace_back(f, id);
    }
  }
  const int ne = (int)c->fxs.size();
  if (ne == 0) {
    for (int64_t k : todo) note(k, "no frontier-exchange engine could be opened");
    return 0;
  }
  std::atomic<size_t> next{0};
  std::vector<int> erc(ne, 0);
  auto run = [&](int e) {
    (void)hipSetDevice(c->fxs[e].second);
    std::vector<lc_op> recs;
    for (;;) {
      const size_t i = next.fetch_add(1);
      if (i >= todo.size()) break;
      const int64_t k = todo[i];
      lc_key_result r;
      if ((erc[e] = fetch(k, recs))) break;
      if (int x = lc_fx_check(c->fxs[e].first, recs.data(), (int64_t)recs.size(), opts, &r)) {
        note(k, std::string("lc_fx_check: ") + lc_fx_last_error(c->fxs[e].first) + " (" +
                    std::to_string(x) + ")");
        continue;
      }
      if ((erc[e] = store(k, r))) break;
    }
  };
  std::vector<std::thread> th;
  for (int e = 0; e < std::min<int>(ne, (int)todo.size()); e++) th.emplace_back(run, e);
  for (auto &t : th) t.join();
  for (int e = 0; e < ne; e++)
    if (erc[e]) return erc[e];
  return 0;
}

// Per-key device cost in record-scan units.  The tier a key
// lands in follows from its records alone (check_kernel.hip, fast_key):
//   * version-order tier (every :ok mutation versioned, nothing crashed):
//     one pass over the records, cost n;
//   * gap tier (crashed writes/CAS, versions pinned): two skeleton passes,
//     the matching and, for an invalid key, the bisection; measured ~6x the
//     fast tier per record on C2 with 5 % crashed ops (crash_leg), plus the
//     matching's share, which grows with the crashed ops;
//   * frontier search (an :ok mutation or a read [nil x] without a version):
//     the frontier grows with the open window w; measured (model_leg,
//     tools/frontier_dist.py) ~1,600x the fast tier per record at
//     concurrency 10 and ~4,700x at 20, i.e. ~12 w^2, and crashed ops
//     multiply the configurations (capped: the search's budget bounds it).
// Plus a fixed 64 per key (launch share, result write).
// (Records of either width: lc_op, or lc_op32 with LC_INF32 for LC_INF.)
inline bool rec_crashed(const lc_op32 &o) { return o.ret == LC_INF32; }
inline int64_t rec_call(const lc_op &o) { return o.call; }
inline int64_t rec_call(const lc_op32 &o) { return (int64_t)o.call; }
inline int64_t rec_ret(const lc_op &o) { return o.ret; }
inline int64_t rec_ret(const lc_op32 &o) { return o.ret == LC_INF32 ? LC_INF : (int64_t)o.ret; }
// a crashed write/CAS, or an :ok op without a version that the version order
// cannot pin (a mutation, or a read of a value)
template <class Op>
inline void rec_kind(const Op &o, bool *crashed_mut, bool *unpinned) {
  const bool mut = o.f == LC_F_WRITE || o.f == LC_F_CAS;
  *crashed_mut = mut && rec_crashed(o);
  *unpinned = !rec_crashed(o) && o.version == (int32_t)LC_NIL &&
              (mut || (o.f == LC_F_READ && o.value != (int32_t)LC_NIL));
}
inline void rec_kind(const lc_op &o, bool *crashed_mut, bool *unpinned) {
  const bool mut = o.f == LC_F_WRITE || o.f == LC_F_CAS;
  *crashed_mut = mut && o.ret == LC_INF;
  *unpinned = o.ret != LC_INF && o.version == LC_NIL &&
              (mut || (o.f == LC_F_READ && o.value != LC_NIL));
}

// An lc_op16 record as the lc_op32 it stands for (include/lincheck.h)
inline lc_op32 as32(const lc_op16 &q) {
  const uint32_t v = q.fve >> 15 & 0x7FFFu, x = q.fve & 0x7FFFu;
  return lc_op32{(int32_t)(q.fve >> 30), v == 0x7FFFu ? -2 : (int32_t)v - 1,
                 x == 0x7FFFu ? -2 : (int32_t)x - 1, q.version, q.call, q.ret};
}
inline int64_t rec_call(const lc_op16 &o) { return (int64_t)o.call; }
inline int64_t rec_ret(const lc_op16 &o) { return o.ret == LC_INF32 ? LC_INF : (int64_t)o.ret; }
inline void rec_kind(const lc_op16 &o, bool *crashed_mut, bool *unpinned) {
  rec_kind(as32(o), crashed_mut, unpinned);
}

template <class Op>
double key_cost(const Op *o, int64_t n) {
  int64_t crashed = 0, unpinned = 0;
  for (int64_t i = 0; i < n; i++) {
    bool cm, un;
    rec_kind(o[i], &cm, &un);
    crashed += cm;
    unpinned += un;
  }
  const double kOverhead = 64;
  if (!unpinned && !crashed) return (double)n + kOverhead;
  if (!unpinned) return (6.0 + 0.01 * (double)crashed) * (double)n + kOverhead;
  // open window: the most ops called and not yet returned at once
  std::vector<int64_t> rets;
  rets.reserve((size_t)n);
  for (int64_t i = 0; i < n; i++) rets.push_back(rec_ret(o[i]));
  std::sort(rets.begin(), rets.end());
  int64_t w = 0;
  size_t j = 0;
  for (int64_t i = 0; i < n; i++) {  // records are sorted by call
    while (j < rets.size() && rets[j] < rec_call(o[i])) j++;
    w = std::max<int64_t>(w, i + 1 - (int64_t)j);
  }
  const double blow = std::pow(2.0, (double)std::min<int64_t>(crashed, 12));
  return (double)n * (1.0 + 12.0 * (double)w * (double)w) * blow + kOverhead;
}


// lc_check's own split over its devices: the same contiguous equal-cost cut
// as lc_plan_partition, but a key is priced by all its records only when a
// sample of them (every kSampleStride-th) shows it is not a clean
// version-pinned key (a crashed write/CAS, an :ok op without a version);
// otherwise it costs its record count, which is what lc_key_cost gives a
// clean key.  And the sample itself is taken only when a first probe — the
// same sample of every kKeyStride-th key — finds an irregular key: a batch
// whose probe is clean is split by record count.  Pricing every record read
// the whole batch on the host (480 MB for C2: several ms even on 16 threads)
// before any copy could start; sampling every key still touched every page
// (0.6-0.9 ms of a 5-ms call on the GPU box, tools/plan_probe.cpp); the
// probe reads ~1/16 of them.  Only the split's balance, never a verdict,
// depends on these estimates.
constexpr int64_t kSampleStride = 64;
constexpr int64_t kKeyStride = 16;
template <class Op>
bool irregular_sample(const Op *o, int64_t n) {
  for (int64_t i = 0; i < n; i += kSampleStride) {
    bool cm, un;
    rec_kind(o[i], &cm, &un);
    if (cm || un) return true;
  }
  return false;
}

template <class Op>
void plan_devices(const Op *ops, const int64_t *key_off, int64_t n_keys, int nd,
                  int64_t *bounds) {
  std::vector<double> pre((size_t)n_keys + 1, 0.0);
  bool any = false;
  for (int64_t k = 0; k < n_keys && !any; k += kKeyStride)
    any = irregular_sample(ops + key_off[k], key_off[k + 1] - key_off[k]);
  auto price = [&](int64_t k0, int64_t k1) {
    for (int64_t k = k0; k < k1; k++) {
      const Op *o = ops + key_off[k];
      const int64_t n = key_off[k + 1] - key_off[k];
      pre[(size_t)k + 1] = any && irregular_sample(o, n) ? key_cost(o, n) : (double)n + 64.0;
    }
  };
  const int nth = any ? (int)std::min<int64_t>(16, std::max<int64_t>(1, n_keys >> 10)) : 1;
  if (nth <= 1) {
    price(0, n_keys);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < nth; t++) th.emplace_back(price, n_keys * t / nth, n_keys * (t + 1) / nth);
    for (auto &x : th) x.join();
  }
  for (int64_t k = 0; k < n_keys; k++) pre[(size_t)k + 1] += pre[(size_t)k];
  const double total = pre[(size_t)n_keys];
  bounds[0] = 0;
  int64_t k = 0;
  for (int p = 1; p < nd; p++) {
    const double goal = total * p / nd;
    while (k < n_keys && pre[(size_t)k] < goal) k++;
    bounds[p] = k;
  }
  bounds[nd] = n_keys;
}

// An lc_op32 record as the lc_op it stands for (include/lincheck.h, ABI 4).
inline lc_op widen_op(const lc_op &o, int64_t) { return o; }
inline lc_op widen_op(const lc_op32 &o, int64_t base) {
  return lc_op{o.f, o.value, o.expected, o.version, base + (int64_t)o.call,
               o.ret == LC_INF32 ? LC_INF : base + (int64_t)o.ret};
}
inline lc_op widen_op(const lc_op16 &o, int64_t base) { return widen_op(as32(o), base); }

// lc_check_ex (48-byte lc_op) and lc_check32 (24-byte lc_op32, ABI 4) from
// host memory: the keys split over the context's devices (plan_devices), one
// host thread per device.  Per device, the key offsets (and lc_check32's key
// bases) are copied first, then the records in chunks of about kChunkBytes
// on the device's copy stream; the compute stream decides each chunk's keys
// with the version-order (or fused) pass as soon as the chunk has landed
// (run_device, Chunks), widening 24-byte records on the way, so the PCIe
// copy of chunk i + 1 overlaps the kernels of chunk i.  The later tiers run
// over the whole range once every chunk is in.  Results and lc_aux outputs
// are copied back into the caller's arrays.  Per call, lc_call_profile keeps
// where the host wall time went.
template <class Op>
int check_host(lc_ctx *c, const Op *ops, const int64_t *key_off, const int64_t *key_base,
               int64_t n_keys, const lc_opts *opts, lc_key_result *out, const lc_aux *aux) {
  constexpr bool k32 = sizeof(Op) == sizeof(lc_op32);
  constexpr bool k16 = sizeof(Op) == sizeof(lc_op16);
  constexpr bool narrow = k32 || k16;  // records widened on the device, key bases
  const auto t0 = std::chrono::steady_clock::now();
  auto since = [&t0]() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  };
  c->stats = lc_stats{};
  c->prof = lc_call_profile{};
  if (n_keys < 0 || (n_keys > 0 && (!ops || !key_off || !out))) {
    set_err(c, "lc_check: null buffer or negative n_keys");
    return -EINVAL;
  }
  if (n_keys == 0) return 0;
  if (key_off[0] < 0) {
    set_err(c, "lc_check: key_off[0] < 0");
    return -EINVAL;
  }
  for (int64_t k = 0; k < n_keys; k++)
    if (key_off[k + 1] < key_off[k]) {
      set_err(c, "lc_check: key_off not monotone at key " + std::to_string(k));
      return -EINVAL;
    }
  lcdev::KParams p;
  int rc = opts_to_params(c, opts, &p);
  if (rc) return rc;
  const int64_t flags = opts ? opts->flags : 0;
  const bool want_wit = aux && aux->witness && aux->witness_kind;
  const bool want_cert = aux && aux->certificate;
  const int nd = (int)c->devs.size();
  c->prof.checked_ms = since();
  std::vector<int64_t> bounds(nd + 1);
  if (nd > 1) plan_devices(ops, key_off, n_keys, nd, bounds.data());
  else bounds[0] = 0, bounds[1] = n_keys;
  c->prof.planned_ms = since();
  // the longest key (the widening's grid); C4's 5,000-op key takes more
  // workgroups than a C2 key
  int64_t max_len = 0;
  if (narrow)
    for (int64_t k = 0; k < n_keys; k++) max_len = std::max(max_len, key_off[k + 1] - key_off[k]);

  std::vector<int> rcs(nd, 0);
  std::vector<int> nchunks(nd, 0);
  auto work = [&](int di) {
    Dev &d = c->devs[di];
    d.t_start = since();
    d.t_end = d.t_start;
    const int64_t a = bounds[di], b = bounds[di + 1];
    const int64_t nk = b - a;
    const auto tw = std::chrono::steady_clock::now();
    d.last = lc_device_stats{};
    d.last.device = d.id;
    d.last.key_begin = a;
    d.last.key_end = b;
    d.kernel_ms = 0;
    if (nk <= 0) return;
    if (hipSetDevice(d.id) != hipSuccess) {
      rcs[di] = -EIO;
      return;
    }
    const int64_t r0 = key_off[a], r1 = key_off[b];
    const int64_t nrec = r1 - r0;
    const size_t ops_bytes = sizeof(lc_op) * (size_t)nrec;  // on the device: 48-byte records
    const size_t in_bytes = sizeof(Op) * (size_t)nrec;      // what crosses PCIe
    int r = ensure(c, reinterpret_cast<char **>(&d.d_ops), &d.ops_cap, ops_bytes);
    // (the narrow records' staging: d_ops32, whichever width)
    if (!r && narrow) r = ensure(c, reinterpret_cast<char **>(&d.d_ops32), &d.ops32_cap, in_bytes);
    if (!r && narrow && key_base) r = ensure(c, &d.d_base, &d.base_cap, sizeof(int64_t) * (size_t)nk);
    if (!r) r = ensure(c, &d.d_off, &d.off_cap, sizeof(int64_t) * (size_t)(nk + 1));
    if (!r) r = ensure(c, &d.d_out, &d.out_cap, sizeof(lc_key_result) * (size_t)nk);
    if (!r && want_wit) r = ensure(c, &d.d_wit, &d.wit_cap, sizeof(int32_t) * (size_t)nrec);
    if (!r && want_wit) r = ensure(c, &d.d_kind, &d.kind_cap, sizeof(int32_t) * (size_t)nk);
    if (!r && want_cert) r = ensure(c, &d.d_cert, &d.cert_cap, 4 * sizeof(int32_t) * (size_t)nk);
    if (!r && want_cert) r = ensure(c, &d.d_cset, &d.cset_cap, sizeof(int32_t) * (size_t)nrec);
    if (r) {
      rcs[di] = r;
      return;
    }
    // small pageable calls: inputs (offsets, bases, records) and outputs
    // (results, lc_aux arrays) through the pinned staging buffer
    auto up = [](size_t x) { return (x + 255) & ~size_t(255); };
    const bool pinned = is_pinned(c, ops + r0, in_bytes);
    const size_t off_bytes = sizeof(int64_t) * (size_t)(nk + 1);
    const size_t base_bytes = narrow && key_base ? sizeof(int64_t) * (size_t)nk : 0;
    const size_t out_bytes =
        up(sizeof(lc_key_result) * (size_t)nk) +
        (want_wit ? up(sizeof(int32_t) * (size_t)nrec) + up(sizeof(int32_t) * (size_t)nk) : 0) +
        (want_cert ? up(4 * sizeof(int32_t) * (size_t)nk) + up(sizeof(int32_t) * (size_t)nrec) : 0);
    const size_t stage_need = up(off_bytes) + up(base_bytes) + up(in_bytes) + out_bytes;
    // (not with lc_aux outputs: the drop-in's C5 call with witnesses and
    // certificates measured 0.05-0.1 ms slower staged)
    const bool stage = !pinned && !want_wit && !want_cert && stage_need <= kStageMax && !stage_off();
    if (stage && !stage_buf(c, d)) {
      rcs[di] = -ENOMEM;
      return;
    }
    char *st_off = stage ? d.h_stage : nullptr;
    char *st_base = stage ? st_off + up(off_bytes) : nullptr;
    char *st_ops = stage ? st_base + up(base_bytes) : nullptr;
    char *st_out = stage ? st_ops + up(in_bytes) : nullptr;
    // chunks: contiguous key ranges of about kChunkBytes of input records,
    // the last ones halving down to kChunkTail (cut at key boundaries)
    Chunks ch;
    std::vector<size_t> sizes;  // from the end of the range
    for (size_t left = in_bytes, want = kChunkTail; left > 0 && (int)sizes.size() < kMaxChunks - 1;) {
      const size_t take = std::min(left, want);
      sizes.push_back(take);
      left -= take;
      want = std::min(kChunkBytes, 2 * want);
    }
    ch.k.push_back(0);
    {
      size_t sum = 0;
      for (size_t z : sizes) sum += z;
      int64_t rec_goal = (int64_t)((in_bytes - sum) / sizeof(Op));  // records before the next cut
      for (size_t i = sizes.size(); i-- > 1;) {
        rec_goal += (int64_t)(sizes[i] / sizeof(Op));
        int64_t k = std::lower_bound(key_off + a, key_off + b, r0 + rec_goal) - (key_off + a);
        if (k > ch.k.back() && k < nk) ch.k.push_back(k);
      }
    }
    ch.k.push_back(nk);
    ch.n = (int)ch.k.size() - 1;
    for (int64_t k : ch.k) ch.r.push_back(key_off[a + k] - r0);
    while ((int)d.cev.size() < ch.n) {
      hipEvent_t e = nullptr;
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
        set_err(c, "hipEventCreateWithFlags failed");
        rcs[di] = -EIO;
        return;
      }
      d.cev.push_back(e);
    }
    ch.ready = d.cev.data();
    ch.max_len = max_len;
    if (k32) ch.d_ops32 = static_cast<const lc_op32 *>(d.d_ops32);
    if (k16) ch.d_ops16 = static_cast<const lc_op16 *>(d.d_ops32);
    if (narrow) ch.d_base = key_base ? d.d_base : nullptr;
    nchunks[di] = ch.n;
    char *dst = static_cast<char *>(narrow ? d.d_ops32 : d.d_ops);
    const char *src = reinterpret_cast<const char *>(ops + r0);
    // the key offsets (and bases) lead; the compute stream waits for the
    // first chunk's event, which follows them on the copy stream
    hipError_t e = hipEventRecord(d.eh0, d.cst);
    const void *src_off = key_off + a, *src_base = narrow && key_base ? key_base + a : nullptr;
    if (stage) {
      std::memcpy(st_off, src_off, off_bytes);
      if (base_bytes) std::memcpy(st_base, src_base, base_bytes);
      src_off = st_off;
      src_base = st_base;
    }
    if (e == hipSuccess)
      e = hipMemcpyAsync(d.d_off, src_off, off_bytes, hipMemcpyHostToDevice, d.cst);
    if (e == hipSuccess && base_bytes)
      e = hipMemcpyAsync(d.d_base, src_base, base_bytes, hipMemcpyHostToDevice, d.cst);
    if (e != hipSuccess) {
      set_err(c, std::string("hipMemcpyAsync H2D: ") + hipGetErrorString(e));
      rcs[di] = -EIO;
      return;
    }
    // the second copy stream starts behind the offsets too
    if (e == hipSuccess) e = hipEventRecord(d.cev[0], d.cst);
    if (e == hipSuccess) e = hipStreamWaitEvent(d.cst2, d.cev[0], 0);
    if (e != hipSuccess) {
      set_err(c, std::string("hipStreamWaitEvent: ") + hipGetErrorString(e));
      rcs[di] = -EIO;
      return;
    }
    // Two copy streams, chunks alternating, the odd ones issued by a helper
    // thread: a copy call returns only once the runtime has staged (pageable)
    // or queued it, so one issuing thread left the link idle between copies —
    // two device contexts copying at once moved 57 GB/s against 52-53 for one
    // thread (tools/host32_probe.py)
    auto copy = [&](int i) -> hipError_t {
      const size_t o = sizeof(Op) * (size_t)ch.r[i];
      const size_t bytes = sizeof(Op) * (size_t)(ch.r[i + 1] - ch.r[i]);
      hipStream_t cs = i % 2 ? d.cst2 : d.cst;
      const char *from = src + o;
      if (stage && bytes) {
        std::memcpy(st_ops + o, from, bytes);
        from = st_ops + o;
      }
      hipError_t x = bytes ? hipMemcpyAsync(dst + o, from, bytes, hipMemcpyHostToDevice, cs)
                           : hipSuccess;
      if (x == hipSuccess) x = hipEventRecord(d.cev[(size_t)i], cs);
      return x;
    };
    std::vector<std::atomic<int>> issued((size_t)ch.n);  // odd chunks: 1 issued, -1 failed
    for (auto &f : issued) f.store(0);
    std::atomic<bool> stop{false};
    std::thread helper;
    if (ch.n >= 4)
      helper = std::thread([&] {
        (void)hipSetDevice(d.id);
        for (int i = 1; i < ch.n && !stop.load(std::memory_order_relaxed); i += 2)
          issued[(size_t)i].store(copy(i) == hipSuccess ? 1 : -1, std::memory_order_release);
      });
    ch.issue = [&](int i) -> int {
      hipError_t x = hipSuccess;
      if (i % 2 == 0 || !helper.joinable()) {
        x = copy(i);
      } else {
        int f;
        while ((f = issued[(size_t)i].load(std::memory_order_acquire)) == 0) std::this_thread::yield();
        if (f < 0) x = hipErrorUnknown;
      }
      if (x == hipSuccess && i == ch.n - 1) {
        // both copy streams done
        if (ch.n > 1) x = hipStreamWaitEvent(d.cst, d.cev[(size_t)i - 1], 0);
        if (x == hipSuccess) x = hipStreamWaitEvent(d.cst, d.cev[(size_t)i], 0);
        if (x == hipSuccess) x = hipEventRecord(d.eh1, d.cst);
      }
      if (x != hipSuccess) {
        set_err(c, std::string("hipMemcpyAsync H2D: ") + hipGetErrorString(x));
        return -EIO;
      }
      return 0;
    };
    auto join_helper = [&] {
      stop.store(true);
      if (helper.joinable()) helper.join();
    };
    d.last.h2d_bytes = (int64_t)(in_bytes + sizeof(int64_t) * (size_t)(nk + 1) +
                                 (narrow && key_base ? sizeof(int64_t) * (size_t)nk : 0));
    d.last.pinned = pinned;
    WitOut wo;
    wo.n_records = nrec;
    if (want_wit) {
      wo.wit = d.d_wit;
      wo.kind = d.d_kind;
    }
    if (want_cert) {
      wo.cert = d.d_cert;
      wo.cset = d.d_cset;
    }
    wo.h_off = key_off + a;
    wo.chunks = &ch;
    if (k32 && !want_wit && !want_cert && !(flags & LC_FLAG_NO_FAST_PATH) && !native32_off()) {
      // decided from the 24-byte records; widened only if a key is handed over
      wo.ops32 = static_cast<const lc_op32 *>(d.d_ops32);
      wo.base32 = key_base ? d.d_base : nullptr;
      wo.widen = [&](const lc_op **out) -> int {
        HIP_TRY(c, lcdev::launch_widen32(static_cast<const lc_op32 *>(d.d_ops32), d.d_off,
                                         key_base ? d.d_base : nullptr, nk, max_len,
                                         static_cast<lc_op *>(d.d_ops), d.stream));
        *out = static_cast<const lc_op *>(d.d_ops);
        return 0;
      };
    }
    r = run_device(c, d, static_cast<const lc_op *>(d.d_ops), d.d_off, nk, p, d.d_out, d.stream,
                   flags, wo);
    join_helper();
    if (!r) r = run_certificates(c, d, static_cast<const lc_op *>(d.d_ops), d.d_off, nk, p,
                                 d.d_out, d.stream, wo);
    if (r) {
      // the copy stream may still read the caller's buffer
      (void)hipStreamSynchronize(d.cst);
      (void)hipStreamSynchronize(d.cst2);
      rcs[di] = r;
      return;
    }
    // outputs: straight into the caller's buffers, or (staged) into the
    // pinned buffer and copied out once the stream is done
    struct OutCopy {
      void *to;
      const void *from;
      size_t bytes;
    };
    OutCopy oc[5];
    int n_oc = 0;
    oc[n_oc++] = {out + a, d.d_out, sizeof(lc_key_result) * (size_t)nk};
    if (want_wit && nrec) oc[n_oc++] = {aux->witness + r0, d.d_wit, sizeof(int32_t) * (size_t)nrec};
    if (want_wit) oc[n_oc++] = {aux->witness_kind + a, d.d_kind, sizeof(int32_t) * (size_t)nk};
    if (want_cert) oc[n_oc++] = {aux->certificate + 4 * a, d.d_cert, 4 * sizeof(int32_t) * (size_t)nk};
    if (want_cert && aux->certificate_set && nrec)
      oc[n_oc++] = {aux->certificate_set + r0, d.d_cset, sizeof(int32_t) * (size_t)nrec};
    size_t so = 0;
    for (int i = 0; i < n_oc && e == hipSuccess; i++) {
      void *to = stage ? st_out + so : oc[i].to;
      so += up(oc[i].bytes);
      e = hipMemcpyAsync(to, oc[i].from, oc[i].bytes, hipMemcpyDeviceToHost, d.stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(d.stream);
    if (e == hipSuccess && stage) {
      so = 0;
      for (int i = 0; i < n_oc; i++) {
        std::memcpy(oc[i].to, st_out + so, oc[i].bytes);
        so += up(oc[i].bytes);
      }
    }
    if (e != hipSuccess) {
      set_err(c, std::string("hipMemcpyAsync D2H: ") + hipGetErrorString(e));
      rcs[di] = -EIO;
      return;
    }
    // eh1 follows the last copy on the copy stream, which the compute stream
    // waited for by the chunk's own event: it may complete a moment after the
    // stream synchronised above (several device threads on one GPU), and an
    // elapsed time read before then fails (h2d_ms would read 0)
    float hms = 0;
    if (hipEventSynchronize(d.eh1) == hipSuccess &&
        hipEventElapsedTime(&hms, d.eh0, d.eh1) == hipSuccess)
      d.last.h2d_ms = hms;
    d.last.kernel_ms = d.kernel_ms;
    d.last.total_ms = std::chrono::duration<double, std::milli>(
                          std::chrono::steady_clock::now() - tw).count();
    d.t_end = since();
  };
  if (nd == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (int di = 0; di < nd; di++) th.emplace_back(work, di);
    for (auto &t : th) t.join();
  }
  c->prof.first_start_ms = c->prof.first_end_ms = 1e300;
  for (int di = 0; di < nd; di++) {
    const Dev &d = c->devs[di];
    if (rcs[di] && !rc) rc = rcs[di];
    c->stats.kernel_ms += d.kernel_ms;
    c->stats.fast_kernel_ms += d.fast_ms;
    c->stats.jit_kernel_ms += d.jit_ms;
    c->stats.n_jit_keys += d.n_jit;
    c->stats.gap_kernel_ms += d.gap_ms;
    c->stats.n_gap_keys += d.n_gap;
    c->stats.hbm_kernel_ms += d.hbm_ms;
    c->stats.n_hbm_keys += d.n_hbm;
    c->stats.n_malformed += d.malformed;
    c->prof.first_start_ms = std::min(c->prof.first_start_ms, d.t_start);
    c->prof.last_start_ms = std::max(c->prof.last_start_ms, d.t_start);
    c->prof.first_end_ms = std::min(c->prof.first_end_ms, d.t_end);
    c->prof.last_end_ms = std::max(c->prof.last_end_ms, d.t_end);
    c->prof.n_chunks += nchunks[di];
  }
  c->prof.joined_ms = since();
  if (!rc && (flags & LC_FLAG_WHOLE_GPU)) {
    std::vector<int64_t> todo, todo_w;
    for (int64_t k = 0; k < n_keys; k++)
      if (out[k].verdict == LC_UNKNOWN && out[k].reason == LC_REASON_CONFIG_BUDGET) todo.push_back(k);
      else if (out[k].verdict == LC_UNKNOWN && out[k].reason == LC_REASON_WINDOW_OVERFLOW)
        todo_w.push_back(k);
    auto fetch = [&](int64_t k, std::vector<lc_op> &v) {
      v.resize((size_t)(key_off[k + 1] - key_off[k]));
      const int64_t base = key_base ? key_base[k] : 0;
      for (size_t i = 0; i < v.size(); i++) v[i] = widen_op(ops[key_off[k] + (int64_t)i], base);
      return 0;
    };
    auto store = [&](int64_t k, const lc_key_result &r) {
      out[k] = r;
      // re-decided by the frontier exchange: no certificate (cert.hip covers
      // the tiers' decisions)
      if (want_cert)
        for (int j = 0; j < 4; j++) aux->certificate[4 * k + j] = j == 0 ? LC_CERT_NONE : j < 3 ? -1 : 0;
      return 0;
    };
    rc = whole_gpu(c, todo, opts, fetch, store);
    if (!rc) rc = whole_gpu(c, todo_w, opts, fetch, store);
  }
  c->prof.whole_gpu_ms = since();
  c->stats.n_keys = n_keys;
  c->stats.n_ops = key_off[n_keys] - key_off[0];
  c->stats.n_devices = nd;
  c->stats.total_ms = since();
  c->prof.total_ms = c->stats.total_ms;
  c->prof.n_devices = nd;
  return rc;
}

}  // namespace

extern "C" {

int lc_abi_version(void) { return LC_ABI_VERSION; }

void lc_default_opts(lc_opts *o) {
  if (!o) return;
  o->init_version = 0;
  o->init_value = LC_NIL;
  o->max_configs_per_key = 0;
  o->time_budget_ms = 0;
  o->flags = 0;
}

// The id is also findable in the file without loading it ("LC_BUILD_ID:"
// marker): tests/conftest.py checks it before anything loads a HIP runtime.
__attribute__((used)) static const char kBuildTag[] = "LC_BUILD_ID:" LC_BUILD_ID;
const char *lc_build_id(void) { return kBuildTag + 12; }

int lc_open(uint32_t device_mask, lc_ctx **out) {
  if (!out) return -EINVAL;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return -ENODEV;
  // LC_VIRTUAL_DEVICES=k: k device contexts on the first selected GPU (tests
  // of the multi-device fan-out on a one-GPU box)
  const char *venv = getenv("LC_VIRTUAL_DEVICES");
  const int virt = venv ? std::max(0, std::min(32, atoi(venv))) : 0;
  lc_ctx *c = new lc_ctx();
  for (int i = 0; i < n && i < 32; i++) {
    if (device_mask && !(device_mask & (1u << i))) continue;
    for (int v = 0; v < (virt >= 2 ? virt : 1); v++) {
      Dev d;
      d.id = i;
      if (hipSetDevice(i) != hipSuccess ||
          hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking) != hipSuccess ||
          hipStreamCreateWithFlags(&d.cst, hipStreamNonBlocking) != hipSuccess ||
          hipStreamCreateWithFlags(&d.cst2, hipStreamNonBlocking) != hipSuccess ||
          hipEventCreateWithFlags(&d.e0, kEventFlags) != hipSuccess ||
          hipEventCreateWithFlags(&d.e1, kEventFlags) != hipSuccess ||
          hipEventCreateWithFlags(&d.e2, kEventFlags) != hipSuccess ||
          hipEventCreateWithFlags(&d.ef, kEventFlags) != hipSuccess ||
          hipEventCreateWithFlags(&d.eg, kEventFlags) != hipSuccess ||
          hipEventCreateWithFlags(&d.el, kEventFlags) != hipSuccess ||
          hipEventCreateWithFlags(&d.eh0, kEventFlags) != hipSuccess ||
          hipEventCreateWithFlags(&d.eh1, kEventFlags) != hipSuccess ||
          hipEventCreateWithFlags(&d.es, kEventFlags) != hipSuccess ||
          hipMalloc(reinterpret_cast<void **>(&d.d_status), sizeof(lcdev::KStatus)) != hipSuccess ||
          hipHostMalloc(reinterpret_cast<void **>(&d.h_status), sizeof(lcdev::KStatus), 0) != hipSuccess ||
          hipHostMalloc(reinterpret_cast<void **>(&d.h_handoff), 2 * sizeof(int32_t),
                        hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
          hipHostGetDevicePointer(reinterpret_cast<void **>(&d.h_handoff_dev), d.h_handoff, 0) != hipSuccess ||
          hipHostMalloc(reinterpret_cast<void **>(&d.h_done), 64,
                        hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
          hipHostGetDevicePointer(reinterpret_cast<void **>(&d.h_done_dev), d.h_done, 0) != hipSuccess) {
        c->devs.push_back(d);  // lc_close frees what was created
        lc_close(c);
        return -ENODEV;
      }
      // pinned memory may be reused from a closed context: the completion
      // word must not already hold this context's first sequence number
      __atomic_store_n(d.h_done, 0u, __ATOMIC_RELEASE);
      __atomic_store_n(d.h_handoff, 0, __ATOMIC_RELEASE);
      __atomic_store_n(d.h_handoff + 1, 0, __ATOMIC_RELEASE);
      c->devs.push_back(d);
    }
    if (virt >= 2) break;
  }
  if (c->devs.empty()) {
    delete c;
    return -ENODEV;
  }
  *out = c;
  return 0;
}

void lc_close(lc_ctx *c) {
  if (!c) return;
  for (auto &f : c->fxs) lc_fx_close(f.first);
  if (c->fx_all) lc_fx_close(c->fx_all);
  for (auto &pr : c->pinned) (void)hipHostUnregister(const_cast<char *>(pr.first));
  for (Dev &d : c->devs) {
    (void)hipSetDevice(d.id);
    (void)res_stop(c, d);
    if (d.rst) (void)hipStreamDestroy(d.rst);
    if (d.res_d) (void)hipFree(d.res_d);
    if (d.res_h) (void)hipHostFree(d.res_h);
    if (d.stream) (void)hipStreamSynchronize(d.stream);
    if (d.d_ops) (void)hipFree(d.d_ops);
    if (d.d_off) (void)hipFree(d.d_off);
    if (d.d_out) (void)hipFree(d.d_out);
    if (d.d_ovf) (void)hipFree(d.d_ovf);
    if (d.d_ovf2) (void)hipFree(d.d_ovf2);
    if (d.d_ws) (void)hipFree(d.d_ws);
    if (d.d_status) (void)hipFree(d.d_status);
    if (d.h_status) (void)hipHostFree(d.h_status);
    if (d.h_handoff) (void)hipHostFree(d.h_handoff);
    if (d.h_done) (void)hipHostFree(d.h_done);
    if (d.h_stage) (void)hipHostFree(d.h_stage);
    if (d.e0) (void)hipEventDestroy(d.e0);
    if (d.e1) (void)hipEventDestroy(d.e1);
    if (d.e2) (void)hipEventDestroy(d.e2);
    if (d.ef) (void)hipEventDestroy(d.ef);
    for (hipEvent_t e : {d.eg, d.el, d.eh0, d.eh1, d.es})
      if (e) (void)hipEventDestroy(e);
    if (d.d_jit) (void)hipFree(d.d_jit);
    if (d.d_jit2) (void)hipFree(d.d_jit2);
    if (d.d_flags) (void)hipFree(d.d_flags);
    if (d.d_gws) (void)hipFree(d.d_gws);
    if (d.d_cex) (void)hipFree(d.d_cex);
    if (d.d_wit) (void)hipFree(d.d_wit);
    if (d.d_kind) (void)hipFree(d.d_kind);
    if (d.d_cert) (void)hipFree(d.d_cert);
    if (d.d_cset) (void)hipFree(d.d_cset);
    if (d.d_cws) (void)hipFree(d.d_cws);
    if (d.d_gap2) (void)hipFree(d.d_gap2);
    if (d.d_ops32) (void)hipFree(d.d_ops32);
    if (d.d_base) (void)hipFree(d.d_base);
    for (hipEvent_t e : d.cev) (void)hipEventDestroy(e);
    for (hipStream_t cs : {d.cst, d.cst2})
      if (cs) {
        (void)hipStreamSynchronize(cs);
        (void)hipStreamDestroy(cs);
      }
    if (d.stream) (void)hipStreamDestroy(d.stream);
  }
  delete c;
}

const char *lc_last_error(lc_ctx *c) { return c ? c->err.c_str() : "null context"; }

int lc_last_stats(lc_ctx *c, lc_stats *out) {
  if (!c || !out) return -EINVAL;
  // a call that returned on the completion signal: its pass's event time
  // (single-device calls only take that path)
  if (c->devs[0].timing_pending) {
    settle_timing(c, c->devs[0]);
    c->stats.fast_kernel_ms = c->devs[0].fast_ms;
    c->stats.kernel_ms = c->devs[0].kernel_ms;
  }
  // the keys the crash-light decision took in a fused call, copied lazily
  for (Dev &d : c->devs) {
    const int64_t n = settle_status(d);
    if (n > 0) c->stats.n_gap_keys += n;
  }
  *out = c->stats;
  return 0;
}

int lc_quiesce(lc_ctx *c) {
  if (!c) return -EINVAL;
  for (Dev &d : c->devs) {
    if (!d.res_grid) continue;
    (void)hipSetDevice(d.id);
    if (int e = res_stop(c, d)) return e;
  }
  return 0;
}

int lc_last_totals(lc_ctx *c, lc_totals *out, int32_t reset) {
  if (!c || !out) return -EINVAL;
  lc_totals t{};
  for (Dev &d : c->devs) {
    settle_timing(c, d);
    t.calls += d.tot.calls;
    t.timed_calls += d.tot.timed_calls;
    t.fast_kernel_ms += d.tot.fast_kernel_ms;
    t.kernel_ms += d.tot.kernel_ms;
    if (reset) d.tot = lc_totals{};
  }
  *out = t;
  return 0;
}

int lc_last_device_stats(lc_ctx *c, int32_t i, lc_device_stats *out) {
  if (!c || !out || i < 0 || i >= (int32_t)c->devs.size()) return -EINVAL;
  *out = c->devs[(size_t)i].last;
  return 0;
}

int lc_host_register(lc_ctx *c, const void *ptr, uint64_t bytes) {
  if (!c || !ptr || !bytes) return -EINVAL;
  std::lock_guard<std::mutex> g(c->pin_mu);
  // portable: page-locked for every device of the process (the fan-out's
  // threads copy from it to each GPU of the context)
  const hipError_t e = hipHostRegister(const_cast<void *>(ptr), (size_t)bytes,
                                       hipHostRegisterPortable);
  if (e != hipSuccess) {
    set_err(c, std::string("hipHostRegister: ") + hipGetErrorString(e));
    return -EIO;
  }
  c->pinned.emplace_back(static_cast<const char *>(ptr), bytes);
  return 0;
}

int lc_host_unregister(lc_ctx *c, const void *ptr) {
  if (!c || !ptr) return -EINVAL;
  std::lock_guard<std::mutex> g(c->pin_mu);
  for (size_t i = 0; i < c->pinned.size(); i++)
    if (c->pinned[i].first == ptr) {
      const hipError_t e = hipHostUnregister(const_cast<void *>(ptr));
      c->pinned.erase(c->pinned.begin() + (long)i);
      if (e != hipSuccess) {
        set_err(c, std::string("hipHostUnregister: ") + hipGetErrorString(e));
        return -EIO;
      }
      return 0;
    }
  set_err(c, "lc_host_unregister: pointer not registered with this context");
  return -EINVAL;
}

int lc_key_cost(const lc_op *ops, const int64_t *key_off, int64_t n_keys, double *costs) {
  if (!ops || !key_off || !costs || n_keys < 0) return -EINVAL;
  for (int64_t k = 0; k < n_keys; k++) {
    const int64_t n = key_off[k + 1] - key_off[k];
    if (n < 0) return -EINVAL;
    costs[k] = key_cost(ops + key_off[k], n);
  }
  return 0;
}

// Contiguous split at equal cost: boundary p is the first key whose cost
// prefix reaches p/n_parts of the total (keys stay in order, so each device
// gets one contiguous slice of the caller's arrays).
int lc_plan_partition(const lc_op *ops, const int64_t *key_off, int64_t n_keys,
                      int32_t n_parts, int64_t *bounds) {
  if (!key_off || !bounds || n_parts < 1 || n_keys < 0) return -EINVAL;
  for (int64_t k = 0; k < n_keys; k++)
    if (key_off[k + 1] < key_off[k]) return -EINVAL;
  std::vector<double> pre((size_t)n_keys + 1, 0.0);
  // each key's cost reads its records once: 10M records (480 MB) is tens of
  // ms on one thread, so large batches are priced on up to 16 threads
  // (lc_check's multi-GPU split runs this on every call)
  const int64_t n_rec = ops && n_keys ? key_off[n_keys] - key_off[0] : 0;
  const int nth = (int)std::min<int64_t>(
      16, std::max<int64_t>(1, std::min<int64_t>(n_keys, n_rec >> 18)));
  auto price = [&](int64_t k0, int64_t k1) {
    for (int64_t k = k0; k < k1; k++) {
      const int64_t n = key_off[k + 1] - key_off[k];
      pre[(size_t)k + 1] = ops ? key_cost(ops + key_off[k], n) : (double)n + 64.0;
    }
  };
  if (nth <= 1) {
    price(0, n_keys);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < nth; t++)
      th.emplace_back(price, n_keys * t / nth, n_keys * (t + 1) / nth);
    for (auto &x : th) x.join();
  }
  for (int64_t k = 0; k < n_keys; k++) pre[(size_t)k + 1] += pre[(size_t)k];
  const double total = pre[(size_t)n_keys];
  bounds[0] = 0;
  int64_t k = 0;
  for (int32_t p = 1; p < n_parts; p++) {
    const double goal = total * p / n_parts;
    while (k < n_keys && pre[(size_t)k] < goal) k++;
    bounds[p] = k;
  }
  bounds[n_parts] = n_keys;
  return 0;
}

int lc_check_ex(lc_ctx *c, const lc_op *ops, const int64_t *key_off,
                int64_t n_keys, const lc_opts *opts, lc_key_result *out, const lc_aux *aux) {
  if (!c) return -EINVAL;
  return check_host(c, ops, key_off, nullptr, n_keys, opts, out, aux);
}

int lc_check(lc_ctx *c, const lc_op *ops, const int64_t *key_off,
             int64_t n_keys, const lc_opts *opts, lc_key_result *out) {
  return lc_check_ex(c, ops, key_off, n_keys, opts, out, nullptr);
}

int lc_check32(lc_ctx *c, const lc_op32 *ops, const int64_t *key_off, const int64_t *key_base,
               int64_t n_keys, const lc_opts *opts, lc_key_result *out, const lc_aux *aux) {
  if (!c) return -EINVAL;
  if (reinterpret_cast<uintptr_t>(ops) % 4) {
    set_err(c, "lc_check32: ops must be 4-byte aligned");
    return -EINVAL;
  }
  return check_host(c, ops, key_off, key_base, n_keys, opts, out, aux);
}

int lc_check16(lc_ctx *c, const lc_op16 *ops, const int64_t *key_off, const int64_t *key_base,
               int64_t n_keys, const lc_opts *opts, lc_key_result *out, const lc_aux *aux) {
  if (!c) return -EINVAL;
  if (reinterpret_cast<uintptr_t>(ops) % 4) {
    set_err(c, "lc_check16: ops must be 4-byte aligned");
    return -EINVAL;
  }
  return check_host(c, ops, key_off, key_base, n_keys, opts, out, aux);
}

int lc_last_call_profile(lc_ctx *c, lc_call_profile *out) {
  if (!c || !out) return -EINVAL;
  *out = c->prof;
  return 0;
}

int lc_check_device_ex(lc_ctx *c, const lc_op *d_ops, const int64_t *d_key_off,
                       int64_t n_keys, const lc_opts *opts, lc_key_result *d_out,
                       void *stream, const lc_aux *aux) {
  if (!c) return -EINVAL;
  const auto t0 = std::chrono::steady_clock::now();
  c->stats = lc_stats{};
  if (n_keys < 0 || (n_keys > 0 && (!d_ops || !d_key_off || !d_out))) {
    set_err(c, "lc_check_device: null buffer or negative n_keys");
    return -EINVAL;
  }
  if (reinterpret_cast<uintptr_t>(d_ops) % 16) {
    set_err(c, "lc_check_device: ops must be 16-byte aligned");
    return -EINVAL;
  }
  lcdev::KParams p;
  int rc = opts_to_params(c, opts, &p);
  if (rc) return rc;
  Dev &d = c->devs[0];
  HIP_TRY(c, hipSetDevice(d.id));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : d.stream;
  WitOut wo;
  const bool want_wit = aux && aux->witness && aux->witness_kind;
  const bool want_cert = aux && aux->certificate;
  if ((want_wit || want_cert) && n_keys > 0) {
    // the record count lives in device memory: key_off[n_keys] - key_off[0]
    int64_t ends[2] = {0, 0};
    HIP_TRY(c, hipMemcpyAsync(&ends[0], d_key_off, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipMemcpyAsync(&ends[1], d_key_off + n_keys, sizeof(int64_t), hipMemcpyDeviceToHost,
                              st));
    HIP_TRY(c, hipStreamSynchronize(st));
    wo.n_records = ends[1] - ends[0];
    if (want_wit) {
      wo.wit = aux->witness;
      wo.kind = aux->witness_kind;
    }
    if (want_cert) {
      wo.cert = aux->certificate;
      wo.cset = aux->certificate_set;
      if (!wo.cset) {  // the position sets still need a home on the device
        if (int e = ensure(c, &d.d_cset, &d.cset_cap, sizeof(int32_t) * (size_t)wo.n_records))
          return e;
        wo.cset = d.d_cset;
      }
    }
  }
  // d_ops points at the record of index d_key_off[0]; the kernels read that
  // base themselves, so a key_off slice of a larger array may be passed.
  rc = run_device(c, d, d_ops, d_key_off, n_keys, p, d_out, st,
                  opts ? opts->flags : 0, wo);
  if (!rc) rc = run_certificates(c, d, d_ops, d_key_off, n_keys, p, d_out, st, wo);
  if (!rc && opts && (opts->flags & LC_FLAG_WHOLE_GPU) && n_keys > 0) {
    // the results and the keys' records are in device memory: read back the
    // verdicts, and each key the frontier exchange takes
    std::vector<lc_key_result> res((size_t)n_keys);
    int64_t base = 0;
    HIP_TRY(c, hipMemcpyAsync(res.data(), d_out, sizeof(lc_key_result) * (size_t)n_keys,
                              hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipMemcpyAsync(&base, d_key_off, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipStreamSynchronize(st));
    std::vector<int64_t> todo, todo_w;
    for (int64_t k = 0; k < n_keys; k++)
      if (res[k].verdict == LC_UNKNOWN && res[k].reason == LC_REASON_CONFIG_BUDGET) todo.push_back(k);
      else if (res[k].verdict == LC_UNKNOWN && res[k].reason == LC_REASON_WINDOW_OVERFLOW)
        todo_w.push_back(k);
    auto fetch = [&](int64_t k, std::vector<lc_op> &v) {
      int64_t se[2];
      if (hipMemcpy(se, d_key_off + k, sizeof se, hipMemcpyDeviceToHost) != hipSuccess) return -EIO;
      v.resize((size_t)(se[1] - se[0]));
      if (!v.empty() && hipMemcpy(v.data(), d_ops + (se[0] - base), sizeof(lc_op) * v.size(),
                                  hipMemcpyDeviceToHost) != hipSuccess)
        return -EIO;
      return 0;
    };
    auto store = [&](int64_t k, const lc_key_result &r) {
      if (want_cert) {
        const int32_t none[4] = {LC_CERT_NONE, -1, -1, 0};
        if (hipMemcpy(aux->certificate + 4 * k, none, sizeof none, hipMemcpyHostToDevice) != hipSuccess)
          return -EIO;
      }
      return hipMemcpy(d_out + k, &r, sizeof r, hipMemcpyHostToDevice) == hipSuccess ? 0 : -EIO;
    };
    rc = whole_gpu(c, todo, opts, fetch, store);
    if (!rc) rc = whole_gpu(c, todo_w, opts, fetch, store);
  }
  c->stats.kernel_ms = d.kernel_ms;
  c->stats.fast_kernel_ms = d.fast_ms;
  c->stats.jit_kernel_ms = d.jit_ms;
  c->stats.n_jit_keys = d.n_jit;
  c->stats.gap_kernel_ms = d.gap_ms;
  c->stats.n_gap_keys = d.n_gap;
  c->stats.hbm_kernel_ms = d.hbm_ms;
  c->stats.n_hbm_keys = d.n_hbm;
  c->stats.n_malformed = d.malformed;
  c->stats.n_keys = n_keys;
  c->stats.n_ops = -1;  // not read back from device memory
  c->stats.n_devices = 1;
  c->stats.total_ms = std::chrono::duration<double, std::milli>(
                          std::chrono::steady_clock::now() - t0).count();
  return rc;
}

int lc_check_device(lc_ctx *c, const lc_op *d_ops, const int64_t *d_key_off,
                    int64_t n_keys, const lc_opts *opts, lc_key_result *d_out,
                    void *stream) {
  return lc_check_device_ex(c, d_ops, d_key_off, n_keys, opts, d_out, stream, nullptr);
}


int lc_check_device32(lc_ctx *c, const lc_op32 *d_ops, const int64_t *d_key_off,
                      const int64_t *d_key_base, int64_t n_keys, const lc_opts *opts,
                      lc_key_result *d_out, void *stream, const lc_aux *aux) {
  if (!c) return -EINVAL;
  if (n_keys < 0 || (n_keys > 0 && (!d_ops || !d_key_off || !d_out))) {
    set_err(c, "lc_check_device32: null buffer or negative n_keys");
    return -EINVAL;
  }
  if (reinterpret_cast<uintptr_t>(d_ops) % 8) {
    set_err(c, "lc_check_device32: ops must be 8-byte aligned");
    return -EINVAL;
  }
  if (n_keys == 0) return lc_check_device_ex(c, nullptr, d_key_off, 0, opts, d_out, stream, aux);
  Dev &d = c->devs[0];
  HIP_TRY(c, hipSetDevice(d.id));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : d.stream;
  const int64_t flags = opts ? opts->flags : 0;
  if (!(aux && (aux->witness || aux->certificate)) &&
      !(flags & (LC_FLAG_NO_FAST_PATH | LC_FLAG_WHOLE_GPU)) && !native32_off()) {
    // decided from the 24-byte records as they are; the 48-byte form (and
    // the record count it needs, read from device memory) only if a key is
    // handed over to the later tiers
    lcdev::KParams p;
    if (int rc = opts_to_params(c, opts, &p)) return rc;
    const auto t0 = std::chrono::steady_clock::now();
    c->stats = lc_stats{};
    WitOut wo;
    wo.ops32 = d_ops;
    wo.base32 = d_key_base;
    wo.widen = [&](const lc_op **out) -> int {
      int64_t *ends = reinterpret_cast<int64_t *>(d.h_status);  // (pinned; read before any later status copy)
      HIP_TRY(c, hipMemcpyAsync(&ends[0], d_key_off, sizeof(int64_t), hipMemcpyDeviceToHost, st));
      HIP_TRY(c, hipMemcpyAsync(&ends[1], d_key_off + n_keys, sizeof(int64_t), hipMemcpyDeviceToHost,
                                st));
      HIP_TRY(c, hipStreamSynchronize(st));
      const int64_t nrec = ends[1] - ends[0];
      if (nrec < 0) {
        set_err(c, "lc_check_device32: key_off[n_keys] < key_off[0]");
        return -EINVAL;
      }
      if (int e = ensure(c, reinterpret_cast<char **>(&d.d_ops), &d.ops_cap,
                         sizeof(lc_op) * (size_t)std::max<int64_t>(nrec, 1)))
        return e;
      HIP_TRY(c, lcdev::launch_widen32(d_ops, d_key_off, d_key_base, n_keys, 4 * (nrec / n_keys + 1),
                                       static_cast<lc_op *>(d.d_ops), st));
      *out = static_cast<const lc_op *>(d.d_ops);
      return 0;
    };
    int rc = run_device(c, d, nullptr, d_key_off, n_keys, p, d_out, st, flags, wo);
    c->stats.kernel_ms = d.kernel_ms;
    c->stats.fast_kernel_ms = d.fast_ms;
    c->stats.jit_kernel_ms = d.jit_ms;
    c->stats.n_jit_keys = d.n_jit;
    c->stats.gap_kernel_ms = d.gap_ms;
    c->stats.n_gap_keys = d.n_gap;
    c->stats.hbm_kernel_ms = d.hbm_ms;
    c->stats.n_hbm_keys = d.n_hbm;
    c->stats.n_malformed = d.malformed;
    c->stats.n_keys = n_keys;
    c->stats.n_ops = -1;
    c->stats.n_devices = 1;
    c->stats.total_ms = std::chrono::duration<double, std::milli>(
                            std::chrono::steady_clock::now() - t0).count();
    return rc;
  }
  // the record count lives in device memory: key_off[n_keys] - key_off[0]
  int64_t *ends = reinterpret_cast<int64_t *>(d.h_status);  // (pinned; free between calls)
  HIP_TRY(c, hipMemcpyAsync(&ends[0], d_key_off, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipMemcpyAsync(&ends[1], d_key_off + n_keys, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipStreamSynchronize(st));
  const int64_t nrec = ends[1] - ends[0];
  if (nrec < 0) {
    set_err(c, "lc_check_device32: key_off[n_keys] < key_off[0]");
    return -EINVAL;
  }
  if (int e = ensure(c, reinterpret_cast<char **>(&d.d_ops), &d.ops_cap, sizeof(lc_op) * (size_t)nrec))
    return e;
  // the grid's second dimension for long keys: sized from the mean length
  // (any size is correct: each workgroup strides its key)
  HIP_TRY(c, lcdev::launch_widen32(d_ops, d_key_off, d_key_base, n_keys, 4 * (nrec / n_keys + 1),
                                   static_cast<lc_op *>(d.d_ops), st));
  return lc_check_device_ex(c, static_cast<const lc_op *>(d.d_ops), d_key_off, n_keys, opts, d_out,
                            stream, aux);
}

int lc_check_frontiers(lc_ctx *c, const lc_op *ops, const int64_t *key_off, int64_t n_keys,
                       const int64_t *stop_op, const lc_opts *opts, lc_fx_config *out,
                       int32_t max_per_key, int32_t *n_out) {
  if (!c) return -EINVAL;
  if (n_keys < 0 || max_per_key < 1 ||
      (n_keys > 0 && (!ops || !key_off || !stop_op || !out || !n_out))) {
    set_err(c, "lc_check_frontiers: null buffer, negative n_keys or max_per_key < 1");
    return -EINVAL;
  }
  if (n_keys == 0) return 0;
  if (key_off[0] < 0) {
    set_err(c, "lc_check_frontiers: key_off[0] < 0");
    return -EINVAL;
  }
  for (int64_t k = 0; k < n_keys; k++)
    if (key_off[k + 1] < key_off[k]) {
      set_err(c, "lc_check_frontiers: key_off not monotone at key " + std::to_string(k));
      return -EINVAL;
    }
  lcdev::KParams p;
  if (int rc = opts_to_params(c, opts, &p)) return rc;
  Dev &d = c->devs[0];
  HIP_TRY(c, hipSetDevice(d.id));
  (void)settle_status(d);  // a fused call's status copy may still be pending
  const int64_t r0 = key_off[0], nrec = key_off[n_keys] - r0;
  const size_t cfg_bytes = sizeof(lc_fx_config) * (size_t)max_per_key * (size_t)n_keys;
  // scratch: the records, offsets, stops and results share the context's
  // lc_check buffers (a context is not re-entrant)
  int e = ensure(c, reinterpret_cast<char **>(&d.d_ops), &d.ops_cap, sizeof(lc_op) * (size_t)nrec);
  if (!e) e = ensure(c, &d.d_off, &d.off_cap, sizeof(int64_t) * (size_t)(2 * n_keys + 1));
  if (!e) e = ensure(c, reinterpret_cast<char **>(&d.d_gws), &d.gws_cap, cfg_bytes);
  if (!e) e = ensure(c, &d.d_jit, &d.jit_cap, sizeof(int32_t) * (size_t)n_keys);
  if (!e) e = ensure(c, &d.d_jit2, &d.jit2_cap, sizeof(int32_t) * (size_t)n_keys);
  if (e) return e;
  int64_t *d_stop = d.d_off + (n_keys + 1);
  lc_fx_config *d_cfg = reinterpret_cast<lc_fx_config *>(d.d_gws);
  const lc_op *d_ops = static_cast<const lc_op *>(d.d_ops);
  hipStream_t st = d.stream;
  // the inputs: through the staging buffer when pageable and small (as lc_check's)
  const void *src_ops = ops + r0, *src_off = key_off, *src_stop = stop_op;
  const size_t ops_b = sizeof(lc_op) * (size_t)nrec, off_b = sizeof(int64_t) * (size_t)(n_keys + 1),
               stop_b = sizeof(int64_t) * (size_t)n_keys;
  if (ops_b + off_b + stop_b + 512 <= kStageMax && !stage_off() && !is_pinned(c, ops + r0, ops_b)) {
    char *sb = stage_buf(c, d);
    if (!sb) return -ENOMEM;
    char *so = sb, *sf = so + ((ops_b + 255) & ~size_t(255)), *ss = sf + ((off_b + 255) & ~size_t(255));
    std::memcpy(so, src_ops, ops_b);
    std::memcpy(sf, src_off, off_b);
    std::memcpy(ss, src_stop, stop_b);
    src_ops = so;
    src_off = sf;
    src_stop = ss;
  }
  HIP_TRY(c, hipMemcpyAsync(d.d_ops, src_ops, ops_b, hipMemcpyHostToDevice, st));
  HIP_TRY(c, hipMemcpyAsync(d.d_off, src_off, off_b, hipMemcpyHostToDevice, st));
  HIP_TRY(c, hipMemcpyAsync(d_stop, src_stop, stop_b, hipMemcpyHostToDevice, st));
  HIP_TRY(c, hipMemsetAsync(d.d_status, 0, sizeof(lcdev::KStatus), st));
  d.status_dirty = true;
  HIP_TRY(c, lcdev::launch_frontier_dump(d_ops, d.d_off, d_stop, n_keys, p, d_cfg, max_per_key, d.d_jit,
                                         d.d_jit2, &d.d_status->n_overflow, st));
  HIP_TRY(c, hipMemcpyAsync(d.h_status, d.d_status, sizeof(lcdev::KStatus), hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipStreamSynchronize(st));
  // keys whose search outgrew the LDS regions: again over HBM tables (the
  // first HBM tier's 16k configurations per set), one wavefront per key
  if (const int32_t n_retry = d.h_status->n_overflow) {
    const int waves = std::min<int>(n_retry, 256);
    if (!(e = ensure(c, reinterpret_cast<char **>(&d.d_ws), &d.ws_cap,
                     lcdev::hbm_tier_ws_bytes(waves, kHbmCap[0]))))
      HIP_TRY(c, lcdev::launch_frontier_dump_hbm(d_ops, d.d_off, d_stop, d.d_jit2, n_retry, p, d.d_ws,
                                                 waves, kHbmCap[0], d_cfg, max_per_key, d.d_jit,
                                                 &d.d_status->hbm_next, st));
    else
      return e;
  }
  HIP_TRY(c, hipMemsetAsync(d.d_status, 0, sizeof(lcdev::KStatus), st));
  HIP_TRY(c, hipMemcpyAsync(n_out, d.d_jit, sizeof(int32_t) * (size_t)n_keys, hipMemcpyDeviceToHost, st));
  // one copy of every key's slots (C5's 94 keys x 10: 0.5 MB) rather than one
  // per key; slots past a key's count keep the device's scratch
  HIP_TRY(c, hipMemcpyAsync(out, d_cfg, cfg_bytes, hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipStreamSynchronize(st));
  d.status_dirty = false;
  return 0;
}

int lc_pack32(const lc_op *ops, const int64_t *key_off, int64_t n_keys, lc_op32 *out,
              int64_t *key_base) {
  if (n_keys < 0 || (n_keys > 0 && (!ops || !key_off || !out || !key_base))) return -EINVAL;
  if (n_keys == 0) return 0;
  if (key_off[0] < 0) return -EINVAL;
  for (int64_t k = 0; k < n_keys; k++)
    if (key_off[k + 1] < key_off[k]) return -EINVAL;
  constexpr int64_t kFieldMax = 0x7FFFFFFE, kNever = 0xFFFFFFFFll;
  // the device's decoding (records.h, decode) of a 48-byte record, applied
  // here: what it reads of each field fits 32 bits
  auto pack = [&](int64_t k0, int64_t k1) {
    for (int64_t k = k0; k < k1; k++) {
      const int64_t b = key_off[k], e = key_off[k + 1];
      const int64_t base = e > b ? ops[b].call : 0;
      key_base[k] = base;
      for (int64_t i = b; i < e; i++) {
        const lc_op &o = ops[i];
        const int64_t rc = o.call - base, rr = o.ret - base;
        const bool bad = o.value < -1 || o.value > kFieldMax || o.expected < -1 ||
                         o.expected > kFieldMax || o.call < 0 || o.ret <= o.call || rc < 0 ||
                         rc >= kNever || (o.ret != LC_INF && rr >= kNever);
        lc_op32 &q = out[i];
        q.f = o.f >= 0 && o.f <= LC_F_CAS ? (int32_t)o.f : 3;
        q.value = bad ? -2 : (int32_t)o.value;  // -2: malformed, in either width
        q.expected = (int32_t)o.expected;
        q.version = o.version < -1 || o.version > kFieldMax ? (int32_t)kFieldMax : (int32_t)o.version;
        q.call = (uint32_t)rc;
        // (a malformed record's return may land on LC_INF32 modulo 2^32: it
        // stays a return, which is what the witness initialisation reads)
        q.ret = o.ret == LC_INF ? LC_INF32 : (uint32_t)rr == LC_INF32 ? LC_INF32 - 1 : (uint32_t)rr;
      }
    }
  };
  const int64_t n_rec = key_off[n_keys] - key_off[0];
  const int nth = (int)std::min<int64_t>(16, std::max<int64_t>(1, std::min<int64_t>(n_keys, n_rec >> 18)));
  if (nth <= 1) {
    pack(0, n_keys);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < nth; t++) th.emplace_back(pack, n_keys * t / nth, n_keys * (t + 1) / nth);
    for (auto &x : th) x.join();
  }
  return 0;
}

int lc_pack16(const lc_op *ops, const int64_t *key_off, int64_t n_keys, lc_op16 *out,
              int64_t *key_base) {
  if (n_keys < 0 || (n_keys > 0 && (!ops || !key_off || !out || !key_base))) return -EINVAL;
  if (n_keys == 0) return 0;
  if (key_off[0] < 0) return -EINVAL;
  for (int64_t k = 0; k < n_keys; k++)
    if (key_off[k + 1] < key_off[k]) return -EINVAL;
  constexpr int64_t kFieldMax = 0x7FFFFFFE, kNever = 0xFFFFFFFFll;
  // lc_pack32's narrowing, then the ids into 15 bits (a record it marks
  // malformed: value field 0x7FFF, its expected field clamped — the device
  // reads nothing else of a malformed key's records)
  std::atomic<bool> range{true};
  auto pack = [&](int64_t k0, int64_t k1) {
    for (int64_t k = k0; k < k1; k++) {
      const int64_t b = key_off[k], e = key_off[k + 1];
      const int64_t base = e > b ? ops[b].call : 0;
      key_base[k] = base;
      for (int64_t i = b; i < e; i++) {
        const lc_op &o = ops[i];
        const int64_t rc = o.call - base, rr = o.ret - base;
        const bool bad = o.value < -1 || o.value > kFieldMax || o.expected < -1 ||
                         o.expected > kFieldMax || o.call < 0 || o.ret <= o.call || rc < 0 ||
                         rc >= kNever || (o.ret != LC_INF && rr >= kNever);
        if (!bad && (o.value > LC_ID15_MAX || o.expected > LC_ID15_MAX)) {
          range.store(false, std::memory_order_relaxed);
          return;
        }
        const uint32_t f = o.f >= 0 && o.f <= LC_F_CAS ? (uint32_t)o.f : 3u;
        const uint32_t v = bad ? 0x7FFFu : (uint32_t)(o.value + 1);
        const uint32_t x = (uint32_t)std::min<int64_t>(0x7FFF, std::max<int64_t>(0, o.expected + 1));
        lc_op16 &q = out[i];
        q.fve = f << 30 | v << 15 | x;
        q.version = o.version < -1 || o.version > kFieldMax ? (int32_t)kFieldMax : (int32_t)o.version;
        q.call = (uint32_t)rc;
        q.ret = o.ret == LC_INF ? LC_INF32 : (uint32_t)rr == LC_INF32 ? LC_INF32 - 1 : (uint32_t)rr;
      }
    }
  };
  const int64_t n_rec = key_off[n_keys] - key_off[0];
  const int nth = (int)std::min<int64_t>(16, std::max<int64_t>(1, std::min<int64_t>(n_keys, n_rec >> 18)));
  if (nth <= 1) {
    pack(0, n_keys);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < nth; t++) th.emplace_back(pack, n_keys * t / nth, n_keys * (t + 1) / nth);
    for (auto &x : th) x.join();
  }
  return range.load() ? 0 : -ERANGE;
}

}  // extern "C"
