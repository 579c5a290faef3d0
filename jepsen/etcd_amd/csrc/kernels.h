// kernels.h — internal interface between the host runtime (lincheck.cpp) and
// the device code (check_kernel.hip).  Not part of the public C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../../include/lincheck.h"
#include "../../../include/lincheck_fx.h"

namespace lcdev {

// Launch parameters shared by both tiers.
struct KParams {
  int32_t init_ver;
  int32_t init_val;
  int64_t budget;      // max configurations generated per key
  uint64_t time_ticks; // max device wall-clock ticks per key in the search tiers (0: none)
};

// Device-side status words, zeroed before every call.
// Longest key the version-order tier and the crash-light pass decide (4
// records per thread of a 256-thread workgroup); longer keys go on to the gap
// tier proper.
constexpr int kFastMaxRecords = 1024;

struct KStatus {
  int32_t malformed;    // keys with LC_REASON_MALFORMED
  int32_t n_overflow;   // keys appended to the overflow list (LDS tier full)
  int32_t n_overflow2;  // keys that also overflowed the first HBM tier
  int32_t n_jit;        // keys handed over by the fast tier
  int32_t max_len;      // longest key among them (records)
  int32_t n_jit2;       // keys the gap tier passes on to the JIT search
  int32_t n_cex;        // gap tier: invalid keys awaiting their counterexample
  int32_t n_open;       // gap tier: counterexample intervals still open after a round
  int32_t max_lds;      // gap tier: largest matching footprint (bytes) of a full decision
  int32_t any_handoff;  // fast tier: some key was handed over (read before the host store)
  int32_t n_gap2;       // crash-light pass: keys it passes on to the gap tier
  int32_t hbm_next;     // HBM tiers: next list entry to claim (zeroed before each launch)
  int32_t n_light;      // fused tier: keys that took the crash-light decision (host: light_count)
  // ... counted on the device in kLightShards counters 128 B apart, by key:
  // one same-address device-scope atomic per key (10,000 on the crash leg)
  // queued behind one another and held up the workgroups' stores and loads
  // (fused pass 0.166 -> 0.121 ms without it)
  int32_t n_light_sh[32 * 32];
};
constexpr int kLightShards = 32, kLightStride = 32;
__host__ __device__ inline int32_t *light_shard(KStatus *s, int64_t key) {
  return &s->n_light_sh[(key & (kLightShards - 1)) * kLightStride];
}
// The sum of the shards, into n_light (host, after the status copy).
inline int32_t light_count(KStatus &s) {
  int32_t n = 0;
  for (int i = 0; i < kLightShards; i++) n += s.n_light_sh[i * kLightStride];
  s.n_light = n;
  return n;
}

constexpr int kWave = 64;
constexpr int kWavesPerWG = 4;   // independent keys per 256-thread workgroup
constexpr int kLdsCap = 128;     // configurations per LDS region (3 regions/wave)

// Fast tier: one 256-thread workgroup per key decides version-pinned keys
// (check_kernel.hip, "Version-order fast tier"); the others are handed over
// to the gap tier or the JIT search (below).
// Status protocol: *d_status is all-zero when the launch starts, and the host
// zeroes *h_handoff (host-coherent memory) before it.  A workgroup that hands
// its key over also stores 1 to *h_handoff, so when every key is decided the
// host needs no memset or copy around this kernel: one launch plus one sync.
// A workgroup hands its key over by a plain store of d_flags[key] (1: for
// the gap tier, 2: jit-only — an :ok mutation without a version, a read
// [nil x], malformed records); launch_handoff_compact then builds the lists
// (d_jit_keys / status->n_jit for the gap tier, status->max_len; with
// route_direct the jit-only keys go to d_direct_keys / status->n_jit2 for the
// JIT search, else to d_jit_keys too) and clears the flags.  (One returning
// same-address atomicAdd per handed-over key serialised: 10k handoffs cost
// the launch 0.16 ms.)
// (A grid-wide "last workgroup" counter instead costs 10k same-address
// atomics per launch: measured 0.115 -> 0.345 ms.)
// The follower of a version-order / fused pass launch on the same stream:
// one thread stores seq to *h_done (host-mapped) once the pass has retired
// (stream order).  The host spins on that word instead of recording events
// around the launch and waiting on the second: an empty 1,250-workgroup
// launch took 10.1 us per step this way against 15.0 (tools/doorbell_probe.hip).
hipError_t launch_done_signal(uint32_t *h_done, uint32_t seq, hipStream_t stream);

// Resident version-order grid (check_kernel.hip, "Resident grid"): for
// lc_check_device calls on batches of at most one key per resident
// workgroup, a grid launched once stays on the GPU and serves request after
// request, so back-to-back calls (a C3 shard's step) pay no launch and no
// follower kernel.  A request is kResWords eight-byte words, each carrying
// the request's number (mod 2^16) in its top 16 bits — the data is its own
// flag: the host writes them to ResHost::req; wave 0 of workgroup 0 polls
// that line (one PCIe read per poll) until every word carries the next
// number, copies the words to ResDev::req with write-through stores, and
// wave 0 of every other workgroup polls those until every word carries it.
// Each workgroup then decides key blockIdx.x exactly as fast_tier_kernel
// does (records, offsets and first calls read with L1-bypassing loads,
// results written through) and, its stores drained, adds to a sharded
// arrival counter; the last arrival stores (number << 32 | wall clock) to
// ResHost::done.  A key the tier hands over is flagged as in
// fast_tier_kernel (the host then stops the grid, whose exit publishes the
// flags, before the later tiers run).  A request with n_keys == kResExitKeys
// ends the grid; workgroup 0 also leaves after idle_ticks of the 100 MHz
// wall clock without a request (ResHost::exited = 1; the others follow its
// exit request), and every wait is bounded by a poll count too, so the grid
// always drains.
constexpr int kResWords = 9;   // ops, key_off, n_keys, out, flags, status, h_handoff, init_ver, init_val
constexpr int kResShards = 16;
constexpr int64_t kResExitKeys = (int64_t(1) << 47) - 1;
__host__ __device__ inline uint64_t res_word(uint64_t v, uint32_t seq) {
  return (v & ((uint64_t(1) << 48) - 1)) | (uint64_t)(seq & 0xFFFFu) << 48;
}
__host__ __device__ inline uint64_t res_val(uint64_t w) { return w & ((uint64_t(1) << 48) - 1); }
struct alignas(128) ResHost {  // hipHostMalloc(Mapped | Coherent)
  uint64_t req[16];            // host: the request words (kResWords used)
  uint64_t done;               // device: (number << 32) | low 32 bits of the wall clock at completion
  uint64_t t0;                 // device: wall clock (low 32 bits) when workgroup 0 saw the request
  uint32_t exited;             // device: 1 once workgroup 0 left on its idle bound
  uint32_t pad[27];
};
struct alignas(128) ResDev {   // hipMalloc, zeroed before each grid launch
  uint64_t req[16];
  uint32_t ticket[kResShards * 32];
  uint32_t top;
  uint32_t pad1[31];
};
hipError_t launch_fast_resident(ResHost *h_res, ResDev *d_res, int64_t grid, uint64_t idle_ticks,
                                hipStream_t stream);
// resident 256-thread workgroups of fast_resident_kernel on this device
int64_t fast_resident_capacity();
hipError_t launch_fast_tier(const lc_op *d_ops, const int64_t *d_key_off,
                            int64_t n_keys, const KParams &p,
                            lc_key_result *d_out, int32_t *d_flags,
                            KStatus *d_status, int32_t *h_handoff, hipStream_t stream);
// The version-order tier and the crash-light decision in one pass over every
// key, for batches where most keys carry crashed writes/CAS: undecided keys
// are flagged for the handoff compaction (as launch_fast_tier), and go to the
// gap tier without a crash-light pass.  status->n_light counts the keys that
// took the crash-light decision.
// The version-order tier / fused pass over lc_op32 records (ABI 4) with the
// keys' bases (null: 0), no witnesses: same decisions as on the widened
// records; the keys they hand over need the 48-byte records (launch_widen32).
hipError_t launch_fast_tier32(const lc_op32 *d_ops, const int64_t *d_key_off, const int64_t *d_key_base,
                              int64_t n_keys, const KParams &p, lc_key_result *d_out, int32_t *d_flags,
                              KStatus *d_status, int32_t *h_handoff, hipStream_t stream);
hipError_t launch_fused_tier32(const lc_op32 *d_ops, const int64_t *d_key_off, const int64_t *d_key_base,
                               int64_t n_keys, const KParams &p, lc_key_result *d_out, int32_t *d_flags,
                               KStatus *d_status, int32_t *h_handoff, hipStream_t stream);
hipError_t launch_fused_tier(const lc_op *d_ops, const int64_t *d_key_off, int64_t n_keys,
                             const KParams &p, lc_key_result *d_out, int32_t *d_flags,
                             KStatus *d_status, int32_t *h_handoff, int32_t *d_witness,
                             int32_t *d_witness_kind, hipStream_t stream);
// Crash-light pass (check_kernel.hip, "Crash-light keys"): over the
// compacted gap-tier list d_keys (status->n_jit keys, at most max_keys), a
// key whose only obstacle is a few crashed writes/CAS is decided valid in
// place (the gap tier's procedure, one record pass), completing its witness
// (d_witness / d_witness_kind may be null); the others go to d_pass
// (status->n_gap2) for the gap tier.
hipError_t launch_gap_light(const lc_op *d_ops, const int64_t *d_key_off, const int32_t *d_keys,
                            int64_t max_keys, const KParams &p, lc_key_result *d_out,
                            int32_t *d_pass, KStatus *d_status, int32_t *d_witness,
                            int32_t *d_witness_kind, hipStream_t stream);
// After a fused pass that handed nothing over: the crash-light key count
// (the sum of the shards) to *h_light (mapped host memory), then *d_status
// zeroed for the next call — one launch instead of a copy and a memset.
hipError_t launch_status_settle(KStatus *d_status, int32_t *h_light, hipStream_t stream);
// With witness_kind, every handed-over key's kind is reset to
// LC_WITNESS_NONE (a later tier that certifies it sets it again).
hipError_t launch_handoff_compact(int32_t *d_flags, const int64_t *d_key_off, int64_t n_keys,
                                  int route_direct, int32_t *d_jit_keys, int32_t *d_direct_keys,
                                  KStatus *d_status, int32_t *d_witness_kind, hipStream_t stream);

// Witness (lc_aux) for the keys the version-order tier decides: their
// linearization is the version order itself, so every record gets its
// pinned position (an :ok write/CAS with version v: v - V0 - 1; everything
// else -1) and every key kind LC_WITNESS_FULL (fast_on) or NONE.  Launched
// before the tiers; later tiers overwrite the keys they take.
hipError_t launch_witness_init(const lc_op *d_ops, const int64_t *d_key_off, int64_t n_keys,
                               int64_t n_records, const KParams &p, int fast_on,
                               int32_t *d_witness, int32_t *d_witness_kind, hipStream_t stream);

// lc_op32 records (ABI 4) widened into lc_op records for the tiers, the key's
// base (d_key_base[k], or 0 when null) added to call / ret; d_in and d_out
// point at the record of index d_key_off[0] (d_in 8-byte aligned, d_out
// 16-byte).  max_len: the longest key's records (sizes the grid).
hipError_t launch_widen32(const lc_op32 *d_in, const int64_t *d_key_off, const int64_t *d_key_base,
                          int64_t n_keys, int64_t max_len, lc_op *d_out, hipStream_t stream);
// The same for lc_op16 records (d_in 16-byte aligned): the 15-bit ids
// unpacked (0x7FFF -> -2) as include/lincheck.h defines them.
hipError_t launch_widen16(const lc_op16 *d_in, const int64_t *d_key_off, const int64_t *d_key_base,
                          int64_t n_keys, int64_t max_len, lc_op *d_out, hipStream_t stream);

// lc_check_frontiers (include/lincheck_fx.h): the LDS tier's search per key
// up to the :ok return of record d_stop[k], its frontier written to
// d_out[k * max ...] (n per key in d_n_out: >= 0 written, -1 not reached).
// Keys whose search outgrows the LDS regions are listed in d_retry (count
// *d_n_retry, zero at launch) for launch_frontier_dump_hbm: the same search
// over HBM tables of `cap` configurations (hbm_tier_ws_bytes(n_waves, cap)
// of workspace; keys claimed from *d_next, zero at launch).
hipError_t launch_frontier_dump(const lc_op *d_ops, const int64_t *d_key_off, const int64_t *d_stop,
                                int64_t n_keys, const KParams &p, ::lc_fx_config *d_out, int max,
                                int32_t *d_n_out, int32_t *d_retry, int32_t *d_n_retry,
                                hipStream_t stream);
hipError_t launch_frontier_dump_hbm(const lc_op *d_ops, const int64_t *d_key_off,
                                    const int64_t *d_stop, const int32_t *d_keys, int32_t n_list,
                                    const KParams &p, void *d_ws, int n_waves, int64_t cap,
                                    ::lc_fx_config *d_out, int max, int32_t *d_n_out, int32_t *d_next,
                                    hipStream_t stream);

// LDS tier (JIT search): one wavefront per key, for the keys in d_keys
// (n_keys of them), or for keys 0..n_keys-1 when d_keys is null.  In every
// tier key_off is indexed by local key id and d_ops points at the record of
// index key_off[0] (a slice of a larger array may be passed); kernels read
// key_off[0] themselves.
// Keys whose frontier outgrows the LDS regions are appended to ovf_keys
// (count in status->n_overflow) with reason LC_REASON_FRONTIER_LDS.
hipError_t launch_lds_tier(const lc_op *d_ops, const int64_t *d_key_off,
                           const int32_t *d_keys, int64_t n_keys,
                           const KParams &p, lc_key_result *d_out, int32_t *d_ovf_keys,
                           KStatus *d_status, hipStream_t stream);

// HBM tier: re-runs the listed keys with configuration sets in global memory
// (open-addressed hash tables, 128-byte buckets).  ws is a workspace of
// hbm_tier_ws_bytes(n_waves, cap) bytes (no initial contents: each
// workgroup zeroes its tag arrays at launch); cap =
// configurations per set.  Keys that overflow again are appended to
// d_ovf_out (count *d_n_ovf_out) unless last_tier, where they become
// LC_REASON_CONFIG_BUDGET (:unknown).
size_t hbm_tier_ws_bytes(int n_waves, int64_t cap);
// Cooperative variant: one workgroup of waves_per_key (4, 8 or 16) wavefronts
// per key, its waves expanding the key's frontier together (for short key
// lists, where a wavefront per key leaves SIMDs idle).  Workspace:
// hbm_tier_ws_bytes(n_wg, cap).
// Both HBM launches count the keys they find malformed in *d_malformed (the
// first frontier-search tier a key reaches reports it: the LDS tier, or the
// HBM tier when few keys skip the LDS tier).  Workgroups claim list entries
// from *d_next (zero at launch), so a workgroup that drew quick keys takes
// more of them.
hipError_t launch_hbm_coop(const lc_op *d_ops, const int64_t *d_key_off, const int32_t *d_keys,
                           int32_t n_list, const KParams &p, lc_key_result *d_out, void *d_ws,
                           int n_wg, int64_t cap, int32_t *d_ovf_out, int32_t *d_n_ovf_out,
                           int32_t *d_malformed, int32_t *d_next, int last_tier,
                           int waves_per_key, hipStream_t stream);
hipError_t launch_hbm_tier(const lc_op *d_ops, const int64_t *d_key_off,
                           const int32_t *d_keys,
                           int32_t n_list, const KParams &p, lc_key_result *d_out,
                           void *d_ws, int n_waves, int64_t cap,
                           int32_t *d_ovf_out, int32_t *d_n_ovf_out, int32_t *d_malformed,
                           int32_t *d_next, int last_tier, hipStream_t stream);

// Gap tier (gap_tier.hip): version-pinned keys with crashed writes/CAS are
// decided by matching gaps to optional ops; keys it cannot decide are
// appended to d_pass_keys (status->n_jit2).  A call runs two kinds of launch
// (GapJob::mode):
//   kGapFull   one 256-thread workgroup per listed key decides the whole
//              history.  With `bisect` the same workgroup then bisects an
//              invalid key's prefixes for its counterexample (many or short
//              keys); without, invalid keys go to the counterexample list
//              (cex_*, status->n_cex) with the interval [0, last return].
//   kGapProbe  P workgroups per open counterexample interval each decide one
//              history prefix (a multisection of the interval), then
//              launch_gap_narrow shrinks the intervals by the probes' verdicts
//              (status->n_open = intervals still open) and writes the results
//              of closed ones.  Rounds repeat until none is open: a single
//              hot key (BASELINE configs[3]) spreads over the whole GPU.
// Workspace: gap_tier_ws_bytes(n_wg, cap) with cap >= longest key + 2.
//   kGapWitness  (lc_aux witnesses only) one workgroup per counterexample
//              closed by the multisection re-decides the prefix just before
//              the failing return and writes its linearization.
// With `wit`, every valid full decision writes its linearization (the
// mutation position of each record, lc_aux) and sets wkind[key] =
// LC_WITNESS_FULL; an invalid key bisected in place gets the witness of
// the prefix before its failing return (LC_WITNESS_PREFIX).
enum { kGapFull = 0, kGapProbe = 1, kGapWitness = 2 };
constexpr int kGapNodeBudget = 4096;  // matching passes per decision (gapmatch.h)
// ... of which the expected-value-first search may spend this many before the
// plain-order rerun takes over with the full budget (C4 decisions take 1-10;
// a search that needs hundreds is better off in the plain order)
constexpr int kGapPrefBudget = 512;
struct GapJob {
  int32_t mode;        // kGapFull / kGapProbe / kGapWitness
  int32_t bisect;      // kGapFull: bisect invalid keys in place
  int32_t P;           // probes per interval (kGapProbe; 1 for kGapWitness)
  int32_t lds_bytes;   // dynamic LDS per workgroup for the matching arrays
  int32_t threads;     // workgroup size: 256, or 64 for short keys (one wave per decision)
  int32_t n_tasks;     // keys (full), intervals x P (probe), intervals (witness)
  int32_t give_up;     // launch_gap_narrow: pass every open interval on to the JIT tier
  int32_t pref_budget; // matching passes of the expected-value-first search before the
                       //   plain-order rerun (gapmatch.h; LC_GAP_PREF_BUDGET tests it)
  int32_t *cex_key;    // per counterexample: the key
  uint32_t *cex_lo;    // key-relative event interval [lo, hi] holding the
  uint32_t *cex_hi;    //   first return whose prefix is not linearizable
  int32_t *cex_gaps;   // gaps of the full history (reported as max_frontier)
  int32_t *cex_state;  // 0 open, 1 closed (decided invalid), 2 passed on to the JIT tier
  int64_t *cex_nodes;  // matching passes spent on the key
  int32_t *probe;      // [n_cex * P] probe verdicts
  int32_t *wit;        // lc_aux witness (per record, indexed like the ops), or null
  int32_t *wkind;      // lc_aux witness kind (per key)
  // kGapFull launched before the host has read the task count (lincheck.cpp,
  // "launched early"): the count on the device, capped by n_tasks; or null
  const int32_t *n_tasks_dev;
};
size_t gap_tier_ws_bytes(int n_wg, int64_t cap);
// 256-thread gap-tier workgroups with lds_bytes of dynamic LDS the device
// holds at once (0 if the runtime cannot tell)
int gap_tier_resident(int lds_bytes, int threads);
hipError_t launch_gap_tier(const lc_op *d_ops, const int64_t *d_key_off, const int32_t *d_keys,
                           const KParams &p, lc_key_result *d_out, int32_t *d_ws, int n_wg,
                           int64_t cap, int32_t *d_pass_keys, KStatus *d_status,
                           const GapJob &job, hipStream_t stream);
hipError_t launch_gap_narrow(const lc_op *d_ops, const int64_t *d_key_off, int32_t n_cex,
                             lc_key_result *d_out, int32_t *d_pass_keys, KStatus *d_status,
                             const GapJob &job, hipStream_t stream);

// Infeasibility certificates (cert.hip, lc_aux ABI 3): one 256-thread
// workgroup per key; every LC_INVALID key of d_out gets {kind, a, b, c} in
// d_cert (4 int32 per key) and, for LC_CERT_HALL, its positions at the start
// of its records' slots of d_cset; other keys LC_CERT_NONE.  Workspace:
// cert_ws_bytes(n_records, n_keys).
size_t cert_ws_bytes(int64_t n_records, int64_t n_keys);
// Every key {LC_CERT_NONE, -1, -1, 0} (what launch_certificates writes for a
// key that is not LC_INVALID), for calls in which no key can be invalid.
hipError_t launch_cert_none(int32_t *d_cert, int64_t n_keys, hipStream_t stream);
hipError_t launch_certificates(const lc_op *d_ops, const int64_t *d_key_off, int64_t n_keys,
                               int64_t n_records, const KParams &p, const lc_key_result *d_out,
                               int32_t *d_ws, int32_t *d_cert, int32_t *d_cset,
                               hipStream_t stream);

}  // namespace lcdev
