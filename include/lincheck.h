/*
 * lincheck.h — C ABI of the MI355X linearizability checker for jepsen.etcd's
 * `register` workload (VersionedRegister model).
 *
 * Drop-in boundary.  The reference wires the check at
 *   /root/reference/src/jepsen/etcd/register.clj:108-112
 *     (independent/checker (checker/compose {:linear (checker/linearizable
 *        {:model (->VersionedRegister 0 nil)}) :timeline (timeline/html)}))
 * and calls it through the jepsen.checker/Checker protocol
 *   (check [this test history opts]) -> {:valid? ...}
 * from checker/compose at /root/reference/src/jepsen/etcd.clj:129-141.
 * The model's step function is register.clj:59-96.
 *
 * This library replaces `independent/checker` + `:linear` as one unit: the JVM
 * (or any host) pairs invoke/completion ops, splits the history by independent
 * key, interns values to dense ids and packs one `lc_op` per operation; one
 * lc_check() call then decides every key.  The cgo-free JNA/Panama binding a
 * maintainer adds on the Clojure side is shown in INTEGRATION.md.
 *
 * Plain C types only; no HIP or torch types appear in any signature.
 */
#ifndef LINCHECK_H
#define LINCHECK_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LC_ABI_VERSION 5  /* 3: lc_aux certificates, lc_device_stats, lc_host_register;
                             4: 24-byte lc_op32 records (lc_pack32, lc_check32,
                             lc_check_device32), lc_last_call_profile;
                             5: 16-byte lc_op16 records (lc_pack16, lc_check16,
                             lc_edn_ops16), lc_quiesce (the resident
                             version-order grid) */

/* Op kinds: the three :f values of register.clj:98-100 (r / w / cas). */
#define LC_F_READ  0
#define LC_F_WRITE 1
#define LC_F_CAS   2

/* nil (Clojure nil) for value / expected / version fields. */
#define LC_NIL ((int64_t)-1)
/* Return index of an op that never completed (:info, or unterminated). */
#define LC_INF INT64_MAX

/*
 * One operation of one key's subhistory, 6 x int64 = 48 bytes.
 *
 *  f        LC_F_READ / LC_F_WRITE / LC_F_CAS
 *  value    read: the value read (:ok value [version value], register.clj:27)
 *           write: the value written ([nil v] invoke, register.clj:99)
 *           cas: the new value v' of [old new] (register.clj:100)
 *           interned id >= 0, or LC_NIL.
 *  expected cas: the old value v; otherwise LC_NIL.
 *  version  the version of the :ok completion (register.clj:27,31,38-39);
 *           LC_NIL for :info ops (whose value stays the invoke's [nil ...]).
 *           Any int64 is accepted: a version no state of the key can reach
 *           (below init_version, above init_version + the key's op count,
 *           beyond int32) makes the op illegal at every step, as in knossos.
 *  call     history index of the invocation.
 *  ret      history index of the completion, or LC_INF for :info/unterminated.
 *
 * :fail pairs are NOT passed (Knossos drops them).  Within a key the records
 * are sorted by strictly increasing `call`, with call < ret.  Indices need
 * only be monotone in history order; they may be global or key-local.
 */
typedef struct lc_op {
  int64_t f;
  int64_t value;
  int64_t expected;
  int64_t version;
  int64_t call;
  int64_t ret;
} lc_op;

/* Options (register.clj:111 initial model (->VersionedRegister 0 nil)). */
typedef struct lc_opts {
  int64_t init_version;        /* 0 */
  int64_t init_value;          /* LC_NIL */
  int64_t max_configs_per_key; /* <=0: library default; exceeding -> :unknown */
  int64_t time_budget_ms;      /* <=0: none; else a key whose frontier search runs longer
                                  than this is :unknown (LC_REASON_TIME_BUDGET) */
  int64_t flags;               /* LC_FLAG_* */
} lc_opts;

#define LC_FLAG_NO_HBM_RETRY 1  /* do not re-run LDS-overflowed keys from HBM */
#define LC_FLAG_NO_FAST_PATH 2  /* skip the version-order and gap tiers: JIT search for every key */
#define LC_FLAG_NO_GAP_TIER  4  /* skip the gap-matching tier: keys the version-order tier
                                   hands over go straight to the JIT search */
#define LC_FLAG_NO_TIMING   16  /* ABI 4, lc_check_device: no HIP events around the version-
                                   order pass (each costs ~2 us of host time per call); its
                                   time is then not measured (lc_last_stats 0, not counted
                                   by lc_last_totals) */
#define LC_FLAG_WHOLE_GPU    8  /* every entry point: a key the tiers leave :unknown at the
                                   configuration budget is searched again by the frontier
                                   exchange (include/lincheck_fx.h), whose budget bounds each
                                   return's configuration sets: with fewer such keys than the
                                   context has GPUs, each over ALL of them (one rank per GPU,
                                   RCCL all-to-all of the hash-partitioned frontier); else
                                   several keys at once, each over a whole GPU.  A failed
                                   re-search leaves that key :unknown (text in lc_last_error);
                                   the call still returns 0 */

/* Verdicts: Knossos :valid? true / false / :unknown. */
#define LC_VALID    1
#define LC_INVALID  0
#define LC_UNKNOWN (-1)

/* Reasons (lc_key_result.reason). */
#define LC_REASON_NONE            0
#define LC_REASON_NONLINEARIZABLE 1 /* frontier emptied at fail_op's return */
#define LC_REASON_CONFIG_BUDGET   2 /* max_configs_per_key exceeded  -> :unknown */
#define LC_REASON_WINDOW_OVERFLOW 3 /* > LC_MAX_WINDOW ops open at once -> :unknown */
#define LC_REASON_MALFORMED       4 /* record out of range / unsorted -> this key :unknown (the call
                                       still returns 0, as jepsen.independent loses only that key) */
#define LC_REASON_UNKNOWN_F       5 /* f not in {read,write,cas}: model throws (register.clj:63) -> :unknown */
#define LC_REASON_FRONTIER_LDS    6 /* internal: LDS tier overflowed (never returned when HBM retry runs) */
#define LC_REASON_TIME_BUDGET     7 /* lc_opts.time_budget_ms exceeded by the frontier search -> :unknown */

/* Largest number of simultaneously open (called, not yet returned, or
 * crashed-but-unlinearized) operations one key may have. */
#define LC_MAX_WINDOW 64

/*
 * Per-key result, 40 bytes.
 *  verdict          LC_VALID / LC_INVALID / LC_UNKNOWN
 *  reason           LC_REASON_*
 *  fail_op          for LC_INVALID: index (within the key's records) of the
 *                   :ok op whose return empties the configuration frontier —
 *                   the canonical minimal non-linearizable prefix; else -1.
 *  fail_prefix_end  for LC_INVALID: that op's `ret` (history index); else -1.
 *  configs_explored configurations generated by the search for this key
 *                   (version-order tier: 0; gap tier: matchings run).
 *  max_frontier     largest configuration set held between two events
 *                   (version-order tier: 1; gap tier: number of version gaps).
 */
typedef struct lc_key_result {
  int32_t verdict;
  int32_t reason;
  int64_t fail_op;
  int64_t fail_prefix_end;
  int64_t configs_explored;
  int64_t max_frontier;
} lc_key_result;

/* Statistics of the most recent lc_check / lc_check_device call. */
typedef struct lc_stats {
  double  kernel_ms;       /* device time of the fast + gap + JIT tiers (HIP events, summed over devices) */
  double  hbm_kernel_ms;   /* device time of the HBM-tier retry kernel(s) */
  double  total_ms;        /* host wall time of the call */
  int64_t n_keys;
  int64_t n_ops;
  int64_t n_hbm_keys;      /* keys re-run on the HBM tier */
  int64_t n_devices;
  double  fast_kernel_ms;  /* version-order tier (every key) */
  double  jit_kernel_ms;   /* JIT search tier (keys the fast tier handed over) */
  int64_t n_jit_keys;      /* keys decided by the JIT search */
  double  gap_kernel_ms;   /* gap-matching tier (keys the version-order tier handed over) */
  int64_t n_gap_keys;      /* keys the gap tier examined */
  int64_t n_malformed;     /* keys left :unknown with LC_REASON_MALFORMED */
} lc_stats;

/*
 * Optional outputs of lc_check_ex / lc_check_device_ex (NULL members are not
 * written; memory of the same kind as ops: host for lc_check_ex, device for
 * lc_check_device_ex).
 *
 *  witness       one int32 per record, indexed like ops.  For a key with
 *                witness_kind FULL: a linearization of the whole history —
 *                witness[r] = p >= 0 when record r is the p-th mutation
 *                (write / successful CAS, 0-based) of the linearization, -1
 *                when r is not linearized as a mutation (reads, which sit
 *                between the mutations their version names, and crashed ops
 *                left out).  For witness_kind PREFIX (invalid keys) the same
 *                for the history prefix at event fail_prefix_end - 1: ops
 *                called after it dropped, ops returning after it pending.
 *                Together with the verdict this certifies a decision: the
 *                order is checkable in O(n) by stepping the model
 *                (register.clj:60-96) and testing real-time order
 *                (tests/test_witness.py does exactly that, independently).
 *  witness_kind  one int32 per key, LC_WITNESS_*.
 */
typedef struct lc_aux {
  int32_t *witness;
  int32_t *witness_kind;
  int32_t *certificate;      /* ABI 3: 4 int32 per key, or NULL (needs witness_kind) */
  int32_t *certificate_set;  /* ABI 3: one int32 per record, indexed like ops, or NULL */
} lc_aux;

#define LC_WITNESS_NONE   0  /* no witness: decided by a search tier, or :unknown */
#define LC_WITNESS_FULL   1  /* valid key: a linearization of the whole history */
#define LC_WITNESS_PREFIX 2  /* invalid key: a linearization of the prefix just before the failing return */

/*
 * Infeasibility certificates (ABI 3).  The PREFIX witness shows that the
 * prefix just before an invalid key's failing return is linearizable; the
 * certificate shows that the prefix AT it is not, so together they certify
 * fail_op as the first failure (linearizability is prefix-closed).  For every
 * LC_INVALID key, certificate[4k .. 4k+3] = {kind, a, b, c}, a / b record
 * indices within the key.  The prefix P: records called at or before
 * fail_prefix_end; "required" = returned at or before it (the others pending,
 * free to be left out).  Mutation = write or CAS; its position = version -
 * init_version - 1.  Each kind names facts that no linearization of P can
 * satisfy together (register.clj:60-96 steps the version by one per
 * mutation, checks CAS expectations :77 and read claims :84-96):
 *   LC_CERT_DUP      a, b: two required mutations with the same version.
 *   LC_CERT_UNREACH  a: a required op whose version no linearization of P
 *                    reaches (a mutation at a version <= init_version, or
 *                    either kind beyond the number of mutations in P), or a
 *                    read of init_version whose value is not the initial one.
 *   LC_CERT_CLAIMS   a, b: two required reads of one version, different values.
 *   LC_CERT_PAIR     c = q: b consumes the value at position q-1 (a CAS
 *                    holding q: its expectation; a read of version init+q:
 *                    its value) and a holds position q-1 (a = -1: q = 0, the
 *                    initial value) with a different value; each of a, b is
 *                    required (and pinned there), or the only op of P that
 *                    can hold its (needed) position.
 *   LC_CERT_ORDER    a, b required: b returned before a was called, yet the
 *                    version order puts a's point before b's (a's lower-bound
 *                    index <= b's upper-bound index).
 *   LC_CERT_HALL     c positions, listed in certificate_set[key's first c
 *                    records]: each needed by a required op and held by none,
 *                    and fewer ops of P can hold any of them than c (Hall's
 *                    condition fails for the gap matching).
 *   LC_CERT_PROOF    (ABI 4) c tokens in certificate_set[0 .. c): a case
 *                    analysis over who holds the open positions (needed, no
 *                    required holder), for infeasibility only the gap
 *                    matching's branching finds.  certificate_set holds only
 *                    BRANCH tokens, in preorder: token = 2 << 30 | a << 15
 *                    | b — position a has exactly b ops able to hold it under
 *                    the choices so far, and b sub-proofs follow, one per op
 *                    in record order, each assuming that op holds a.  Forced
 *                    choices (a position with exactly one able op, which then
 *                    holds it) and closing positions (no able op) are NOT
 *                    written: a checker re-derives them by propagation before
 *                    each token, as oracle/cert.c proof_ok does, and rejects
 *                    a token whose position is forced or closed there.
 *                    "Able" is HALL's list of conditions, plus: an op chosen
 *                    at a+1 that is a CAS fixes the value a's holder writes,
 *                    one chosen at a-1 the value a CAS at a expects, and a
 *                    chosen op holds no other position.  Keys and positions
 *                    below 2^15.
 * LC_CERT_NONE: no certificate (valid or :unknown keys, keys only a search
 * decided where none of these applies).  oracle/cert.c checks them from
 * the records alone (tests/).
 */
#define LC_CERT_NONE    0
#define LC_CERT_DUP     1
#define LC_CERT_UNREACH 2
#define LC_CERT_CLAIMS  3
#define LC_CERT_PAIR    4
#define LC_CERT_ORDER   5
#define LC_CERT_HALL    6
#define LC_CERT_PROOF   7

typedef struct lc_ctx lc_ctx;

/* Open a context on the GPUs in device_mask (bit i = HIP device i).
 * device_mask == 0 selects every visible device.  Returns 0, or -ENODEV when
 * no requested GPU is usable (there is no CPU fallback).
 * The environment variable LC_VIRTUAL_DEVICES=k (k >= 2) opens k independent
 * device contexts (own stream and buffers) on the first selected GPU, so the
 * multi-device fan-out of lc_check can be exercised on a one-GPU machine. */
int lc_open(uint32_t device_mask, lc_ctx **out);

/* Check n_keys keys.  ops/key_off/out are host memory owned by the caller;
 * key k's records are ops[key_off[k] .. key_off[k+1]).  Synchronous.
 * Keys are partitioned over the context's GPUs in contiguous cost-balanced
 * ranges (lc_plan_partition).  Returns 0 (keys with malformed records are
 * :unknown with LC_REASON_MALFORMED; the others are decided), -EINVAL
 * (unusable arguments: null buffers, key_off not monotone, bad opts),
 * -ENOMEM, or -EIO (HIP failure); text in lc_last_error(). */
int lc_check(lc_ctx *ctx, const lc_op *ops, const int64_t *key_off,
             int64_t n_keys, const lc_opts *opts, lc_key_result *out);

/* lc_check plus the optional outputs of `aux` (may be NULL). */
int lc_check_ex(lc_ctx *ctx, const lc_op *ops, const int64_t *key_off,
                int64_t n_keys, const lc_opts *opts, lc_key_result *out,
                const lc_aux *aux);

/* Same, with ops / key_off / out already resident in device memory of the
 * context's first GPU; `stream` is a hipStream_t (NULL: the context's own).
 * Returns when every key is decided: d_out is complete for work ordered
 * after the call on `stream` (another stream reads it after synchronising
 * `stream`: a call that every key's version-order pass decided returns on
 * the pass's completion signal, a few microseconds before the kernel
 * retires; ABI 4). */
int lc_check_device(lc_ctx *ctx, const lc_op *d_ops, const int64_t *d_key_off,
                    int64_t n_keys, const lc_opts *opts,
                    lc_key_result *d_out, void *stream);

/* lc_check_device plus the optional outputs of `aux` (device pointers; the
 * lc_aux struct itself is host memory; may be NULL). */
int lc_check_device_ex(lc_ctx *ctx, const lc_op *d_ops, const int64_t *d_key_off,
                       int64_t n_keys, const lc_opts *opts, lc_key_result *d_out,
                       void *stream, const lc_aux *aux);

int lc_last_stats(lc_ctx *ctx, lc_stats *out);

/* ABI 4: sums over the calls since the last reset (reset != 0 zeroes them
 * after the read).  lc_check_device returns as soon as the version-order (or
 * fused) pass signals that every key is decided, before the kernel has
 * retired; the pass's HIP-event time is read afterwards — here, by
 * lc_last_stats, or at the next call — so a loop that times calls reads the
 * device time of all of them at once without waiting inside the loop. */
typedef struct lc_totals {
  int64_t calls;           /* run on the context's devices (one per device per call) */
  int64_t timed_calls;     /* those whose pass was timed (without LC_FLAG_NO_TIMING) */
  double fast_kernel_ms;   /* the version-order / fused pass (HIP events on the launch stream) */
  double kernel_ms;        /* every tier */
} lc_totals;

int lc_last_totals(lc_ctx *ctx, lc_totals *out, int32_t reset);

/* Per-device share of the most recent lc_check / lc_check_ex call (the
 * multi-GPU fan-out: one host thread and one HIP stream per device, each over
 * its contiguous cost-balanced key range, register.clj:108's independent
 * keys).  Device i of lc_stats.n_devices; -EINVAL past the last. */
typedef struct lc_device_stats {
  int32_t device;      /* HIP device id */
  int32_t pinned;      /* the records came from page-locked host memory (lc_host_register) */
  int64_t key_begin;   /* [key_begin, key_end) of the call's keys */
  int64_t key_end;
  int64_t h2d_bytes;   /* records + key offsets copied to the device */
  double  h2d_ms;      /* the host-to-device copies (HIP events on the device's stream) */
  double  kernel_ms;   /* the tiers (as lc_stats.kernel_ms, this device's) */
  double  total_ms;    /* host wall time of this device's thread, copies included */
} lc_device_stats;

int lc_last_device_stats(lc_ctx *ctx, int32_t i, lc_device_stats *out);

/* Page-lock a caller buffer that will be handed to lc_check repeatedly (a
 * JVM DirectByteBuffer / MemorySegment that outlives the call), so the
 * host-to-device copies of every GPU of the context DMA straight from it
 * instead of staging through the runtime's pageable-copy path (SURVEY.md
 * §8(b): "the library copies to device, or pins with hipHostRegister").
 * Registration costs about as much as one pageable copy of the buffer, so it
 * pays from the second call on.  Unregister before freeing the buffer.
 * Returns 0, -EINVAL, or -EIO (text in lc_last_error). */
int lc_host_register(lc_ctx *ctx, const void *ptr, uint64_t bytes);
int lc_host_unregister(lc_ctx *ctx, const void *ptr);

/*
 * ABI 4: the same op in 24 bytes.  The device reads every field of an lc_op
 * as int32 (key-relative 32-bit indices, int32 values and
 * versions), so half of the 48-byte record the JVM hands over crosses PCIe
 * for nothing.  lc_op32 carries exactly what the device reads:
 *
 *  f, value, expected, version   as in lc_op (int32; LC_NIL = -1)
 *  call, ret   history indices relative to the key's base (key_base[k],
 *              any int64; the key's first call when packed by lc_pack32);
 *              ret = LC_INF32 for :info / unterminated ops.
 *
 * Meaning: record r of key k stands for the lc_op
 *   {f, value, expected, version, key_base[k] + call,
 *    ret == LC_INF32 ? LC_INF : key_base[k] + ret}
 * (all int32 fields sign-extended, call/ret zero-extended; key_base NULL =
 * all zero), and lc_check32 returns exactly what lc_check returns for those
 * records — fail_prefix_end included, as an absolute history index.
 *
 * lc_pack32 narrows lc_op records key by key with the device's own rules, so
 * that lc_check32(lc_pack32(x)) == lc_check(x) field for field (witnesses and
 * certificates too):
 *   - key_base[k] = the key's first call, call/ret relative to it;
 *   - a version outside [-1, 2^31-2] (one no state can reach) becomes
 *     2^31-2, which no state reaches either (the device saturates it so);
 *   - an :f outside read/write/cas becomes 3 (unknown :f);
 *   - a record the device rejects as malformed (a value or expected id
 *     outside [-1, 2^31-2], call < 0, ret <= call, a key spanning 2^32-1 or
 *     more indices) gets value = -2, which keeps it malformed; its other
 *     fields are kept modulo 2^32, which is all the device reads of them.
 * A JVM (or any) packer may emit lc_op32 directly by the same rules (the
 * Clojure shim does: INTEGRATION.md §2).
 */
typedef struct lc_op32 {
  int32_t f;
  int32_t value;
  int32_t expected;
  int32_t version;
  uint32_t call;
  uint32_t ret;
} lc_op32;

#define LC_INF32 0xFFFFFFFFu

/* Narrow n_keys keys of lc_op records into out (indexed like ops: key k's
 * records are out[key_off[k] .. key_off[k+1])) and key_base (n_keys entries).
 * Host-only, multi-threaded for large batches; usable without a GPU.
 * Returns 0 or -EINVAL (null buffers, key_off not monotone). */
int lc_pack32(const lc_op *ops, const int64_t *key_off, int64_t n_keys, lc_op32 *out,
              int64_t *key_base);

/* lc_check_ex on 24-byte records from host memory (aux may be NULL; ops and
 * key_off indexed as in lc_check, key_base per key or NULL).  Each
 * device's key range is copied in chunks on a copy stream while the
 * version-order tier decides the chunks already copied. */
int lc_check32(lc_ctx *ctx, const lc_op32 *ops, const int64_t *key_off, const int64_t *key_base,
               int64_t n_keys, const lc_opts *opts, lc_key_result *out, const lc_aux *aux);

/* lc_check_device_ex on 24-byte records resident on the context's first GPU
 * (d_key_base may be NULL). */
int lc_check_device32(lc_ctx *ctx, const lc_op32 *d_ops, const int64_t *d_key_off,
                      const int64_t *d_key_base, int64_t n_keys, const lc_opts *opts,
                      lc_key_result *d_out, void *stream, const lc_aux *aux);

/*
 * ABI 5: the same op in 16 bytes, for batches whose value ids fit
 * 15 bits — the drop-in's host-to-device copy is PCIe-bound, and every value
 * a key's history holds is interned per key to a small dense id:
 *
 *  fve       f << 30 | (value + 1) << 15 | (expected + 1): 2 + 15 + 15 bits;
 *            value / expected ids in [-1, LC_ID15_MAX] (nil = -1 -> 0); a
 *            value field of 0x7FFF marks a record lc_pack32 would mark
 *            malformed (value -2)
 *  version   as in lc_op32 (int32)
 *  call, ret as in lc_op32 (relative to key_base[k]; LC_INF32: no return)
 *
 * Record r of key k stands for the lc_op32
 *   {fve >> 30, v - 1 (v = fve >> 15 & 0x7FFF; 0x7FFF: -2),
 *    (fve & 0x7FFF) - 1 (0x7FFF: -2), version, call, ret}
 * and lc_check16 returns exactly what lc_check32 returns for those records
 * (and so what lc_check returns for the records lc_pack16 was given).
 * lc_pack16 narrows lc_op records by lc_pack32's rules, or returns -ERANGE
 * (nothing written that the caller may use) when a record that is not
 * malformed holds a value or expected id above LC_ID15_MAX: such a batch
 * goes as lc_op32.
 */
typedef struct lc_op16 {
  uint32_t fve;
  int32_t version;
  uint32_t call;
  uint32_t ret;
} lc_op16;

#define LC_ID15_MAX 0x7FFD

int lc_pack16(const lc_op *ops, const int64_t *key_off, int64_t n_keys, lc_op16 *out,
              int64_t *key_base);

/* lc_check_ex on 16-byte records from host memory (as lc_check32: chunked
 * copies on the copy streams; each chunk widened on the device and decided
 * while the next one crosses PCIe). */
int lc_check16(lc_ctx *ctx, const lc_op16 *ops, const int64_t *key_off, const int64_t *key_base,
               int64_t n_keys, const lc_opts *opts, lc_key_result *out, const lc_aux *aux);

/* Where the host wall time of the last lc_check / lc_check_ex / lc_check32
 * call went (ABI 4): the argument checks, the split over devices, the start
 * of the per-device threads, their ends, the frontier-exchange re-search
 * (LC_FLAG_WHOLE_GPU), all as milliseconds since the call began. */
typedef struct lc_call_profile {
  double total_ms;          /* the whole call */
  double checked_ms;        /* arguments checked, options converted */
  double planned_ms;        /* keys split over the devices (plan_devices) */
  double first_start_ms;    /* first per-device thread running */
  double last_start_ms;     /* last per-device thread running */
  double first_end_ms;      /* first per-device thread done (results copied back) */
  double last_end_ms;       /* last per-device thread done */
  double joined_ms;         /* every thread joined, statistics summed */
  double whole_gpu_ms;      /* LC_FLAG_WHOLE_GPU re-search done (= joined_ms without it) */
  int64_t n_devices;
  int64_t n_chunks;         /* host-to-device chunks issued over all devices */
} lc_call_profile;

int lc_last_call_profile(lc_ctx *ctx, lc_call_profile *out);

/* ABI 5: lc_check_device on a batch of at most one key per resident
 * workgroup (1,536 on an MI355X) is served by a version-order grid that
 * stays resident on the GPU between calls (no launch per call); it leaves on
 * its own after LC_RESIDENT_IDLE_US microseconds (default 50) without a
 * call, before any other work of the context runs on that GPU, and at
 * lc_close.  lc_quiesce stops it now (a caller that is done calling, or
 * wants the GPU to itself); the next call launches it again.  Returns 0, or
 * -EIO.  LC_RESIDENT=0 in the environment disables the resident grid. */
int lc_quiesce(lc_ctx *ctx);

const char *lc_last_error(lc_ctx *ctx);
void lc_close(lc_ctx *ctx);

/* Default options (init state (0, nil)). */
void lc_default_opts(lc_opts *out);

/* Contiguous cost-balanced partition of keys over n_parts workers (the
 * static multi-GPU split).  Writes n_parts+1 key boundaries
 * to bounds.  With ops, each key is priced by the tier that will decide it
 * (lc_key_cost); with ops == NULL by its record count.  Host-only; usable
 * without a GPU. */
int lc_plan_partition(const lc_op *ops, const int64_t *key_off, int64_t n_keys,
                      int32_t n_parts, int64_t *bounds);

/* Estimated device cost of each key, in record-scan units (a record the
 * version-order tier decides costs 1).  Calibrated from measured tier times
 * (DESIGN.md §7): a key with crashed writes/CAS goes to the gap tier, one
 * with version-less :ok mutations to the frontier search, whose cost grows
 * with the number of concurrently open ops and crashed ops.  costs[n_keys]. */
int lc_key_cost(const lc_op *ops, const int64_t *key_off, int64_t n_keys, double *costs);

int lc_abi_version(void);

/* Hash of the sources the library was built from (hex string); callers that
 * build the library from a source tree compare it against the tree's own
 * hash to refuse a stale binary. */
const char *lc_build_id(void);

#ifdef __cplusplus
}
#endif

#endif /* LINCHECK_H */
