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

#define LC_ABI_VERSION 1

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

/* Verdicts: Knossos :valid? true / false / :unknown. */
#define LC_VALID    1
#define LC_INVALID  0
#define LC_UNKNOWN (-1)

/* Reasons (lc_key_result.reason). */
#define LC_REASON_NONE            0
#define LC_REASON_NONLINEARIZABLE 1 /* frontier emptied at fail_op's return */
#define LC_REASON_CONFIG_BUDGET   2 /* max_configs_per_key exceeded  -> :unknown */
#define LC_REASON_WINDOW_OVERFLOW 3 /* > LC_MAX_WINDOW ops open at once -> :unknown */
#define LC_REASON_MALFORMED       4 /* record out of range / unsorted -> :unknown, call returns -EINVAL */
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
} lc_stats;

typedef struct lc_ctx lc_ctx;

/* Open a context on the GPUs in device_mask (bit i = HIP device i).
 * device_mask == 0 selects every visible device.  Returns 0, or -ENODEV when
 * no requested GPU is usable (there is no CPU fallback). */
int lc_open(uint32_t device_mask, lc_ctx **out);

/* Check n_keys keys.  ops/key_off/out are host memory owned by the caller;
 * key k's records are ops[key_off[k] .. key_off[k+1]).  Synchronous.
 * Keys are partitioned over the context's GPUs in contiguous cost-balanced
 * ranges.  Returns 0, -EINVAL (malformed input; per-key reasons are still
 * written), -ENOMEM, or -EIO (HIP failure); text in lc_last_error(). */
int lc_check(lc_ctx *ctx, const lc_op *ops, const int64_t *key_off,
             int64_t n_keys, const lc_opts *opts, lc_key_result *out);

/* Same, with ops / key_off / out already resident in device memory of the
 * context's first GPU; `stream` is a hipStream_t (NULL: the context's own).
 * Synchronous with respect to the host. */
int lc_check_device(lc_ctx *ctx, const lc_op *d_ops, const int64_t *d_key_off,
                    int64_t n_keys, const lc_opts *opts,
                    lc_key_result *d_out, void *stream);

int lc_last_stats(lc_ctx *ctx, lc_stats *out);
const char *lc_last_error(lc_ctx *ctx);
void lc_close(lc_ctx *ctx);

/* Default options (init state (0, nil)). */
void lc_default_opts(lc_opts *out);

/* Contiguous cost-balanced partition of keys over n_parts workers (the
 * static multi-GPU split).  Writes n_parts+1 key boundaries to bounds.
 * Host-only; usable without a GPU. */
int lc_plan_partition(const lc_op *ops, const int64_t *key_off, int64_t n_keys,
                      int32_t n_parts, int64_t *bounds);

int lc_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* LINCHECK_H */
