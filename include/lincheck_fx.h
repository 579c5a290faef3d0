/*
 * lincheck_fx.h — frontier exchange: ONE oversized key's JIT frontier search
 * spread over a whole GPU, and over several GPUs by hash ownership.
 *
 * SURVEY.md §8(e), "the one exception": a key too large for one workgroup of
 * the HBM tier (lincheck.h) — a version-less model (cas-register, register,
 * mutex: lock.clj:244) with a long, highly concurrent history, where knossos'
 * search (knossos.linear, called through checker/linearizable at
 * register.clj:110-111) holds frontiers of 10^5..10^7 configurations.
 *
 * The search is knossos.linear's (Lowe's JIT linearization) with the exact
 * reductions of the other tiers (eager read closure, deadline order,
 * retirement: DESIGN.md §4), restated by the oracle as JITC; on every key
 * the verdict, the canonical fail op, the configurations explored and the
 * largest frontier equal the oracle's.  A return's expansion is level-
 * synchronous over the whole device: every wave takes configurations of the
 * current level, generates their successors (lane = window slot) and
 * inserts them into open-addressed device tables.
 *
 * Over n ranks each configuration is owned by hash(configuration) mod n (a
 * Zobrist hash over every op it has linearized, retired ones included, so
 * retirement never moves a configuration).  While the frontier holds more
 * than `part_above` configurations it is partitioned: each rank expands the
 * configurations it owns and sends every successor to its owner (counts
 * first, then payload: an all-to-all-v), and a small sum-reduction per level
 * detects the end of the level.  Below `repl_below` the frontier is
 * gathered back and every rank holds (and expands) all of it, with no
 * traffic.
 *
 * Collectives, three ways:
 *  - native RCCL (librccl, loaded at run time): lc_fx_open_devices runs one
 *    rank per listed GPU of this process, each on a host thread of its own,
 *    over communicators from ncclCommInitAll; lc_fx_open_rccl makes this
 *    process one rank of a multi-process search (ncclCommInitRank, the id
 *    from lc_fx_rccl_unique_id passed around by the caller).  Counts are
 *    exchanged on the device (ncclAllToAll), configurations by grouped
 *    ncclSend / ncclRecv straight from the per-owner regions on the engine's
 *    stream, reductions by ncclAllReduce.  lincheck.h's LC_FLAG_WHOLE_GPU uses
 *    lc_fx_open_devices over every GPU of the lc_ctx;
 *  - the caller's callbacks (`lc_fx_transport`; jepsen/etcd_amd/fx.py's
 *    TorchTransport implements them with torch.distributed);
 *  - transport == NULL and virtual_ranks = k: k ranks as threads on one
 *    device with an in-process transport (device copies), so the partitioned
 *    path is testable on one GPU.
 *
 * Plain C types only.
 */
#ifndef LINCHECK_FX_H
#define LINCHECK_FX_H

#include <stdint.h>

#include "lincheck.h"

#ifdef __cplusplus
extern "C" {
#endif

#define LC_FX_SUM 0
#define LC_FX_MAX 1

/* Collectives over the ranks of one search.  Every callback is called by
 * every rank in the same order; each returns 0 or a negative error.
 *  exchange_counts  send[j] = entries this rank sends to rank j; fills
 *                   recv[j] = entries rank j sends to this rank (n_ranks each).
 *  alltoallv        d_send (device memory) holds this rank's entries grouped
 *                   by destination rank, send_counts[j] of them for rank j;
 *                   writes the entries received, grouped by source rank, to
 *                   d_recv (device, room for the sum of recv_counts).
 *  allreduce        in-place element-wise reduction (LC_FX_SUM / LC_FX_MAX)
 *                   of n int64 values in host memory. */
typedef struct lc_fx_transport {
  void *user;
  int32_t rank;
  int32_t n_ranks;
  int (*exchange_counts)(void *user, const int64_t *send, int64_t *recv);
  int (*alltoallv)(void *user, const void *d_send, const int64_t *send_counts,
                   void *d_recv, const int64_t *recv_counts, int64_t entry_bytes);
  int (*allreduce)(void *user, int64_t *vals, int32_t n, int32_t op);
} lc_fx_transport;

typedef struct lc_fx_params {
  int32_t device;         /* HIP device ordinal */
  int32_t virtual_ranks;  /* transport == NULL: ranks run as threads on `device` (>= 1) */
  int64_t part_above;     /* partition while the frontier exceeds this (< 0: default 65536) */
  int64_t repl_below;     /* replicate again below this (< 0: default part_above / 4) */
  int64_t table_log2;     /* log2 of each dedup table's entries (0: from the budget) */
  int64_t flags;          /* LC_FX_FLAG_* */
} lc_fx_params;

/* Always use the 16-byte-key tables (epoch tags, fenced publication) instead
 * of one-word entries: for tests of that path. */
#define LC_FX_FLAG_WIDE_TABLES 1
/* Run the multi-rank protocol even with one rank, and send each rank's own
 * configurations through the exchange like every other owner's: with one
 * rank on a one-device RCCL communicator every configuration then moves
 * through ncclSend / ncclRecv to itself (tests of the transport on a one-GPU
 * machine; RCCL refuses two ranks on one device). */
#define LC_FX_FLAG_EXCHANGE_SELF 2

typedef struct lc_fx_stats {
  double  total_ms;         /* host wall time of the last lc_fx_check */
  int64_t returns;          /* :ok returns whose frontier was expanded */
  int64_t levels;           /* BFS levels run (replicated + partitioned) */
  int64_t part_returns;     /* returns expanded with the frontier partitioned */
  int64_t part_levels;      /* levels run partitioned (one exchange each) */
  int64_t sent_configs;     /* configurations this rank sent to other ranks (and to itself,
                               with LC_FX_FLAG_EXCHANGE_SELF) */
  int64_t gathers;          /* partitioned -> replicated switches */
  int64_t max_local_frontier; /* largest frontier share held by this rank */
  int64_t redos;            /* returns redone with a larger dedup table */
  int64_t wide_returns;     /* returns on 16-byte-key tables (an open slot at or above 64 minus the
                               key's value-id bits, over 2^20 - 1 values, or LC_FX_FLAG_WIDE_TABLES) */
} lc_fx_stats;

typedef struct lc_fx lc_fx;

/* Open an engine.  transport == NULL: params->virtual_ranks in-process ranks.
 * Returns 0, -EINVAL, -ENODEV, -ENOMEM or -EIO (text in lc_fx_last_error). */
int lc_fx_open(const lc_fx_params *params, const lc_fx_transport *transport, lc_fx **out);

/* One engine over the GPUs devices[0 .. n_devices) of this process: rank i
 * on devices[i] (distinct devices; RCCL refuses two ranks on one), one host
 * thread per rank inside lc_fx_check.  -ENOSYS without a loadable librccl,
 * -EINVAL for a list RCCL rejects (duplicates). */
int lc_fx_open_devices(const lc_fx_params *params, const int32_t *devices, int32_t n_devices,
                       lc_fx **out);

/* Multi-process RCCL: rank 0 makes an id, every rank opens with it (params->
 * device = this process's GPU).  ncclGetUniqueId / ncclCommInitRank. */
#define LC_FX_RCCL_ID_BYTES 128
int lc_fx_rccl_unique_id(uint8_t *id /* LC_FX_RCCL_ID_BYTES */);
int lc_fx_open_rccl(const lc_fx_params *params, const uint8_t *id, int32_t rank, int32_t n_ranks,
                    lc_fx **out);

/* Decide one key: ops[0..n) are its records (lincheck.h layout, host memory,
 * sorted by call).  Every rank calls it with the same key.  `out` gets the
 * same result lc_check gives (verdict, reason, fail_op, fail_prefix_end,
 * configs_explored, max_frontier), identical on every rank.  Keys with more
 * than LC_MAX_WINDOW open ops are :unknown (LC_REASON_WINDOW_OVERFLOW). */
int lc_fx_check(lc_fx *fx, const lc_op *ops, int64_t n, const lc_opts *opts,
                lc_key_result *out);

/* One configuration of a key's search frontier — knossos's `:configs` entry
 * (`{:model (->VersionedRegister version value), :pending [...]}`,
 * register.clj:55, checker/linearizable's result at register.clj:110-111):
 * the model state and the ops (record indices of the key) that have been
 * called but are not linearized in it.  Ops linearized in every
 * configuration are retired and never pending; reads that can never
 * constrain (crashed, [nil nil]) take no part in the search. */
typedef struct lc_fx_config {
  int64_t version;
  int64_t value;        /* the caller's value id; LC_NIL for nil */
  int64_t n_pending;
  int64_t pending[64];  /* sorted */
} lc_fx_config;

/* Run the key's search up to the :ok return of record stop_op and copy up
 * to `max` configurations of the frontier that return expands — for an
 * invalid key with fail_op = stop_op, the configurations just before the
 * failure, which knossos reports as :configs.  One-rank engines only.
 * *n_out = configurations copied (0 when stop_op's return is a no-op: the op
 * was retired). */
int lc_fx_frontier(lc_fx *fx, const lc_op *ops, int64_t n, const lc_opts *opts, int64_t stop_op,
                   lc_fx_config *out, int32_t max, int32_t *n_out);

/* ABI 4: the same for many keys in one call on an lc_check context (its
 * first GPU).  Key k (records ops[key_off[k] .. key_off[k+1]), host memory)
 * is searched on the device — one wavefront per key, the JIT search of the
 * LDS tier, the same reductions as the frontier exchange — up to the :ok
 * return of its record stop_op[k], and up to max_per_key configurations of
 * the frontier that return expands go to out[k * max_per_key ...]:
 * knossos's :configs of an invalid key whose stop_op is its fail_op
 * (register.clj:110-111).  n_out[k] = configurations copied; 0 when
 * stop_op's return is a no-op (the op was retired); -1 when the search could
 * not get there on the LDS tier (a frontier beyond 128 configurations, more
 * than LC_MAX_WINDOW open ops, the budget, an earlier failure, a stop_op that
 * is not an :ok op): lc_fx_frontier decides those one by one.  Returns 0,
 * -EINVAL, -ENOMEM or -EIO. */
int lc_check_frontiers(lc_ctx *ctx, const lc_op *ops, const int64_t *key_off, int64_t n_keys,
                       const int64_t *stop_op, const lc_opts *opts, lc_fx_config *out,
                       int32_t max_per_key, int32_t *n_out);

/* From another thread: stop a search in progress.  Every RCCL communicator
 * of the engine is aborted (ncclCommAbort), so ranks waiting in a collective
 * return and lc_fx_check fails; an RCCL engine is unusable afterwards.  For
 * in-process ranks the hub is aborted.  A watchdog's way out of a hang. */
void lc_fx_abort(lc_fx *fx);

int lc_fx_last_stats(lc_fx *fx, lc_fx_stats *out);   /* rank 0's (or this rank's) */
const char *lc_fx_last_error(lc_fx *fx);
void lc_fx_close(lc_fx *fx);

#ifdef __cplusplus
}
#endif

#endif /* LINCHECK_FX_H */
