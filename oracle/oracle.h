/*
 * oracle.h — CPU restatement of the reference's linearizability check for the
 * `register` workload.  TEST INFRASTRUCTURE ONLY: tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg are the only permitted users.  The product
 * path (jepsen/etcd_amd) never links or calls this.
 *
 * Parity status: the reference's hot path is Clojure (register.clj) running on
 * Knossos (a JVM dependency, not in /root/reference, pulled in by
 * [jepsen "0.3.3-SNAPSHOT"] at project.clj:7).  No JVM exists in this image, so
 * the reference cannot be run here, and the reference holds no tests, golden
 * histories or fixtures for this path.  This oracle is
 * therefore pinned only by hand-derived known-answer histories
 * (tests/golden/kat.json, from the step semantics at register.clj:60-96) and by
 * agreement of three independent algorithms (brute force, JIT-linear, WGL):
 * PARITY UNPINNED against outputs of the reference itself.
 */
#ifndef LC_ORACLE_H
#define LC_ORACLE_H

#include "../include/lincheck.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ORACLE_JIT 0  /* knossos.linear (Lowe's just-in-time linearization) */
#define ORACLE_WGL 1  /* knossos.wgl (Wing-Gong with Lowe's cache)          */
/* OR into algo with ORACLE_JIT: exact reductions (see oracle.c); tests/
 * check each against the faithful mode. */
#define ORACLE_FLAG_READ_CLOSURE   0x100
#define ORACLE_FLAG_CRASH_SYMMETRY 0x200
#define ORACLE_FLAG_RETIRE         0x400
#define ORACLE_FLAG_DEADLINE_ORDER 0x800

/* Check every key with the chosen algorithm on n_threads host threads.
 * Same record format, options and result struct as lc_check().
 * JIT reports the canonical fail op; WGL reports verdicts only (fail_op -1).
 * Returns 0 or -EINVAL (malformed key; reason LC_REASON_MALFORMED). */
int oracle_check(const lc_op *ops, const int64_t *key_off, int64_t n_keys,
                 const lc_opts *opts, lc_key_result *out, int algo,
                 int n_threads);

/* The JIT search (algo = ORACLE_JIT | reductions) of one key, stopped at the
 * :ok return of record stop_op: the frontier that return expands, up to max
 * configurations of ORACLE_CFG_WORDS int64 each — version, value, number of
 * pending ops, then the pending ops (record indices, sorted; at most 64).
 * *n_out = the frontier's size (0 when stop_op's return is a no-op). */
#define ORACLE_CFG_WORDS 67
int oracle_frontier(const lc_op *ops, int64_t n, const lc_opts *opts, int algo,
                    int64_t stop_op, int64_t *out, int64_t max, int64_t *n_out);

/* The VersionedRegister step (register.clj:60-96) on int64 fields.
 * Returns 1 and writes the next state if legal, 0 if inconsistent,
 * -1 for an unknown f (the reference's condp has no default, :63). */
int oracle_step(int64_t ver, int64_t val, const lc_op *op,
                int64_t *nver, int64_t *nval);

/* Witness certification (witness.c): rebuild the total order a witness
 * (lc_aux, include/lincheck.h) names and check it against the definition —
 * every :ok op present, model steps legal (oracle_step), real-time order
 * respected.  Per key status: ORACLE_WIT_OK, ORACLE_WIT_NONE (kind NONE), or
 * a negative ORACLE_WIT_* code.  cut[k] is the prefix end for kind PREFIX
 * (fail_prefix_end - 1; may be NULL when no key has that kind).  order_len
 * (may be NULL) receives the length of each rebuilt order. */
#define ORACLE_WIT_OK                 1
#define ORACLE_WIT_NONE               0
#define ORACLE_WIT_BAD_POSITION     (-1) /* positions not exactly 0..m-1, once each */
#define ORACLE_WIT_NOT_AN_OP        (-2) /* a position on a read / an op after the cut / unknown f */
#define ORACLE_WIT_READ_UNPLACEABLE (-3) /* a read's version names no segment of the order */
#define ORACLE_WIT_INCONSISTENT     (-4) /* the model rejects an op of the order */
#define ORACLE_WIT_REAL_TIME        (-5) /* an op ordered after one called after it returned */
#define ORACLE_WIT_MISSING_OK_OP    (-6) /* an :ok write/CAS left out */
int oracle_check_witness(const lc_op *ops, const int64_t *key_off, int64_t n_keys,
                         const lc_opts *opts, const int32_t *witness, const int32_t *kind,
                         const int64_t *cut, int32_t *status, int64_t *order_len,
                         int n_threads);

/* Infeasibility certificates (cert.c): check each key's certificate
 * (lc_aux.certificate, 4 int32 per key; certificate_set, per record) against
 * the prefix at cut[k] (fail_prefix_end) from the records alone.  Per key
 * ORACLE_CERT_OK, ORACLE_CERT_NONE (kind LC_CERT_NONE) or ORACLE_CERT_BAD
 * (the facts named do not rule out every linearization). */
#define ORACLE_CERT_OK    1
#define ORACLE_CERT_NONE  0
#define ORACLE_CERT_BAD (-1)
int oracle_check_certificate(const lc_op *ops, const int64_t *key_off, int64_t n_keys,
                             const lc_opts *opts, const int32_t *cert, const int32_t *cert_set,
                             const int64_t *cut, int32_t *status, int n_threads);

#ifdef __cplusplus
}
#endif

#endif
