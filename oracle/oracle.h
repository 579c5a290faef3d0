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

/* Check every key with the chosen algorithm on n_threads host threads.
 * Same record format, options and result struct as lc_check().
 * JIT reports the canonical fail op; WGL reports verdicts only (fail_op -1).
 * Returns 0 or -EINVAL (malformed key; reason LC_REASON_MALFORMED). */
int oracle_check(const lc_op *ops, const int64_t *key_off, int64_t n_keys,
                 const lc_opts *opts, lc_key_result *out, int algo,
                 int n_threads);

/* The VersionedRegister step (register.clj:60-96) on int64 fields.
 * Returns 1 and writes the next state if legal, 0 if inconsistent,
 * -1 for an unknown f (the reference's condp has no default, :63). */
int oracle_step(int64_t ver, int64_t val, const lc_op *op,
                int64_t *nver, int64_t *nval);

#ifdef __cplusplus
}
#endif

#endif
