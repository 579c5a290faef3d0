/*
 * lincheck_synth.h — seeded synthetic `register` histories.
 *
 * Simulates, per independent key, the workload of
 *   /root/reference/src/jepsen/etcd/register.clj:113-119
 * (2n worker processes per key, n of them read-only via gen/reserve, the rest
 * gen/mix [w cas] with values uniform in 0..4, register.clj:98-100) against a
 * linearizable etcd-like register that tracks the per-key version
 * (register.clj:30-43: ok write/cas report prev-version+1; a CAS whose old
 * value mismatches is :fail, :44).  Every op gets a linearization point inside
 * [call, ret], so un-injected histories are linearizable by construction.
 * Crashed writes/CAS become :info (ret = LC_INF) and take effect with p = 0.5;
 * the crashed process is replaced by a fresh one (Jepsen process semantics).
 *
 * With info_frac, the crash count is made exact (see lc_synth_params).
 *
 * Anomalies (p_anomaly per key): a stale read (a read reports the state before
 * a mutation that returned before the read was invoked) or a lost CAS (a CAS
 * reported :ok whose effect never reaches the register).
 */
#ifndef LINCHECK_SYNTH_H
#define LINCHECK_SYNTH_H

#include <stdint.h>

#include "lincheck.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct lc_synth_params {
  int64_t  n_keys;
  int64_t  ops_per_key;  /* exact packed (non-:fail) records per key */
  int32_t  concurrency;  /* processes per key (reference: 2n = 10) */
  int32_t  n_values;     /* value domain (reference: 5) */
  double   p_info;       /* P(a write/cas crashes -> :info) */
  double   p_anomaly;    /* P(a key gets one injected anomaly) */
  uint64_t seed;
  double   info_frac;    /* > 0: exactly round(info_frac * ops_per_key) of a key's
                            records are crashed writes/CAS (BASELINE configs[3]:
                            20 %).  After the p_info crashes, uniformly chosen :ok
                            writes/CAS are reported :info instead (a client timeout
                            on an op that took effect; its process is replaced),
                            which keeps the history linearizable.  0: off. */
} lc_synth_params;

/* Labels written per key by lc_synth_register. */
#define LC_SYNTH_CLEAN      0
#define LC_SYNTH_STALE_READ 1
#define LC_SYNTH_LOST_CAS   2

/* Status of an op in lc_synth_key's full stream. */
#define LC_SYNTH_FAIL 0
#define LC_SYNTH_OK   1
#define LC_SYNTH_INFO 2

/* All keys, packed records only (:fail pairs dropped, as the checker's host
 * preprocessing does).  ops holds n_keys*ops_per_key records, key_off
 * n_keys+1 offsets; labels (n_keys) and n_invocations (total invocations,
 * :fail included) may be NULL.  Deterministic in (params, key) regardless of
 * n_threads.  Returns 0 or -EINVAL. */
int lc_synth_register(const lc_synth_params *p, lc_op *ops, int64_t *key_off,
                      int32_t *labels, int64_t *n_invocations, int n_threads);

/* One key's full stream including :fail ops (sorted by call), with the
 * Jepsen process id and status of each op.  *n_out receives the count; if it
 * exceeds cap nothing is written and -ENOSPC is returned. */
int lc_synth_key(const lc_synth_params *p, int64_t key, lc_op *ops,
                 int32_t *proc, int32_t *status, int64_t cap, int64_t *n_out,
                 int32_t *label);

#ifdef __cplusplus
}
#endif

#endif
