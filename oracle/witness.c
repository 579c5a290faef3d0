/*
 * witness.c — independent certification of the GPU's decisions from their
 * witnesses (lc_aux, include/lincheck.h).  TEST INFRASTRUCTURE ONLY (see
 * oracle.h for who may use it).
 *
 * A witness names, for every record, its mutation position in a claimed
 * linearization (or -1).  This file turns it into one total order of the
 * (prefix) history's ops and checks that order against the definition the
 * verdicts stand on ("parity-critical definition"):
 *   - it holds every op that completed :ok, and only ops of the history;
 *   - stepping the model from the initial state through it never becomes
 *     inconsistent: oracle_step, the restatement of register.clj:60-96;
 *   - it respects real time: no op comes after an op that was called after
 *     it returned (ret(b) < call(a) with a before b is a violation).
 * The check is O(n log n) per key and shares nothing with the device code
 * that produced the witness: a wrong witness fails here, whatever produced it.
 *
 * Reads are not named by the witness: a read whose version is v sits between
 * the (v - V0)-th and the (v - V0 + 1)-th mutation; among the reads of one
 * such segment the order is by return (which respects real time among them);
 * a read with no version goes to the earliest segment after every placed op
 * that returned before it was called (and, with a value, whose value it
 * reads).  Any order this builds is still checked in full above, so the
 * placement rules can only make a correct witness fail, never a wrong one
 * pass.
 */
#include <errno.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef struct {
  int64_t k1, k2, k3;
  int64_t rec;
} ord_t;

static int ord_cmp(const void *a, const void *b) {
  const ord_t *x = (const ord_t *)a, *y = (const ord_t *)b;
  if (x->k1 != y->k1) return x->k1 < y->k1 ? -1 : 1;
  if (x->k2 != y->k2) return x->k2 < y->k2 ? -1 : 1;
  if (x->k3 != y->k3) return x->k3 < y->k3 ? -1 : 1;
  return 0;
}

typedef struct {
  int64_t ret;
  int64_t seg;  /* segment an op returning at `ret` forces later ops into */
} done_t;

static int done_cmp(const void *a, const void *b) {
  const done_t *x = (const done_t *)a, *y = (const done_t *)b;
  return x->ret < y->ret ? -1 : x->ret > y->ret;
}

/* One key.  Returns ORACLE_WIT_OK or a negative ORACLE_WIT_* code. */
static int check_key(const lc_op *o, int64_t n, const int32_t *wit, int64_t cut,
                     int64_t V0, int64_t init, int64_t *order_len) {
  int rc = ORACLE_WIT_OK;
  int64_t m = 0;
  for (int64_t i = 0; i < n; i++)
    if (wit[i] >= 0) m++;
  int64_t *mut = (int64_t *)malloc(sizeof(int64_t) * (size_t)(m + 1));
  int64_t *segval = (int64_t *)malloc(sizeof(int64_t) * (size_t)(m + 1));
  ord_t *ord = (ord_t *)malloc(sizeof(ord_t) * (size_t)(n + 1));
  done_t *done = (done_t *)malloc(sizeof(done_t) * (size_t)(n + 1));
  int64_t *rseg = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n + 1));
  if (!mut || !segval || !ord || !done || !rseg) {
    rc = -ENOMEM;
    goto out;
  }
  for (int64_t p = 0; p < m; p++) mut[p] = -1;
  /* mutations: positions 0..m-1, each held once, by an op of the prefix */
  for (int64_t i = 0; i < n; i++) {
    if (wit[i] < -1) { rc = ORACLE_WIT_BAD_POSITION; goto out; }
    if (wit[i] < 0) continue;
    if (wit[i] >= m || mut[wit[i]] != -1) { rc = ORACLE_WIT_BAD_POSITION; goto out; }
    if (o[i].call > cut || (o[i].f != LC_F_WRITE && o[i].f != LC_F_CAS)) {
      rc = ORACLE_WIT_NOT_AN_OP;
      goto out;
    }
    mut[wit[i]] = i;
  }
  /* the value in each segment (after p mutations), for value-only reads */
  segval[0] = init;
  for (int64_t p = 0; p < m; p++) segval[p + 1] = o[mut[p]].value;
  /* every :ok op of the prefix must be in the order */
  int64_t nd = 0;
  for (int64_t i = 0; i < n; i++) {
    rseg[i] = -1;
    if (o[i].call > cut) continue;
    const int64_t ret = o[i].ret <= cut ? o[i].ret : LC_INF;
    if (o[i].f == LC_F_READ) {
      if (ret == LC_INF) continue;  /* a pending read may be left out */
      if (o[i].version != LC_NIL) {
        const int64_t s = o[i].version - V0;
        if (s < 0 || s > m) { rc = ORACLE_WIT_READ_UNPLACEABLE; goto out; }
        rseg[i] = s;
        done[nd].ret = ret;
        done[nd].seg = s;
        nd++;
      }
    } else if (o[i].f == LC_F_WRITE || o[i].f == LC_F_CAS) {
      if (wit[i] < 0) {
        if (ret != LC_INF) { rc = ORACLE_WIT_MISSING_OK_OP; goto out; }
        continue;
      }
      if (ret != LC_INF) {
        done[nd].ret = ret;
        done[nd].seg = wit[i] + 1;
        nd++;
      }
    } else if (ret != LC_INF) {
      rc = ORACLE_WIT_NOT_AN_OP; /* an :ok op the model cannot step (register.clj:63) */
      goto out;
    }
  }
  /* version-less reads: after everything that returned before their call */
  qsort(done, (size_t)nd, sizeof(done_t), done_cmp);
  for (int64_t j = 1; j < nd; j++)
    if (done[j].seg < done[j - 1].seg) done[j].seg = done[j - 1].seg;
  for (int64_t i = 0; i < n; i++) {
    if (o[i].f != LC_F_READ || o[i].call > cut || o[i].ret > cut || o[i].version != LC_NIL)
      continue;
    int64_t lo = 0, hi = nd; /* first done with ret >= call */
    while (lo < hi) {
      const int64_t mid = (lo + hi) / 2;
      if (done[mid].ret < o[i].call) lo = mid + 1; else hi = mid;
    }
    int64_t s = lo > 0 ? done[lo - 1].seg : 0;
    if (o[i].value != LC_NIL)
      while (s <= m && segval[s] != o[i].value) s++;
    if (s > m) { rc = ORACLE_WIT_READ_UNPLACEABLE; goto out; }
    rseg[i] = s;
  }
  /* the total order: slot 2p+1 = mutation p, slot 2s = reads of segment s
   * (by return, then record) */
  int64_t len = 0;
  for (int64_t p = 0; p < m; p++) {
    ord[len].k1 = 2 * p + 1;
    ord[len].k2 = 0;
    ord[len].k3 = 0;
    ord[len].rec = mut[p];
    len++;
  }
  for (int64_t i = 0; i < n; i++)
    if (rseg[i] >= 0) {
      ord[len].k1 = 2 * rseg[i];
      ord[len].k2 = o[i].ret;
      ord[len].k3 = i;
      ord[len].rec = i;
      len++;
    }
  qsort(ord, (size_t)len, sizeof(ord_t), ord_cmp);
  *order_len = len;
  /* the definition: model steps and real-time order */
  int64_t ver = V0, val = init, maxcall = -1;
  for (int64_t j = 0; j < len; j++) {
    const lc_op *op = &o[ord[j].rec];
    const int64_t ret = op->ret <= cut ? op->ret : LC_INF;
    if (ret < maxcall) { rc = ORACLE_WIT_REAL_TIME; goto out; }
    if (op->call > maxcall) maxcall = op->call;
    int64_t nv, nl;
    if (oracle_step(ver, val, op, &nv, &nl) != 1) { rc = ORACLE_WIT_INCONSISTENT; goto out; }
    ver = nv;
    val = nl;
  }
out:
  free(mut);
  free(segval);
  free(ord);
  free(done);
  free(rseg);
  return rc;
}

typedef struct {
  const lc_op *ops;
  const int64_t *key_off;
  int64_t n_keys;
  const int32_t *wit, *kind;
  const int64_t *cut;
  int64_t V0, init;
  int32_t *status;
  int64_t *order_len;
  atomic_long next;
} wjob;

static void *wworker(void *arg) {
  wjob *j = (wjob *)arg;
  for (;;) {
    const int64_t k = atomic_fetch_add(&j->next, 1);
    if (k >= j->n_keys) break;
    const int64_t b = j->key_off[k] - j->key_off[0], n = j->key_off[k + 1] - j->key_off[k];
    int64_t len = 0;
    if (j->kind[k] == LC_WITNESS_NONE) {
      j->status[k] = ORACLE_WIT_NONE;
    } else {
      const int64_t cut = j->kind[k] == LC_WITNESS_FULL ? INT64_MAX : j->cut[k];
      j->status[k] = check_key(j->ops + b, n, j->wit + b, cut, j->V0, j->init, &len);
    }
    if (j->order_len) j->order_len[k] = len;
  }
  return NULL;
}

int oracle_check_witness(const lc_op *ops, const int64_t *key_off, int64_t n_keys,
                         const lc_opts *opts, const int32_t *witness, const int32_t *kind,
                         const int64_t *cut, int32_t *status, int64_t *order_len,
                         int n_threads) {
  if (n_keys < 0 || (n_keys > 0 && (!ops || !key_off || !witness || !kind || !status)))
    return -EINVAL;
  wjob j;
  j.ops = ops;
  j.key_off = key_off;
  j.n_keys = n_keys;
  j.wit = witness;
  j.kind = kind;
  j.cut = cut;
  j.V0 = opts ? opts->init_version : 0;
  j.init = opts ? opts->init_value : LC_NIL;
  j.status = status;
  j.order_len = order_len;
  atomic_init(&j.next, 0);
  for (int64_t k = 0; k < n_keys; k++)
    if (kind[k] == LC_WITNESS_PREFIX && !cut) return -EINVAL;
  if (n_threads <= 1) {
    wworker(&j);
  } else {
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)n_threads);
    if (!th) return -ENOMEM;
    for (int i = 0; i < n_threads; i++) pthread_create(&th[i], NULL, wworker, &j);
    for (int i = 0; i < n_threads; i++) pthread_join(th[i], NULL);
    free(th);
  }
  return 0;
}
