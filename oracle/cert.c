/*
 * cert.c — independent check of infeasibility certificates (lc_aux
 * certificate / certificate_set, include/lincheck.h).  TEST INFRASTRUCTURE
 * ONLY (see oracle.h for who may use it).
 *
 * A PREFIX witness (witness.c) shows that the history prefix just before an
 * invalid key's failing return is linearizable.  The certificate checked
 * here shows that the prefix AT the failing return is not; by prefix closure
 * the two certify the reported fail op as the first failure.  The check uses
 * the records and the definition only (every :ok op, any
 * subset of the pending/crashed ones, real-time order, the model of
 * register.clj:60-96) — no skeleton, matching or search code of the device:
 *
 *   P = the records called at or before `cut` (fail_prefix_end); required =
 *   returned at or before it.  In any linearization of P the k-th mutation
 *   (write / successful CAS) takes the version from V0+k-1 to V0+k (:64-75),
 *   so a mutation claiming version v holds position v-V0-1 (it is
 *   "pinned"), and a read of version v is linearized between the mutations
 *   at positions v-V0-1 and v-V0 and reads the value written at v-V0-1
 *   (:84-96; V0's value is the initial one).  A CAS at position q expects the
 *   value written at q-1 (:77).  Points respect real time: ret(b) < call(a)
 *   puts b before a.
 *
 * Each certificate kind is a set of facts these rules make contradictory:
 *   DUP      two required mutations claiming one version hold one position.
 *   UNREACH  a required op claims a version no linearization of P reaches.
 *   CLAIMS   two required reads of one version read one value.
 *   PAIR     the value at q-1 (held by a, or the initial value) is consumed
 *            at q by b with another value; a and b are each required, or the
 *            only op of P able to hold their needed positions.
 *   ORDER    a's point comes before b's by the version order, b returned
 *            before a was called.
 *   HALL     c needed positions no required op holds, fewer ops of P able
 *            to hold any of them (the necessary conditions below) than c.
 *   PROOF    a case analysis over who holds the open positions: the case
 *            splits a search needed (every op able to hold a position, one
 *            case each), the forced choices in between re-derived here by
 *            propagation (a position exactly one op can hold), each case
 *            ending at a position no remaining op can hold — "able" under
 *            the choices made so far (an op assumed next to a position
 *            fixes the value it writes or expects; an assumed op holds
 *            nothing else).  Sound because each position needed and held by
 *            no required op is held by one of its candidates.
 *
 * "Able to hold position p" (cand) is a set of NECESSARY conditions on the
 * op x that holds a needed position p no required op holds: x is a mutation
 * of P other than a required pinned one, pinned (if at all) to p; x's point
 * t_p is after call(x) and before the return of every required op whose
 * point follows t_p by the version order (mutations at positions > p, reads
 * of versions > V0+p), so call(x) < that minimum; x writes the value the
 * required reads of version V0+p+1 claim and the required CAS at p+1
 * expects; a CAS x expects the value at p-1 where P fixes it (the initial
 * value, a required op at p-1, the required reads of version V0+p).  Any
 * over-approximation only makes a valid certificate fail here, never an
 * invalid one pass.
 */
#include <errno.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>

#include "oracle.h"

typedef struct {
  const lc_op *o;
  int64_t n, cut, V0, init;
  int64_t n_mut;  /* mutations in P */
  int64_t M;      /* positions needed by the required ops */
} pfx_t;

static int in_p(const pfx_t *P, int64_t i) { return P->o[i].call <= P->cut; }
static int req(const pfx_t *P, int64_t i) { return in_p(P, i) && P->o[i].ret <= P->cut; }
static int is_mut(const lc_op *x) { return x->f == LC_F_WRITE || x->f == LC_F_CAS; }
static int pinned(const lc_op *x) { return is_mut(x) && x->version != LC_NIL; }
static int64_t pos_of(const pfx_t *P, const lc_op *x) { return x->version - P->V0 - 1; }
static int ok_rec(const pfx_t *P, int64_t i) { return i >= 0 && i < P->n; }

/* A required pinned mutation at position p, or -1. */
static int64_t held_by(const pfx_t *P, int64_t p) {
  for (int64_t i = 0; i < P->n; i++)
    if (req(P, i) && pinned(&P->o[i]) && pos_of(P, &P->o[i]) == p) return i;
  return -1;
}

/* The value P fixes at position p-1 (the one a CAS at p expects): *det = 0
 * when P leaves it open. */
static int64_t value_before(const pfx_t *P, int64_t p, int *det) {
  *det = 1;
  if (p == 0) return P->init;
  const int64_t h = held_by(P, p - 1);
  if (h >= 0) return P->o[h].value;
  for (int64_t i = 0; i < P->n; i++) {
    const lc_op *x = &P->o[i];
    if (req(P, i) && x->f == LC_F_READ && x->version != LC_NIL && x->version - P->V0 == p &&
        x->value != LC_NIL)
      return x->value;
  }
  *det = 0;
  return 0;
}

/* Assumptions of a PROOF certificate: asg[p] = the op assumed to hold open
 * position p (-1: none), used[x] = op x holds some assumed position. */
typedef struct {
  int64_t *asg;          /* M entries */
  unsigned char *used;   /* n entries */
} assume_t;

/* cand(p), for a needed position no required op holds: the number of ops
 * able to hold it; *one = the op when there is exactly one; mark[x] set for
 * each (may be NULL); list[] the ops in record order (may be NULL).  Under
 * assumptions A (may be NULL): an op assumed at p+1 that is a CAS fixes the
 * value p must write, one assumed at p-1 the value before p, and an op
 * assumed anywhere holds nothing else. */
static int64_t cand_a(const pfx_t *P, int64_t p, int64_t *one, unsigned char *mark,
                      const assume_t *A, int64_t *list) {
  const lc_op *o = P->o;
  /* deadline: returns of the required ops whose points follow t_p */
  int64_t dl = LC_INF;
  for (int64_t i = 0; i < P->n; i++) {
    if (!req(P, i)) continue;
    const lc_op *y = &o[i];
    if ((pinned(y) && pos_of(P, y) > p) ||
        (y->f == LC_F_READ && y->version != LC_NIL && y->version - P->V0 - 1 >= p))
      if (y->ret < dl) dl = y->ret;
  }
  int det;
  int64_t before = value_before(P, p, &det);
  if (A && !det && p >= 1 && A->asg[p - 1] >= 0) {
    det = 1;
    before = o[A->asg[p - 1]].value;
  }
  /* the value the holder of p must write: claimed by the required reads of
   * version V0+p+1, expected by a required CAS at p+1 (two different: none) */
  int has_want = 0, clash = 0;
  int64_t want = 0;
  for (int64_t i = 0; i < P->n; i++) {
    if (!req(P, i)) continue;
    const lc_op *y = &o[i];
    int64_t v;
    if (y->f == LC_F_READ && y->version != LC_NIL && y->version - P->V0 == p + 1 &&
        y->value != LC_NIL)
      v = y->value;
    else if (y->f == LC_F_CAS && y->version != LC_NIL && pos_of(P, y) == p + 1)
      v = y->expected;
    else
      continue;
    if (has_want && v != want) clash = 1;
    has_want = 1;
    want = v;
  }
  if (A && p + 1 < P->M && A->asg[p + 1] >= 0 && o[A->asg[p + 1]].f == LC_F_CAS) {
    const int64_t v = o[A->asg[p + 1]].expected;
    if (has_want && v != want) clash = 1;
    has_want = 1;
    want = v;
  }
  if (clash) return 0;
  int64_t cnt = 0;
  for (int64_t j = 0; j < P->n; j++) {
    const lc_op *x = &o[j];
    if (!in_p(P, j) || !is_mut(x) || (req(P, j) && pinned(x))) continue;
    if (pinned(x) && pos_of(P, x) != p) continue;
    if (x->call >= dl) continue;
    if (x->f == LC_F_CAS && det && x->expected != before) continue;
    if (has_want && x->value != want) continue;
    if (A && A->used[j]) continue;
    if (mark) mark[j] = 1;
    if (one) *one = j;
    if (list) list[cnt] = j;
    cnt++;
  }
  return cnt;
}

static int64_t cand(const pfx_t *P, int64_t p, int64_t *one, unsigned char *mark) {
  return cand_a(P, p, one, mark, NULL, NULL);
}

/* Position p is needed by a required op and held by none. */
static int open_gap(const pfx_t *P, int64_t p) {
  return p >= 0 && p < P->M && held_by(P, p) < 0;
}

/* Op i (a mutation) certainly holds position p: it is required and pinned
 * there, or p is an open needed position whose only candidate it is. */
static int forced_at(const pfx_t *P, int64_t i, int64_t p) {
  if (!ok_rec(P, i) || !is_mut(&P->o[i])) return 0;
  if (req(P, i) && pinned(&P->o[i])) return pos_of(P, &P->o[i]) == p;
  if (!open_gap(P, p)) return 0;
  int64_t one = -1;
  return cand(P, p, &one, NULL) == 1 && one == i;
}

/* A PROOF certificate's proof, from token *at on (include/lincheck.h
 * LC_CERT_PROOF).  Forced choices are derived, not listed: the open
 * positions are propagated — a position no op can hold under the choices so
 * far closes the case; else the lowest position exactly one op can hold is
 * assumed held by it, and again — and only where propagation stops does the
 * next token name a case split, BRANCH(g, k): g open and unassigned with
 * exactly k >= 2 candidates, whose k sub-proofs follow, one per candidate in
 * record order, each assuming it holds g.  (As a SAT proof checker's unit
 * propagation: deterministic deduction, no search.)  Every assumption is
 * undone before returning.  1: the (sub)proof holds. */
static int proof_ok(const pfx_t *P, const int32_t *tok, int64_t len, int64_t *at, assume_t *A,
                    int64_t *scratch, int depth) {
  if (depth > 64) return 0;
  int64_t *forced = scratch + (int64_t)depth * 2 * (P->n + 2);  /* this level's assumptions */
  int64_t *list = forced + (P->n + 2);
  int64_t nf = 0;
  int ok = 0;
  for (;;) {
    /* propagate: an empty position closes the case; else the lowest forced */
    int64_t fp = -1, fo = -1, empty = 0;
    for (int64_t p = 0; p < P->M; p++) {
      if (A->asg[p] >= 0 || !open_gap(P, p)) continue;
      int64_t one = -1;
      const int64_t k = cand_a(P, p, &one, NULL, A, NULL);
      if (k == 0) {
        empty = 1;
        break;
      }
      if (k == 1 && fp < 0) fp = p, fo = one;
    }
    if (empty) {
      ok = 1;
      break;
    }
    if (fp >= 0) {
      A->asg[fp] = fo;
      A->used[fo] = 1;
      forced[nf++] = fp;
      continue;
    }
    /* a case split, named by the next token */
    if (*at >= len) break;
    const uint32_t t = (uint32_t)tok[(*at)++];
    const int64_t g = (t >> 15) & 0x7FFF, k = t & 0x7FFF;
    if ((t >> 30) != 2 || !open_gap(P, g) || A->asg[g] >= 0 || k < 2) break;
    if (cand_a(P, g, NULL, NULL, A, list) != k) break;
    ok = 1;
    for (int64_t i = 0; i < k && ok; i++) {
      const int64_t x = list[i];
      A->asg[g] = x;
      A->used[x] = 1;
      ok = proof_ok(P, tok, len, at, A, scratch, depth + 1);
      A->asg[g] = -1;
      A->used[x] = 0;
    }
    break;
  }
  while (nf > 0) {
    const int64_t p = forced[--nf];
    A->used[A->asg[p]] = 0;
    A->asg[p] = -1;
  }
  return ok;
}

static int check_cert(const lc_op *o, int64_t n, const int32_t *c, const int32_t *cset,
                      int64_t cut, int64_t V0, int64_t init) {
  if (c[0] == LC_CERT_NONE) return ORACLE_CERT_NONE;
  pfx_t P = {o, n, cut, V0, init, 0, 0};
  for (int64_t i = 0; i < n; i++) {
    if (in_p(&P, i) && is_mut(&o[i])) P.n_mut++;
    if (!req(&P, i)) continue;
    int64_t need = 0;
    if (pinned(&o[i])) need = pos_of(&P, &o[i]) + 1;
    else if (o[i].f == LC_F_READ && o[i].version != LC_NIL) need = o[i].version - V0;
    if (need > P.M) P.M = need;
  }
  const int64_t a = c[1], b = c[2];
  const lc_op *A = ok_rec(&P, a) ? &o[a] : NULL, *B = ok_rec(&P, b) ? &o[b] : NULL;
  switch (c[0]) {
    case LC_CERT_DUP:
      if (A && B && a != b && req(&P, a) && req(&P, b) && pinned(A) && pinned(B) &&
          A->version == B->version)
        return ORACLE_CERT_OK;
      break;
    case LC_CERT_UNREACH:
      if (!A || !req(&P, a)) break;
      if (pinned(A) && (A->version <= V0 || A->version - V0 > P.n_mut)) return ORACLE_CERT_OK;
      if (A->f == LC_F_READ && A->version != LC_NIL &&
          (A->version < V0 || A->version - V0 > P.n_mut ||
           (A->version == V0 && A->value != LC_NIL && A->value != init)))
        return ORACLE_CERT_OK;
      break;
    case LC_CERT_CLAIMS:
      if (A && B && a != b && req(&P, a) && req(&P, b) && A->f == LC_F_READ &&
          B->f == LC_F_READ && A->version != LC_NIL && A->version == B->version &&
          A->value != LC_NIL && B->value != LC_NIL && A->value != B->value)
        return ORACLE_CERT_OK;
      break;
    case LC_CERT_PAIR: {
      const int64_t q = c[3];
      if (!B || q < 0) break;
      int64_t want;
      if (B->f == LC_F_CAS) {
        want = B->expected;
        if (!forced_at(&P, b, q)) break;
      } else if (B->f == LC_F_READ && B->version != LC_NIL && B->value != LC_NIL &&
                 B->version - V0 == q) {
        want = B->value;
        if (!req(&P, b)) break;
      } else {
        break;
      }
      int64_t have;
      if (a == -1) {
        if (q != 0) break;
        have = init;
      } else {
        if (!A || q < 1 || !forced_at(&P, a, q - 1)) break;
        have = A->value;
      }
      if (have != want) return ORACLE_CERT_OK;
      break;
    }
    case LC_CERT_ORDER: {
      if (!A || !B || !req(&P, a) || !req(&P, b) || !(A->call > B->ret)) break;
      int64_t lo, hi;
      if (pinned(A)) lo = pos_of(&P, A);
      else if (A->f == LC_F_READ && A->version != LC_NIL) lo = A->version - V0;
      else break;
      if (pinned(B)) hi = pos_of(&P, B);
      else if (B->f == LC_F_READ && B->version != LC_NIL) hi = B->version - V0 - 1;
      else break;
      if (lo >= 0 && lo <= hi) return ORACLE_CERT_OK;
      break;
    }
    case LC_CERT_HALL: {
      const int64_t cnt = c[3];
      if (cnt < 1 || cnt > n || !cset) break;
      unsigned char *mark = (unsigned char *)calloc((size_t)n, 1);
      unsigned char *seen = (unsigned char *)calloc((size_t)n + 2, 1);
      if (!mark || !seen) {
        free(mark);
        free(seen);
        return -ENOMEM;
      }
      int good = 1;
      for (int64_t g = 0; g < cnt && good; g++) {
        const int64_t p = cset[g];
        /* distinct, needed, held by no required op */
        if (!open_gap(&P, p) || p > n || seen[p]) good = 0;
        else seen[p] = 1;
        if (good) cand(&P, p, NULL, mark);
      }
      int64_t u = 0;
      for (int64_t j = 0; j < n; j++) u += mark[j];
      free(mark);
      free(seen);
      if (good && u < cnt) return ORACLE_CERT_OK;
      break;
    }
    case LC_CERT_PROOF: {
      const int64_t len = c[3];
      if (len < 0 || len > n || !cset || P.M < 1) break;
      int64_t *asg = (int64_t *)malloc(sizeof(int64_t) * (size_t)P.M);
      unsigned char *used = (unsigned char *)calloc((size_t)n, 1);
      int64_t *scratch = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n + 2) * 2 * 66);
      if (!asg || !used || !scratch) {
        free(asg);
        free(used);
        free(scratch);
        return -ENOMEM;
      }
      for (int64_t p = 0; p < P.M; p++) asg[p] = -1;
      assume_t A = {asg, used};
      int64_t at = 0;
      /* the whole proof, and nothing after it */
      const int ok = proof_ok(&P, cset, len, &at, &A, scratch, 0) && at == len;
      free(asg);
      free(used);
      free(scratch);
      if (ok) return ORACLE_CERT_OK;
      break;
    }
    default:
      break;
  }
  return ORACLE_CERT_BAD;
}

typedef struct {
  const lc_op *ops;
  const int64_t *key_off, *cut;
  int64_t n_keys, V0, init;
  const int32_t *cert, *cset;
  int32_t *status;
  atomic_long next;
} cjob;

static void *cworker(void *arg) {
  cjob *j = (cjob *)arg;
  for (;;) {
    const int64_t k = atomic_fetch_add(&j->next, 1);
    if (k >= j->n_keys) break;
    const int64_t b = j->key_off[k] - j->key_off[0], n = j->key_off[k + 1] - j->key_off[k];
    j->status[k] = check_cert(j->ops + b, n, j->cert + 4 * k, j->cset ? j->cset + b : NULL,
                              j->cut[k], j->V0, j->init);
  }
  return NULL;
}

int oracle_check_certificate(const lc_op *ops, const int64_t *key_off, int64_t n_keys,
                             const lc_opts *opts, const int32_t *cert, const int32_t *cert_set,
                             const int64_t *cut, int32_t *status, int n_threads) {
  if (n_keys < 0 || (n_keys > 0 && (!ops || !key_off || !cert || !cut || !status)))
    return -EINVAL;
  cjob j;
  j.ops = ops;
  j.key_off = key_off;
  j.cut = cut;
  j.n_keys = n_keys;
  j.V0 = opts ? opts->init_version : 0;
  j.init = opts ? opts->init_value : LC_NIL;
  j.cert = cert;
  j.cset = cert_set;
  j.status = status;
  atomic_init(&j.next, 0);
  if (n_threads <= 1) {
    cworker(&j);
  } else {
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)n_threads);
    if (!th) return -ENOMEM;
    for (int i = 0; i < n_threads; i++) pthread_create(&th[i], NULL, cworker, &j);
    for (int i = 0; i < n_threads; i++) pthread_join(th[i], NULL);
    free(th);
  }
  return 0;
}
