/*
 * oracle.c — CPU restatement of the reference path (TEST INFRASTRUCTURE ONLY;
 * see oracle.h for who may use it and for its parity status: PARITY UNPINNED
 * against outputs of the reference itself, pinned by hand-derived KATs and by
 * three-way algorithm agreement).
 *
 * What it restates:
 *  - the model: VersionedRegister.step, /root/reference/src/jepsen/etcd/register.clj:59-96
 *    (write :64-68, cas :70-82, read :84-96), initial state (->VersionedRegister 0 nil) :111;
 *  - the checker: jepsen.checker/linearizable over knossos (register.clj:110-111), whose
 *    two analyzers knossos.linear (JIT linearization, Lowe 2017) and knossos.wgl
 *    (Wing & Gong with Lowe's (linearized-set, state) cache) are third-party code pulled in
 *    by [jepsen "0.3.3-SNAPSHOT"] (project.clj:7; knossos 0.3.x, exact version unverifiable
 *    offline).  Both are restated from their published algorithms, faithfully: no
 *    model-specific pruning (the GPU path's eager read closure is NOT used here), so the
 *    oracle checks that pruning rather than sharing it.
 *  - the per-key split of jepsen.independent/checker (register.clj:108) is the caller's
 *    key_off partition; :fail pairs are already dropped and :info ops carry ret = LC_INF
 *    (knossos history completion: crashed ops may take effect any time after their call).
 */
#include "oracle.h"

#include <errno.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- model */

int oracle_step(int64_t ver, int64_t val, const lc_op *op, int64_t *nver,
                int64_t *nval) {
  /* (let [[op-version op-value] (:value op) version' (inc version)] ...) :61-62 */
  const int64_t opver = op->version;
  const int64_t ver1 = ver + 1;
  switch (op->f) {
    case LC_F_WRITE: /* :64-68 */
      if (opver != LC_NIL && opver != ver1) return 0;
      *nver = ver1;
      *nval = op->value;
      return 1;
    case LC_F_CAS: /* :70-82 — version check first, then (not= value v) */
      if (opver != LC_NIL && opver != ver1) return 0;
      if (val != op->expected) return 0; /* nil == nil passes, :77 */
      *nver = ver1;
      *nval = op->value;
      return 1;
    case LC_F_READ: /* :84-96 — state unchanged */
      if (opver != LC_NIL && opver != ver) return 0;
      if (op->value != LC_NIL && op->value != val) return 0;
      *nver = ver;
      *nval = val;
      return 1;
    default: /* condp = without a default clause throws, :63 */
      return -1;
  }
}

/* ------------------------------------------------- configuration hash set */

/* A configuration is `nw` words: bitset words then (version, value). */
typedef struct {
  int nw;
  uint64_t *arena;
  size_t n, cap;
  uint32_t *tab; /* index+1, 0 = empty */
  size_t tcap;   /* power of two */
} cset;

static uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

static uint64_t cfg_hash(const uint64_t *c, int nw) {
  uint64_t h = 0x9E3779B97F4A7C15ULL;
  for (int i = 0; i < nw; i++) h = mix64(h ^ c[i]) + (uint64_t)i;
  return h;
}

static int cset_init(cset *s, int nw) {
  memset(s, 0, sizeof(*s));
  s->nw = nw;
  s->cap = 64;
  s->arena = (uint64_t *)malloc(sizeof(uint64_t) * s->cap * nw);
  s->tcap = 128;
  s->tab = (uint32_t *)calloc(s->tcap, sizeof(uint32_t));
  return (s->arena && s->tab) ? 0 : -ENOMEM;
}

static void cset_free(cset *s) {
  free(s->arena);
  free(s->tab);
  memset(s, 0, sizeof(*s));
}

static void cset_clear(cset *s) {
  s->n = 0;
  memset(s->tab, 0, s->tcap * sizeof(uint32_t));
}

static const uint64_t *cset_get(const cset *s, size_t i) {
  return s->arena + i * (size_t)s->nw;
}

static int cset_rehash(cset *s, size_t tcap) {
  uint32_t *t = (uint32_t *)calloc(tcap, sizeof(uint32_t));
  if (!t) return -ENOMEM;
  for (size_t i = 0; i < s->n; i++) {
    size_t h = (size_t)cfg_hash(cset_get(s, i), s->nw) & (tcap - 1);
    while (t[h]) h = (h + 1) & (tcap - 1);
    t[h] = (uint32_t)(i + 1);
  }
  free(s->tab);
  s->tab = t;
  s->tcap = tcap;
  return 0;
}

/* Returns 1 if inserted, 0 if already present, <0 on ENOMEM. */
static int cset_add(cset *s, const uint64_t *c) {
  const int nw = s->nw;
  size_t h = (size_t)cfg_hash(c, nw) & (s->tcap - 1);
  while (s->tab[h]) {
    const uint64_t *e = cset_get(s, s->tab[h] - 1);
    if (memcmp(e, c, sizeof(uint64_t) * nw) == 0) return 0;
    h = (h + 1) & (s->tcap - 1);
  }
  if (s->n == s->cap) {
    size_t ncap = s->cap * 2;
    uint64_t *a = (uint64_t *)realloc(s->arena, sizeof(uint64_t) * ncap * nw);
    if (!a) return -ENOMEM;
    s->arena = a;
    s->cap = ncap;
  }
  memcpy(s->arena + s->n * (size_t)nw, c, sizeof(uint64_t) * nw);
  s->n++;
  s->tab[h] = (uint32_t)s->n;
  if (s->n * 2 > s->tcap) return cset_rehash(s, s->tcap * 2) < 0 ? -ENOMEM : 1;
  return 1;
}

/* ------------------------------------------------------------ utilities */

static void result_init(lc_key_result *r) {
  r->verdict = LC_VALID;
  r->reason = LC_REASON_NONE;
  r->fail_op = -1;
  r->fail_prefix_end = -1;
  r->configs_explored = 0;
  r->max_frontier = 0;
}

static void result_unknown(lc_key_result *r, int reason) {
  r->verdict = LC_UNKNOWN;
  r->reason = reason;
  r->fail_op = -1;
  r->fail_prefix_end = -1;
}

/* Structural validation shared with the device path: calls strictly
 * increasing, call < ret, fields >= -1.  Unknown f is not malformed
 * (the model throws at step time -> :unknown). */
static int key_malformed(const lc_op *o, int64_t n) {
  for (int64_t i = 0; i < n; i++) {
    if (o[i].call < 0 || o[i].ret <= o[i].call) return 1;
    if (i > 0 && o[i].call <= o[i - 1].call) return 1;
    /* any version is well-formed: one no state reaches (< -1 included) makes
     * the op illegal at every step, as in knossos */
    if (o[i].value < -1 || o[i].expected < -1) return 1;
  }
  return 0;
}

static int key_has_unknown_f(const lc_op *o, int64_t n) {
  for (int64_t i = 0; i < n; i++)
    if (o[i].f != LC_F_READ && o[i].f != LC_F_WRITE && o[i].f != LC_F_CAS)
      return 1;
  return 0;
}

/* Events in history order; at equal index a call precedes a return (a
 * precedes b in real time only when ret(a) < call(b)). */
typedef struct {
  int64_t idx;
  int32_t is_ret;
  int32_t op;
} event;

static int event_cmp(const void *a, const void *b) {
  const event *x = (const event *)a, *y = (const event *)b;
  if (x->idx != y->idx) return x->idx < y->idx ? -1 : 1;
  if (x->is_ret != y->is_ret) return x->is_ret - y->is_ret;
  return x->op - y->op;
}

static event *build_events(const lc_op *o, int64_t n, int64_t *ne) {
  event *ev = (event *)malloc(sizeof(event) * (size_t)(2 * n + 1));
  if (!ev) return NULL;
  int64_t k = 0;
  for (int64_t i = 0; i < n; i++) {
    ev[k].idx = o[i].call;
    ev[k].is_ret = 0;
    ev[k].op = (int32_t)i;
    k++;
    if (o[i].ret != LC_INF) {
      ev[k].idx = o[i].ret;
      ev[k].is_ret = 1;
      ev[k].op = (int32_t)i;
      k++;
    }
  }
  qsort(ev, (size_t)k, sizeof(event), event_cmp);
  *ne = k;
  return ev;
}

/* ------------------------------------------ knossos.linear (JIT) restated */

/* Frontier of configurations (model state, set of linearized ops among the
 * open calls).  On each :ok return of x every configuration lacking x is
 * expanded by linearizing pending ops (any order the model allows) until x
 * is linearized; expansion stops at x.  An empty frontier at x's return means
 * the history prefix up to that return has no linearization: x is the
 * canonical counterexample.  Slots index the open calls; crashed ops keep
 * their slot (until retired, below).
 *
 * `reduce` (ORACLE_FLAG_*) enables exact reductions, each checked by tests/
 * against the faithful mode (reduce == 0), which is knossos.linear's search:
 *  READ_CLOSURE   a pending read legal in a configuration is linearized at
 *                 once, and reads that can never constrain (crashed, or
 *                 [nil nil]) get no slot.  A read never changes the state
 *                 (register.clj:84-96), so (s, L+{r}) dominates (s, L).
 *  CRASH_SYMMETRY crashed writes/CAS with equal (f, value, expected) are
 *                 interchangeable once called (their version is always nil:
 *                 the completion never arrived), so only the earliest-called
 *                 unlinearized member of such a class may be linearized next.
 *  DEADLINE_ORDER writes/CAS with equal (f, value, expected, version) have the
 *                 same precondition and effect, so among the pending members
 *                 of such a class only the one with the earliest deadline
 *                 (return index; crashed = never, ties by call) may be
 *                 linearized next.  Exchange argument: if a and b are both
 *                 pending, ret(a) <= ret(b), and a linearization puts b at p
 *                 and a later at q <= ret(a), swapping them keeps every op
 *                 within its interval (p >= now >= call(a), q <= ret(a) <=
 *                 ret(b)) and every state unchanged; a crashed b may also
 *                 stay unlinearized.  So the configuration that took a
 *                 dominates the one that took b.  This generalises
 *                 CRASH_SYMMETRY (crashed ops: equal deadlines) to :ok ops,
 *                 which matters for version-less models, where equal writes
 *                 are common (round 2).
 *  RETIRE         an op linearized in every configuration is done for good:
 *                 a crashed op has no return, and an :ok op's return would
 *                 keep every configuration unchanged (JIT keeps the configs
 *                 that already linearized it), so its slot is freed and its
 *                 return skipped.  Real time stays respected: anything
 *                 called later is linearized after it in every config. */
static int is_trivial_read(const lc_op *op) {
  return op->f == LC_F_READ &&
         (op->ret == LC_INF || (op->version == LC_NIL && op->value == LC_NIL));
}

static int is_crashed_mutation(const lc_op *op) {
  return op->ret == LC_INF && op->f != LC_F_READ;
}

static int same_class(const lc_op *a, const lc_op *b) {
  return a->f == b->f && a->value == b->value && a->expected == b->expected &&
         a->version == b->version;
}

static void close_reads(const lc_op *o, const int32_t *slot_op, const uint64_t *occ,
                        int bw, uint64_t *cfg) {
  for (int w = 0; w < bw; w++) {
    uint64_t pend = occ[w] & ~cfg[w];
    while (pend) {
      const int b = __builtin_ctzll(pend);
      pend &= pend - 1;
      const lc_op *op = &o[slot_op[w * 64 + b]];
      int64_t nv, nval;
      if (op->f == LC_F_READ &&
          oracle_step((int64_t)cfg[bw], (int64_t)cfg[bw + 1], op, &nv, &nval) == 1)
        cfg[w] |= 1ULL << b;
    }
  }
}

#define BIT(a, s) (((a)[(s) >> 6] >> ((s) & 63)) & 1)

/* oracle_frontier: stop at the return of stop_op and dump the frontier that
 * return expands (every configuration: state + sorted pending ops). */
typedef struct frontier_req {
  int64_t stop_op;
  int64_t *out;  /* max entries of ORACLE_CFG_WORDS int64 */
  int64_t max;
  int64_t n;     /* configurations in the frontier (may exceed max) */
} frontier_req;

static void check_key_jit_fr(const lc_op *o, int64_t n, const lc_opts *opts,
                             int64_t budget, int reduce, lc_key_result *res,
                             frontier_req *fr);

static void check_key_jit(const lc_op *o, int64_t n, const lc_opts *opts,
                          int64_t budget, int reduce, lc_key_result *res) {
  check_key_jit_fr(o, n, opts, budget, reduce, res, NULL);
}

static void check_key_jit_fr(const lc_op *o, int64_t n, const lc_opts *opts,
                             int64_t budget, int reduce, lc_key_result *res,
                             frontier_req *fr) {
  const int closure = (reduce & ORACLE_FLAG_READ_CLOSURE) != 0;
  const int symmetry = (reduce & ORACLE_FLAG_CRASH_SYMMETRY) != 0;
  const int retire = (reduce & ORACLE_FLAG_RETIRE) != 0;
  const int deadline = (reduce & ORACLE_FLAG_DEADLINE_ORDER) != 0;
  result_init(res);
  if (n == 0) return;
  int64_t ne = 0;
  event *ev = build_events(o, n, &ne);
  if (!ev) {
    result_unknown(res, LC_REASON_CONFIG_BUDGET);
    return;
  }
  /* Window size bound: simulate open-slot count (retirement only lowers it). */
  int64_t open = 0, maxopen = 0;
  for (int64_t e = 0; e < ne; e++) {
    if (!ev[e].is_ret) {
      open++;
      if (open > maxopen) maxopen = open;
    } else {
      open--;
    }
  }
  const int bw = (int)((maxopen + 63) / 64);
  const int nw = bw + 2;
  int32_t *slot_of = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
  int32_t *slot_op = (int32_t *)malloc(sizeof(int32_t) * (size_t)(bw * 64));
  int32_t *pred = (int32_t *)malloc(sizeof(int32_t) * (size_t)(bw * 64));
  uint8_t *latest = (uint8_t *)calloc((size_t)(bw * 64), 1);
  uint64_t *occ = (uint64_t *)calloc((size_t)bw, sizeof(uint64_t));
  uint64_t *crashed = (uint64_t *)calloc((size_t)bw, sizeof(uint64_t));
  uint64_t *all = (uint64_t *)calloc((size_t)bw, sizeof(uint64_t));
  uint64_t *tmp = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)nw);
  /* DEADLINE_ORDER: per slot, the same-class slots to linearize before it */
  uint64_t *before = (uint64_t *)calloc((size_t)(bw * 64) * (size_t)bw, sizeof(uint64_t));
  cset F, R, V;
  int ok = slot_of && slot_op && pred && latest && occ && crashed && all && tmp && before;
  ok = ok && cset_init(&F, nw) == 0 && cset_init(&R, nw) == 0 &&
       cset_init(&V, nw) == 0;
  if (!ok) {
    result_unknown(res, LC_REASON_CONFIG_BUDGET);
    goto done;
  }
  for (int u = 0; u < bw * 64; u++) pred[u] = -1;
  memset(tmp, 0, sizeof(uint64_t) * (size_t)nw);
  tmp[bw] = (uint64_t)opts->init_version;
  tmp[bw + 1] = (uint64_t)opts->init_value;
  cset_add(&F, tmp);
  res->max_frontier = 1;
  int64_t explored = 1;

  for (int64_t e = 0; e < ne; e++) {
    const int32_t x = ev[e].op;
    if (!ev[e].is_ret) {
      if (closure && is_trivial_read(&o[x])) {
        slot_of[x] = -1;
        continue;
      }
      int s = 0;
      while (BIT(occ, s)) s++;
      occ[s >> 6] |= 1ULL << (s & 63);
      slot_of[x] = s;
      slot_op[s] = x;
      pred[s] = -1;
      latest[s] = 0;
      if (deadline && o[x].f != LC_F_READ) {
        uint64_t *bs_row = before + (size_t)s * (size_t)bw;
        memset(bs_row, 0, sizeof(uint64_t) * (size_t)bw);
        for (int u = 0; u < bw * 64; u++) {
          if (u == s || !BIT(occ, u)) continue;
          const lc_op *ou = &o[slot_op[u]];
          if (ou->f == LC_F_READ || !same_class(ou, &o[x])) continue;
          if (ou->ret <= o[x].ret) /* earlier deadline (equal: both crashed, u called first) */
            bs_row[u >> 6] |= 1ULL << (u & 63);
          else
            before[(size_t)u * (size_t)bw + (size_t)(s >> 6)] |= 1ULL << (s & 63);
        }
      }
      if (is_crashed_mutation(&o[x])) {
        crashed[s >> 6] |= 1ULL << (s & 63);
        if (symmetry) {
          for (int u = 0; u < bw * 64; u++)
            if (u != s && BIT(crashed, u) && latest[u] &&
                same_class(&o[slot_op[u]], &o[x])) {
              pred[s] = u;
              latest[u] = 0;
              break;
            }
          latest[s] = 1;
        }
      }
      if (closure && o[x].f == LC_F_READ) {
        /* linearize the new read in every configuration where it is legal;
         * configurations stay distinct (equal states decide alike) */
        for (size_t i = 0; i < F.n; i++) {
          uint64_t *c = F.arena + i * (size_t)nw;
          int64_t nv, nval;
          if (oracle_step((int64_t)c[bw], (int64_t)c[bw + 1], &o[x], &nv, &nval) == 1)
            c[s >> 6] |= 1ULL << (s & 63);
        }
        /* masks changed in place: rebuild F's hash index */
        cset_rehash(&F, F.tcap);
      }
      continue;
    }
    if (slot_of[x] < 0) continue; /* trivial read: nothing to do */
    if (fr && x == fr->stop_op) {
      fr->n = (int64_t)F.n;
      for (size_t i = 0; i < F.n && (int64_t)i < fr->max; i++) {
        const uint64_t *c = cset_get(&F, i);
        int64_t *d = fr->out + i * ORACLE_CFG_WORDS;
        d[0] = (int64_t)c[bw];
        d[1] = (int64_t)c[bw + 1];
        int64_t np = 0;
        for (int u = 0; u < bw * 64 && np < 64; u++)
          if (BIT(occ, u) && !BIT(c, u)) d[3 + np++] = slot_op[u];
        d[2] = np;
        /* sorted by op index */
        for (int64_t a = 1; a < np; a++)
          for (int64_t b = a; b > 0 && d[3 + b - 1] > d[3 + b]; b--) {
            const int64_t t = d[3 + b];
            d[3 + b] = d[3 + b - 1];
            d[3 + b - 1] = t;
          }
      }
      goto done;
    }
    const int sx = slot_of[x];
    const int wx = sx >> 6;
    const uint64_t bx = 1ULL << (sx & 63);
    cset_clear(&R);
    cset_clear(&V);
    for (size_t i = 0; i < F.n; i++) {
      const uint64_t *c = cset_get(&F, i);
      if (c[wx] & bx) {
        memcpy(tmp, c, sizeof(uint64_t) * (size_t)nw);
        tmp[wx] &= ~bx;
        cset_add(&R, tmp);
      } else {
        cset_add(&V, c);
      }
    }
    for (size_t h = 0; h < V.n; h++) {
      for (int w = 0; w < bw; w++) {
        const uint64_t *c = cset_get(&V, h); /* arena may move: re-fetch */
        uint64_t pend = occ[w] & ~c[w];
        while (pend) {
          const int b = __builtin_ctzll(pend);
          pend &= pend - 1;
          const int t = w * 64 + b;
          c = cset_get(&V, h);
          if (symmetry && pred[t] >= 0 && !BIT(c, pred[t])) continue;
          if (deadline) {
            const uint64_t *row = before + (size_t)t * (size_t)bw;
            int blocked = 0;
            for (int w2 = 0; w2 < bw; w2++) blocked |= (row[w2] & ~c[w2]) != 0;
            if (blocked) continue;
          }
          int64_t nv, nval;
          const int st = oracle_step((int64_t)c[bw], (int64_t)c[bw + 1],
                                     &o[slot_op[t]], &nv, &nval);
          if (st < 0) {
            result_unknown(res, LC_REASON_UNKNOWN_F);
            goto done;
          }
          if (!st) continue;
          memcpy(tmp, c, sizeof(uint64_t) * (size_t)nw);
          tmp[w] |= 1ULL << b;
          tmp[bw] = (uint64_t)nv;
          tmp[bw + 1] = (uint64_t)nval;
          if (closure) {
            if (o[slot_op[t]].f == LC_F_READ) continue; /* closed already */
            close_reads(o, slot_op, occ, bw, tmp);
          }
          explored++;
          int r;
          if (tmp[wx] & bx) { /* x linearized (directly, or by the closure) */
            tmp[wx] &= ~bx;
            r = cset_add(&R, tmp);
          } else {
            r = cset_add(&V, tmp);
          }
          if (r < 0 || (int64_t)(R.n + V.n) > budget) {
            res->configs_explored = explored;
            result_unknown(res, LC_REASON_CONFIG_BUDGET);
            goto done;
          }
        }
      }
    }
    /* F := R */
    cset t = F;
    F = R;
    R = t;
    occ[wx] &= ~bx;
    if (deadline) /* x is linearized in every configuration from here on */
      for (int u = 0; u < bw * 64; u++) before[(size_t)u * (size_t)bw + (size_t)wx] &= ~bx;
    if ((int64_t)F.n > res->max_frontier) res->max_frontier = (int64_t)F.n;
    if (F.n == 0) {
      res->verdict = LC_INVALID;
      res->reason = LC_REASON_NONLINEARIZABLE;
      res->fail_op = x;
      res->fail_prefix_end = o[x].ret;
      break;
    }
    if (retire) {
      /* an op linearized in every configuration is finished: a crashed op has
       * no return to wait for, and an :ok op's return would keep every
       * configuration as it is (all of them already linearized it) */
      int any = 0;
      for (int w = 0; w < bw; w++) {
        all[w] = occ[w];
        for (size_t i = 0; i < F.n; i++) all[w] &= cset_get(&F, i)[w];
        any |= all[w] != 0;
      }
      if (any) {
        for (size_t i = 0; i < F.n; i++) {
          uint64_t *c = F.arena + i * (size_t)nw;
          for (int w = 0; w < bw; w++) c[w] &= ~all[w];
        }
        cset_rehash(&F, F.tcap);
        for (int u = 0; u < bw * 64; u++) {
          if (BIT(all, u)) {
            latest[u] = 0;
            pred[u] = -1;
            slot_of[slot_op[u]] = -1; /* its return (if any) is now a no-op */
          }
          if (BIT(occ, u) && pred[u] >= 0 && BIT(all, pred[u])) pred[u] = -1;
        }
        for (int w = 0; w < bw; w++) {
          occ[w] &= ~all[w];
          crashed[w] &= ~all[w];
        }
        if (deadline)
          for (int u = 0; u < bw * 64; u++)
            for (int w = 0; w < bw; w++) before[(size_t)u * (size_t)bw + (size_t)w] &= ~all[w];
      }
    }
  }
  res->configs_explored = explored;
done:
  cset_free(&F);
  cset_free(&R);
  cset_free(&V);
  free(slot_of);
  free(slot_op);
  free(pred);
  free(latest);
  free(occ);
  free(crashed);
  free(all);
  free(tmp);
  free(before);
  free(ev);
}

/* ------------------------------------------------ knossos.wgl restated */

typedef struct wnode {
  struct wnode *prev, *next;
  struct wnode *match; /* call -> its return node (NULL for :info) */
  int32_t op;
  int32_t is_ret;
} wnode;

static void lift(wnode *c) {
  c->prev->next = c->next;
  if (c->next) c->next->prev = c->prev;
  wnode *r = c->match;
  if (r) {
    r->prev->next = r->next;
    if (r->next) r->next->prev = r->prev;
  }
}

static void unlift(wnode *c) {
  wnode *r = c->match;
  if (r) {
    r->prev->next = r;
    if (r->next) r->next->prev = r;
  }
  c->prev->next = c;
  if (c->next) c->next->prev = c;
}

/* Depth-first search over the call/return entry list: at a call entry try to
 * linearize it (model step legal and (linearized ∪ {op}, state') not cached);
 * at a return entry of an op not yet linearized, backtrack.  Crashed ops have
 * no return entry, so they may stay unlinearized.  Valid once every :ok op is
 * linearized. */
static void check_key_wgl(const lc_op *o, int64_t n, const lc_opts *opts,
                          int64_t budget, lc_key_result *res) {
  result_init(res);
  if (n == 0) return;
  int64_t ne = 0;
  event *ev = build_events(o, n, &ne);
  wnode *nodes = (wnode *)calloc((size_t)ne + 1, sizeof(wnode));
  wnode **callnode = (wnode **)calloc((size_t)n, sizeof(wnode *));
  const int bw = (int)((n + 63) / 64);
  const int nw = bw + 2;
  uint64_t *L = (uint64_t *)calloc((size_t)nw, sizeof(uint64_t));
  typedef struct {
    wnode *e;
    int64_t ver, val;
  } frame;
  frame *stack = (frame *)malloc(sizeof(frame) * (size_t)(n + 1));
  cset cache;
  int have_cache = 0;
  if (!ev || !nodes || !callnode || !L || !stack ||
      cset_init(&cache, nw) != 0) {
    result_unknown(res, LC_REASON_CONFIG_BUDGET);
    goto done;
  }
  have_cache = 1;
  wnode *head = &nodes[ne];
  head->prev = NULL;
  wnode *prev = head;
  int64_t remaining_ok = 0;
  for (int64_t e = 0; e < ne; e++) {
    wnode *w = &nodes[e];
    w->op = ev[e].op;
    w->is_ret = ev[e].is_ret;
    w->prev = prev;
    prev->next = w;
    prev = w;
    if (!w->is_ret) {
      callnode[w->op] = w;
    } else {
      callnode[w->op]->match = w;
      remaining_ok++;
    }
  }
  prev->next = NULL;

  int64_t ver = opts->init_version, val = opts->init_value;
  int64_t sp = 0, explored = 0;
  wnode *entry = head->next;
  for (;;) {
    if (remaining_ok == 0) break; /* valid */
    if (!entry) {                 /* unreachable while an :ok op remains */
      result_unknown(res, LC_REASON_CONFIG_BUDGET);
      goto done;
    }
    if (!entry->is_ret) {
      const int32_t x = entry->op;
      int64_t nv, nval;
      const int st = oracle_step(ver, val, &o[x], &nv, &nval);
      if (st < 0) {
        result_unknown(res, LC_REASON_UNKNOWN_F);
        goto done;
      }
      if (st) {
        L[x >> 6] |= 1ULL << (x & 63);
        L[bw] = (uint64_t)nv;
        L[bw + 1] = (uint64_t)nval;
        const int r = cset_add(&cache, L);
        if (r < 0 || (int64_t)cache.n > budget) {
          res->configs_explored = (int64_t)cache.n;
          result_unknown(res, LC_REASON_CONFIG_BUDGET);
          goto done;
        }
        if (r == 1) {
          explored++;
          stack[sp].e = entry;
          stack[sp].ver = ver;
          stack[sp].val = val;
          sp++;
          ver = nv;
          val = nval;
          lift(entry);
          if (o[x].ret != LC_INF) remaining_ok--;
          entry = head->next;
          continue;
        }
        L[x >> 6] &= ~(1ULL << (x & 63));
      }
      entry = entry->next;
    } else {
      if (sp == 0) {
        res->verdict = LC_INVALID;
        res->reason = LC_REASON_NONLINEARIZABLE;
        break;
      }
      sp--;
      wnode *c = stack[sp].e;
      ver = stack[sp].ver;
      val = stack[sp].val;
      L[c->op >> 6] &= ~(1ULL << (c->op & 63));
      unlift(c);
      if (o[c->op].ret != LC_INF) remaining_ok++;
      entry = c->next;
    }
  }
  res->configs_explored = explored;
  res->max_frontier = (int64_t)cache.n;
done:
  if (have_cache) cset_free(&cache);
  free(ev);
  free(nodes);
  free(callnode);
  free(L);
  free(stack);
}

/* ------------------------------------------------------------- driver */

typedef struct {
  const lc_op *ops;
  const int64_t *key_off;
  int64_t n_keys;
  const lc_opts *opts;
  lc_key_result *out;
  int algo;
  int reduce;
  int64_t budget;
  _Atomic int64_t next;
  _Atomic int malformed;
} job;

static void *worker(void *arg) {
  job *j = (job *)arg;
  for (;;) {
    const int64_t k = atomic_fetch_add(&j->next, 1);
    if (k >= j->n_keys) break;
    const lc_op *o = j->ops + j->key_off[k];
    const int64_t n = j->key_off[k + 1] - j->key_off[k];
    lc_key_result *r = &j->out[k];
    if (n < 0 || key_malformed(o, n)) {
      result_init(r);
      result_unknown(r, LC_REASON_MALFORMED);
      atomic_store(&j->malformed, 1);
      continue;
    }
    if (key_has_unknown_f(o, n)) {
      /* The reference throws inside step the first time such an op is
       * stepped; jepsen's check-safe turns that into :unknown.  The JIT
       * search may legitimately never step it (an unlinearized :info op),
       * so decide like the device path: any unknown f -> :unknown. */
      result_init(r);
      result_unknown(r, LC_REASON_UNKNOWN_F);
      continue;
    }
    if (j->algo == ORACLE_WGL)
      check_key_wgl(o, n, j->opts, j->budget, r);
    else
      check_key_jit(o, n, j->opts, j->budget, j->reduce, r);
  }
  return NULL;
}

int oracle_frontier(const lc_op *ops, int64_t n, const lc_opts *opts, int algo,
                    int64_t stop_op, int64_t *out, int64_t max, int64_t *n_out) {
  if (!ops || n < 0 || !n_out || stop_op < 0 || stop_op >= n || (max > 0 && !out)) return -EINVAL;
  if ((algo & 0xff) != ORACLE_JIT || key_malformed(ops, n)) return -EINVAL;
  lc_opts dflt = {0, LC_NIL, 0, 0, 0};
  if (!opts) opts = &dflt;
  frontier_req fr = {stop_op, out, max, 0};
  lc_key_result r;
  check_key_jit_fr(ops, n, opts,
                   opts->max_configs_per_key > 0 ? opts->max_configs_per_key : (int64_t)4000000,
                   algo & ~0xff, &r, &fr);
  *n_out = fr.n;
  return 0;
}

int oracle_check(const lc_op *ops, const int64_t *key_off, int64_t n_keys,
                 const lc_opts *opts, lc_key_result *out, int algo,
                 int n_threads) {
  lc_opts dflt;
  if (!opts) {
    dflt.init_version = 0;
    dflt.init_value = LC_NIL;
    dflt.max_configs_per_key = 0;
    dflt.time_budget_ms = 0;
    dflt.flags = 0;
    opts = &dflt;
  }
  if (n_keys < 0 || (n_keys > 0 && (!ops || !key_off || !out))) return -EINVAL;
  job j;
  j.ops = ops;
  j.key_off = key_off;
  j.n_keys = n_keys;
  j.opts = opts;
  j.out = out;
  j.algo = algo & 0xff;
  j.reduce = algo & ~0xff;
  j.budget = opts->max_configs_per_key > 0 ? opts->max_configs_per_key
                                           : (int64_t)4000000;
  atomic_init(&j.next, 0);
  atomic_init(&j.malformed, 0);
  if (n_threads < 1) n_threads = 1;
  if (n_threads == 1) {
    worker(&j);
  } else {
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)n_threads);
    if (!th) return -ENOMEM;
    for (int i = 0; i < n_threads; i++) pthread_create(&th[i], NULL, worker, &j);
    for (int i = 0; i < n_threads; i++) pthread_join(th[i], NULL);
    free(th);
  }
  return atomic_load(&j.malformed) ? -EINVAL : 0;
}
