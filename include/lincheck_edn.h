/*
 * lincheck_edn.h — offline ingestion of a Jepsen `history.edn` (SURVEY.md
 * §8(f) rank 2): the on-disk form of the history the reference's checker is
 * handed, turned into the packed records of lincheck.h without a JVM.
 *
 * What it replaces on the reference side is the host half of the checker
 * boundary: jepsen.independent's per-key split
 * (register.clj:108; values are independent tuples [k v], register.clj:28,
 * 34,43) and knossos's history completion, done in Clojure before the model's
 * step (register.clj:59-96) ever runs.  The rules are those of
 * jepsen/etcd_amd/history.py (the Python mirror) and of the JVM shim
 * jepsen/etcd_amd/clojure/jepsen/etcd/mi355x.clj:
 *
 *   - client ops only: `:process` is an integer (nemesis ops have no model
 *     step, register.clj:63);
 *   - LC_EDN_INDEPENDENT: a client op whose `:value` is a 2-element vector
 *     [k v] belongs to key k with value v; other client ops go to every key.
 *     Keys are numbered in order of first appearance.  (EDN has no
 *     MapEntry, so a tuple is recognised by shape: the register workload
 *     always wraps values, register.clj:28,34,43.)  Without the flag the
 *     whole history is one key;
 *   - per key, an :invoke is paired with the next completion of the same
 *     process: :ok copies the completion value in and sets ret = its index,
 *     :fail drops the pair, :info (or no completion) leaves the op pending
 *     forever (ret = LC_INF);
 *   - `:index` gives call/ret; an op without one gets its position in the
 *     file (0-based, all ops counted);
 *   - :f :read/:write/:cas with a value [version x] (version nil or an
 *     integer; x = [old new] for :cas) packs to (f, value, expected,
 *     version); anything else packs as f = 3 (the device reports :unknown,
 *     as the model's condp would throw).  Other models: LC_EDN_*_REGISTER,
 *     LC_EDN_MUTEX below;
 *   - values are interned per key by EDN equality (nil -> LC_NIL; integers
 *     and big integers by value, floats apart from integers, vectors equal
 *     to lists, maps and sets order-free), in the order history.py interns
 *     them (per record: cas new before old).
 *
 * EDN accepted: maps, vectors, lists, sets, strings, characters, keywords,
 * symbols, nil/true/false, integers (N suffix), floats (M suffix), ratios,
 * tagged forms (#jepsen.history.Op{...}, #inst "..." — the tag is kept in
 * the value's identity but not interpreted), #_ discards, ; comments, commas.
 * Top level: a stream of op maps (one per line, as jepsen writes it) or a
 * single vector of them.
 *
 * Threading: lc_edn_parse scans form boundaries once, then parses the forms
 * on n_threads threads; the per-key split and pairing run on one thread.
 */
#ifndef LINCHECK_EDN_H
#define LINCHECK_EDN_H

#include <stddef.h>
#include <stdint.h>

#include "lincheck.h"

#ifdef __cplusplus
extern "C" {
#endif

#define LC_EDN_INDEPENDENT 1 /* values are [k v] tuples: split per key */

/* Model (flags bits 8..11), as in jepsen/etcd_amd/history.py: how an op's
 * value becomes (value, expected, version).  The initial state is the
 * model's nil / free state (lc_opts.init_value = LC_NIL, or 0 for MUTEX). */
#define LC_EDN_VERSIONED_REGISTER (0 << 8) /* register.clj:55-96: [version x] */
#define LC_EDN_CAS_REGISTER       (1 << 8) /* knossos cas-register: x, cas [old new] */
#define LC_EDN_REGISTER           (2 << 8) /* knossos register: no :cas step */
#define LC_EDN_MUTEX              (3 << 8) /* knossos mutex (lock.clj:244): :acquire/:release
                                              as CAS free(0)->held(1) / held->free */
#define LC_EDN_MODEL_MASK         (15 << 8)

typedef struct lc_edn_history lc_edn_history;

/* Parse `len` bytes of EDN text.  On success *out owns the packed history
 * (free with lc_edn_free) and 0 is returned; on a syntax error -EINVAL and
 * a message with the byte offset in err[0..errlen). */
int lc_edn_parse(const char *text, size_t len, int64_t flags, int n_threads,
                 lc_edn_history **out, char *err, size_t errlen);

int64_t lc_edn_n_keys(const lc_edn_history *h);
int64_t lc_edn_n_ops(const lc_edn_history *h);     /* packed records */
int64_t lc_edn_n_events(const lc_edn_history *h);  /* op maps read */

/* Packed records (n_ops) and key offsets (n_keys + 1): the inputs of
 * lc_check.  Pointers stay valid until lc_edn_free. */
const lc_op *lc_edn_ops(const lc_edn_history *h);
const int64_t *lc_edn_key_off(const lc_edn_history *h);

/* The same records as 24-byte lc_op32 (n_ops) and each key's base (n_keys):
 * the inputs of lc_check32 (ABI 4), narrowed by lc_pack32's rules on the
 * first call; valid until lc_edn_free.  NULL on a null history. */
const lc_op32 *lc_edn_ops32(lc_edn_history *h);
const int64_t *lc_edn_key_base(lc_edn_history *h);

/* The same records as 16-byte lc_op16 (n_ops; round 6), the inputs of
 * lc_check16 with lc_edn_key_base's bases, packed by lc_pack16's rules on the
 * first call; NULL when some value id does not fit 15 bits (use
 * lc_edn_ops32) or on a null history.  Valid until lc_edn_free. */
const lc_op16 *lc_edn_ops16(lc_edn_history *h);

/* EDN text of key i as it first appeared (NUL-terminated). */
const char *lc_edn_key(const lc_edn_history *h, int64_t key);

/* Source text of the op maps behind packed record `rec` (global record
 * number): which = 0 the :invoke, 1 its completion (NULL when none). */
const char *lc_edn_op_text(const lc_edn_history *h, int64_t rec, int which);

/* EDN text of interned value `id` of key `key` (NULL for LC_NIL / out of
 * range). */
const char *lc_edn_value(const lc_edn_history *h, int64_t key, int64_t id);

void lc_edn_free(lc_edn_history *h);

#ifdef __cplusplus
}
#endif

#endif /* LINCHECK_EDN_H */
