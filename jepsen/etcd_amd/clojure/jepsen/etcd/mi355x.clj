(ns jepsen.etcd.mi355x
  "Drop-in jepsen.checker/Checker for the register workload's hot path.

  Replaces, as one unit, the checker built at
  src/jepsen/etcd/register.clj:108-112:

    (independent/checker
      (checker/compose
        {:linear   (checker/linearizable {:model (->VersionedRegister 0 nil)})
         :timeline (timeline/html)}))

  The JVM side does the host preprocessing (client ops only, the independent
  per-key split, knossos-style invoke/completion pairing with :fail pairs
  dropped and :info ops pending forever, per-key value interning by Clojure
  =) and packs one 16-byte lc_op16 record per operation (24-byte lc_op32
  when some value id does not fit 15 bits) into off-heap memory
  (ABI 5: a third of the PCIe bytes of the 48-byte lc_op; the 24-byte form
  holds the int32 fields the device reads).  One lc_check16 / lc_check32
  call (JNA, liblincheck.so; C ABI in
  include/lincheck.h) then decides every key on the MI355X GPUs of the
  control node.  The result has
  jepsen.independent/checker's shape, and each key's entry has
  checker/compose's shape: {:valid? merged, :linear <the GPU verdict>,
  :timeline <jepsen's own timeline/html over that key's subhistory, written
  under the key's independent/ subdirectory>}.  Only :linear moves to the
  GPU; the timeline stays jepsen's renderer (pass :timeline? false to skip
  it, e.g. for benchmarks).

  Usage, in register.clj's workload:

    :checker (jepsen.etcd.mi355x/checker)

  An invalid key's :linear map carries knossos's diagnostics: :op,
  :previous-ok, :configs and :final-paths — up to 10 configurations of the
  JIT search's frontier just before the failing return, for every invalid
  key from one batched device search (lc_check_frontiers,
  include/lincheck_fx.h) and, for a key whose frontier outgrows it, from the
  frontier exchange alone (lc_fx_frontier); for keys the version-order and
  gap tiers decided, also the :last-op of the prefix witness (lc_aux); the
  witness's one configuration stands in where no frontier could be had.  :final-paths step the reference's own model
  (jepsen.etcd.register/->VersionedRegister, register.clj:55-96) through
  knossos.model/step, so the messages are the model's own
  (jepsen/etcd_amd/diagnostics.py restates the same).  A key with malformed
  records is :unknown alone.

  Untested in the build container (no JVM there); the same contract is
  exercised from Python by tests/test_gpu.py::test_register_checker_end_to_end."
  (:require [jepsen.checker :as checker]
            [jepsen.checker.timeline :as timeline]
            [jepsen.independent :as independent]
            [knossos.model :as model])
  (:import (com.sun.jna Function Memory NativeLibrary Pointer)
           (com.sun.jna.ptr PointerByReference)))

(def ^:const LC_NIL -1)
(def ^:const LC_FLAG_WHOLE_GPU 8)  ; include/lincheck.h
(def ^:const LC_INF Long/MAX_VALUE)
(def ^:const op-bytes 48)      ; lc_op (the frontier searches)
(def ^:const op32-bytes 24)    ; lc_op32 (lc_check32, ABI 4)
(def ^:const op16-bytes 16)    ; lc_op16 (lc_check16, round 6): value ids within 15 bits
(def ^:const id15-max 0x7FFD)  ; LC_ID15_MAX
(def ^:const field-max 0x7FFFFFFE)
(def ^:const never 0xFFFFFFFF)
(def ^:const result-bytes 40)

(defonce ^:private lib
  (delay (NativeLibrary/getInstance
           (or (System/getenv "LINCHECK_LIB") "lincheck"))))

(defn- fun ^Function [name] (.getFunction ^NativeLibrary @lib name))

(def ^:const abi-min 5)  ; lc_check16 / lc_check32 / lc_check_frontiers (include/lincheck.h LC_ABI_VERSION)

(defonce ^:private ctx
  (delay
    (let [abi (.invokeInt (fun "lc_abi_version") (object-array []))
          _   (when (< abi abi-min)
                (throw (ex-info "liblincheck.so is older than this shim's ABI"
                                {:abi abi :need abi-min})))
          out (PointerByReference.)
          rc  (.invokeInt (fun "lc_open") (object-array [(int 0) out]))]
      (when-not (zero? rc)
        (throw (ex-info "lc_open failed: no usable GPU (no CPU fallback)"
                        {:rc rc})))
      (.getValue out))))

(defn- client-op? [op] (integer? (:process op)))

(defn- subhistories
  "{k [op ...]}: jepsen.independent's split of the client ops in one pass
  over the history; tuple values are unwrapped, non-tuple ops go to every
  key (in history order, interleaved with the key's own ops)."
  [history]
  (let [ops   (filterv client-op? history)
        ;; first pass over the ops: the keys, in order of appearance
        order (->> ops
                   (keep (fn [op] (let [v (:value op)] (when (independent/tuple? v) (key v)))))
                   distinct
                   vec)
        ;; second pass: route each op to its key (or to every key)
        subs  (reduce (fn [m op]
                        (let [v (:value op)]
                          (if (independent/tuple? v)
                            (assoc! m (key v) (conj! (get m (key v)) (assoc op :value (val v))))
                            (reduce (fn [m k] (assoc! m k (conj! (get m k) op))) m order))))
                      (transient (zipmap order (repeatedly #(transient []))))
                      ops)
        subs  (persistent! subs)]
    (into (array-map) (for [k order] [k (persistent! (get subs k))]))))

(defn- complete
  "knossos-style completion of one key: [{:op invoke-with-completed-value
  :call i :ret j-or-INF :completion c}] in invoke order, :fail pairs dropped."
  [ops]
  (loop [ops ops, pending {}, out []]
    (if-let [op (first ops)]
      (let [p (:process op)]
        (case (:type op)
          :invoke (recur (rest ops) (assoc pending p (count out))
                         (conj out {:op op :call (:index op) :ret LC_INF}))
          (:ok :fail :info)
          (if-let [i (pending p)]
            (recur (rest ops) (dissoc pending p)
                   (update out i
                           (fn [r]
                             (case (:type op)
                               :ok   (assoc r :op (assoc (:op r) :value (:value op))
                                              :ret (:index op) :completion op)
                               :fail (assoc r :fail? true)
                               :info (assoc r :completion op)))))
            (recur (rest ops) pending out))
          (recur (rest ops) pending out)))
      (vec (remove :fail? out)))))

(defn- interner
  "A value -> dense id fn (nil -> LC_NIL); (intern) with no argument returns
  the id -> value map."
  []
  (let [ids (volatile! {})]
    (fn
      ([] (into {} (map (fn [[v i]] [i v])) @ids))
      ([v]
       (if (nil? v)
         LC_NIL
         (or (@ids v)
             (let [i (count @ids)] (vswap! ids assoc v i) i)))))))

(defn- record
  "[f value expected version call ret] for one completed op under model
  (register.clj:22-44, 98-100 for :versioned-register); f 3 (unknown) if the
  shape does not match, which the GPU reports as :unknown like the model's
  throwing step (:63).  Other knossos models are packings of the same
  records (jepsen/etcd_amd/history.py, \"Models\"): :cas-register and
  :register values carry no version; :mutex (lock.clj:244) packs :acquire
  as a CAS free(0) -> held(1) and :release as the reverse."
  [model intern {:keys [op call ret]}]
  (case model
    :mutex
    (case (:f op)
      :acquire [2 1 0 LC_NIL call ret]
      :release [2 0 1 LC_NIL call ret]
      [3 LC_NIL LC_NIL LC_NIL call ret])

    (:cas-register :register)
    (let [v (:value op)
          f (case (:f op) :read 0 :write 1 :cas (if (= model :register) 3 2) 3)]
      (cond (= f 3)                                 [3 LC_NIL LC_NIL LC_NIL call ret]
            (and (= f 2) (not (and (sequential? v) (= 2 (count v)))))
                                                    [3 LC_NIL LC_NIL LC_NIL call ret]
            (= f 2) [2 (intern (second v)) (intern (first v)) LC_NIL call ret]
            :else   [f (intern v) LC_NIL LC_NIL call ret]))

    (let [[version v] (:value op)
          f (case (:f op) :read 0 :write 1 :cas 2 3)]
      (if (or (= f 3) (and (some? version) (not (integer? version)))
              (and (= f 2) (not (sequential? v))))
        [3 LC_NIL LC_NIL LC_NIL call ret]
        (let [ver (if (nil? version) LC_NIL (long version))]
          (if (= f 2)
            [2 (intern (second v)) (intern (first v)) ver call ret]
            [f (intern v) LC_NIL ver call ret]))))))

(defn- narrow
  "One record [f v e ver call ret] as the six int32 words of an lc_op32, by
  lc_pack32's rules (include/lincheck.h): call / ret relative to the key's
  base (its first call), -1 (LC_INF32) for a pending op; a version no state
  reaches becomes 2^31-2, an unknown :f 3, and a record the device rejects as
  malformed keeps value -2 (the arithmetic wraps as the library's does)."
  [^long base [f v e ver call ret]]
  (let [f (long f), v (long v), e (long e), ver (long ver), call (long call), ret (long ret)
        rc  (unchecked-subtract call base)
        rr  (unchecked-subtract ret base)
        inf (= ret LC_INF)
        bad (or (< v -1) (> v field-max) (< e -1) (> e field-max) (neg? call) (<= ret call)
                (neg? rc) (>= rc never) (and (not inf) (>= rr never)))
        lo  (fn [^long x] (unchecked-int (bit-and x 0xFFFFFFFF)))]
    [(if (<= 0 f 2) f 3)
     (if bad -2 (unchecked-int v))
     (unchecked-int e)
     (if (or (< ver -1) (> ver field-max)) field-max ver)
     (lo rc)
     (cond inf -1                                        ; LC_INF32
           (= (bit-and rr 0xFFFFFFFF) 0xFFFFFFFF) -2     ; LC_INF32 - 1
           :else (lo rr))]))

(defn- key-records
  "One key's records [f v e ver call ret], values interned in record order
  (so the ids are the ones its packing used), and its id -> value map."
  [model d]
  (let [intern (interner)
        rs     (mapv #(record model intern %) d)]
    [rs (intern)]))

(defn- fits16?
  "Whether an lc_op32 record (six ints) fits an lc_op16 (include/lincheck.h,
  round 6): a malformed one always (value -2), else value and expected ids
  within [-1, LC_ID15_MAX]."
  [^ints arr ^long b]
  (let [v (aget arr (+ b 1)), e (aget arr (+ b 2))]
    (or (= v -2) (and (<= -1 v id15-max) (<= -1 e id15-max)))))

(defn- to16
  "lc_pack16's record from lc_pack32's (six ints at b): f << 30 | (value + 1)
  << 15 | (expected + 1), version, call, ret; a malformed record's value field
  0x7FFF, its expected clamped."
  [^ints arr ^long b]
  (let [f (long (aget arr b)), v (long (aget arr (+ b 1))), e (long (aget arr (+ b 2)))
        v15 (if (= v -2) 0x7FFF (inc v))
        x15 (max 0 (min 0x7FFF (inc e)))]
    [(unchecked-int (bit-or (bit-shift-left f 30) (bit-shift-left v15 15) x15))
     (aget arr (+ b 3)) (aget arr (+ b 4)) (aget arr (+ b 5))]))

(defn- pack
  "Packs all keys as 16-byte lc_op16 records when every value id fits 15
  bits, else as 24-byte lc_op32 records: returns [keys completed-per-key
  ^Memory ops ^Memory key-off ^Memory key-base n-records values-per-key
  record-bytes] (values: each key's id -> value map).  Records are filled
  into one int[] and written to the off-heap buffer in a single bulk copy."
  [model subs]
  (let [keys  (vec (keys subs))
        nk    (count keys)
        done  (mapv (fn [k] (complete (get subs k))) keys)
        n     (long (reduce + (map count done)))
        arr   (int-array (* 6 n))
        offs  (long-array (inc nk))
        bases (long-array (max 1 nk))
        vals  (transient [])]
    (loop [ki 0, i 0]
      (aset offs ki i)
      (when (< ki nk)
        (let [[rs vm] (key-records model (nth done ki))
              base    (if (seq rs) (long (nth (first rs) 4)) 0)
              i'      (reduce (fn [^long i r]
                                (let [w (narrow base r), b (* 6 i)]
                                  (dotimes [j 6] (aset arr (+ b j) (unchecked-int (nth w j))))
                                  (inc i)))
                              i rs)]
          (aset bases ki base)
          (conj! vals vm)
          (recur (inc ki) i'))))
    (let [w16 (loop [i 0] (cond (>= i n) true
                                (fits16? arr (* 6 i)) (recur (inc i))
                                :else false))
          rb  (if w16 op16-bytes op32-bytes)
          ops (Memory. (max 1 (* rb n)))
          off (Memory. (* 8 (inc nk)))
          bm  (Memory. (* 8 (max 1 nk)))]
      (if w16
        (let [a16 (int-array (* 4 n))]
          (dotimes [i n]
            (let [q (to16 arr (* 6 i))]
              (dotimes [j 4] (aset a16 (+ (* 4 i) j) (unchecked-int (nth q j))))))
          (.write ops 0 a16 0 (alength a16)))
        (.write ops 0 arr 0 (alength arr)))
      (.write off 0 offs 0 (alength offs))
      (.write bm 0 bases 0 (alength bases))
      [keys done ops off bm n (persistent! vals) rb])))

(defn- pack48
  "The 48-byte lc_op records of some keys (the frontier searches take
  them): [^Memory ops long[] key-off]."
  [model done kis]
  (let [rss  (mapv #(first (key-records model (nth done %))) kis)
        n    (long (reduce + (map count rss)))
        arr  (long-array (max 1 (* 6 n)))
        offs (long-array (inc (count kis)))]
    (loop [j 0, i 0]
      (aset offs j i)
      (when (< j (count kis))
        (recur (inc j)
               (reduce (fn [^long i r]
                         (dotimes [x 6] (aset arr (+ (* 6 i) x) (long (nth r x))))
                         (inc i))
                       i (nth rss j)))))
    (let [ops (Memory. (max 1 (* op-bytes n)))]
      (.write ops 0 arr 0 (alength arr))
      [ops offs])))

;; ---- knossos's invalid-analysis keys (diagnostics.py restates the same)

(defn- ref-model
  "The reference's own model, register.clj:55 (->VersionedRegister version
  value), resolved at run time from the test's classpath: :final-paths step
  it through knossos.model/step, so every message is the model's own."
  [version value]
  ((requiring-resolve 'jepsen.etcd.register/->VersionedRegister) version value))

(defn- model-map [m] (if (model/inconsistent? m) m {:version (:version m) :value (:value m)}))

(defn- op-map [r] (if (not= LC_INF (:ret r)) (:completion r) (:op r)))

(defn- final-paths
  "From each [model last-index pending-indices] configuration, the paths that
  try to linearize the failing op — directly, or after one pending op — and
  end inconsistent; at most 10, as knossos keeps."
  [done fail-op configs]
  (let [try-op (fn [m i] (let [m' (model/step m (:op (nth done i)))]
                           [m' {:op (op-map (nth done i)) :model (model-map m')}]))]
    (->> (for [[m last-i pending] configs
               :let [head   {:op (when last-i (op-map (nth done last-i))) :model (model-map m)}
                     [d end] (try-op m fail-op)]
               path (cons (when (model/inconsistent? d) [head end])
                          (for [i pending :when (not= i fail-op)
                                :let [[m' mid] (try-op m i)]
                                :when (or (model/inconsistent? m')
                                          (model/inconsistent? (first (try-op m' fail-op))))]
                            (if (model/inconsistent? m')
                              [head mid]
                              [head mid (second (try-op m' fail-op))])))
               :when path]
           path)
         (take 10)
         vec)))

(defn- previous-ok [done fail-ret]
  (let [oks (filter #(and (= :ok (:type (:completion %))) (< (:ret %) fail-ret)) done)]
    (when (seq oks) (:completion (apply max-key :ret oks)))))

(defn- witness-analysis
  ":configs [the one configuration the prefix witness names], :last-op and
  :final-paths, for keys the version-order / gap tiers decided."
  [done fail-op fail-ret witness [v0 x0]]
  (let [cut   (dec fail-ret)
        muts  (->> (map-indexed vector witness) (filter #(>= (second %) 0))
                   (sort-by second) (map first))
        state (reduce (fn [m i] (if (model/inconsistent? m) m (model/step m (:op (nth done i)))))
                      (ref-model v0 x0) muts)]
    (when-not (model/inconsistent? state)
      (let [lin      (set muts)
            freads   (->> (map-indexed vector done)
                          (filter (fn [[_ r]] (and (= :read (:f (:op r))) (<= (:ret r) cut)
                                                   (= (first (:value (:op r))) (:version state)))))
                          (map first))
            last-i   (if (seq freads) (apply max-key #(:ret (nth done %)) freads) (last muts))
            last-op  (when last-i (op-map (nth done last-i)))
            pending  (->> (range (count done))
                          (filter #(let [r (nth done %)]
                                     (and (<= (:call r) cut) (not (lin %)) (> (:ret r) cut)))))]
        {:configs     [{:model (model-map state) :last-op last-op
                        :pending (mapv #(:op (nth done %)) pending)}]
         :last-op     last-op
         :final-paths (final-paths done fail-op [[state last-i pending]])}))))

(def ^:const fx-config-bytes 536)  ; lc_fx_config: version, value, n_pending, pending[64]

(defonce ^:private fx-engine
  (delay
    (let [prm (doto (Memory. 40) (.clear)
                (.setInt 0 0) (.setInt 4 1)            ; device 0, one rank
                (.setLong 8 -1) (.setLong 16 -1))      ; default thresholds
          out (PointerByReference.)
          rc  (.invokeInt (fun "lc_fx_open") (object-array [prm nil out]))]
      (when-not (zero? rc) (throw (ex-info "lc_fx_open failed" {:rc rc})))
      (.getValue out))))

(defn- configs-analysis
  ":configs and :final-paths from [[version value-id pending-record-indices]
  ...], a frontier search's configurations just before the failing return."
  [model done fail-op vals configs]
  (let [configs (for [[ver vid pending] configs]
                  [ver (when (not= vid LC_NIL) (get vals vid vid)) pending])]
    (cond-> {:configs (vec (for [[ver x pending] configs]
                             {:model (if (= model :versioned-register)
                                       {:version ver :value x}
                                       {:value x})
                              :pending (mapv #(:op (nth done %)) pending)}))}
      (= model :versioned-register)
      (assoc :final-paths
             (final-paths done fail-op
                          (for [[ver x pending] configs] [(ref-model ver x) nil pending]))))))

(defn- read-configs
  "n lc_fx_config structs from buf at byte offset b0."
  [^Memory buf b0 n]
  (vec (for [i (range n)
             :let [b (+ b0 (* i fx-config-bytes))]]
         [(.getLong buf b) (.getLong buf (+ b 8))
          (vec (for [j (range (.getLong buf (+ b 16)))] (.getLong buf (+ b 24 (* 8 j)))))])))

(defn- batched-configs
  "knossos's :configs of every invalid key in one device call
  (lc_check_frontiers, include/lincheck_fx.h): {:configs {key-index
  configurations}, :ops ^Memory, :off long[], :at {key-index j}} — the keys the
  device search could not take (a frontier beyond its tiers) are left out of
  :configs; :ops / :off / :at hold their 48-byte records for lc_fx_frontier."
  [model done inv o]
  (let [kis         (mapv first inv)
        [ops offs]  (pack48 model done kis)
        nk          (count kis)
        off         (doto (Memory. (* 8 (inc nk))) (.write 0 offs 0 (alength offs)))
        stops       (long-array (map second inv))
        stop        (doto (Memory. (* 8 (max 1 nk))) (.write 0 stops 0 (alength stops)))
        buf         (Memory. (* (max 1 nk) 10 fx-config-bytes))
        cnt         (Memory. (* 4 (max 1 nk)))
        rc          (try
                      (locking ctx
                        (.invokeInt (fun "lc_check_frontiers")
                                    (object-array [@ctx ops off (long nk) stop o buf (int 10) cnt])))
                      ;; diagnostics only: the verdict stands whatever happens here
                      (catch Exception e e))
        ok?         (and (number? rc) (zero? rc))]
    {:ops ops :off offs :at (zipmap kis (range))
     :configs (if-not ok?
                {}
                (into {} (for [j (range nk)
                               :let [c (.getInt cnt (* 4 j))]
                               :when (>= c 0)]
                           [(nth kis j) (read-configs buf (* j 10 fx-config-bytes) c)])))}))

(defn- fx-frontier
  "One key's frontier search alone, up to its failing return
  (lc_fx_frontier): its configurations, or {:configs-error ...}."
  [^Memory ops ^long k0 n fail-op opts]
  (let [buf (Memory. (* 10 fx-config-bytes))
        cnt (Memory. 4)
        rc  (try
              (locking fx-engine
                (.invokeInt (fun "lc_fx_frontier")
                            (object-array [@fx-engine (.share ops (* op-bytes k0))
                                           (long n) opts (long fail-op) buf (int 10) cnt])))
              ;; diagnostics only: the verdict stands whatever happens here
              (catch Exception e e))]
    (if (and (number? rc) (zero? rc))
      (read-configs buf 0 (.getInt cnt 0))
      {:configs-error (if (number? rc) [:lc-fx-frontier rc] (str rc))})))

(def ^:private cert-kinds {0 :none 1 :dup 2 :unreach 3 :claims 4 :pair 5 :order 6 :hall 7 :proof})

;; an invalid key the batched device search could not take gets :configs from
;; the frontier exchange alone when the frontier search decided it, or the
;; version-order / gap tiers did and it has at most this many crashed ops; at
;; most frontier-max-keys such searches per check (checker.py counts the same
;; way: a search is counted when it runs, and runs while the count is below
;; the cap)
(def ^:private frontier-max-crashed 16)
(def ^:private frontier-max-keys 1000)

(defn- merge-valid [vs]
  (cond (some false? vs)          false
        (some #{:unknown} vs)     :unknown
        :else                     true))

(def ^:private reasons
  {2 :config-budget 3 :window-overflow 4 :malformed 5 :unknown-f 7 :time-budget})

(defn- check-keys
  "One lc_check32 over subs {k [op ...]}: {k result-map}.  Malformed keys
  come back :unknown one by one; lc_check32 fails (and this throws, for
  check-safe) only on unusable arguments or a GPU error."
  [model max-configs-per-key time-budget-ms flags subs]
  (let [[keys done ops off base n vals rb] (pack model subs)
        check-fn (if (= rb op16-bytes) "lc_check16" "lc_check32")
        n-fallback (atom 0)
        nk   (count keys)
        out  (Memory. (* result-bytes nk))
        wit  (Memory. (max 4 (* 4 n)))
        kind (Memory. (max 4 (* 4 nk)))
        cert (Memory. (max 16 (* 16 nk)))       ; lc_aux certificates (ABI 3): 4 int32 per key
        cset (Memory. (max 4 (* 4 n)))
        aux  (doto (Memory. 32) (.setPointer 0 wit) (.setPointer 8 kind)
               (.setPointer 16 cert) (.setPointer 24 cset))
        o    (doto (Memory. 40)
               (.setLong 0 0) (.setLong 8 (if (= model :mutex) 0 LC_NIL))
               (.setLong 16 max-configs-per-key)
               (.setLong 24 time-budget-ms) (.setLong 32 flags))
        rc   (locking ctx
               (.invokeInt (fun check-fn)
                           (object-array [@ctx ops off base (long nk) o out aux])))]
    (when-not (zero? rc)
      (throw (ex-info (str check-fn " failed")
                      {:rc rc :error (.invoke (fun "lc_last_error")
                                              String (object-array [@ctx]))})))
    (let [inv (vec (for [ki (range nk)
                         :let [b (* ki result-bytes)]
                         :when (zero? (.getInt out b))]
                     [ki (.getLong out (+ b 8))]))
          bc  (when (seq inv) (batched-configs model done inv o))]
      (into (array-map)
            (for [ki (range nk)]
              (let [b       (* ki result-bytes)
                    verdict (.getInt out b)
                    reason  (.getInt out (+ b 4))
                    fail-op (.getLong out (+ b 8))
                    fail-at (.getLong out (+ b 16))
                    v       (case verdict 1 true 0 false :unknown)
                    d       (nth done ki)
                    k0      (.getLong off (* 8 ki))
                    witnessed (and (false? v) (= model :versioned-register)
                                   (= 2 (.getInt kind (* 4 ki))))  ; LC_WITNESS_PREFIX
                    witness (when witnessed (vec (.getIntArray wit (* 4 k0) (count d))))]
                [(nth keys ki)
                 ;; the same keys as checker.py's map for the same history
                 (cond-> {:valid?   v
                          :analyzer :mi355x
                          :configs-explored (.getLong out (+ b 24))
                          :max-frontier (.getLong out (+ b 32))}
                   (false? v)     (merge {:op (op-map (nth d fail-op))
                                          :fail-prefix-end fail-at
                                          :previous-ok (previous-ok d fail-at)
                                          ;; why the prefix at the failing return has no
                                          ;; linearization (include/lincheck.h LC_CERT_*)
                                          :certificate
                                          (let [c (.getIntArray cert (* 16 ki) 4)
                                                kd (get cert-kinds (aget c 0) :none)
                                                rec #(when (>= % 0) (op-map (nth d %)))]
                                            (cond-> {:kind kd}
                                              (#{:dup :unreach :claims :pair :order} kd)
                                              (assoc :ops (vec (keep rec [(aget c 1) (aget c 2)])))
                                              (= kd :hall)
                                              (assoc :positions
                                                     (vec (.getIntArray cset (* 4 k0) (aget c 3))))
                                              ;; the case splits, [position cases] in preorder
                                              (= kd :proof)
                                              (assoc :splits
                                                     (mapv (fn [t] [(bit-and (bit-shift-right t 15) 0x7FFF)
                                                                    (bit-and t 0x7FFF)])
                                                           (.getIntArray cset (* 4 k0) (aget c 3))))))}
                                         (let [wa (when witness
                                                    (witness-analysis d fail-op fail-at witness
                                                                      [0 nil]))
                                               ;; knossos's :configs: the frontier search's
                                               ;; own, up to the failing return — batched on
                                               ;; the device, else this key alone
                                               cs (or (get-in bc [:configs ki])
                                                      (when (and (< @n-fallback frontier-max-keys)
                                                                 (or (not witnessed)
                                                                     (<= (count (filter
                                                                                 #(= LC_INF (:ret %)) d))
                                                                         frontier-max-crashed)))
                                                        (swap! n-fallback inc)
                                                        (fx-frontier (:ops bc)
                                                                     (aget ^longs (:off bc)
                                                                           (get (:at bc) ki))
                                                                     (count d) fail-op o)))
                                               fa (cond (vector? cs)
                                                        (configs-analysis model d fail-op (nth vals ki) cs)
                                                        (map? cs) cs)]
                                           (cond (and fa (:configs fa))
                                                 (cond-> fa (:last-op wa) (assoc :last-op (:last-op wa)))
                                                 wa (merge wa (select-keys fa [:configs-error]))
                                                 :else fa)))
                   (= v :unknown) (assoc :cause (reasons reason reason)
                                         :error [:lincheck-reason (reasons reason reason)]))]))))))

(defn linearizable
  "(checker/linearizable {:model m}) over the whole history, for the knossos
  models this library packs: opts :model one of :versioned-register,
  :cas-register, :register, :mutex.  The lock workload's checker
  (lock.clj:243-244) becomes (linearizable {:model :mutex})."
  [{:keys [model max-configs-per-key time-budget-ms whole-gpu?]
    :or {model :versioned-register max-configs-per-key 0 time-budget-ms 0 whole-gpu? true}}]
  (reify checker/Checker
    (check [_ test history _opts]
      (let [ops (filterv client-op? history)]
        (if (empty? ops)
          {:valid? true :analyzer :mi355x}
          (get (check-keys model max-configs-per-key time-budget-ms
                           (if whole-gpu? LC_FLAG_WHOLE_GPU 0) {nil ops}) nil))))))

(defn- render-linear!
  "What jepsen's checker/linearizable does with a failed analysis: knossos's
  own renderer draws it into the key's directory as linear.svg.  A rendering
  error is swallowed (jepsen only warns); it never changes the verdict."
  [test subdir sub linear]
  (when (and (false? (:valid? linear)) (seq (:final-paths linear)))
    (try
      (let [render! (requiring-resolve 'knossos.linear.report/render-analysis!)
            path!   (requiring-resolve 'jepsen.store/path!)
            ^java.io.File f (path! test subdir "linear.svg")]
        (render! sub linear (.getCanonicalPath f)))
      (catch Throwable _ nil))))

(defn- composed
  "checker/compose's per-key map (register.clj:109-112): the GPU's :linear
  result beside jepsen's own timeline/html, which renders into the key's
  independent/ subdirectory as jepsen.independent/checker would direct it
  (plus linear.svg for an invalid key, as checker/linearizable writes it)."
  [test opts k sub linear timeline?]
  (if-not timeline?
    {:valid? (:valid? linear) :linear linear}
    (let [subdir (concat (:subdirectory opts) ["independent" k])
          _      (render-linear! test subdir sub linear)
          tl     (checker/check-safe (timeline/html) test sub
                                     {:subdirectory subdir :history-key k})]
      {:valid?   (merge-valid [(:valid? linear) (:valid? tl)])
       :linear   linear
       :timeline tl})))

(defn checker
  "The drop-in (see ns doc).  opts: :max-configs-per-key (0 = default),
  :model (default :versioned-register, register.clj:111), :timeline?
  (default true: keep register.clj:112's timeline/html per key),
  :time-budget-ms (0 = none: a key whose frontier search runs longer is
  :unknown, as knossos's aborts are), :whole-gpu? (default true: a key one
  workgroup's search leaves :unknown at the configuration budget is searched
  again over the whole GPU, LC_FLAG_WHOLE_GPU, include/lincheck_fx.h, as
  knossos keeps searching until it runs out of memory or time)."
  ([] (checker {}))
  ([{:keys [max-configs-per-key model timeline? time-budget-ms whole-gpu?]
     :or {max-configs-per-key 0 model :versioned-register timeline? true time-budget-ms 0
          whole-gpu? true}}]
   (reify checker/Checker
     (check [_ test history opts]
       (let [subs (subhistories history)]
         (if (empty? subs)
           {:valid? true :results {} :failures []}
           (let [linear  (check-keys model max-configs-per-key time-budget-ms
                                     (if whole-gpu? LC_FLAG_WHOLE_GPU 0) subs)
                 results (into (array-map)
                               (for [[k r] linear]
                                 [k (composed test opts k (get subs k) r timeline?)]))]
             {:valid?   (merge-valid (map :valid? (vals results)))
              :results  results
              :failures (vec (for [[k r] results :when (false? (:valid? r))] k))})))))))
