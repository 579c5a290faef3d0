;; JVM parity kit: the reference's own checker over the exported golden
;; histories, diffed against the verdicts the GPU tests pin.
;;
;; Run from a checkout of the reference (bsbds/jepsen.etcd, whose project.clj
;; pulls jepsen 0.3.x and knossos), with this repo's tests/golden/edn on disk:
;;
;;   lein run -m clojure.main /path/to/repo/tools/jvm_parity/parity.clj \
;;       /path/to/repo/tests/golden/edn [c1 c5 info tiny kat]
;;
;; For each name it reads <name>.edn.gz (one Jepsen op map per line, written
;; by tests/golden/make_edn.py), rebuilds the independent tuples, runs
;;
;;   (independent/checker (checker/linearizable
;;                          {:model (register/->VersionedRegister 0 nil)}))
;;
;; — the checker register.clj:108-111 builds, with the model taken from the
;; reference's own jepsen.etcd.register namespace (never a copy) — and compares
;; every key's :valid? with <name>.expected.edn, and an invalid key's :op
;; :index with the expected failing completion.  Knossos returns :unknown when
;; it runs out of memory or time; those keys are counted apart, not as
;; mismatches.  Prints one summary line per file and exits non-zero on any
;; verdict mismatch.  (Knossos's reported :op can legitimately differ from the
;; canonical first failing return when its WGL analyzer wins the race, so op
;; differences are reported but do not fail the run.)
;;
;; With MI355X_SHIM set to this repo's jepsen/etcd_amd/clojure/jepsen/etcd/
;; mi355x.clj (and LINCHECK_LIB to the built liblincheck.so, ABI >= 4 — the
;; shim checks lc_abi_version), the drop-in runs on the same history too:
;; (jepsen.etcd.mi355x/checker {:timeline? false}), i.e. lc_check32 plus
;; lc_check_frontiers for the invalid keys' :configs.  Its verdicts must equal
;; the expected ones on every key (the drop-in never answers :unknown on these
;; fixtures), its invalid keys' :op :index the expected failing completion, and
;; every key knossos decides must get the same verdict from both.
(ns mi355x.parity
  (:require [clojure.edn :as edn]
            [clojure.java.io :as io]
            [clojure.string :as str]
            [jepsen.checker :as checker]
            [jepsen.independent :as independent]
            [jepsen.etcd.register :as register])
  (:import (java.util.zip GZIPInputStream)))

(defn- read-history [path]
  (with-open [r (io/reader (GZIPInputStream. (io/input-stream path)))]
    (->> (line-seq r)
         (remove str/blank?)
         (mapv (fn [line]
                 (let [op (edn/read-string line)
                       v  (:value op)]
                   ;; EDN has no MapEntry: [k v] values become independent tuples
                   (if (and (vector? v) (= 2 (count v)))
                     (assoc op :value (independent/tuple (first v) (second v)))
                     op)))))))

(defn- as-history
  "jepsen 0.3.x checkers take a jepsen.history when that namespace exists,
  a vector of op maps before it."
  [ops]
  (if-let [f (try (requiring-resolve 'jepsen.history/history)
                  (catch Exception _ nil))]
    (f ops)
    ops))

(def ^:private dropin
  (delay (when-let [shim (System/getenv "MI355X_SHIM")]
           (load-file shim)
           ((requiring-resolve 'jepsen.etcd.mi355x/checker) {:timeline? false}))))

(defn- check-dropin
  "The drop-in on the same history: its verdicts and fail ops against the
  expected ones, and against knossos's where knossos decided.  True when
  there is no mismatch (or no shim)."
  [name hist expected res]
  (if-let [chk @dropin]
    (let [t0   (System/nanoTime)
          dres (checker/check chk {:name (str "mi355x-dropin-" name)} (as-history hist) {})
          secs (/ (- (System/nanoTime) t0) 1e9)
          rows (for [[k {:keys [valid? op-index]}] expected]
                 (let [d (get-in dres [:results k])
                       r (get-in res [:results k :valid?])]
                   {:key k :want valid? :got (:valid? d) :knossos r
                    :op-want op-index :op-got (get-in d [:linear :op :index])}))
          bad  (filter #(or (not= (:want %) (:got %))
                            (and (false? (:want %)) (not= (:op-want %) (:op-got %)))
                            (and (boolean? (:knossos %)) (not= (:knossos %) (:got %))))
                       rows)]
      (println (format "%s: drop-in %d keys, %d mismatches (verdict, fail op or vs knossos), %.2f s"
                       name (count rows) (count bad) secs))
      (doseq [m (take 10 bad)] (println "  drop-in mismatch" m))
      (empty? bad))
    true))

(defn- check-file [dir name]
  (let [hist     (read-history (io/file dir (str name ".edn.gz")))
        expected (edn/read-string (slurp (io/file dir (str name ".expected.edn"))))
        chk      (independent/checker
                   (checker/linearizable {:model (register/->VersionedRegister 0 nil)}))
        t0       (System/nanoTime)
        res      (checker/check chk {:name (str "mi355x-parity-" name)} (as-history hist) {})
        secs     (/ (- (System/nanoTime) t0) 1e9)
        rows     (for [[k {:keys [valid? op-index]}] expected]
                   (let [r (get-in res [:results k])
                         v (:valid? r)]
                     {:key k :want valid? :got v
                      :op-want op-index :op-got (get-in r [:op :index])}))
        unknown  (filter #(= :unknown (:got %)) rows)
        mismatch (remove #(or (= :unknown (:got %)) (= (:want %) (:got %))) rows)
        op-diff  (filter #(and (false? (:got %)) (false? (:want %))
                               (not= (:op-want %) (:op-got %))) rows)]
    (println (format "%s: %d keys, %d verdict mismatches, %d knossos :unknown, %d op differences, %.1f s"
                     name (count rows) (count mismatch) (count unknown) (count op-diff) secs))
    (doseq [m (take 10 mismatch)] (println "  mismatch" m))
    (and (empty? mismatch) (check-dropin name hist expected res))))

(let [[dir & names] *command-line-args*
      names (or (seq names) ["kat" "c1" "tiny" "c5" "info"])
      ok    (doall (map #(check-file dir %) names))]
  (shutdown-agents)
  (System/exit (if (every? true? ok) 0 1)))
