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
    (empty? mismatch)))

(let [[dir & names] *command-line-args*
      names (or (seq names) ["kat" "c1" "tiny" "c5" "info"])
      ok    (doall (map #(check-file dir %) names))]
  (shutdown-agents)
  (System/exit (if (every? true? ok) 0 1)))
