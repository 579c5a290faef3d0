// synth.cpp — seeded synthetic register histories (see include/lincheck_synth.h).
//
// Workload shape follows /root/reference/src/jepsen/etcd/register.clj:98-119:
// half the processes only read (gen/reserve n r, :118), the rest mix writes and
// CAS 50/50 (gen/mix [w cas], :117) with values uniform in 0..n_values-1
// (:99-100).  Completion values follow the client at :22-44: an ok read reports
// [version value] ([nil nil] while the key does not exist), an ok write/CAS
// reports [prev-version+1 ...], a CAS whose expected value mismatches is :fail.
#include <errno.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <queue>
#include <thread>
#include <vector>
#include <atomic>

#include "../../../include/lincheck_synth.h"

namespace {

struct Rng {
  uint64_t s[4];
  static uint64_t splitmix(uint64_t &x) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
  }
  Rng(uint64_t seed, uint64_t key) {
    uint64_t x = seed ^ (key * 0xD1B54A32D192ED03ULL);
    for (auto &v : s) v = splitmix(x);
  }
  static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {  // xoshiro256**
    const uint64_t r = rotl(s[1] * 5, 7) * 9;
    const uint64_t t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 45);
    return r;
  }
  double uniform() { return (double)(next() >> 11) * 0x1.0p-53; }
  double expo(double mean) { return -std::log1p(-uniform()) * mean; }
  int below(int n) { return (int)((next() >> 33) % (uint64_t)n); }
};

struct SimOp {
  int f;
  int64_t value, expected, version;
  double call_t, lin_t, ret_t;  // ret_t = inf for crashed
  int status;                   // LC_SYNTH_*
  bool effect;                  // crashed op takes effect
  bool lost;                    // the injected lost CAS (never made :info)
  int32_t slot;                 // worker slot (process ids: slot + conc * crashes so far)
  int32_t proc;
  int64_t call_i, ret_i;
};

enum { EV_LIN = 0, EV_RET = 1, EV_FREE = 2 };

struct Ev {
  double t;
  int kind;
  int64_t arg;  // op index (LIN/RET) or process slot (FREE)
  bool operator>(const Ev &o) const {
    if (t != o.t) return t > o.t;
    return kind > o.kind;
  }
};

// Simulate one key; returns all ops (fails included) sorted by call.
void simulate(const lc_synth_params &p, int64_t key, std::vector<SimOp> &out,
              int32_t *label_out) {
  Rng rng(p.seed, (uint64_t)key);
  const int conc = std::max(1, p.concurrency);
  const int readers = conc / 2;
  const int nvals = std::max(1, p.n_values);
  const double inf = INFINITY;
  const int64_t target = p.ops_per_key;

  int anomaly = LC_SYNTH_CLEAN;
  if (p.p_anomaly > 0 && rng.uniform() < p.p_anomaly)
    anomaly = rng.uniform() < 0.5 ? LC_SYNTH_STALE_READ : LC_SYNTH_LOST_CAS;
  // Which successful CAS gets lost (counted in lin order).
  int64_t lost_cas_at = anomaly == LC_SYNTH_LOST_CAS
                            ? (int64_t)(rng.uniform() * std::max<int64_t>(1, target / 20))
                            : -1;

  out.clear();
  std::priority_queue<Ev, std::vector<Ev>, std::greater<Ev>> pq;
  std::vector<int32_t> proc_id(conc);
  for (int i = 0; i < conc; i++) {
    proc_id[i] = i;
    pq.push({rng.expo(0.2), EV_FREE, i});
  }
  std::vector<int> idle;
  int64_t packed = 0, inflight = 0;
  int64_t ver = 0, val = LC_NIL;
  std::vector<int64_t> vals_at;  // value after version v (index v)
  vals_at.push_back(LC_NIL);
  int64_t ok_cas_seen = 0;
  bool lost_done = false;

  auto start_op = [&](int slot, double t) {
    SimOp o{};
    const bool reader = slot < readers;
    if (reader) {
      o.f = LC_F_READ;
      o.expected = LC_NIL;
    } else if (rng.uniform() < 0.5) {
      o.f = LC_F_WRITE;
      o.value = rng.below(nvals);
      o.expected = LC_NIL;
    } else {
      o.f = LC_F_CAS;
      o.expected = rng.below(nvals);
      o.value = rng.below(nvals);
    }
    o.version = LC_NIL;
    const double d = 0.05 + rng.expo(1.0);
    o.call_t = t;
    o.lin_t = t + rng.uniform() * d;
    o.proc = proc_id[slot];
    o.slot = slot;
    bool crash = !reader && p.p_info > 0 && rng.uniform() < p.p_info;
    const int64_t idx = (int64_t)out.size();
    if (crash) {
      o.status = LC_SYNTH_INFO;
      o.effect = rng.uniform() < 0.5;
      o.ret_t = inf;
      proc_id[slot] += conc;  // the crashed process is replaced
      pq.push({t + d, EV_FREE, slot});
    } else {
      o.status = LC_SYNTH_OK;
      o.effect = true;
      o.ret_t = t + d;
      pq.push({o.ret_t, EV_RET, slot});
    }
    pq.push({o.lin_t, EV_LIN, idx});
    out.push_back(o);
    inflight++;
  };

  while (!pq.empty()) {
    const Ev e = pq.top();
    pq.pop();
    if (e.kind == EV_FREE || e.kind == EV_RET) {
      const int slot = (int)e.arg;
      if (packed + inflight < target)
        start_op(slot, e.t + (e.kind == EV_RET ? rng.expo(0.2) : 0.0));
      else
        idle.push_back(slot);
      continue;
    }
    // EV_LIN: the op takes effect now.
    SimOp &o = out[(size_t)e.arg];
    inflight--;
    if (o.f == LC_F_READ) {
      if (o.status == LC_SYNTH_OK) {
        o.version = ver == 0 ? LC_NIL : ver;  // missing key reads [nil nil]
        o.value = ver == 0 ? LC_NIL : val;
      }
      packed++;
    } else if (o.status == LC_SYNTH_INFO) {
      if (o.effect && (o.f == LC_F_WRITE || val == o.expected)) {
        ver++;
        val = o.value;
        vals_at.push_back(val);
      }
      packed++;
    } else if (o.f == LC_F_WRITE) {
      ver++;
      val = o.value;
      vals_at.push_back(val);
      o.version = ver;
      packed++;
    } else {  // CAS
      if (val == o.expected) {
        if (!lost_done && ok_cas_seen == lost_cas_at) {
          // Lost CAS: reported ok with the next version, effect dropped.
          o.version = ver + 1;
          o.lost = true;
          lost_done = true;
        } else {
          ver++;
          val = o.value;
          vals_at.push_back(val);
          o.version = ver;
        }
        ok_cas_seen++;
        packed++;
      } else {
        o.status = LC_SYNTH_FAIL;
        // A failed CAS frees its budget slot: wake an idle process.
        if (!idle.empty() && packed + inflight < target) {
          const int slot = idle.back();
          idle.pop_back();
          start_op(slot, e.t);
        }
      }
    }
  }

  // info_frac: top the crashed records up to the exact target by reporting
  // uniformly chosen :ok writes/CAS as :info (they did take effect, so the
  // history stays linearizable).  Each such process is replaced: the later
  // ops of its worker slot move to the next process id.
  if (p.info_frac > 0) {
    const int64_t want = std::llround(p.info_frac * (double)target);
    int64_t have = 0;
    std::vector<size_t> cand;
    for (size_t i = 0; i < out.size(); i++) {
      const SimOp &o = out[i];
      if (o.status == LC_SYNTH_INFO) have++;
      else if (o.status == LC_SYNTH_OK && o.f != LC_F_READ && !o.lost) cand.push_back(i);
    }
    for (size_t j = 0; have < want && j < cand.size(); j++, have++) {
      const size_t pick = j + (size_t)rng.below((int)(cand.size() - j));
      std::swap(cand[j], cand[pick]);
      SimOp &o = out[cand[j]];
      o.status = LC_SYNTH_INFO;
      o.ret_t = inf;
      for (SimOp &q : out)
        if (q.slot == o.slot && q.call_t > o.call_t) q.proc += conc;
    }
  }

  // History indices: rank every call / finite return by time.
  struct TE {
    double t;
    int64_t op;
    int is_ret;
  };
  std::vector<TE> te;
  te.reserve(out.size() * 2);
  for (size_t i = 0; i < out.size(); i++) {
    te.push_back({out[i].call_t, (int64_t)i, 0});
    if (out[i].status != LC_SYNTH_INFO) te.push_back({out[i].ret_t, (int64_t)i, 1});
  }
  std::sort(te.begin(), te.end(), [](const TE &a, const TE &b) {
    if (a.t != b.t) return a.t < b.t;
    return a.is_ret > b.is_ret;
  });
  for (size_t r = 0; r < te.size(); r++) {
    SimOp &o = out[(size_t)te[r].op];
    if (te[r].is_ret)
      o.ret_i = (int64_t)r;
    else
      o.call_i = (int64_t)r;
  }
  for (auto &o : out)
    if (o.status == LC_SYNTH_INFO) o.ret_i = LC_INF;
  std::sort(out.begin(), out.end(),
            [](const SimOp &a, const SimOp &b) { return a.call_i < b.call_i; });

  if (anomaly == LC_SYNTH_STALE_READ) {
    // Mutation that produced version V (ok write/cas) and returned at ret_i;
    // pick a read invoked after that return which observed version >= V >= 2
    // and make it report state V-1.
    std::vector<int64_t> ret_of_version(vals_at.size(), -1);
    for (auto &o : out)
      if (o.status == LC_SYNTH_OK && o.f != LC_F_READ && o.version >= 0 &&
          (size_t)o.version < ret_of_version.size())
        ret_of_version[(size_t)o.version] = o.ret_i;
    std::vector<size_t> cand;
    for (size_t i = 0; i < out.size(); i++) {
      const SimOp &o = out[i];
      if (o.f != LC_F_READ || o.status != LC_SYNTH_OK || o.version < 2) continue;
      const int64_t r = ret_of_version[(size_t)o.version];
      if (r >= 0 && r < o.call_i) cand.push_back(i);
    }
    if (!cand.empty()) {
      SimOp &o = out[cand[(size_t)rng.below((int)cand.size())]];
      o.version -= 1;
      o.value = vals_at[(size_t)o.version];
    } else {
      anomaly = LC_SYNTH_CLEAN;
    }
  }
  if (anomaly == LC_SYNTH_LOST_CAS && !lost_done) anomaly = LC_SYNTH_CLEAN;
  if (label_out) *label_out = anomaly;
}

void to_record(const SimOp &o, lc_op *r) {
  r->f = o.f;
  r->value = o.value;
  r->expected = o.f == LC_F_CAS ? o.expected : LC_NIL;
  r->version = o.status == LC_SYNTH_OK ? o.version : LC_NIL;
  r->call = o.call_i;
  r->ret = o.ret_i;
}

}  // namespace

extern "C" int lc_synth_register(const lc_synth_params *p, lc_op *ops,
                                 int64_t *key_off, int32_t *labels,
                                 int64_t *n_invocations, int n_threads) {
  if (!p || !ops || !key_off || p->n_keys < 0 || p->ops_per_key < 0)
    return -EINVAL;
  const int64_t nk = p->n_keys, per = p->ops_per_key;
  for (int64_t k = 0; k <= nk; k++) key_off[k] = k * per;
  std::atomic<int64_t> next{0}, inv{0};
  std::atomic<int> err{0};
  auto work = [&]() {
    std::vector<SimOp> buf;
    int64_t local_inv = 0;
    for (;;) {
      const int64_t k = next.fetch_add(1);
      if (k >= nk) break;
      int32_t lab = 0;
      simulate(*p, k, buf, &lab);
      int64_t w = 0;
      for (const SimOp &o : buf) {
        local_inv++;
        if (o.status == LC_SYNTH_FAIL) continue;
        if (w < per) to_record(o, &ops[k * per + w]);
        w++;
      }
      if (w != per) err.store(1);
      if (labels) labels[k] = lab;
    }
    inv.fetch_add(local_inv);
  };
  n_threads = std::max(1, std::min(n_threads, 64));
  std::vector<std::thread> th;
  for (int i = 1; i < n_threads; i++) th.emplace_back(work);
  work();
  for (auto &t : th) t.join();
  if (n_invocations) *n_invocations = inv.load();
  return err.load() ? -EINVAL : 0;
}

extern "C" int lc_synth_key(const lc_synth_params *p, int64_t key, lc_op *ops,
                            int32_t *proc, int32_t *status, int64_t cap,
                            int64_t *n_out, int32_t *label) {
  if (!p || !n_out) return -EINVAL;
  std::vector<SimOp> buf;
  simulate(*p, key, buf, label);
  *n_out = (int64_t)buf.size();
  if ((int64_t)buf.size() > cap) return -ENOSPC;
  for (size_t i = 0; i < buf.size(); i++) {
    const SimOp &o = buf[i];
    if (ops) {
      to_record(o, &ops[i]);
      if (o.status == LC_SYNTH_FAIL) {
        ops[i].version = LC_NIL;  // a :fail completion carries no version
      }
    }
    if (proc) proc[i] = o.proc;
    if (status) status[i] = o.status;
  }
  return 0;
}
