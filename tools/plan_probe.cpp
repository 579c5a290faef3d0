// Host cost of lc_check's device split (lincheck.cpp plan_devices) on a
// C2-sized batch: the sampled irregularity scan at several strides and
// thread counts, and the cost of creating the threads alone.
//   g++ -O2 -std=c++17 -pthread tools/plan_probe.cpp -o /tmp/plan_probe && /tmp/plan_probe
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

struct Op { int64_t f, value, expected, version, call, ret; };

int main() {
  const int64_t nk = 10000, per = 1000, n = nk * per;
  std::vector<Op> ops((size_t)n);
  for (int64_t i = 0; i < n; i++) ops[(size_t)i] = Op{i % 3, 1, -1, i % per + 1, i % per, i % per + 5};
  std::vector<int64_t> off((size_t)nk + 1);
  for (int64_t k = 0; k <= nk; k++) off[(size_t)k] = k * per;
  std::vector<double> pre((size_t)nk + 1);
  for (int64_t stride : {32, 64, 128, 256}) {
    for (int nth : {1, 4, 9, 16, 32}) {
      double best = 1e9;
      for (int rep = 0; rep < 5; rep++) {
        auto t0 = std::chrono::steady_clock::now();
        auto price = [&](int64_t k0, int64_t k1) {
          for (int64_t k = k0; k < k1; k++) {
            const Op *o = ops.data() + off[(size_t)k];
            const int64_t m = off[(size_t)k + 1] - off[(size_t)k];
            bool irr = false;
            for (int64_t i = 0; i < m && !irr; i += stride) {
              const bool mut = o[i].f == 1 || o[i].f == 2;
              irr = (mut && o[i].ret == INT64_MAX) || (o[i].version == -1 && mut);
            }
            pre[(size_t)k + 1] = irr ? 6.0 * m : (double)m + 64.0;
          }
        };
        if (nth == 1) {
          price(0, nk);
        } else {
          std::vector<std::thread> th;
          for (int t = 0; t < nth; t++) th.emplace_back(price, nk * t / nth, nk * (t + 1) / nth);
          for (auto &x : th) x.join();
        }
        const double ms =
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (ms < best) best = ms;
      }
      printf("stride %3ld threads %2d: %.3f ms\n", (long)stride, nth, best);
    }
  }
  for (int nth : {1, 8, 16}) {
    double best = 1e9;
    for (int rep = 0; rep < 5; rep++) {
      auto t0 = std::chrono::steady_clock::now();
      std::vector<std::thread> th;
      for (int t = 0; t < nth; t++) th.emplace_back([] {});
      for (auto &x : th) x.join();
      const double ms =
          std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (ms < best) best = ms;
    }
    printf("create+join %2d empty threads: %.3f ms\n", nth, best);
  }
  return 0;
}
