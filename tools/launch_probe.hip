// Dev probe: host-side cost of submitting one kernel launch, by launch API
// (and a captured two-kernel graph against the two launches)
// and argument size (the frontier exchange submits two launches per return,
// the first with its ~2.7 KB window by value).  Batches of 200 launches of a
// one-workgroup kernel are enqueued and timed on the host, then the stream is
// synchronised (so the queue never fills and the time is the submission's).
//   hipcc --offload-arch=gfx950 -O2 tools/launch_probe.hip -o tools/launch_probe_bin
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

struct Big {
  unsigned long long w[340];  // 2,720 bytes, about the frontier exchange's Win
};

__global__ void k_small(int *p, int v) {
  if (threadIdx.x == 0) p[0] = v;
}
__global__ void k_big(int *p, const Big b) {
  if (threadIdx.x == 0) p[1] = (int)b.w[threadIdx.x + 7];
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  int *d;
  CK(hipMalloc(&d, 4096));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  Big big{};
  for (int i = 0; i < 340; i++) big.w[i] = i;
  hipFunction_t fs = nullptr, fb = nullptr;
  CK(hipGetFuncBySymbol(&fs, reinterpret_cast<const void *>(k_small)));
  CK(hipGetFuncBySymbol(&fb, reinterpret_cast<const void *>(k_big)));
  const int B = 200, R = 50;
  auto run = [&](const char *name, auto &&launch) -> int {
    for (int i = 0; i < B; i++) launch(i);  // warm
    if (hipStreamSynchronize(st) != hipSuccess) return 1;
    double host = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < R; r++) {
      const auto a = std::chrono::steady_clock::now();
      for (int i = 0; i < B; i++) launch(i);
      host += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
      if (hipStreamSynchronize(st) != hipSuccess) return 1;
    }
    const double all = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    printf("%-34s submit %.2f us/launch, with the GPU %.2f us/launch\n", name, host / (B * R),
           all / (B * R));
    return 0;
  };
  if (run("<<<>>> small args", [&](int i) { k_small<<<1, 64, 0, st>>>(d, i); })) return 1;
  if (run("<<<>>> 2.7 KB by value", [&](int i) { big.w[0] = i; k_big<<<1, 64, 0, st>>>(d, big); }))
    return 1;
  if (run("hipModuleLaunchKernel small", [&](int i) {
        void *args[] = {&d, &i};
        (void)hipModuleLaunchKernel(fs, 1, 1, 1, 64, 1, 1, 0, st, args, nullptr);
      }))
    return 1;
  if (run("hipModuleLaunchKernel 2.7 KB", [&](int i) {
        big.w[0] = i;
        void *args[] = {&d, &big};
        (void)hipModuleLaunchKernel(fb, 1, 1, 1, 64, 1, 1, 0, st, args, nullptr);
      }))
    return 1;
  if (run("hipExtLaunchKernelGGL small", [&](int i) {
        hipExtLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, st, nullptr, nullptr, 0, d, i);
      }))
    return 1;
  // a captured graph of two launches (a step's pass and its follower) against
  // the two launches themselves
  if (run("two <<<>>> launches", [&](int i) {
        k_small<<<1, 64, 0, st>>>(d, i);
        k_small<<<1, 64, 0, st>>>(d + 4, i);
      }))
    return 1;
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
  k_small<<<1, 64, 0, st>>>(d, 1);
  k_small<<<1, 64, 0, st>>>(d + 4, 1);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  if (run("hipGraphLaunch (2 kernels)", [&](int) { (void)hipGraphLaunch(ge, st); })) return 1;
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
