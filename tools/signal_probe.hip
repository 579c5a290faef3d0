// Dev probe: completion signal of a launch, follower kernel against
// hipStreamWriteValue32 into host-mapped memory, both spun on by the host
// (every wait bounded at 100 ms; the grid is an empty kernel).
//   hipcc --offload-arch=gfx950 -O2 tools/signal_probe.hip -o tools/signal_probe_bin
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void empty_k(int *p) {
  if (threadIdx.x == 0) p[blockIdx.x] = blockIdx.x;
}
__global__ void follow_k(uint32_t *h_done, uint32_t s) {
  if (threadIdx.x == 0) __hip_atomic_store(h_done, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

static bool spin_until(volatile uint32_t *w, uint32_t want) {
  const auto t0 = std::chrono::steady_clock::now();
  while (__atomic_load_n(w, __ATOMIC_ACQUIRE) != want)
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(100)) return false;
  return true;
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  int *d_out;
  CK(hipMalloc(&d_out, 1 << 20));
  uint32_t *h_done, *hd_dev;
  CK(hipHostMalloc(&h_done, 64, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer((void **)&hd_dev, h_done, 0));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const int N = 500;
  for (int grid : {1, 1250, 10000}) {
    for (int w = 0; w < 50; w++) hipLaunchKernelGGL(empty_k, dim3(grid), dim3(256), 0, st, d_out);
    CK(hipStreamSynchronize(st));
    for (int mode = 0; mode < 2; mode++) {
      *(volatile uint32_t *)h_done = 0;
      const auto t0 = std::chrono::steady_clock::now();
      uint32_t i = 1;
      for (; i <= (uint32_t)N; i++) {
        hipLaunchKernelGGL(empty_k, dim3(grid), dim3(256), 0, st, d_out);
        if (mode == 0)
          hipLaunchKernelGGL(follow_k, dim3(1), dim3(64), 0, st, hd_dev, i);
        else
          CK(hipStreamWriteValue32(st, hd_dev, i, 0));
        if (!spin_until(h_done, i)) {
          printf("grid %d mode %d: request %u not seen in 100 ms\n", grid, mode, i);
          break;
        }
      }
      const auto t1 = std::chrono::steady_clock::now();
      CK(hipStreamSynchronize(st));
      printf("grid %5d %-22s %.2f us per launch+signal\n", grid,
             mode == 0 ? "follower kernel:" : "hipStreamWriteValue32:",
             std::chrono::duration<double, std::micro>(t1 - t0).count() / (i - 1));
    }
  }
  return 0;
}
