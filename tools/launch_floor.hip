// Dev probe: the host-side floor of one step (launch + completion wait) on
// this box, for an empty kernel and for a 1,250-workgroup kernel that only
// writes one word per workgroup (C3 at 8 GPUs has 1,250 keys per rank).
//   hipcc --offload-arch=gfx950 -O2 tools/launch_floor.hip -o /tmp/lf && /tmp/lf [spin]
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>

__global__ void empty_k(int *p) {
  if (threadIdx.x == 0 && p) p[blockIdx.x] = blockIdx.x;
}

#define CK(x) do { hipError_t e = (x); if (e) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main(int argc, char **argv) {
  if (argc > 1 && !strcmp(argv[1], "spin")) CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
  int *d;
  CK(hipMalloc(&d, 1 << 20));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreateWithFlags(&e0, hipEventDisableSystemFence));
  CK(hipEventCreateWithFlags(&e1, hipEventDisableSystemFence));
  for (int grid : {1, 1250, 10000}) {
    for (int mode = 0; mode < 3; mode++) {
      const int N = 2000;
      for (int w = 0; w < 50; w++) { hipLaunchKernelGGL(empty_k, dim3(grid), dim3(256), 0, st, d); }
      CK(hipStreamSynchronize(st));
      auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < N; i++) {
        if (mode == 0) {  // events around the launch, wait on the event (lc_check_device)
          CK(hipEventRecord(e0, st));
          hipLaunchKernelGGL(empty_k, dim3(grid), dim3(256), 0, st, d);
          CK(hipEventRecord(e1, st));
          CK(hipEventSynchronize(e1));
        } else if (mode == 1) {  // stream sync only
          hipLaunchKernelGGL(empty_k, dim3(grid), dim3(256), 0, st, d);
          CK(hipStreamSynchronize(st));
        } else {  // event wait by polling hipEventQuery
          hipLaunchKernelGGL(empty_k, dim3(grid), dim3(256), 0, st, d);
          CK(hipEventRecord(e1, st));
          while (hipEventQuery(e1) == hipErrorNotReady) {}
        }
      }
      auto t1 = std::chrono::steady_clock::now();
      printf("grid %5d mode %d (%s): %.2f us per step\n", grid, mode,
             mode == 0 ? "events+EventSynchronize" : mode == 1 ? "StreamSynchronize" : "EventQuery poll",
             std::chrono::duration<double, std::micro>(t1 - t0).count() / N);
    }
  }
  return 0;
}
