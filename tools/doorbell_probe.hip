// Dev probe: what a step costs when the kernel is already resident.  A
// persistent grid waits on a host-mapped doorbell (one lane of workgroup 0
// polls host memory and forwards the sequence number to a device word the
// other workgroups poll), does one pass of trivial work (a word per
// workgroup), and the last workgroup (sharded counters) writes the sequence
// number to a host-mapped completion word the host spins on.  Compared with
// launch + event sync and launch + a kernel-written completion flag.  Every
// wave leaves on an exit request or after an idle timeout (wall clock), so
// the grid always drains.
//   hipcc --offload-arch=gfx950 -O2 tools/doorbell_probe.hip -o /tmp/db && /tmp/db
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>

#define CK(x) do { hipError_t e = (x); if (e) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr uint32_t kExit = 0xFFFFFFFFu;
constexpr int kShards = 32;

__device__ __forceinline__ uint32_t ld_sys(const uint32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t ld_dev(const uint32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}

// ctr: kShards counters 128 B apart, then the top counter; all zero at launch
__global__ void resident_k(const uint32_t *h_bell, uint32_t *d_bell, uint32_t *h_done, uint32_t *ctr,
                           int *out, unsigned long long idle_ticks) {
  __shared__ uint32_t seq_s;
  uint32_t seq = 0;
  const int nshard = (int)min((unsigned)kShards, gridDim.x);
  const int shard = blockIdx.x % nshard;
  // workgroups per shard
  const uint32_t per = gridDim.x / nshard + (shard < (int)(gridDim.x % nshard) ? 1 : 0);
  for (;;) {
    if (threadIdx.x == 0) {
      const unsigned long long t0 = wall_clock64();
      uint32_t s;
      for (;;) {
        if (blockIdx.x == 0) {
          s = ld_sys(h_bell);
          if (s != seq) __hip_atomic_store(d_bell, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          s = ld_dev(d_bell);
        }
        if (s != seq) break;
        if (wall_clock64() - t0 > idle_ticks) {
          s = kExit;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      seq_s = s;
    }
    __syncthreads();
    const uint32_t s = seq_s;
    __syncthreads();
    if (s == kExit) return;
    seq = s;
    // the work: one word per workgroup
    if (threadIdx.x == 0) out[blockIdx.x] = (int)s;
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      uint32_t *c = ctr + shard * 32;
      const uint32_t v = __hip_atomic_fetch_add(c, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1;
      if (v % per == 0) {  // this shard's last workgroup of this request
        uint32_t *top = ctr + kShards * 32;
        const uint32_t t = __hip_atomic_fetch_add(top, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1;
        if (t % (uint32_t)nshard == 0) {
          __hip_atomic_store(h_done, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
    }
  }
}

__global__ void flag_k(uint32_t *h_done, uint32_t *ctr, int *out, uint32_t s) {
  const int nshard = (int)min((unsigned)kShards, gridDim.x);
  const int shard = blockIdx.x % nshard;
  const uint32_t per = gridDim.x / nshard + (shard < (int)(gridDim.x % nshard) ? 1 : 0);
  if (threadIdx.x == 0) {
    out[blockIdx.x] = (int)s;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const uint32_t v = __hip_atomic_fetch_add(ctr + shard * 32, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1;
    if (v % per == 0) {
      const uint32_t t = __hip_atomic_fetch_add(ctr + kShards * 32, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1;
      if (t % (uint32_t)nshard == 0) __hip_atomic_store(h_done, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// the same without the per-workgroup release and with relaxed counters: the
// last workgroup alone fences (system scope) before its host store
__global__ void flag_relaxed_k(uint32_t *h_done, uint32_t *ctr, int *out, uint32_t s) {
  const int nshard = (int)min((unsigned)kShards, gridDim.x);
  const int shard = blockIdx.x % nshard;
  const uint32_t per = gridDim.x / nshard + (shard < (int)(gridDim.x % nshard) ? 1 : 0);
  if (threadIdx.x == 0) {
    out[blockIdx.x] = (int)s;
    const uint32_t v = __hip_atomic_fetch_add(ctr + shard * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    if (v % per == 0) {
      const uint32_t t = __hip_atomic_fetch_add(ctr + kShards * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
      if (t % (uint32_t)nshard == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __hip_atomic_store(h_done, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

__global__ void follow_k(uint32_t *h_done, uint32_t s) {
  if (threadIdx.x == 0) __hip_atomic_store(h_done, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void empty_k(int *p) {
  if (threadIdx.x == 0) p[blockIdx.x] = blockIdx.x;
}

// spin on a host word until it equals want, at most 100 ms
static bool spin_until(volatile uint32_t *w, uint32_t want) {
  const auto t0 = std::chrono::steady_clock::now();
  while (__atomic_load_n(w, __ATOMIC_ACQUIRE) != want)
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(100)) return false;
  return true;
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  int *d_out;
  uint32_t *ctr, *d_bell;
  CK(hipMalloc(&d_out, 1 << 20));
  CK(hipMalloc(&ctr, 4 * (kShards + 1) * 32));
  CK(hipMalloc(&d_bell, 64));
  uint32_t *h_bell, *h_done, *hb_dev, *hd_dev;
  CK(hipHostMalloc(&h_bell, 64, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostMalloc(&h_done, 64, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer((void **)&hb_dev, h_bell, 0));
  CK(hipHostGetDevicePointer((void **)&hd_dev, h_done, 0));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreateWithFlags(&e0, hipEventDisableSystemFence));
  CK(hipEventCreateWithFlags(&e1, hipEventDisableSystemFence));
  int khz = 100000;
  (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
  const int N = 500;
  for (int grid : {1, 1250, 1792, 10000}) {
    printf("grid %4d launch ...\n", grid);
    // launch + events + event sync (lc_check_device today)
    for (int w = 0; w < 50; w++) hipLaunchKernelGGL(empty_k, dim3(grid), dim3(256), 0, st, d_out);
    CK(hipStreamSynchronize(st));
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < N; i++) {
      CK(hipEventRecord(e0, st));
      hipLaunchKernelGGL(empty_k, dim3(grid), dim3(256), 0, st, d_out);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
    }
    auto t1 = std::chrono::steady_clock::now();
    printf("grid %4d launch+events+EventSynchronize: %.2f us\n", grid,
           std::chrono::duration<double, std::micro>(t1 - t0).count() / N);
    // launch, the kernel's last workgroup writes a host-mapped flag, host spins
    CK(hipMemset(ctr, 0, 4 * (kShards + 1) * 32));
    *(volatile uint32_t *)h_done = 0;
    t0 = std::chrono::steady_clock::now();
    printf("grid %4d kernel flag ...\n", grid);
    for (uint32_t i = 1; i <= (uint32_t)N; i++) {
      hipLaunchKernelGGL(flag_k, dim3(grid), dim3(256), 0, st, hd_dev, ctr, d_out, i);
      if (!spin_until(h_done, i)) {
        printf("grid %4d kernel flag: request %u not seen in 100 ms (h_done %u)\n", grid, i, *h_done);
        break;
      }
    }
    t1 = std::chrono::steady_clock::now();
    CK(hipStreamSynchronize(st));
    printf("grid %4d launch+kernel flag spin: %.2f us\n", grid,
           std::chrono::duration<double, std::micro>(t1 - t0).count() / N);
    // the same, relaxed counters, one fence by the last workgroup
    CK(hipMemset(ctr, 0, 4 * (kShards + 1) * 32));
    *(volatile uint32_t *)h_done = 0;
    t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 1; i <= (uint32_t)N; i++) {
      hipLaunchKernelGGL(flag_relaxed_k, dim3(grid), dim3(256), 0, st, hd_dev, ctr, d_out, i);
      if (!spin_until(h_done, i)) {
        printf("grid %4d relaxed flag: request %u not seen in 100 ms (h_done %u)\n", grid, i, *h_done);
        break;
      }
    }
    t1 = std::chrono::steady_clock::now();
    CK(hipStreamSynchronize(st));
    printf("grid %4d launch+relaxed kernel flag spin: %.2f us\n", grid,
           std::chrono::duration<double, std::micro>(t1 - t0).count() / N);
    // launch, then a one-thread follower kernel writes the host flag (it
    // starts once the first kernel has retired, in stream order)
    *(volatile uint32_t *)h_done = 0;
    printf("grid %4d follower flag ...\n", grid);
    t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 1; i <= (uint32_t)N; i++) {
      hipLaunchKernelGGL(empty_k, dim3(grid), dim3(256), 0, st, d_out);
      hipLaunchKernelGGL(follow_k, dim3(1), dim3(64), 0, st, hd_dev, i);
      if (!spin_until(h_done, i)) {
        printf("grid %4d follower: request %u not seen in 100 ms\n", grid, i);
        break;
      }
    }
    t1 = std::chrono::steady_clock::now();
    CK(hipStreamSynchronize(st));
    printf("grid %4d launch+follower flag spin: %.2f us\n", grid,
           std::chrono::duration<double, std::micro>(t1 - t0).count() / N);
    // the same with events around the first kernel (timing kept)
    *(volatile uint32_t *)h_done = 0;
    t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 1; i <= (uint32_t)N; i++) {
      CK(hipEventRecord(e0, st));
      hipLaunchKernelGGL(empty_k, dim3(grid), dim3(256), 0, st, d_out);
      CK(hipEventRecord(e1, st));
      hipLaunchKernelGGL(follow_k, dim3(1), dim3(64), 0, st, hd_dev, i);
      if (!spin_until(h_done, i)) {
        printf("grid %4d follower+events: request %u not seen in 100 ms\n", grid, i);
        break;
      }
    }
    t1 = std::chrono::steady_clock::now();
    CK(hipStreamSynchronize(st));
    printf("grid %4d events+launch+follower flag spin: %.2f us\n", grid,
           std::chrono::duration<double, std::micro>(t1 - t0).count() / N);
  }
  return 0;
}
