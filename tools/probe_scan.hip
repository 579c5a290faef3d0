// Dev probe (not product code): read-rate ceilings for the fast tier's access
// shape.  One 256-thread workgroup per 48-KB "key" (1,000 records x 48 B),
// 10,000 keys = the 480 MB C2 launch.  Variants:
//   strided  - lane i loads record i as three 16-B loads (the fast tier today)
//   coal     - each wave-instruction loads 1 KB contiguous (lane i, chunk i)
//   coal_lds - coalesced loads, then the 3 KB per wave transposed through LDS
//   persistN - N workgroups walk the keys, next key's loads issued early
// Each variant folds what it loaded into one word per workgroup so nothing is
// dead code.  Build: hipcc --offload-arch=gfx950 -O3 tools/probe_scan.hip -o tools/probe_scan
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

constexpr int kRec = 1000, kKeys = 10000, kT = 256;

__global__ __launch_bounds__(kT) void strided(const longlong2 *__restrict__ p, const int64_t *__restrict__ off,
                                               int64_t *__restrict__ out) {
  const int64_t beg = off[blockIdx.x], n = off[blockIdx.x + 1] - beg;
  const longlong2 *q = p + beg * 3;
  int64_t acc = 0;
  longlong2 a[4], b[4], c[4];
#pragma unroll
  for (int u = 0; u < 4; u++) {
    const int r = threadIdx.x + u * kT;
    if (r < n) { a[u] = q[3 * r]; b[u] = q[3 * r + 1]; c[u] = q[3 * r + 2]; }
    else { a[u] = b[u] = c[u] = make_longlong2(0, 0); }
  }
#pragma unroll
  for (int u = 0; u < 4; u++) acc += a[u].x ^ a[u].y ^ b[u].x ^ b[u].y ^ c[u].x ^ c[u].y;
  __shared__ int64_t s;
  if (threadIdx.x == 0) s = 0;
  __syncthreads();
  atomicXor((unsigned long long *)&s, (unsigned long long)acc);
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = s;
}

__global__ __launch_bounds__(kT) void coal(const longlong2 *__restrict__ p, const int64_t *__restrict__ off,
                                           int64_t *__restrict__ out) {
  const int64_t beg = off[blockIdx.x], n = off[blockIdx.x + 1] - beg;
  const longlong2 *q = p + beg * 3;
  const int nch = (int)n * 3;
  int64_t acc = 0;
  longlong2 a[12];
#pragma unroll
  for (int u = 0; u < 12; u++) {
    const int ch = threadIdx.x + u * kT;
    a[u] = ch < nch ? q[ch] : make_longlong2(0, 0);
  }
#pragma unroll
  for (int u = 0; u < 12; u++) acc += a[u].x ^ a[u].y;
  __shared__ int64_t s;
  if (threadIdx.x == 0) s = 0;
  __syncthreads();
  atomicXor((unsigned long long *)&s, (unsigned long long)acc);
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = s;
}

// coalesced loads, records re-assembled through LDS (48 KB per workgroup)
__global__ __launch_bounds__(kT) void coal_lds(const longlong2 *__restrict__ p, const int64_t *__restrict__ off,
                                               int64_t *__restrict__ out) {
  __shared__ longlong2 L[3 * 1024];
  const int64_t beg = off[blockIdx.x], n = off[blockIdx.x + 1] - beg;
  const longlong2 *q = p + beg * 3;
  const int nch = (int)n * 3;
  longlong2 a[12];
#pragma unroll
  for (int u = 0; u < 12; u++) {
    const int ch = threadIdx.x + u * kT;
    a[u] = ch < nch ? q[ch] : make_longlong2(0, 0);
  }
#pragma unroll
  for (int u = 0; u < 12; u++) L[threadIdx.x + u * kT] = a[u];
  __syncthreads();
  int64_t acc = 0;
#pragma unroll
  for (int u = 0; u < 4; u++) {
    const int r = threadIdx.x + u * kT;
    const longlong2 x = L[3 * r], y = L[3 * r + 1], z = L[3 * r + 2];
    acc += x.x ^ y.y ^ z.x ^ z.y;
  }
  __shared__ int64_t s;
  if (threadIdx.x == 0) s = 0;
  __syncthreads();
  atomicXor((unsigned long long *)&s, (unsigned long long)acc);
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = s;
}

// Persistent: grid of G workgroups walks keys blockIdx.x, +G, ...; coalesced
// loads of the next key issued before folding the current one.
__global__ __launch_bounds__(kT) void persist(const longlong2 *__restrict__ p, const int64_t *__restrict__ off,
                                              int64_t *__restrict__ out, int nkeys) {
  __shared__ int64_t s;
  longlong2 a[12];
  int key = blockIdx.x;
  auto issue = [&](int k) {
    const int64_t beg = off[k], n = off[k + 1] - beg;
    const longlong2 *q = p + beg * 3;
    const int nch = (int)n * 3;
#pragma unroll
    for (int u = 0; u < 12; u++) {
      const int ch = threadIdx.x + u * kT;
      a[u] = ch < nch ? q[ch] : make_longlong2(0, 0);
    }
  };
  if (key < nkeys) issue(key);
  for (; key < nkeys; key += gridDim.x) {
    int64_t acc = 0;
#pragma unroll
    for (int u = 0; u < 12; u++) acc += a[u].x ^ a[u].y;
    if (key + (int)gridDim.x < nkeys) issue(key + gridDim.x);
    if (threadIdx.x == 0) s = 0;
    __syncthreads();
    atomicXor((unsigned long long *)&s, (unsigned long long)acc);
    __syncthreads();
    if (threadIdx.x == 0) out[key] = s;
    __syncthreads();
  }
}

// strided with non-temporal register loads (global_load_dwordx4 ... nt)
typedef long long v2ll __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(kT) void strided_nt(const longlong2 *__restrict__ p, const int64_t *__restrict__ off,
                                                  int64_t *__restrict__ out) {
  const int64_t beg = off[blockIdx.x], n = off[blockIdx.x + 1] - beg;
  const v2ll *q = reinterpret_cast<const v2ll *>(p + beg * 3);
  int64_t acc = 0;
  v2ll a[4], b[4], c[4];
#pragma unroll
  for (int u = 0; u < 4; u++) {
    const int r = threadIdx.x + u * kT;
    if (r < n) { a[u] = __builtin_nontemporal_load(q + 3 * r); b[u] = __builtin_nontemporal_load(q + 3 * r + 1); c[u] = __builtin_nontemporal_load(q + 3 * r + 2); }
    else { a[u] = b[u] = c[u] = (v2ll){0, 0}; }
  }
#pragma unroll
  for (int u = 0; u < 4; u++) acc += a[u].x ^ a[u].y ^ b[u].x ^ b[u].y ^ c[u].x ^ c[u].y;
  __shared__ int64_t s;
  if (threadIdx.x == 0) s = 0;
  __syncthreads();
  atomicXor((unsigned long long *)&s, (unsigned long long)acc);
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = s;
}

// LDS-DMA: the key's 48 KB straight into LDS (global_load_lds_dwordx4, 1 KB
// per wave-instruction), then folded from LDS.  AUX 0 = default policy, 2 = nt.
template <int AUX>
__global__ __launch_bounds__(kT) void glds(const longlong2 *__restrict__ p, const int64_t *__restrict__ off,
                                           int64_t *__restrict__ out) {
  __shared__ longlong2 L[3 * 1024];
  const int64_t beg = off[blockIdx.x], n = off[blockIdx.x + 1] - beg;
  const longlong2 *q = p + beg * 3;
  const int nch = (int)n * 3;
  const int w = threadIdx.x / 64;
#pragma unroll
  for (int u = 0; u < 12; u++) {
    const int ch = threadIdx.x + u * kT;
    if (u * kT + w * 64 < nch)  // wave-uniform: the whole 1 KB row is in range (n = 1000)
      __builtin_amdgcn_global_load_lds((const void *)(q + ch), (__attribute__((address_space(3))) void *)(L + u * kT + w * 64), 16, 0, AUX);
  }
  __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) lgkmcnt(0) expcnt(0)
  __syncthreads();
  int64_t acc = 0;
#pragma unroll
  for (int u = 0; u < 4; u++) {
    const int r = threadIdx.x + u * kT;
    if (r < n) {
      const longlong2 x = L[3 * r], y = L[3 * r + 1], z = L[3 * r + 2];
      acc += x.x ^ y.y ^ z.x ^ z.y;
    }
  }
  __shared__ int64_t s;
  if (threadIdx.x == 0) s = 0;
  __syncthreads();
  atomicXor((unsigned long long *)&s, (unsigned long long)acc);
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = s;
}

// Hybrid: per record, chunks a and b by register loads, chunk c (call, ret)
// by LDS-DMA nt into a 16 KB per-workgroup LDS array (per-lane source
// addresses, contiguous LDS destination).
__global__ __launch_bounds__(kT) void hybrid(const longlong2 *__restrict__ p, const int64_t *__restrict__ off,
                                             int64_t *__restrict__ out) {
  __shared__ longlong2 C[1024];
  const int64_t beg = off[blockIdx.x], n = off[blockIdx.x + 1] - beg;
  const longlong2 *q = p + beg * 3;
  const int w = threadIdx.x / 64;
  longlong2 a[4], b[4];
#pragma unroll
  for (int u = 0; u < 4; u++) {
    const int r = threadIdx.x + u * kT;
    if (r < n) {
      __builtin_amdgcn_global_load_lds((const void *)(q + 3 * r + 2),
                                       (__attribute__((address_space(3))) void *)(C + u * kT + w * 64), 16, 0, 2);
      a[u] = q[3 * r];
      b[u] = q[3 * r + 1];
    } else {
      a[u] = b[u] = make_longlong2(0, 0);
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  int64_t acc = 0;
#pragma unroll
  for (int u = 0; u < 4; u++) {
    const int r = threadIdx.x + u * kT;
    const longlong2 c = r < n ? C[r] : make_longlong2(0, 0);
    acc += a[u].x ^ a[u].y ^ b[u].x ^ b[u].y ^ c.x ^ c.y;
  }
  __shared__ int64_t s;
  if (threadIdx.x == 0) s = 0;
  __syncthreads();
  atomicXor((unsigned long long *)&s, (unsigned long long)acc);
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = s;
}

int main() {
  const size_t nrec = (size_t)kRec * kKeys;
  std::vector<int64_t> h(nrec * 6), ho(kKeys + 1);
  for (size_t i = 0; i < h.size(); i++) h[i] = (int64_t)(i * 2654435761u);
  for (int k = 0; k <= kKeys; k++) ho[k] = (int64_t)k * kRec;
  longlong2 *d;
  int64_t *doff, *dout;
  CK(hipMalloc(&d, nrec * 48));
  CK(hipMalloc(&doff, (kKeys + 1) * 8));
  CK(hipMalloc(&dout, kKeys * 8));
  CK(hipMemcpy(d, h.data(), nrec * 48, hipMemcpyHostToDevice));
  CK(hipMemcpy(doff, ho.data(), (kKeys + 1) * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char *name, auto launch) {
    for (int i = 0; i < 3; i++) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    const int it = 30;
    for (int i = 0; i < it; i++) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= it;
    printf("%-12s %.4f ms  %.0f GB/s\n", name, ms, nrec * 48.0 / ms / 1e6);
    return 0;
  };
  run("strided", [&] { strided<<<kKeys, kT>>>(d, doff, dout); });
  run("coal", [&] { coal<<<kKeys, kT>>>(d, doff, dout); });
  run("coal_lds", [&] { coal_lds<<<kKeys, kT>>>(d, doff, dout); });
  run("strided_nt", [&] { strided_nt<<<kKeys, kT>>>(d, doff, dout); });
  run("hybrid", [&] { hybrid<<<kKeys, kT>>>(d, doff, dout); });
  run("glds", [&] { glds<0><<<kKeys, kT>>>(d, doff, dout); });
  run("glds_nt", [&] { glds<2><<<kKeys, kT>>>(d, doff, dout); });
  run("strided", [&] { strided<<<kKeys, kT>>>(d, doff, dout); });
  run("strided_nt", [&] { strided_nt<<<kKeys, kT>>>(d, doff, dout); });
  run("hybrid", [&] { hybrid<<<kKeys, kT>>>(d, doff, dout); });
  for (int g : {256, 512, 1024, 2048})
  {
    char nm[32];
    snprintf(nm, sizeof nm, "persist%d", g);
    run(nm, [&] { persist<<<g, kT>>>(d, doff, dout, kKeys); });
  }
  return 0;
}
