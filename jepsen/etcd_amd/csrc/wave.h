// wave.h — wave-level helpers shared by the kernels (64-lane wavefronts).
#pragma once
#include <stdint.h>

#include "kernels.h"

namespace lcdev {
namespace {

// Number of set bits of m in lanes below this one (prefix-sum compaction).
__device__ __forceinline__ int lanes_below(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                        __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }
// Minimum of v over the 64 lanes as a wave-uniform (SGPR) value: four DPP
// min steps inside each 16-lane row (quad_perm [1,0,3,2], quad_perm
// [2,3,0,1], row_half_mirror, row_mirror), then the four row minima are read
// with v_readlane and combined on the scalar unit.  No LDS round trip.
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
  v = umin(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false));
  v = umin(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false));
  v = umin(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x141, 0xF, 0xF, false));
  v = umin(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x140, 0xF, 0xF, false));
  const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
  const uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
  const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 32);
  const uint32_t r3 = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
  return umin(umin(r0, r1), umin(r2, r3));
}
// Signed minimum over the wave (wave-uniform): wave_min_u32 on the
// order-preserving flip of the sign bit.
__device__ __forceinline__ int wave_min_i32(int v) {
  return (int)(wave_min_u32((uint32_t)v ^ 0x80000000u) ^ 0x80000000u);
}
__device__ __forceinline__ int first_lane(uint64_t b) { return (int)__builtin_ctzll(b); }
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int4 uni4(int4 v) {
  return make_int4(uni(v.x), uni(v.y), uni(v.z), uni(v.w));
}
// Makes this wave's earlier stores visible to all of its lanes (LDS:
// lgkmcnt; global memory: vmcnt, same CU so L1-coherent).
__device__ __forceinline__ void wave_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

}  // namespace
}  // namespace lcdev
