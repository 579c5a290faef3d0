// records.h — device-side decoding of lc_op records, shared by the kernels
// (check_kernel.hip: version-order and JIT tiers; gap_tier.hip).
#pragma once
#include <climits>

#include "kernels.h"

namespace lcdev {
namespace {

constexpr int64_t kInf = INT64_MAX;
constexpr int64_t kFieldMax = 0x7FFFFFFE;  // int32 range for value/expected/version
constexpr uint32_t kNever = 0xFFFFFFFFu;   // key-relative index of "no return"

// One record, decoded by one lane.  Event indices become key-relative 32-bit
// (index - first call of the key; LC_INF -> kNever) so event selection is a
// 32-bit compare.  A key whose indices span >= 2^32-1 is rejected as
// malformed (documented limit).  The op's precondition on the state it is
// stepped from is precomputed as (nv, nvm, nl, nlm):
//     legal(ver, val)  <=>  (((ver ^ nv) & nvm) | ((val ^ nl) & nlm)) == 0
// (register.clj:60-96: read needs version == op-version and value ==
// op-value where non-nil; write needs version+1 == op-version where non-nil;
// cas additionally needs value == expected), so legality over all 64 window
// slots is a handful of VALU ops and one compare — no per-lane boolean
// logic on lane masks.
struct Rec {
  int f, val, exp, ver;  // raw fields (int32; f = 3 for an unknown :f)
  int nv, nvm, nl, nlm;  // precondition
  uint32_t call, ret;    // key-relative; kNever = none
  int bad;
};

// Raw 48-byte record as loaded (three 16-byte loads per lane).  Decoding is
// deferred to the chunk switch so the prefetch of the next 64 records stays
// in flight while the current chunk is processed.
struct Raw {
  longlong2 a, b, c;
};

__device__ __forceinline__ Raw load_raw(const lc_op *__restrict__ o, int i, int n) {
  Raw r;
  if (i < n) {
    const longlong2 *p = reinterpret_cast<const longlong2 *>(o + i);
    r.a = p[0];
    r.b = p[1];
    r.c = p[2];
  } else {
    r.a = make_longlong2(0, -1);
    r.b = make_longlong2(-1, -1);
    r.c = make_longlong2(-1, -1);  // call = ret = -1 marks "past the end"
  }
  return r;
}

__device__ __forceinline__ Rec decode(const Raw &w, int64_t base_idx) {
  Rec r;
  const int64_t f = w.a.x, value = w.a.y, expected = w.b.x, version = w.b.y;
  const int64_t call = w.c.x, ret = w.c.y;
  if (call == -1 && ret == -1) {  // past the end of the key
    r.f = 0;
    r.val = r.exp = r.ver = -1;
    r.nv = r.nvm = r.nl = r.nlm = 0;
    r.bad = 0;
    r.call = kNever;
    r.ret = kNever;
    return r;
  }
  const int64_t rc = call - base_idx, rr = ret - base_idx;
  r.bad = (value < -1) | (value > kFieldMax) | (expected < -1) |
          (expected > kFieldMax) |
          (call < 0) | (ret <= call) | (rc < 0) | (rc >= (int64_t)kNever) |
          ((ret != kInf) & (rr >= (int64_t)kNever));
  r.f = (f >= 0 && f <= 2) ? (int)f : 3;
  r.val = (int)value;
  r.exp = (int)expected;
  // A version outside [-1, kFieldMax] is one no state of the key can hold
  // (states run from V0 >= 0 up to V0 + n < kFieldMax): knossos rejects the
  // op at every step, so it is saturated to kFieldMax, which is equally
  // unreachable, instead of failing the key as malformed.
  r.ver = (version < -1 || version > kFieldMax) ? (int)kFieldMax : (int)version;
  r.call = (uint32_t)rc;
  r.ret = ret == kInf ? kNever : (uint32_t)rr;
  const int vchk = r.ver != -1 ? -1 : 0;
  if (r.f == LC_F_READ) {
    r.nv = r.ver;
    r.nvm = vchk;
    r.nl = r.val;
    r.nlm = r.val != -1 ? -1 : 0;
  } else {
    r.nv = r.ver - 1;
    r.nvm = vchk;
    r.nl = r.exp;
    r.nlm = r.f == LC_F_CAS ? -1 : 0;
  }
  return r;
}

}  // namespace
}  // namespace lcdev
