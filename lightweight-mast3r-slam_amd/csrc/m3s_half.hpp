// binary16 helpers shared by the refine kernels (matching.hip, refine.hip).
#pragma once
#include "m3s_common.hpp"

namespace m3s {

typedef _Float16 h1;
typedef _Float16 h2 __attribute__((ext_vector_type(2)));

// NaN-propagating max (fmaxf drops a NaN operand; the refine screen's norm bound must see one)
__device__ __forceinline__ float fmaxf_nan(float a, float b) { return (a > b || a != a) ? a : b; }

// D21 row source: f16 (reference signature, caller did .half()) or f32 (fused path: RNE convert here,
// identical to torch's .half()).
template <int F, bool D21_F32>
__device__ __forceinline__ void load_query(const void* D21, size_t row, h2* q) {
  if constexpr (D21_F32) {
    const float4* s = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(D21) + row * F);
#pragma unroll
    for (int k = 0; k < F / 4; k++) {
      const float4 v = s[k];
      q[2 * k + 0] = h2{(h1)v.x, (h1)v.y};
      q[2 * k + 1] = h2{(h1)v.z, (h1)v.w};
    }
  } else {
    const uint4* s = reinterpret_cast<const uint4*>(reinterpret_cast<const h1*>(D21) + row * F);
#pragma unroll
    for (int k = 0; k < F / 8; k++) {
      const uint4 t = s[k];
      q[4 * k + 0] = *reinterpret_cast<const h2*>(&t.x);
      q[4 * k + 1] = *reinterpret_cast<const h2*>(&t.y);
      q[4 * k + 2] = *reinterpret_cast<const h2*>(&t.z);
      q[4 * k + 3] = *reinterpret_cast<const h2*>(&t.w);
    }
  }
}

// score += sum_{k<8} half(q_k * c_k), one rounding per product and per add (c10::Half semantics).
// Files using this are compiled with -ffp-contract=off so no v_fma_f16 can fuse a pair.
__device__ __forceinline__ void add8(h1& s, const h2* q4, uint4 c) {
  const h2* cv = reinterpret_cast<const h2*>(&c);
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const h2 pr = q4[k] * cv[k];
    s = s + pr.x;
    s = s + pr.y;
  }
}

}  // namespace m3s
