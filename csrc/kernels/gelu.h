// GELU (tanh "gelu_new" and erf forms) shared by the elementwise kernels and the GEMM epilogues.
#pragma once
#include <hip/hip_runtime.h>

namespace pdt {

constexpr float kSqrt2OverPi = 0.7978845608028654f;
constexpr float kGeluC = 0.044715f;
constexpr float kInvSqrt2 = 0.7071067811865476f;

// tanh-form GELU through the sigmoid identity 0.5 (1 + tanh z) = sigmoid(2z): one v_exp_f32 and one
// v_rcp_f32 per element instead of libm tanhf (~30 VALU ops; at 268M elements per GPT-2 1.3B MLP call the
// tanhf form made bias+GELU VALU-bound at ~50 % of HBM bandwidth).  exp overflow -> s = 0, underflow -> 1.
// sigmoid(2z) = 1 / (1 + 2^(u (A + B u^2))) with the constants folded: A = -2 sqrt(2/pi) log2(e), B = A * 0.044715
// (v_exp_f32 is exp2: no extra multiply; 2 fewer VALU ops per element than the z-then-__expf form)
constexpr float kGeluA = -2.f * 0.7978845608028654f * 1.4426950408889634f;
constexpr float kGeluB = kGeluA * 0.044715f;
__device__ __forceinline__ float sigmoid2z(float u) {
  const float a = u * __builtin_fmaf(kGeluB, u * u, kGeluA);
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(a));
}

// GELU value AND derivative of two pre-activations per packed instruction (v_pk_fma / v_pk_mul; exp2 / rcp stay
// scalar), sharing the one sigmoid: y = u s, d = s + u s (1 - s) 2 sqrt(2/pi) (1 + 3 c u^2).  The GEMM epilogue of
// GPT-2's c_fc stores d instead of the pre-activation, so the backward's GELU step is one multiply (no
// transcendentals where the matrix pipe idles, gemm.hip E_DGELU) -- both GEMM kernels call this one function,
// so their results stay bitwise equal.
typedef float gelu_f32x2 __attribute__((ext_vector_type(2)));
constexpr float kGeluD1 = 2.f * 0.7978845608028654f;
constexpr float kGeluD3 = kGeluD1 * 3.f * 0.044715f;
__device__ __forceinline__ void gelu_fwd_grad2(gelu_f32x2 u, gelu_f32x2& y, gelu_f32x2& d) {
  const gelu_f32x2 u2 = u * u;
  const gelu_f32x2 a = u * __builtin_elementwise_fma(gelu_f32x2{kGeluB, kGeluB}, u2, gelu_f32x2{kGeluA, kGeluA});
  const gelu_f32x2 e = gelu_f32x2{__builtin_amdgcn_exp2f(a[0]), __builtin_amdgcn_exp2f(a[1])} + gelu_f32x2{1.f, 1.f};
  const gelu_f32x2 s = gelu_f32x2{__builtin_amdgcn_rcpf(e[0]), __builtin_amdgcn_rcpf(e[1])};
  y = u * s;
  const gelu_f32x2 t = __builtin_elementwise_fma(-s, s, s);                                   // s (1 - s)
  const gelu_f32x2 q = __builtin_elementwise_fma(gelu_f32x2{kGeluD3, kGeluD3}, u2, gelu_f32x2{kGeluD1, kGeluD1});
  d = __builtin_elementwise_fma(u * t, q, s);
}

template <bool TANH>
__device__ __forceinline__ float gelu_f(float u) {
  if (TANH) {
    return u * sigmoid2z(u);
  } else {
    return 0.5f * u * (1.f + erff(u * kInvSqrt2));
  }
}
template <bool TANH>
__device__ __forceinline__ float gelu_grad(float u) {
  if (TANH) {
    // d/du [u s(2z)] = s + u * 2 s (1 - s) * dz/du, with 1 - tanh^2 = 4 s (1 - s)
    const float s = sigmoid2z(u);
    return s + 2.f * u * s * (1.f - s) * kSqrt2OverPi * (1.f + 3.f * kGeluC * u * u);
  } else {
    const float cdf = 0.5f * (1.f + erff(u * kInvSqrt2));
    const float pdf = 0.3989422804014327f * __expf(-0.5f * u * u);
    return cdf + u * pdf;
  }
}

}  // namespace pdt
