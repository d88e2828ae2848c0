// Device helpers shared by the BPLA kernels (bpla.hip) and the BPLA gradient
// kernels (bpla_grad.hip): lane shifts of the systolic schedule and the
// table-driven exp of the dyadic fast path.
#pragma once
#include <hip/hip_runtime.h>

#include "launch.h"

namespace sk {

// lane l receives lane l-1's value (lane 0 receives `low`): DPP wave_shr:1
__device__ __forceinline__ double wave_shr1(double v, double low) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const int llo = __double2loint(low), lhi = __double2hiint(low);
  const int rlo = __builtin_amdgcn_update_dpp(llo, lo, 0x138, 0xf, 0xf, false);
  const int rhi = __builtin_amdgcn_update_dpp(lhi, hi, 0x138, 0xf, 0xf, false);
  return __hiloint2double(rhi, rlo);
}

// lane l receives lane l+1's value (lane 63 receives `high`): DPP wave_shl:1
__device__ __forceinline__ double wave_shl1_to(double v, double high) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const int hlo = __double2loint(high), hhi = __double2hiint(high);
  const int rlo = __builtin_amdgcn_update_dpp(hlo, lo, 0x130, 0xf, 0xf, false);
  const int rhi = __builtin_amdgcn_update_dpp(hhi, hi, 0x130, 0xf, 0xf, false);
  return __hiloint2double(rhi, rlo);
}

// The reference's float expressions a*b + c*d and n + a*b, every operation
// rounded on its own: no fused multiply-add (a contracted one differs by an
// ulp of float, ~1e-8 relative in K after the exponentials).
__device__ __forceinline__ float f32_dot2(float a, float b, float c, float d) {
#pragma clang fp contract(off)
  return a * b + c * d;
}
__device__ __forceinline__ float f32_madd(float n, float a, float b) {
#pragma clang fp contract(off)
  return n + a * b;
}

// exp(x), |x| << 700: x = (64m + j) ln2/64 + r, |r| <= ln2/128, e^r by its
// Taylor series to degree 5 (truncation < 4e-17 relative), times 2^(j/64)
// from an LDS table, times 2^m.
__device__ __forceinline__ double fast_exp(double x, const double* etab, const double (&ec)[4]) {
  const double k = __builtin_rint(x * 92.332482616893657);  // 64 / ln2
  const int ki = (int)k;
  double r = __builtin_fma(-k, 1.0830424693267560e-02, x);  // ln2/64, high part (exact k*hi)
  r = __builtin_fma(-k, 2.9815858269852933e-12, r);         // ln2/64, low part
  double p = ec[0];
  p = __builtin_fma(p, r, ec[1]);
  p = __builtin_fma(p, r, ec[2]);
  p = __builtin_fma(p, r, ec[3]);
  p = __builtin_fma(p, r, 1.0);
  p = __builtin_fma(p, r, 1.0);
  return __builtin_amdgcn_ldexp(etab[ki & 63] * p, ki >> 6);
}

// 2^(j/64), j < 64, into the workgroup's exp table (first kBplaExpLds bytes)
__device__ __forceinline__ void fill_exp_table(double* etab) {
  if (threadIdx.x < 64) etab[threadIdx.x] = exp2((double)threadIdx.x / 64.0);
  __syncthreads();
}

}  // namespace sk
