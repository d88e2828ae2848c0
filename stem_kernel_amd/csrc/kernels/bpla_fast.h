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

// exp(x) for |x| < 2^40 (overflow to inf past ~709, underflow to 0):
// x = (1024 m + j) ln2/1024 + r, |r| <= ln2/2048; k = 1024 m + j rounded by
// the 1.5 * 2^52 shifter (its low word is k), r = fma(-k, C, x) with C the
// double nearest ln2/1024 (one rounding: |k| |C - ln2/1024| <= 7.7e-14
// relative for |x| <= 709, where exp is finite; a two-part Cody-Waite
// constant buys nothing against the polynomial and cost one VALU), e^r by
// its Taylor series to degree 2 (truncation r^3/6 < 6.5e-12 relative: over
// the <= 2L factors of one alignment path below 1e-8, against the 1e-6 parity
// gate), times 2^(j/1024) from the workgroup's LDS table, times 2^m.  9 VALU
// and one LDS read (two-part reduction: 10; degree 3: 11; the degree-5 form
// over a 64-entry table took 16).
__device__ __forceinline__ double fast_exp(double x, const double* etab) {
  const double t = __builtin_fma(x, 1477.3197218702985, 6755399441055744.0);  // 1024/ln2, 1.5*2^52
  const int ki = __double2loint(t);
  const double k = t - 6755399441055744.0;
  const double r = __builtin_fma(-k, 6.769015435155716e-04, x);  // ln2/1024
  double p = __builtin_fma(r, 0.5, 1.0);
  p = __builtin_fma(p, r, 1.0);
  return __builtin_amdgcn_ldexp(etab[ki & 1023] * p, ki >> 10);
}

// 2^(j/1024), j < 1024, into the workgroup's exp table (first kBplaExpLds bytes)
__device__ __forceinline__ void fill_exp_table(double* etab) {
  for (int j = threadIdx.x; j < 1024; j += blockDim.x) etab[j] = exp2((double)j / 1024.0);
  __syncthreads();
}

}  // namespace sk
