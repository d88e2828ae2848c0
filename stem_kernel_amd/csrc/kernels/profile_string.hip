// Profile string-alignment kernel on CDNA4 (gfx950).
//
// Reference: StringKernel<double,MData>::operator()
//   stem_kernel_lite/string_kernel.cpp:66-132 (DP), :81-100 (subst_score),
//   ctors :46-70 (exp(alpha*ribosum_s) or match/mismatch).
//
// Systolic schedule: one wavefront per (x,y) pair; lane l owns DP row
// i = 64*strip + l + 1 and at step t computes column j = t - l + 1, so the
// wave sweeps a 64-row strip in Ly+64 steps.  The up / diagonal neighbours
// come from lane l-1 through cross-lane shuffles; the strip boundary row goes
// through a per-wave LDS row.  Row-local K1/G1 stay in registers.
#include <hip/hip_runtime.h>

#include "device_set.h"
#include "launch.h"

namespace sk {

__device__ __forceinline__ int onehot_code(float4 c) {
  // column of a single unambiguous residue -> its code, else -1
  if (c.x == 1.0f && c.y == 0.0f && c.z == 0.0f && c.w == 0.0f) return 0;
  if (c.x == 0.0f && c.y == 1.0f && c.z == 0.0f && c.w == 0.0f) return 1;
  if (c.x == 0.0f && c.y == 0.0f && c.z == 1.0f && c.w == 0.0f) return 2;
  if (c.x == 0.0f && c.y == 0.0f && c.z == 0.0f && c.w == 1.0f) return 3;
  return -1;
}

// subst_score(st, Column x, Column y): string_kernel.cpp:81-100.  Every
// operation rounded as the reference's (no fused multiply-add: a contracted
// float weight n is off by an ulp of float)
__device__ __forceinline__ double prof_subst(const double* __restrict__ st, float4 xc, float4 yc) {
#pragma clang fp contract(off)
  const float xa[4] = {xc.x, xc.y, xc.z, xc.w};
  const float yb[4] = {yc.x, yc.y, yc.z, yc.w};
  double v_c = 0.0;
  float n = 0.0f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (xa[i] == 0.0f) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (yb[j] == 0.0f) continue;
      n += xa[i] * yb[j];
      v_c += st[i * 4 + j] * xa[i] * yb[j];
    }
  }
  return n == 0.0f ? 1.0 : v_c / (double)n;
}

__global__ void __launch_bounds__(256) sk_profile_string_kernel(StrLaunch P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const DevSet& sx = P.xset;
  const DevSet& sy = P.yset;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int maxlen = P.lds_max_len;
  const int nwaves = blockDim.x >> 6;
  // LDS: st[16] | per wave rowK,rowG [maxlen+2] | yprof float4 | ywt | ycode
  double* st = reinterpret_cast<double*>(smem);
  double* rows = st + 16;
  double* rowK = rows + (size_t)wave * 2 * (maxlen + 2);
  double* rowG = rowK + (maxlen + 2);
  float4* yprof_all = reinterpret_cast<float4*>(rows + (size_t)nwaves * 2 * (maxlen + 2));
  float4* yprof = yprof_all + (size_t)wave * maxlen;
  float* ywt_all = reinterpret_cast<float*>(yprof_all + (size_t)nwaves * maxlen);
  float* ywt = ywt_all + (size_t)wave * maxlen;
  int* ycode = reinterpret_cast<int*>(ywt_all + (size_t)nwaves * maxlen) + (size_t)wave * maxlen;

  if (threadIdx.x < 16) st[threadIdx.x] = P.st[threadIdx.x];
  __syncthreads();
  const double gap = P.gap;

  for (;;) {
    unsigned long long pr = 0;
    if (lane == 0) pr = atomicAdd(P.pair_counter, 1ull);
    // broadcast lane 0's ticket through an SGPR (wave-uniform from here on)
    pr = ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(pr >> 32)) << 32) |
         (unsigned)__builtin_amdgcn_readfirstlane((unsigned)pr);
    if ((int64_t)pr >= P.n_pairs) break;
    const int x = P.xs[pr], y = P.ys[pr];
    const int Lx = sx.ex_len[x], Ly = sy.ex_len[y];
    const int xpb = sx.ex_pos_base[x], ypb = sy.ex_pos_base[y];
    const bool naive = P.naive != 0;
    const bool use_w = !naive && sx.ex_has_w[x] && sy.ex_has_w[y];
    for (int j = lane; j < Ly; j += 64) {
      const float4 c = sy.pos_prof[ypb + j];
      yprof[j] = c;
      ywt[j] = use_w ? sy.pos_w[ypb + j] : 1.0f;
      // naive kernel: the raw character (codes >= 16 never meet the profile path)
      ycode[j] = naive ? 16 + (int)sy.pos_chr[ypb + j] : onehot_code(c);
    }
    // row 0: K0[0][j] = 1, G0[0][j] = G0[0][j-1]*gap
    for (int j = lane; j <= Ly; j += 64) {
      rowK[j] = 1.0;
      rowG[j] = P.gpow[j];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    double result = 1.0;  // K0[Lx][Ly] for Lx==0 or Ly==0 is 1
    const int nstrips = (Lx + 63) / 64;
    for (int strip = 0; strip < nstrips; ++strip) {
      const int i = strip * 64 + lane + 1;  // my DP row (1-based)
      const bool row_ok = i <= Lx;
      float4 xc = make_float4(0.f, 0.f, 0.f, 0.f);
      float xw = 1.0f;
      int xcode = -1;
      if (row_ok) {
        xc = sx.pos_prof[xpb + i - 1];
        xw = use_w ? sx.pos_w[xpb + i - 1] : 1.0f;
        xcode = naive ? 16 + (int)sx.pos_chr[xpb + i - 1] : onehot_code(xc);
      }
      const double g0col = row_ok ? P.gpow[i] : 0.0;  // G0[i][0] = G0[i-1][0]*gap
      // outputs of steps t-1 (myK0, myG0) and t-2 (myG0p).  Lane l reaches
      // column 0 at step l-1; lane 0's column-0 output is the initial state.
      double myK0 = 1.0, myG0 = g0col, myG0p = 0.0;
      double K1p = 0.0, G1p = 0.0;
      for (int t = 0; t < Ly + 64; ++t) {
        const int j = t - lane + 1;
        double upK = __shfl_up(myK0, 1, 64);
        double upG = __shfl_up(myG0, 1, 64);
        double dG = __shfl_up(myG0p, 1, 64);
        if (lane == 0 && j >= 1 && j <= Ly) {
          upK = rowK[j];
          upG = rowG[j];
          dG = rowG[j - 1];
        }
        double nK0 = myK0, nG0 = myG0;
        if (j == 0) {
          nK0 = 1.0;
          nG0 = g0col;
          K1p = 0.0;
          G1p = 0.0;
        } else if (j >= 1 && j <= Ly && row_ok) {
          double v = use_w ? dG * (double)xw * (double)ywt[j - 1] : dG;
          const int yc = ycode[j - 1];
          if (naive) {
            // string_kernel.cpp:41-44: K1/G1 += G0[i-1][j-1]*g2 on x[i-1]==y[j-1]
            v = (xcode == yc) ? dG * (gap * gap) : 0.0;
          } else {
            v *= (xcode >= 0 && yc >= 0) ? st[xcode * 4 + yc] : prof_subst(st, xc, yprof[j - 1]);
          }
          const double K1 = v + K1p;
          const double G1 = v + G1p * gap;
          nK0 = K1 + upK;
          nG0 = G1 + upG * gap;
          K1p = K1;
          G1p = G1;
          if (i == Lx && j == Ly) result = nK0;
        }
        if (lane == 63 && j >= 0 && j <= Ly) {
          rowK[j] = nK0;
          rowG[j] = nG0;
        }
        myG0p = myG0;
        myK0 = nK0;
        myG0 = nG0;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    // the lane that owned row Lx holds the result
    const int owner = Lx == 0 ? 0 : ((Lx - 1) & 63);
    result = (Lx == 0 || Ly == 0) ? 1.0 : __shfl(result, owner, 64);
    if (lane == 0) P.out[pr] = result;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

size_t str_lds_bytes(const StrLaunch& P, int nwaves) {
  const size_t L = (size_t)P.lds_max_len;
  return 16 * 8 + (size_t)nwaves * (2 * (L + 2) * 8 + L * 16 + L * 4 + L * 4);
}

hipError_t launch_str(const StrLaunch& P, int grid, int nwaves, hipStream_t st) {
  const size_t lds = str_lds_bytes(P, nwaves);
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute((const void*)sk_profile_string_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(sk_profile_string_kernel, dim3(grid), dim3(64 * nwaves),
                     str_lds_bytes(P, nwaves), st, P);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Kernel combinators (common/conv_kernel.h:12-100) as an epilogue.
__global__ void sk_combine_kernel(const double* __restrict__ stem, const double* __restrict__ str,
                                  double* __restrict__ out, int64_t n, int32_t mode, double alpha,
                                  double beta) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  double r;
  switch (mode) {
    case kCombineStem: r = stem[k]; break;
    case kCombineStr: r = str[k]; break;
    case kCombineAdd: r = stem[k] + str[k]; break;
    case kCombineLogStem: r = beta * log(stem[k]) + 0.0; break;
    default: r = (beta * log(stem[k]) + 0.0) + (alpha * log(str[k]) + 0.0); break;
  }
  out[k] = r;
}

hipError_t launch_combine(const double* stem, const double* str, double* out, int64_t n,
                          int32_t mode, double alpha, double beta, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const int bs = 256;
  const int64_t grid = (n + bs - 1) / bs;
  hipLaunchKernelGGL(sk_combine_kernel, dim3((unsigned)grid), dim3(bs), 0, st, stem, str, out, n,
                     mode, alpha, beta);
  return hipGetLastError();
}

}  // namespace sk
