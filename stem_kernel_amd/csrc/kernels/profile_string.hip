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

#include <type_traits>

#include "bpla_fast.h"
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
    pr = ((unsigned long long)__builtin_amdgcn_readlane((unsigned)(pr >> 32), 0) << 32) |
         (unsigned)__builtin_amdgcn_readlane((unsigned)pr, 0);
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
    if (lane == 0) P.out[P.oidx ? P.oidx[pr] : (int64_t)pr] = result;
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
// Fast path: profiles whose columns are dyadic (multiples of 1/256: single
// sequences, alignments of 2^k rows, IUPAC codes) and never empty.  There
// subst_score's float weight n = xs * ys exactly, so with per-position
// operands (sk_str_tab_kernel) the weighted score of a cell is
// sum_l vx_l vy_l: four FMAs instead of 16 products, a float sum and a
// divide.  The DP (string_kernel.cpp:10-62, as the general kernel above):
//   v = G0[i-1][j-1] * w_x w_y subst;  K1 = v + K1[i][j-1];  G1 = v + G1[i][j-1] g
//   K0 = K1 + K0[i-1][j];  G0 = G1 + G0[i-1][j] g;  row 0: (1, g^j); column 0: (1, g^i)
// runs on the systolic schedule of the BPLA fast path (bpla.hip): lane l
// owns row 64s + l + 1, the row above arrives from lane l-1 by DPP
// wave_shr, strips are streamed, and the steps fall in wave-uniform windows
// (lane w starts its next row) and interiors (no per-lane control flow).
// The result K0[Lx][Ly] is the last output of the lane that owns row Lx.
__global__ void __launch_bounds__(256) sk_str_tab_kernel(const float4* __restrict__ prof,
                                                         const float* __restrict__ pos_w, int64_t n,
                                                         const double* __restrict__ st,
                                                         StrPos* __restrict__ xrole,
                                                         StrPos* __restrict__ yrole) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const float4 c = prof[p];
  const double s = (double)(c.x + c.y + c.z + c.w);  // exact for dyadic columns
  const double w = (double)pos_w[p];
  const float cv[4] = {c.x, c.y, c.z, c.w};
  StrPos X, Y;
#pragma unroll
  for (int l = 0; l < 4; ++l) {
    const double u = st[l] * (double)c.x + st[4 + l] * (double)c.y + st[8 + l] * (double)c.z +
                     st[12 + l] * (double)c.w;
    X.v[l] = s > 0.0 ? u / s * w : 0.0;
    Y.v[l] = s > 0.0 ? (double)cv[l] / s * w : 0.0;
  }
  xrole[p] = X;
  yrole[p] = Y;
}

hipError_t launch_str_tab(const float4* prof, const float* pos_w, int64_t n, const double* st, StrPos* xrole,
                          StrPos* yrole, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(sk_str_tab_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, prof, pos_w,
                     n, st, xrole, yrole);
  return hipGetLastError();
}

__global__ void __launch_bounds__(256) sk_str_code_tab_kernel(const float4* __restrict__ prof,
                                                              const float* __restrict__ pos_w, int64_t n,
                                                              StrCode* __restrict__ tab) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  StrCode c;
  c.w = pos_w[p];
  c.code = onehot_code(prof[p]);
  tab[p] = c;
}

hipError_t launch_str_code_tab(const float4* prof, const float* pos_w, int64_t n, StrCode* tab,
                               hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(sk_str_code_tab_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, prof,
                     pos_w, n, tab);
  return hipGetLastError();
}

// One pair on one wavefront; ycol: the y operands (LDS), bnd: the strip
// boundary row {K0, G0} per column (LDS, row 0 on entry).  OH: one-hot
// columns, subst = st[code_x][code_y] w_x w_y (the general kernel's one-hot
// case); else the dyadic factors.
template <bool OH>
__device__ __forceinline__ double str_fast_pair(const StrFastLaunch& P, int x, int Ly, const void* ycol,
                                                double* bnd, const double* st, int lane) {
  typedef typename std::conditional<OH, StrCode, StrPos>::type Op;
  const Op* xtab = reinterpret_cast<const Op*>(P.xtab);
  const double gap = P.gap;
  const int Lx = __builtin_amdgcn_readfirstlane(P.xset.ex_len[x]);
  const int xpb = __builtin_amdgcn_readfirstlane(P.xset.ex_pos_base[x]);
  if (Lx == 0 || Ly == 0) return 1.0;
  const int Lys = max(Ly, 64);
  const int nstrips = (Lx + 63) / 64;
  const int T = (nstrips - 1) * Lys + ((Lx - 1) & 63) + Ly;
  const char* ybase = reinterpret_cast<const char*>(ycol);
  // my row operands and G0 of the row above at column 0, the next strip's
  Op xn = xtab[xpb + min(lane, Lx - 1)];
  double dn = P.gpow[lane];  // G0[i-1][0] = g^(i-1)
  Op xr = xn;
  unsigned yofs = 0;
  double lK1 = 0.0, lG1 = 0.0, lK0 = 0.0, lG0 = 0.0;  // my (i, j-1) values
  double dG = 0.0;                                     // G0[i-1][j-1]

  auto cell = [&](double uK, double uG, bool c1) __attribute__((always_inline)) {
    const Op yc = *reinterpret_cast<const Op*>(ybase + yofs);
    double v;
    if constexpr (OH) {
      v = dG * (double)xr.w * (double)yc.w * st[xr.code * 4 + yc.code];
    } else {
      double s = xr.v[0] * yc.v[0];
      s = __builtin_fma(xr.v[1], yc.v[1], s);
      s = __builtin_fma(xr.v[2], yc.v[2], s);
      s = __builtin_fma(xr.v[3], yc.v[3], s);
      v = dG * s;
    }
    const double K1 = c1 ? v : v + lK1;
    const double G1 = c1 ? v : __builtin_fma(lG1, gap, v);
    lK1 = K1;
    lG1 = G1;
    lK0 = K1 + uK;
    lG0 = __builtin_fma(uG, gap, G1);
  };
  // interior step: every lane inside strip s; lane 0 at column jb
  auto interior = [&](int jb) __attribute__((always_inline)) {
    const double* bj = bnd + 2 * jb;
    const double uK = wave_shr1(lK0, bj[0]);
    const double uG = wave_shr1(lG0, bj[1]);
    cell(uK, uG, false);
    if (lane == 63) {
      double* bw = bnd + 2 * (jb - 63);
      bw[0] = lK0;
      bw[1] = lG0;
    }
    dG = uG;
    yofs += (unsigned)sizeof(Op);
  };
  // window step w of strip s: lane w starts its row at column 1
  auto window = [&](int s, int w) __attribute__((always_inline)) {
    const bool wrap = lane == w;
    if (wrap) {
      xr = xn;
      dG = dn;
      yofs = 0;
    }
    const int jl = lane <= w ? w - lane + 1 : Lys + w - lane + 1;
    const bool on = jl <= Ly && (lane <= w ? s < nstrips : s > 0);
    const int jb = w + 1;
    const double* bj = bnd + 2 * (jb <= Ly ? jb : 0);
    const double uK = wave_shr1(lK0, bj[0]);
    const double uG = wave_shr1(lG0, bj[1]);
    if (on) {
      cell(uK, uG, wrap);
      if (lane == 63) {
        double* bw = bnd + 2 * jl;
        bw[0] = lK0;
        bw[1] = lG0;
      }
    }
    dG = uG;
    yofs += (unsigned)sizeof(Op);
  };
  for (int s = 0; s <= nstrips; ++s) {
    const int Ws = s * Lys;
    const int wend = min(64, T - Ws);
    if (wend <= 0) break;
    for (int w = 0; w < wend; ++w) window(s, w);
    if (s + 1 < nstrips) {
      const int i1 = 64 * (s + 1) + lane;  // 0-based row of my next strip
      xn = xtab[xpb + min(i1, Lx - 1)];
      dn = P.gpow[min(i1, Lx)];
    }
    const int tend = s < nstrips ? min(Ws + Lys, T) : 0;
    for (int t = Ws + 64; t < tend; ++t) interior(t - Ws + 1);
  }
  const int owner = (Lx - 1) & 63;
  const double r = __shfl(lK0, owner, 64);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return r;
}

template <bool OH>
__global__ void __launch_bounds__(256) sk_str_fast_kernel(StrFastLaunch P) {
  typedef typename std::conditional<OH, StrCode, StrPos>::type Op;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int maxlen = P.lds_max_len;
  double* st = reinterpret_cast<double*>(smem);
  if (threadIdx.x < 16) st[threadIdx.x] = OH ? P.st[threadIdx.x] : 0.0;
  __syncthreads();
  unsigned char* wbase = smem + kStrFastLds0 + (size_t)wave * str_fast_wave_lds_bytes(maxlen, OH);
  Op* ycol = reinterpret_cast<Op*>(wbase);
  double* bnd = reinterpret_cast<double*>(ycol + maxlen);
  const Op* ytab = reinterpret_cast<const Op*>(P.ytab);
  // pairs dealt cyclically to the waves (costs within a call are alike)
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t pr = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave; pr < P.n_pairs; pr += nw) {
    const int x = __builtin_amdgcn_readfirstlane(P.xs[pr]);
    const int y = __builtin_amdgcn_readfirstlane(P.ys[pr]);
    const int Ly = __builtin_amdgcn_readfirstlane(P.yset.ex_len[y]);
    const int ypb = P.yset.ex_pos_base[y];
    const int Lys = max(Ly, 64);
    for (int j = lane; j < Ly; j += 64) ycol[j] = ytab[ypb + j];
    for (int j = lane; j <= Lys; j += 64) {  // row 0: K0 = 1, G0 = g^j
      bnd[2 * j] = 1.0;
      bnd[2 * j + 1] = j <= Ly ? P.gpow[j] : 0.0;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const double r = str_fast_pair<OH>(P, x, Ly, ycol, bnd, st, lane);
    if (lane == 0) P.out[P.oidx ? P.oidx[pr] : pr] = r;
  }
}

hipError_t launch_str_fast(const StrFastLaunch& P, int grid, int nwaves, hipStream_t stream) {
  const size_t lds = kStrFastLds0 + (size_t)nwaves * str_fast_wave_lds_bytes(P.lds_max_len, P.onehot != 0);
  const void* fn = P.onehot ? (const void*)sk_str_fast_kernel<true> : (const void*)sk_str_fast_kernel<false>;
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  if (P.onehot)
    hipLaunchKernelGGL(sk_str_fast_kernel<true>, dim3(grid), dim3(64 * nwaves), lds, stream, P);
  else
    hipLaunchKernelGGL(sk_str_fast_kernel<false>, dim3(grid), dim3(64 * nwaves), lds, stream, P);
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
