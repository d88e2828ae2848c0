// PairHMM alignment constraints of the 4-D stem kernel (-a option) on CDNA4.
//
// Reference: StemKernel::alignment_constraints  stem_kernel/stem_kernel.cpp:14-81,
//   PairHMM<Ribosum>::forward / backward / forward_backward  stem_kernel/phmm.cpp:10-115,
//   MAP forward + traceback  phmm.cpp:117-236, Ribosum scores  phmm.cpp:247-320,
//   LogValue<double> arithmetic  stem_kernel/log_value.h:55-389 (FAST_LOG1EXP0, :28).
//
// One wavefront per (x, y) pair of a 4-D batch, sweeping 64-row strips of
// the |x| x |y| tables along anti-diagonals (see sk_phmm_kernel).  Lane 0
// writes c_low / c_high (|x|+1 each) straight into the band arrays the 4-D
// kernel reads, so nothing returns to the host.
//
// Bit-level agreement with the host restatement: log1exp0 is the probcons
// polynomial (no libm), evaluated without FMA contraction (this file is built
// with -ffp-contract=off), and every log-space sum keeps the reference's
// operand order.  Only exp() of the posterior comes from the device libm.
#include <hip/hip_runtime.h>

#include "device_set.h"
#include "launch.h"

namespace sk {
namespace {

enum { kM = 0, kIX = 1, kIY = 2 };

// ribosum_trans / ribosum_emit (phmm.cpp:262-276), kept as logs (ExpOf)
__constant__ double kTrans[3][3] = {{0.0, -5.0, -5.0}, {-10.0, -5.0, -15.0}, {-10.0, -5.0, -15.0}};
__constant__ double kEmit[4][4] = {{2.22, -1.86, -1.46, -1.39},
                                   {-1.86, 1.16, -2.48, -1.05},
                                   {-1.46, -2.48, 1.03, -1.74},
                                   {-1.39, -1.05, -1.74, 1.65}};

// log(exp(x)+1) as LogValue::log1exp0 with FAST_LOG1EXP0 (log_value.h:312-347).
// The four cubic segments use float constants; they are evaluated in the
// quartic's Horner form with a leading 0 (0*x + b == b exactly), so every
// segment is one straight-line polynomial.  x is >= 0 or NaN here.
__device__ __forceinline__ double log1exp0(double x) {
  double a = 0.0, b, c, d, e;
  if (x <= 1.00) {
    b = (double)-0.009350833524763f, c = (double)0.130659527668286f;
    d = (double)0.498799810682272f, e = (double)0.693203116424741f;
  } else if (x <= 2.50) {
    b = (double)-0.014532321752540f, c = (double)0.139942324101744f;
    d = (double)0.495635523139337f, e = (double)0.692140569840976f;
  } else if (x <= 4.50) {
    b = (double)-0.004605031767994f, c = (double)0.063427417320019f;
    d = (double)0.695956496475118f, e = (double)0.514272634594009f;
  } else if (x <= 7.50) {
    b = (double)-0.000458661602210f, c = (double)0.009695946122598f;
    d = (double)0.930734667215156f, e = (double)0.168037164329057f;
  } else {
    a = 0.00000051726300753785, b = -0.00002720671238876090, c = 0.00053403733818413500;
    d = 0.99536021775747900000, e = 0.01507065715532010000;
  }
  const double r = (((a * x + b) * x + c) * x + d) * x + e;
  return x > 10.0 ? x : r;
}

// LogValue::operator+= (log_value.h:212-224).  fixed: zerop detects -inf;
// otherwise zerop is never true (std::isinf(...) < 0 with a bool isinf).
__device__ __forceinline__ double lv_add(double a, double b, bool fixed) {
  if (fixed) {
    if (b == -__builtin_inf()) return a;
    if (a == -__builtin_inf()) return b;
  }
  return a < b ? a + log1exp0(b - a) : b + log1exp0(a - b);
}

__device__ __forceinline__ int base_code(uint8_t c) {
  switch (c) {
    case 'a': case 'A': return 0;
    case 'c': case 'C': return 1;
    case 'g': case 'G': return 2;
    default: return 3;  // 'u' / 'U' (the host rejects anything else)
  }
}

// MAP step of PairHMM::forward(fb, tr) (phmm.cpp:160-183): the first state
// sets the cell, later ones replace it only when strictly larger.
__device__ __forceinline__ void best3(double v0, double v1, double v2, double& best, int& arg) {
  best = v0, arg = 0;
  if (best < v1) best = v1, arg = 1;
  if (best < v2) best = v2, arg = 2;
}

// DPP: lane l receives lane l-1's value (lane 0 receives `low`), wave_shr:1
__device__ __forceinline__ double shr1(double v, double low) {
  const int rlo = __builtin_amdgcn_update_dpp(__double2loint(low), __double2loint(v), 0x138, 0xf, 0xf, false);
  const int rhi = __builtin_amdgcn_update_dpp(__double2hiint(low), __double2hiint(v), 0x138, 0xf, 0xf, false);
  return __hiloint2double(rhi, rlo);
}
// lane l receives lane l+1's value (lane 63 receives `high`), wave_shl:1
__device__ __forceinline__ double shl1(double v, double high) {
  const int rlo = __builtin_amdgcn_update_dpp(__double2loint(high), __double2loint(v), 0x130, 0xf, 0xf, false);
  const int rhi = __builtin_amdgcn_update_dpp(__double2hiint(high), __double2hiint(v), 0x130, 0xf, 0xf, false);
  return __hiloint2double(rhi, rlo);
}

// One WAVEFRONT per pair.  Rows 1..|x| are cut into strips of 64, lane l of
// strip s owning row i = 64s + 1 + l; the strip sweeps anti-diagonals, lane l
// handling column j = t - l at step t (t - (63 - l) counted from the right in
// the backward pass), so a cell's row-above neighbours come from lane l-1 by
// DPP (one and two steps old) and its left neighbour is the lane's own
// previous output.  Row 0 (whose recurrences differ) is done by lane 0 alone.
// The strip's boundary row lives in LDS.  Tables are stored skewed,
// element (strip s, step t, state, lane) at ((s*T + t)*3 + state)*64 + lane,
// so every store and load of a step is 512 contiguous bytes.
__global__ void __launch_bounds__(64) sk_phmm_kernel(PhmmLaunch P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int pidx = blockIdx.x;
  const int l = threadIdx.x;
  const Stem4dPair pr = P.pairs[pidx];
  const int n = pr.n, m = pr.m;
  const int M1 = P.m1;
  const int T = m + 64;          // steps of a strip
  const int nS = (n + 63) / 64;  // strips
  double* FBS = reinterpret_cast<double*>(P.scratch + (size_t)pidx * P.pair_bytes);
  uint8_t* TRS = reinterpret_cast<uint8_t*>(FBS + (size_t)nS * T * 3 * 64);
  // LDS: boundary row (3 x M1), row 0 (3 x M1), y codes (M1), path (N1 + M1)
  double* buf = reinterpret_cast<double*>(smem);
  double* row0 = buf + 3 * M1;
  int32_t* yc = reinterpret_cast<int32_t*>(row0 + 3 * M1);
  int32_t* path = yc + M1;
  const uint8_t* xs = P.chars + pr.x_chr;
  const uint8_t* ys = P.chars_y + pr.y_chr;
  const bool fx = P.zerop_fixed != 0;
  const double NEG = -__builtin_inf();
#define SKW(s_, t_, st_) (((size_t)(s_) * T + (t_)) * 3 + (st_)) * 64 + l
  for (int j = l; j < M1; j += 64) yc[j] = j < m ? base_code(ys[j]) : 0;
  __syncthreads();

  // ---- forward (phmm.cpp:10-50), log values
  double wlog = 0.0;  // fw[M][n][m]
  if (l == 0) {       // row 0: M = IX = 0 past (0,0), IY from the left
    double f0 = 0.0, f1 = NEG, f2 = NEG;
    row0[0] = buf[0] = f0, row0[M1] = buf[M1] = f1, row0[2 * M1] = buf[2 * M1] = f2;
    for (int j = 1; j <= m; ++j) {
      double y2 = NEG;
      y2 = lv_add(y2, f0 + kTrans[0][kIY], fx);
      y2 = lv_add(y2, f1 + kTrans[1][kIY], fx);
      y2 = lv_add(y2, f2 + kTrans[2][kIY], fx);
      f0 = NEG, f1 = NEG, f2 = y2;
      row0[j] = buf[j] = f0, row0[M1 + j] = buf[M1 + j] = f1, row0[2 * M1 + j] = buf[2 * M1 + j] = f2;
    }
    if (n == 0) wlog = row0[m];
  }
  __syncthreads();
  for (int s = 0; s < nS; ++s) {
    const int i = 64 * s + 1 + l;
    const bool row_ok = i <= n;
    const int xc = row_ok ? base_code(xs[i - 1]) : 0;
    double o0 = NEG, o1 = NEG, o2 = NEG;  // own output of the previous step: (i, j-1)
    double d0 = NEG, d1 = NEG, d2 = NEG;  // lane l-1's output two steps ago: (i-1, j-1)
    for (int t = 0; t < T; ++t) {
      const int j = t - l;
      // (i-1, j): lane l-1's previous output, lane 0 from the boundary row
      const bool b0 = l == 0 && t <= m;
      const double u0 = shr1(o0, b0 ? buf[t] : 0.0);
      const double u1 = shr1(o1, b0 ? buf[M1 + t] : 0.0);
      const double u2 = shr1(o2, b0 ? buf[2 * M1 + t] : 0.0);
      double M = NEG, X = NEG, Y = NEG;
      if (j == 0) {  // column 0: M = IY = 0, IX from above
        X = lv_add(X, u0 + kTrans[0][kIX], fx);
        X = lv_add(X, u1 + kTrans[1][kIX], fx);
        X = lv_add(X, u2 + kTrans[2][kIX], fx);
      } else {
        const double e = kEmit[xc][yc[min(max(j - 1, 0), M1 - 1)]];
        M = lv_add(M, d0 + (kTrans[0][kM] + e), fx);
        X = lv_add(X, u0 + kTrans[0][kIX], fx);
        Y = lv_add(Y, o0 + kTrans[0][kIY], fx);
        M = lv_add(M, d1 + (kTrans[1][kM] + e), fx);
        X = lv_add(X, u1 + kTrans[1][kIX], fx);
        Y = lv_add(Y, o1 + kTrans[1][kIY], fx);
        M = lv_add(M, d2 + (kTrans[2][kM] + e), fx);
        X = lv_add(X, u2 + kTrans[2][kIX], fx);
        Y = lv_add(Y, o2 + kTrans[2][kIY], fx);
      }
      const bool ok = row_ok && j >= 0 && j <= m;
      if (ok) {
        FBS[SKW(s, t, 0)] = M, FBS[SKW(s, t, 1)] = X, FBS[SKW(s, t, 2)] = Y;
        if (i == n && j == m) wlog = M;
        if (l == 63) buf[j] = M, buf[M1 + j] = X, buf[2 * M1 + j] = Y;  // next strip's row above
      }
      d0 = u0, d1 = u1, d2 = u2;
      o0 = M, o1 = X, o2 = Y;
    }
    __syncthreads();
  }
  wlog = __shfl(wlog, n == 0 ? 0 : (n - 1) & 63, 64);

  // ---- backward (phmm.cpp:52-93) in gather form + posterior (:95-115);
  // contributions in the reference's scatter order (see the oracle): main
  // loop (a+1,b+1) [M], (a+1,b) [IX], (a,b+1) [IY], then the column-0 loop
  // (and, for row 0, the row-0 loop) with their resets.
  for (int s = nS - 1; s >= 0; --s) {
    const int a = 64 * s + 1 + l;
    const bool row_ok = a <= n;
    const int xc = a < n ? base_code(xs[a]) : 0;
    double o0 = NEG, o1 = NEG, o2 = NEG;  // own previous output: (a, b+1)
    double dM = NEG;                      // lane l+1's output two steps ago: bk(M, a+1, b+1)
    for (int t = 0; t < T; ++t) {
      const int b = m + 63 - l - t;
      const bool b63 = l == 63 && b >= 0 && b <= m && a < n;
      // (a+1, b): lane l+1's previous output, lane 63 from the boundary row
      const double vM = shl1(o0, b63 ? buf[b] : 0.0);
      const double vX = shl1(o1, b63 ? buf[M1 + b] : 0.0);
      double acc[3];
#pragma unroll
      for (int q = 0; q < 3; ++q) acc[q] = (q == kM && a == n && b == m) ? 0.0 : NEG;
      if (a < n) {
        if (b < m) {
          const double e = kEmit[xc][yc[min(max(b, 0), M1 - 1)]];
#pragma unroll
          for (int q = 0; q < 3; ++q) acc[q] = lv_add(acc[q], dM + (kTrans[q][kM] + e), fx);
        }
        if (b >= 1) {
#pragma unroll
          for (int q = 0; q < 3; ++q) acc[q] = lv_add(acc[q], vX + kTrans[q][kIX], fx);
        }
      }
      if (b < m) {
#pragma unroll
        for (int q = 0; q < 3; ++q) acc[q] = lv_add(acc[q], o2 + kTrans[q][kIY], fx);
      }
      if (b == 0) {  // column-0 loop: source (a+1, 0), then the reset
        if (a < n) {
#pragma unroll
          for (int q = 0; q < 3; ++q) acc[q] = lv_add(acc[q], vX + kTrans[q][kIX], fx);
        }
        acc[kM] = acc[kIY] = NEG;
      }
      const bool ok = row_ok && b >= 0 && b <= m;
      if (ok) {
        const int tf = b + l;  // forward step of cell (a, b)
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const size_t o = SKW(s, tf, q);
          FBS[o] = exp((FBS[o] + acc[q]) - wlog);
        }
        if (l == 0) buf[b] = acc[0], buf[M1 + b] = acc[1], buf[2 * M1 + b] = acc[2];
      }
      dM = vM;
      o0 = acc[0], o1 = acc[1], o2 = acc[2];
    }
    __syncthreads();
  }
  if (l == 0) {  // row 0 (a = 0): main loop from row 1, row-0 loop, column-0 loop
    const int xc = n > 0 ? base_code(xs[0]) : 0;
    double c2 = NEG;  // bk(IY, 0, b+1)
    for (int b = m; b >= 0; --b) {
      double acc[3];
#pragma unroll
      for (int q = 0; q < 3; ++q) acc[q] = (q == kM && n == 0 && b == m) ? 0.0 : NEG;
      if (n >= 1) {
        if (b < m) {
          const double e = kEmit[xc][yc[b]];
#pragma unroll
          for (int q = 0; q < 3; ++q) acc[q] = lv_add(acc[q], buf[b + 1] + (kTrans[q][kM] + e), fx);
        }
        if (b >= 1) {
#pragma unroll
          for (int q = 0; q < 3; ++q) acc[q] = lv_add(acc[q], buf[M1 + b] + kTrans[q][kIX], fx);
        }
      }
      if (b < m) {
#pragma unroll
        for (int q = 0; q < 3; ++q) acc[q] = lv_add(acc[q], c2 + kTrans[q][kIY], fx);
      }
      if (b >= 1) {
        acc[kM] = acc[kIX] = NEG;
      } else if (n >= 1) {
#pragma unroll
        for (int q = 0; q < 3; ++q) acc[q] = lv_add(acc[q], buf[M1] + kTrans[q][kIX], fx);
      }
#pragma unroll
      for (int q = 0; q < 3; ++q) row0[q * M1 + b] = exp((row0[q * M1 + b] + acc[q]) - wlog);
      c2 = acc[2];
    }
  }
  __syncthreads();

  // ---- MAP path over the posteriors: PairHMM::forward(fb, tr) (phmm.cpp:117-185)
  if (l == 0) {  // row 0
    double p0 = row0[0], p1 = row0[M1], p2 = row0[2 * M1];
    buf[0] = p0, buf[M1] = p1, buf[2 * M1] = p2;
    for (int j = 1; j <= m; ++j) {
      const double fy = row0[2 * M1 + j];
      double bst;
      int k;
      best3(p0 + fy, p1 + fy, p2 + fy, bst, k);
      p0 = 0.0, p1 = 0.0, p2 = bst;
      buf[j] = p0, buf[M1 + j] = p1, buf[2 * M1 + j] = p2;
    }
  }
  __syncthreads();
  for (int s = 0; s < nS; ++s) {
    const int i = 64 * s + 1 + l;
    const bool row_ok = i <= n;
    double o0 = 0.0, o1 = 0.0, o2 = 0.0, d0 = 0.0, d1 = 0.0, d2 = 0.0;
    for (int t = 0; t < T; ++t) {
      const int j = t - l;
      const bool b0 = l == 0 && t <= m;
      const double u0 = shr1(o0, b0 ? buf[t] : 0.0);
      const double u1 = shr1(o1, b0 ? buf[M1 + t] : 0.0);
      const double u2 = shr1(o2, b0 ? buf[2 * M1 + t] : 0.0);
      const bool ok = row_ok && j >= 0 && j <= m;
      double fM = 0.0, fX = 0.0, fY = 0.0;
      if (ok) fM = FBS[SKW(s, t, 0)], fX = FBS[SKW(s, t, 1)], fY = FBS[SKW(s, t, 2)];
      double bm = 0.0, bx, by = 0.0;
      int km = 3, kx, ky = 3;
      if (j == 0) {
        best3(u0 + fX, u1 + fX, u2 + fX, bx, kx);
      } else {
        best3(d0 + fM, d1 + fM, d2 + fM, bm, km);
        best3(u0 + fX, u1 + fX, u2 + fX, bx, kx);
        best3(o0 + fY, o1 + fY, o2 + fY, by, ky);
      }
      if (ok) {
        TRS[((size_t)s * T + t) * 64 + l] = (uint8_t)(km | (kx << 2) | (ky << 4));
        if (l == 63) buf[j] = bm, buf[M1 + j] = bx, buf[2 * M1 + j] = by;
      }
      d0 = u0, d1 = u1, d2 = u2;
      o0 = bm, o1 = bx, o2 = by;
    }
    __syncthreads();
  }

  // ---- traceback (phmm.cpp:187-216) and anchors (stem_kernel.cpp:40-67)
  if (l == 0) {
    int len = 0;
    int st = kM, x = n, y = m;
    path[len++] = (st << 30) | (x << 15) | y;
    while (x != 0 && y != 0) {
      const int sx = (x - 1) >> 6, lx = (x - 1) & 63;
      const int code = (TRS[((size_t)sx * T + y + lx) * 64 + lx] >> (2 * st)) & 3;
      if (st == kM) --x, --y;
      else if (st == kIX) --x;
      else --y;
      if (code == 3) break;  // unreachable: interior cells always have a predecessor
      st = code;
      path[len++] = (st << 30) | (x << 15) | y;
    }
    int32_t* clo = P.band_lo + pr.band_off;
    int32_t* chi = P.band_hi + pr.band_off;
    int low_x = 0, low_y = 0;
    for (int k = len - 1; k >= 0; --k) {
      const int32_t v = path[k];
      const int ps = (v >> 30) & 3, px = (v >> 15) & 0x7fff, py = v & 0x7fff;
      if (ps != kM) continue;
      double post;
      if (px == 0) {
        post = row0[py];
      } else {
        const int sx = (px - 1) >> 6, lx = (px - 1) & 63;
        post = FBS[(((size_t)sx * T + py + lx) * 3 + kM) * 64 + lx];
      }
      if (post >= (double)P.ali_bound) {
        for (int i = low_x; i < px; ++i) clo[i] = low_y, chi[i] = py;
        clo[px] = py, chi[px] = py;
        low_x = px + 1, low_y = py;
      }
    }
    for (int i = low_x; i <= n; ++i) clo[i] = low_y, chi[i] = m;
    const int band = (int)P.band;
    if (band > 0)
      for (int i = 0; i <= n; ++i)
        if (chi[i] - clo[i] < band * 2) {
          const int j = (chi[i] + clo[i]) / 2;
          clo[i] = j < band ? 0 : j - band;
          chi[i] = j + band > m ? m : j + band;
        }
  }
#undef SKW
}

}  // namespace

size_t phmm_pair_bytes(int n1, int m1) {
  const size_t nS = (size_t)(n1 - 1 + 63) / 64, T = (size_t)m1 - 1 + 64;
  return (nS * T * (3 * 64 * 8 + 64) + 255) & ~(size_t)255;
}

size_t phmm_lds_bytes(int n1, int m1) { return (size_t)m1 * (6 * 8 + 4) + (size_t)(n1 + m1) * 4 + 16; }

hipError_t launch_phmm(const PhmmLaunch& P, hipStream_t st) {
  if (P.n_pairs == 0) return hipSuccess;
  const size_t lds = phmm_lds_bytes(P.n1, P.m1);
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(sk_phmm_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(sk_phmm_kernel, dim3((unsigned)P.n_pairs), dim3(64), lds, st, P);
  return hipGetLastError();
}

}  // namespace sk
