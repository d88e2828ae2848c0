// PairHMM alignment constraints of the 4-D stem kernel (-a option) on CDNA4.
//
// Reference: StemKernel::alignment_constraints  stem_kernel/stem_kernel.cpp:14-81,
//   PairHMM<Ribosum>::forward / backward / forward_backward  stem_kernel/phmm.cpp:10-115,
//   MAP forward + traceback  phmm.cpp:117-236, Ribosum scores  phmm.cpp:247-320,
//   LogValue<double> arithmetic  stem_kernel/log_value.h:55-389 (FAST_LOG1EXP0, :28).
//
// One thread per (x, y) pair of a 4-D batch: the PairHMM is O(|x||y|) per pair
// against the 4-D DP's O(|x|^2 |y|^2), so it only has to stay out of the way
// (it costs < 1 % of a batch).  Per-pair tables are interleaved across the
// pairs of the launch (element e of pair t at e*P + t, laid out for the
// launch's largest |x|, |y|), so the 64 lanes of a wave touch 512 contiguous
// bytes per access.  The thread writes c_low / c_high (|x|+1 each) straight
// into the band arrays the 4-D kernel reads, so nothing returns to the host.
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

__global__ void __launch_bounds__(64) sk_phmm_kernel(PhmmLaunch P) {
  const int64_t t = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (t >= P.n_pairs) return;
  const Stem4dPair pr = P.pairs[t];
  const int n = pr.n, m = pr.m;
  const int64_t S = P.n_pairs, N1 = P.n1, M1 = P.m1;
  double* FB = reinterpret_cast<double*>(P.scratch);  // 3 x N1 x M1: log fw, then posterior
  double* BR = FB + 3 * N1 * M1 * S;                   // 2 rows x 3 x M1: backward
  double* MR = BR + 6 * M1 * S;                        // 2 rows x 3 x M1: MAP forward
  int32_t* PATH = reinterpret_cast<int32_t*>(MR + 6 * M1 * S);  // N1 + M1 steps
  uint8_t* TR = reinterpret_cast<uint8_t*>(PATH + (N1 + M1) * S);  // N1 x M1, 2 bits per state
#define FBA(s, i, j) FB[(((int64_t)(s) * N1 + (i)) * M1 + (j)) * S + t]
#define BRA(r, s, j) BR[(((int64_t)(r) * 3 + (s)) * M1 + (j)) * S + t]
#define MRA(r, s, j) MR[(((int64_t)(r) * 3 + (s)) * M1 + (j)) * S + t]
#define TRA(i, j) TR[((int64_t)(i) * M1 + (j)) * S + t]
  const uint8_t* xs = P.chars + pr.x_chr;
  const uint8_t* ys = P.chars + pr.y_chr;
  const bool fx = P.zerop_fixed != 0;
  const double NEG = -__builtin_inf();

  // Every pass streams its thread's previous row (and, backward, the forward
  // values) from HBM/L2 in chunks, issuing the next chunk's loads before the
  // current chunk's arithmetic, so the latency of a load is paid once per
  // chunk rather than once per cell.
  constexpr int CF = 4, CB = 4, CM = 4;

  // ---- forward (phmm.cpp:10-50): log fw into FB
  {
    double f0 = 0.0, f1 = NEG, f2 = NEG;  // fw(., 0, 0): M = log 1
    FBA(0, 0, 0) = f0, FBA(1, 0, 0) = f1, FBA(2, 0, 0) = f2;
    for (int j = 1; j <= m; ++j) {  // row 0: M = IX = 0, IY from the left
      double y2 = NEG;
      y2 = lv_add(y2, f0 + kTrans[0][kIY], fx);
      y2 = lv_add(y2, f1 + kTrans[1][kIY], fx);
      y2 = lv_add(y2, f2 + kTrans[2][kIY], fx);
      f0 = NEG, f1 = NEG, f2 = y2;
      FBA(0, 0, j) = f0, FBA(1, 0, j) = f1, FBA(2, 0, j) = f2;
    }
  }
  for (int i = 1; i <= n; ++i) {
    const int xc = base_code(xs[i - 1]);
    // column 0: M = IY = 0, IX from above
    double u0 = FBA(0, i - 1, 0), u1 = FBA(1, i - 1, 0), u2 = FBA(2, i - 1, 0);  // (i-1, j-1)
    double c0 = NEG, c1 = NEG, c2 = NEG;                                        // (i, j-1)
    c1 = lv_add(c1, u0 + kTrans[0][kIX], fx);
    c1 = lv_add(c1, u1 + kTrans[1][kIX], fx);
    c1 = lv_add(c1, u2 + kTrans[2][kIX], fx);
    FBA(0, i, 0) = c0, FBA(1, i, 0) = c1, FBA(2, i, 0) = c2;
    double A0[CF], A1[CF], A2[CF], Q0[CF], Q1[CF], Q2[CF];  // (i-1, j) of this / next chunk
    int Ay[CF], Ny[CF];
    auto load = [&](int j0, double* B0, double* B1, double* B2, int* By) {
#pragma unroll
      for (int k = 0; k < CF; ++k) {
        const int j = j0 + k;
        B0[k] = B1[k] = B2[k] = 0.0;
        By[k] = 0;
        if (j <= m) {
          B0[k] = FBA(0, i - 1, j), B1[k] = FBA(1, i - 1, j), B2[k] = FBA(2, i - 1, j);
          By[k] = base_code(ys[j - 1]);
        }
      }
    };
    load(1, A0, A1, A2, Ay);
    for (int j0 = 1; j0 <= m; j0 += CF) {
      load(j0 + CF, Q0, Q1, Q2, Ny);
#pragma unroll
      for (int k = 0; k < CF; ++k) {
        if (j0 + k <= m) {
          const double e = kEmit[xc][Ay[k]];
          const double v0 = A0[k], v1 = A1[k], v2 = A2[k];
          double M = NEG, X = NEG, Y = NEG;
          M = lv_add(M, u0 + (kTrans[0][kM] + e), fx);
          X = lv_add(X, v0 + kTrans[0][kIX], fx);
          Y = lv_add(Y, c0 + kTrans[0][kIY], fx);
          M = lv_add(M, u1 + (kTrans[1][kM] + e), fx);
          X = lv_add(X, v1 + kTrans[1][kIX], fx);
          Y = lv_add(Y, c1 + kTrans[1][kIY], fx);
          M = lv_add(M, u2 + (kTrans[2][kM] + e), fx);
          X = lv_add(X, v2 + kTrans[2][kIX], fx);
          Y = lv_add(Y, c2 + kTrans[2][kIY], fx);
          FBA(0, i, j0 + k) = M, FBA(1, i, j0 + k) = X, FBA(2, i, j0 + k) = Y;
          c0 = M, c1 = X, c2 = Y;
          u0 = v0, u1 = v1, u2 = v2;
        }
      }
#pragma unroll
      for (int k = 0; k < CF; ++k) A0[k] = Q0[k], A1[k] = Q1[k], A2[k] = Q2[k], Ay[k] = Ny[k];
    }
  }
  const double wlog = FBA(0, n, m);  // fw[M][|x|][|y|]

  // ---- backward (phmm.cpp:52-93) in gather form, posterior fw*bk/w (:95-115)
  // Contributions to bk(s,a,b) arrive in the reference's scatter order: from
  // (a+1,b+1) [M], (a+1,b) [IX], (a,b+1) [IY] in the main loop, then the
  // row-0 and column-0 loops, which also reset M,IX of row 0 and M,IY of
  // column 0 after their last contribution.
  for (int a = n; a >= 0; --a) {
    const int r = a & 1, q = r ^ 1;
    const int xc = a < n ? base_code(xs[a]) : 0;
    double c2 = NEG;  // bk(IY, a, b+1)
    // per cell b: fw(s,a,b), bk(M,a+1,b+1), bk(IX,a+1,b), y code
    double AF0[CB], AF1[CB], AF2[CB], AM[CB], AX[CB], NF0[CB], NF1[CB], NF2[CB], NM[CB], NX[CB];
    int Ay[CB], Ny[CB];
    auto load = [&](int b0, double* F0, double* F1, double* F2, double* BM, double* BX, int* By) {
#pragma unroll
      for (int k = 0; k < CB; ++k) {
        const int b = b0 - k;
        F0[k] = F1[k] = F2[k] = BM[k] = BX[k] = 0.0;
        By[k] = 0;
        if (b >= 0) {
          F0[k] = FBA(0, a, b), F1[k] = FBA(1, a, b), F2[k] = FBA(2, a, b);
          if (a < n) {
            BX[k] = BRA(q, kIX, b);
            if (b < m) BM[k] = BRA(q, kM, b + 1), By[k] = base_code(ys[b]);
          }
        }
      }
    };
    load(m, AF0, AF1, AF2, AM, AX, Ay);
    for (int b0 = m; b0 >= 0; b0 -= CB) {
      load(b0 - CB, NF0, NF1, NF2, NM, NX, Ny);
#pragma unroll
      for (int k = 0; k < CB; ++k) {
        const int b = b0 - k;
        if (b >= 0) {
          double acc[3];
#pragma unroll
          for (int s = 0; s < 3; ++s) acc[s] = (s == kM && a == n && b == m) ? 0.0 : NEG;
          const double nX = AX[k];
          if (a < n) {
            if (b < m) {
              const double e = kEmit[xc][Ay[k]];
#pragma unroll
              for (int s = 0; s < 3; ++s) acc[s] = lv_add(acc[s], AM[k] + (kTrans[s][kM] + e), fx);
            }
            if (b >= 1) {
#pragma unroll
              for (int s = 0; s < 3; ++s) acc[s] = lv_add(acc[s], nX + kTrans[s][kIX], fx);
            }
          }
          if (a >= 1 && b < m) {
#pragma unroll
            for (int s = 0; s < 3; ++s) acc[s] = lv_add(acc[s], c2 + kTrans[s][kIY], fx);
          }
          if (a == 0) {
            if (b < m) {  // row-0 loop, source (0, b+1)
#pragma unroll
              for (int s = 0; s < 3; ++s) acc[s] = lv_add(acc[s], c2 + kTrans[s][kIY], fx);
            }
            if (b >= 1) {
              acc[kM] = acc[kIX] = NEG;
            } else if (n >= 1) {  // (0,0): column-0 loop, source (1, 0)
#pragma unroll
              for (int s = 0; s < 3; ++s) acc[s] = lv_add(acc[s], nX + kTrans[s][kIX], fx);
            }
          } else if (b == 0) {
            if (a < n) {  // column-0 loop, source (a+1, 0)
#pragma unroll
              for (int s = 0; s < 3; ++s) acc[s] = lv_add(acc[s], nX + kTrans[s][kIX], fx);
            }
            acc[kM] = acc[kIY] = NEG;
          }
          BRA(r, 0, b) = acc[0], BRA(r, 1, b) = acc[1], BRA(r, 2, b) = acc[2];
          FBA(0, a, b) = exp((AF0[k] + acc[0]) - wlog);
          FBA(1, a, b) = exp((AF1[k] + acc[1]) - wlog);
          FBA(2, a, b) = exp((AF2[k] + acc[2]) - wlog);
          c2 = acc[2];
        }
      }
#pragma unroll
      for (int k = 0; k < CB; ++k) {
        AF0[k] = NF0[k], AF1[k] = NF1[k], AF2[k] = NF2[k], AM[k] = NM[k], AX[k] = NX[k];
        Ay[k] = Ny[k];
      }
    }
  }

  // ---- MAP path over the posteriors: PairHMM::forward(fb, tr) (phmm.cpp:117-185)
  {
    double p0 = FBA(0, 0, 0), p1 = FBA(1, 0, 0), p2 = FBA(2, 0, 0);
    MRA(0, 0, 0) = p0, MRA(0, 1, 0) = p1, MRA(0, 2, 0) = p2;
    TRA(0, 0) = 0x3f;
    for (int j = 1; j <= m; ++j) {
      double bst;
      int k;
      const double fy = FBA(kIY, 0, j);
      best3(p0 + fy, p1 + fy, p2 + fy, bst, k);
      p0 = 0.0, p1 = 0.0, p2 = bst;
      MRA(0, 0, j) = p0, MRA(0, 1, j) = p1, MRA(0, 2, j) = p2;
      TRA(0, j) = (uint8_t)(3 | (3 << 2) | (k << 4));
    }
  }
  for (int i = 1; i <= n; ++i) {
    const int r = i & 1, q = r ^ 1;
    double u0 = MRA(q, 0, 0), u1 = MRA(q, 1, 0), u2 = MRA(q, 2, 0);  // (i-1, j-1)
    double bst;
    int kx;
    const double fx0 = FBA(kIX, i, 0);
    best3(u0 + fx0, u1 + fx0, u2 + fx0, bst, kx);
    double c0 = 0.0, c1 = bst, c2 = 0.0;  // (i, j-1)
    MRA(r, 0, 0) = c0, MRA(r, 1, 0) = c1, MRA(r, 2, 0) = c2;
    TRA(i, 0) = (uint8_t)(3 | (kx << 2) | (3 << 4));
    for (int j0 = 1; j0 <= m; j0 += CM) {
      double V0[CM], V1[CM], V2[CM], PM[CM], PX[CM], PY[CM];
#pragma unroll
      for (int k = 0; k < CM; ++k) {
        const int j = j0 + k;
        V0[k] = V1[k] = V2[k] = PM[k] = PX[k] = PY[k] = 0.0;
        if (j <= m) {
          V0[k] = MRA(q, 0, j), V1[k] = MRA(q, 1, j), V2[k] = MRA(q, 2, j);  // (i-1, j)
          PM[k] = FBA(kM, i, j), PX[k] = FBA(kIX, i, j), PY[k] = FBA(kIY, i, j);
        }
      }
#pragma unroll
      for (int k = 0; k < CM; ++k) {
        const int j = j0 + k;
        if (j <= m) {
          double bm, bx, by;
          int km, kx2, ky;
          best3(u0 + PM[k], u1 + PM[k], u2 + PM[k], bm, km);
          best3(V0[k] + PX[k], V1[k] + PX[k], V2[k] + PX[k], bx, kx2);
          best3(c0 + PY[k], c1 + PY[k], c2 + PY[k], by, ky);
          MRA(r, 0, j) = bm, MRA(r, 1, j) = bx, MRA(r, 2, j) = by;
          TRA(i, j) = (uint8_t)(km | (kx2 << 2) | (ky << 4));
          c0 = bm, c1 = bx, c2 = by;
          u0 = V0[k], u1 = V1[k], u2 = V2[k];
        }
      }
    }
  }

  // ---- traceback (phmm.cpp:187-216), then the anchors (stem_kernel.cpp:40-67)
  int len = 0;
  {
    int s = kM, x = n, y = m;
    PATH[(int64_t)len++ * S + t] = (s << 30) | (x << 15) | y;
    while (x != 0 && y != 0) {
      const int code = (TRA(x, y) >> (2 * s)) & 3;
      if (s == kM) --x, --y;
      else if (s == kIX) --x;
      else --y;
      if (code == 3) break;  // unreachable: every interior cell has a predecessor
      s = code;
      PATH[(int64_t)len++ * S + t] = (s << 30) | (x << 15) | y;
    }
  }
  int32_t* clo = P.band_lo + pr.band_off;
  int32_t* chi = P.band_hi + pr.band_off;
  int low_x = 0, low_y = 0;
  for (int k = len - 1; k >= 0; --k) {
    const int32_t v = PATH[(int64_t)k * S + t];
    const int s = (v >> 30) & 3, x = (v >> 15) & 0x7fff, y = v & 0x7fff;
    if (s == kM && FBA(kM, x, y) >= (double)P.ali_bound) {
      for (int i = low_x; i < x; ++i) clo[i] = low_y, chi[i] = y;
      clo[x] = y, chi[x] = y;
      low_x = x + 1, low_y = y;
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
#undef FBA
#undef BRA
#undef MRA
#undef TRA
}

}  // namespace

size_t phmm_scratch_bytes(int64_t n_pairs, int n1, int m1) {
  const int64_t c = (int64_t)n1 * m1;
  return (size_t)n_pairs * (size_t)(8 * (3 * c + 12 * (int64_t)m1) + 4 * ((int64_t)n1 + m1) + c) + 256;
}

hipError_t launch_phmm(const PhmmLaunch& P, hipStream_t st) {
  if (P.n_pairs == 0) return hipSuccess;
  const dim3 grid((unsigned)((P.n_pairs + 63) / 64)), block(64);
  hipLaunchKernelGGL(sk_phmm_kernel, grid, block, 0, st, P);
  return hipGetLastError();
}

}  // namespace sk
