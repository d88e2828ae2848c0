// BPLA gradients on CDNA4: the per-pair step of the reference's bpla_optimizer.
//
// Reference: BPLAKernel::compute_gradients  bpla_kernel/bpla_kernel.cpp:385-401
//   BPLA_Forward (:178-243), BPLA_Backward (:245-305), BPLA_ForwardBackword
//   (:325-383) with update_alpha_beta / update_beta_gap_ext (:307-323),
//   LAScore (:16-44), fill_weight (bpla_kernel/data.cpp:19-45).
//
// One thread per (x, y) pair.  The seven forward and seven backward tables of
// a pair live in HBM, interleaved across the pairs of the launch (element e
// of pair t at e*P + t, laid out for the launch's largest |x|, |y|), so the
// 64 lanes of a wave touch 512 contiguous bytes per access; the loops are the
// reference's, in its order (scatter form included).  The hyperparameter
// search calls this once per pair and optimizer step, so it is a throughput
// kernel over many pairs, not a latency one.  Built with -ffp-contract=off
// (float products of the scores as the reference rounds them).
#include <hip/hip_runtime.h>

#include "device_set.h"
#include "launch.h"

namespace sk {
namespace {

enum { gM = 0, gIX, gIY, gLX, gLY, gRX, gRY, gN };

// LAScore::operator() (bpla_kernel.cpp:24-43)
__device__ __forceinline__ double la_score(const double* tb, float4 xc, float4 yc) {
  const float xa[4] = {xc.x, xc.y, xc.z, xc.w}, yb[4] = {yc.x, yc.y, yc.z, yc.w};
  double v = 0.0;
  float n = 0.0f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (xa[k] == 0.0f) continue;
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      if (yb[l] == 0.0f) continue;
      n += xa[k] * yb[l];
      v += tb[k * 4 + l] * (double)xa[k] * (double)yb[l];
    }
  }
  return n == 0.0f ? 0.0 : v / (double)n;
}

__global__ void __launch_bounds__(64) sk_bpla_grad_kernel(BplaGradLaunch P) {
  const int64_t t = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (t >= P.n_pairs) return;
  const DevSet& sx = P.xset;
  const DevSet& sy = P.yset;
  const int x = P.xs[t], y = P.ys[t];
  const int n = sx.ex_len[x], m = sy.ex_len[y];
  const int xpb = sx.ex_pos_base[x], ypb = sy.ex_pos_base[y];
  const int64_t S = P.n_pairs, M1 = P.m1, C1 = (int64_t)P.n1 * P.m1;
  double* F = P.scratch;
  double* B = P.scratch + gN * C1 * S;
#define TF(s, i, j) F[(((int64_t)(s) * C1) + (int64_t)(i) * M1 + (j)) * S + t]
#define TB(s, i, j) B[(((int64_t)(s) * C1) + (int64_t)(i) * M1 + (j)) * S + t]
  double tb[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) tb[k] = P.table[k];
  const double alpha = P.alpha, beta = P.beta, gap = P.gap, ext = P.ext;
  const double beta_gap = P.beta_gap, beta_ext = P.beta_ext;
  // score operands of cell (i, j) (positions i-1, j-1): w_pair (float sum of
  // float products), pu*pu' (float) and LAScore
  auto score = [&](int i, int j, double& wp, double& wu) {
    const float4 lx = sx.pos_lru[xpb + i - 1], ly = sy.pos_lru[ypb + j - 1];  // pl, pr, pu
    wp = (double)(lx.y * ly.y + lx.x * ly.x);
    wu = (double)(lx.z * ly.z) * la_score(tb, sx.pos_prof[xpb + i - 1], sy.pos_prof[ypb + j - 1]);
  };

  for (int s = 0; s < gN; ++s)
    for (int i = 0; i <= n; ++i)
      for (int j = 0; j <= m; ++j) TF(s, i, j) = 0.0, TB(s, i, j) = 0.0;

  // ---- BPLA_Forward
  TF(gM, 0, 0) = 1;
  TF(gLX, 0, 0) = 1;
  TF(gLY, 0, 0) = 1;
  for (int i = 1; i <= n; ++i) TF(gLX, i, 0) += TF(gLX, i - 1, 0);
  for (int j = 1; j <= m; ++j) TF(gLY, 0, j) += TF(gLY, 0, j - 1);
  for (int i = 1; i <= n; ++i) {
    const double lx0 = TF(gLX, i - 1, 0);
    for (int j = 1; j <= m; ++j) {
      double wp, wu;
      score(i, j, wp, wu);
      const double bs = exp(beta * (alpha * wp + wu));
      double M = TF(gM, i, j);
      M += bs * TF(gM, i - 1, j - 1);
      M += bs * TF(gIX, i - 1, j - 1);
      M += bs * TF(gIY, i - 1, j - 1);
      M += bs * TF(gLX, i - 1, j - 1);
      M += bs * TF(gLY, i - 1, j - 1);
      TF(gM, i, j) = M;
      const double Mu = TF(gM, i - 1, j), Ml = TF(gM, i, j - 1);
      double X = TF(gIX, i, j);
      X += beta_gap * Mu;
      X += beta_ext * TF(gIX, i - 1, j);
      TF(gIX, i, j) = X;
      double Y = TF(gIY, i, j);
      Y += beta_gap * Ml;
      Y += beta_gap * TF(gIX, i, j - 1);
      Y += beta_ext * TF(gIY, i, j - 1);
      TF(gIY, i, j) = Y;
      TF(gLX, i, j) += lx0;
      double LY = TF(gLY, i, j);
      LY += TF(gLX, i, j - 1);
      LY += TF(gLY, i, j - 1);
      TF(gLY, i, j) = LY;
      double RX = TF(gRX, i, j);
      RX += Mu;
      RX += TF(gRX, i - 1, j);
      TF(gRX, i, j) = RX;
      double RY = TF(gRY, i, j);
      RY += Ml;
      RY += TF(gRX, i, j - 1);
      RY += TF(gRY, i, j - 1);
      TF(gRY, i, j) = RY;
    }
  }

  // ---- BPLA_Backward (scatter form, as written)
  TB(gM, n, m) = 1;
  TB(gRX, n, m) = 1;
  TB(gRY, n, m) = 1;
  for (int i = n; i != 0; --i)
    for (int j = m; j != 0; --j) {
      double wp, wu;
      score(i, j, wp, wu);
      const double bs = exp(beta * (alpha * wp + wu));
      const double bm = TB(gM, i, j), bx = TB(gIX, i, j), by = TB(gIY, i, j);
      const double blx = TB(gLX, i, j), bly = TB(gLY, i, j);
      const double brx = TB(gRX, i, j), bry = TB(gRY, i, j);
      TB(gM, i - 1, j - 1) += bs * bm;
      TB(gIX, i - 1, j - 1) += bs * bm;
      TB(gIY, i - 1, j - 1) += bs * bm;
      TB(gLX, i - 1, j - 1) += bs * bm;
      TB(gLY, i - 1, j - 1) += bs * bm;
      TB(gM, i - 1, j) += beta_gap * bx;
      TB(gIX, i - 1, j) += beta_ext * bx;
      TB(gM, i, j - 1) += beta_gap * by;
      TB(gIX, i, j - 1) += beta_gap * by;
      TB(gIY, i, j - 1) += beta_ext * by;
      TB(gLX, i - 1, 0) += blx;
      TB(gLX, i, j - 1) += bly;
      TB(gLY, i, j - 1) += bly;
      TB(gM, i - 1, j) += brx;
      TB(gRX, i - 1, j) += brx;
      TB(gM, i, j - 1) += bry;
      TB(gRX, i, j - 1) += bry;
      TB(gRY, i, j - 1) += bry;
    }
  for (int i = n; i != 0; --i) TB(gLX, i - 1, 0) += TB(gLX, i, 0);
  for (int j = m; j != 0; --j) TB(gLY, 0, j - 1) += TB(gLY, 0, j);

  // ---- BPLA_ForwardBackword
  double da = 0.0, db = 0.0, dg = 0.0, de = 0.0;
  for (int i = 1; i <= n; ++i)
    for (int j = 1; j <= m; ++j) {
      double wp, wu;
      score(i, j, wp, wu);
      const double bs = exp(beta * (alpha * wp + wu));
      const double bm = TB(gM, i, j);
#pragma unroll
      for (int q = 0; q < 5; ++q) {  // M, IX, IY, LX, LY at (i-1, j-1)
        const double v = TF(q, i - 1, j - 1) * bs * bm;
        da += beta * wp * v;
        db += (alpha * wp + wu) * v;
      }
      const double bx = TB(gIX, i, j), by = TB(gIY, i, j);
      double v = TF(gM, i - 1, j) * beta_gap * bx;
      db += gap * v, dg += beta * v;
      v = TF(gIX, i - 1, j) * beta_ext * bx;
      db += ext * v, de += beta * v;
      v = TF(gM, i, j - 1) * beta_gap * by;
      db += gap * v, dg += beta * v;
      v = TF(gIX, i, j - 1) * beta_gap * by;
      db += gap * v, dg += beta * v;
      v = TF(gIY, i, j - 1) * beta_ext * by;
      db += ext * v, de += beta * v;
    }
  P.value[t] = 1 + TF(gM, n, m) + TF(gRX, n, m) + TF(gRY, n, m);
  P.grad[4 * t + 0] = da;
  P.grad[4 * t + 1] = db;
  P.grad[4 * t + 2] = dg;
  P.grad[4 * t + 3] = de;
#undef TF
#undef TB
}

}  // namespace

size_t bpla_grad_pair_bytes(int n1, int m1) { return (size_t)2 * 7 * n1 * m1 * sizeof(double); }

hipError_t launch_bpla_grad(const BplaGradLaunch& P, hipStream_t st) {
  if (P.n_pairs == 0) return hipSuccess;
  hipLaunchKernelGGL(sk_bpla_grad_kernel, dim3((unsigned)((P.n_pairs + 63) / 64)), dim3(64), 0, st, P);
  return hipGetLastError();
}

}  // namespace sk
