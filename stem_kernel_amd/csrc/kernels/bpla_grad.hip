// BPLA gradients on CDNA4: the per-pair step of the reference's bpla_optimizer.
//
// Reference: BPLAKernel::compute_gradients  bpla_kernel/bpla_kernel.cpp:385-401
//   BPLA_Forward (:178-243), BPLA_Backward (:245-305), BPLA_ForwardBackword
//   (:325-383) with update_alpha_beta / update_beta_gap_ext (:307-323),
//   LAScore (:16-44), fill_weight (bpla_kernel/data.cpp:19-45).
//
// One thread per (x, y) pair.  The seven forward and seven backward tables of
// a pair (and exp(beta*s) per cell) live in HBM, interleaved across the pairs
// of the launch (element e of pair t at e*P + t, laid out for the launch's
// largest |x|, |y|), so the 64 lanes of a wave touch 512 contiguous bytes per
// access.  The hyperparameter
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
  double* BS = P.scratch + 2 * gN * C1 * S;  // exp(beta*s) per cell (forward -> the other passes)
#define TF(s, i, j) F[(((int64_t)(s) * C1) + (int64_t)(i) * M1 + (j)) * S + t]
#define TB(s, i, j) B[(((int64_t)(s) * C1) + (int64_t)(i) * M1 + (j)) * S + t]
#define TS(i, j) BS[((int64_t)(i) * M1 + (j)) * S + t]
  double tb[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) tb[k] = P.table[k];
  const double alpha = P.alpha, beta = P.beta, gap = P.gap, ext = P.ext;
  const double beta_gap = P.beta_gap, beta_ext = P.beta_ext;

  // Every recurrence keeps its same-row neighbour in registers and reads the
  // previous row (written a row earlier) one cell ahead, so no load waits on
  // a store of the same pass.

  // ---- BPLA_Forward (:178-243): rows 0 and column 0 are the closed forms of
  // the init loops (M = LX = LY = 1 at (0,0), LX = 1 down column 0, LY = 1
  // along row 0)
  for (int j = 0; j <= m; ++j) {
#pragma unroll
    for (int q = 0; q < gN; ++q) TF(q, 0, j) = (q == gLY || (j == 0 && (q == gM || q == gLX))) ? 1.0 : 0.0;
  }
  for (int i = 1; i <= n; ++i) {
    const float4 lx = sx.pos_lru[xpb + i - 1];  // pl, pr, pu
    const float4 px = sx.pos_prof[xpb + i - 1];
#pragma unroll
    for (int q = 0; q < gN; ++q) TF(q, i, 0) = q == gLX ? 1.0 : 0.0;
    double c[gN];  // (i, j-1)
#pragma unroll
    for (int q = 0; q < gN; ++q) c[q] = q == gLX ? 1.0 : 0.0;
    double u[gN], v[gN];  // (i-1, j-1), (i-1, j)
#pragma unroll
    for (int q = 0; q < gN; ++q) u[q] = TF(q, i - 1, 0), v[q] = TF(q, i - 1, 1);
    const double lx0 = u[gLX];  // LX(i-1, 0)
    float4 ly = sy.pos_lru[ypb], py = sy.pos_prof[ypb];
    for (int j = 1; j <= m; ++j) {
      // next cell's operands
      double vn[gN];
      float4 lyn = ly, pyn = py;
      if (j < m) {
#pragma unroll
        for (int q = 0; q < gN; ++q) vn[q] = TF(q, i - 1, j + 1);
        lyn = sy.pos_lru[ypb + j];
        pyn = sy.pos_prof[ypb + j];
      }
      const double wp = (double)(lx.y * ly.y + lx.x * ly.x);
      const double wu = (double)(lx.z * ly.z) * la_score(tb, px, py);
      const double bs = exp(beta * (alpha * wp + wu));
      TS(i, j) = bs;
      double M = 0.0;
      M += bs * u[gM];
      M += bs * u[gIX];
      M += bs * u[gIY];
      M += bs * u[gLX];
      M += bs * u[gLY];
      double X = 0.0;
      X += beta_gap * v[gM];
      X += beta_ext * v[gIX];
      double Y = 0.0;
      Y += beta_gap * c[gM];
      Y += beta_gap * c[gIX];
      Y += beta_ext * c[gIY];
      const double LX = 0.0 + lx0;
      double LY = 0.0;
      LY += c[gLX];
      LY += c[gLY];
      double RX = 0.0;
      RX += v[gM];
      RX += v[gRX];
      double RY = 0.0;
      RY += c[gM];
      RY += c[gRX];
      RY += c[gRY];
      c[gM] = M, c[gIX] = X, c[gIY] = Y, c[gLX] = LX, c[gLY] = LY, c[gRX] = RX, c[gRY] = RY;
#pragma unroll
      for (int q = 0; q < gN; ++q) TF(q, i, j) = c[q];
#pragma unroll
      for (int q = 0; q < gN; ++q) u[q] = v[q], v[q] = vn[q];
      ly = lyn, py = pyn;
    }
  }
  const double value = 1 + TF(gM, n, m) + TF(gRX, n, m) + TF(gRY, n, m);

  // ---- BPLA_Backward (:245-305) in the reference's scatter order, with the
  // contributions a source (i,j) makes to (i, j-1) carried in registers and
  // those to row i-1 completed in registers and stored once: the row-below
  // cell (i-1, c) receives only from the sources (i, c+1) (diagonal) and
  // (i, c) (vertical), plus the row's LX sum into (i-1, 0).
  for (int j = 0; j <= m; ++j) {  // row n: the init (M = RX = RY = 1 at (n, m))
#pragma unroll
    for (int q = 0; q < gN; ++q) TB(q, n, j) = (j == m && (q == gM || q == gRX || q == gRY)) ? 1.0 : 0.0;
  }
  for (int i = n; i >= 1; --i) {
    double cc[gN];    // to (i, j-1) from (i, j)
    double pend[gN];  // to (i-1, j) from (i, j+1) (diagonal)
#pragma unroll
    for (int q = 0; q < gN; ++q) cc[q] = 0.0, pend[q] = 0.0;
    double lxsum = 0.0;  // LX(i-1, 0) += LX(i, j), j = m..1
    double mb[gN];
#pragma unroll
    for (int q = 0; q < gN; ++q) mb[q] = TB(q, i, m);
    double bsj = TS(i, m);
    for (int j = m; j >= 1; --j) {
      double mbn[gN];
      double bsn = 0.0;
      if (j > 1) {
#pragma unroll
        for (int q = 0; q < gN; ++q) mbn[q] = TB(q, i, j - 1);
        bsn = TS(i, j - 1);
      }
      double b[gN];  // B(i, j): row i+1's contributions + (i, j+1)'s
#pragma unroll
      for (int q = 0; q < gN; ++q) b[q] = mb[q] + cc[q];
      // vertical contributions to (i-1, j) complete it
      double dn[gN];
#pragma unroll
      for (int q = 0; q < gN; ++q) dn[q] = pend[q];
      dn[gM] += beta_gap * b[gIX];
      dn[gIX] += beta_ext * b[gIX];
      dn[gM] += b[gRX];
      dn[gRX] += b[gRX];
#pragma unroll
      for (int q = 0; q < gN; ++q) TB(q, i - 1, j) = dn[q];
      // diagonal contributions to (i-1, j-1)
      const double d = bsj * b[gM];
#pragma unroll
      for (int q = 0; q < gN; ++q) pend[q] = 0.0;
      pend[gM] += d;
      pend[gIX] += d;
      pend[gIY] += d;
      pend[gLX] += d;
      pend[gLY] += d;
      lxsum += b[gLX];
      // same-row contributions to (i, j-1)
#pragma unroll
      for (int q = 0; q < gN; ++q) cc[q] = 0.0;
      cc[gM] += beta_gap * b[gIY];
      cc[gIX] += beta_gap * b[gIY];
      cc[gIY] += beta_ext * b[gIY];
      cc[gLX] += b[gLY];
      cc[gLY] += b[gLY];
      cc[gM] += b[gRY];
      cc[gRX] += b[gRY];
      cc[gRY] += b[gRY];
      // B(i, j) is final: the gradient pass reads M, IX, IY
      TB(gM, i, j) = b[gM];
      TB(gIX, i, j) = b[gIX];
      TB(gIY, i, j) = b[gIY];
#pragma unroll
      for (int q = 0; q < gN; ++q) mb[q] = mbn[q];
      bsj = bsn;
    }
    // (i-1, 0): the diagonal from (i, 1) and the row's LX sum
    pend[gLX] += lxsum;
#pragma unroll
    for (int q = 0; q < gN; ++q) TB(q, i - 1, 0) = pend[q];
  }
  // column 0 and row 0 only feed the backward total (and the column/row
  // loops after the main loop), which the gradients do not read

  // ---- BPLA_ForwardBackword (:325-383)
  double da = 0.0, db = 0.0, dg = 0.0, de = 0.0;
  for (int i = 1; i <= n; ++i) {
    const float4 lx = sx.pos_lru[xpb + i - 1];
    const float4 px = sx.pos_prof[xpb + i - 1];
#pragma unroll 2
    for (int j = 1; j <= m; ++j) {
      const float4 ly = sy.pos_lru[ypb + j - 1], py = sy.pos_prof[ypb + j - 1];
      const double wp = (double)(lx.y * ly.y + lx.x * ly.x);
      const double wu = (double)(lx.z * ly.z) * la_score(tb, px, py);
      const double bs = TS(i, j);
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
  }
  P.value[t] = value;
  P.grad[4 * t + 0] = da;
  P.grad[4 * t + 1] = db;
  P.grad[4 * t + 2] = dg;
  P.grad[4 * t + 3] = de;
#undef TF
#undef TB
#undef TS
}

}  // namespace

size_t bpla_grad_pair_bytes(int n1, int m1) { return (size_t)(2 * 7 + 1) * n1 * m1 * sizeof(double); }

hipError_t launch_bpla_grad(const BplaGradLaunch& P, hipStream_t st) {
  if (P.n_pairs == 0) return hipSuccess;
  hipLaunchKernelGGL(sk_bpla_grad_kernel, dim3((unsigned)((P.n_pairs + 63) / 64)), dim3(64), 0, st, P);
  return hipGetLastError();
}

}  // namespace sk
