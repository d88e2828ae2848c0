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

#include "bpla_fast.h"
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

// ===========================================================================
// Wave-per-pair gradients for dyadic profiles (the operand tables and exp of
// bpla.hip's fast path; every profile entry a multiple of 1/256).
//
// The gradient sums (BPLA_ForwardBackword, :325-383) read the forward states
// around a cell and the backward states M, IX, IY at the cell, so:
//   1. the BACKWARD pass runs first, on the forward kernel's streamed-strip
//      systolic schedule played in reverse time (lane l owns rows 64s+l+1;
//      row a+1 lives one lane up: wave_shl; the strip boundary row goes
//      through LDS, written by lane 0, read by lane 63), and stores B_M, B_IX,
//      B_IY in a per-wave HBM table laid out by (state, step, lane) -- 512
//      contiguous bytes per state per step;
//   2. the FORWARD pass recomputes F step by step and adds the gradient terms
//      with the stored B of the same (step, lane).
// The reference's scatter backward (:245-305) is gathered:
//   B_M(a,b)  = [a<n,b<m] bs(a+1,b+1) B_M(a+1,b+1) + [a<n] (e^{bg} B_IX(a+1,b) + B_RX(a+1,b))
//             + [b<m] (e^{bg} B_IY(a,b+1) + B_RY(a,b+1))
//   B_IX(a,b) = [a<n,b<m] bs B_M(a+1,b+1) + [a<n] e^{be} B_IX(a+1,b) + [b<m] e^{bg} B_IY(a,b+1)
//   B_IY(a,b) = [a<n,b<m] bs B_M(a+1,b+1) + [b<m] e^{be} B_IY(a,b+1)
// with B_RX(a,b) = [b >= 1 or a = n] and B_RY(a,b) = [a = n] in closed form
// (they only ever add 1s), and B_LX, B_LY never feeding M, IX, IY.  Forward,
// F_LX = 1 and F_LY = j on rows i >= 1 (row 0: F_M = F_LX = 1 at (0,0),
// F_LY = 1), and 1 + F_M + F_RX + F_RY at (n,m) = 1 + sum of F_M over cells
// i, j >= 1.  Per pair: two exps per cell, 24 B per cell written and read
// back.  Sums run in another order than the reference's (~1e-15 relative).
__device__ void bpla_grad_wave_pair(const BplaGradLaunch& P, int x, int y, const BplaPos* ycol,
                                    double* bnd, const double* etab, double* __restrict__ Bt,
                                    int lane, double& value, double (&g)[4]) {
  const double alpha = P.alpha, beta = P.beta, gap = P.gap, ext = P.ext;
  const double bg = P.beta_gap, be = P.beta_ext;
  const int Lx = __builtin_amdgcn_readfirstlane(P.xset.ex_len[x]);
  const int Ly = __builtin_amdgcn_readfirstlane(P.yset.ex_len[y]);
  const int xpb = __builtin_amdgcn_readfirstlane(P.xset.ex_pos_base[x]);
  const int Lys = max(Ly, 64);
  const int T = bpla_steps(Lx, Ly);
  const int64_t TS = (int64_t)T * 64;
  double* __restrict__ BM = Bt;
  double* __restrict__ BX = Bt + TS;
  double* __restrict__ BY = Bt + 2 * TS;
  auto wave_sync = []() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  // BPLAScore (bpla_kernel.cpp:45-62): the pair weight in float as written,
  // the LAScore from the tabulated factors
  auto score = [&](const BplaPos& xr, const BplaPos& yc, double& wp) {
    double la = xr.v[0] * yc.v[0];
    la = __builtin_fma(xr.v[1], yc.v[1], la);
    la = __builtin_fma(xr.v[2], yc.v[2], la);
    la = __builtin_fma(xr.v[3], yc.v[3], la);
    const float pp = f32_dot2(xr.pr, yc.pr, xr.pl, yc.pl);
    const float uu = xr.pu * yc.pu;
    wp = (double)pp;
    return alpha * (double)pp + (double)uu * la;
  };

  // ---------------------------------------------------------------- backward
  double* bndX = bnd;              // B_IX of row 64s+1 (lane 0), column b
  double* bndP = bnd + (Lys + 2);  // bs * B_M of the same cells
  for (int j = lane; j < 2 * (Lys + 2); j += 64) bnd[j] = 0.0;
  wave_sync();
  {
    double oX = 0.0, oP = 0.0, oY = 0.0;  // my outputs of the previous (reverse) step
    double dP = 0.0;                      // P(a+1, b+1): received a step earlier
    int xs_cur = -1;
    BplaPos xr;
    for (int t = T - 1; t >= 0; --t) {
      const int u = t - lane;
      const int s = u >= 0 ? u / Lys : -1;
      const int b = u - s * Lys + 1;
      const int a = 64 * s + lane + 1;
      // lane 63's row a+1 is lane 0 of the next strip (boundary row)
      const int b63 = __builtin_amdgcn_readlane(b, 63);
      const int bi = (b63 >= 1 && b63 <= Ly) ? b63 : 0;
      const double rX = wave_shl1_to(oX, bndX[bi]);
      const double rP = wave_shl1_to(oP, bndP[bi]);
      double M = 0.0, X = 0.0, Y = 0.0, Pn = 0.0;
      if (u >= 0 && b <= Ly && a <= Lx) {
        if (s != xs_cur) {
          xr = P.xtab[xpb + a - 1];
          xs_cur = s;
        }
        const bool an = a < Lx, bm = b < Ly;
        const double diag = (an && bm) ? dP : 0.0;
        const double iyr = bm ? oY : 0.0;
        const double ixd = an ? rX : 0.0;
        M = diag + (an ? __builtin_fma(bg, ixd, 1.0) : 0.0) +
            (bm ? __builtin_fma(bg, iyr, a == Lx ? 1.0 : 0.0) : 0.0);
        X = diag + (an ? be * ixd : 0.0) + (bm ? bg * iyr : 0.0);
        Y = diag + (bm ? be * iyr : 0.0);
        if (!an && !bm) {  // (n, m): B_M = B_RX = B_RY = 1
          M = 1.0;
          X = Y = 0.0;
        }
        const BplaPos yc = ycol[b - 1];
        double wp;
        const double sc = score(xr, yc, wp);
        Pn = fast_exp(beta * sc, etab) * M;
        BM[(int64_t)t * 64 + lane] = M;
        BX[(int64_t)t * 64 + lane] = X;
        BY[(int64_t)t * 64 + lane] = Y;
        if (lane == 0) {
          bndX[b] = X;
          bndP[b] = Pn;
        }
      }
      oX = X;
      oP = Pn;
      oY = Y;
      dP = rP;
    }
  }
  wave_sync();

  // ---------------------------------------------------------------- forward + gradients
  for (int j = lane; j < 3 * (Lys + 1); j += 64) bnd[j] = 0.0;  // row 0 (M, IX, IY)
  wave_sync();
  int j = 1 - lane, i = lane + 1;
  bool row_ok = i <= Lx;
  BplaPos xr = P.xtab[xpb + (row_ok ? i - 1 : 0)];
  BplaPos xnext = P.xtab[xpb + (i + 64 <= Lx ? i + 63 : 0)];
  double lM = 0.0, lX = 0.0, lY = 0.0;  // (i, j-1)
  double dM = 0.0, dX = 0.0, dY = 0.0;  // (i-1, j-1): received a step earlier
  double acc = 0.0, ga = 0.0, gb = 0.0, gg = 0.0, ge = 0.0;
  // B at (step t, lane), prefetched a step ahead
  double nbm = T > 0 ? BM[lane] : 0.0, nbx = T > 0 ? BX[lane] : 0.0, nby = T > 0 ? BY[lane] : 0.0;
  for (int t = 0; t < T; ++t) {
    const double bm = nbm, bx = nbx, by = nby;
    if (t + 1 < T) {
      nbm = BM[(int64_t)(t + 1) * 64 + lane];
      nbx = BX[(int64_t)(t + 1) * 64 + lane];
      nby = BY[(int64_t)(t + 1) * 64 + lane];
    }
    const int jb = __builtin_amdgcn_readfirstlane(j);
    const double* bj = bnd + 3 * (jb >= 1 && jb <= Ly ? jb : 0);
    const double uM = wave_shr1(lM, bj[0]);
    const double uX = wave_shr1(lX, bj[1]);
    const double uY = wave_shr1(lY, bj[2]);
    if (j >= 1 && j <= Ly) {
      const BplaPos yc = ycol[j - 1];
      double wp;
      const double sc = score(xr, yc, wp);
      const double bs = fast_exp(beta * sc, etab);
      const bool c1 = j == 1;
      // diagonal F_M + F_IX + F_IY + F_LX + F_LY at (i-1, j-1)
      const double extra = i == 1 ? (c1 ? 3.0 : 1.0) : (double)j;
      const double nM = bs * (dM + dX + dY + extra);
      const double nX = bg * uM + be * uX;
      const double lMX = c1 ? 0.0 : lM + lX, lYc = c1 ? 0.0 : lY;
      const double nY = bg * lMX + be * lYc;
      if (row_ok) {
        acc += nM;
        const double vd = nM * bm;
        const double vgx = uM * bg * bx, vex = uX * be * bx;
        const double vgy = lMX * bg * by, vey = lYc * be * by;
        ga += beta * wp * vd;
        gb += sc * vd + gap * (vgx + vgy) + ext * (vex + vey);
        gg += beta * (vgx + vgy);
        ge += beta * (vex + vey);
      }
      lM = nM;
      lX = nX;
      lY = nY;
      if (lane == 63) {
        double* bw = bnd + 3 * j;
        bw[0] = nM;
        bw[1] = nX;
        bw[2] = nY;
      }
    }
    dM = uM;
    dX = uX;
    dY = uY;
    if (++j > Lys) {  // next strip: row i + 64, column 1
      j = 1;
      i += 64;
      row_ok = i <= Lx;
      xr = xnext;
      if (i + 64 <= Lx) xnext = P.xtab[xpb + i + 63];
      dM = dX = dY = 0.0;
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    acc += __shfl_xor(acc, off, 64);
    ga += __shfl_xor(ga, off, 64);
    gb += __shfl_xor(gb, off, 64);
    gg += __shfl_xor(gg, off, 64);
    ge += __shfl_xor(ge, off, 64);
  }
  value = 1.0 + acc;
  g[0] = ga;
  g[1] = gb;
  g[2] = gg;
  g[3] = ge;
  wave_sync();
}

__global__ void __launch_bounds__(256) sk_bpla_grad_wave_kernel(BplaGradLaunch P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int maxlen = P.lds_max_len;
  double* etab = reinterpret_cast<double*>(smem);
  unsigned char* wbase = smem + kBplaExpLds + (size_t)wave * bpla_grad_wave_lds_bytes(maxlen);
  BplaPos* ycol = reinterpret_cast<BplaPos*>(wbase);
  double* bnd = reinterpret_cast<double*>(ycol + maxlen);
  double* Bt = P.scratch + (int64_t)(blockIdx.x * (blockDim.x >> 6) + wave) * P.bt_doubles;
  fill_exp_table(etab);
  auto next_pair = [&]() {
    unsigned long long v = 0;
    if (lane == 0) v = atomicAdd(P.pair_counter, 1ull);
    return (int64_t)(((unsigned long long)__builtin_amdgcn_readlane((unsigned)(v >> 32), 0) << 32) |
                     (unsigned)__builtin_amdgcn_readlane((unsigned)v, 0));
  };
  for (int64_t pr = next_pair(); pr < P.n_pairs; pr = next_pair()) {
    const int x = __builtin_amdgcn_readfirstlane(P.xs[pr]);
    const int y = __builtin_amdgcn_readfirstlane(P.ys[pr]);
    const int Ly = P.yset.ex_len[y], ypb = P.yset.ex_pos_base[y];
    for (int j = lane; j < Ly; j += 64) ycol[j] = P.ytab[ypb + j];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    double v, g[4];
    bpla_grad_wave_pair(P, x, y, ycol, bnd, etab, Bt, lane, v, g);
    if (lane == 0) {
      const int64_t o = P.oidx ? P.oidx[pr] : pr;
      P.value[o] = v;
      P.grad[4 * o + 0] = g[0];
      P.grad[4 * o + 1] = g[1];
      P.grad[4 * o + 2] = g[2];
      P.grad[4 * o + 3] = g[3];
    }
  }
}

hipError_t launch_bpla_grad_wave(const BplaGradLaunch& P, int grid, int nwaves, hipStream_t st) {
  if (P.n_pairs == 0 || grid <= 0) return hipSuccess;
  const size_t lds = kBplaExpLds + (size_t)nwaves * bpla_grad_wave_lds_bytes(P.lds_max_len);
  hipError_t e = hipFuncSetAttribute((const void*)sk_bpla_grad_wave_kernel,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(sk_bpla_grad_wave_kernel, dim3(grid), dim3(64 * nwaves), lds, st, P);
  return hipGetLastError();
}

size_t bpla_grad_pair_bytes(int n1, int m1) { return (size_t)(2 * 7 + 1) * n1 * m1 * sizeof(double); }

hipError_t launch_bpla_grad(const BplaGradLaunch& P, hipStream_t st) {
  if (P.n_pairs == 0) return hipSuccess;
  hipLaunchKernelGGL(sk_bpla_grad_kernel, dim3((unsigned)((P.n_pairs + 63) / 64)), dim3(64), 0, st, P);
  return hipGetLastError();
}

}  // namespace sk
