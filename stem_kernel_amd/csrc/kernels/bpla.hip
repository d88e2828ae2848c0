// BPLA kernel on CDNA4 (gfx950): local-alignment partition function (or
// Smith-Waterman score) over profile columns with base-pairing scores.
//
// Reference: BPLAKernel<double,MData>::operator()  bpla_kernel/bpla_kernel.cpp:159-174
//   local_alignment_exp :64-115 (M, X, Y, X2, Y2; result 1 + X2 + Y2 + M)
//   local_alignment_max :117-157 (M, X, Y; result max M)
//   LAScore :16-43, BPLAScore :45-62, fill_weight bpla_kernel/data.cpp:19-45.
//
// Systolic schedule: one wavefront per pair, lane l owns DP rows
// i = 64*strip + l + 1 and computes column j of its current row at step t.
// Row i-1 lives one lane down and one step ahead, so the "up" cell (i-1, j)
// is lane l-1's previous output (one DPP wave_shr), and the diagonal
// (i-1, j-1) is what lane l received one step earlier.  Strips are streamed:
// a lane starts its next row as soon as it finishes one, so the 64-step fill
// and drain is paid once per pair, not per strip; the strip boundary row goes
// through a per-wave LDS row of the four states lane 0 reads.
// FP64 throughout; one exp per cell is the bound.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "bpla_fast.h"
#include "device_set.h"
#include "launch.h"

namespace sk {

// Column sum of a profile column if every entry is a multiple of 1/256
// (then every product, partial sum and the total weight of LAScore are exact
// in float, whatever the order), else -1.
__device__ __forceinline__ float dyadic_sum(float4 c) {
  const bool ex = c.x * 256.0f == rintf(c.x * 256.0f) && c.y * 256.0f == rintf(c.y * 256.0f) &&
                  c.z * 256.0f == rintf(c.z * 256.0f) && c.w * 256.0f == rintf(c.w * 256.0f);
  return ex ? c.x + c.y + c.z + c.w : -1.0f;
}

// LAScore::operator() (bpla_kernel.cpp:24-43), 0 when either column is empty.
// Branch-free numerator from the row's factored u; the float weight n is
// xs*ys when both columns are dyadic (exact, see dyadic_sum), else every
// product added in the reference's (k, l) order (the skipped ones are exact
// zeros).
__device__ __forceinline__ double la_score_f(const double (&u)[4], float4 xc, float4 yc, float xs,
                                             float ys) {
  const float yb[4] = {yc.x, yc.y, yc.z, yc.w};
  float n;
  if (xs >= 0.0f && ys >= 0.0f) {
    n = xs * ys;
  } else {
    const float xa[4] = {xc.x, xc.y, xc.z, xc.w};
    n = 0.0f;
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int l = 0; l < 4; ++l) n = f32_madd(n, xa[k], yb[l]);
  }
  const double v = u[0] * (double)yb[0] + u[1] * (double)yb[1] + u[2] * (double)yb[2] +
                   u[3] * (double)yb[3];
  return n == 0.0f ? 0.0 : v / (double)n;
}

__global__ void __launch_bounds__(256) sk_bpla_kernel(BplaLaunch P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const DevSet& sx = P.xset;
  const DevSet& sy = P.yset;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nwaves = blockDim.x >> 6;
  const int maxlen = P.lds_max_len;  // even
  // LDS: table[16] | per wave: bM,bX,bY,bX2 [maxlen+2] | yprof, ylru float4 [maxlen]
  double* tb = reinterpret_cast<double*>(smem);
  const size_t wbytes = bpla_wave_lds_bytes(maxlen);
  unsigned char* wbase = smem + 16 * 8 + (size_t)wave * wbytes;
  double* bM = reinterpret_cast<double*>(wbase);
  double* bX = bM + (maxlen + 2);
  double* bY = bX + (maxlen + 2);
  double* bX2 = bY + (maxlen + 2);
  float4* yprof = reinterpret_cast<float4*>(bX2 + (maxlen + 2));
  float4* ylru = yprof + maxlen;
  (void)nwaves;

  if (threadIdx.x < 16) tb[threadIdx.x] = P.table[threadIdx.x];
  __syncthreads();
  const bool sw = P.sw != 0, bp = P.bp != 0;
  const double beta = P.beta, alpha = P.alpha, gap = P.gap, ext = P.ext;
  const double bg = P.beta_gap, be = P.beta_ext;

  for (;;) {
    unsigned long long pr = 0;
    if (lane == 0) pr = atomicAdd(P.pair_counter, 1ull);
    pr = ((unsigned long long)__builtin_amdgcn_readlane((unsigned)(pr >> 32), 0) << 32) |
         (unsigned)__builtin_amdgcn_readlane((unsigned)pr, 0);
    if ((int64_t)pr >= P.n_pairs) break;
    const int x = P.xs[pr], y = P.ys[pr];
    const int Lx = sx.ex_len[x], Ly = sy.ex_len[y];
    const int xpb = sx.ex_pos_base[x], ypb = sy.ex_pos_base[y];
    for (int j = lane; j < Ly; j += 64) {
      const float4 c = sy.pos_prof[ypb + j];
      yprof[j] = c;
      float4 w = sy.pos_lru[ypb + j];
      w.w = dyadic_sum(c);  // (the 4th weight slot is unused)
      ylru[j] = w;
    }
    // streamed strips: a strip takes Lys = max(Ly, 64) steps, so lane 0
    // reads boundary column j of strip s (row 64s, written by lane 63 one
    // strip earlier) at least one step after it was written, and before
    // lane 63 overwrites it with strip s's own row
    const int Lys = max(Ly, 64);
    for (int j = lane; j <= Lys; j += 64) {  // row 0 (bpla_kernel.cpp:90-96)
      bM[j] = 0.0;
      bX[j] = 0.0;
      bY[j] = 0.0;
      bX2[j] = 0.0;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    double result = 0.0, mmax = 0.0;
    const int nstrips = (Lx + 63) / 64;
    // lane l owns rows l+1, l+65, ...: at step t it is at strip
    // s = (t-l) / Lys, column j = (t-l) % Lys + 1 (nothing before t = l)
    int strip = 0, j = 1 - lane;
    int i = lane + 1;
    bool row_ok = i <= Lx;
    // x column of the current row, the next row's prefetched
    float4 xc = make_float4(0.f, 0.f, 0.f, 0.f), xw = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row_ok) {
      xc = sx.pos_prof[xpb + i - 1];
      xw = sx.pos_lru[xpb + i - 1];
    }
    float4 nxc = make_float4(0.f, 0.f, 0.f, 0.f), nxw = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i + 64 <= Lx) {
      nxc = sx.pos_prof[xpb + i + 63];
      nxw = sx.pos_lru[xpb + i + 63];
    }
    // LAScore numerator factored per row: v = sum_l u_l y_l with
    // u_l = sum_k table[k][l] x_k (one-hot columns give table[k][l] exactly)
    double u[4];
#pragma unroll
    for (int l = 0; l < 4; ++l)
      u[l] = tb[l] * (double)xc.x + tb[4 + l] * (double)xc.y + tb[8 + l] * (double)xc.z +
             tb[12 + l] * (double)xc.w;
    float xsum = dyadic_sum(xc);
    // my outputs of the previous step (row i, column j-1)
    double lM = 0.0, lX = 0.0, lY = 0.0, lX2 = 0.0, lY2 = 0.0;
    // what I received last step: (i-1, j-1)
    double dM = 0.0, dX = 0.0, dY = 0.0;
    const int T = (nstrips - 1) * Lys + ((Lx - 1) & 63) + Ly;
    for (int t = 0; t < T; ++t) {
      // lane 0 takes row i-1 from the boundary row (a wave-uniform column)
      const int jb = __builtin_amdgcn_readfirstlane(j);
      const int jr = jb >= 1 && jb <= Ly ? jb : 0;
      const double b0M = bM[jr], b0X = bX[jr], b0Y = bY[jr], b0X2 = bX2[jr];
      const double upM = wave_shr1(lM, strip == 0 ? 0.0 : b0M);
      const double upX = wave_shr1(lX, strip == 0 ? 0.0 : b0X);
      const double upY = wave_shr1(lY, strip == 0 ? 0.0 : b0Y);
      const double upX2 = wave_shr1(lX2, strip == 0 ? 0.0 : b0X2);
      if (j >= 1 && j <= Ly) {
        const float4 yc = yprof[j - 1];
        const float4 yw = ylru[j - 1];
        double s = la_score_f(u, xc, yc, xsum, yw.w);
        if (bp) {
          // BPLAScore (bpla_kernel.cpp:55-60): float products as written
          const float pp = f32_dot2(xw.y, yw.y, xw.x, yw.x);
          const float uu = xw.z * yw.z;
          s = alpha * (double)pp + (double)uu * s;
        }
        // the left cell (i, j-1); column 0 is zero.  (lM.. keep the last
        // column of the previous row until lane l+1 has taken it.)
        const bool c1 = j == 1;
        const double aM = c1 ? 0.0 : lM, aX = c1 ? 0.0 : lX, aY = c1 ? 0.0 : lY;
        const double aX2 = c1 ? 0.0 : lX2, aY2 = c1 ? 0.0 : lY2;
        double nM, nX, nY, nX2 = 0.0, nY2 = 0.0;
        if (!sw) {
          nM = exp(beta * s) * (1.0 + dX + dY + dM);
          nX = bg * upM + be * upX;
          nY = bg * (aM + aX) + be * aY;
          nX2 = upM + upX2;
          nY2 = aM + aX2 + aY2;
        } else {
          double v = fmax(0.0, dM);
          v = fmax(v, dX);
          v = fmax(v, dY);
          nM = v + s;
          nX = fmax(upM + gap, upX + ext);
          nY = fmax(fmax(aM + gap, aX + gap), aY + ext);
        }
        if (row_ok) {
          lM = nM;
          lX = nX;
          lY = nY;
          lX2 = nX2;
          lY2 = nY2;
          mmax = fmax(mmax, nM);
          if (i == Lx && j == Ly) result = 1.0 + nX2 + nY2 + nM;
        }
        if (lane == 63) {
          bM[j] = nM;
          bX[j] = nX;
          bY[j] = nY;
          bX2[j] = nX2;
        }
      }
      dM = upM;
      dX = upX;
      dY = upY;
      if (++j > Lys) {  // next strip: row i + 64, column 1 (column 0 is zero)
        j = 1;
        ++strip;
        i += 64;
        row_ok = i <= Lx;
        xc = nxc;
        xw = nxw;
        if (i + 64 <= Lx) {
          nxc = sx.pos_prof[xpb + i + 63];
          nxw = sx.pos_lru[xpb + i + 63];
        }
#pragma unroll
        for (int l = 0; l < 4; ++l)
          u[l] = tb[l] * (double)xc.x + tb[4 + l] * (double)xc.y + tb[8 + l] * (double)xc.z +
                 tb[12 + l] * (double)xc.w;
        xsum = dyadic_sum(xc);
        dM = dX = dY = 0.0;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    double r;
    if (sw) {
      for (int off = 32; off > 0; off >>= 1) mmax = fmax(mmax, __shfl_xor(mmax, off, 64));
      r = mmax;
    } else {
      const int owner = Lx == 0 ? 0 : ((Lx - 1) & 63);
      r = (Lx == 0 || Ly == 0) ? 1.0 : __shfl(result, owner, 64);
    }
    if (lane == 0) P.out[P.oidx ? P.oidx[pr] : (int64_t)pr] = r;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

size_t bpla_lds_bytes(const BplaLaunch& P, int nwaves) {
  return 16 * 8 + (size_t)nwaves * bpla_wave_lds_bytes(P.lds_max_len);
}

hipError_t launch_bpla(const BplaLaunch& P, int grid, int nwaves, hipStream_t st) {
  hipLaunchKernelGGL(sk_bpla_kernel, dim3(grid), dim3(64 * nwaves), bpla_lds_bytes(P, nwaves), st,
                     P);
  return hipGetLastError();
}

// ===========================================================================
// Fast path for pairs whose profile columns are all dyadic (every entry a
// multiple of 1/256: single sequences and alignments of 1, 2, 4, 8, ... rows,
// IUPAC codes included).  There LAScore's float weight is n = xs * ys exactly
// (dyadic_sum), so v / n = sum_l (u_l / xs) (y_l / ys): the per-position
// factors are tabulated once per call (sk_bpla_tab_kernel) and a cell costs
// four FMAs instead of 16 products and an FP64 divide.  Two identities of the
// reference recurrences remove work per cell:
//   - X2/Y2 only sum M: X2[i][j] = sum_{i'<i} M[i'][j] and Y2[i][j] =
//     sum_{j'<j} (M[i][j'] + X2[i][j']), so 1 + X2[n][m] + Y2[n][m] + M[n][m]
//     = 1 + sum over all cells of M (bpla_kernel.cpp:104-114): each lane sums
//     its cells and one wave reduction ends the pair;
//   - exp(beta * s) by a table-driven reduction (2^(j/64) in LDS) and a
//     degree-5 Taylor polynomial (relative error ~1e-16), no special-case
//     handling (|beta * s| stays far from the double range).
// The sums run in another order than the reference's (all terms positive,
// ~1e-15 relative); the score keeps the reference's float products
// (BPLAScore, bpla_kernel.cpp:55-60).  A lane's next strip row is prefetched
// from the operand table one strip ahead; the per-wave LDS holds the y
// columns and the strip boundary row only (72 B per column).

__global__ void __launch_bounds__(256) sk_bpla_tab_kernel(const float4* __restrict__ prof,
                                                          const float4* __restrict__ lru,
                                                          int64_t n, const double* __restrict__ tb,
                                                          double xscale, BplaPos* __restrict__ xrole,
                                                          BplaPos* __restrict__ yrole) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const float4 c = prof[p];
  const float4 w = lru[p];
  const float s = dyadic_sum(c);
  BplaPos X, Y;
  const float cv[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
  for (int l = 0; l < 4; ++l) {
    const double u = tb[l] * (double)c.x + tb[4 + l] * (double)c.y + tb[8 + l] * (double)c.z +
                     tb[12 + l] * (double)c.w;
    X.v[l] = s > 0.0f ? u / (double)s * xscale : 0.0;
    Y.v[l] = s > 0.0f ? (double)cv[l] / (double)s : 0.0;
  }
  X.pr = Y.pr = w.y;
  X.pl = Y.pl = w.x;
  X.pu = Y.pu = w.z;
  X.dyadic = Y.dyadic = s >= 0.0f ? 1.0f : 0.0f;
  xrole[p] = X;
  yrole[p] = Y;
}

hipError_t launch_bpla_tab(const float4* prof, const float4* lru, int64_t n, const double* table,
                           double xscale, BplaPos* xrole, BplaPos* yrole, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(sk_bpla_tab_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     prof, lru, n, table, xscale, xrole, yrole);
  return hipGetLastError();
}

template <bool BP, bool FULL>
__device__ __forceinline__ void bpla_fast_chunk2(const BplaLaunch& P, int np, const int4* ci, double* ksum,
                                                 int Ly, const BplaPos* ycol, double* bnd, const double* etab,
                                                 int lane);
template <bool BP, bool FULL>
__device__ __forceinline__ void bpla_fast_chunk3(const BplaLaunch& P, int np, const int4* ci, double* ksum,
                                                 int Ly, const BplaPos* ycol, double* bnd, const double* etab,
                                                 int lane);
// rows per lane of the exp path (2 or 3) and a pair's rows padded to them
// (3: C4 18.71M / 18.80M against 17.95M / 18.01M pairs/s, r04o2)
#ifndef SK_BPLA_ROWS
#define SK_BPLA_ROWS 3
#endif
__device__ __forceinline__ int bpla_pad_rows(int len) {
  return SK_BPLA_ROWS == 3 ? len + (3 - len % 3) % 3 : len + (len & 1);
}

// A chunk of np pairs sharing y on one wavefront: their x rows are streamed
// back to back as one sequence of rows (chunk row G = first row of pair p +
// local row i), so a strip may end one pair's rows and start the next's and
// the drain of a partly filled last strip is paid once per chunk, not per
// pair.  ci[p] = {xtab base, Lx, first chunk row, -} (LDS), ksum[p] receives
// the pair's sum of M cells (exp) or its max (SW: np == 1).  ycol holds y's
// operand columns (LDS), bnd is the wave's boundary row.
//
// Lane l computes chunk row 64s + l + 1 of strip s, one column per step, a
// step behind lane l-1 (DPP wave_shr); a lane moves on to its row of the
// next strip right after its last column.  The steps fall in wave-uniform
// phases: the 64-step WINDOW of strip s (step w: lane w starts its new row
// at column 1, lanes above it finish strip s-1's row), then the INTERIOR
// (every lane inside strip s, columns 2..Ly: no per-lane control flow at
// all).  The next strip's row operands are loaded for all lanes at the end
// of a window, a strip ahead of their use.  The first row of a pair sees row
// 0 (zero) above it: its "up" and "diagonal" inputs are scaled by fb = 0
// (folded into the coefficients, no extra instruction per cell).
template <bool SW, bool BP>
__device__ __forceinline__ void bpla_fast_chunk(const BplaLaunch& P, int np, const int4* ci,
                                                double* ksum, int Ly, const BplaPos* ycol,
                                                double* bnd, const double* etab, int lane) {
  if (!SW) {  // the exp path runs two rows per lane
    if (Ly >= 64)
      SK_BPLA_ROWS == 3 ? bpla_fast_chunk3<BP, true>(P, np, ci, ksum, Ly, ycol, bnd, etab, lane)
                        : bpla_fast_chunk2<BP, true>(P, np, ci, ksum, Ly, ycol, bnd, etab, lane);
    else
      SK_BPLA_ROWS == 3 ? bpla_fast_chunk3<BP, false>(P, np, ci, ksum, Ly, ycol, bnd, etab, lane)
                        : bpla_fast_chunk2<BP, false>(P, np, ci, ksum, Ly, ycol, bnd, etab, lane);
    return;
  }
  const double alpha = P.alpha, beta = P.beta, gap = P.gap, ext = P.ext;
  const double bg = P.beta_gap, be = P.beta_ext;
  const int4 last = ci[np - 1];
  const int Rt = __builtin_amdgcn_readfirstlane(last.z + last.y);  // rows of the chunk
  const int Lys = max(Ly, 64);
  for (int j = lane; j < 3 * (Lys + 1); j += 64) bnd[j] = 0.0;  // row 0
  if (lane < np) ksum[lane] = 0.0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (Rt == 0 || Ly == 0) return;  // no cells: K = 1 (exp) / 0 (SW)
  const int nstrips = (Rt + 63) / 64;
  const int T = (nstrips - 1) * Lys + ((Rt - 1) & 63) + Ly;  // steps
  const char* ybase = reinterpret_cast<const char*>(ycol);

  // chunk row G (1-based) -> its pair, whether it exists, fb, xtab index
  auto map_row = [&](int G, int& pp, bool& ok, double& fbv, int& xi) __attribute__((always_inline)) {
    int q = 0;
    for (int k = 1; k < np; ++k) q += G - 1 >= ci[k].z ? 1 : 0;
    const int4 c = ci[q];
    const int i = G - c.z;
    ok = G <= Rt;
    pp = q;
    fbv = i == 1 ? 0.0 : 1.0;
    xi = ok ? c.x + i - 1 : ci[0].x;
  };
  int pn, xi;
  bool okn;
  double fbn;
  map_row(lane + 1, pn, okn, fbn, xi);
  BplaPos xn = P.xtab[xi];  // the next strip's row operands (strip 0 first)
  BplaPos xr = xn;
  int p = 0;                // my row's pair
  bool row_ok = false;      // my row exists (and has started)
  double fb = 1.0, cbg = bg, cbe = be;  // 0 / 0 / 0 on a pair's first row
  unsigned yofs = 0;        // byte offset of my column j-1 in ycol
  double lM = 0.0, lX = 0.0, lY = 0.0;  // (i, j-1): my previous output
  double acc = 0.0;                      // sum of my row's M cells (exp) / max (SW)

  // cell (i, j) from d = (i-1, j-1), u = (i-1, j) and l = (i, j-1); c1: j == 1
  auto cell = [&](const BplaPos& yc, double dM, double dX, double dY, double uM, double uX, double uY,
                  bool c1, double& nM, double& nX, double& nY) __attribute__((always_inline)) {
    double s = xr.v[0] * yc.v[0];
    s = __builtin_fma(xr.v[1], yc.v[1], s);
    s = __builtin_fma(xr.v[2], yc.v[2], s);
    s = __builtin_fma(xr.v[3], yc.v[3], s);
    if (BP) {
      // BPLAScore (bpla_kernel.cpp:55-60): float products as written
      const float pp = f32_dot2(xr.pr, yc.pr, xr.pl, yc.pl);
      const float uu = xr.pu * yc.pu;
      s = alpha * (double)pp + (double)uu * s;
    }
    if (!SW) {
      nM = fast_exp(beta * s, etab) * __builtin_fma(fb, dX + dY + dM, 1.0);
      nX = cbg * uM + cbe * uX;
      nY = c1 ? 0.0 : bg * (lM + lX) + be * lY;  // column 0 is zero
      // every lane sums its cells; a row that does not exist (past the
      // chunk's last row, never an input of a real one) is dropped at its
      // hand-off, so no per-cell select
      acc += nM;
    } else {
      nM = fmax(fmax(fmax(0.0, fb * dM), fb * dX), fb * dY) + s;
      nX = fmax(fb * uM + gap, fb * uX + ext);
      // column 0 is zero: max(0 + gap, 0 + gap, 0 + ext)
      nY = c1 ? fmax(gap, ext) : fmax(fmax(lM + gap, lX + gap), lY + ext);
      if (row_ok) acc = fmax(acc, nM);
    }
  };

  // step of an interior: lane 0's column jb (uniform); every lane active
  // (SK_BPLA_PF: this step's y column and boundary values were loaded a step
  // earlier, the next step's are loaded here, so the LDS latency overlaps the
  // cell's arithmetic; the last step's loads land past the row, never used)
#ifdef SK_BPLA_PF
  BplaPos ycp;
  double bp0 = 0.0, bp1 = 0.0, bp2 = 0.0;
  auto interior_load = [&](int jb) __attribute__((always_inline)) {
    ycp = *reinterpret_cast<const BplaPos*>(ybase + yofs);
    const double* bj = bnd + 3 * jb;
    bp0 = bj[0];
    bp1 = bj[1];
    bp2 = bj[2];
  };
#endif
  auto interior = [&](int jb, double& dM, double& dX, double& dY, double& uM, double& uX,
                      double& uY) __attribute__((always_inline)) {
#ifdef SK_BPLA_PF
    const BplaPos yc = ycp;
    uM = wave_shr1(lM, bp0);
    uX = wave_shr1(lX, bp1);
    uY = wave_shr1(lY, bp2);
    {
      ycp = *reinterpret_cast<const BplaPos*>(ybase + yofs + (unsigned)sizeof(BplaPos));
      const double* bj = bnd + 3 * (jb + 1);
      bp0 = bj[0];
      bp1 = bj[1];
      bp2 = bj[2];
    }
#else
    const BplaPos yc = *reinterpret_cast<const BplaPos*>(ybase + yofs);
    const double* bj = bnd + 3 * jb;
    uM = wave_shr1(lM, bj[0]);
    uX = wave_shr1(lX, bj[1]);
    uY = wave_shr1(lY, bj[2]);
#endif
    double nM, nX, nY;
    cell(yc, dM, dX, dY, uM, uX, uY, false, nM, nX, nY);
    lM = nM;
    lX = nX;
    lY = nY;
    if (lane == 63) {  // lane 63's column is jb - 63
      double* bw = bnd + 3 * (jb - 63);
      bw[0] = nM;
      bw[1] = nX;
      bw[2] = nY;
    }
    yofs += (unsigned)sizeof(BplaPos);
  };

  // step w of strip s's window: lane w starts its row of strip s at column 1
  // (diagonal and left are column 0: zero), handing its finished row's sum
  // to the pair; lanes below it are at column w - lane + 1 of strip s, lanes
  // above at column Lys + w - lane + 1 of strip s-1 (none for s = 0).  The
  // window of s = nstrips is the drain: only the last strip's lanes above w
  // are still working.
  auto window = [&](int s, int w, double& dM, double& dX, double& dY, double& uM, double& uX,
                    double& uY) __attribute__((always_inline)) {
    const bool wrap = lane == w;
    if (wrap) {
      if (row_ok) {
        if (SW) ksum[p] = fmax(ksum[p], acc);
        else ksum[p] += acc;
      }
      acc = 0.0;
      xr = xn;
      p = pn;
      row_ok = okn;
      fb = fbn;
      cbg = bg * fbn;
      cbe = be * fbn;
      yofs = 0;
      dM = dX = dY = 0.0;
    }
    const int jl = lane <= w ? w - lane + 1 : Lys + w - lane + 1;
    const bool on = jl <= Ly && (lane <= w ? s < nstrips : s > 0);
    const int jb = w + 1;  // lane 0's column (strip s)
    const double* bj = bnd + 3 * (jb <= Ly ? jb : 0);
    uM = wave_shr1(lM, bj[0]);
    uX = wave_shr1(lX, bj[1]);
    uY = wave_shr1(lY, bj[2]);
    if (on) {
      const BplaPos yc = *reinterpret_cast<const BplaPos*>(ybase + yofs);
      double nM, nX, nY;
      cell(yc, dM, dX, dY, uM, uX, uY, wrap, nM, nX, nY);
      lM = nM;
      lX = nX;
      lY = nY;
      if (lane == 63) {
        double* bw = bnd + 3 * jl;
        bw[0] = nM;
        bw[1] = nX;
        bw[2] = nY;
      }
    }
    yofs += (unsigned)sizeof(BplaPos);
  };

  // d* = values received a step earlier, u* = this step's; the unrolled
  // pairs of steps swap their roles (no register copies)
  double aM = 0.0, aX = 0.0, aY = 0.0, bM = 0.0, bX = 0.0, bY = 0.0;
  for (int s = 0; s <= nstrips; ++s) {
    const int Ws = s * Lys;
    const int wend = min(64, T - Ws);
    if (wend <= 0) break;
    int w = 0;
    for (; w + 1 < wend; w += 2) {
      window(s, w, aM, aX, aY, bM, bX, bY);
      window(s, w + 1, bM, bX, bY, aM, aX, aY);
    }
    if (w < wend) {
      window(s, w, aM, aX, aY, bM, bX, bY);
      aM = bM;
      aX = bX;
      aY = bY;
    }
    if (s + 1 < nstrips) {
      map_row(64 * (s + 1) + lane + 1, pn, okn, fbn, xi);
      xn = P.xtab[xi];
    }
    const int tend = s < nstrips ? min(Ws + Lys, T) : 0;
    int t = Ws + 64;
#ifdef SK_BPLA_PF
    if (t < tend) interior_load(t - Ws + 1);
#endif
    for (; t + 1 < tend; t += 2) {
      interior(t - Ws + 1, aM, aX, aY, bM, bX, bY);
      interior(t - Ws + 2, bM, bX, bY, aM, aX, aY);
    }
    if (t < tend) {
      interior(t - Ws + 1, aM, aX, aY, bM, bX, bY);
      aM = bM;
      aX = bX;
      aY = bY;
    }
  }
  // the rows still held
  if (SW) {  // (acc >= 0: it starts at 0)
    for (int off = 32; off > 0; off >>= 1) acc = fmax(acc, __shfl_xor(acc, off, 64));
    if (lane == 0) ksum[0] = fmax(ksum[0], acc);
  } else if (row_ok) {
    __hip_atomic_fetch_add(&ksum[p], acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The exp path (local_alignment_exp) with TWO rows per lane: lane l of
// strip s computes chunk rows A = 128s + 2l + 1 and B = A + 1 at one column
// per step, a step behind lane l-1, so a 64-step window serves 128 rows and
// the per-step shared work -- the y column read from LDS, the three DPP
// shifts of the row above, the boundary-row traffic of lane 63, the
// window's per-lane control -- is paid once per two cells.  Row A's "up" is
// lane l-1's row B (DPP; lane 0: the boundary row in LDS), row B's "up" is
// this lane's row A of the same step and its diagonal row A's previous
// output (registers).  Every pair is padded to an even row count (a dummy
// row after an odd last row; its cells are computed and dropped) so a lane's
// two rows always belong to one pair and a pair's first row is always an A
// row (fb = 0 there).  Rows that do not exist are dropped at the hand-off
// (okA / okB), as in the one-row schedule.  xtab holds the x operands with
// beta folded in (v[l] * beta), so the exponent is
// fma(uu, s, alpha * beta * pp) (BP) or s (LA).
template <bool BP, bool FULL>
__device__ __forceinline__ void bpla_fast_chunk2(const BplaLaunch& P, int np, const int4* ci, double* ksum,
                                                 int Ly, const BplaPos* ycol, double* bnd, const double* etab,
                                                 int lane) {
  const double ab = P.alpha * P.beta;
  const double bg = P.beta_gap, be = P.beta_ext;
  const int4 last = ci[np - 1];
  const int Rt = __builtin_amdgcn_readfirstlane(last.z + last.y + (last.y & 1));  // padded rows
  const int Lys = max(Ly, 64);
  for (int j = lane; j < 3 * (Lys + 1); j += 64) bnd[j] = 0.0;  // row 0
  if (lane < np) ksum[lane] = 0.0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (Rt == 0 || Ly == 0) return;  // no cells: K = 1
  const int Rp = Rt >> 1;          // row pairs
  const int nstrips = (Rp + 63) / 64;
  const int T = (nstrips - 1) * Lys + ((Rp - 1) & 63) + Ly;  // steps
  const char* ybase = reinterpret_cast<const char*>(ycol);

  // row pair (chunk rows GA = 2 * Q + 1, GA + 1) -> pair, existence, fb, xtab index
  auto map_pair = [&](int Q, int& pp, bool& oka, bool& okb, double& fbv, int& xi) __attribute__((always_inline)) {
    const int G = 2 * Q + 1;
    int q = 0;
    for (int k = 1; k < np; ++k) q += G - 1 >= ci[k].z ? 1 : 0;
    const int4 c = ci[q];
    const int i = G - c.z;  // odd, <= c.y when the row exists
    oka = G <= Rt;
    okb = oka && i + 1 <= c.y;
    pp = q;
    fbv = i == 1 ? 0.0 : 1.0;
    xi = oka ? c.x + i - 1 : ci[0].x;
  };
  int pn, xi;
  bool okan, okbn;
  double fbn;
  map_pair(lane, pn, okan, okbn, fbn, xi);
  BplaPos xnA = P.xtab[xi], xnB = P.xtab[okbn ? xi + 1 : xi];  // the next strip's operands
  BplaPos xA = xnA, xB = xnB;
  int p = 0;
  bool okA = false, okB = false;
  double fb = 1.0, cbg = bg, cbe = be;  // row A's: 0 / 0 / 0 on a pair's first row
  unsigned yofs = 0;
  double aM = 0.0, aX = 0.0, aY = 0.0;  // row A at (., j-1)
  double bM = 0.0, bX = 0.0, bY = 0.0;  // row B at (., j-1)
  double accA = 0.0, accB = 0.0;

  auto expo = [&](const BplaPos& xr, const BplaPos& yc) __attribute__((always_inline)) {
    double s = xr.v[0] * yc.v[0];
    s = __builtin_fma(xr.v[1], yc.v[1], s);
    s = __builtin_fma(xr.v[2], yc.v[2], s);
    s = __builtin_fma(xr.v[3], yc.v[3], s);
    if (BP) {
      // BPLAScore (bpla_kernel.cpp:55-60): float products as written
      const float pp = f32_dot2(xr.pr, yc.pr, xr.pl, yc.pl);
      const float uu = xr.pu * yc.pu;
      s = __builtin_fma((double)uu, s, ab * (double)pp);
    }
    return fast_exp(s, etab);
  };
  // both cells of a step: dS = M + X + Y of the row above at (j-1) (lane
  // l-1 sends its row B's sum, bS), u = row above at j (lane l-1's row B);
  // c1: column 1 (left is column 0: zero).  A row's left sum M + X is
  // shared by its Y recurrence and the diagonal sum it hands on.
  // sB1 = bM + bX and sB2 = sB1 + bY of row B's latest outputs, carried from
  // step to step: each is formed once per step (the row-B Y recurrence, the
  // diagonal sum handed on, lane 63's boundary write), not once per use
  double sB1 = 0.0, sB2 = 0.0;
  auto cells = [&](const BplaPos& yc, double dS, double uM, double uX, bool c1) __attribute__((always_inline)) {
    const double eA = expo(xA, yc);
    const double eB = expo(xB, yc);
    const double sA = aM + aX;
    const double nMA = eA * __builtin_fma(fb, dS, 1.0);
    const double nXA = cbg * uM + cbe * uX;
    const double nYA = c1 ? 0.0 : bg * sA + be * aY;
    const double nMB = __builtin_fma(eB, sA + aY, eB);  // diagonal: row A at j-1
    const double nXB = bg * nMA + be * nXA;
    const double nYB = c1 ? 0.0 : bg * sB1 + be * bY;
    aM = nMA;
    aX = nXA;
    aY = nYA;
    bM = nMB;
    bX = nXB;
    bY = nYB;
    accA += nMA;
    accB += nMB;
    sB1 = nMB + nXB;
    sB2 = sB1 + nYB;
    __asm__ volatile("" : "+v"(sB2));  // formed here, once, ahead of lane 63's write
  };

  // interior step: lane 0's column jb, every lane active
  // (the boundary row holds {M, X, M + X + Y} of row B per column)
  // Interior operands are read a step ahead (the y column and lane 0's
  // boundary values of the next step land during this step's arithmetic):
  // (yc, b*) this step's, (ycn, n*) the next step's.
  auto iload = [&](int jb, BplaPos& yc, double& b0, double& b1, double& b2) __attribute__((always_inline)) {
    yc = *reinterpret_cast<const BplaPos*>(ybase + yofs);
    const double* bj = bnd + 3 * jb;
    b0 = bj[0];
    b1 = bj[1];
    b2 = bj[2];
  };
  auto interior = [&](int jb, double& dS, double& uS, const BplaPos& yc, double b0, double b1, double b2,
                      BplaPos& ycn, double& n0, double& n1, double& n2) __attribute__((always_inline)) {
    ycn = *reinterpret_cast<const BplaPos*>(ybase + yofs + (unsigned)sizeof(BplaPos));
    {
      const double* bj = bnd + 3 * (jb + 1);
      n0 = bj[0];
      n1 = bj[1];
      n2 = bj[2];
    }
    const double uM = wave_shr1(bM, b0);
    const double uX = wave_shr1(bX, b1);
    uS = wave_shr1(sB2, b2);
    cells(yc, dS, uM, uX, false);
    if (lane == 63) {  // lane 63's column is jb - 63
      double* bw = bnd + 3 * (jb - 63);
      bw[0] = bM;
      bw[1] = bX;
      bw[2] = sB2;
    }
    yofs += (unsigned)sizeof(BplaPos);
  };

  // window step w of strip s: lane w starts its rows of strip s at column 1,
  // handing its finished rows' sums to their pair (rows that exist only);
  // lanes below are at column w - lane + 1 of strip s, lanes above at column
  // Lys + w - lane + 1 of strip s-1
  // FULL (Ly >= 64, so Lys = Ly): every lane computes every window step.
  // The cells of lanes that have not started strip 0 yet are garbage that
  // their wrap discards (sums and left / diagonal values reset, row B's left
  // masked at column 1), and those of lanes past the last strip belong to
  // rows that do not exist (dropped at the hand-off); lane 63's stray
  // boundary writes in strip 0 land on columns it overwrites with the real
  // values before lane 0 of strip 1 reads them.  Otherwise (Ly < 64: columns
  // past Ly in every strip) the cells of columns past Ly are skipped.
  auto window = [&](int s, int w, double& dM, double& dX, double& dS, double& uM, double& uX, double& uS)
                    __attribute__((always_inline)) {
    (void)dM;
    (void)dX;
    const bool wrap = lane == w;
    if (wrap) {
      // the finished rows' sums stay in the lane while its next rows belong
      // to the same pair; they go to the pair's sum when the pair changes
      const double h = accA + (okB ? accB : 0.0);
      const bool cont = okA && okan && pn == p;
      // (an LDS add without return: no read round trip inside the window;
      // one lane, this wave's own sums, so the order of additions is kept)
      if (okA && !cont) __hip_atomic_fetch_add(&ksum[p], h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
      accA = cont ? h : 0.0;
      accB = 0.0;
      xA = xnA;
      xB = xnB;
      p = pn;
      okA = okan;
      okB = okbn;
      fb = fbn;
      cbg = bg * fbn;
      cbe = be * fbn;
      yofs = 0;
      dS = 0.0;
      aM = aX = aY = 0.0;  // row A's column 0 (row B's diagonal at column 1)
    }
    const int jb = w + 1;  // lane 0's column (strip s)
    const double* bj = bnd + 3 * (jb <= Ly ? jb : 0);
    uM = wave_shr1(bM, bj[0]);
    uX = wave_shr1(bX, bj[1]);
    uS = wave_shr1(sB2, bj[2]);
    if (FULL) {
      const BplaPos yc = *reinterpret_cast<const BplaPos*>(ybase + yofs);
      cells(yc, dS, uM, uX, wrap);
      // lane 63's column: w - 62 once it wrapped (w = 63), else Lys + w - 62
      const int j63 = w == 63 ? 1 : Lys + w - 62;
      if (lane == 63) {
        double* bw = bnd + 3 * j63;
        bw[0] = bM;
        bw[1] = bX;
        bw[2] = sB2;
      }
    } else {
      const int jl = lane <= w ? w - lane + 1 : Lys + w - lane + 1;
      const bool on = jl <= Ly && (lane <= w ? s < nstrips : s > 0);
      if (on) {
        const BplaPos yc = *reinterpret_cast<const BplaPos*>(ybase + yofs);
        cells(yc, dS, uM, uX, wrap);
        if (lane == 63) {
          double* bw = bnd + 3 * jl;
          bw[0] = bM;
          bw[1] = bX;
          bw[2] = sB2;
        }
      }
    }
    yofs += (unsigned)sizeof(BplaPos);
  };

  // d* = values received a step earlier, u* = this step's; the unrolled
  // pairs of steps swap their roles (no register copies)
  double pM = 0.0, pX = 0.0, pY = 0.0, qM = 0.0, qX = 0.0, qY = 0.0;
  for (int s = 0; s <= nstrips; ++s) {
    const int Ws = s * Lys;
    const int wend = min(64, T - Ws);
    if (wend <= 0) break;
    int w = 0;
    for (; w + 1 < wend; w += 2) {
      window(s, w, pM, pX, pY, qM, qX, qY);
      window(s, w + 1, qM, qX, qY, pM, pX, pY);
    }
    if (w < wend) {
      window(s, w, pM, pX, pY, qM, qX, qY);
      pM = qM;
      pX = qX;
      pY = qY;
    }
    if (s + 1 < nstrips) {
      map_pair(64 * (s + 1) + lane, pn, okan, okbn, fbn, xi);
      xnA = P.xtab[xi];
      xnB = P.xtab[okbn ? xi + 1 : xi];
    } else {
      // the drain: a lane that wraps past the last strip holds no rows (its
      // cells there are computed, FULL, and must not be handed on)
      okan = okbn = false;
    }
    const int tend = s < nstrips ? min(Ws + Lys, T) : 0;
    int t = Ws + 64;
    if (t < tend) {
      BplaPos yc0, yc1;
      double a0, a1, a2, c0, c1, c2;
      iload(t - Ws + 1, yc0, a0, a1, a2);
      for (; t + 1 < tend; t += 2) {
        interior(t - Ws + 1, pY, qY, yc0, a0, a1, a2, yc1, c0, c1, c2);
        interior(t - Ws + 2, qY, pY, yc1, c0, c1, c2, yc0, a0, a1, a2);
      }
      if (t < tend) {
        interior(t - Ws + 1, pY, qY, yc0, a0, a1, a2, yc1, c0, c1, c2);
        pY = qY;
      }
    }
  }
  // the rows still held
  if (okA) {
    const double h = accA + (okB ? accB : 0.0);
    __hip_atomic_fetch_add(&ksum[p], h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// SK_BPLA_ROWS 3: THREE rows per lane (rows A, B, C = 192s + 3l + 1 ..
// + 3): the per-step shared work (y column, DPP shifts of the row above,
// lane 63's boundary row, the window's per-lane control) is paid once per
// three cells; pairs are padded to a multiple of three rows; row C is the
// lane's last row (handed to lane l+1 and to the boundary row).  Same
// operations per cell as the two-row schedule.
template <bool BP, bool FULL>
__device__ __forceinline__ void bpla_fast_chunk3(const BplaLaunch& P, int np, const int4* ci, double* ksum,
                                                 int Ly, const BplaPos* ycol, double* bnd, const double* etab,
                                                 int lane) {
  const double ab = P.alpha * P.beta;
  const double bg = P.beta_gap, be = P.beta_ext;
  const int4 last = ci[np - 1];
  const int Rt = __builtin_amdgcn_readfirstlane(last.z + bpla_pad_rows(last.y));  // padded rows
  const int Lys = max(Ly, 64);
  for (int j = lane; j < 3 * (Lys + 1); j += 64) bnd[j] = 0.0;  // row 0
  if (lane < np) ksum[lane] = 0.0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (Rt == 0 || Ly == 0) return;  // no cells: K = 1
  const int Rp = Rt / 3;           // row triples
  const int nstrips = (Rp + 63) / 64;
  const int T = (nstrips - 1) * Lys + ((Rp - 1) & 63) + Ly;  // steps
  const char* ybase = reinterpret_cast<const char*>(ycol);

  // row triple (chunk rows GA = 3 * Q + 1, GA + 1, GA + 2) -> pair,
  // existence, fb, xtab index
  auto map_pair = [&](int Q, int& pp, bool& oka, bool& okb, bool& okc, double& fbv, int& xi)
                      __attribute__((always_inline)) {
    const int G = 3 * Q + 1;
    int q = 0;
    for (int k = 1; k < np; ++k) q += G - 1 >= ci[k].z ? 1 : 0;
    const int4 c = ci[q];
    const int i = G - c.z;  // 1 mod 3, <= c.y when the row exists
    oka = G <= Rt;
    okb = oka && i + 1 <= c.y;
    okc = oka && i + 2 <= c.y;
    pp = q;
    fbv = i == 1 ? 0.0 : 1.0;
    xi = oka ? c.x + i - 1 : ci[0].x;
  };
  int pn, xi;
  bool okan, okbn, okcn;
  double fbn;
  map_pair(lane, pn, okan, okbn, okcn, fbn, xi);
  BplaPos xnA = P.xtab[xi], xnB = P.xtab[okbn ? xi + 1 : xi], xnC = P.xtab[okcn ? xi + 2 : xi];
  BplaPos xA = xnA, xB = xnB, xC = xnC;
  int p = 0;
  bool okA = false, okB = false, okC = false;
  double fb = 1.0, cbg = bg, cbe = be;  // row A's: 0 / 0 / 0 on a pair's first row
  unsigned yofs = 0;
  double aM = 0.0, aX = 0.0, aY = 0.0;  // row A at (., j-1)
  double bY = 0.0;  // row B's Y at (., j-1) (its M + X: sB1)
  double cM = 0.0, cX = 0.0, cY = 0.0;  // row C at (., j-1)
  double accA = 0.0, accB = 0.0, accC = 0.0;

  auto expo = [&](const BplaPos& xr, const BplaPos& yc) __attribute__((always_inline)) {
    double s = xr.v[0] * yc.v[0];
    s = __builtin_fma(xr.v[1], yc.v[1], s);
    s = __builtin_fma(xr.v[2], yc.v[2], s);
    s = __builtin_fma(xr.v[3], yc.v[3], s);
    if (BP) {
      // BPLAScore (bpla_kernel.cpp:55-60): float products as written
      const float pp = f32_dot2(xr.pr, yc.pr, xr.pl, yc.pl);
      const float uu = xr.pu * yc.pu;
      s = __builtin_fma((double)uu, s, ab * (double)pp);
    }
    return fast_exp(s, etab);
  };
  // both cells of a step: dS = M + X + Y of the row above at (j-1) (lane
  // l-1 sends its row B's sum, bS), u = row above at j (lane l-1's row B);
  // c1: column 1 (left is column 0: zero).  A row's left sum M + X is
  // shared by its Y recurrence and the diagonal sum it hands on.
  // sB1 = bM + bX and sB2 = sB1 + bY of row B's latest outputs, carried from
  // step to step: each is formed once per step (the row-B Y recurrence, the
  // diagonal sum handed on, lane 63's boundary write), not once per use
  // (three rows: row C is the lane's last -- its sums go down and to the
  // boundary row; rows B and C take up and diagonal from the row before)
  double sB1 = 0.0, sC1 = 0.0, sC2 = 0.0;
  auto cells = [&](const BplaPos& yc, double dS, double uM, double uX, bool c1) __attribute__((always_inline)) {
    (void)c1;
    const double eA = expo(xA, yc);
    const double eB = expo(xB, yc);
    const double eC = expo(xC, yc);
    const double sA = aM + aX;
    const double nMA = eA * __builtin_fma(fb, dS, 1.0);
    const double nXA = cbg * uM + cbe * uX;
    // (column 1, c1: the wrap reset every left value, so these are 0 -- no select)
    const double nYA = bg * sA + be * aY;
    const double nMB = __builtin_fma(eB, sA + aY, eB);  // diagonal: row A at j-1
    const double nXB = bg * nMA + be * nXA;
    const double nYB = bg * sB1 + be * bY;
    const double nMC = __builtin_fma(eC, sB1 + bY, eC);  // diagonal: row B at j-1
    const double nXC = bg * nMB + be * nXB;
    const double nYC = bg * sC1 + be * cY;
    aM = nMA;
    aX = nXA;
    aY = nYA;
    bY = nYB;
    cM = nMC;
    cX = nXC;
    cY = nYC;
    accA += nMA;
    accB += nMB;
    accC += nMC;
    sB1 = nMB + nXB;
    sC1 = nMC + nXC;
    sC2 = sC1 + nYC;
    __asm__ volatile("" : "+v"(sC2));  // formed here, once, ahead of lane 63's write
  };

  // interior step: lane 0's column jb, every lane active
  // (the boundary row holds {M, X, M + X + Y} of row B per column)
  // Interior operands are read a step ahead (the y column and lane 0's
  // boundary values of the next step land during this step's arithmetic):
  // (yc, b*) this step's, (ycn, n*) the next step's.
  auto iload = [&](int jb, BplaPos& yc, double& b0, double& b1, double& b2) __attribute__((always_inline)) {
    yc = *reinterpret_cast<const BplaPos*>(ybase + yofs);
    const double* bj = bnd + 3 * jb;
    b0 = bj[0];
    b1 = bj[1];
    b2 = bj[2];
  };
  auto interior = [&](int jb, double& dS, double& uS, const BplaPos& yc, double b0, double b1, double b2,
                      BplaPos& ycn, double& n0, double& n1, double& n2) __attribute__((always_inline)) {
    ycn = *reinterpret_cast<const BplaPos*>(ybase + yofs + (unsigned)sizeof(BplaPos));
    {
      const double* bj = bnd + 3 * (jb + 1);
      n0 = bj[0];
      n1 = bj[1];
      n2 = bj[2];
    }
    const double uM = wave_shr1(cM, b0);
    const double uX = wave_shr1(cX, b1);
    uS = wave_shr1(sC2, b2);
    cells(yc, dS, uM, uX, false);
    if (lane == 63) {  // lane 63's column is jb - 63
      double* bw = bnd + 3 * (jb - 63);
      bw[0] = cM;
      bw[1] = cX;
      bw[2] = sC2;
    }
    yofs += (unsigned)sizeof(BplaPos);
  };

  // window step w of strip s: lane w starts its rows of strip s at column 1,
  // handing its finished rows' sums to their pair (rows that exist only);
  // lanes below are at column w - lane + 1 of strip s, lanes above at column
  // Lys + w - lane + 1 of strip s-1
  // FULL (Ly >= 64, so Lys = Ly): every lane computes every window step.
  // The cells of lanes that have not started strip 0 yet are garbage that
  // their wrap discards (sums and left / diagonal values reset, row B's left
  // masked at column 1), and those of lanes past the last strip belong to
  // rows that do not exist (dropped at the hand-off); lane 63's stray
  // boundary writes in strip 0 land on columns it overwrites with the real
  // values before lane 0 of strip 1 reads them.  Otherwise (Ly < 64: columns
  // past Ly in every strip) the cells of columns past Ly are skipped.
  auto window = [&](int s, int w, double& dM, double& dX, double& dS, double& uM, double& uX, double& uS)
                    __attribute__((always_inline)) {
    (void)dM;
    (void)dX;
    const bool wrap = lane == w;
    if (wrap) {
      // the finished rows' sums stay in the lane while its next rows belong
      // to the same pair; they go to the pair's sum when the pair changes
      const double h = accA + (okB ? accB : 0.0) + (okC ? accC : 0.0);
      const bool cont = okA && okan && pn == p;
      // (an LDS add without return: no read round trip inside the window;
      // one lane, this wave's own sums, so the order of additions is kept)
      if (okA && !cont) __hip_atomic_fetch_add(&ksum[p], h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
      accA = cont ? h : 0.0;
      accB = accC = 0.0;
      xA = xnA;
      xB = xnB;
      xC = xnC;
      p = pn;
      okA = okan;
      okB = okbn;
      okC = okcn;
      fb = fbn;
      cbg = bg * fbn;
      cbe = be * fbn;
      yofs = 0;
      dS = 0.0;
      aM = aX = aY = 0.0;  // row A's column 0 (row B's diagonal at column 1)
      sB1 = bY = 0.0;      // row B's column 0 (row C's diagonal at column 1)
      sC1 = cY = 0.0;      // row C's left at column 1 (cM, cX, sC2 stay: lane w+1's row above)
    }
    const int jb = w + 1;  // lane 0's column (strip s)
    const double* bj = bnd + 3 * (jb <= Ly ? jb : 0);
    uM = wave_shr1(cM, bj[0]);
    uX = wave_shr1(cX, bj[1]);
    uS = wave_shr1(sC2, bj[2]);
    if (FULL) {
      const BplaPos yc = *reinterpret_cast<const BplaPos*>(ybase + yofs);
      cells(yc, dS, uM, uX, wrap);
      // lane 63's column: w - 62 once it wrapped (w = 63), else Lys + w - 62
      const int j63 = w == 63 ? 1 : Lys + w - 62;
      if (lane == 63) {
        double* bw = bnd + 3 * j63;
        bw[0] = cM;
        bw[1] = cX;
        bw[2] = sC2;
      }
    } else {
      const int jl = lane <= w ? w - lane + 1 : Lys + w - lane + 1;
      const bool on = jl <= Ly && (lane <= w ? s < nstrips : s > 0);
      if (on) {
        const BplaPos yc = *reinterpret_cast<const BplaPos*>(ybase + yofs);
        cells(yc, dS, uM, uX, wrap);
        if (lane == 63) {
          double* bw = bnd + 3 * jl;
          bw[0] = cM;
          bw[1] = cX;
          bw[2] = sC2;
        }
      }
    }
    yofs += (unsigned)sizeof(BplaPos);
  };

  // d* = values received a step earlier, u* = this step's; the unrolled
  // pairs of steps swap their roles (no register copies)
  double pM = 0.0, pX = 0.0, pY = 0.0, qM = 0.0, qX = 0.0, qY = 0.0;
  for (int s = 0; s <= nstrips; ++s) {
    const int Ws = s * Lys;
    const int wend = min(64, T - Ws);
    if (wend <= 0) break;
    int w = 0;
    for (; w + 1 < wend; w += 2) {
      window(s, w, pM, pX, pY, qM, qX, qY);
      window(s, w + 1, qM, qX, qY, pM, pX, pY);
    }
    if (w < wend) {
      window(s, w, pM, pX, pY, qM, qX, qY);
      pM = qM;
      pX = qX;
      pY = qY;
    }
    if (s + 1 < nstrips) {
      map_pair(64 * (s + 1) + lane, pn, okan, okbn, okcn, fbn, xi);
      xnA = P.xtab[xi];
      xnB = P.xtab[okbn ? xi + 1 : xi];
      xnC = P.xtab[okcn ? xi + 2 : xi];
    } else {
      // the drain: a lane that wraps past the last strip holds no rows (its
      // cells there are computed, FULL, and must not be handed on)
      okan = okbn = okcn = false;
    }
    const int tend = s < nstrips ? min(Ws + Lys, T) : 0;
    int t = Ws + 64;
    if (t < tend) {
      BplaPos yc0, yc1;
      double a0, a1, a2, c0, c1, c2;
      iload(t - Ws + 1, yc0, a0, a1, a2);
      for (; t + 1 < tend; t += 2) {
        interior(t - Ws + 1, pY, qY, yc0, a0, a1, a2, yc1, c0, c1, c2);
        interior(t - Ws + 2, qY, pY, yc1, c0, c1, c2, yc0, a0, a1, a2);
      }
      if (t < tend) {
        interior(t - Ws + 1, pY, qY, yc0, a0, a1, a2, yc1, c0, c1, c2);
        pY = qY;
      }
    }
  }
  // the rows still held
  if (okA) {
    const double h = accA + (okB ? accB : 0.0) + (okC ? accC : 0.0);
    __hip_atomic_fetch_add(&ksum[p], h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Pairs dealt one per wave: each wave stages its own y columns.
template <bool SW, bool BP>
__global__ void __launch_bounds__(256) sk_bpla_fast_kernel(BplaLaunch P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int maxlen = P.lds_max_len;  // even, >= 64
  double* etab = reinterpret_cast<double*>(smem);
  unsigned char* wbase = smem + kBplaExpLds + (size_t)wave * bpla_fast_wave_lds_bytes(maxlen);
  BplaPos* ycol = reinterpret_cast<BplaPos*>(wbase);
  double* bnd = reinterpret_cast<double*>(ycol + maxlen);
  int4* ci = reinterpret_cast<int4*>(bnd + 3 * (maxlen + 2));
  double* ksum = reinterpret_cast<double*>(ci + kBplaChunkMax);
  fill_exp_table(etab);
  // the wave's next pair: lane 0 draws, the value goes through SGPRs
  auto next_pair = [&]() {
    unsigned long long v = 0;
    if (lane == 0) v = atomicAdd(P.pair_counter, 1ull);
    return (int64_t)(((unsigned long long)__builtin_amdgcn_readlane((unsigned)(v >> 32), 0) << 32) |
                     (unsigned)__builtin_amdgcn_readlane((unsigned)v, 0));
  };
  for (int64_t pr = next_pair(); pr < P.n_pairs; pr = next_pair()) {
    const int x = __builtin_amdgcn_readfirstlane(P.xs[pr]);
    const int y = __builtin_amdgcn_readfirstlane(P.ys[pr]);
    const int Ly = __builtin_amdgcn_readfirstlane(P.yset.ex_len[y]);
    const int ypb = P.yset.ex_pos_base[y];
    for (int j = lane; j < Ly; j += 64) ycol[j] = P.ytab[ypb + j];
    if (lane == 0) ci[0] = make_int4(P.xset.ex_pos_base[x], P.xset.ex_len[x], 0, 0);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    bpla_fast_chunk<SW, BP>(P, 1, ci, ksum, Ly, ycol, bnd, etab, lane);
    if (lane == 0) P.out[P.oidx ? P.oidx[pr] : (int64_t)pr] = SW ? ksum[0] : 1.0 + ksum[0];
  }
}

// Pairs grouped by y into items {first, count} of one y: a workgroup stages
// the y columns once in LDS for all its waves, and its waves take chunks of
// the item's pairs (P.chunk at a time) from an LDS counter.  Per wave only
// the boundary row (24 B per column) and the chunk table, so 16 waves fit a
// CU.
// SK_BPLA_WPE (build-time): ask the register allocator for that many waves
// per SIMD (96 VGPRs give 5)
#ifdef SK_BPLA_WPE
#define SK_BPLA_ITEMS_ATTR __attribute__((amdgpu_waves_per_eu(SK_BPLA_WPE)))
#else
#define SK_BPLA_ITEMS_ATTR
#endif
template <bool SW, bool BP>
__global__ void __launch_bounds__(64 * kBplaItemsWavesMax) SK_BPLA_ITEMS_ATTR
    sk_bpla_fast_items_kernel(BplaLaunch P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int maxlen = P.lds_max_len;
  double* etab = reinterpret_cast<double*>(smem);
  int* sh = reinterpret_cast<int*>(smem + kBplaExpLds);  // [0] item, [1] in-item counter
  BplaPos* ycol = reinterpret_cast<BplaPos*>(smem + kBplaExpLds + 16);
  unsigned char* wb = reinterpret_cast<unsigned char*>(ycol + maxlen) +
                      (size_t)wave * (3 * (maxlen + 2) * 8 + kBplaChunkLds);
  double* bnd = reinterpret_cast<double*>(wb);
  int4* ci = reinterpret_cast<int4*>(bnd + 3 * (maxlen + 2));
  double* ksum = reinterpret_cast<double*>(ci + kBplaChunkMax);
  // P.chunk = 0: per item, the fewest pairs per chunk that give every wave
  // one chunk (the workgroup waits for its slowest wave at the item's end)
  const int nw = (int)(blockDim.x >> 6);
  fill_exp_table(etab);
  for (;;) {
    if (threadIdx.x == 0) {
      sh[0] = (int)atomicAdd(P.pair_counter, 1ull);
      sh[1] = 0;
    }
    __syncthreads();
    const int it = __builtin_amdgcn_readfirstlane(sh[0]);
    if (it >= P.n_items) break;
    const int2 item0 = P.items[it];
    const int2 item = make_int2(__builtin_amdgcn_readfirstlane(item0.x),
                                __builtin_amdgcn_readfirstlane(item0.y));
    const int y = __builtin_amdgcn_readfirstlane(P.ys[item.x]);
    const int Ly = __builtin_amdgcn_readfirstlane(P.yset.ex_len[y]);
    const int ypb = P.yset.ex_pos_base[y];
    for (int j = threadIdx.x; j < Ly; j += blockDim.x) ycol[j] = P.ytab[ypb + j];
    __syncthreads();
    const int chunk = SW ? 1
                         : __builtin_amdgcn_readfirstlane(
                               min(max(P.chunk > 0 ? P.chunk : (item.y + nw - 1) / nw, 1), kBplaChunkMax));
    // the wave's next chunk of the item: lane 0 draws, through an SGPR
    auto next_k = [&]() {
      int v = 0;
      if (lane == 0) v = atomicAdd(&sh[1], chunk);
      return __builtin_amdgcn_readlane(v, 0);
    };
    for (int k = next_k(); k < item.y; k = next_k()) {
      const int np = min(chunk, item.y - k);
      // chunk table: first rows by an exclusive prefix sum over the pairs
      int len = 0, pb = 0;
      if (lane < np) {
        const int x = P.xs[item.x + k + lane];
        len = P.xset.ex_len[x];
        pb = P.xset.ex_pos_base[x];
      }
      int start = 0;
      for (int q = 0; q < np - 1; ++q) {
        const int lq = __shfl(len, q, 64);
        start += lane > q ? (SW ? lq : bpla_pad_rows(lq)) : 0;  // the exp path pads pairs (SK_BPLA_ROWS)
      }
      if (lane < np) ci[lane] = make_int4(pb, len, start, 0);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      bpla_fast_chunk<SW, BP>(P, np, ci, ksum, Ly, ycol, bnd, etab, lane);
      double kv = lane < np ? ksum[lane] : 0.0;
      // A pair whose sums overflow to inf (long rows, as in the reference)
      // poisons the pairs after it in the chunk: their first row sees its
      // last row through the fb = 0 coefficients, and 0 * inf = NaN.  Such a
      // chunk (rare: never on finite sums) is redone one pair at a time.
      if (!SW && np > 1 && __builtin_amdgcn_ballot_w64(lane < np && !__builtin_isfinite(kv)) != 0) {
        for (int q = 0; q < np; ++q) {
          const int lq = __shfl(len, q, 64), bq = __shfl(pb, q, 64);
          if (lane == 0) ci[0] = make_int4(bq, lq, 0, 0);
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          bpla_fast_chunk<SW, BP>(P, 1, ci, ksum, Ly, ycol, bnd, etab, lane);
          const double v = ksum[0];
          if (lane == q) kv = v;
        }
      }
      if (lane < np) {
        const int64_t pr = (int64_t)item.x + k + lane;
        P.out[P.oidx ? P.oidx[pr] : pr] = SW ? kv : 1.0 + kv;
      }
    }
    __syncthreads();
  }
}

hipError_t launch_bpla_fast(const BplaLaunch& P, int grid, int nwaves, hipStream_t st) {
  const bool items = P.items != nullptr;
  const size_t lds = items ? bpla_items_lds_bytes(P.lds_max_len, nwaves)
                           : kBplaExpLds + (size_t)nwaves * bpla_fast_wave_lds_bytes(P.lds_max_len);
#define SK_BF(K, A, B)                                                                       \
  do {                                                                                       \
    hipError_t e = hipFuncSetAttribute((const void*)K<A, B>,                                 \
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
    if (e != hipSuccess) return e;                                                           \
    hipLaunchKernelGGL((K<A, B>), dim3(grid), dim3(64 * nwaves), lds, st, P);                \
  } while (0)
#define SK_BF2(K)                      \
  if (P.sw) {                          \
    if (P.bp) SK_BF(K, true, true);    \
    else SK_BF(K, true, false);        \
  } else {                             \
    if (P.bp) SK_BF(K, false, true);   \
    else SK_BF(K, false, false);       \
  }
  if (items) {
    SK_BF2(sk_bpla_fast_items_kernel)
  } else {
    SK_BF2(sk_bpla_fast_kernel)
  }
#undef SK_BF2
#undef SK_BF
  return hipGetLastError();
}

}  // namespace sk
