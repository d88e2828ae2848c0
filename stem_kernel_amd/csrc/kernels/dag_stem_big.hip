// DAG stem-kernel DP for y examples beyond the register classes (gfx950).
//
// Reference: StemKernel<ST,MData>::operator()  stem_kernel_lite/stem_kernel.cpp:14-95
// (node scores score_table.cpp:14-53, 118-134; edge scores :60-101), which
// has no size limit.  sk_dag_stem_kernel (dag_stem.hip) holds a y example's
// non-leaf nodes in 64 x MAXK register slots (MAXK <= 32: 2048 nodes) and its
// IY sweep records as child:11 | parent:11 | gaps:10; a y example with more
// nodes, or a stem edge gap over 1023, comes here instead.
//
// Same reformulation as dag_stem.hip (K never stored: path sums P_x M P_y;
// leaf rows / columns in closed form; one weighted child row S per x row),
// but the y DAG is read in LEVEL order from the packed x-role arrays
// (nd_*, ed, lvl; 16-bit local ids) straight from HBM (L2-resident per y),
// and the per-row vectors live in per-wave scratch instead of registers and
// LDS:
//   A. S[q]  = sum_{c in ch(p)} g^gaps G0[c][q]            (lane-strided q)
//   B. level by level (children first), a pull per node, no atomics:
//        M[q]  = node_score(p,q) * H[q] inside the length band,
//        H[q]  = sum_{cy in ch(q)} g^gy S[cy]   (loop q: closed form),
//        G1[q] = M[q] + sum_{cy} G1[cy] * (gap^2 w_y(q)) * g^gy,
//        K    += P_x[p] * M[q] * P_y[q];
//   C. G0[p][q] = G1[q] + v_s(p) S[q] -> p's recycled slot.
// One wavefront per pair; the lanes of a wave exchange S / G1 through
// global memory, so the phases are separated by workgroup-scope fences
// (all lanes of a wave share one CU's vector L1).
#include <hip/hip_runtime.h>

#include "device_set.h"
#include "launch.h"

namespace sk {

__device__ __forceinline__ void lane_exchange_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// node_match_score (score_table.cpp:162-201 Subst / :14-53 Simple): the
// bp-frequency double sum in the reference's order, then the two gap-column
// terms.  co = exp(beta * ribosum) or the match / mismatch table.
__device__ __forceinline__ double big_node_score(const double* __restrict__ co, const DevSet& xs,
                                                 int xbf, int xnbf, double x_nbp, double x_nseq,
                                                 double xwg, const DevSet& ys, int ybf, int ynbf,
                                                 double y_nbp, double y_nseq, double ywg) {
  double v = 0.0;
  for (int a = 0; a < xnbf; ++a) {
    const double cx = (double)xs.bpf_p[xbf + a];
    const uint32_t ca = xs.bpf_code[xbf + a] * 16u;
    for (int b = 0; b < ynbf; ++b) v += co[ca + ys.bpf_code[ybf + b]] * cx * (double)ys.bpf_p[ybf + b];
  }
  v += ywg * x_nbp / x_nseq;
  v += xwg * y_nbp / y_nseq;
  return v;
}

__device__ double big_pair(const StemBigLaunch& P, double* __restrict__ S, double* __restrict__ G,
                           double* __restrict__ slab, int x, int y, int lane) {
  const DevSet& s = P.xset;
  const DevSet& ys = P.yset;
  const int nlx = s.ex_nl[x], nly = ys.ex_nl[y];
  if (nlx == 0 || nly == 0) return 0.0;
  const double* __restrict__ gp = P.gpow;
  const double* __restrict__ co = P.co_subst;
  const int64_t stride = P.stride;
  const double gap2 = P.gap2;
  const int band = (int)P.band;
  const int xnb = s.ex_node_base[x], xbb = s.ex_bpf_base[x];
  const double x_nseq = (double)s.ex_nseqs[x];
  int chp = s.ex_xch_base[x];
  const int ynb = ys.ex_node_base[y], yeb = ys.ex_edge_base[y], ybb = ys.ex_bpf_base[y];
  const int32_t* __restrict__ ylv = ys.lvl + ys.ex_lvl_base[y];
  const int nlev = ys.ex_nlev[y];
  const double y_nseq = (double)ys.ex_nseqs[y];
  double kacc = 0.0;  // this lane's share of K

  for (int r = 0; r < nlx; ++r) {
    const XRow xr = s.xrow[xnb + r];
    const int xne = xr.a & 0xff, xnbf = (xr.a >> 8) & 0xff;
    const bool xloop = xne == 0;
    const double xeg0 = gp[xr.a >> 16];
    const int xlen = xr.b & 0xffff;
    const uint32_t pslot = xr.b >> 16;
    const int xbf = xbb + (int)(xr.c & 0xffff);
    const double xwg = gap2 * (double)xr.w;
    const double x_nbp = (double)xr.nbp;
    const double xSL = P.pn.xr_SL[xnb + r];

    // ---- A: weighted child-row sum (x loop rows have only a leaf child: S = 0)
    for (int q = lane; q < nly; q += 64) {
      double acc = 0.0;
      for (int t = 0; t < xne; ++t) {
        const uint32_t c = s.xr_ch[chp + t];
        acc += gp[c >> 16] * slab[(int64_t)(c & 0xffff) * stride + q];
      }
      S[q] = acc;
    }
    chp += xne;
    lane_exchange_fence();

    // ---- B: MATCH and IY, level by level
    double rowk = 0.0;
    for (int lv = 0; lv < nlev; ++lv) {
      const int q1 = ylv[lv + 1];
      for (int q = ylv[lv] + lane; q < q1; q += 64) {
        const uint32_t a = ys.nd_a[ynb + q];
        const int ne = (a >> 16) & 0xff, e0 = a & 0xffff, ynbf = a >> 24;
        const uint32_t b = ys.nd_b[ynb + q];
        const int ylen = b & 0xffff;
        const double wy = (double)ys.nd_w[ynb + q];
        double M = 0.0;
        if (band == 0 || abs(xlen - ylen) <= band) {
          double H = 0.0;
          if (ne == 0) {  // loop node: its single leaf child, G0[*][leaf] closed form
            H = (xloop ? xeg0 : xSL) * gp[ys.nd_c[ynb + q]];
          } else if (!xloop) {
            for (int t = 0; t < ne; ++t) {
              const uint32_t e = ys.ed[yeb + e0 + t].x;
              H += gp[e >> 16] * S[e & 0xffff];
            }
          }
          if (H != 0.0)
            M = big_node_score(co, s, xbf, xnbf, x_nbp, x_nseq, xwg, ys, ybb + (int)(b >> 16), ynbf,
                               (double)ys.nd_nbp[ynb + q], y_nseq, gap2 * wy) *
                H;
        }
        double g1 = M;
        if (ne > 0) {  // G1[q] += G1[cy] * v_s * e_s  (stem_kernel.cpp:61-77 order)
          const double vsy = gap2 * wy;
          for (int t = 0; t < ne; ++t) {
            const uint32_t e = ys.ed[yeb + e0 + t].x;
            g1 += G[e & 0xffff] * vsy * gp[e >> 16];
          }
        }
        G[q] = g1;
        rowk += M * ys.nd_P[ynb + q];
      }
      lane_exchange_fence();
    }
    kacc += xr.P * rowk;

    // ---- C: G0 row p (rows nobody reads are not stored)
    if (pslot != 0xffffu) {
      double* __restrict__ orow = slab + (int64_t)pslot * stride;
      for (int q = lane; q < nly; q += 64) orow[q] = G[q] + xwg * S[q];
    }
    lane_exchange_fence();
  }
  for (int off = 32; off > 0; off >>= 1) kacc += __shfl_xor(kacc, off, 64);
  return kacc;
}

__global__ void __launch_bounds__(64 * kStemBigWaves) sk_dag_stem_big_kernel(StemBigLaunch P) {
  const int lane = threadIdx.x & 63;
  // wave index as an SGPR value: the pair loop and everything in big_pair
  // that depends on the pair is wave-uniform
  const int gw = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * kStemBigWaves + (threadIdx.x >> 6)));
  const int nw = (int)gridDim.x * kStemBigWaves;
  double* base = P.scratch + (int64_t)gw * P.wave_doubles;
  double* S = base;
  double* G = base + P.stride;
  double* slab = base + 2 * P.stride;
  // pairs dealt cyclically (the host orders them costliest y first)
  for (int64_t k = gw; k < P.n_pairs; k += nw) {
    const double v = big_pair(P, S, G, slab, P.xs[k], P.ys[k], lane);
    if (lane == 0) P.out[P.oidx ? P.oidx[k] : k] = v;
  }
}

hipError_t launch_stem_big(const StemBigLaunch& P, int grid, hipStream_t st) {
  if (grid <= 0 || P.n_pairs <= 0) return hipSuccess;
  hipLaunchKernelGGL(sk_dag_stem_big_kernel, dim3(grid), dim3(64 * kStemBigWaves), 0, st, P);
  return hipGetLastError();
}

}  // namespace sk
