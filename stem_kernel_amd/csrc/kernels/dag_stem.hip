// DAG stem-kernel DP on CDNA4 (gfx950).
//
// Reference: StemKernel<ST,MData>::operator()  stem_kernel_lite/stem_kernel.cpp:49-130
// with SubstNodeScore / SimpleNodeScore / SimpleEdgeScore  score_table.cpp:193-380.
//
// Reformulation (exact in real arithmetic):
//   * The reference carries four tables K0,G0 (|Vx|x|Vy|) and K1,G1 (rows).
//     K1/K0 are pure path sums of the MATCH term M:
//        K(x,y) = sum_{p,q non-leaf} P_x[p] * M[p][q] * P_y[q]
//     with P[v] = number of root->v paths (host-precomputed), so K tables are
//     never stored.
//   * Leaf rows/columns of G0 are closed forms: G0[leaf][leaf]=1,
//     G0[leaf][q]=0, G0[p][leaf]=L[p] (per-x, from sk_prep_kernel).
//   * Only G0 over non-leaf x non-leaf nodes is materialised, one row per
//     x-node, in a per-wave HBM slab; G1 (the IY recurrence of a row) lives in
//     LDS and is swept level by level (levels of the y-DAG are contiguous).
//
// Parallel structure: one WAVEFRONT per (x,y) pair; a workgroup of W waves
// shares one y example (its DAG staged once in LDS) and pulls x examples from
// a per-item LDS cursor; workgroups pull items from a global counter
// (persistent grid).  No MFMA: this is a recurrence, not a contraction.
#include <hip/hip_runtime.h>

#include "device_set.h"
#include "launch.h"

namespace sk {

// ---------------------------------------------------------------------------
// Per-call prep: L[p] = G0[p][y-leaf column] and SL[p] = sum_e g^gaps L[child]
// (one thread per example, nodes in level order = children first).
// L reproduces the reference's G0[i][leaf] cells exactly:
//   G0[i][j] = G1[j](=0) ; G0[i][j] += G0[ex.to][j]*v_s*e_s   (stem_kernel.cpp:105-112)
__global__ void sk_prep_kernel(DevSet s, DevParamNodes pn, const double* __restrict__ gpow,
                               double gap2) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= s.n_examples) return;
  const int nl = s.ex_nl[e];
  const int nb = s.ex_node_base[e], eb = s.ex_edge_base[e];
  for (int k = 0; k < nl; ++k) {
    const uint32_t a = s.nd_a[nb + k];
    const int e0 = a & 0xffff, ne = (a >> 16) & 0xff;
    const double v_s = gap2 * (double)s.nd_w[nb + k];
    double L = 0.0, SL = 0.0;
    for (int t = 0; t < ne; ++t) {
      const uint32_t ed = s.ed[eb + e0 + t];
      const uint32_t c = ed & 0xffff;
      const double gp = gpow[ed >> 16];
      const double Lc = (c == kLeafChild) ? 1.0 : pn.nd_L[nb + c];
      L += Lc * v_s * gp;
      if (c != kLeafChild) SL += gp * Lc;
    }
    pn.nd_L[nb + k] = L;
    pn.nd_SL[nb + k] = SL;
  }
}

// ---------------------------------------------------------------------------
struct YView {  // the y example staged in LDS
  const uint32_t* a;
  const uint32_t* b;
  const float* w;
  const float* nbp;
  const double* P;
  const uint32_t* ed;
  const uint32_t* bc;
  const float* bp;
  const int32_t* lv;
  int nl, nlev;
  float nseqs;
};

__device__ __forceinline__ void wave_sync() {
  // LDS traffic of one wave is processed in issue order; this only pins the
  // compiler's instruction order.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// node_score(xx,yy,i,j): score_table.cpp:343-380 (Subst) / 193-232 (Simple);
// co[] holds exp(beta*ribosum) or the match/mismatch table.
__device__ __forceinline__ double match_node_score(const double* __restrict__ co,
                                                   const DevSet& s, int xbb, int xb0, int xnb,
                                                   const YView& Y, int yb0, int ynb, double xwg,
                                                   double ywg, double x_nbp, double y_nbp,
                                                   double x_nseq) {
  double v = 0.0;
  for (int a = 0; a < xnb; ++a) {
    const double cx = (double)s.bpf_p[xbb + xb0 + a];
    const uint32_t ca = s.bpf_code[xbb + xb0 + a] * 16u;
    for (int b = 0; b < ynb; ++b) {
      const double cy = (double)Y.bp[yb0 + b];
      v += co[ca + Y.bc[yb0 + b]] * cx * cy;
    }
  }
  v += ywg * x_nbp / x_nseq;
  v += xwg * y_nbp / (double)Y.nseqs;
  return v;
}

__device__ double stem_pair(const StemLaunch& P, const YView& Y, double* __restrict__ G1,
                            const double* __restrict__ co, const double* __restrict__ gp,
                            double* __restrict__ slab, int x, int lane) {
  const DevSet& s = P.xset;
  const int nlx = s.ex_nl[x];
  const int NLy = Y.nl;
  if (nlx == 0 || NLy == 0) return 0.0;
  const int xnb = s.ex_node_base[x], xeb = s.ex_edge_base[x], xbb = s.ex_bpf_base[x];
  const double x_nseq = (double)s.ex_nseqs[x];
  const int nloop_y = Y.lv[1];  // level 0 = loop nodes
  const double gap2 = P.gap2;
  const uint32_t band = P.band;
  double kacc = 0.0;

  for (int p = 0; p < nlx; ++p) {
    // ---- x node p (wave-uniform: scalar loads)
    const uint32_t xa = s.nd_a[xnb + p], xb = s.nd_b[xnb + p];
    const int xe0 = xa & 0xffff, xne = (xa >> 16) & 0xff, xnbf = xa >> 24;
    const int xlen = xb & 0xffff, xb0 = xb >> 16;
    const double xwg = gap2 * (double)s.nd_w[xnb + p];
    const double x_nbp = (double)s.nd_nbp[xnb + p];
    const double xP = s.nd_P[xnb + p];
    const uint32_t xed0 = s.ed[xeb + xe0];
    const bool xloop = (xed0 & 0xffff) == kLeafChild;
    const double xSL = P.pn.nd_SL[xnb + p];
    const double xeg0 = gp[xed0 >> 16];

    // ---- pass A: MATCH term of every y node, into G1; K contribution
    double rowk = 0.0;
    for (int q = lane; q < NLy; q += 64) {
      const uint32_t ya = Y.a[q], yb = Y.b[q];
      const int ylen = yb & 0xffff;
      double M = 0.0;
      const int dl = xlen - ylen;
      if (band == 0 || (uint32_t)(dl < 0 ? -dl : dl) <= band) {
        const int ye0 = ya & 0xffff, yne = (ya >> 16) & 0xff;
        double H;
        if (q < nloop_y) {
          const double egy = gp[Y.ed[ye0] >> 16];
          H = xloop ? xeg0 * egy : xSL * egy;
        } else if (xloop) {
          H = 0.0;
        } else {
          H = 0.0;
          for (int t = 0; t < xne; ++t) {
            const uint32_t e = s.ed[xeb + xe0 + t];
            const double* __restrict__ row = slab + (size_t)(e & 0xffff) * NLy;
            double inner = 0.0;
            for (int u = 0; u < yne; ++u) {
              const uint32_t f = Y.ed[ye0 + u];
              inner += gp[f >> 16] * row[f & 0xffff];
            }
            H += gp[e >> 16] * inner;
          }
        }
        if (H != 0.0) {
          const double ywg = gap2 * (double)Y.w[q];
          const double vs = match_node_score(co, s, xbb, xb0, xnbf, Y, yb >> 16, ya >> 24, xwg,
                                             ywg, x_nbp, (double)Y.nbp[q], x_nseq);
          M = vs * H;
        }
      }
      G1[q] = M;
      rowk += M * Y.P[q];
    }
    kacc += xP * rowk;
    wave_sync();

    // ---- pass B: IY recurrence, level by level (levels >= 1 are stems)
    for (int l = 1; l < Y.nlev; ++l) {
      const int q1 = Y.lv[l + 1];
      for (int q = Y.lv[l] + lane; q < q1; q += 64) {
        const uint32_t ya = Y.a[q];
        const int ye0 = ya & 0xffff, yne = (ya >> 16) & 0xff;
        const double v_s = gap2 * (double)Y.w[q];
        double acc = G1[q];
        for (int u = 0; u < yne; ++u) {
          const uint32_t f = Y.ed[ye0 + u];
          acc += G1[f & 0xffff] * v_s * gp[f >> 16];
        }
        G1[q] = acc;
      }
      wave_sync();
    }

    // ---- pass C: IX term, G0 row p to the slab
    double* __restrict__ orow = slab + (size_t)p * NLy;
    for (int q = lane; q < NLy; q += 64) {
      double g0 = G1[q];
      if (!xloop) {
        for (int t = 0; t < xne; ++t) {
          const uint32_t e = s.ed[xeb + xe0 + t];
          g0 += slab[(size_t)(e & 0xffff) * NLy + q] * xwg * gp[e >> 16];
        }
      }
      orow[q] = g0;
    }
    // make row p visible to the other lanes' loads of the next rows
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  // wave reduction of the K partial sums (fixed order -> deterministic)
  for (int off = 32; off > 0; off >>= 1) kacc += __shfl_xor(kacc, off, 64);
  return kacc;
}

__global__ void __launch_bounds__(1024) sk_dag_stem_kernel(StemLaunch P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const DevSet& s = P.yset;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nwaves = blockDim.x >> 6;
  const int maxnl = P.lds_max_nl;

  // LDS carve (every region a multiple of 16 bytes)
  double* co = reinterpret_cast<double*>(smem);             // 256
  double* gp = co + 256;                                     // n_gpow_pad
  double* yP = gp + P.n_gpow_pad;                            // maxnl
  double* G1all = yP + maxnl;                                // nwaves*maxnl
  uint32_t* ya = reinterpret_cast<uint32_t*>(G1all + (size_t)nwaves * maxnl);
  uint32_t* yb = ya + maxnl;
  float* yw = reinterpret_cast<float*>(yb + maxnl);
  float* ynbp = yw + maxnl;
  uint32_t* yed = reinterpret_cast<uint32_t*>(ynbp + maxnl);  // lds_max_edges
  uint32_t* ybc = yed + P.lds_max_edges;                      // lds_max_bpf
  float* ybp = reinterpret_cast<float*>(ybc + P.lds_max_bpf);
  int32_t* ylv = reinterpret_cast<int32_t*>(ybp + P.lds_max_bpf);  // lds_max_nlev+1
  int32_t* ctl = ylv + P.lds_max_nlev_pad;                    // 4 ints

  for (int k = threadIdx.x; k < 256; k += blockDim.x) co[k] = P.co_subst[k];
  for (int k = threadIdx.x; k < P.n_gpow; k += blockDim.x) gp[k] = P.gpow[k];

  double* G1 = G1all + (size_t)wave * maxnl;
  double* slab = P.scratch + (size_t)(blockIdx.x * nwaves + wave) * P.slab_doubles;

  // wave index as an SGPR value: every branch below on it is wave-uniform
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  for (;;) {
    __syncthreads();
    if (threadIdx.x == 0) ctl[0] = atomicAdd(P.item_counter, 1);
    __syncthreads();
    const int it = __builtin_amdgcn_readfirstlane(ctl[0]);
    if (it >= P.n_items) break;
    const int4 item = P.items[it];  // {y, base, count, -}
    const int y = item.x;
    YView Y;
    Y.nl = s.ex_nl[y];
    Y.nlev = s.ex_nlev[y];
    Y.nseqs = s.ex_nseqs[y];
    {
      const int nb = s.ex_node_base[y], eb = s.ex_edge_base[y], bb = s.ex_bpf_base[y];
      const int ne = s.ex_edge_base[y + 1] - eb, nbf = s.ex_bpf_base[y + 1] - bb;
      const int lb = s.ex_lvl_base[y];
      for (int k = threadIdx.x; k < Y.nl; k += blockDim.x) {
        ya[k] = s.nd_a[nb + k];
        yb[k] = s.nd_b[nb + k];
        yw[k] = s.nd_w[nb + k];
        ynbp[k] = s.nd_nbp[nb + k];
        yP[k] = s.nd_P[nb + k];
      }
      for (int k = threadIdx.x; k < ne; k += blockDim.x) yed[k] = s.ed[eb + k];
      for (int k = threadIdx.x; k < nbf; k += blockDim.x) {
        ybc[k] = s.bpf_code[bb + k];
        ybp[k] = s.bpf_p[bb + k];
      }
      for (int k = threadIdx.x; k <= Y.nlev; k += blockDim.x) ylv[k] = s.lvl[lb + k];
    }
    Y.a = ya; Y.b = yb; Y.w = yw; Y.nbp = ynbp; Y.P = yP;
    Y.ed = yed; Y.bc = ybc; Y.bp = ybp; Y.lv = ylv;
    __syncthreads();

    // static round-robin of the item's pairs over the waves (uniform loop)
    for (int t = wave_u; t < item.z; t += nwaves) {
      const int x = P.xs[item.y + t];
      const double k = stem_pair(P, Y, G1, co, gp, slab, x, lane);
      if (lane == 0) P.out[P.oidx[item.y + t]] = k;
    }
  }
}

// ---------------------------------------------------------------------------
hipError_t launch_prep(const DevSet& s, const DevParamNodes& pn, const double* gpow, double gap2,
                       hipStream_t st) {
  const int bs = 64;
  const int grid = (s.n_examples + bs - 1) / bs;
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(sk_prep_kernel, dim3(grid), dim3(bs), 0, st, s, pn, gpow, gap2);
  return hipGetLastError();
}

size_t stem_lds_bytes(const StemLaunch& P, int nwaves) {
  size_t b = 0;
  b += 256 * 8;
  b += (size_t)P.n_gpow_pad * 8;
  b += (size_t)P.lds_max_nl * 8;                   // yP
  b += (size_t)nwaves * P.lds_max_nl * 8;          // G1 rows
  b += (size_t)P.lds_max_nl * 16;                  // ya,yb,yw,ynbp
  b += (size_t)P.lds_max_edges * 4;
  b += (size_t)P.lds_max_bpf * 8;
  b += (size_t)P.lds_max_nlev_pad * 4;
  b += 16;
  return b;
}

hipError_t launch_stem(const StemLaunch& P, int grid, int nwaves, hipStream_t st) {
  const size_t lds = stem_lds_bytes(P, nwaves);
  hipLaunchKernelGGL(sk_dag_stem_kernel, dim3(grid), dim3(64 * nwaves), lds, st, P);
  return hipGetLastError();
}

hipError_t stem_kernel_attr(int* max_dyn_lds) {
  hipFuncAttributes attr;
  hipError_t e = hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(sk_dag_stem_kernel));
  if (e != hipSuccess) return e;
  *max_dyn_lds = 163840 - (int)attr.sharedSizeBytes;
  return hipSuccess;
}

}  // namespace sk
