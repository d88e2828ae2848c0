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
    if (ne == 0) {  // loop node: its single child is a leaf (G0[leaf][leaf] = 1)
      L += 1.0 * v_s * gpow[s.nd_c[nb + k]];
    } else {
      for (int t = 0; t < ne; ++t) {
        const uint32_t ed = s.ed[eb + e0 + t].x;
        const double gp = gpow[ed >> 16];
        const double Lc = pn.nd_L[nb + (ed & 0xffff)];
        L += Lc * v_s * gp;
        SL += gp * Lc;
      }
    }
    pn.nd_L[nb + k] = L;
    pn.nd_SL[nb + k] = SL;
  }
  for (int r = 0; r < nl; ++r) pn.xr_SL[nb + r] = pn.nd_SL[nb + s.xr_node[nb + r]];
}

// ---------------------------------------------------------------------------
struct YView {  // the y example staged in LDS
  const uint32_t* b;   // len:16 | bpf_beg:16
  const uint32_t* c;   // loop gaps
  const float* w;
  const float* nbp;
  const double* P;
  const uint2* ed;
  const uint32_t* bc;
  const float* bp;
  const int32_t* lv;   // level -> first node
  const int32_t* lve;  // level -> first edge
  int nl, nlev;
  float nseqs;
};

__device__ __forceinline__ void wave_sync() {
  // LDS traffic of one wave is processed in issue order; this pins the
  // compiler's instruction order and waits for outstanding LDS operations.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

#ifdef SK_STAMPS
#define STAMP(i)                                                  \
  do {                                                            \
    __builtin_amdgcn_sched_barrier(0);                            \
    const unsigned long long _t = __builtin_amdgcn_s_memtime();   \
    tacc[i] += _t - tlast;                                        \
    tlast = _t;                                                   \
    __builtin_amdgcn_sched_barrier(0);                            \
  } while (0)
#else
#define STAMP(i) do {} while (0)
#endif

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

// One (x,y) pair on one wavefront.
//
// Rows p of G0 (x non-leaf nodes) are produced in the reference's post-order
// (x_order), each into a recycled HBM row slot (nd_slot; 0xffff = never read,
// not stored).  Lane l owns the y nodes q = l + 64k (k < MAXK) for phases A,
// B and D; their y-structure fields are hoisted into registers per item.
//
// Both x-child sums of the reference are linear in the child rows, so one
// weighted row suffices:   S[q] = sum_{c in ch(p)} g^gaps(p,c) * G0[c][q]
//   IX term   : sum_c G0[c][q] * v_s(p) * g^gaps = v_s(p) * S[q]
//   MATCH sum : sum_c sum_cy g^gx g^gy G0[c][cy] = sum_{cy in ch(q)} g^gy S[cy]
// For a stem row p:
//   A. stream the child rows from HBM (coalesced, pipelined) into S (regs);
//      S -> per-wave LDS row R; H[k] = sum_{cy in ch(q)} g^gy R[cy] (in band);
//   B. M[q] = node_score(p,q) * H (closed forms for loop nodes) -> R (G1);
//      K += P_x[p] * sum_q M[q] P_y[q];
//   C. IY sweep over the y levels, edge-parallel: G1[q] += G1[cy]*w(q,cy)
//      with w = gap^2*w_y(q)*g^gaps precomputed per item (LDS f64 atomics);
//   D. G0[p][q] = G1[q] + v_s(p)*S[k] -> slot of p.
template <int MAXK>
__device__ double stem_pair(const StemLaunch& P, const YView& Y, const uint32_t (&qe)[MAXK],
                            const uint32_t (&ql)[MAXK / 2], double* __restrict__ R,
                            const double* __restrict__ yew, const double* __restrict__ co,
                            const double* __restrict__ gp, double* __restrict__ slab, int x,
                            int lane) {
  const DevSet& s = P.xset;
  const int nlx = s.ex_nl[x];
  const int NLy = Y.nl;
  if (nlx == 0 || NLy == 0) return 0.0;
  const int xnb = s.ex_node_base[x], xbb = s.ex_bpf_base[x];
  int chp = s.ex_xch_base[x];
  const double x_nseq = (double)s.ex_nseqs[x];
  const int nloop_y = Y.lv[1];  // level 0 = loop nodes
  const double gap2 = P.gap2;
  const int band = (int)P.band;
  double kacc = 0.0;
#ifdef SK_STAMPS
  unsigned long long tacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tlast = __builtin_amdgcn_s_memtime();
#endif

  // x-row header and first child records, prefetched one row ahead
  uint32_t na = s.xr_a[xnb], nbw = s.xr_b[xnb], nc = s.xr_c[xnb];
  float nw = s.xr_w[xnb], nnbp = s.xr_nbp[xnb], nbp0 = s.xr_bp0[xnb];
  double nP = s.xr_P[xnb], nSL = P.pn.xr_SL[xnb];
  uint32_t nch[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) nch[j] = s.xr_ch[chp + j];

  for (int r = 0; r < nlx; ++r) {
    const uint32_t xa = na, xb = nbw, xc = nc;
    const double xwg = gap2 * (double)nw;
    const double x_nbp = (double)nnbp;
    const double xP = nP, xSL = nSL, xpf = (double)nbp0;
    uint32_t ch[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) ch[j] = nch[j];
    const int xne = xa & 0xff, xnbf = (xa >> 8) & 0xff;
    const int chp_r = chp;
    chp += xne;
    if (r + 1 < nlx) {
      na = s.xr_a[xnb + r + 1];
      nbw = s.xr_b[xnb + r + 1];
      nc = s.xr_c[xnb + r + 1];
      nw = s.xr_w[xnb + r + 1];
      nnbp = s.xr_nbp[xnb + r + 1];
      nbp0 = s.xr_bp0[xnb + r + 1];
      nP = s.xr_P[xnb + r + 1];
      nSL = P.pn.xr_SL[xnb + r + 1];
#pragma unroll
      for (int j = 0; j < 4; ++j) nch[j] = s.xr_ch[chp + j];
    }
    const int xlen = xb & 0xffff;
    const uint32_t pslot = xb >> 16;
    const int xb0 = xc & 0xffff;
    const bool xloop = xne == 0;
    const double xeg0 = gp[xa >> 16];
    // single bp-frequency entry of x (the common single-sequence case)
    const bool x_one = xnbf == 1 && x_nbp == 0.0;
    const uint32_t xcode = (xc >> 16) * 16u;
    // band mask of my y nodes for this row
    uint32_t inb = 0;
#pragma unroll
    for (int k = 0; k < MAXK; ++k) {
      const int dl = xlen - (int)((ql[k >> 1] >> (16 * (k & 1))) & 0xffff);
      if (qe[k] != 0xffffffffu && (band == 0 || (dl < 0 ? -dl : dl) <= band)) inb |= 1u << k;
    }
    STAMP(0);

    // ---- A: S = sum_c g^gaps G0[c][*]  (coalesced HBM row streams)
    double S[MAXK];
#pragma unroll
    for (int k = 0; k < MAXK; ++k) S[k] = 0.0;
    for (int t = 0; t < xne; t += 2) {
      const uint32_t c0 = t < 4 ? ch[t] : s.xr_ch[chp_r + t];
      const bool two = t + 1 < xne;
      const uint32_t c1 = two ? (t + 1 < 4 ? ch[t + 1] : s.xr_ch[chp_r + t + 1]) : c0;
      const double eg0 = gp[c0 >> 16], eg1 = two ? gp[c1 >> 16] : 0.0;
      const double* __restrict__ r0 = slab + (size_t)(c0 & 0xffff) * NLy;
      const double* __restrict__ r1 = slab + (size_t)(c1 & 0xffff) * NLy;
#pragma unroll
      for (int k = 0; k < MAXK; ++k) {
        const int q = lane + 64 * k;
        if (q < NLy) S[k] += eg0 * r0[q] + eg1 * r1[q];
      }
    }
    STAMP(1);
    double H[MAXK];
#pragma unroll
    for (int k = 0; k < MAXK; ++k) H[k] = 0.0;
    if (!xloop) {
#pragma unroll
      for (int k = 0; k < MAXK; ++k) {
        const int q = lane + 64 * k;
        if (q < NLy) R[q] = S[k];
      }
      wave_sync();
      // MATCH sums over y-children: up to 4 edges per node in one predicated
      // pass (all LDS reads independent), longer edge lists after it
      uint32_t more = 0;
#pragma unroll
      for (int k = 0; k < MAXK; ++k) {
        const int q = lane + 64 * k;
        const bool on = (inb >> k & 1u) && q >= nloop_y;
        const int e0 = qe[k] & 0xffff, ne = on ? (int)((qe[k] >> 16) & 0xff) : 0;
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (j < ne) {
            const uint32_t f = Y.ed[e0 + j].x;
            acc += gp[f >> 16] * R[f & 0xffff];
          }
        }
        H[k] = acc;
        if (ne > 4) more |= 1u << k;
      }
      if (__builtin_amdgcn_read_exec() && __any(more != 0)) {
#pragma unroll
        for (int k = 0; k < MAXK; ++k) {
          if (more >> k & 1u) {
            const int e0 = qe[k] & 0xffff, ne = (qe[k] >> 16) & 0xff;
            double acc = H[k];
            for (int j = 4; j < ne; ++j) {
              const uint32_t f = Y.ed[e0 + j].x;
              acc += gp[f >> 16] * R[f & 0xffff];
            }
            H[k] = acc;
          }
        }
      }
      wave_sync();
    }
    STAMP(2);

    // ---- B: MATCH term (node score, closed forms for loops) -> R, K part
    double rowk = 0.0;
#pragma unroll
    for (int k = 0; k < MAXK; ++k) {
      const int q = lane + 64 * k;
      if (q < NLy) {
        double M = 0.0;
        if (inb >> k & 1u) {
          double Hq;
          if (q < nloop_y) {
            const double egy = gp[Y.c[q]];
            Hq = xloop ? xeg0 * egy : xSL * egy;
          } else {
            Hq = H[k];
          }
          if (Hq != 0.0) {
            const uint32_t e = qe[k], b = Y.b[q];
            const float ynbp = Y.nbp[q];
            double vs;
            if (x_one && (e >> 24) == 1u && ynbp == 0.0f) {
              // co[a][b][c][d]*cx*cy, no gap columns (score_table.cpp:350-364)
              vs = co[xcode + Y.bc[b >> 16]] * xpf * (double)Y.bp[b >> 16];
            } else {
              const double ywg = gap2 * (double)Y.w[q];
              vs = match_node_score(co, s, xbb, xb0, xnbf, Y, b >> 16, e >> 24, xwg, ywg, x_nbp,
                                    (double)ynbp, x_nseq);
            }
            M = vs * Hq;
          }
        }
        R[q] = M;
        rowk += M * Y.P[q];
      }
    }
    kacc += xP * rowk;
    wave_sync();
    STAMP(3);

    // ---- C: IY recurrence, level by level, edge-parallel (levels >= 1).
    //         Level bounds are read two levels ahead and edge records one
    //         level ahead, so only the R reads stay on the dependency chain.
    if (Y.nlev > 1) {
      int fa = Y.lve[1], fb = Y.lve[2];
      int fc = Y.lve[Y.nlev > 2 ? 3 : 2];
      uint2 rec = make_uint2(0, 0);
      double w = 0.0;
      if (fa + lane < fb) {
        rec = Y.ed[fa + lane];
        w = yew[fa + lane];
      }
      for (int l = 1; l < Y.nlev; ++l) {
        // next level [fb, fc); level after next ends at fd
        const int fd = (l + 3 <= Y.nlev) ? Y.lve[l + 3] : fc;
        uint2 rec2 = make_uint2(0, 0);
        double w2 = 0.0;
        if (fb + lane < fc) {
          rec2 = Y.ed[fb + lane];
          w2 = yew[fb + lane];
        }
        if (fa + lane < fb) atomicAdd(&R[rec.y], R[rec.x & 0xffff] * w);
        for (int f = fa + 64 + lane; f < fb; f += 64) {  // levels with > 64 edges
          const uint2 rr = Y.ed[f];
          atomicAdd(&R[rr.y], R[rr.x & 0xffff] * yew[f]);
        }
        wave_sync();
        fa = fb;
        fb = fc;
        fc = fd;
        rec = rec2;
        w = w2;
      }
    }
    STAMP(4);

    // ---- D: G0 row p = G1 + v_s*S, to p's slot (roots are never read).
    // Every later read of element q of this row is by the same lane (q =
    // lane + 64k), so per-thread program order makes it visible: no fence.
    if (pslot != 0xffffu) {
      double* __restrict__ orow = slab + (size_t)pslot * NLy;
#pragma unroll
      for (int k = 0; k < MAXK; ++k) {
        const int q = lane + 64 * k;
        if (q < NLy) orow[q] = R[q] + xwg * S[k];
      }
    }
    wave_sync();
    STAMP(5);
  }
#ifdef SK_STAMPS
  if (lane == 0 && P.stamps) {
    for (int i = 0; i < 6; ++i) atomicAdd(&P.stamps[i], tacc[i]);
    atomicAdd(&P.stamps[6], (unsigned long long)nlx);
    atomicAdd(&P.stamps[7], 1ull);
  }
#endif
  // wave reduction of the K partial sums (fixed order -> deterministic)
  for (int off = 32; off > 0; off >>= 1) kacc += __shfl_xor(kacc, off, 64);
  return kacc;
}

template <int MAXK>
__global__ void __launch_bounds__(512) sk_dag_stem_kernel(StemLaunch P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const DevSet& s = P.yset;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nwaves = blockDim.x >> 6;
  const int maxnl = P.lds_max_nl;

  // LDS carve (every region a multiple of 16 bytes)
  double* co = reinterpret_cast<double*>(smem);             // 256
  double* gp = co + 256;                                     // n_gpow_pad
  double* yP = gp + P.n_gpow_pad;                            // maxnl
  double* Rall = yP + maxnl;                                 // nwaves*maxnl
  double* yew = Rall + (size_t)nwaves * maxnl;               // lds_max_edges
  uint2* yed = reinterpret_cast<uint2*>(yew + P.lds_max_edges);  // lds_max_edges
  uint32_t* yb = reinterpret_cast<uint32_t*>(yed + P.lds_max_edges);
  uint32_t* yc = yb + maxnl;
  float* yw = reinterpret_cast<float*>(yc + maxnl);
  float* ynbp = yw + maxnl;
  uint32_t* ybc = reinterpret_cast<uint32_t*>(ynbp + maxnl);  // lds_max_bpf
  float* ybp = reinterpret_cast<float*>(ybc + P.lds_max_bpf);
  int32_t* ylv = reinterpret_cast<int32_t*>(ybp + P.lds_max_bpf);  // lds_max_nlev_pad
  int32_t* ylve = ylv + P.lds_max_nlev_pad;                   // lds_max_nlev_pad
  int32_t* ctl = ylve + P.lds_max_nlev_pad;                   // 4 ints

  for (int k = threadIdx.x; k < 256; k += blockDim.x) co[k] = P.co_subst[k];
  for (int k = threadIdx.x; k < P.n_gpow; k += blockDim.x) gp[k] = P.gpow[k];

  double* R = Rall + (size_t)wave * maxnl;
  double* slab = P.scratch + (size_t)(blockIdx.x * nwaves + wave) * P.slab_doubles;
  const double gap2 = P.gap2;

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
    const int nb = s.ex_node_base[y], eb = s.ex_edge_base[y], bb = s.ex_bpf_base[y];
    {
      const int ne = s.ex_edge_base[y + 1] - eb, nbf = s.ex_bpf_base[y + 1] - bb;
      const int lb = s.ex_lvl_base[y];
      for (int k = threadIdx.x; k < Y.nl; k += blockDim.x) {
        yb[k] = s.nd_b[nb + k];
        yc[k] = s.nd_c[nb + k];
        yw[k] = s.nd_w[nb + k];
        ynbp[k] = s.nd_nbp[nb + k];
        yP[k] = s.nd_P[nb + k];
      }
      for (int k = threadIdx.x; k < ne; k += blockDim.x) {
        const uint2 rec = s.ed[eb + k];
        yed[k] = rec;
        // IY weight of the edge: node gap score of the parent * g^gaps (the
        // reference multiplies G1[child]*v_s*e_s, stem_kernel.cpp:96-102)
        yew[k] = gap2 * (double)s.nd_w[nb + rec.y] * gp[rec.x >> 16];
      }
      for (int k = threadIdx.x; k < nbf; k += blockDim.x) {
        ybc[k] = s.bpf_code[bb + k];
        ybp[k] = s.bpf_p[bb + k];
      }
      for (int k = threadIdx.x; k <= Y.nlev; k += blockDim.x) {
        const int q = s.lvl[lb + k];
        ylv[k] = q;
        // first edge of level k (levels are contiguous node and edge ranges)
        ylve[k] = q < Y.nl ? (int)(s.nd_a[nb + q] & 0xffff) : ne;
      }
    }
    Y.b = yb; Y.c = yc; Y.w = yw; Y.nbp = ynbp; Y.P = yP;
    Y.ed = yed; Y.bc = ybc; Y.bp = ybp; Y.lv = ylv; Y.lve = ylve;
    uint32_t qe[MAXK], ql[MAXK / 2];
#pragma unroll
    for (int k = 0; k < MAXK / 2; ++k) ql[k] = 0;
#pragma unroll
    for (int k = 0; k < MAXK; ++k) {
      const int q = lane + 64 * k;
      qe[k] = q < Y.nl ? s.nd_a[nb + q] : 0xffffffffu;
      if (q < Y.nl) ql[k >> 1] |= (s.nd_b[nb + q] & 0xffffu) << (16 * (k & 1));
    }
    __syncthreads();

    // static round-robin of the item's pairs over the waves (uniform loop)
    for (int t = wave_u; t < item.z; t += nwaves) {
      const int x = P.xs[item.y + t];
      const double k = stem_pair<MAXK>(P, Y, qe, ql, R, yew, co, gp, slab, x, lane);
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
  b += (size_t)nwaves * P.lds_max_nl * 8;          // one row per wave
  b += (size_t)P.lds_max_edges * 16;               // yew + yed
  b += (size_t)P.lds_max_nl * 16;                  // yb,yc,yw,ynbp
  b += (size_t)P.lds_max_bpf * 8;
  b += (size_t)P.lds_max_nlev_pad * 8;
  b += 16;
  return b;
}

static const void* stem_kernel_ptr(int maxk) {
  switch (maxk) {
    case 8: return reinterpret_cast<const void*>(sk_dag_stem_kernel<8>);
    case 16: return reinterpret_cast<const void*>(sk_dag_stem_kernel<16>);
    case 24: return reinterpret_cast<const void*>(sk_dag_stem_kernel<24>);
    default: return reinterpret_cast<const void*>(sk_dag_stem_kernel<32>);
  }
}

int stem_maxk(int max_nl) {
  const int k = (max_nl + 63) / 64;
  if (k <= 8) return 8;
  if (k <= 16) return 16;
  if (k <= 24) return 24;
  if (k <= 32) return 32;
  return -1;
}

hipError_t launch_stem(const StemLaunch& P, int grid, int nwaves, hipStream_t st) {
  const size_t lds = stem_lds_bytes(P, nwaves);
  const int maxk = stem_maxk(P.lds_max_nl);
  const void* fn = stem_kernel_ptr(maxk);
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  switch (maxk) {
    case 8: hipLaunchKernelGGL(sk_dag_stem_kernel<8>, dim3(grid), dim3(64 * nwaves), lds, st, P); break;
    case 16: hipLaunchKernelGGL(sk_dag_stem_kernel<16>, dim3(grid), dim3(64 * nwaves), lds, st, P); break;
    case 24: hipLaunchKernelGGL(sk_dag_stem_kernel<24>, dim3(grid), dim3(64 * nwaves), lds, st, P); break;
    default: hipLaunchKernelGGL(sk_dag_stem_kernel<32>, dim3(grid), dim3(64 * nwaves), lds, st, P); break;
  }
  return hipGetLastError();
}

hipError_t stem_kernel_attr(int max_nl, int* max_dyn_lds, int* vgprs) {
  hipFuncAttributes attr;
  const int maxk = stem_maxk(max_nl);
  if (maxk < 0) return hipErrorInvalidValue;
  hipError_t e = hipFuncGetAttributes(&attr, stem_kernel_ptr(maxk));
  if (e != hipSuccess) return e;
  *max_dyn_lds = 163840 - (int)attr.sharedSizeBytes;
  *vgprs = attr.numRegs;
  return hipSuccess;
}

}  // namespace sk
