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

#include <algorithm>

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
// LDS (address space 3) pointer types: every access below is a ds_* op,
// whatever the register allocator does with the view structs.
typedef __attribute__((address_space(3))) double lds_f64;
typedef __attribute__((address_space(3))) float lds_f32;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) int32_t lds_i32;

struct YView {  // the y example staged in LDS
  const lds_u32* b;   // len:16 | bpf_beg:16
  const lds_u32* c;   // loop gaps
  const lds_f32* w;
  const lds_f32* nbp;
  const lds_f64* P;
  const lds_u32* ed;  // child:11 | parent:11 | gaps:10
  const lds_u32* bc;
  const lds_f32* bp;
  const lds_i32* lv;   // level -> first node
  const lds_i32* lve;  // level -> first edge
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
__device__ __forceinline__ double match_node_score(const lds_f64* co, const DevSet& s, int xbb,
                                                int xb0, int xnb, const YView& Y, int yb0, int ynb,
                                                double xwg, double ywg, double x_nbp, double y_nbp,
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
// Rows p of G0 (x non-leaf nodes) are produced in the reference's post-order,
// each into a recycled HBM row slot (0xffff = never read, not stored).  Lane
// l owns the y nodes q = l + 64k, k < kused = ceil(|Vy|/64) (wave-uniform);
// rows are padded to a multiple of 64 in LDS and in the slab, so the per-k
// loops need no lane predicates (padded q are masked by selects only where
// they could reach a valid value).
//
// Both x-child sums of the reference are linear in the child rows, so one
// weighted row suffices:   S[q] = sum_{c in ch(p)} g^gaps(p,c) * G0[c][q]
//   IX term   : sum_c G0[c][q] * v_s(p) * g^gaps = v_s(p) * S[q]
//   MATCH sum : sum_c sum_cy g^gx g^gy G0[c][cy] = sum_{cy in ch(q)} g^gy S[cy]
// For a stem row p:
//   A. stream the child rows from HBM (coalesced) into S (registers);
//      S -> per-wave LDS row R; H[k] = sum_{cy in ch(q)} g^gy R[cy] (band);
//   B. M[q] = node_score(p,q) * H (closed forms for loop nodes) -> R (G1);
//      K += P_x[p] * sum_q M[q] P_y[q];
//   C. IY sweep over the y levels, edge-parallel: G1[q] += G1[cy]*w(q,cy)
//      with w = gap^2*w_y(q)*g^gaps precomputed per item (LDS f64 atomics);
//   D. G0[p][q] = G1[q] + v_s(p)*S[k] -> slot of p.
template <int MAXK>
__device__ double stem_pair(const StemLaunch& P, const YView& Y, lds_f64* R,
                            const lds_f64* co, const lds_f64* gp, const lds_u32* ya,
                            double* __restrict__ slab, int x, int lane, int kused, int stride) {
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
  const XRow* __restrict__ xrows = s.xrow + xnb;
  const double* __restrict__ xsl = P.pn.xr_SL + xnb;
  const uint32_t* __restrict__ xch = s.xr_ch;
  double kacc = 0.0;
#ifdef SK_STAMPS
  unsigned long long tacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tlast = __builtin_amdgcn_s_memtime();
#endif

  // x-row header and first child records, prefetched one row ahead
  XRow nx = xrows[0];
  double nSL = xsl[0];
  uint32_t nch[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) nch[j] = xch[chp + j];

  for (int r = 0; r < nlx; ++r) {
    const uint32_t xa = nx.a, xb = nx.b, xc = nx.c;
    const double xwg = gap2 * (double)nx.w;
    const double x_nbp = (double)nx.nbp;
    const double xP = nx.P, xSL = nSL, xpf = (double)nx.bp0;
    uint32_t ch[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) ch[j] = nch[j];
    const int xne = xa & 0xff, xnbf = (xa >> 8) & 0xff;
    const int chp_r = chp;
    chp += xne;
    if (r + 1 < nlx) {
      nx = xrows[r + 1];
      nSL = xsl[r + 1];
#pragma unroll
      for (int j = 0; j < 4; ++j) nch[j] = xch[chp + j];
    }
    const int xlen = xb & 0xffff;
    const uint32_t pslot = xb >> 16;
    const int xb0 = xc & 0xffff;
    const bool xloop = xne == 0;
    const double xeg0 = gp[xa >> 16];
    // single bp-frequency entry of x (the common single-sequence case)
    const bool x_one = xnbf == 1 && x_nbp == 0.0;
    const uint32_t xcode = (xc >> 16) * 16u;
    STAMP(0);

    // ---- A: S = sum_c g^gaps G0[c][*]  (coalesced HBM row streams)
    double S[MAXK];
#pragma unroll
    for (int k = 0; k < MAXK; ++k) S[k] = 0.0;
    for (int t = 0; t < xne; t += 2) {
      const uint32_t c0 = t < 4 ? ch[t] : xch[chp_r + t];
      const bool two = t + 1 < xne;
      const uint32_t c1 = two ? (t + 1 < 4 ? ch[t + 1] : xch[chp_r + t + 1]) : c0;
      const double eg0 = gp[c0 >> 16], eg1 = two ? gp[c1 >> 16] : 0.0;
      const double* __restrict__ r0 = slab + (size_t)(c0 & 0xffff) * stride + lane;
      const double* __restrict__ r1 = slab + (size_t)(c1 & 0xffff) * stride + lane;
#pragma unroll
      for (int k = 0; k < MAXK; ++k)
        if (k < kused) S[k] += eg0 * r0[64 * k] + eg1 * r1[64 * k];
    }
    STAMP(1);
    double H[MAXK];
#pragma unroll
    for (int k = 0; k < MAXK; ++k) H[k] = 0.0;
    if (!xloop) {
#pragma unroll
      for (int k = 0; k < MAXK; ++k)
        if (k < kused) R[lane + 64 * k] = S[k];
      wave_sync();
      // MATCH sums over y-children: up to 4 edges per node in one pass with
      // selects (reads past a node's edges stay inside the padded edge
      // array), longer edge lists after it
      bool more = false;
#pragma unroll
      for (int k = 0; k < MAXK; ++k) {
        if (k < kused) {
          const uint32_t a = ya[lane + 64 * k];
          const int e0 = a & 0xffff, ne = (a >> 16) & 0xff;
          double acc = 0.0;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const uint32_t f = Y.ed[e0 + j];
            const double v = gp[f >> 22] * R[f & 0x7ff];
            acc += j < ne ? v : 0.0;
          }
          H[k] = acc;
          more |= ne > 4;
        }
      }
      if (__any(more)) {
#pragma unroll
        for (int k = 0; k < MAXK; ++k) {
          if (k < kused) {
            const uint32_t a = ya[lane + 64 * k];
            const int e0 = a & 0xffff, ne = (a >> 16) & 0xff;
            double acc = H[k];
            for (int j = 4; j < ne; ++j) {
              const uint32_t f = Y.ed[e0 + j];
              acc += gp[f >> 22] * R[f & 0x7ff];
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
      if (k < kused) {
        const int q = lane + 64 * k;
        const uint32_t bq = Y.b[q];
        const int dl = xlen - (int)(bq & 0xffff);
        const bool inb = q < NLy && (band == 0 || (dl < 0 ? -dl : dl) <= band);
        const double egy = gp[Y.c[q]];
        const double Hq = q < nloop_y ? (xloop ? xeg0 : xSL) * egy : H[k];
        const uint32_t a = ya[q];
        const float ynbp = Y.nbp[q];
        double vs = co[xcode + Y.bc[bq >> 16]] * xpf * (double)Y.bp[bq >> 16];
        const bool fast = x_one && (a >> 24) == 1u && ynbp == 0.0f;
        if (!fast && inb && Hq != 0.0) {
          // general bp-frequency lists / gap columns (score_table.cpp:343-380)
          const double ywg = gap2 * (double)Y.w[q];
          vs = match_node_score(co, s, xbb, xb0, xnbf, Y, bq >> 16, a >> 24, xwg, ywg, x_nbp,
                                (double)ynbp, x_nseq);
        }
        const double M = inb ? vs * Hq : 0.0;
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
      // IY weight of an edge: node gap score of the parent * g^gaps (the
      // reference multiplies G1[child]*v_s*e_s, stem_kernel.cpp:96-102)
      int fa = Y.lve[1], fb = Y.lve[2];
      int fc = Y.lve[Y.nlev > 2 ? 3 : 2];
      uint32_t rec = 0;
      double w = 0.0;
      if (fa + lane < fb) {
        rec = Y.ed[fa + lane];
        w = gap2 * (double)Y.w[(rec >> 11) & 0x7ff] * gp[rec >> 22];
      }
      for (int l = 1; l < Y.nlev; ++l) {
        // next level [fb, fc); level after next ends at fd
        const int fd = (l + 3 <= Y.nlev) ? Y.lve[l + 3] : fc;
        uint32_t rec2 = 0;
        double w2 = 0.0;
        if (fb + lane < fc) {
          rec2 = Y.ed[fb + lane];
          w2 = gap2 * (double)Y.w[(rec2 >> 11) & 0x7ff] * gp[rec2 >> 22];
        }
        if (fa + lane < fb)
          __hip_atomic_fetch_add(&R[(rec >> 11) & 0x7ff], R[rec & 0x7ff] * w, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WAVEFRONT);
        for (int f = fa + 64 + lane; f < fb; f += 64) {  // levels with > 64 edges
          const uint32_t rr = Y.ed[f];
          const double wr = gap2 * (double)Y.w[(rr >> 11) & 0x7ff] * gp[rr >> 22];
          __hip_atomic_fetch_add(&R[(rr >> 11) & 0x7ff], R[rr & 0x7ff] * wr, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WAVEFRONT);
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
      double* __restrict__ orow = slab + (size_t)pslot * stride + lane;
#pragma unroll
      for (int k = 0; k < MAXK; ++k)
        if (k < kused) orow[64 * k] = R[lane + 64 * k] + xwg * S[k];
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

// Workgroup size bound per register template: MAXK <= 16 keeps <= 168 VGPRs,
// so 12 waves (3 per SIMD) fit; the wider templates need up to 256.
template <int MAXK>
struct StemWaves {
  static constexpr int value = MAXK <= 16 ? 12 : 8;
};

template <int MAXK>
__global__ void __launch_bounds__(64 * StemWaves<MAXK>::value) sk_dag_stem_kernel(StemLaunch P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const DevSet& s = P.yset;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nwaves = blockDim.x >> 6;
  const int maxnl = P.lds_max_nl;  // multiple of 64

  // LDS carve (every region a multiple of 16 bytes)
  lds_f64* co = (lds_f64*)(smem);                             // 256
  lds_f64* gp = co + 256;                                     // n_gpow_pad
  lds_f64* yP = gp + P.n_gpow_pad;                            // maxnl
  lds_f64* Rall = yP + maxnl;                                 // nwaves*maxnl
  lds_u32* yed = (lds_u32*)(Rall + (size_t)nwaves * maxnl);   // lds_max_edges (mult. of 4)
  lds_u32* ya = yed + P.lds_max_edges;                        // maxnl
  lds_u32* yb = ya + maxnl;
  lds_u32* yc = yb + maxnl;
  lds_f32* yw = (lds_f32*)(yc + maxnl);
  lds_f32* ynbp = yw + maxnl;
  lds_u32* ybc = (lds_u32*)(ynbp + maxnl);                    // lds_max_bpf
  lds_f32* ybp = (lds_f32*)(ybc + P.lds_max_bpf);
  lds_i32* ylv = (lds_i32*)(ybp + P.lds_max_bpf);             // lds_max_nlev_pad
  lds_i32* ylve = ylv + P.lds_max_nlev_pad;                   // lds_max_nlev_pad
  lds_i32* ctl = ylve + P.lds_max_nlev_pad;                   // 4 ints

  for (int k = threadIdx.x; k < 256; k += blockDim.x) co[k] = P.co_subst[k];
  for (int k = threadIdx.x; k < P.n_gpow; k += blockDim.x) gp[k] = P.gpow[k];

  lds_f64* R = Rall + (size_t)wave * maxnl;
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
    const int kused = (Y.nl + 63) >> 6;
    const int stride = kused * 64;
    {
      const int ne = s.ex_edge_base[y + 1] - eb, nbf = s.ex_bpf_base[y + 1] - bb;
      const int lb = s.ex_lvl_base[y];
      // node fields, zero padded to a multiple of 64 (padded q: no edges)
      for (int k = threadIdx.x; k < stride; k += blockDim.x) {
        const bool v = k < Y.nl;
        ya[k] = v ? s.nd_a[nb + k] : 0u;
        yb[k] = v ? s.nd_b[nb + k] : 0u;
        yc[k] = v ? s.nd_c[nb + k] : 0u;
        yw[k] = v ? s.nd_w[nb + k] : 0.0f;
        ynbp[k] = v ? s.nd_nbp[nb + k] : 0.0f;
        yP[k] = v ? s.nd_P[nb + k] : 0.0;
      }
      // edges (+4 padding records: the predicated gather reads past the end)
      for (int k = threadIdx.x; k < ne + 4; k += blockDim.x) {
        if (k < ne) {
          const uint2 rec = s.ed[eb + k];  // {child | gaps<<16, parent}
          yed[k] = (rec.x & 0x7ffu) | ((rec.y & 0x7ffu) << 11) | ((rec.x >> 16) << 22);
        } else {
          yed[k] = 0u;
        }
      }
      for (int k = threadIdx.x; k < nbf + 1; k += blockDim.x) {
        ybc[k] = k < nbf ? s.bpf_code[bb + k] : 0u;
        ybp[k] = k < nbf ? s.bpf_p[bb + k] : 0.0f;
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
    __syncthreads();

    // static round-robin of the item's pairs over the waves (uniform loop)
    for (int t = wave_u; t < item.z; t += nwaves) {
      const int x = P.xs[item.y + t];
      const double k = stem_pair<MAXK>(P, Y, R, co, gp, ya, slab, x, lane, kused, stride);
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
  b += (size_t)P.lds_max_edges * 4;                // packed edges
  b += (size_t)P.lds_max_nl * 20;                  // ya,yb,yc,yw,ynbp
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

hipError_t stem_kernel_attr(int max_nl, int* max_dyn_lds, int* vgprs, int* max_waves) {
  hipFuncAttributes attr;
  const int maxk = stem_maxk(max_nl);
  if (maxk < 0) return hipErrorInvalidValue;
  hipError_t e = hipFuncGetAttributes(&attr, stem_kernel_ptr(maxk));
  if (e != hipSuccess) return e;
  *max_dyn_lds = 163840 - (int)attr.sharedSizeBytes;
  *vgprs = attr.numRegs;
  *max_waves = std::max(1, attr.maxThreadsPerBlock / 64);
  return hipSuccess;
}

}  // namespace sk
