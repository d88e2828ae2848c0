// DAG stem-kernel DP on CDNA4 (gfx950).
//
// Reference: StemKernel<ST,MData>::operator()  stem_kernel_lite/stem_kernel.cpp:14-95
// with SubstNodeScore / SimpleNodeScore / SimpleEdgeScore  score_table.cpp:14-201.
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
  // child-edge weights of both x schedules
  {
    int k = s.ex_xch_base[e];
    for (int r = 0; r < nl; ++r) {
      const int ne = s.xrow[nb + r].a & 0xff;
      for (int t = 0; t < ne; ++t, ++k) pn.xr_chw[k] = gpow[s.xr_ch[k] >> 16];
    }
  }
  if (s.n_gam > 0) {
    const int gb = s.ex_xg_base[e], nlg = s.ex_nlxg[e];
    int k = s.ex_xgch_base[e];
    int pk = s.n_phi > 0 ? s.ex_phk_base[e] : 0;
    for (int r = 0; r < nlg; ++r) {
      const double SLr = pn.nd_SL[nb + s.xg_node[gb + r]];
      pn.xg_SL[gb + r] = SLr;
      const XRow xr = s.xgrow[gb + r];
      const int ne = xr.a & 0xff;
      for (int t = 0; t < ne; ++t, ++k) {
        // the record's weight recipe (device_set.h)
        const uint32_t c = s.xg_ch[k];
        const double wc = gpow[c >> 16] * gpow[s.xg_clg[k]] * (double)s.xg_cpf[k];
        double w;
        switch (s.xg_cty[k]) {
          case 0: w = gpow[c >> 16]; break;
          case 1: w = wc; break;
          case 2: w = (double)xr.bp0 * wc; break;
          case 3: w = (double)xr.bp0 * SLr; break;
          default: w = gap2 * (double)xr.w * wc; break;
        }
        pn.xg_chw[k] = w;
        if (s.xg_cty[k] == 2) pn.phk_w[pk++] = xr.P * w;
      }
    }
    double* h = pn.gam_h + (int64_t)e * s.n_gam;
    for (int g = 0; g < s.n_gam; ++g) h[g] = 0.0;
    for (int i = s.ex_gr_base[e]; i < s.ex_gr_base[e + 1]; ++i) {
      const uint32_t inf = s.gr_info[i];
      h[inf & 0xffff] += s.gr_P[i] * (gpow[inf >> 16] * (double)s.gr_pf[i]);
    }
    if (s.n_phi > 0)  // phi rows' Gamma_{code,len} terms: P pf xSL
      for (int i = s.ex_gra_base[e]; i < s.ex_gra_base[e + 1]; ++i) {
        const uint32_t r = s.gra_row[i];
        h[s.gra_gidx[i]] += s.xgrow[r].P * ((double)s.xgrow[r].bp0 * pn.xg_SL[r]);
      }
  }
}

// ---------------------------------------------------------------------------
// LDS (address space 3) pointer types: every access below is a ds_* op,
// whatever the register allocator does with the view structs.
typedef __attribute__((address_space(3))) double lds_f64;
typedef __attribute__((address_space(3))) float lds_f32;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) int32_t lds_i32;

// One y node record (16 B, one global_load_dwordx4):
//   a = first edge in the node-major edge array:16 | n_edges:8 | n_bpf:8
//   c = loop leaf-edge gaps:16 | code of the first bp-freq entry:4 @16 |
//       single-entry flag @24 (one bp-freq entry and no gap column)
//   w = node weight, p0 = probability of the first bp-freq entry (float bits)
struct YView {  // the y example (staged in LDS unless noted)
  const uint4* __restrict__ nrg;  // node records {a, c, w, p0} (HBM, L2-resident)
  const lds_u32* sc;   // sweep schedule: (nch + 2) chunks of 64 child:11 | parent:11 | gaps:10
  const lds_f64* ew;   // their weights gap^2 w(parent) g^gaps (0 for dummies), or
                       // (node_weights<MAXK>) per node gap^2 w(q), or
  const lds_f32* ewf;  // (node_weights_f32<MAXK>) per node w(q): gap^2 w(q) g^gaps in the sweep
  const lds_f64* gp;   // g^k
  double gap2;
  const lds_u32* ed2;  // edges node-major (sorted ids)
  const uint32_t* __restrict__ ed2g;  // the same in HBM (L2-resident; edges_global<MAXK>)
  const lds_i32* lfirst;  // length v -> first node (nodes sorted by length), v <= lmax+1
  const lds_i32* ycs;     // length v -> first sweep chunk reaching v, v <= lmax+1
  int lmax;               // largest node length of the example
  int nl, nch;
  float nseqs;
  int nb, bb;             // node / bp-freq base of the example in the y set (HBM)
};

// read-only global data through the constant address space (scalar loads)
#if defined(__HIP_DEVICE_COMPILE__)
template <typename T>
using cst_ptr = const __attribute__((address_space(4))) T*;
#else
template <typename T>
using cst_ptr = const T*;
#endif

__device__ __forceinline__ void wave_sync() {
  // LDS traffic of one wave is processed in issue order; this pins the
  // compiler's instruction order and waits for outstanding LDS operations.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// scheduling fence: keeps the compiler from hoisting every slot's memory ops
// to the top of a phase (which would exceed the register budget)
#define SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
// waves per workgroup of the MAXK 16 / 20 classes (8: two prefetched rows; 12: one)
#ifndef SK_W20
#define SK_W20 8
#endif
#ifndef SK_W16  // waves per workgroup of the MAXK 16 class
#define SK_W16 8
#endif
#ifndef SK_NPF12  // rows prefetched per row in the MAXK <= 12 classes
#define SK_NPF12 2
#endif
#ifndef SK_NPF20  // rows prefetched per row in the MAXK 20 class (8 waves)
#define SK_NPF20 2
#endif
#ifndef SK_NPF16  // rows prefetched per row in the MAXK 16 class
#define SK_NPF16 1
#endif
#ifndef SK_NPF17  // ... in the MAXK 17 class: none (with one, the row loop spilled; r06h: +2.5 % without)
#define SK_NPF17 0
#endif
#ifndef SK_PW  // MATCH pass width in 64-node groups
#define SK_PW 3  // NS 193.7k against 192.2k pairs/s with 4 (r03, same box)
#endif
#ifndef SK_SEGSUM  // MATCH: same-parent runs summed per quad before the atomic (0 = off)
#define SK_SEGSUM 1
#endif
#ifndef SK_SEGSUM_MAXK  // the widest class that sums runs per quad
#define SK_SEGSUM_MAXK 20
#endif
#ifndef SK_MU  // MATCH edge rounds: 64-edge groups whose reads are issued together
#define SK_MU 3
#endif
#ifndef SK_NODEW_MIN  // the narrowest class whose sweep weights are per node (LDS for waves)
#define SK_NODEW_MIN 20
#endif
// The MAXK 16 class: 1 = 12 waves (3 per SIMD at 168 VGPRs: phases A / D in
// halves, 128-node MATCH passes, per-node sweep weights; r06: 32 scratch
// bytes, item-loop values reloaded per work item, none in the row loop),
// NS 198.1k against 190.5k pairs/s with 0 (8 waves, one prefetched child row,
// 196 VGPRs) over two alternating rounds (r04c); 2 = 1 without the
// prefetched row (no spills): 196.0k.
#ifndef SK_M16
#define SK_M16 1
#endif
// The MAXK 17 class (y of 1,025-1,088 non-leaf nodes: a third of the NS
// set, L = 200) runs the 12-wave layout of MAXK 16 instead of the 8-wave
// MAXK 20 class (SK_K17 = 0: no such class)
#ifndef SK_K17
#define SK_K17 1
#endif
template <int MAXK>
constexpr bool m16_wide() {
  return (MAXK == 16 || MAXK == 17) && SK_M16 != 0;
}
// Sweep weights per y node (gap^2 w(q), 8 B per node; the widest classes
// w(q) itself, the float, 4 B) instead of per schedule slot (8 B per slot of
// (nch + 2) x 64): a third of the schedule's LDS, for one more LDS read per
// slot (g^gaps) and the product(s) the staging formed (same operands, same
// order: the same double).  The wide classes are LDS-bound in
// waves per CU (C5's MAXK 24: 5 waves with slot weights, 7 without), so they
// trade; MAXK 16 holds 8 waves either way (VGPRs).
template <int MAXK>
constexpr bool node_weights() {
  return MAXK >= SK_NODEW_MIN || m16_wide<MAXK>();
}
#ifndef SK_NODEF_MIN  // the narrowest class whose node weights are the floats w(q)
#define SK_NODEF_MIN 24
#endif
template <int MAXK>
constexpr bool node_weights_f32() {
  return node_weights<MAXK>() && MAXK >= SK_NODEF_MIN;
}
#ifndef SK_PW2_MIN  // the narrowest class whose MATCH passes are 128 nodes (LDS for waves)
#define SK_PW2_MIN 24
#endif
// MATCH pass width in 64-node groups: SK_PW, 2 in the widest classes (the
// per-wave accumulator is 64 * PW doubles of LDS)
template <int MAXK>
#ifndef SK_PW17  // MATCH pass width of the MAXK 17 class
#define SK_PW17 2
#endif
constexpr int pass_width() {
  return MAXK == 17 ? SK_PW17 : (MAXK >= SK_PW2_MIN || m16_wide<MAXK>()) ? 2 : SK_PW;
}
// host mirror of pass_width (stem_lds_bytes)
static inline bool m16_wide_of(int maxk) { return (maxk == 16 || maxk == 17) && SK_M16 != 0; }
static inline int pass_width_of(int maxk) {
  return maxk == 17 ? SK_PW17 : (maxk >= SK_PW2_MIN || m16_wide_of(maxk)) ? 2 : SK_PW;
}
static inline bool node_weights_of(int maxk) { return maxk >= SK_NODEW_MIN || m16_wide_of(maxk); }
#ifndef SK_EDG_MIN  // the narrowest class whose MATCH reads the node-major edges from L2, not LDS
#define SK_EDG_MIN 64  // off: C5 100.7k against 102.3k pairs/s (r03 A/B; MATCH 14.4k against 9.9k cycles per row)
#endif
// The node-major edges (4 B per edge) read by MATCH from HBM / L2 instead of
// LDS: one more wave per CU in the widest classes, for an L2 round trip per
// MATCH round (issued a round ahead).
template <int MAXK>
constexpr bool edges_global() {
  return MAXK >= SK_EDG_MIN;
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

// node_score(xx,yy,i,j): score_table.cpp:162-201 (Subst) / 193-232 (Simple);
// co[] holds exp(beta*ribosum) or the match/mismatch table.
// General case (several bp-freq entries or gap columns; rare): the y
// entries are read from HBM.
__device__ __forceinline__ double match_node_score(const lds_f64* co, const DevSet& s, int xbb,
                                                int xb0, int xnb, const DevSet& ys, const YView& Y,
                                                int yb0, int ynb, double xwg, double ywg,
                                                double x_nbp, double y_nbp, double x_nseq) {
  double v = 0.0;
  for (int a = 0; a < xnb; ++a) {
    const double cx = (double)s.bpf_p[xbb + xb0 + a];
    const uint32_t ca = s.bpf_code[xbb + xb0 + a] * 16u;
    for (int b = 0; b < ynb; ++b) {
      const double cy = (double)ys.bpf_p[Y.bb + yb0 + b];
      v += co[ca + ys.bpf_code[Y.bb + yb0 + b]] * cx * cy;
    }
  }
  v += ywg * x_nbp / x_nseq;
  v += xwg * y_nbp / (double)Y.nseqs;
  return v;
}

// A G0 row slot as a buffer resource whose range is the y example's NLy
// valid columns: loads of the padded tail return 0 without touching memory
// (the tail is never needed).  Built from wave-uniform values only.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const double* base, int nly) {
  const uint64_t a = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  // (the record count through readfirstlane too: a value the compiler
  // cannot prove uniform turns every load through the descriptor into a
  // waterfall loop)
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                           __builtin_amdgcn_readfirstlane(nly * 8), 0x00020000);
}

// cache policy bits of the G0 row loads / stores (experiments: 2 = nt)
#ifndef SK_ROW_LD_POL
#define SK_ROW_LD_POL 0
#endif
#ifndef SK_ROW_ST_POL
#define SK_ROW_ST_POL 0
#endif
typedef unsigned int u32x2 __attribute__((__vector_size__(2 * sizeof(unsigned int))));

// element lane + 64k of a row
__device__ __forceinline__ double row_ld(__amdgpu_buffer_rsrc_t r, int lane, int k) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, lane * 8, k * 512, SK_ROW_LD_POL));
}

// S[k] += eg0 * r0[lane + 64k] + eg1 * r1[lane + 64k]: every load of both rows
// is issued before the first is consumed (one memory round trip, not one per
// slot).
// The widest classes (MAXK > SK_HALF_A) load the two rows in two halves of
// slots: half the peak registers of phase A (which otherwise holds S and
// both rows at once) for a second memory round trip.
#ifndef SK_HALF_A
#define SK_HALF_A 64  // off: C5 90.7k against 89.5k pairs/s halved (tools/ab.sh, r03l)
#endif
#ifndef SK_HALF_D  // phase D likewise
#define SK_HALF_D 64
#endif
#ifndef SK_M16_HALFA  // the 12-wave MAXK 16 class loads A in halves
#define SK_M16_HALFA 1
#endif
#ifndef SK_M16_HALFD  // ... and reads D's G1 in halves
#define SK_M16_HALFD 1
#endif
template <int MAXK>
__device__ __forceinline__ void add_rows2(double (&S)[MAXK], __amdgpu_buffer_rsrc_t r0,
                                          __amdgpu_buffer_rsrc_t r1, double eg0, double eg1,
                                          int lane) {
  constexpr int H = (MAXK > SK_HALF_A || (m16_wide<MAXK>() && SK_M16_HALFA)) ? (MAXK + 1) / 2 : MAXK;
#pragma unroll
  for (int h0 = 0; h0 < MAXK; h0 += H) {
    double a[H], b[H];
#pragma unroll
    for (int k = 0; k < H; ++k) {
      a[k] = h0 + k < MAXK ? row_ld(r0, lane, h0 + k) : 0.0;
      b[k] = h0 + k < MAXK ? row_ld(r1, lane, h0 + k) : 0.0;
    }
    SCHED_FENCE();
#pragma unroll
    for (int k = 0; k < H; ++k)
      if (h0 + k < MAXK) S[h0 + k] += eg0 * a[k] + eg1 * b[k];
  }
}

// One (x,y) pair on one wavefront.
//
// Rows p of G0 (x non-leaf nodes) are produced in the reference's post-order,
// each into a recycled HBM row slot (0xffff = never read, not stored).  Lane
// l owns the y nodes q = l + 64k, k < MAXK (the launch's register class: the
// y example has at most 64*MAXK non-leaf nodes).  LDS node data and the slab
// rows are padded to 64*MAXK, and every per-slot loop is straight-line code
// (no branches on k or on the lane), so the compiler can overlap the memory
// round trips of all slots; padded nodes are masked by selects.
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
//      with w = gap^2*w_y(q)*g^gaps (LDS f64 atomics);
//   D. G0[p][q] = G1[q] + v_s(p)*S[k] -> slot of p.
// ---- C of a row (and the Gamma rows of an item): the IY recurrence
// G1[q] += w(q,cy) G1[cy], w = gap^2 w_y(q) g^gaps, over the y example's
// sweep schedule from chunk c0: chunks of 64 edges, each placed after every
// edge of its children (host list schedule).  A chunk's R reads are issued
// after the previous chunk's atomics and a wave's LDS ops execute in issue
// order, so nothing drains between chunks: only the data a lane consumes is
// waited for.  Records are read two chunks ahead, weights one; dummy records
// (weight 0) pad the chunks.  Ends with a wave barrier.
template <bool NW, bool NWF>
__device__ __forceinline__ void iy_sweep(const YView& Y, lds_f64* R, int c0, int lane) {
  const lds_u32* rp = Y.sc + c0 * 64 + lane;
  const lds_f64* wp = Y.ew + (NW ? 0 : c0 * 64 + lane);
  // NW: the slot's weight from its parent's node weight and g^gaps.  A
  // dummy record reads and writes a free slot past the y's nodes (the
  // staging's choice, by lane; the classes keep one slot free at least): its
  // R entry and node weight are 0, so it adds 0 * 0 -- no select needed
  auto nweight = [&](uint32_t rec) __attribute__((always_inline)) -> double {
    const uint32_t pa = (rec >> 11) & 0x7ff;
    return (NWF ? Y.gap2 * (double)Y.ewf[pa] : Y.ew[pa]) * Y.gp[rec >> 22];
  };
  // three chunk slots in rotation (the loop is unrolled by three, so no
  // loaded register is ever copied, which would force a wait for it)
  struct Ck {
    uint32_t rec;
    double w, rv;
  };
  Ck A, B, C;
  A.rec = rp[0];
  B.rec = rp[64];
  A.w = NW ? nweight(A.rec) : wp[0];
  B.w = 0.0;
  C.rec = 0u;
  C.w = C.rv = B.rv = 0.0;
  A.rv = R[A.rec & 0x7ff];
  int c = c0;
  const int nch = Y.nch;
  // chunk X now, Y next, Z after: false after the last chunk; each chunk's
  // R reads after the previous chunk's atomics
  auto step = [&](Ck& X, Ck& Yc, Ck& Z) __attribute__((always_inline)) -> bool {
    Z.rec = rp[128];
    Yc.w = NW ? nweight(Yc.rec) : wp[64];
    __hip_atomic_fetch_add(&R[(X.rec >> 11) & 0x7ff], X.rv * X.w, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WAVEFRONT);
    Yc.rv = R[Yc.rec & 0x7ff];
    rp += 64;
    wp += 64;
    return ++c < nch;
  };
  for (;;) {
    if (!step(A, B, C)) break;
    if (!step(B, C, A)) break;
    if (!step(C, A, B)) break;
  }
  wave_sync();
}

// base of child row c of an x schedule: a slab slot, (bit 15) the y's Gamma
// row of a gamma child or component, or (bit 14) the y's Phi row of a phi
// component
__device__ __forceinline__ const double* child_row(uint32_t c, const double* slab, const double* gamtab,
                                                   const double* phitab, int stride) {
  const double* base = (c & 0x8000u) ? gamtab : (c & 0x4000u) ? phitab : slab;
  return base + (size_t)(c & 0x3fffu) * stride;
}

template <int MAXK>
__device__ double stem_pair(const StemLaunch& P, const YView& Y, lds_f64* R, lds_f64* hb,
                            const lds_f64* co, const lds_f64* gp, double* __restrict__ slab, int x,
                            int lane, bool gam, const double* __restrict__ gamtab,
                            const lds_f64* kap, const double* __restrict__ phitab,
                            const double* __restrict__ phikap) {
  constexpr int stride = 64 * MAXK;
  constexpr int PW = pass_width<MAXK>();
  const DevSet& s = P.xset;
  const DevSet& ys = P.yset;
  const double* __restrict__ yPg = ys.yn_P + Y.nb;  // path counts of y (HBM, L2-resident)
  const int NLy = Y.nl;
  if (s.ex_nl[x] == 0 || NLy == 0) return 0.0;
  const int xnb = s.ex_node_base[x], xbb = s.ex_bpf_base[x];
  // the x schedule: every non-leaf row, or (gamma) all but the gamma rows,
  // whose K terms come from the y's Gamma sums: sum_g h_x[g] kappa_y[g]
  const int xgb = gam ? s.ex_xg_base[x] : 0;
  const int nlx = gam ? s.ex_nlxg[x] : s.ex_nl[x];
  int chp = gam ? s.ex_xgch_base[x] : s.ex_xch_base[x];
  const double x_nseq = (double)s.ex_nseqs[x];
  const double gap2 = P.gap2;
  const int band = (int)P.band;
  const XRow* __restrict__ xrows = gam ? s.xgrow + xgb : s.xrow + xnb;
  const double* __restrict__ xsl = gam ? P.pn.xg_SL + xgb : P.pn.xr_SL + xnb;
  const uint32_t* __restrict__ xch = gam ? s.xg_ch : s.xr_ch;
  const double* __restrict__ xchw = gam ? P.pn.xg_chw : P.pn.xr_chw;
  double kacc = 0.0;
  if (gam) {
    const double* __restrict__ h = P.pn.gam_h + (int64_t)x * s.n_gam;
    for (int g = lane; g < s.n_gam; g += 64) kacc += h[g] * kap[g];
    if (P.phi_on)  // phi rows' Phi components: sum P_p w kappa_Phi
      for (int j = s.ex_phk_base[x] + lane; j < s.ex_phk_base[x + 1]; j += 64)
        kacc += P.pn.phk_w[j] * phikap[s.phk_idx[j]];
  }
  if (nlx == 0) {
    for (int off = 32; off > 0; off >>= 1) kacc += __shfl_xor(kacc, off, 64);
    return kacc;
  }
#ifdef SK_STAMPS
  unsigned long long tacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long cnt[4] = {0, 0, 0, 0};  // A-loaded rows, levels, passes, band nodes
  unsigned long long tlast = __builtin_amdgcn_s_memtime();
#endif

  // x-row header, its child-sum leaf term and its first four child records,
  // prefetched one row ahead with scalar loads (constant address space: the
  // x set is read-only here).  A vector load of these uniform values would
  // be moved to SGPRs, i.e. waited for, right away, behind the previous
  // row's stores; a scalar load is waited for at the next LDS wait, issued
  // where the next one is a phase away.
  const cst_ptr<XRow> xrows_c = (cst_ptr<XRow>)xrows;
  const cst_ptr<double> xsl_c = (cst_ptr<double>)xsl;
  const cst_ptr<uint32_t> xch_c = (cst_ptr<uint32_t>)xch;
  const cst_ptr<double> xchw_c = (cst_ptr<double>)xchw;
  XRow nx = xrows_c[0];
  double nSL = xsl_c[0];
  uint32_t nch[4];
  double ncw[4];  // their weights (g^gaps, times g^lg pf for a gamma child)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    nch[j] = xch_c[chp + j];
    ncw[j] = xchw_c[chp + j];
  }

  double S[MAXK];  // this row's weighted child sum (carried over rows)
#pragma unroll
  for (int k = 0; k < MAXK; ++k) S[k] = 0.0;
  uint32_t done = 0;  // first-four children already in S

  for (int r = 0; r < nlx; ++r) {
    const uint32_t xa = nx.a, xb = nx.b, xc = nx.c;
    const double xwg = gap2 * (double)nx.w;
    const double x_nbp = (double)nx.nbp;
    const double xP = nx.P, xSL = nSL, xpf = (double)nx.bp0;
    uint32_t ch[4];
    double cw[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      ch[j] = nch[j];
      cw[j] = ncw[j];
    }
    const int xne = xa & 0xff, xnbf = (xa >> 8) & 0xff;
    const int chp_r = chp;
    chp += xne;
    const int xlen = xb & 0xffff;
    const uint32_t pslot = xb >> 16;
    const int xb0 = xc & 0xffff;
    const bool xloop = xne == 0;
    const double xeg0 = gp[xa >> 16];
    // single bp-frequency entry of x (the common single-sequence case)
    const bool x_one = xnbf == 1 && x_nbp == 0.0;
    const uint32_t xcode = ((xc >> 16) & 0xffu) * 16u;
    // a phi (combination) row: G0 = S, the weighted sum of its component
    // rows; no MATCH, no sweep (its K terms come with the y's Phi sums)
    const bool combo = (xc >> 31) != 0u;
    // MATCH node range [qa, qb): y nodes are numbered by length, so the
    // length band [xlen-band, xlen+band] is one index range; its first
    // pass's node records are requested now, ahead of the child rows
    int qa = 0, qb = NLy;
    if (band > 0) {
      qa = Y.lfirst[min(max(xlen - band, 0), Y.lmax + 1)];
      qb = Y.lfirst[min(max(xlen + band + 1, 0), Y.lmax + 1)];
    }
    qa = __builtin_amdgcn_readfirstlane(qa);
    qb = __builtin_amdgcn_readfirstlane(qb);
    uint4 nd_first[PW];
    double Pq_first[PW];
#pragma unroll
    for (int j = 0; j < PW; ++j) {
      nd_first[j] = make_uint4(0u, 0u, 0u, 0u);
      Pq_first[j] = 0.0;
    }
    if (qa < qb) {
#pragma unroll
      for (int j = 0; j < PW; ++j) {
        const int qf = min(max(qb - 64 * PW, qa) + 64 * j + lane, qb - 1);
        nd_first[j] = Y.nrg[qf];
        Pq_first[j] = yPg[qf];
      }
    }
    STAMP(0);

    // next row's header (see above): issued ahead of A, which has no LDS
    // waits
    SCHED_FENCE();
    if (r + 1 < nlx) {
      nx = xrows_c[r + 1];
      nSL = xsl_c[r + 1];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        nch[j] = xch_c[chp + j];
        ncw[j] = xchw_c[chp + j];
      }
    }
    SCHED_FENCE();

    // ---- A: S = sum_c g^gaps G0[c][*]  (coalesced HBM row streams).
    //      S arrives partly filled: the previous row added the child rows it
    //      prefetched during its sweep and itself (a distance-1 child) from
    //      registers; `done` marks those among the first four children.
    {
      uint32_t c[4] = {0u, 0u, 0u, 0u};
      double w[4] = {0.0, 0.0, 0.0, 0.0};
      int na = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool take = j < xne && !(done >> j & 1u);
        c[0] = (take && na == 0) ? ch[j] : c[0];
        c[1] = (take && na == 1) ? ch[j] : c[1];
        c[2] = (take && na == 2) ? ch[j] : c[2];
        c[3] = (take && na == 3) ? ch[j] : c[3];
        w[0] = (take && na == 0) ? cw[j] : w[0];
        w[1] = (take && na == 1) ? cw[j] : w[1];
        w[2] = (take && na == 2) ? cw[j] : w[2];
        w[3] = (take && na == 3) ? cw[j] : w[3];
        na += take ? 1 : 0;
      }
      for (int h = 0; h < 4; h += 2) {
        if (na > h) {
          const bool two = na > h + 1;
          const uint32_t c0 = c[h], c1 = two ? c[h + 1] : c[h];
          const double eg0 = w[h], eg1 = two ? w[h + 1] : 0.0;
          add_rows2<MAXK>(S, row_rsrc(child_row(c0, slab, gamtab, phitab, stride), NLy),
                          row_rsrc(child_row(c1, slab, gamtab, phitab, stride), NLy), eg0, eg1, lane);
        }
      }
    }
#ifdef SK_STAMPS
    {
      int nl_ = 0;
      for (int j = 0; j < 4; ++j) nl_ += (j < xne && !(done >> j & 1u)) ? 1 : 0;
      cnt[0] += nl_ + (xne > 4 ? xne - 4 : 0);
    }
#endif
    for (int t = 4; t < xne; t += 2) {  // children past the fourth
      const uint32_t c0 = xch[chp_r + t];
      const bool two = t + 1 < xne;
      const uint32_t c1 = two ? xch[chp_r + t + 1] : c0;
      const double eg0 = xchw[chp_r + t], eg1 = two ? xchw[chp_r + t + 1] : 0.0;
      add_rows2<MAXK>(S, row_rsrc(child_row(c0, slab, gamtab, phitab, stride), NLy),
                      row_rsrc(child_row(c1, slab, gamtab, phitab, stride), NLy), eg0, eg1, lane);
    }
    STAMP(1);

    // ---- MATCH term, only where it can be non-zero.  y nodes are numbered
    //      by length, so the nodes inside the length band [xlen-band,
    //      xlen+band] are one index range [qa, qb) (looked up per row).  They
    //      are processed longest first, 64 per pass: a node's MATCH sum reads
    //      S of its children, which are strictly shorter, so a pass may
    //      overwrite R (S -> M) for the nodes it finished without affecting a
    //      later pass.  Everything outside the range gets M = 0 afterwards.
    //      Within a pass the child sums are edge-parallel: the pass's nodes
    //      own one contiguous range of the node-major edge array, each lane
    //      takes edges of it and adds g^gy S[child] into the per-wave
    //      accumulator hb[parent - q0] (LDS atomics), so the cost follows
    //      the pass's edge count, not its largest node degree.
    //      (LDS ops of a wave complete in issue order.)
    // (nodes from qb up have M = 0 and are never read as children here)
    if (!combo) {
#pragma unroll
      for (int k = 0; k < MAXK; ++k) R[lane + 64 * k] = lane + 64 * k < qb ? S[k] : 0.0;
    }
    double rowk = 0.0;
    STAMP(2);
#ifdef SK_STAMPS
    cnt[3] += qb > qa ? qb - qa : 0;
#endif
    if (!combo && qa < qb) {
      // node records and path counts come from HBM (L2-resident per y),
      // the first pass's issued before A, each later pass's during the
      // pass before.  A pass covers NW = 64*PW nodes [q0, top], lane l
      // scoring nodes q0 + 64j + l.
      constexpr int NW = 64 * PW;
      int top = qb - 1, q0 = max(top - NW + 1, qa);
      uint4 nd_n[PW];
      double Pq_n[PW];
#pragma unroll
      for (int j = 0; j < PW; ++j) {
        nd_n[j] = nd_first[j];
        Pq_n[j] = Pq_first[j];
      }
      for (;;) {
        uint4 nd[PW];
        double Pq[PW];
#pragma unroll
        for (int j = 0; j < PW; ++j) {
          nd[j] = nd_n[j];
          Pq[j] = Pq_n[j];
        }
        const int ntop = top - NW, nq0 = max(ntop - NW + 1, qa);
        if (ntop >= qa) {
#pragma unroll
          for (int j = 0; j < PW; ++j) {
            nd_n[j] = Y.nrg[min(nq0 + 64 * j + lane, ntop)];
            Pq_n[j] = yPg[min(nq0 + 64 * j + lane, ntop)];
          }
        }
        // node-score operands, requested ahead of the child sums
        double co_v[PW], gl_v[PW];
#pragma unroll
        for (int j = 0; j < PW; ++j) {
          co_v[j] = co[xcode + ((nd[j].y >> 16) & 0xf)];
          gl_v[j] = gp[nd[j].y & 0xffff];
        }
        double Hq[PW];  // x leaf child against a y stem: G0[leaf][*] = 0
#pragma unroll
        for (int j = 0; j < PW; ++j) Hq[j] = 0.0;
        if (!xloop) {
          // edge range of nodes [q0, top]: E(q0) .. E(top) + n_edges(top),
          // 64*SK_MU edges per round: all reads of a round are issued
          // before its first accumulate (two LDS round trips per round, not
          // per 64 edges)
          const int ea = __builtin_amdgcn_readfirstlane(nd[0].x & 0xffff);
          const int jt = (top - q0) >> 6;
          uint32_t ndt = nd[0].x;
#pragma unroll
          for (int j = 1; j < PW; ++j) ndt = jt == j ? nd[j].x : ndt;
          const uint32_t at = __builtin_amdgcn_readlane(ndt, (top - q0) & 63);
          const int eb = (int)((at & 0xffff) + ((at >> 16) & 0xff));
          constexpr bool EG = edges_global<MAXK>();
          uint32_t en[SK_MU];  // (EG) the round's edges, loaded a round ahead
          if constexpr (EG) {
#pragma unroll
            for (int u = 0; u < SK_MU; ++u) en[u] = Y.ed2g[min(ea + 64 * u + lane, eb - 1)];
          }
          for (int f0 = ea; f0 < eb; f0 += 64 * SK_MU) {
            uint32_t e[SK_MU];
            if constexpr (EG) {
#pragma unroll
              for (int u = 0; u < SK_MU; ++u) {
                e[u] = en[u];
                en[u] = Y.ed2g[min(f0 + 64 * (SK_MU + u) + lane, eb - 1)];
              }
            } else {
#pragma unroll
              for (int u = 0; u < SK_MU; ++u) e[u] = Y.ed2[min(f0 + 64 * u + lane, eb - 1)];
            }
            // unconditional accumulates (lanes past the range add 0 to their
            // own slot), so no read is sunk into a branch
            double g[SK_MU], rv[SK_MU];
#pragma unroll
            for (int u = 0; u < SK_MU; ++u) {
              g[u] = gp[e[u] >> 22];
              rv[u] = R[e[u] & 0x7ff];
            }
#pragma unroll
            for (int u = 0; u < SK_MU; ++u) {
              const bool ok = f0 + 64 * u + lane < eb;
              // (a product, not a select: a select lets the compiler sink
              // this round's reads into a branch)
              const double w = g[u] * rv[u] * (ok ? 1.0 : 0.0);
              const int h = ok ? (int)((e[u] >> 11) & 0x7ff) - q0 : lane;
              if constexpr (SK_SEGSUM && MAXK <= SK_SEGSUM_MAXK) {
                // Node-major edges put a parent's edges in adjacent lanes:
                // each run is summed within its quad (DPP quad_perm,
                // Hillis-Steele on contiguous keys) and only the run's last
                // lane in the quad issues the atomic.  Lanes past the range
                // carry a unique negative key, so they neither join a run nor
                // write.  (Wider classes sit at the register cap: off there.)
                const int key = ok ? h : -1 - lane;
                const int ql = lane & 3;
                double sw = w;
                {  // lane - 1: quad_perm(0,0,1,2)
                  const int ks = __builtin_amdgcn_mov_dpp(key, 0x90, 0xf, 0xf, false);
                  const double ws = __hiloint2double(
                      __builtin_amdgcn_mov_dpp(__double2hiint(sw), 0x90, 0xf, 0xf, false),
                      __builtin_amdgcn_mov_dpp(__double2loint(sw), 0x90, 0xf, 0xf, false));
                  sw += (ql >= 1 && ks == key) ? ws : 0.0;
                }
                {  // lane - 2: quad_perm(0,0,0,1)
                  const int ks = __builtin_amdgcn_mov_dpp(key, 0x40, 0xf, 0xf, false);
                  const double ws = __hiloint2double(
                      __builtin_amdgcn_mov_dpp(__double2hiint(sw), 0x40, 0xf, 0xf, false),
                      __builtin_amdgcn_mov_dpp(__double2loint(sw), 0x40, 0xf, 0xf, false));
                  sw += (ql >= 2 && ks == key) ? ws : 0.0;
                }
                const int kn = __builtin_amdgcn_mov_dpp(key, 0xF9, 0xf, 0xf, false);  // lane + 1
                if (ok && (ql == 3 || kn != key))
                  __hip_atomic_fetch_add(&hb[h], sw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
              } else {
                __hip_atomic_fetch_add(&hb[h], w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
              }
            }
          }
#pragma unroll
          for (int j = 0; j < PW; ++j) {
            Hq[j] = hb[64 * j + lane];
            hb[64 * j + lane] = 0.0;
          }
        }
#pragma unroll
        for (int j = 0; j < PW; ++j) {
          const int q = q0 + 64 * j + lane;
          const bool on = q <= top;
          const uint32_t nda = nd[j].x, ndc = nd[j].y;
          double H = Hq[j];
          if (((nda >> 16) & 0xff) == 0)  // loop node: closed form over the two leaf children
            H = (xloop ? xeg0 : xSL) * gl_v[j];
          double vs;
          if (x_one && (ndc >> 24) != 0u) {
            // co[a][b][c][d]*cx*cy, no gap columns (score_table.cpp:171-185)
            vs = co_v[j] * xpf * (double)__uint_as_float(nd[j].w);
          } else {
            // general bp-frequency lists / gap columns (score_table.cpp:162-201)
            const int qq = on ? q : top;
            vs = H != 0.0 ? match_node_score(co, s, xbb, xb0, xnbf, ys, Y, ys.yn_b[Y.nb + qq] >> 16,
                                             nda >> 24, xwg, gap2 * (double)__uint_as_float(nd[j].z),
                                             x_nbp, (double)ys.yn_nbp[Y.nb + qq], x_nseq)
                          : 0.0;
          }
          const double M = vs * H;
          if (on) {
            R[q] = M;
            rowk += M * Pq[j];
          }
        }
#ifdef SK_STAMPS
        cnt[2] += 1;
#endif
        if (ntop < qa) break;
        top = ntop;
        q0 = nq0;
      }
    }
    STAMP(3);
    // below the band: M = 0 (above it R was filled with 0)
#pragma unroll
    for (int k = 0; k < MAXK; ++k) {
      const int q = lane + 64 * k;
      if (!combo && 64 * k < qa && q < qa) R[q] = 0.0;
    }
    kacc += xP * rowk;
    wave_sync();
    STAMP(4);

    // ---- next row's children: the ones this row cannot produce are loaded
    //      now (two at most, into registers the MATCH sums have freed) and
    //      land during the sweep; this row itself, when a child of the next,
    //      is added from registers in D.
    // rows prefetched per row: two where the register budget allows
    constexpr int NPF = MAXK == 17 ? SK_NPF17
                        : (MAXK == 16 && (SK_NPF16 == 0 || SK_M16 == 2)) ? 0
                        : ((MAXK <= 12 && SK_NPF12 == 2) || (MAXK == 16 && SK_NPF16 == 2) ||
                           (MAXK == 20 && SK_W20 == 8 && SK_NPF20 == 2)) ? 2 : 1;
    uint32_t nxt_done = 0;
    double egd = 0.0, egt0 = 0.0, egt1 = 0.0;
    double T0[MAXK], T1[MAXK];
#pragma unroll
    for (int k = 0; k < MAXK; ++k) T0[k] = T1[k] = 0.0;
    if (r + 1 < nlx) {
      const int nne = nx.a & 0xff;
      uint32_t pf0 = 0, pf1 = 0;
      int npf = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j < nne) {
          const uint32_t c = nch[j];
          const double g = ncw[j];
          if ((c & 0xffff) == pslot) {
            egd += g;
            nxt_done |= 1u << j;
          } else if (npf < NPF) {
            if (npf == 0) {
              pf0 = c;
              egt0 = g;
            } else {
              pf1 = c;
              egt1 = g;
            }
            ++npf;
            nxt_done |= 1u << j;
          }
        }
      }
      if (NPF >= 1 && npf >= 1) {
        const __amdgpu_buffer_rsrc_t r0 = row_rsrc(child_row(pf0, slab, gamtab, phitab, stride), NLy);
#pragma unroll
        for (int k = 0; k < MAXK; ++k) T0[k] = row_ld(r0, lane, k);
      }
      if (NPF >= 2 && npf >= 2) {
        const __amdgpu_buffer_rsrc_t r1 = row_rsrc(child_row(pf1, slab, gamtab, phitab, stride), NLy);
#pragma unroll
        for (int k = 0; k < MAXK; ++k) T1[k] = row_ld(r1, lane, k);
      }
    }

    // ---- C: IY recurrence G1[q] += w(q,cy) G1[cy], w = gap^2 w_y(q) g^gaps,
    //      over the y example's sweep schedule: chunks of 64 edges, each
    //      placed after every edge of its children (host list schedule).  A
    //      chunk's R reads are issued after the previous chunk's atomics and
    //      a wave's LDS ops execute in issue order, so nothing drains between
    //      chunks: only the data a lane consumes is waited for.  Records are
    //      read two chunks ahead, weights one; dummy records (weight 0) pad
    //      the chunks.
    //      With a length band, every y node shorter than xlen - band has G1 =
    //      0 exactly (its MATCH terms are masked and so are all its
    //      descendants'), so chunks whose children are all that short add
    //      only zeros: the sweep starts at the first chunk whose running
    //      maximum child length reaches the threshold.
    int c0 = 0;
    if (band > 0) c0 = Y.ycs[min(max(xlen - band, 0), Y.lmax + 1)];
    c0 = __builtin_amdgcn_readfirstlane(c0);
#ifdef SK_STAMPS
    cnt[1] += Y.nch - c0;
#endif
    // a row nobody reads (a root: pslot 0xffff) needs only its MATCH terms
    // (K is the path sum of M), so it skips the sweep and the store
    if (!combo && c0 < Y.nch && pslot != 0xffffu) {
      iy_sweep<node_weights<MAXK>(), node_weights_f32<MAXK>()>(Y, R, c0, lane);
      wave_sync();
    }
    STAMP(5);

    // ---- D: G0 row p = G1 + v_s*S, to p's slot.  Every later read of
    // element q of this row is by the same lane (q = lane + 64k), so
    // per-thread program order makes it visible: no fence.  A row nobody
    // reads (a root) is not stored; it is no child of the next row either.
    // (the widest classes read G1 back in two halves: fewer live registers)
    constexpr int HD = (MAXK > SK_HALF_D || (m16_wide<MAXK>() && SK_M16_HALFD)) ? (MAXK + 1) / 2 : MAXK;
    if (pslot == 0xffffu) {
#pragma unroll
      for (int k = 0; k < MAXK; ++k) S[k] = egt0 * T0[k] + (NPF >= 2 ? egt1 * T1[k] : 0.0);
    } else if (pslot == 0xfffeu) {
      // read only by the next row, from registers: not stored
      const double cw = combo ? 1.0 : xwg;
#pragma unroll
      for (int h0 = 0; h0 < MAXK; h0 += HD) {
        double g1[HD];
#pragma unroll
        for (int k = 0; k < HD; ++k) g1[k] = combo ? 0.0 : R[lane + 64 * (h0 + k)];
        SCHED_FENCE();
#pragma unroll
        for (int k = 0; k < HD; ++k)
          S[h0 + k] = egd * (g1[k] + cw * S[h0 + k]) + egt0 * T0[h0 + k] + (NPF >= 2 ? egt1 * T1[h0 + k] : 0.0);
      }
    } else {
#ifdef SK_FULL_STORE
      double* __restrict__ orow = slab + (size_t)pslot * stride + lane;
#else
      // stores through the slot's buffer resource: the padded tail (q >=
      // NLy, never read) is dropped by the range check, not written
      const __amdgpu_buffer_rsrc_t orsrc = row_rsrc(slab + (size_t)pslot * stride, NLy);
#endif
      // all R reads issued before the first store (one LDS round trip)
      const double cw = combo ? 1.0 : xwg;
#pragma unroll
      for (int h0 = 0; h0 < MAXK; h0 += HD) {
        double g1[HD];
#pragma unroll
        for (int k = 0; k < HD; ++k) g1[k] = combo ? 0.0 : R[lane + 64 * (h0 + k)];
        SCHED_FENCE();
#pragma unroll
        for (int k = 0; k < HD; ++k) {
          const double o = g1[k] + cw * S[h0 + k];
#ifndef SK_XNOSTORE
#ifdef SK_FULL_STORE
          orow[64 * (h0 + k)] = o;
#else
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o), orsrc, lane * 8,
                                                (h0 + k) * 512, SK_ROW_ST_POL);
#endif
#endif
          // the next row's partial sum: itself (distance-1) + prefetched rows
          S[h0 + k] = egd * o + egt0 * T0[h0 + k] + (NPF >= 2 ? egt1 * T1[h0 + k] : 0.0);
        }
      }
    }
    done = nxt_done;
    wave_sync();
    STAMP(6);
  }
#ifdef SK_STAMPS
  if (lane == 0 && P.stamps) {
    for (int i = 0; i < 8; ++i) atomicAdd(&P.stamps[i], tacc[i]);
    atomicAdd(&P.stamps[8], (unsigned long long)nlx);
    atomicAdd(&P.stamps[9], 1ull);
    for (int i = 0; i < 4; ++i) atomicAdd(&P.stamps[10 + i], cnt[i]);
  }
#endif
  // wave reduction of the K partial sums (fixed order -> deterministic)
  for (int off = 32; off > 0; off >>= 1) kacc += __shfl_xor(kacc, off, 64);
  return kacc;
}

template <int MAXK>
struct StemWaves {
  static constexpr int value = MAXK <= 12 ? 12 : MAXK <= 17 ? (SK_M16 ? 12 : SK_W16) : MAXK <= 20 ? SK_W20 : 8;
};

template <int MAXK>
__global__ void __launch_bounds__(64 * StemWaves<MAXK>::value) sk_dag_stem_kernel(StemLaunch P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const DevSet& s = P.yset;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nwaves = blockDim.x >> 6;
  const int maxnl = P.lds_max_nl;  // multiple of 64
  constexpr int PW = pass_width<MAXK>();

  // LDS carve (every region a multiple of 16 bytes)
  lds_f64* co = (lds_f64*)(smem);                             // 256
  lds_f64* gp = co + 256;                                     // n_gpow_pad
  lds_f64* Rall = gp + P.n_gpow_pad;                          // nwaves*maxnl
  lds_f64* hball = Rall + (size_t)nwaves * maxnl;             // nwaves*64*PW (MATCH sums)
  constexpr bool NW = node_weights<MAXK>();
  lds_f64* yew = hball + (size_t)nwaves * 64 * PW;         // lds_max_nch*64 weights (NW: maxnl)
  lds_u32* ysc = (lds_u32*)(yew + (node_weights_f32<MAXK>() ? (size_t)maxnl / 2
                                   : NW ? (size_t)maxnl : (size_t)P.lds_max_nch * 64));  // lds_max_nch*64 records
  lds_u32* yed2 = ysc + (size_t)P.lds_max_nch * 64;           // lds_max_edges (mult. of 4)
  lds_i32* ylf = (lds_i32*)(yed2 + (edges_global<MAXK>() ? 0 : P.lds_max_edges));  // lds_max_len_pad
  lds_i32* ycs = ylf + P.lds_max_len_pad;                     // lds_max_len_pad
  lds_i32* ctl = ycs + P.lds_max_len_pad;                     // 4 ints
  lds_f64* kap = (lds_f64*)(ctl + 4);                         // xset.n_gam (gam_on)

  for (int k = threadIdx.x; k < 256; k += blockDim.x) co[k] = P.co_subst[k];
  for (int k = threadIdx.x; k < P.n_gpow; k += blockDim.x) gp[k] = P.gpow[k];

  lds_f64* R = Rall + (size_t)wave * maxnl;
  lds_f64* hb = hball + (size_t)wave * 64 * PW;
  for (int j = 0; j < PW; ++j) hb[64 * j + lane] = 0.0;  // kept zero between MATCH passes
  double* slab = P.scratch + (size_t)(blockIdx.x * nwaves + wave) * P.slab_doubles;
  double* gamtab = P.gam_on ? P.gam + (size_t)blockIdx.x * P.gam_doubles : nullptr;
  // the workgroup's Phi table: n_phi rows of 64*MAXK, then their sums kappa
  double* phitab = P.phi_on ? P.phi + (size_t)blockIdx.x * P.phi_doubles : nullptr;
  double* phikap = P.phi_on ? phitab + (size_t)P.xset.n_phi * (64 * MAXK) : nullptr;
  const double gap2 = P.gap2;
  const int band = (int)P.band;

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
    Y.nch = s.ex_nch[y];
    Y.nseqs = s.ex_nseqs[y];
    const int nb = s.ex_node_base[y], eb = s.ex_edge_base[y], bb = s.ex_bpf_base[y];
    Y.lmax = Y.nl ? (int)(s.yn_b[nb + Y.nl - 1] & 0xffff) : 0;
    {
      const int ne = s.ex_edge_base[y + 1] - eb;
      // sweep schedule + two dummy chunks (read ahead past the end), with
      // the edge weights (weight 0 for the dummies)
      const int sb = s.ex_ysc_base[y] * 64, nrec = Y.nch * 64;
      // dummy records (the schedule's padding and two trailing chunks read
      // ahead) read and write a free slot past the y's nodes: the classes
      // hold y of at most 64 MAXK - 1 nodes (stem_maxk(nl + 1)), so there is
      // one at least, its R entry stays 0 through every sweep and its node
      // weight is 0 -- a dummy adds 0 * 0 to it, without a select in the sweep
      // (spread over the free slots by lane: one target for every dummy of a
      // chunk would serialize their atomics)
      const int nfree = max(maxnl - Y.nl, 1);
      for (int k = threadIdx.x; k < nrec + 128; k += blockDim.x) {
        uint32_t r = k < nrec ? s.ysc[sb + k] : 0u;
        const uint32_t ch = r & 0x7ff, pa = (r >> 11) & 0x7ff;
        const uint32_t zs = (uint32_t)(maxnl - 1 - (k & 63) % nfree);
        if (k >= nrec || ch == pa) r = zs | (zs << 11);
        ysc[k] = r;
        if (!NW) yew[k] = (k >= nrec || ch == pa) ? 0.0 : gap2 * (double)s.yn_w[nb + pa] * gp[r >> 22];
      }
      if (node_weights_f32<MAXK>())
        for (int q = threadIdx.x; q < maxnl; q += blockDim.x) ((lds_f32*)yew)[q] = q < Y.nl ? s.yn_w[nb + q] : 0.0f;
      else if (NW)  // (gap2 w) gp: the slot weights' rounding
        for (int q = threadIdx.x; q < maxnl; q += blockDim.x) yew[q] = q < Y.nl ? gap2 * (double)s.yn_w[nb + q] : 0.0;
      if (!edges_global<MAXK>())
        for (int k = threadIdx.x; k < ne; k += blockDim.x) yed2[k] = s.ye2[eb + k];
      const int cb = s.ex_ycs_base[y];
      for (int v = threadIdx.x; v <= Y.lmax + 1; v += blockDim.x) ycs[v] = s.ycs[cb + v];
    }
    Y.nrg = s.yrec + nb;
    Y.sc = ysc; Y.ew = yew; Y.ed2 = yed2; Y.lfirst = ylf; Y.ycs = ycs; Y.gp = gp;
    Y.ewf = (const lds_f32*)yew; Y.gap2 = gap2;
    Y.ed2g = s.ye2 + eb;
    Y.nb = nb; Y.bb = bb;
    __syncthreads();
    // length -> first node index (nodes are sorted by length)
    for (int v = threadIdx.x; v <= Y.lmax + 1; v += blockDim.x) {
      int lo = 0, hi = Y.nl;  // first q with len(q) >= v
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((int)(s.yn_b[nb + mid] & 0xffff) < v) lo = mid + 1; else hi = mid;
      }
      ylf[v] = lo;
    }
    __syncthreads();

    // Gamma rows of this y (gapless y only): for every gamma key g = (code,
    // len) of the x set, Gamma_g = the IY sweep of M_g[q] = co[code][bp(q)]
    // p(q) g^{leaf gaps(q)} over the y loop nodes q in len's length band (an
    // x gamma row's G0 row is g^lg pf Gamma_g; its MATCH row is that times
    // M_g), into this workgroup's table; kappa_g = sum_q M_g[q] P_y[q].
    const bool gam = P.gam_on && s.ex_gapless[y];
    if (gam) {
      const DevSet& xset = P.xset;
      for (int g = wave_u; g < xset.n_gam; g += nwaves) {
        const uint32_t key = xset.gam_key[g];
        const int gcode = (int)(key >> 16) * 16, glen = (int)(key & 0xffff);
        double kp = 0.0;
        for (int k = 0; k < MAXK; ++k) {
          const int q = lane + 64 * k;
          double M = 0.0;
          if (q < Y.nl) {
            const uint4 nd = Y.nrg[q];
            const int ylen = (int)(s.yn_b[nb + q] & 0xffff);
            if (((nd.x >> 16) & 0xff) == 0 && (band == 0 || abs(glen - ylen) <= band)) {
              double vs;
              if ((nd.y >> 24) != 0u) {
                vs = co[gcode + ((nd.y >> 16) & 0xf)] * (double)__uint_as_float(nd.w);
              } else {
                vs = 0.0;
                const int yb0 = (int)(s.yn_b[nb + q] >> 16), ynb = (int)(nd.x >> 24);
                for (int b = 0; b < ynb; ++b)
                  vs += co[gcode + s.bpf_code[bb + yb0 + b]] * (double)s.bpf_p[bb + yb0 + b];
              }
              M = vs * gp[nd.y & 0xffff];
              kp += M * s.yn_P[nb + q];
            }
          }
          R[q] = M;
        }
        for (int off = 32; off > 0; off >>= 1) kp += __shfl_xor(kp, off, 64);
        if (lane == 0) kap[g] = kp;
        wave_sync();
        int c0 = 0;
        if (band > 0) c0 = Y.ycs[min(max(glen - band, 0), Y.lmax + 1)];
        c0 = __builtin_amdgcn_readfirstlane(c0);
        if (c0 < Y.nch) iy_sweep<node_weights<MAXK>(), node_weights_f32<MAXK>()>(Y, R, c0, lane);
        double* grow = gamtab + (size_t)g * (64 * MAXK);
        for (int k = 0; k < MAXK; ++k)
          if (lane + 64 * k < Y.nl) grow[lane + 64 * k] = R[lane + 64 * k];  // (the tail is never read)
        wave_sync();
      }
      __syncthreads();  // the table and kappa, for every wave's pairs

      // Phi rows of the item's phi keys t = (code a, len, gamma key g):
      // M_t[q] = co[a][bp(q)] p(q) sum_{cy in ch(q)} g^gy Gamma_g[cy] over
      // the y stems q in len's band; Phi_t = its IY sweep; kappa_t = sum_q
      // M_t[q] P_y[q] (a phi row's MATCH row is pf_p sum_c w_c M_{t(c)} plus
      // its Gamma_{a,len} part)
      if (P.phi_on) {
        // the item's keys come sorted by gamma key: wave w takes the w-th
        // contiguous share, and H_g[q] = sum_{cy in ch(q)} g^gy Gamma_g[cy]
        // (independent of the key's code and length) is formed once per
        // gamma key from the Gamma row staged in the wave's LDS row
        const DevSet& xset = P.xset;
        const int pb = P.item_phi_off[it], pe = P.item_phi_off[it + 1];
        const int share = (pe - pb + nwaves - 1) / nwaves;
        const int t0 = pb + wave_u * share, t1 = min(pe, t0 + share);
        int gcur = -1;
        double Hr[MAXK];
#pragma unroll
        for (int k = 0; k < MAXK; ++k) Hr[k] = 0.0;
        for (int t = t0; t < t1; ++t) {
          const int idx = __builtin_amdgcn_readfirstlane(P.item_phi[t]);
          const int g = __builtin_amdgcn_readfirstlane((int)xset.phi_g[idx]);
          if (g != gcur) {
            gcur = g;
            const double* __restrict__ grow = gamtab + (size_t)g * (64 * MAXK);
#pragma unroll
            for (int k = 0; k < MAXK; ++k) R[lane + 64 * k] = grow[lane + 64 * k];
            wave_sync();
            for (int k = 0; k < MAXK; ++k) {
              const int q = lane + 64 * k;
              double H = 0.0;
              if (q < Y.nl) {
                const uint32_t na = Y.nrg[q].x;
                const int ne = (int)((na >> 16) & 0xff), e0 = (int)(na & 0xffff);
                for (int e = 0; e < ne; ++e) {
                  const uint32_t rec = edges_global<MAXK>() ? Y.ed2g[e0 + e] : Y.ed2[e0 + e];
                  H += gp[rec >> 22] * R[rec & 0x7ff];
                }
              }
              Hr[k] = H;
            }
            wave_sync();
          }
          const uint32_t al = xset.phi_al[idx];
          const int acode = (int)(al >> 16) * 16, alen = (int)(al & 0xffff);
          double kp = 0.0;
#pragma unroll
          for (int k = 0; k < MAXK; ++k) {
            const int q = lane + 64 * k;
            double M = 0.0;
            if (q < Y.nl) {
              const uint4 nd = Y.nrg[q];
              const int ylen = (int)(s.yn_b[nb + q] & 0xffff);
              if (Hr[k] != 0.0 && (band == 0 || abs(alen - ylen) <= band)) {
                double vs;
                if ((nd.y >> 24) != 0u) {
                  vs = co[acode + ((nd.y >> 16) & 0xf)] * (double)__uint_as_float(nd.w);
                } else {
                  vs = 0.0;
                  const int yb0 = (int)(s.yn_b[nb + q] >> 16), ynb = (int)(nd.x >> 24);
                  for (int b = 0; b < ynb; ++b)
                    vs += co[acode + s.bpf_code[bb + yb0 + b]] * (double)s.bpf_p[bb + yb0 + b];
                }
                M = vs * Hr[k];
                kp += M * s.yn_P[nb + q];
              }
            }
            R[q] = M;
          }
          for (int off = 32; off > 0; off >>= 1) kp += __shfl_xor(kp, off, 64);
          if (lane == 0) phikap[idx] = kp;
          wave_sync();
          int c0 = 0;
          if (band > 0) c0 = Y.ycs[min(max(alen - band, 0), Y.lmax + 1)];
          c0 = __builtin_amdgcn_readfirstlane(c0);
          if (c0 < Y.nch) iy_sweep<node_weights<MAXK>(), node_weights_f32<MAXK>()>(Y, R, c0, lane);
          double* prow = phitab + (size_t)idx * (64 * MAXK);
#pragma unroll
          for (int k = 0; k < MAXK; ++k)
            if (lane + 64 * k < Y.nl) prow[lane + 64 * k] = R[lane + 64 * k];
          wave_sync();
        }
        __syncthreads();
      }
    }

    // the item's pairs (costliest first) go to whichever wave is free next
    // (the first nwaves dealt statically; ctl[1] counts the pairs taken), so
    // the workgroup waits at the item boundary for one pair, not a round
    if (threadIdx.x == 0) ctl[1] = nwaves;
    __syncthreads();
    for (int t = wave_u; t < item.z;) {
      const int x = P.xs[item.y + t];
      const double k = stem_pair<MAXK>(P, Y, R, hb, co, gp, slab, x, lane, gam, gamtab, kap, phitab, phikap);
      if (lane == 0) P.out[P.oidx[item.y + t]] = k;
      int nt = 0;
      // generic-pointer atomic on the LDS counter
      if (lane == 0) nt = atomicAdd(reinterpret_cast<int*>(const_cast<int32_t*>((const int32_t*)ctl)) + 1, 1);
      t = __builtin_amdgcn_readlane(nt, 0);
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
  b += (size_t)nwaves * P.lds_max_nl * 8;          // one row per wave
  b += (size_t)nwaves * 64 * pass_width_of(stem_maxk(P.lds_max_nl)) * 8;  // MATCH accumulators
  const int maxk = stem_maxk(P.lds_max_nl);
  if (node_weights_of(maxk))                       // sweep schedule: records, node weights
    b += (size_t)P.lds_max_nch * 64 * 4 + (size_t)P.lds_max_nl * (maxk >= SK_NODEF_MIN ? 4 : 8);
  else                                             // sweep schedule: weights + records
    b += (size_t)P.lds_max_nch * 64 * 12;
  if (stem_maxk(P.lds_max_nl) < SK_EDG_MIN) b += (size_t)P.lds_max_edges * 4;  // node-major edges
  b += (size_t)P.lds_max_len_pad * 4 * 2 + 16;     // length tables, control
  if (P.gam_on) b += (size_t)P.xset.n_gam * 8;     // Gamma sums kappa
  return b;
}

#define SK_STEM_CLASSES(X) X(4) X(8) X(12) X(16) X(17) X(20) X(24) X(28) X(32)

static const void* stem_kernel_ptr(int maxk) {
  switch (maxk) {
#define SK_CASE(K) \
  case K: return reinterpret_cast<const void*>(sk_dag_stem_kernel<K>);
    SK_STEM_CLASSES(SK_CASE)
#undef SK_CASE
    default: return nullptr;
  }
}

int stem_maxk(int max_nl) {
  const int s = (std::max(max_nl, 1) + 63) / 64;  // 64-node slots per lane
  if (SK_K17 && s == 17) return 17;
  const int k = (s + 3) & ~3;
  return k <= 32 ? k : -1;
}

hipError_t launch_stem(const StemLaunch& P, int grid, int nwaves, hipStream_t st) {
  const size_t lds = stem_lds_bytes(P, nwaves);
  const int maxk = stem_maxk(P.lds_max_nl);
  const void* fn = stem_kernel_ptr(maxk);
  if (!fn) return hipErrorInvalidValue;
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  switch (maxk) {
#define SK_CASE(K)                                                                          \
  case K:                                                                                  \
    hipLaunchKernelGGL(sk_dag_stem_kernel<K>, dim3(grid), dim3(64 * nwaves), lds, st, P); \
    break;
    SK_STEM_CLASSES(SK_CASE)
#undef SK_CASE
    default: return hipErrorInvalidValue;
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
