// 4-D stem kernel on CDNA4 (gfx950).
//
// Reference: StemKernel<double,BPMat>::full_dp  stem_kernel/stem_kernel.cpp:282-351,
//   dp_init / dp_update :85-111, BPMat::prob :354-421.
//
// The DP runs over pairs of substrings, x[i,j) and y[k,l): eight states
// K0..K3, G0..G3 per cell (i,j,k,l).  Dependencies, by x span d1 = j-i and
// y span d2 = l-k:
//   K0,G0 <- (i, j-1)          span d1-1, same (k,l)
//   K1,G1 <- (i+1, j)          span d1-1, same (k,l)
//   G0    <- (i+1, j-1)        span d1-2, cell (k+1, l-1)   (stacking term)
//   K2,G2 <- (k, l-1)          same plane, span d2-1
//   K3,G3 <- (k+1, l)          same plane, span d2-1
// so one launch per x span d1 computes every plane (i, i+d1) of every pair in
// the batch in parallel, one WAVEFRONT per plane, sweeping the plane's y
// spans d2 = 0..m in order.  K2/G2/K3/G3 never leave registers (lane owns
// CPL consecutive k, the k+1 neighbour of the last one comes from the next
// lane by DPP); only K0,G0,K1,G1 of each cell go to HBM, once, and are read
// back once by the next span (72 B per cell: SURVEY.md §8d's roofline).
//
// HBM layout of one plane: four state arrays (K0,G0,K1,G1) over cells stored
// row by row in d2, row d2 holding k = 0..m-d2 padded to a multiple of 4.
// Per pair, a ring of three span buffers of n+1 planes each.
#include <hip/hip_runtime.h>

#include "device_set.h"
#include "launch.h"

namespace sk {

// lane l receives lane l+1's value (lane 63 receives `high`): DPP wave_shl:1
__device__ __forceinline__ double wave_shl1(double v, double high) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const int rlo = __builtin_amdgcn_update_dpp(__double2loint(high), lo, 0x130, 0xf, 0xf, false);
  const int rhi = __builtin_amdgcn_update_dpp(__double2hiint(high), hi, 0x130, 0xf, 0xf, false);
  return __hiloint2double(rhi, rlo);
}

__device__ __forceinline__ int pad4(int v) { return (v + 3) & ~3; }

__device__ __forceinline__ double bcast_lane0(double v) {
  const int lo = __builtin_amdgcn_readfirstlane(__double2loint(v));
  const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(v));
  return __hiloint2double(hi, lo);
}

// offset of row d2 in a plane: sum_{e<d2} pad4(m+1-e)
__device__ __forceinline__ int row_off(int m, int d2) {
  const int q = d2 >> 2;
  int r = 4 * q * (m + 1) - (4 * q) * (4 * q - 1) / 2 + 6 * q;  // whole groups of four rows
  for (int e = 4 * q; e < d2; ++e) r += pad4(m + 1 - e);
  return r;
}

// A range-checked buffer over `bytes` from `base` (wave-uniform): loads past
// the range return 0, stores past it are dropped -- a row's slots need no
// per-slot guard, so a step is straight-line code.  The whole element offset
// goes in the VGPR offset (the SGPR offset is not range-checked on gfx9).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t s4c_rsrc(const void* base, int bytes) {
  const uint64_t a = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, bytes, 0x00020000);
}
typedef unsigned int s4c_u32x2 __attribute__((__vector_size__(2 * sizeof(unsigned int))));
// slot c (elements 64c .. 64c + 63) of a row of nk valid elements: a
// buffer per slot, lane offset in the VGPR (range-checked), so the slot
// offset costs no VGPR
template <class T>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t s4c_slot(const T* base, int nk, int c) {
  return s4c_rsrc(base + 64 * c, (nk > 64 * c ? nk - 64 * c : 0) * (int)sizeof(T));
}
__device__ __forceinline__ double s4c_ld64(const double* base, int nk, int c, int lane) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(s4c_slot(base, nk, c), lane * 8, 0, 0));
}
__device__ __forceinline__ float s4c_ld32(const float* base, int nk, int c, int lane) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(s4c_slot(base, nk, c), lane * 4, 0, 0));
}
__device__ __forceinline__ uint8_t s4c_ld8(const uint8_t* base, int nk, int c, int lane) {
  return __builtin_amdgcn_raw_buffer_load_b8(s4c_slot(base, nk, c), lane, 0, 0);
}
__device__ __forceinline__ void s4c_st64(double* base, int nk, int c, int lane, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(s4c_u32x2, v), s4c_slot(base, nk, c), lane * 8, 0, 0);
}

// BAND: partial_dp (stem_kernel.cpp:113-280) with the -b band constraints:
// cells outside the band stay zero, K0 past c_high[j-1] and K1 below
// c_low[i+1] take the reference's boundary approximations.
#ifndef SK4_PF  // K-sum kernel: rows fetched ahead (1 or 2)
#define SK4_PF 2
#endif
#ifndef SK4_MINB  // minimum 4-wave workgroups per CU (register budget knob)
#define SK4_MINB 1
#endif
template <int CPL, bool BAND>
__global__ void __launch_bounds__(256, SK4_MINB) sk_stem4d_kernel(Stem4dLaunch P) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t it = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave;
  if (it >= P.n_items) return;
  const int2 item = P.items[it];  // {pair slot, i}
  const Stem4dPair pr = P.pairs[item.x];
  const int i = item.y, d1 = P.d1, j = i + d1;
  const int n = pr.n, m = pr.m;
  const int64_t cp = pr.plane_doubles;  // per state
  double* span_cur = P.scratch + pr.scratch_off + (int64_t)(d1 % 3) * (n + 1) * 4 * cp;
  double* __restrict__ cur = span_cur + (int64_t)i * 4 * cp;
  const double g = P.gap;
  // k tiles of 64*CPL cells: lane owns k = kb + lane + 64c (every state
  // access of a wave instruction is 512 contiguous bytes).  y longer than one
  // tile (|y| >= 512 at CPL 8) is swept tile by tile, right to left: the
  // only dependence across k is K3/G3 at (k+1, l) of span d2-1, which the
  // tile to the right leaves in a per-plane boundary column (P.kbound).
  constexpr int TW = 64 * CPL;
  const int ntile = (m + TW) / TW;

  if (d1 == 0) {  // plane (j,j): K0 = 1, G0 = g^(l-k), K1 = G1 = 0  (:297-309)
    for (int kt = 0; kt < ntile; ++kt) {
      const int k0 = kt * TW + lane;
      int R = 0;
      for (int d2 = 0; d2 <= m; ++d2) {
        const double gd = P.gpow[d2];
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          const int k = k0 + 64 * c;
          if (k <= m - d2) {
            cur[R + k] = 1.0;
            cur[cp + R + k] = gd;
            cur[2 * cp + R + k] = 0.0;
            cur[3 * cp + R + k] = 0.0;
          }
        }
        R += pad4(m + 1 - d2);
      }
    }
    if (n == 0 && lane == 0) P.out[pr.out_index] = 1.0;
    return;
  }

  const double* span_p1 = P.scratch + pr.scratch_off + (int64_t)((d1 - 1) % 3) * (n + 1) * 4 * cp;
  const double* __restrict__ A = span_p1 + (int64_t)i * 4 * cp;        // plane (i, j-1)
  const double* __restrict__ B = span_p1 + (int64_t)(i + 1) * 4 * cp;  // plane (i+1, j)
  const double* Cg = nullptr;                              // plane (i+1, j-1), G0
  if (d1 >= 2)
    Cg = P.scratch + pr.scratch_off + (int64_t)((d1 - 2) % 3) * (n + 1) * 4 * cp +
         (int64_t)(i + 1) * 4 * cp + cp;
  const float* bpx = P.bpdiag + pr.x_bp;  // prob(a, a+e) at e*n - e*(e-1)/2 + a
  const float* bpy = P.bpdiag + pr.y_bp;
  const uint8_t* xs = P.chars + pr.x_chr;
  const uint8_t* ys = P.chars + pr.y_chr;
  const float bound = P.bp_bound;
  // bp_ij = prob(i, j-1): diagonal e = j-1-i = d1-1 of x  (:320)
  const int e1 = d1 - 1;
  const float bp_ij = bpx[(int64_t)e1 * n - (int64_t)e1 * (e1 - 1) / 2 + i];
  const bool stack_on = bp_ij > bound;
  const uint8_t xi = xs[i], xj = xs[j - 1];
  const double stk = P.stack, sub = P.subst;
  int clj = 0, chj = m, cli = 0, chi = m, chjm1 = m, cli1 = 0, cljm1 = 0, chi1 = m;
  // y spans with cells inside the constraints: l in [clj, chj], k in [cli, chi]
  int d2_lo = 1, d2_hi = m;
  if (BAND) {
    const int32_t* cl = P.band_lo + pr.band_off;
    const int32_t* ch = P.band_hi + pr.band_off;
    clj = cl[j];
    chj = ch[j];
    cli = cl[i];
    chi = ch[i];
    chjm1 = ch[j - 1];
    cli1 = cl[i + 1];
    cljm1 = cl[j - 1];
    chi1 = ch[i + 1];
    d2_lo = max(1, clj - chi);
    d2_hi = min(m, chj - cli);
    if (i == 0 && j == n && lane == 0) P.out[pr.out_index] = 0.0;  // K0(0,n,0,m) may lie outside
  }
  // Partial DP: only the spans [d2_lo, d2_hi] are swept and only cells inside
  // the constraints are read or written.  Nothing outside them is ever read:
  // A and B are read at cells inside their own planes' constraints (or at the
  // boundary cells of the approximations), and the stacking read of plane
  // (i+1,j-1) is guarded by that plane's constraints unless it is the fully
  // initialised plane (j-1,j-1).
  const bool cg_guard = BAND && d1 >= 3;
  // boundary columns of this plane: [2 parities][K3, G3][span d2]
  double* kbnd = ntile > 1 ? P.kbound + it * P.kbound_stride : nullptr;
  const int bstride = m + 1;

  for (int kt = ntile - 1; kt >= 0; --kt) {
  const int kb = kt * TW;
  const int k0 = kb + lane;
  double* bnd_w = kbnd ? kbnd + (int64_t)(kt & 1) * 2 * bstride : nullptr;        // for tile kt-1
  const double* bnd_r = kbnd ? kbnd + (int64_t)((kt + 1) & 1) * 2 * bstride : nullptr;  // of tile kt+1
  const bool has_right = kt + 1 < ntile;
  if (bnd_w && lane == 0) {  // nothing swept below d2_lo: the state there is zero
    bnd_w[max(d2_lo - 1, 0)] = 0.0;
    bnd_w[bstride + max(d2_lo - 1, 0)] = 0.0;
  }

  double K2[CPL], G2[CPL], K3[CPL], G3[CPL];
  uint8_t yk[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    K2[c] = G2[c] = K3[c] = G3[c] = 0.0;
    const int k = k0 + 64 * c;
    yk[c] = k < m ? ys[k] : 0;
  }

  // d2 = 0: cells (l,l): K0 = 1, G0 = G0(i+1,j,l,l)*g, K1 = G1 = 0  (:313-316);
  // partial DP: only l in [clj, chj] (the others are never read)
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int k = k0 + 64 * c;
    if (k <= m && (!BAND || (k >= clj && k <= chj))) {
      cur[k] = 1.0;
      cur[cp + k] = B[cp + k] * g;
      cur[2 * cp + k] = 0.0;
      cur[3 * cp + k] = 0.0;
    }
  }
  // Row d2's inputs are prefetched during row d2-1 (they do not depend on
  // it): K0,G0 of (i,j-1), K1,G1 of (i+1,j), and, for the stacking term,
  // prob_y(k, l-1) and G0(i+1,j-1) at (k+1, l-1).
  double pK0[CPL], pG0[CPL], pK1[CPL], pG1[CPL], pGs[CPL];
  float pbp[CPL];
  uint8_t pyl[CPL];
  // row offsets of d2-1 and d2
  int Rm1 = BAND ? row_off(m, d2_lo - 1) : 0, R = BAND ? row_off(m, d2_lo) : pad4(m + 1);
  auto fetch = [&](int d2, int Rd, int Rd2) {
    const int kmax = m - d2;
    const int e2 = d2 - 1;
    const int64_t ye = (int64_t)e2 * m - (int64_t)e2 * (e2 - 1) / 2;
    const int klo = max(cli, clj - d2), khi = min(min(chi, chj - d2), kmax);
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int k = k0 + 64 * c;
      const int l = k + d2;
      if (BAND && (kb + 64 * c > khi || kb + 64 * c + 63 < klo)) continue;  // whole slot outside
      pbp[c] = 0.0f;
      pGs[c] = 0.0;
      pyl[c] = 0;
      if (BAND) pK0[c] = pG0[c] = pK1[c] = pG1[c] = 0.0;
      const bool on = !BAND || (l >= clj && l <= chj && k >= cli && k <= chi);
      if (k <= kmax && on) {
        if (!BAND || l <= chjm1) {
          pK0[c] = A[Rd + k];
          pG0[c] = A[cp + Rd + k];
        }
        if (!BAND || k >= cli1) {
          pK1[c] = B[2 * cp + Rd + k];
          pG1[c] = B[3 * cp + Rd + k];
        }
        if (stack_on) {
          pbp[c] = bpy[ye + k];
          pyl[c] = ys[k + d2 - 1];
          // cell (k+1, l-1) of plane (i+1, j-1): inside its constraints (on
          // its diagonal row, l-1 inside them) unless that plane is (j-1,j-1)
          const bool cg_on = !cg_guard || (l - 1 >= cljm1 && l - 1 <= chjm1 &&
                                           (d2 == 2 || (k + 1 >= cli1 && k + 1 <= chi1)));
          if (d2 >= 2 && cg_on) pGs[c] = Cg[Rd2 + k + 1];
        }
      }
    }
  };
  if (d2_lo <= d2_hi) fetch(d2_lo, R, d2_lo >= 2 ? row_off(m, d2_lo - 2) : 0);
  for (int d2 = d2_lo; d2 <= d2_hi; ++d2) {
    double cK0[CPL], cG0[CPL], cK1[CPL], cG1[CPL], cGs[CPL];
    float cbp[CPL];
    uint8_t cyl[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      cK0[c] = pK0[c];
      cG0[c] = pG0[c];
      cK1[c] = pK1[c];
      cG1[c] = pG1[c];
      cGs[c] = pGs[c];
      cbp[c] = pbp[c];
      cyl[c] = pyl[c];
    }
    const int Rn = R + pad4(m + 1 - d2);
    if (d2 + 1 <= d2_hi) fetch(d2 + 1, Rn, Rm1);
    // K3/G3 of (k+1, l): my next cell, or the next lane's first (span d2-1)
    double K3n[CPL], G3n[CPL];
    // the last slot's neighbour: the right tile's first cell, span d2-1
    double rk = 0.0, rg = 0.0;
    if (has_right) {
      rk = bnd_r[d2 - 1];
      rg = bnd_r[bstride + d2 - 1];
    }
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      // lane 63's neighbour k+1 is lane 0 of the next slot
      const double hk = c + 1 < CPL ? bcast_lane0(K3[c + 1 < CPL ? c + 1 : c]) : rk;
      const double hg = c + 1 < CPL ? bcast_lane0(G3[c + 1 < CPL ? c + 1 : c]) : rg;
      K3n[c] = wave_shl1(K3[c], hk);
      G3n[c] = wave_shl1(G3[c], hg);
    }
    const int kmax = m - d2;
    // partial DP: the row's cells inside the constraints, k in [klo, khi]
    const int klo = max(cli, clj - d2), khi = min(min(chi, chj - d2), kmax);
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      if (BAND && (kb + 64 * c > khi || kb + 64 * c + 63 < klo)) {  // whole slot outside (wave-uniform)
        K2[c] = G2[c] = K3[c] = G3[c] = 0.0;
        continue;
      }
      const int k = k0 + 64 * c;
      if (k <= kmax) {
        const int l = k + d2;
        const bool on = !BAND || (l >= clj && l <= chj && k >= cli && k <= chi);
        // dp_init (:85-96); banded: partial_dp's boundary cases (:179-236)
        double K0 = cK0[c];
        double G0 = cG0[c] * g;
        double K1 = cK1[c];
        double G1 = cG1[c] * g;
        double k2 = K2[c], g2 = G2[c] * g;
        double k3 = K3n[c], g3 = G3n[c] * g;
        if (BAND && on) {
          if (l > chjm1) {  // K0(i,j-1,k,c_high[j-1]), G0 * g * g
            const int o = row_off(m, chjm1 - k) + k;
            K0 = A[o];
            G0 = A[cp + o] * g * g;
          }
          if (k < cli1) {  // K1(i+1,j,c_low[i+1],l), G1 * g * g
            const int o = row_off(m, l - cli1) + cli1;
            K1 = B[2 * cp + o];
            G1 = B[3 * cp + o] * g * g;
          }
          if (!(l - 1 >= clj || k == l - 1)) k2 = g2 = 0.0;  // diagonal K3/G3 are zero
          if (!(k + 1 <= chi)) k3 = g3 = 0.0;
        }
        if (stack_on && on) {  // :327-340
          const float bp_kl = cbp[c];
          if (bp_kl > bound) {
            const double g0 = cGs[c];
            if (xi == yk[c] && xj == cyl[c]) {
              k3 += g0 * stk * (double)bp_ij * (double)bp_kl;
              g3 += g0;
            } else {
              k3 += g0 * stk * sub * (double)bp_ij * (double)bp_kl;
            }
          }
        }
        // dp_update (:98-111)
        k2 += k3;
        g2 += g3;
        K1 += k2;
        G1 += g2;
        K0 += K1;
        G0 += G1;
        if (BAND && !on) K0 = G0 = K1 = G1 = k2 = g2 = k3 = g3 = 0.0;  // outside: zero state
        if (on) {
          cur[R + k] = K0;
          cur[cp + R + k] = G0;
          cur[2 * cp + R + k] = K1;
          cur[3 * cp + R + k] = G1;
        }
        K2[c] = k2;
        G2[c] = g2;
        K3[c] = k3;
        G3[c] = g3;
        if (d2 == m && i == 0 && j == n) P.out[pr.out_index] = K0;  // K0(0,n,0,m)
      }
    }
    if (bnd_w && lane == 0) {
      bnd_w[d2] = K3[0];
      bnd_w[bstride + d2] = G3[0];
    }
    Rm1 = R;
    R = Rn;
  }
  if (kbnd) {  // the next tile's lanes read what lane 0 stored
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  }  // k tiles
  if (m == 0 && i == 0 && j == n && lane == 0) P.out[pr.out_index] = 1.0;
}

// full_dp (no band) with the K chain summed.  For k < l, dp_init/dp_update
// (:85-111) make K3(c) = K3(i,j,k+1,l) + src(c), K2(c) = K2(i,j,k,l-1) + K3(c),
// K1(c) = K1(i+1,j,k,l) + K2(c), K0(c) = K0(i,j-1,k,l) + K1(c), where src(c)
// is the stacking term (:325-331), K1/K2/K3 are zero on their boundaries
// (the (j,j) planes and the diagonal cells, :294-297, :311-314) and K0 is 1 on
// the (j,j) planes.  Unrolled, K0(0,n,0,m) = 1 + sum of src over every cell
// i < j, k < l: each source reaches the result with coefficient one, and no
// K value is read for anything else.  So only G0 and G1 go to HBM (16 B
// written and 16 + 8 B read per cell instead of 32 + 40), K2/K3 leave the
// registers, each plane's wave sums its sources (fixed lane order) into the
// pair's accumulator of its i (acc[i], one writer per launch; a pair's spans
// run in order on one stream), and the wave of the last plane (0, n) forms
// 1 + sum_i acc[i] in i order: deterministic, equal to the reference's chain
// up to the association of non-negative sums.  Plane layout: G0 at 0, G1 at
// cp; acc follows the pair's ring.  k tiles (|y| >= 512) hand G3 on as in the
// 4-state kernel.
template <int CPL>
__global__ void __launch_bounds__(256) sk_stem4d_gsum_kernel(Stem4dLaunch P) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t it = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave;
  if (it >= P.n_items) return;
  const int2 item = P.items[it];  // {pair slot, i}
  const Stem4dPair pr = P.pairs[item.x];
  const int i = item.y, d1 = P.d1, j = i + d1;
  const int n = pr.n, m = pr.m;
  const int64_t cp = pr.plane_doubles;  // per state
  const int64_t ps = 2 * cp;            // plane stride (G0, G1)
  double* ring = P.scratch + pr.scratch_off;
  double* acc = ring + (int64_t)3 * (n + 1) * ps;
  double* __restrict__ cur = ring + (int64_t)(d1 % 3) * (n + 1) * ps + (int64_t)i * ps;
  const double g = P.gap;
  constexpr int TW = 64 * CPL;
  const int ntile = (m + TW) / TW;

  if (d1 == 0) {  // plane (j,j): G0 = g^(l-k), G1 = 0  (:297-309); acc[j] = 0
    for (int kt = 0; kt < ntile; ++kt) {
      const int k0 = kt * TW + lane;
      int R = 0;
      for (int d2 = 0; d2 <= m; ++d2) {
        const double gd = P.gpow[d2];
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          const int k = k0 + 64 * c;
          if (k <= m - d2) {
            cur[R + k] = gd;
            cur[cp + R + k] = 0.0;
          }
        }
        R += pad4(m + 1 - d2);
      }
    }
    if (lane == 0) {
      acc[i] = 0.0;
      if (n == 0) P.out[pr.out_index] = 1.0;
    }
    return;
  }

  const double* span_p1 = ring + (int64_t)((d1 - 1) % 3) * (n + 1) * ps;
  const double* __restrict__ A = span_p1 + (int64_t)i * ps;        // plane (i, j-1): G0
  const double* __restrict__ B = span_p1 + (int64_t)(i + 1) * ps;  // plane (i+1, j): G0, G1
  const double* Cg = d1 >= 2 ? ring + (int64_t)((d1 - 2) % 3) * (n + 1) * ps + (int64_t)(i + 1) * ps
                             : nullptr;  // plane (i+1, j-1), G0
  const float* bpx = P.bpdiag + pr.x_bp;  // prob(a, a+e) at e*n - e*(e-1)/2 + a
  const float* bpy = P.bpdiag + pr.y_bp;
  const uint8_t* xs = P.chars + pr.x_chr;
  const uint8_t* ys = P.chars + pr.y_chr;
  const float bound = P.bp_bound;
  const int e1 = d1 - 1;  // bp_ij = prob(i, j-1) (:320)
  const float bp_ij = bpx[(int64_t)e1 * n - (int64_t)e1 * (e1 - 1) / 2 + i];
  const bool stack_on = bp_ij > bound && Cg != nullptr;
  const uint8_t xi = xs[i], xj = xs[j - 1];
  const double stk = P.stack, sub = P.subst;
  double ksrc = 0.0;  // this plane's sources
  // boundary columns of this plane: [2 parities][G3][span d2]
  double* kbnd = ntile > 1 ? P.kbound + it * P.kbound_stride : nullptr;
  const int bstride = m + 1;

  for (int kt = ntile - 1; kt >= 0; --kt) {
    const int kb = kt * TW;
    const int k0 = kb + lane;
    double* bnd_w = kbnd ? kbnd + (int64_t)(kt & 1) * bstride : nullptr;              // for tile kt-1
    const double* bnd_r = kbnd ? kbnd + (int64_t)((kt + 1) & 1) * bstride : nullptr;  // of tile kt+1
    const bool has_right = kt + 1 < ntile;
    if (bnd_w && lane == 0) bnd_w[0] = 0.0;  // span 0 (the diagonal): G3 = 0
    double G2[CPL], G3[CPL];
    uint8_t yk[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      G2[c] = G3[c] = 0.0;
      const int k = k0 + 64 * c;
      yk[c] = k < m ? ys[k] : 0;
    }
    // d2 = 0: cells (l,l): G0 = G0(i+1,j,l,l) g, G1 = 0  (:313-317)
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int k = k0 + 64 * c;
      if (k <= m) {
        cur[k] = B[k] * g;
        cur[cp + k] = 0.0;
      }
    }
    // row d2's inputs, prefetched during row d2-1: G0 of (i,j-1), G1 of
    // (i+1,j), prob_y(k, l-1), y[l-1] and G0(i+1,j-1) at (k+1, l-1)
    struct Row {
      double G0[CPL], G1[CPL], Gs[CPL];
      float bp[CPL];
      uint8_t yl[CPL];
    };
    Row p, q;
    int Rm1 = 0, R = pad4(m + 1);
    auto fetch = [&](Row& r, int d2, int Rd, int Rd2) __attribute__((always_inline)) {
      const int kmax = m - d2;
      const int e2 = d2 - 1;
      const int64_t ye = (int64_t)e2 * m - (int64_t)e2 * (e2 - 1) / 2;
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const int k = k0 + 64 * c;
        r.bp[c] = 0.0f;
        r.Gs[c] = 0.0;
        r.yl[c] = 0;
        if (k <= kmax) {
          r.G0[c] = A[Rd + k];
          r.G1[c] = B[cp + Rd + k];
          if (stack_on) {
            r.bp[c] = bpy[ye + k];
            r.yl[c] = ys[k + d2 - 1];
            if (d2 >= 2) r.Gs[c] = Cg[Rd2 + k + 1];
          }
        }
      }
    };
    // rows are fetched SK4_PF rows ahead (row 2 reads the stacking row 0)
    if (m >= 1) fetch(p, 1, R, 0);
    if (SK4_PF == 2 && m >= 2) fetch(q, 2, R + pad4(m), 0);
    for (int d2 = 1; d2 <= m; ++d2) {
      const Row cr = p;
      const double* cG0 = cr.G0;
      const double* cG1 = cr.G1;
      const double* cGs = cr.Gs;
      const float* cbp = cr.bp;
      const uint8_t* cyl = cr.yl;
      const int Rn = R + pad4(m + 1 - d2);
      if (SK4_PF == 2) {
        p = q;
        if (d2 + 2 <= m) fetch(q, d2 + 2, Rn + pad4(m - d2), R);
      } else if (d2 + 1 <= m) {
        fetch(p, d2 + 1, Rn, Rm1);
      }
      // G3 of (k+1, l): my next cell, or the next lane's first (span d2-1)
      const double rg = has_right ? bnd_r[d2 - 1] : 0.0;
      double G3n[CPL];
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const double hg = c + 1 < CPL ? bcast_lane0(G3[c + 1 < CPL ? c + 1 : c]) : rg;
        G3n[c] = wave_shl1(G3[c], hg);
      }
      const int kmax = m - d2;
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const int k = k0 + 64 * c;
        if (k <= kmax) {
          // dp_init (:85-96): G terms; the K terms are the sources below
          double G0 = cG0[c] * g;
          double G1 = cG1[c] * g;
          double g2 = G2[c] * g;
          double g3 = G3n[c] * g;
          if (stack_on) {  // :321-333
            const float bp_kl = cbp[c];
            if (bp_kl > bound) {
              const double g0 = cGs[c];
              if (xi == yk[c] && xj == cyl[c]) {
                ksrc += g0 * stk * (double)bp_ij * (double)bp_kl;
                g3 += g0;
              } else {
                ksrc += g0 * stk * sub * (double)bp_ij * (double)bp_kl;
              }
            }
          }
          // dp_update (:100-111)
          g2 += g3;
          G1 += g2;
          G0 += G1;
          cur[R + k] = G0;
          cur[cp + R + k] = G1;
          G2[c] = g2;
          G3[c] = g3;
        }
      }
      if (bnd_w && lane == 0) bnd_w[d2] = G3[0];
      Rm1 = R;
      R = Rn;
    }
    if (kbnd) {  // the next tile's lanes read what lane 0 stored
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
  }  // k tiles
  for (int off = 32; off > 0; off >>= 1) ksrc += __shfl_xor(ksrc, off, 64);
  if (lane == 0) acc[i] += ksrc;
  if (i == 0 && j == n) {  // the last plane: K0(0,n,0,m) = 1 + sum_i acc[i]
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane == 0) {
      double K = 0.0;
      for (int t = 0; t <= n; ++t) K += acc[t];
      P.out[pr.out_index] = 1.0 + K;
    }
  }
}

// full_dp with the K chain summed and each plane's stacking chain produced one
// span early.  A plane's G2 / G3 (and so its G1 = G1(i+1,j) g + G2) depend
// only on its stacking sources, s(k,l) = G0(i+1,j-1,k+1,l-1) when
// bp(i,j-1) and bp(k,l-1) pass the bound and the end bases match (:321-333).
// The wave of plane (i+1, j) streams exactly those G0 rows one span earlier
// (they are its A input, G0(i+1, j-1)), so it runs the chain of its consumer
// (i, j) too and writes, beside its own G0, the consumer's G1 pre-combined:
// B'(k,l) = G1(i+1,j,k,l) g + G2_(i,j)(k,l) -- the consumer's G1 in the
// reference's own operation order.  A plane then reads G0 of (i, j-1) and its
// B' (16 B per cell) and writes G0 and its consumer's B' (16 B): 32 B per cell
// against the K-sum kernel's 40 (no stacking read); its consumer's sources
// go to its own accumulator acc[i].  Single k tile (|y| < 512; the host runs
// the K-sum kernel otherwise).  Plane layout: G0 at 0, B' (for the plane
// (i-1, j)) at cp.
// SK4P_RANGE: the span kernel's rows as straight-line slots over
// range-checked buffers -- off: 318.5 / 315.8 against 336.5 pairs/s with the
// per-slot guards on one box (r04k), although it fits 128 VGPRs
#ifndef SK4P_RANGE
#define SK4P_RANGE 0
#endif
// SK4P_WPE (build-time): ask the register allocator for that many waves per
// SIMD (4: <= 128 VGPRs)
#ifdef SK4P_WPE
#define SK4P_ATTR __attribute__((amdgpu_waves_per_eu(SK4P_WPE)))
#else
#define SK4P_ATTR
#endif
template <int CPL>
__global__ void __launch_bounds__(256) SK4P_ATTR sk_stem4d_pre_kernel(Stem4dLaunch P) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t it = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave;
  if (it >= P.n_items) return;
  const int2 item = P.items[it];  // {pair slot, i}
  const Stem4dPair pr = P.pairs[item.x];
  const int i = item.y, d1 = P.d1, j = i + d1;
  const int n = pr.n, m = pr.m;
  const int64_t cp = pr.plane_doubles;
  const int64_t ps = 2 * cp;
  double* ring = P.scratch + pr.scratch_off;
  double* acc = ring + (int64_t)3 * (n + 1) * ps;
  double* __restrict__ cur = ring + (int64_t)(d1 % 3) * (n + 1) * ps + (int64_t)i * ps;
  const double g = P.gap;
  const int k0 = lane;

  if (d1 == 0) {  // plane (j,j): G0 = g^(l-k); B' of (j-1, j) = 0 (no sources: bp(j-1,j-1) = 0)
    int R = 0;
    for (int d2 = 0; d2 <= m; ++d2) {
      const double gd = P.gpow[d2];
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const int k = k0 + 64 * c;
        if (k <= m - d2) {
          cur[R + k] = gd;
          cur[cp + R + k] = 0.0;
        }
      }
      R += pad4(m + 1 - d2);
    }
    if (lane == 0) {
      acc[i] = 0.0;
      if (n == 0) P.out[pr.out_index] = 1.0;
    }
    return;
  }

  const double* span_p1 = ring + (int64_t)((d1 - 1) % 3) * (n + 1) * ps;
  const double* __restrict__ A = span_p1 + (int64_t)i * ps;        // plane (i, j-1): G0
  const double* __restrict__ B = span_p1 + (int64_t)(i + 1) * ps;  // plane (i+1, j): G0, this plane's B'
  const float* bpx = P.bpdiag + pr.x_bp;
  const float* bpy = P.bpdiag + pr.y_bp;
  const uint8_t* xs = P.chars + pr.x_chr;
  const uint8_t* ys = P.chars + pr.y_chr;
  const float bound = P.bp_bound;
  // the consumer: plane (i-1, j) of span d1+1, bp_c = prob(i-1, j-1) (:320)
  const bool cons = i >= 1;
  float bp_c = 0.0f;
  uint8_t xci = 0, xcj = 0;
  if (cons) {  // (wave-uniform: into SGPRs)
    const int e = d1;
    bp_c = __uint_as_float(__builtin_amdgcn_readfirstlane(
        __float_as_uint(bpx[(int64_t)e * n - (int64_t)e * (e - 1) / 2 + (i - 1)])));
    xci = (uint8_t)__builtin_amdgcn_readfirstlane(xs[i - 1]);
    xcj = (uint8_t)__builtin_amdgcn_readfirstlane(xs[j - 1]);
  }
  const bool stack_c = cons && bp_c > bound;
  const double stk = P.stack, sub = P.subst;
  double ksrc = 0.0;  // the consumer's sources

  uint8_t yk[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int k = k0 + 64 * c;
    yk[c] = k < m ? ys[k] : 0;
  }
  // d2 = 0: cells (l,l): G0 = G0(i+1,j,l,l) g (:313-317); the consumer's
  // G1 there is 0 (it reads its own diagonal from this plane's G0)
  double Am1[CPL], Am2[CPL], G2c[CPL], G3c[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int k = k0 + 64 * c;
    if (k <= m) {
      cur[k] = B[k] * g;
      cur[cp + k] = 0.0;
    }
    Am1[c] = (stack_c && k <= m) ? A[k] : 0.0;  // G0(i, j-1) diagonal: the sources of row 2
    Am2[c] = 0.0;
    G2c[c] = G3c[c] = 0.0;
  }
  struct Row {
    double A[CPL], Bp[CPL];
    float bp[CPL];
    uint8_t yl[CPL];
  };
  Row p, q;
  int R = pad4(m + 1);
  auto fetch = [&](Row& r, int d2, int Rd) __attribute__((always_inline)) {
    const int kmax = m - d2;
    const int e2 = d2 - 1;
    const int64_t ye = (int64_t)e2 * m - (int64_t)e2 * (e2 - 1) / 2;
#if SK4P_RANGE
    // range-checked buffers: loads past kmax return 0, no per-slot guards
    const int nk = kmax + 1;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      r.A[c] = s4c_ld64(A + Rd, nk, c, lane);
      r.Bp[c] = s4c_ld64(B + cp + Rd, nk, c, lane);
      r.bp[c] = 0.0f;
      r.yl[c] = 0;
    }
    if (stack_c) {
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        r.bp[c] = s4c_ld32(bpy + ye, nk, c, lane);
        r.yl[c] = s4c_ld8(ys + d2 - 1, nk, c, lane);
      }
    }
    return;
#endif
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int k = k0 + 64 * c;
      r.A[c] = 0.0;
      r.Bp[c] = 0.0;
      r.bp[c] = 0.0f;
      r.yl[c] = 0;
      if (k <= kmax) {
        r.A[c] = A[Rd + k];
        r.Bp[c] = B[cp + Rd + k];
        if (stack_c) {
          r.bp[c] = bpy[ye + k];
          r.yl[c] = ys[k + d2 - 1];
        }
      }
    }
  };
  if (m >= 1) fetch(p, 1, R);
  if (SK4_PF == 2 && m >= 2) fetch(q, 2, R + pad4(m));
  for (int d2 = 1; d2 <= m; ++d2) {
    const Row cr = p;
    const int Rn = R + pad4(m + 1 - d2);
    if (SK4_PF == 2) {
      p = q;
      if (d2 + 2 <= m) fetch(q, d2 + 2, Rn + pad4(m - d2));
    } else if (d2 + 1 <= m) {
      fetch(p, d2 + 1, Rn);
    }
    // the consumer's G3 at (k+1, l) (row d2-1) and G0(i, j-1) at (k+1, l-1)
    // (row d2-2): the next lane's, or the next slot's lane 0
    double G3n[CPL], A2[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const double hg = c + 1 < CPL ? bcast_lane0(G3c[c + 1 < CPL ? c + 1 : c]) : 0.0;
      const double ha = c + 1 < CPL ? bcast_lane0(Am2[c + 1 < CPL ? c + 1 : c]) : 0.0;
      G3n[c] = wave_shl1(G3c[c], hg);
      A2[c] = wave_shl1(Am2[c], ha);
    }
    const int kmax = m - d2;
#if SK4P_RANGE
    {  // straight-line slots (as in sk_stem4d_col_kernel): stores past kmax are
       // dropped by the buffer range, lanes past it feed no valid cell and add
       // nothing to K
      const bool stk_row = stack_c && d2 >= 2;
      const double bpc = (double)bp_c;
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const int k = k0 + 64 * c;
        const double G1 = cr.Bp[c];
        double G0 = cr.A[c] * g;
        G0 += G1;
        s4c_st64(cur + R, kmax + 1, c, lane, G0);
        if (cons) {
          double g3 = G3n[c] * g;
          if (stk_row) {
            const float bp_kl = cr.bp[c];
            const bool src = bp_kl > bound && k <= kmax;
            const bool match = xci == yk[c] && xcj == cr.yl[c];
            const double g0 = A2[c];
            const double t0 = g0 * stk;
            const double tm = match ? t0 : t0 * sub;
            const double term = tm * bpc * (double)bp_kl;
            ksrc += src ? term : 0.0;
            g3 += src && match ? g0 : 0.0;
          }
          double g2 = G2c[c] * g;
          g2 += g3;
          double Bn = G1 * g;
          Bn += g2;
          s4c_st64(cur + cp + R, kmax + 1, c, lane, Bn);
          G2c[c] = g2;
          G3c[c] = g3;
        }
      }
    }
    if (SK4P_RANGE) {
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        Am2[c] = Am1[c];
        Am1[c] = cr.A[c];
      }
      R = Rn;
      continue;
    }
#endif
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int k = k0 + 64 * c;
      if (k <= kmax) {
        // this plane: G1 = B' (its G1, formed by the plane (i+1, j)), G0 (:85-111)
        const double G1 = cr.Bp[c];
        double G0 = cr.A[c] * g;
        G0 += G1;
        cur[R + k] = G0;
        if (cons) {  // the consumer (i-1, j): dp_init / stacking / dp_update of its G chain
          double g3 = G3n[c] * g;
          if (stack_c && d2 >= 2) {
            const float bp_kl = cr.bp[c];
            if (bp_kl > bound) {
              const double g0 = A2[c];
              if (xci == yk[c] && xcj == cr.yl[c]) {
                ksrc += g0 * stk * (double)bp_c * (double)bp_kl;
                g3 += g0;
              } else {
                ksrc += g0 * stk * sub * (double)bp_c * (double)bp_kl;
              }
            }
          }
          double g2 = G2c[c] * g;
          g2 += g3;
          double Bn = G1 * g;
          Bn += g2;
          cur[cp + R + k] = Bn;
          G2c[c] = g2;
          G3c[c] = g3;
        }
      }
    }
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      Am2[c] = Am1[c];
      Am1[c] = cr.A[c];
    }
    R = Rn;
  }
  for (int off = 32; off > 0; off >>= 1) ksrc += __shfl_xor(ksrc, off, 64);
  if (lane == 0) acc[i] += ksrc;
  if (i == 0 && j == n) {  // the last plane: K0(0,n,0,m) = 1 + sum_i acc[i]
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane == 0) {
      double K = 0.0;
      for (int t = 0; t <= n; ++t) K += acc[t];
      P.out[pr.out_index] = 1.0 + K;
    }
  }
}

// full_dp, column-pipelined (r04): one WORKGROUP per pair walks the x
// columns j = 1..n, and in column j the planes i = j-1, j-2, ..., 0, which
// its W waves take in turn, each wave one row (y span d2) behind the previous.
// Plane (i, j) needs G0(i, j-1) (the previous column's plane i, HBM) and its
// pre-combined G1, B'(i, j) = G1(i+1, j) g + G2_(i,j), which the wave of plane
// (i+1, j) forms from ITS A input -- G0(i+1, j-1), the stacking sources of
// (i, j) -- one step earlier (the scheme of sk_stem4d_pre_kernel).  Here B'
// goes from wave w to wave w+1 through an LDS double buffer instead of HBM,
// so a cell costs the G0 read of (i, j-1) and the G0 write of (i, j) (in
// place: plane slot i holds G0(i, j) of the latest column): 16 B, plus 16 B
// for every W-th plane, whose B' crosses the round wrap (wave W-1 -> wave 0,
// R - W + 1 steps later) through one plane-sized HBM buffer per pair.
//
// Schedule: positions p = 0, 1, ... run column by column; column j holds its
// j planes (i = j-1 at offset 0) and then bubbles up to c_j = max(j, PF + 1)
// positions, PF = 2 rows fetched ahead.  Position p is wave p % W's plane of
// round p / W, and wave w processes row s of it at step T(p) + s, T(p) =
// (p / W) R + p % W, R = m + 1 rows; one workgroup barrier per step.  Since
// R >= W + PF + 1 (the host's choice of W), T is increasing with
// T(p2) - T(p1) >= p2 - p1, so:
//  * B' of row s is written by wave w-1 at step t-1 and read by wave w at
//    step t (LDS slot t & 1), or, at the wrap, at least PF + 1 steps later;
//  * the A row s + PF that a plane prefetches at step T(p) + s was written
//    (by the previous column's plane i, >= PF + 2 positions earlier) at a
//    step before that;
//  * row 0 is never stored: G0(i, j, l, l) = g^(j-i) (the repeated products
//    of gap_powers, as the chain G0(i+1,j,l,l) g forms it, :313-317).
// The K chain is summed (sk_stem4d_gsum_kernel): every lane keeps one running
// sum of its consumers' stacking sources over all its planes; the pair's
// K = 1 + the waves' lane-reduced sums in wave order.
#ifndef SK4C_PF
#define SK4C_PF 2  // rows fetched ahead
#endif

// Barriers: between steps only the LDS B' rows need to be visible, so most
// barriers wait for LDS traffic alone (lgkmcnt) -- a workgroup release of
// global memory would wait for every outstanding vector memory op (vmcnt:
// the prefetched rows too), i.e. pay the HBM latency every step.  Every F-th
// barrier (P.col_f; the one before step t, t % F == 0) is a full one, so a
// global store of step u is visible from the first multiple of F above u
// on: readers of global data need a lag of F + PF steps -- column j holds
// c_j = max(j, F + 2) positions, and W <= m - F - 1 (the round wrap).
//
// Between the full barriers the waves need not run in lockstep (SK4C_P2P):
// wave w publishes in LDS the number of steps it has completed, and waits
// only for what it touches -- its producer's step t-1 before it reads link
// slot (t-1) % D, its consumer's step t-D+1 before it overwrites slot t % D
// -- so a wave held up by a late row delays its consumers alone and not the
// whole workgroup.  Every wait is on a strictly earlier step, so there is no
// cycle; a wait that runs past ~0.5 s gives up and the pair's K is NaN.
#ifndef SK4C_RANGE  // 1: the row step as straight-line slots over range-checked buffers
#define SK4C_RANGE 0   // (off: 260 against 306 pairs/s with the per-slot guards, r04k)
#endif
#ifndef SK4C_P2P  // off: 278 against 305 pairs/s lockstep on C3 (r04e)
#define SK4C_P2P 0
#endif
#ifndef SK4C_D  // link slots per wave (a power of 2; 2 when lockstep)
#define SK4C_D (SK4C_P2P ? 4 : 2)
#endif
static_assert(SK4C_D >= 2 && (SK4C_D & (SK4C_D - 1)) == 0, "SK4C_D: a power of 2");

__device__ __forceinline__ void s4c_publish(int* done, int v) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __hip_atomic_store(done, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void s4c_wait_ge(const int* done, int v, bool& bad) {
  if (bad) return;
  int it = 0;
  while (__builtin_amdgcn_readfirstlane(
             __hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < v) {
    __builtin_amdgcn_s_sleep(1);
    if (++it > (1 << 23)) {
      bad = true;
      break;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}


__device__ __forceinline__ int s4c_cols(int j, int F) { return j > F + SK4C_PF ? j : F + SK4C_PF; }

// position -> plane of the column schedule; advance() moves on by W positions
struct S4cPos {
  int j = 1, off = 0;  // column, offset in the column (i = j - 1 - off; off >= j: bubble)
  __device__ void advance(int W, int n, int F) {
    off += W;
    while (j <= n && off >= s4c_cols(j, F)) {
      off -= s4c_cols(j, F);
      ++j;
    }
  }
  __device__ bool valid(int n) const { return j <= n; }
  __device__ bool plane(int n) const { return j <= n && off < j; }
  __device__ int i() const { return j - 1 - off; }
};

// waves per workgroup at most: 4, 3 and 2 per SIMD (the register budget)
#ifndef SK4C_W4  // waves per workgroup of the CPL 4 class (12: 3 per SIMD; 16 needs SK4C_PF 1)
#define SK4C_W4 12
#endif
template <int CPL>
constexpr int s4c_max_waves() {
  return CPL <= 2 ? 16 : CPL == 4 ? SK4C_W4 : 8;
}

template <int CPL>
__global__ void __launch_bounds__(64 * s4c_max_waves<CPL>()) sk_stem4d_col_kernel(Stem4dLaunch P) {
  extern __shared__ __attribute__((aligned(16))) double s4c_lds[];
  constexpr int TW = 64 * CPL;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int W = blockDim.x >> 6;
  const Stem4dPair pr = P.pairs[blockIdx.x];
  const int n = pr.n, m = pr.m, R = m + 1;
  const int64_t cp = pr.plane_doubles;
  double* __restrict__ planes = P.scratch + pr.scratch_off;  // slot i: G0(i, latest j)
  double* __restrict__ wrapb = planes + (int64_t)n * cp;     // B' across the round wrap
  const float* bpx = P.bpdiag + pr.x_bp;
  const float* bpy = P.bpdiag + pr.y_bp;
  const uint8_t* xs = P.chars + pr.x_chr;
  const uint8_t* ys = P.chars + pr.y_chr;
  const double* gpow = P.gpow;
  const float bound = P.bp_bound;
  const double g = P.gap, stk = P.stack, sub = P.subst;
  const int F = max(P.col_f, 1);
  // links: wave w writes link w (slot t % D), wave w+1 reads it a step later
  constexpr int D = SK4C_D;
  double* link_out = s4c_lds + (int64_t)w * D * TW;
  const double* link_in = s4c_lds + (int64_t)(w - 1) * D * TW;
  double* red = s4c_lds + (int64_t)W * D * TW;  // W per-wave sums
  int* done = reinterpret_cast<int*>(red + W);  // W step counters (SK4C_P2P)
  bool bad = false;

  // steps: T(last position) + R
  int64_t np = 0;
  for (int j = 1; j <= n; ++j) np += s4c_cols(j, F);
  const int64_t total = np > 0 ? ((np - 1) / W) * R + (np - 1) % W + R : 0;

  // per-plane constants of the plane at a position
  struct Plane {
    int i, j;
    bool on, first, cons, stack;
    float bp_c;
    uint8_t xci, xcj;
  };
  auto describe = [&](const S4cPos& q) __attribute__((always_inline)) -> Plane {
    Plane d;
    d.on = q.plane(n);
    d.i = d.on ? q.i() : 0;
    d.j = d.on ? q.j : 1;
    d.first = d.i == d.j - 1;
    d.cons = d.on && d.i >= 1;
    d.bp_c = 0.0f;
    d.xci = d.xcj = 0;
    if (d.cons) {  // the consumer (i-1, j): bp(i-1, j-1) (:320)
      // (wave-uniform loads made uniform in SGPRs: the plane's branches on
      // them are then scalar branches, not exec-mask juggling per slot)
      const int e = d.j - d.i;
      d.bp_c = __uint_as_float(__builtin_amdgcn_readfirstlane(
          __float_as_uint(bpx[(int64_t)e * n - (int64_t)e * (e - 1) / 2 + (d.i - 1)])));
      d.xci = (uint8_t)__builtin_amdgcn_readfirstlane(xs[d.i - 1]);
      d.xcj = (uint8_t)__builtin_amdgcn_readfirstlane(xs[d.j - 1]);
    }
    d.stack = d.cons && d.bp_c > bound;
    return d;
  };
  // one row's HBM inputs, fetched PF rows ahead: G0(i, j-1) (A), the wrap
  // B' (wave 0 of a non-first plane), prob_y(k, l-1), y[l-1]
  struct Row {
    double A[CPL], Bw[CPL];
    float bp[CPL];
    uint8_t yl[CPL];  // y[l-1], compared at the row's step: an operation on a
                      // loaded value here would wait for the load (no prefetch)
  };
#if SK4C_RANGE
  auto fetch = [&](Row& r, const Plane& d, int s) __attribute__((always_inline)) {
    // cells k <= m - s of the row; past them every load returns 0 (buffer
    // range), the branches below are on wave-uniform values
    const int nk = d.on && s >= 1 ? m - s + 1 : 0;
    const int ro = row_off(m, s);
    const int e2 = s - 1;
    const int64_t ye = (int64_t)e2 * m - (int64_t)e2 * (e2 - 1) / 2;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      r.A[c] = r.Bw[c] = 0.0;
      r.bp[c] = 0.0f;
      r.yl[c] = 0;
    }
    if (nk == 0) return;
    if (d.first) {  // G0(j-1, j-1) = g^(l-k)
      const double gs = gpow[s];
#pragma unroll
      for (int c = 0; c < CPL; ++c) r.A[c] = lane + 64 * c < nk ? gs : 0.0;
    } else {
#pragma unroll
      for (int c = 0; c < CPL; ++c) r.A[c] = s4c_ld64(planes + (int64_t)d.i * cp + ro, nk, c, lane);
      if (w == 0) {  // the round wrap's B'
#pragma unroll
        for (int c = 0; c < CPL; ++c) r.Bw[c] = s4c_ld64(wrapb + ro, nk, c, lane);
      }
    }
    if (d.stack) {
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        r.bp[c] = s4c_ld32(bpy + ye, nk, c, lane);
        r.yl[c] = s4c_ld8(ys + s - 1, nk, c, lane);
      }
    }
  };
#else
  auto fetch = [&](Row& r, const Plane& d, int s) __attribute__((always_inline)) {
    const int kmax = m - s;
    const int ro = row_off(m, s);
    const int e2 = s - 1;
    const int64_t ye = (int64_t)e2 * m - (int64_t)e2 * (e2 - 1) / 2;
    const double* Ai = planes + (int64_t)d.i * cp + ro;
    const bool wrap_in = w == 0 && !d.first;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int k = lane + 64 * c;
      r.A[c] = 0.0;
      r.Bw[c] = 0.0;
      r.bp[c] = 0.0f;
      r.yl[c] = 0;

      if (d.on && s >= 1 && k <= kmax) {
        r.A[c] = d.first ? gpow[s] : Ai[k];  // G0(j-1, j-1) = g^(l-k)
        if (wrap_in) r.Bw[c] = wrapb[ro + k];
        if (d.stack) {
          r.bp[c] = bpy[ye + k];
          r.yl[c] = ys[k + s - 1];
        }
      }
    }
  };
#endif

  uint32_t yk = 0;  // y[k] of slot c in byte c (CPL <= 4), else reread per plane
#pragma unroll
  for (int c = 0; c < CPL && c < 4; ++c) {
    const int k = lane + 64 * c;
    yk |= (uint32_t)(k < m ? ys[k] : 0) << (8 * c);
  }
  uint32_t xkm = 0;  // bit c: y[k] == x[i-1] of the consumer (per plane)
  double ksrc = 0.0;
  double Am1[CPL], Am2[CPL], G2c[CPL], G3c[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) Am1[c] = Am2[c] = G2c[c] = G3c[c] = 0.0;

  // this wave's position (p = w) and the fetch cursor PF rows ahead
  S4cPos cur;
  cur.advance(w, n, F);  // from position 0
  Plane dc = describe(cur);
  S4cPos fpos = cur;
  Plane df = dc;
  int fs = 0;  // fetch cursor: (fpos, fs)
  Row rq[SK4C_PF];  // rows fetched ahead, oldest first
  auto fetch_next = [&](Row& r) __attribute__((always_inline)) {
    fetch(r, df, fs);
    if (++fs == R) {
      fs = 0;
      fpos.advance(W, n, F);
      df = describe(fpos);
    }
  };
  // a wave's first rows are fetched PF steps before its first step (t = w),
  // not earlier: their A rows may be written in the steps before
#pragma unroll
  for (int q = 0; q < SK4C_PF; ++q)
    if (w - SK4C_PF + q < 0) fetch_next(rq[q]);
  int s = 0;
#if SK4C_P2P
  done[w] = cur.valid(n) ? 0 : INT_MAX;
  __syncthreads();
#endif

  for (int64_t t = 0; t < total; ++t) {
    if (t > 0) {  // (every wave takes every barrier)
      if (t % F == 0) {
        __syncthreads();
      } else if (!SK4C_P2P) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
      }
    }
    if (!cur.valid(n)) continue;
    if (t < w) {
#pragma unroll
      for (int q = 0; q < SK4C_PF; ++q)
        if (t == w - SK4C_PF + q) fetch_next(rq[q]);
      if (SK4C_P2P) s4c_publish(done + w, (int)t + 1);
      continue;
    }
    const Row cr = rq[0];
#pragma unroll
    for (int q = 0; q + 1 < SK4C_PF; ++q) rq[q] = rq[q + 1];
    fetch_next(rq[SK4C_PF - 1]);
    if (dc.on) {
      const int kmax = m - s;
      if (s == 0) {  // cells (l, l): G0 = g^(j-i), never stored; chain registers reset
        xkm = 0u;
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          const int k = lane + 64 * c;
          const uint32_t ykc = c < 4 ? (yk >> (8 * (c & 3))) & 0xffu : (k < m ? ys[k] : 0u);
          xkm |= (dc.stack && ykc == dc.xci ? 1u : 0u) << c;
        }
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          const int k = lane + 64 * c;
          Am1[c] = (dc.stack && k <= m) ? gpow[dc.j - 1 - dc.i] : 0.0;  // G0(i, j-1, l, l)
          Am2[c] = G2c[c] = G3c[c] = 0.0;
        }
#if SK4C_RANGE
      } else {
        // Straight-line slots: lanes past kmax compute values that are never
        // stored (the output buffers' range ends at kmax) nor read by a valid
        // cell of a later row (a cell reads k+1 of the row before, valid
        // there), and add nothing to K (their bp loads are 0 and masked)
        const int ro = row_off(m, s);
        const int nk = kmax + 1;
        double* const gout = planes + (int64_t)dc.i * cp + ro;
        const bool wrap_in = w == 0;
        const double* lin = link_in + ((t - 1) & (D - 1)) * TW;
        double* lout = dc.cons && w + 1 < W ? link_out + (t & (D - 1)) * TW : nullptr;
        const int nk_wrap = dc.cons && !lout ? nk : 0;
        if (SK4C_P2P) {
          if (!dc.first && !wrap_in) s4c_wait_ge(done + w - 1, (int)t, bad);
          if (lout) s4c_wait_ge(done + w + 1, (int)t - D + 2, bad);
        }
        const bool stk_row = dc.stack && s >= 2;
        const double bpc = (double)dc.bp_c;
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          // the consumer's G3 at (k+1, l) (row s-1) and G0(i, j-1) at
          // (k+1, l-1): the next lane's, or the next slot's lane 0 -- formed
          // here, before slot c's update, while slot c+1's is still the old
          // row's (short live ranges: the registers of 4 waves per SIMD)
          const double hg = c + 1 < CPL ? bcast_lane0(G3c[c + 1 < CPL ? c + 1 : c]) : 0.0;
          const double ha = c + 1 < CPL ? bcast_lane0(Am2[c + 1 < CPL ? c + 1 : c]) : 0.0;
          const double G3n = wave_shl1(G3c[c], hg);
          const double A2 = wave_shl1(Am2[c], ha);
          const int k = lane + 64 * c;
          // this plane: G1 = B' (formed by the plane (i+1, j)), G0 (:85-111)
          const double G1 = dc.first ? 0.0 : wrap_in ? cr.Bw[c] : lin[k];
          double G0 = cr.A[c] * g;
          G0 += G1;
          s4c_st64(gout, nk, c, lane, G0);
          if (dc.cons) {  // the consumer (i-1, j): dp_init / stacking / dp_update of its G chain
            double g3 = G3n * g;
            if (stk_row) {
              const float bp_kl = cr.bp[c];
              const bool src = bp_kl > bound && k <= kmax;
              const bool match = ((xkm >> c) & 1u) && cr.yl[c] == dc.xcj;
              const double g0 = A2;
              // the reference's products in its order; +0 where no source
              const double t0 = g0 * stk;
              const double tm = match ? t0 : t0 * sub;
              const double term = tm * bpc * (double)bp_kl;
              ksrc += src ? term : 0.0;
              g3 += src && match ? g0 : 0.0;
            }
            double g2 = G2c[c] * g;
            g2 += g3;
            double Bn = G1 * g;
            Bn += g2;
            if (lout) lout[k] = Bn;
            else s4c_st64(wrapb + ro, nk_wrap, c, lane, Bn);
            G2c[c] = g2;
            G3c[c] = g3;
          }
        }
#else
      } else {
        const int ro = row_off(m, s);
        double* __restrict__ out = planes + (int64_t)dc.i * cp + ro;
        const bool wrap_in = w == 0;
        const double* lin = link_in + ((t - 1) & (D - 1)) * TW;
        double* lout = dc.cons && w + 1 < W ? link_out + (t & (D - 1)) * TW : nullptr;
        if (SK4C_P2P) {
          if (!dc.first && !wrap_in) s4c_wait_ge(done + w - 1, (int)t, bad);
          if (lout) s4c_wait_ge(done + w + 1, (int)t - D + 2, bad);
        }
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          // the consumer's G3 at (k+1, l) (row s-1) and G0(i, j-1) at
          // (k+1, l-1): the next lane's, or the next slot's lane 0 -- formed
          // here, before slot c's update, while slot c+1's is still the old
          // row's (short live ranges: the registers of 4 waves per SIMD)
          const double hg = c + 1 < CPL ? bcast_lane0(G3c[c + 1 < CPL ? c + 1 : c]) : 0.0;
          const double ha = c + 1 < CPL ? bcast_lane0(Am2[c + 1 < CPL ? c + 1 : c]) : 0.0;
          const double G3n = wave_shl1(G3c[c], hg);
          const double A2 = wave_shl1(Am2[c], ha);
          const int k = lane + 64 * c;
          if (k <= kmax) {
            // this plane: G1 = B' (formed by the plane (i+1, j)), G0 (:85-111)
            const double G1 = dc.first ? 0.0 : wrap_in ? cr.Bw[c] : lin[k];
            double G0 = cr.A[c] * g;
            G0 += G1;
            out[k] = G0;
            if (dc.cons) {  // the consumer (i-1, j): dp_init / stacking / dp_update of its G chain
              double g3 = G3n * g;
              if (dc.stack && s >= 2) {
                const float bp_kl = cr.bp[c];
                if (bp_kl > bound) {
                  const double g0 = A2;
                  if (((xkm >> c) & 1u) && cr.yl[c] == dc.xcj) {
                    ksrc += g0 * stk * (double)dc.bp_c * (double)bp_kl;
                    g3 += g0;
                  } else {
                    ksrc += g0 * stk * sub * (double)dc.bp_c * (double)bp_kl;
                  }
                }
              }
              double g2 = G2c[c] * g;
              g2 += g3;
              double Bn = G1 * g;
              Bn += g2;
              if (lout) lout[k] = Bn;
              else wrapb[ro + k] = Bn;
              G2c[c] = g2;
              G3c[c] = g3;
            }
          }
        }
#endif
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          Am2[c] = Am1[c];
          Am1[c] = cr.A[c];
        }
      }
    }
    if (++s == R) {
      s = 0;
      cur.advance(W, n, F);
      dc = describe(cur);
    }
    if (SK4C_P2P) s4c_publish(done + w, cur.valid(n) ? (int)t + 1 : INT_MAX);
  }
  for (int off = 32; off > 0; off >>= 1) ksrc += __shfl_xor(ksrc, off, 64);
  if (lane == 0) red[w] = bad ? __builtin_nan("") : ksrc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double K = 0.0;
    for (int v = 0; v < W; ++v) K += red[v];
    P.out[pr.out_index] = 1.0 + K;
  }
}

int stem4d_col_max_waves(int cpl) {
  return cpl <= 2 ? s4c_max_waves<2>() : cpl == 4 ? s4c_max_waves<4>() : s4c_max_waves<8>();
}

size_t stem4d_col_lds_bytes(int cpl, int waves) {
  return ((size_t)waves * SK4C_D * 64 * cpl + 2 * waves) * sizeof(double);
}

hipError_t launch_stem4d_col(const Stem4dLaunch& P, int64_t n_pairs, int cpl, int waves,
                             hipStream_t st) {
  if (n_pairs == 0) return hipSuccess;
  const size_t lds = stem4d_col_lds_bytes(cpl, waves);
  const dim3 grid((unsigned)n_pairs), block(64 * waves);
#define SK_L(C)                                                                                   \
  {                                                                                               \
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(sk_stem4d_col_kernel<C>),    \
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);     \
    if (e != hipSuccess) return e;                                                                \
    hipLaunchKernelGGL((sk_stem4d_col_kernel<C>), grid, block, lds, st, P);                       \
  }
  switch (cpl) {
    case 1: SK_L(1) break;
    case 2: SK_L(2) break;
    case 4: SK_L(4) break;
    default: SK_L(8) break;
  }
#undef SK_L
  return hipGetLastError();
}

int stem4d_cpl(int m) {
  if (m + 1 <= 64) return 1;
  if (m + 1 <= 128) return 2;
  if (m + 1 <= 256) return 4;
  return 8;  // tiles of 512 beyond
}

hipError_t launch_stem4d(const Stem4dLaunch& P, int cpl, hipStream_t st) {
  if (P.n_items == 0) return hipSuccess;
  const int wpb = 4;
  const dim3 grid((unsigned)((P.n_items + wpb - 1) / wpb)), block(64 * wpb);
  const bool band = P.band_lo != nullptr;
#define SK_L(C)                                                                      \
  if (band)                                                                          \
    hipLaunchKernelGGL((sk_stem4d_kernel<C, true>), grid, block, 0, st, P);         \
  else if (P.gsum == 2)                                                              \
    hipLaunchKernelGGL((sk_stem4d_pre_kernel<C>), grid, block, 0, st, P);           \
  else if (P.gsum)                                                                   \
    hipLaunchKernelGGL((sk_stem4d_gsum_kernel<C>), grid, block, 0, st, P);          \
  else                                                                               \
    hipLaunchKernelGGL((sk_stem4d_kernel<C, false>), grid, block, 0, st, P);
  switch (cpl) {
    case 1: SK_L(1) break;
    case 2: SK_L(2) break;
    case 4: SK_L(4) break;
    default: SK_L(8) break;
  }
#undef SK_L
  return hipGetLastError();
}

}  // namespace sk
