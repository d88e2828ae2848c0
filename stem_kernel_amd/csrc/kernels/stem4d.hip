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

#include <algorithm>
#include <type_traits>

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

// lane l receives lane l+1's value of v, lane 63 zero (DPP bound_ctrl): two
// moves, for a slot whose lane 63 holds no valid cell
__device__ __forceinline__ double wave_shl1_z(double v) {
  const int rlo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x130, 0xf, 0xf, true);
  const int rhi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x130, 0xf, 0xf, true);
  return __hiloint2double(rhi, rlo);
}

// lane l receives lane l+1's value of v, lane 63 lane 0's of `next` (the
// slot after v's): lane 63's value comes by DPP wave_rol:1 of `next` and
// stays where the wave_shl:1 of v has no source -- four DPP moves, no trip
// through SGPRs (wave_shl1 with bcast_lane0(next) as `high`: six VALU)
__device__ __forceinline__ double wave_shl1_next(double v, double next) {
  const int nlo = __builtin_amdgcn_mov_dpp(__double2loint(next), 0x134, 0xf, 0xf, false);
  const int nhi = __builtin_amdgcn_mov_dpp(__double2hiint(next), 0x134, 0xf, 0xf, false);
  const int rlo = __builtin_amdgcn_update_dpp(nlo, __double2loint(v), 0x130, 0xf, 0xf, false);
  const int rhi = __builtin_amdgcn_update_dpp(nhi, __double2hiint(v), 0x130, 0xf, 0xf, false);
  return __hiloint2double(rhi, rlo);
}

__device__ __forceinline__ int pad4(int v) { return (v + 3) & ~3; }

// read-only, wave-uniform global data through the constant address space
// (scalar loads: no vector-memory wait behind the prefetched rows)
template <typename T>
using s4_cst = const __attribute__((address_space(4))) T*;

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
  const float* bpy = P.bpdiag_y + pr.y_bp;
  const uint8_t* xs = P.chars + pr.x_chr;
  const uint8_t* ys = P.chars_y + pr.y_chr;
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
  const float* bpy = P.bpdiag_y + pr.y_bp;
  const uint8_t* xs = P.chars + pr.x_chr;
  const uint8_t* ys = P.chars_y + pr.y_chr;
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
  const float* bpy = P.bpdiag_y + pr.y_bp;
  const uint8_t* xs = P.chars + pr.x_chr;
  const uint8_t* ys = P.chars_y + pr.y_chr;
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

// full_dp, column groups (r05): one WORKGROUP per pair walks the x columns in
// groups of NB, j = gNB+1 .. j_hi = min(gNB+NB, n), and in group g the planes
// i = j_hi-1, ..., 0 in turn ("positions"), which its W waves take in turn,
// each wave one row (y span d2) behind the previous.  A position runs its
// group's columns as NB CHAINS in the same step: chain c is the plane
// (i, j_lo + c), and the G0 row it forms is the A row (G0(i, j-1)) of chain
// c+1, so only chain 0 reads a G0 row from HBM (written in plane slot i by
// the previous group's last chain) and only the last chain writes one: 16/NB
// B per cell.  Each chain also forms its consumer's pre-combined G1,
// B'(i-1, j) = G1(i, j) g + G2_(i-1,j), from its own A rows (the stacking
// sources of (i-1, j), the scheme of sk_stem4d_pre_kernel) and hands it to
// the next wave through an LDS double buffer (slot = step parity); the wave
// of every W-th position hands it across the round wrap through one plane per
// chain in HBM (16/W B per cell).  A consumer whose x pair is no stacking
// pair (prob(i-1, j-1) <= bound) has G3 = G2 = 0 in every cell, so its chain
// costs one FMA and one multiply per cell (stem_kernel.cpp:320-334).
// Schedule (tests/test_stem4d_col_schedule.py emulates it step by step
// against the oracle): group g holds c_g = max(j_hi, PF + V) positions (its
// planes, then bubbles); position p is wave p % W's plane of round p / W,
// row s at step T(p) + s, T(p) = (p / W) R + p % W, R = m + 1 rows, one
// LDS-only workgroup barrier per step (lgkmcnt: only the LDS link rows must
// be visible across it).  With W <= m - PF - V (the host's W; m - PF - V + 1
// is exact in the emulator) T is increasing with T(p2) - T(p1) >= p2 - p1, so:
//  * B' of row s is written by wave w-1 at step t-1 and read by wave w at
//    step t (LDS slot t & 1), or, at the wrap, >= PF + V steps later;
//  * the A row that position (g, i) fetches PF rows ahead was written by
//    position (g-1, i), >= c_{g-1} >= PF + V positions earlier;
//  * row 0 is never stored: G0(i, j, l, l) = g^(j-i), the repeated products
//    of gap_powers, as the chain G0(i+1, j, l, l) g forms it (:313-317).
// Global visibility without full barriers: every step ends with a vector
// load issued after its stores (the fence load), and the next step waits for
// it (vmcnt counts loads and stores together, in issue order), so a store of
// step u is complete when its wave ends step u + 1 and seen by the other
// waves after the barrier of step u + 2: V = 2.
// Wave 0's round-wrap rows (one plane per chain in HBM) are staged by all
// waves: each loads its share of the (chain, slot) segments PF + 1 steps
// ahead and writes it into an LDS staging slot the step before wave 0 reads
// it -- in a row step inside the first chain, where the scalar work
// interleaves with vector work (in the tail all waves reached it together and
// the CU's one scalar unit serialised them).
// The K chain is summed (sk_stem4d_gsum_kernel): each lane sums its sources
// over every chain of every position, the waves' sums are added in wave
// order.  Lanes past a row's end compute values that are never stored (the
// range-checked buffers end at the row) nor read by a valid cell of a later
// row (a cell reads k and k+1 of earlier rows, both valid there), and add
// nothing to K (their bp loads return 0, and bound >= 0).
// Every load of a step is issued whether its row exists or not (a
// range-checked buffer of 0 bytes returns 0 without a memory access): a load
// on one path only leaves a phi whose register copy waits for it, right where
// the copy sits.  The next row is fetched (PF = 1) right after a row's
// prologue, into the registers it just left -- but in the widest rows (NS =
// CPL = 4) in the tail, where the early fetch held the kernel's peak
// registers.  PF = 1 with NB = 4 at CPL 4 from the C3 (1,024 x L200) A/B,
// pairs/s: PF 1 NB 4 698, PF 2 NB 3 677, PF 1 NB 3 612, PF 4 NB 2 519 on the
// kernel of then (wider groups halve the row traffic per cell; the registers
// they take come out of the prefetch depth); NB 3 1,106 against NB 4 1,306
// on the final one.
#ifndef SK4C_PF
#define SK4C_PF 1
#endif
constexpr int kS4cV = 2;
// longest x of the column kernel: its x characters sit in LDS (sized per
// launch from the batch's longest x), and with |x| <= 2,048 and |y| < 512 the
// step count fits an int for any W >= 1 (sum of group lengths <= 2.1M
// positions, times R <= 512); longer x go to the span kernels
constexpr int kS4cMaxN = 2048;
#ifndef SK4C_STAGE_IN_ROW  // row steps stage wave 0's wrap rows inside their first chain
#define SK4C_STAGE_IN_ROW 1
#endif
#ifndef SK4C_NB4  // column-group width of the CPL 4 class (|y| 128..255)
#define SK4C_NB4 4
#endif

template <int CPL>
constexpr int s4c_nb() {
  return CPL <= 2 ? 4 : CPL == 4 ? SK4C_NB4 : 1;
}
// waves per workgroup at most (registers: two waves per SIMD)
template <int CPL>
constexpr int s4c_max_waves() {
  return 8;
}

__device__ __forceinline__ int s4c_group_len(int g, int n, int nb, int fp) {
  const int jh = min((g + 1) * nb, n);
  return jh > fp ? jh : fp;
}

// position -> (column group, offset in the group); advance() moves on by W
struct S4cPos {
  int g = 0, off = 0;
  __device__ __forceinline__ void advance(int W, int n, int nb, int fp) {
    off += W;
    while (g * nb < n) {
      const int c = s4c_group_len(g, n, nb, fp);
      if (off < c) break;
      off -= c;
      ++g;
    }
    g = __builtin_amdgcn_readfirstlane(g);  // (uniform: keeps the cursors in SGPRs)
    off = __builtin_amdgcn_readfirstlane(off);
  }
  __device__ __forceinline__ bool valid(int n, int nb) const { return g * nb < n; }
};

// a range-checked buffer over one row of nk elements (loads past them return
// 0, stores are dropped); slot c of the row at voffset (lane + 64 c) * size
template <class T>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t s4c_rowbuf(const T* base, int nk) {
  // (wave-uniform by construction; readfirstlane tells the compiler, which
  // otherwise may build the descriptor in VGPRs and waterfall every access)
  return s4c_rsrc(base, __builtin_amdgcn_readfirstlane(nk * (int)sizeof(T)));
}
__device__ __forceinline__ double s4c_rld64(__amdgpu_buffer_rsrc_t r, int c, int lane) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (lane + 64 * c) * 8, 0, 0));
}
__device__ __forceinline__ float s4c_rld32(__amdgpu_buffer_rsrc_t r, int c, int lane) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (lane + 64 * c) * 4, 0, 0));
}
__device__ __forceinline__ void s4c_rst64(__amdgpu_buffer_rsrc_t r, int c, int lane, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(s4c_u32x2, v), r, (lane + 64 * c) * 8, 0, 0);
}
// the same row as a window [off, off + nk) of a buffer whose base does not
// move from row to row: the range check covers voffset + soffset (gfx950,
// tools/calib/buf_soffset.hip), so records = off + nk and soffset = off
// bound the row exactly -- two scalar shifts per row instead of a 64-bit
// base address and its descriptor words
struct S4cWin {
  __amdgpu_buffer_rsrc_t r;
  int so;
};
template <class T>
__device__ __forceinline__ S4cWin s4c_win(const T* base, int off, int nk) {
  return {s4c_rsrc(base, __builtin_amdgcn_readfirstlane((off + nk) * (int)sizeof(T))),
          __builtin_amdgcn_readfirstlane(off * (int)sizeof(T))};
}
__device__ __forceinline__ double s4c_rld64(S4cWin w, int c, int lane) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(w.r, (lane + 64 * c) * 8, w.so, 0));
}
__device__ __forceinline__ float s4c_rld32(S4cWin w, int c, int lane) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(w.r, (lane + 64 * c) * 4, w.so, 0));
}
__device__ __forceinline__ void s4c_rst64(S4cWin w, int c, int lane, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(s4c_u32x2, v), w.r, (lane + 64 * c) * 8, w.so, 0);
}

template <int CPL>
__global__ void __launch_bounds__(64 * s4c_max_waves<CPL>()) sk_stem4d_col_kernel(Stem4dLaunch P) {
  constexpr int NB = s4c_nb<CPL>();
  constexpr int TW = 64 * CPL;
  constexpr int NSEG = NB * CPL;         // a step's round-wrap rows: segments (chain, slot) of 64 doubles
  constexpr int SEGR = (NSEG + 7) / 8;   // segments a wave stages through registers (W >= NSEG / SEGR)
  constexpr int PF = SK4C_PF;
  constexpr int FP = PF + kS4cV;  // positions per group at least
  extern __shared__ __attribute__((aligned(16))) double s4c_lds[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int W = blockDim.x >> 6;
  const Stem4dPair pr = P.pairs[blockIdx.x];
  const int n = pr.n, m = pr.m, R = m + 1;
  if (m <= 1) {  // no y pair (k, l-1) with k < l-1: no stacking source, K = 1 (the host's W ignores it)
    if (threadIdx.x == 0) P.out[pr.out_index] = 1.0;
    return;
  }
  const int cp = (int)pr.plane_doubles;  // (< 2^17 doubles: |y| < 512)
  double* __restrict__ planes = P.scratch + pr.scratch_off;  // slot i: G0(i, latest column)
  double* __restrict__ wrapb = planes + (int64_t)n * cp;     // NB planes: B' across the round wrap
  const s4_cst<float> bpx = (s4_cst<float>)(P.bpdiag + pr.x_bp);
  const float* bpy = P.bpdiag_y + pr.y_bp;
  const s4_cst<double> gpow = (s4_cst<double>)P.gpow;
  const float bound = P.bp_bound;
  // LDS: links [W][2][NB][TW] (wave w writes link w, wave w+1 reads it a step
  // later), the round-wrap staging [2][NB][TW] (wave 0's link in), W per-wave
  // sums, y (zero padded: y[k + s - 1] for every slot) and x.  The links and
  // the staging start at 0, so every value any lane computes is finite.
  double* link_out = s4c_lds + (int64_t)w * 2 * NB * TW;
  double* wst = s4c_lds + (int64_t)W * 2 * NB * TW;
  const double* link_in = w == 0 ? wst : link_out - 2 * NB * TW;
  double* red = wst + 2 * NB * TW;
  uint8_t* ysl = reinterpret_cast<uint8_t*>(red + W);
  uint8_t* xsl = ysl + TW + R + 8;
  for (int k = threadIdx.x; k < (W + 1) * 2 * NB * TW; k += blockDim.x) s4c_lds[k] = 0.0;
  for (int k = threadIdx.x; k < TW + R + 8; k += blockDim.x) ysl[k] = k < m ? P.chars_y[pr.y_chr + k] : 0;
  for (int k = threadIdx.x; k < n; k += blockDim.x) xsl[k] = P.chars[pr.x_chr + k];
  __syncthreads();

  // steps: T(last position) + R
  int np = 0;
  for (int gg = 0; gg * NB < n; ++gg) np += s4c_group_len(gg, n, NB, FP);
  const int total = np > 0 ? ((np - 1) / W) * R + (np - 1) % W + R : 0;  // (< 2^31: |x| <= kS4cMaxN, |y| < 512)

  // Every position runs all NB chains: a group cut short by n runs virtual
  // columns past n (no stacking sources; the last group's G0 store is never
  // read), and in a group's top triangle (i >= j_lo - 1) the chains before
  // the plane (i, i+1) -- the boundary chain c0 = i + 1 - j_lo, whose A row is
  // G0(i, i) = g^(l-k) and G1 0 -- compute values that are discarded (their
  // A is replaced at c0, their consumers have no sources, their B' rows reach
  // no real chain: the next position reads them only at its boundary chain,
  // which reads none).
  struct Plane {
    int i, c0;          // plane row, the boundary chain (c0 < 0: none)
    bool on;            // a plane (not a bubble)
    uint32_t stack;     // bit c: chain c's consumer (i-1, j_lo+c) is a stacking pair
    uint32_t xci, xcj;  // x[i-1], x[j_lo+c-1] in byte c
    float bpc[NB];      // bp(i-1, j_lo+c-1) of the stacking consumers
  };
  auto describe = [&](const S4cPos& q) __attribute__((always_inline)) -> Plane {
    Plane d;
    d.on = false;
    d.i = 0;
    d.c0 = -1;
    d.stack = d.xci = d.xcj = 0u;
#pragma unroll
    for (int c = 0; c < NB; ++c) d.bpc[c] = 0.0f;
    if (!q.valid(n, NB)) return d;
    const int j_lo = q.g * NB + 1, j_hi = min(q.g * NB + NB, n);
    if (q.off >= j_hi) return d;  // a bubble
    d.on = true;
    const int i = j_hi - 1 - q.off;
    d.i = i;
    d.c0 = i + 1 >= j_lo ? i + 1 - j_lo : -1;
    if (i >= 1) {
      d.xci = __builtin_amdgcn_readfirstlane(xsl[i - 1]);
#pragma unroll
      for (int c = 0; c < NB; ++c) {
        const int jp = j_lo + c, e = jp - i;  // bp(i-1, jp-1): diagonal e
        if (c < (d.c0 < 0 ? 0 : d.c0) || jp > n) continue;
        const float bc = bpx[(int64_t)e * n - (int64_t)e * (e - 1) / 2 + (i - 1)];
        d.xcj |= (uint32_t)__builtin_amdgcn_readfirstlane(xsl[jp - 1]) << (8 * c);
        if (bc > bound) {
          d.stack |= 1u << c;
          d.bpc[c] = bc;
        }
      }
    }
    // (the compiler's divergence analysis loses these through the LDS / the
    // loops: without readfirstlane the per-chain branches become exec-mask
    // branches with both sides executed)
    d.i = __builtin_amdgcn_readfirstlane(d.i);
    d.c0 = __builtin_amdgcn_readfirstlane(d.c0);
    d.stack = __builtin_amdgcn_readfirstlane(d.stack);
    d.xci = __builtin_amdgcn_readfirstlane(d.xci);
    d.xcj = __builtin_amdgcn_readfirstlane(d.xcj);
    return d;
  };
  auto pos_of = [&](const S4cPos& q, bool& on) __attribute__((always_inline)) -> int {
    on = false;
    if (!q.valid(n, NB)) return 0;
    const int j_hi = min(q.g * NB + NB, n);
    on = q.off < j_hi;
    return j_hi - 1 - q.off;
  };
  // a cursor over this wave's (or wave 0's) rows: position, row, the row's
  // offset in a plane and in prob_y
  struct Cur {
    S4cPos q;
    bool on;
    int i, s, ro, ye;
  };
  auto cur_init = [&](Cur& c, int p) __attribute__((always_inline)) {
    c.q = S4cPos();
    c.q.advance(p, n, NB, FP);
    c.i = pos_of(c.q, c.on);
    c.s = c.ro = c.ye = 0;
  };
  auto cur_next = [&](Cur& c) __attribute__((always_inline)) {
    c.ro = __builtin_amdgcn_readfirstlane(c.ro + pad4(m + 1 - c.s));
    c.ye = __builtin_amdgcn_readfirstlane(c.ye + (c.s >= 1 ? m + 1 - c.s : 0));  // prob_y row s at ((s-1) m - (s-1)(s-2)/2)
    c.s = __builtin_amdgcn_readfirstlane(c.s + 1);
    if (c.s == R) {
      c.s = c.ro = c.ye = 0;
      c.q.advance(W, n, NB, FP);
      c.i = __builtin_amdgcn_readfirstlane(pos_of(c.q, c.on));
    }
  };

  // one row's HBM inputs, fetched PF rows ahead: G0(i, j_lo - 1) (chain 0's
  // A row) and prob_y(k, l-1)
  struct Row {
    double A[CPL];
    float bp[CPL];
  };
  Row rq[PF];  // oldest first: the row of step t is fetched at step t - PF
#pragma unroll
  for (int q = 0; q < PF; ++q)
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      rq[q].A[c] = 0.0;
      rq[q].bp[c] = 0.0f;
    }
  Cur fc;  // fetch cursor, from the wave's first step on (fdelay: the steps before)
  cur_init(fc, w);
  int fdelay = w;
  auto fetch_next = [&](Row& r) __attribute__((always_inline)) {
    const bool ld = fdelay <= 0 && fc.q.valid(n, NB) && fc.on && fc.s >= 1;
    const int nk = ld ? m - fc.s + 1 : 0;  // valid cells of the row
    const auto ra = s4c_rowbuf(planes + (ld ? (int64_t)fc.i * cp + fc.ro : 0), nk);
    const auto rb = s4c_rowbuf(bpy + (ld ? fc.ye : 0), nk);
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      r.A[c] = s4c_rld64(ra, c, lane);
      r.bp[c] = s4c_rld32(rb, c, lane);
    }
    if (fdelay > 0) --fdelay;
    else if (fc.q.valid(n, NB)) cur_next(fc);
  };

  // The round wrap: wave 0's positions are 0, W, 2W, ..., so at step u it
  // runs row u mod R of position (u div R) W, whose chains read their B'
  // rows from the wrap planes.  Every wave stages a share of them: the
  // segments (chain, slot) w, w + W, ... of wave 0's rows of step u are
  // loaded at step u - PF - 1, written to wst[(u - 1) & 1] at step u-1 (the
  // slot a link of step u-1 takes) and read by wave 0 at step u after the
  // barrier.  zc: the rows of the last staging load, yc: of the next store
  // (with PF = 1 the same rows: zc serves both, and yc is dead).
  Cur zc, yc;
  cur_init(zc, 0);
  cur_init(yc, 0);
  cur_next(yc);  // wave 0's rows of step 1 are the first the stores write
  double wrq[PF][SEGR];  // staged segments in flight, oldest first
#pragma unroll
  for (int q = 0; q < PF; ++q)
#pragma unroll
    for (int e = 0; e < SEGR; ++e) wrq[q][e] = 0.0;
  auto zload = [&](double (&wr)[SEGR]) __attribute__((always_inline)) {
    const bool ld = zc.q.valid(n, NB) && zc.on && zc.s != 0;
    const int nk = ld ? m - zc.s + 1 : 0;
    const int ro = ld ? zc.ro : 0;
#pragma unroll
    for (int q = 0; q < SEGR; ++q) {
      const int sg = w + q * W, ch = sg / CPL, c = sg % CPL;
      // (sg >= NSEG: wave w has no q-th segment -- W > NSEG / SEGR -- nothing to load)
      wr[q] = s4c_rld64(s4c_win(wrapb + (int64_t)(ch < NB ? ch : 0) * cp, ro, sg < NSEG ? nk : 0), c % CPL, lane);
    }
  };
  // (segments past this wave's SEGR: only with few waves; one flag)
  const bool zrest = __builtin_amdgcn_readfirstlane(w + SEGR * W < NSEG ? 1 : 0) != 0;
  auto zstore = [&](double* dst, const double (&wr)[SEGR], const Cur& yc) __attribute__((always_inline)) {
    if (!yc.on || yc.s == 0) return;
#pragma unroll
    for (int q = 0; q < SEGR; ++q) {
      const int sg = w + q * W, ch = sg / CPL, c = sg % CPL;
      if (sg < NSEG) dst[ch * TW + 64 * c + lane] = wr[q];
    }
    if (zrest) {  // few waves (short y): the rest loaded here
      const int nk = m - yc.s + 1;
      for (int sg = w + SEGR * W; sg < NSEG; sg += W) {
        const int ch = sg / CPL, c = sg % CPL;
        dst[ch * TW + 64 * c + lane] = s4c_rld64(s4c_win(wrapb + (int64_t)ch * cp, yc.ro, nk), c, lane);
      }
    }
  };
  // the fence load: one 4-byte load at the end of every step, waited for at
  // the end of the next, so every step's stores complete by then (kS4cV)
  float fq = 0.0f;
  const auto fence_buf = s4c_rowbuf(bpy, 1);

  // steps -PF .. -1: this wave's first rows (of steps 0 .. PF-1; before its
  // first step, t = w, nothing) and the staging loads of wave 0's rows of
  // steps 1 .. PF
#pragma unroll
  for (int q = 0; q < PF; ++q) fetch_next(rq[q]);
#pragma unroll
  for (int q = 0; q < PF; ++q) {
    cur_next(zc);
    zload(wrq[q]);
  }
  fq = s4c_rld32(fence_buf, 0, lane);

#ifdef SK4C_TIMING  // diagnostic build: cycles per step part, printed for two blocks
  uint64_t tm_bar = 0, tm_fence = 0, tm_row = 0, tm_tail = 0, tm_a = 0, tm_b = 0;
  int tm_steps = 0;
#define S4C_TICK(v) (v = (uint64_t)clock64())
#else
#define S4C_TICK(v) ((void)0)
#endif
  // every step: the barrier (this wave's row of the step is rq[0]) ...
  auto head = [&](int t) __attribute__((always_inline)) {
#ifdef SK4C_TIMING
    uint64_t t0, t1;
    S4C_TICK(t0);
    if (tm_a) tm_tail += t0 - tm_a;
#endif
    if (t > 0) {  // (every wave takes every barrier) LDS-only: the global stores by vmcnt (kS4cV)
      asm volatile("" ::: "memory");
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
      asm volatile("" ::: "memory");
    }
#ifdef SK4C_TIMING
    S4C_TICK(t1);
#endif
#ifdef SK4C_TIMING
    S4C_TICK(tm_b);
    tm_bar += t1 - t0;
    tm_fence += tm_b - t1;
    tm_a = tm_b;
    ++tm_steps;
#endif
  };
  // ... and after the step's compute: wave 0's wrap rows of step t+1 into
  // LDS, the wait for the previous step's fence load, the queue moved on,
  // the row of step t + PF and wave 0's wrap rows of step t+PF+1 loaded, the
  // fence load
  // (FETCHED: a row step with PF = 1 issued the fetch after its prologue)
  // (STAGED: a row step ran the staging part -- wave 0's wrap rows and the
  // fence wait -- inside its first chain, where its scalar work interleaves
  // with the chain's vector work: in the tail all waves reach it together,
  // and the CU's one scalar unit serialises them)
  auto stage = [&](int t) __attribute__((always_inline)) {
    if constexpr (PF == 1) {
      if (zc.q.valid(n, NB)) zstore(wst + (t & 1) * NB * TW, wrq[0], zc);
    } else if (yc.q.valid(n, NB)) {
      zstore(wst + (t & 1) * NB * TW, wrq[0], yc);
      cur_next(yc);
    }
    asm volatile("" ::"v"(fq));  // this wave's stores of step t-1 are complete
#pragma unroll
    for (int q = 0; q + 1 < PF; ++q)
#pragma unroll
      for (int e = 0; e < SEGR; ++e) wrq[q][e] = wrq[q + 1][e];
    if (zc.q.valid(n, NB)) cur_next(zc);
    zload(wrq[PF - 1]);
  };
  auto tail = [&](int t, auto fetched_tag, auto staged_tag) __attribute__((always_inline)) {
    constexpr bool STAGED = decltype(staged_tag)::value;
    if constexpr (!STAGED) {
      if constexpr (PF == 1) {
        if (zc.q.valid(n, NB)) zstore(wst + (t & 1) * NB * TW, wrq[0], zc);
      } else if (yc.q.valid(n, NB)) {
        zstore(wst + (t & 1) * NB * TW, wrq[0], yc);
        cur_next(yc);
      }
      asm volatile("" ::"v"(fq));  // this wave's stores of step t-1 are complete
    }
    if constexpr (!decltype(fetched_tag)::value) {
#pragma unroll
      for (int q = 0; q + 1 < PF; ++q) rq[q] = rq[q + 1];
      fetch_next(rq[PF - 1]);
    }
    if constexpr (!STAGED) {
#pragma unroll
      for (int q = 0; q + 1 < PF; ++q)
#pragma unroll
        for (int e = 0; e < SEGR; ++e) wrq[q][e] = wrq[q + 1][e];
      if (zc.q.valid(n, NB)) cur_next(zc);
      zload(wrq[PF - 1]);
    }
    fq = s4c_rld32(fence_buf, 0, lane);  // (lane 0 reads bpy[0], the rest nothing)
  };

  double ksrc = 0.0, kacc[NB];
  double Am1[NB][CPL], Am2[NB][CPL], G2c[NB][CPL], G3c[NB][CPL];
#pragma unroll
  for (int ch = 0; ch < NB; ++ch) {
    kacc[ch] = 0.0;
#pragma unroll
    for (int c = 0; c < CPL; ++c) Am1[ch][c] = Am2[ch][c] = G2c[ch][c] = G3c[ch][c] = 0.0;
  }
  // loop-invariant kernel constants in VGPRs (SGPRs are the scarce ones here)
  double gv = P.gap, subv = P.subst;
  asm volatile("" : "+v"(gv), "+v"(subv));
  uint32_t xk = 0u;  // bit c: y[k] == x[i-1] (the consumer's left base), per position
  Plane dc;

  // row s >= 1 of the position: NS slots hold its cells (64 (NS-1) <= m - s
  // + 1 < 64 NS), chain by chain (one uniform branch per chain on its consumer's
  // stacking); BND: a boundary chain c0 (a top-triangle position)
  auto row = [&](int t, int s, int ro, int ye, const double* pbase, auto bnd_tag, auto ns_tag, auto last_tag)
                 __attribute__((always_inline)) {
    constexpr bool BND = decltype(bnd_tag)::value;
    constexpr int NS = decltype(ns_tag)::value;
    // the last wave hands its B' rows on through the wrap planes, the others
    // through their LDS links (the last wave's link has no reader)
    constexpr bool LASTW = decltype(last_tag)::value;
    const int nk = m - s + 1;
    const double* lin = link_in + ((t - 1) & 1) * NB * TW;
    double* lout = link_out + (t & 1) * NB * TW;
    const double gs = gpow[s];
    // per slot, shared by the chains: prob_y(k, l-1) where a source, y[l-1]
    double A[NS], bpd[NS];
    uint32_t yl[NS];
    const Row& X = rq[0];
#pragma unroll
    for (int c = 0; c < NS; ++c) {
      // (explicit copies: the queue's registers end here, so the loads below
      // can land in them; a renamed A would leave them live and the loads
      // in other registers, copied -- and waited for -- at the loop latch)
      asm volatile("v_mov_b64 %0, %1" : "=v"(A[c]) : "v"(X.A[c]));
      float b;
      asm volatile("v_mov_b32 %0, %1" : "=v"(b) : "v"(X.bp[c]));
      bpd[c] = b > bound ? (double)b : 0.0;
      yl[c] = ysl[lane + 64 * c + s - 1];
    }
    // the queue's row is in A / bpd now: with PF = 1 the next row's loads go
    // out here, into the same registers, a whole step ahead of their use
    // (not in the widest rows, where the registers they hold through the row
    // are the kernel's peak: there the tail issues them)
    // (the row is this position's s + 1, when s < m: its offsets follow from
    // this row's, the plane's base is the position's -- no cursor arithmetic;
    // the fetch cursor stands still, and the position's end sets it again)
    if constexpr (PF == 1 && (NS < CPL || CPL < 4)) {
      // (at s = m the window is empty: nothing is read)
      const int nk = m - s;
      const auto ra = s4c_win(pbase, ro + pad4(m + 1 - s), nk);
      const auto rb = s4c_win(bpy, ye + m + 1 - s, nk);
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        rq[0].A[c] = s4c_rld64(ra, c, lane);
        rq[0].bp[c] = s4c_rld32(rb, c, lane);
      }
    }
    const uint32_t stk_mask = __builtin_amdgcn_readfirstlane(dc.stack);
    const int bch = BND ? __builtin_amdgcn_readfirstlane(dc.c0) : -1;
    // the B' rows from the neighbour (G1), every chain's at once: a chain
    // whose consumer does not stack (most of them) is a few VALU after its
    // read, so reads issued chain by chain leave one LDS round trip per
    // chain exposed.  Not in the widest phase, whose registers are the
    // kernel's peak (there each chain reads its own)
    constexpr bool HOIST = NB >= 2 && NB * NS <= 12 && (NS < CPL || CPL <= 2);
    double G1h[NB][HOIST ? NS : 1];
    if constexpr (HOIST) {
#pragma unroll
      for (int ch = 0; ch < NB; ++ch)
#pragma unroll
        for (int c = 0; c < NS; ++c) G1h[ch][c] = lin[ch * TW + lane + 64 * c];
    }
#pragma unroll
    for (int ch = 0; ch < NB; ++ch) {
      // (one chain at a time: the scheduler would otherwise hoist every
      // chain's LDS reads to the top, past the register budget)
      if (NB >= 4) __builtin_amdgcn_sched_barrier(0);
      if (SK4C_STAGE_IN_ROW && ch == 0) stage(t);
      const bool bz = BND && ch == bch;  // G0(i, i) row and no G1
      const auto rw = s4c_win(wrapb + (int64_t)ch * cp, ro, LASTW ? nk : 0);
      if constexpr (HOIST) {
        // the part every chain runs, then the stacking consumer's terms in
        // one branch without an else (a non-stacking chain: G0, B' and the
        // store; an if / else costs two branches and its phi copies)
        double G0v[NS], Bnv[NS];
#pragma unroll
        for (int c = 0; c < NS; ++c) {
          double G1 = 0.0;
          if (bz) A[c] = gs;
          else G1 = G1h[ch][HOIST ? c : 0];
          G0v[c] = A[c] * gv + G1;
          Bnv[c] = G1 * gv;
        }
        if ((stk_mask >> ch) & 1u) {
          const uint32_t xcj = (dc.xcj >> (8 * ch)) & 0xffu;
#pragma unroll
          for (int c = 0; c < NS; ++c) {
            const double G3n = c + 1 < NS ? wave_shl1_next(G3c[ch][c], G3c[ch][c + 1 < CPL ? c + 1 : c])
                                          : wave_shl1_z(G3c[ch][c]);
            const double A2 = c + 1 < NS ? wave_shl1_next(Am2[ch][c], Am2[ch][c + 1 < CPL ? c + 1 : c])
                                         : wave_shl1_z(Am2[ch][c]);
            const double bp_kl = bpd[c];
            const bool mt = ((xk >> c) & 1u) && yl[c] == xcj && bp_kl != 0.0;
            kacc[ch] += A2 * bp_kl * (mt ? 1.0 : subv);
            double g3 = G3n * gv;
            g3 += mt ? A2 : 0.0;
            double g2 = G2c[ch][c] * gv;
            g2 += g3;
            Bnv[c] += g2;
            G2c[ch][c] = g2;
            G3c[ch][c] = g3;
            Am2[ch][c] = Am1[ch][c];
            Am1[ch][c] = A[c];
          }
        }
#pragma unroll
        for (int c = 0; c < NS; ++c) {
          if (LASTW) s4c_rst64(rw, c, lane, Bnv[c]);
          else lout[ch * TW + lane + 64 * c] = Bnv[c];
          A[c] = G0v[c];
        }
      } else if ((stk_mask >> ch) & 1u) {
        const uint32_t xcj = (dc.xcj >> (8 * ch)) & 0xffu;
#pragma unroll
        for (int c = 0; c < NS; ++c) {
          const int k = lane + 64 * c;
          double G1 = 0.0;
          if (bz) A[c] = gs;
          else G1 = HOIST ? G1h[ch][HOIST ? c : 0] : lin[ch * TW + k];
          double G0 = A[c] * gv;
          G0 += G1;
          // the consumer's G3 at (k+1, l) (row s-1) and G0(i, j-1) at
          // (k+1, l-1) (row s-2): the next lane's, or the next slot's lane 0
          // (slot c+1 not yet updated this row); the phase's last slot has
          // no valid cell in lane 63 (a phase's rows hold < 64 NS cells), so
          // nothing comes from the slot after it
          const double G3n = c + 1 < NS ? wave_shl1_next(G3c[ch][c], G3c[ch][c + 1 < CPL ? c + 1 : c])
                                        : wave_shl1_z(G3c[ch][c]);
          const double A2 = c + 1 < NS ? wave_shl1_next(Am2[ch][c], Am2[ch][c + 1 < CPL ? c + 1 : c])
                                       : wave_shl1_z(Am2[ch][c]);
          const double bp_kl = bpd[c];
          const uint32_t y_l = yl[c];
          const bool mt = ((xk >> c) & 1u) && y_l == xcj && bp_kl != 0.0;
          // the source (:320-331) without its stack * bp(i-1, j-1) factor,
          // which the position's sum takes at its end
          kacc[ch] += A2 * bp_kl * (mt ? 1.0 : subv);
          double g3 = G3n * gv;
          g3 += mt ? A2 : 0.0;
          double g2 = G2c[ch][c] * gv;
          g2 += g3;
          double Bn = G1 * gv;
          Bn += g2;
          G2c[ch][c] = g2;
          G3c[ch][c] = g3;
          Am2[ch][c] = Am1[ch][c];
          Am1[ch][c] = A[c];
          if (LASTW) s4c_rst64(rw, c, lane, Bn);
          else lout[ch * TW + k] = Bn;
          A[c] = G0;
        }
      } else {
#pragma unroll
        for (int c = 0; c < NS; ++c) {
          const int k = lane + 64 * c;
          double G1 = 0.0;
          if (bz) A[c] = gs;
          else G1 = HOIST ? G1h[ch][HOIST ? c : 0] : lin[ch * TW + k];
          double G0 = A[c] * gv;
          G0 += G1;
          const double Bn = G1 * gv;
          if (LASTW) s4c_rst64(rw, c, lane, Bn);
          else lout[ch * TW + k] = Bn;
          A[c] = G0;
        }
      }
    }
    const auto rg = s4c_win(pbase, ro, nk);
#pragma unroll
    for (int c = 0; c < NS; ++c) s4c_rst64(rg, c, lane, A[c]);  // the last chain's G0 (i, j_hi)
  };

  int t = 0;
  auto run = [&](auto last_tag) __attribute__((always_inline)) {
  for (; t < w && t < total; ++t) {  // before the wave's first position
    head(t);
    tail(t, std::false_type(), std::false_type());
  }
  // a position's rows 1 .. m in phases of NS active slots, CPL down to 1:
  // phase NS takes the rows of 64 (NS-1) .. 64 NS - 1 cells (m - s + 1), so
  // lane 63 of its last slot never holds a valid cell (m < 64 CPL)
  auto rows = [&](auto bnd_tag) __attribute__((always_inline)) {
    int s = 1, ro = pad4(m + 1), ye = 0;
    const double* pbase = planes + (int64_t)dc.i * cp;
    auto phase = [&](auto ns_tag) __attribute__((always_inline)) {
      constexpr int NS = decltype(ns_tag)::value;
      const int s_end = NS > 1 ? m + 1 - 64 * (NS - 1) : m;
      for (; s <= s_end; ++s, ++t) {
        head(t);
        row(t, s, ro, ye, pbase, bnd_tag, ns_tag, last_tag);
#ifdef SK4C_TIMING
        {
          uint64_t tr;
          S4C_TICK(tr);
          tm_row += tr - tm_a;
          tm_a = tr;
        }
#endif
        tail(t, std::integral_constant<bool, PF == 1 && (NS < CPL || CPL < 4)>(),
             std::integral_constant<bool, SK4C_STAGE_IN_ROW != 0>());
        ro += pad4(m + 1 - s);
        ye += m + 1 - s;
      }
    };
    if constexpr (CPL >= 8) {
      phase(std::integral_constant<int, 8>());
      phase(std::integral_constant<int, 7>());
      phase(std::integral_constant<int, 6>());
      phase(std::integral_constant<int, 5>());
    }
    if constexpr (CPL >= 4) {
      phase(std::integral_constant<int, 4>());
      phase(std::integral_constant<int, 3>());
    }
    if constexpr (CPL >= 2) phase(std::integral_constant<int, 2>());
    phase(std::integral_constant<int, 1>());
  };
  S4cPos cur;
  cur.advance(w, n, NB, FP);  // from position 0
  while (cur.valid(n, NB)) {
    dc = describe(cur);
    if (!dc.on) {  // a bubble
      for (int s = 0; s < R; ++s, ++t) {
        head(t);
        tail(t, std::false_type(), std::false_type());
      }
    } else {
      head(t);  // row 0, cells (l, l): G0 = g^(j-i), never stored; the chains' registers reset
      xk = 0u;
#pragma unroll
      for (int c = 0; c < CPL; ++c) xk |= (ysl[lane + 64 * c] == dc.xci ? 1u : 0u) << c;
#pragma unroll
      for (int ch = 0; ch < NB; ++ch) {
        const double a0 = (dc.stack >> ch) & 1u ? gpow[cur.g * NB + ch - dc.i] : 0.0;  // G0(i, j-1, l, l)
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          Am1[ch][c] = a0;
          Am2[ch][c] = G2c[ch][c] = G3c[ch][c] = 0.0;
        }
      }
      tail(t, std::false_type(), std::false_type());
      ++t;
      if (dc.c0 >= 0) rows(std::true_type());
      else rows(std::false_type());
#pragma unroll
      for (int ch = 0; ch < NB; ++ch) {  // the position's sources: times stack * bp(i-1, j-1)
        ksrc += kacc[ch] * (P.stack * (double)dc.bpc[ch]);
        kacc[ch] = 0.0;
      }
      // the fetch cursor resumes at the next position's row 1, which that
      // position's first step fetches (the row steps fetched without it)
      if constexpr (PF == 1) {
        fc.q = cur;
        fc.q.advance(W, n, NB, FP);
        fc.i = __builtin_amdgcn_readfirstlane(pos_of(fc.q, fc.on));
        fc.s = 1;
        fc.ro = pad4(m + 1);
        fc.ye = 0;
        fdelay = 0;
      }
    }
    cur.advance(W, n, NB, FP);
  }
  for (; t < total; ++t) {  // after the wave's last position
    head(t);
    tail(t, std::false_type(), std::false_type());
  }
  };
  if (w + 1 == W) run(std::true_type());
  else run(std::false_type());
#ifdef SK4C_TIMING
  if (lane == 0 && (blockIdx.x == 0 || blockIdx.x == gridDim.x / 2))
    printf("sk4c b%d w%d steps %d bar %lu fence %lu row %lu tail %lu\n", (int)blockIdx.x, w, tm_steps,
           (unsigned long)tm_bar, (unsigned long)tm_fence, (unsigned long)tm_row, (unsigned long)tm_tail);
#endif
  for (int off = 32; off > 0; off >>= 1) ksrc += __shfl_xor(ksrc, off, 64);
  if (lane == 0) red[w] = ksrc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double K = 0.0;
    for (int v = 0; v < W; ++v) K += red[v];
    P.out[pr.out_index] = 1.0 + K;
  }
}

int stem4d_col_w_max(int m) { return m - SK4C_PF - kS4cV; }
int stem4d_col_pf() { return SK4C_PF; }

int stem4d_col_max_waves(int cpl) {
  return cpl <= 1 ? s4c_max_waves<1>() : cpl == 2 ? s4c_max_waves<2>() : cpl == 4 ? s4c_max_waves<4>()
                                                                          : s4c_max_waves<8>();
}

int stem4d_col_nb(int cpl) {
  return cpl <= 1 ? s4c_nb<1>() : cpl == 2 ? s4c_nb<2>() : cpl == 4 ? s4c_nb<4>() : s4c_nb<8>();
}

int stem4d_col_max_n() { return kS4cMaxN; }

size_t stem4d_col_lds_bytes(int cpl, int waves, int m, int n) {
  const int nb = stem4d_col_nb(cpl);
  return ((size_t)(waves + 1) * 2 * nb * 64 * cpl + waves) * sizeof(double) +
         (size_t)(64 * cpl + m + 1 + 8 + std::max(n, 0) + 15) / 16 * 16;  // y, x
}

hipError_t launch_stem4d_col(const Stem4dLaunch& P, int64_t n_pairs, int cpl, int waves, int max_m,
                             int max_n, hipStream_t st) {
  if (n_pairs == 0) return hipSuccess;
  if (max_n > kS4cMaxN || max_m + 1 > 64 * cpl) return hipErrorInvalidValue;
  const size_t lds = stem4d_col_lds_bytes(cpl, waves, max_m, max_n);
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
