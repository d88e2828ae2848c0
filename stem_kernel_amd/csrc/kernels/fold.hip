// McCaskill base-pairing probabilities on CDNA4 (gfx950): SURVEY.md §8 f1.
//
// Replaces ViennaRNA's pf_fold as the reference calls it for every example
// (BPMatrix FOLD, common/bpmatrix.cpp:151-177; PFWrapper::fold,
// common/pf_wrapper.cpp:15-36; twice per pair in stem_kernel/stem_kernel.cpp:290-291).
// ViennaRNA and its parameter files are not in this image: the loop model is
// the Turner-1999 core the legacy library compiles in (stacks, hairpin /
// bulge / interior initiation, Ninio asymmetry, terminal AU/GU, linear
// multiloop) without its mismatch, dangle and special-loop tables
// (parity against ViennaRNA unpinned, the recursions pinned by
// exhaustive enumeration in oracle/fold_oracle.c).
//
// One workgroup per sequence.  Inside tables Qb (pair closes a loop), Qm1
// (one multiloop branch starting at i), Qm (>= 1 branch) and the exterior
// prefix Q5; outside values as adjoints of the inside rules (Hb, Hm1, Hm,
// H5), each cell PULLING from larger spans, so a span's cells are
// independent: one thread per cell, a barrier per span.  Tables are n x n
// doubles in HBM (L2-resident for n up to ~250), with transposed copies of
// the ones read down a column.  All quantities of a subsequence carry a
// per-nucleotide scale sc^len (Vienna's pf_scale), so Z stays in range for
// n up to ~1,400; P(i,j) = Qb Hb / Z is scale-free.
#include <hip/hip_runtime.h>

#include "launch.h"

namespace sk {

// pair type of codes (a, b), a * 4 + b -> 4 bits of a 64-bit constant (no
// memory access: a __constant__ table indexed per thread is a vector load):
// {0,0,0,5, 0,0,1,0, 0,2,0,4, 6,0,3,0}  CG1 GC2 GU3 UG4 AU5 UA6
constexpr uint64_t kFoldPairBits = 0x306402001005000ull;

struct FoldTables {  // views into P.tab (FoldLaunch::tab layout)
  const double *st, *hp, *bu, *in, *ni, *au, *scp;
  double mlc, mli;
};

__device__ __forceinline__ int pair_raw(int a, int b) {
  return (a < 0 || b < 0) ? 0 : (int)((kFoldPairBits >> (4 * (a * 4 + b))) & 0xfu);
}
__device__ __forceinline__ bool is_gu(int t) { return t == 3 || t == 4; }

// interior / bulge / stack loop factor (unscaled), t1 = type(i,j), t2 = type(q,p)
__device__ __forceinline__ double fold_interior(const FoldTables& T, int t1, int t2, int n1, int n2,
                                                bool ncg) {
  const int n = n1 + n2;
  if (n == 0) return T.st[t1 * 7 + t2];
  if (ncg && (is_gu(t1) || is_gu(t2))) return 0.0;
  if (n1 == 0 || n2 == 0) return n == 1 ? T.bu[1] * T.st[t1 * 7 + t2] : T.bu[n] * T.au[t1] * T.au[t2];
  return T.in[n] * T.ni[abs(n1 - n2)] * T.au[t1] * T.au[t2];
}

// block-wide sum (at most 8 waves), result in every thread
__device__ __forceinline__ double block_sum(double v, double* red) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int k = 0; k < nw; ++k) s += red[k];
  return s;
}

// sum over a team of G (1, 2, 4, 8) adjacent lanes, in every lane of the team
__device__ __forceinline__ double team_sum(double v, int G) {
  if (G >= 2) v += __shfl_xor(v, 1, 64);
  if (G >= 4) v += __shfl_xor(v, 2, 64);
  if (G >= 8) v += __shfl_xor(v, 4, 64);
  return v;
}

// lanes per cell of a span of ncell cells: the most (up to 8) that keep
// every cell of the span in one pass of the block's threads
__device__ __forceinline__ int team_of(int ncell, int nt) {
  int G = 1;
  while (G < 8 && ncell * (2 * G) <= nt) G *= 2;
  return G;
}

// Tables are stored by DIAGONAL: cell (i, i+d) of a table at d*n + i.  A
// span's cells are the threads (consecutive i), and every read of a loop
// iteration sits at a fixed offset from the cell -- (i+a, j-b) lies on
// diagonal d-a-b at index i+a -- so the threads of a wave read consecutive
// doubles: coalesced, where the row-major tables gave each thread its own
// row (one cache line per lane per iteration).  The interior-loop windows
// (the 31 diagonals below the span inside, above it outside) are also kept
// in an LDS ring of kFoldRing diagonals when the sequences are short enough
// (RING: 33 n doubles), and the Boltzmann tables and the codes sit in LDS.
constexpr int kFoldRing = 33;  // 31 diagonals read + the one written, distinct slots

// 512 threads (8 waves; 94 VGPRs: two workgroups per CU by LDS at L = 200)
// GTAB: the hairpin and scale tables (the tail of P.tab, sized by the
// batch's longest sequence) are read from HBM, only the fixed-size head sits
// in LDS -- long sequences, whose tables would not fit beside the codes
template <bool RING, bool GTAB>
__global__ void __launch_bounds__(512) sk_fold_kernel(FoldLaunch P) {
  extern __shared__ __attribute__((aligned(16))) double fsm[];
  __shared__ double red[8];
  const FoldSeq sq = P.seqs[blockIdx.x];
  const int n = sq.n;
  const int tid = threadIdx.x, nt = blockDim.x;
  const size_t N2 = (size_t)n * n;
  double* W = P.work + sq.work_off;
  double *Qb = W, *Qm = W + N2, *Qm1 = W + 2 * N2, *Hb = W + 3 * N2, *Hm = W + 4 * N2, *Hm1 = W + 5 * N2;
  double *Q5 = W + 6 * N2, *H5 = Q5 + n + 1;
  // LDS: the Boltzmann tables, the ring (RING), the codes
  double* tl = fsm;
  const int n_lds = GTAB ? P.n_small : P.n_tab;  // table entries copied to LDS
  double* ring = tl + ((n_lds + 1) & ~1);
  int8_t* c = reinterpret_cast<int8_t*>(ring + (RING ? kFoldRing * P.ring_n : 0));
  for (int k = tid; k < n_lds; k += nt) tl[k] = P.tab[k];
  for (int k = tid; k < n; k += nt) c[k] = P.codes[sq.seq_off + k];
  __syncthreads();
  FoldTables T;
  T.st = tl + P.o_st;
  T.hp = GTAB ? P.tab + P.o_hp : tl + P.o_hp;
  T.bu = tl + P.o_bu;
  T.in = tl + P.o_in;
  T.ni = tl + P.o_ni;
  T.au = tl + P.o_au;
  T.scp = GTAB ? P.tab + P.o_scp : tl + P.o_scp;
  T.mlc = tl[P.o_ml];
  T.mli = tl[P.o_ml + 1];
  const double* scp = T.scp;
  const bool ngu = P.no_gu != 0, ncg = P.no_closing_gu != 0;
  const uint8_t* __restrict__ lp = P.lp ? P.lp + sq.lp_off : nullptr;
  auto ptype = [&](int i, int j) {
    const int t = pair_raw(c[i], c[j]);
    if (lp && !lp[(size_t)i * n + j]) return 0;  // --noLonelyPairs (host table)
    return (ngu && is_gu(t)) ? 0 : t;
  };
  auto D = [&](int d, int i) { return (size_t)d * n + i; };
  // ring slot of diagonal d, and the slot of d - 1 / d + 1 given d's
  auto slot = [](int d) { return d % kFoldRing; };
  auto dn = [](int sl) { return sl == 0 ? kFoldRing - 1 : sl - 1; };
  auto up = [](int sl) { return sl == kFoldRing - 1 ? 0 : sl + 1; };
#ifdef SK_FOLD_TIMING  // diagnostic build: cycles per pass, printed for blocks 0 and 1
  const uint64_t tk0 = clock64();
#endif

  // ---------------------------------------------------------------- inside
  // A span's cells go to TEAMS of G lanes (team_of: as many as the block's
  // threads allow, up to 8 -- the long spans, with the most work per cell,
  // have the fewest cells): lane r of a team takes every G-th iteration of
  // each sum, and the team adds its partial sums by a butterfly (the same
  // fixed order for every cell).
  for (int d = 4; d < n; ++d) {
    const int ncell = n - d;
    const int G = team_of(ncell, nt);
    for (int base = 0; base < ncell; base += nt / G) {
      const int i0 = base + tid / G, r = tid % G;
      const bool on = i0 < ncell;
      const int i = on ? i0 : 0, j = i + d;
      const int t = on ? ptype(i, j) : 0;
      double part = 0.0;
      if (t) {
        // interior loops closed by (p, q) = (i+1+n1, j-1-n2), n1 + n2 <= 30,
        // q >= p + 4: diagonal d-2-n1-n2
        for (int n1 = r; n1 <= min(30, d - 6); n1 += G) {
          const int p = i + 1 + n1;
          const int n2m = min(30 - n1, d - 6 - n1);
          const int cp = c[p];
          int sl = slot(d - 2 - n1);
          for (int n2 = 0; n2 <= n2m; ++n2) {
            const double v = RING ? ring[(size_t)sl * P.ring_n + p] : Qb[D(d - 2 - n1 - n2, p)];
            sl = dn(sl);
            if (v != 0.0)
              part += v * fold_interior(T, t, pair_raw(c[j - 1 - n2], cp), n1, n2, ncg) * scp[n1 + n2 + 2];
          }
        }
        if (!(ncg && is_gu(t))) {
          // multiloop closed by (i, j): Qm(i+1, u) Qm1(u+1, j-1), u = i+e
          double ml = 0.0;
#pragma unroll 4
          for (int e = 5 + r; e + 6 <= d; e += G) ml += Qm[D(e - 1, i + 1)] * Qm1[D(d - e - 2, i + e + 1)];
          part += ml * T.mlc * T.au[t] * scp[2];
        }
      }
      part = team_sum(part, G);
      const double qb = t ? (!(ncg && is_gu(t)) ? T.hp[d - 1] * T.au[t] * scp[d + 1] : 0.0) + part : 0.0;
      if (on && r == 0) {
        Qb[D(d, i)] = qb;
        if (RING) ring[(size_t)slot(d) * P.ring_n + i] = qb;
      }
      double m1 = 0.0;  // Qm1(i, j): Qb(i, l) closing the branch, l = i+4 .. j
      if (on) {
#pragma unroll 4
        for (int l = i + 4 + r; l <= j; l += G) {
          const double v = l == j ? qb : Qb[D(l - i, i)];
          if (v != 0.0) m1 += v * T.mli * T.au[pair_raw(c[i], c[l])] * scp[j - l];
        }
      }
      m1 = team_sum(m1, G);
      if (on && r == 0) Qm1[D(d, i)] = m1;
      double m = 0.0;  // Qm(i, j) = sum_u (sc^(u-i) + Qm(i, u-1)) Qm1(u, j)
      if (on) {
#pragma unroll 4
        for (int u = i + r; u + 4 <= j; u += G)
          m += (scp[u - i] + (u - 1 >= i ? Qm[D(u - 1 - i, i)] : 0.0)) * (u == i ? m1 : Qm1[D(j - u, u)]);
      }
      m = team_sum(m, G);
      if (on && r == 0) Qm[D(d, i)] = m;
    }
    __syncthreads();
  }
#ifdef SK_FOLD_TIMING
  const uint64_t tk1 = clock64();
#endif

  // ---------------------------------------------------------------- exterior
  if (tid == 0) Q5[0] = 1.0;
  __syncthreads();
  for (int j = 0; j < n; ++j) {
    double s = 0.0;
    for (int k = tid; k + 4 <= j; k += nt) {
      const double v = Qb[D(j - k, k)];
      if (v != 0.0) s += Q5[k] * v * T.au[pair_raw(c[k], c[j])];
    }
    s = block_sum(s, red);
    if (tid == 0) Q5[j + 1] = Q5[j] * scp[1] + s;
    __syncthreads();
  }
  const double Z = Q5[n];
  if (tid == 0 && P.log_z) P.log_z[blockIdx.x] = log(Z) - (double)n * P.log_sc;
  if (tid == 0) H5[n] = 1.0;
  __syncthreads();
  for (int k = n - 1; k >= 0; --k) {
    double s = 0.0;
    for (int j = k + 4 + tid; j < n; j += nt) {
      const double v = Qb[D(j - k, k)];
      if (v != 0.0) s += H5[j + 1] * v * T.au[pair_raw(c[k], c[j])];
    }
    s = block_sum(s, red);
    if (tid == 0) H5[k] = H5[k + 1] * scp[1] + s;
    __syncthreads();
  }
#ifdef SK_FOLD_TIMING
  const uint64_t tk2 = clock64();
#endif

  // ---------------------------------------------------------------- outside
  // (the ring now holds the Hb diagonals above the span: every one read was
  // written by an earlier span of this pass)
  double* __restrict__ out = P.out + sq.out_off;
  for (int d = n - 1; d >= 4; --d) {
    const int ncell = n - d;
    const int G = team_of(ncell, nt);
    for (int base = 0; base < ncell; base += nt / G) {
      const int i0 = base + tid / G, r = tid % G;
      const bool on = i0 < ncell;
      const int i = on ? i0 : 0, j = i + d;
      // Hm(i,j): Qm(i,j2) += Qm(i,j) Qm1(j+1,j2);  Qb(i-1,j') ML rule with u = j
      double hm = 0.0;
      if (on) {
#pragma unroll 4
        for (int j2 = j + 5 + r; j2 < n; j2 += G) hm += Hm[D(j2 - i, i)] * Qm1[D(j2 - j - 1, j + 1)];
        if (i >= 1) {
          for (int jp = j + 6 + r; jp < n; jp += G) {
            const double v = Hb[D(jp - i + 1, i - 1)];
            if (v == 0.0) continue;
            const int t1 = ptype(i - 1, jp);
            if (!t1 || (ncg && is_gu(t1))) continue;
            hm += v * T.mlc * T.au[t1] * scp[2] * Qm1[D(jp - j - 2, j + 1)];
          }
        }
      }
      hm = team_sum(hm, G);
      if (on && r == 0) Hm[D(d, i)] = hm;
      // Hm1(i,j): Qm(ii,j) += (sc^(i-ii) + Qm(ii,i-1)) Qm1(i,j), ii <= i;
      //           Qb(i',j+1) ML rule with u + 1 = i
      // (ii = i - e, e up: the threads read consecutive doubles)
      double hm1 = 0.0;
      if (on) {
#pragma unroll 4
        for (int e = r; e <= i; e += G) {
          const double v = e == 0 ? hm : Hm[D(d + e, i - e)];
          if (v != 0.0) hm1 += v * (scp[e] + (e >= 1 ? Qm[D(e - 1, i - e)] : 0.0));
        }
        if (j + 1 < n) {
          for (int e = 6 + r; e <= i; e += G) {  // ip = i - e
            const double v = Hb[D(d + 1 + e, i - e)];
            if (v == 0.0) continue;
            const int t1 = ptype(i - e, j + 1);
            if (!t1 || (ncg && is_gu(t1))) continue;
            hm1 += v * T.mlc * T.au[t1] * scp[2] * Qm[D(e - 2, i - e + 1)];
          }
        }
      }
      hm1 = team_sum(hm1, G);
      if (on && r == 0) Hm1[D(d, i)] = hm1;
      // Hb(i,j): exterior branch, Qm1(i,jj) += Qb(i,j) (branch) sc^(jj-j),
      //          enclosing interior loops (ip, jp) = (i-1-n1, j+1+n2):
      //          diagonal d+2+n1+n2
      const int t = on ? ptype(i, j) : 0;
      double part = 0.0;
      if (t) {
        double s = r == 0 ? hm1 : 0.0;
#pragma unroll 4
        for (int jj = j + 1 + r; jj < n; jj += G) s += Hm1[D(jj - i, i)] * scp[jj - j];
        part = s * T.mli * T.au[t];
        const int t2 = pair_raw(c[j], c[i]);
        for (int n1 = r; n1 <= min(30, i - 1); n1 += G) {
          const int ip = i - 1 - n1;
          const int n2m = min(30 - n1, n - 2 - j);
          int sl = slot(d + 2 + n1);
          for (int n2 = 0; n2 <= n2m; ++n2) {
            const double v = RING ? ring[(size_t)sl * P.ring_n + ip] : Hb[D(d + 2 + n1 + n2, ip)];
            sl = up(sl);
            if (v == 0.0) continue;
            const int t1 = ptype(ip, j + 1 + n2);
            if (!t1) continue;
            part += v * fold_interior(T, t1, t2, n1, n2, ncg) * scp[n1 + n2 + 2];
          }
        }
      }
      part = team_sum(part, G);
      if (on && r == 0) {
        const double hb = t ? H5[j + 1] * Q5[i] * T.au[t] + part : 0.0;
        const double qbij = Qb[D(d, i)];
        Hb[D(d, i)] = hb;
        if (RING) ring[(size_t)slot(d) * P.ring_n + i] = hb;
        out[(size_t)i * n - (size_t)i * (i + 1) / 2 + (size_t)(j - i - 1)] = qbij != 0.0 ? qbij * hb / Z : 0.0;
      }
    }
    __syncthreads();
  }
#ifdef SK_FOLD_TIMING
  if (tid == 0 && blockIdx.x < 2)
    printf("fold b%d n %d inside %lu exterior %lu outside %lu\n", (int)blockIdx.x, n, (unsigned long)(tk1 - tk0),
           (unsigned long)(tk2 - tk1), (unsigned long)(clock64() - tk2));
#endif
}

static size_t fold_lds_bytes_t(const FoldLaunch& P, int max_n, bool gtab) {
  const bool ring = fold_ring(max_n);
  const size_t ntab = gtab ? (size_t)((P.n_small + 1) & ~1) : (size_t)P.n_tab_pad;
  return (ntab + (ring ? (size_t)kFoldRing * max_n : 0)) * 8 + (size_t)(max_n + 15) / 16 * 16;
}

bool fold_gtab(const FoldLaunch& P, int max_n) { return fold_lds_bytes_t(P, max_n, false) > kFoldLdsMax; }

size_t fold_lds_bytes(const FoldLaunch& P, int max_n) {
  return fold_lds_bytes_t(P, max_n, fold_gtab(P, max_n));
}

bool fold_ring(int max_n) { return max_n <= kFoldRingMaxN; }

template <bool RING, bool GTAB>
static hipError_t launch_fold_t(const FoldLaunch& P, int n_seqs, size_t lds, hipStream_t st) {
  hipError_t e = hipFuncSetAttribute((const void*)sk_fold_kernel<RING, GTAB>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((sk_fold_kernel<RING, GTAB>), dim3(n_seqs), dim3(512), lds, st, P);
  return hipGetLastError();
}

hipError_t launch_fold(const FoldLaunch& P0, int n_seqs, int max_n, hipStream_t st) {
  if (n_seqs <= 0) return hipSuccess;
  FoldLaunch P = P0;
  P.ring_n = fold_ring(max_n) ? max_n : 0;
  const size_t lds = fold_lds_bytes(P, max_n);
  if (lds > kFoldLdsMax) return hipErrorInvalidValue;
  if (fold_ring(max_n)) return launch_fold_t<true, false>(P, n_seqs, lds, st);  // (tables always fit)
  return fold_gtab(P, max_n) ? launch_fold_t<false, true>(P, n_seqs, lds, st)
                             : launch_fold_t<false, false>(P, n_seqs, lds, st);
}

}  // namespace sk
