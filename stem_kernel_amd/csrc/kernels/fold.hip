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

__constant__ int8_t kFoldPair[16] = {0, 0, 0, 5, 0, 0, 1, 0, 0, 2, 0, 4, 6, 0, 3, 0};  // CG1 GC2 GU3 UG4 AU5 UA6

struct FoldTables {  // views into P.tab (FoldLaunch::tab layout)
  const double *st, *hp, *bu, *in, *ni, *au, *scp;
  double mlc, mli;
};

__device__ __forceinline__ int pair_raw(int a, int b) { return (a < 0 || b < 0) ? 0 : kFoldPair[a * 4 + b]; }
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

// block-wide sum (256 threads), result in every thread
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

__global__ void __launch_bounds__(256) sk_fold_kernel(FoldLaunch P) {
  __shared__ double red[8];
  const FoldSeq sq = P.seqs[blockIdx.x];
  const int n = sq.n;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int8_t* __restrict__ c = P.codes + sq.seq_off;
  const size_t N2 = (size_t)n * n;
  double* W = P.work + sq.work_off;
  double *Qb = W, *Qm = W + N2, *QmT = W + 2 * N2, *Qm1 = W + 3 * N2, *Qm1T = W + 4 * N2;
  double *Hb = W + 5 * N2, *HbT = W + 6 * N2, *Hm = W + 7 * N2, *HmT = W + 8 * N2, *Hm1 = W + 9 * N2;
  double *Q5 = W + 10 * N2, *H5 = Q5 + n + 1;
  FoldTables T;
  T.st = P.tab + P.o_st;
  T.hp = P.tab + P.o_hp;
  T.bu = P.tab + P.o_bu;
  T.in = P.tab + P.o_in;
  T.ni = P.tab + P.o_ni;
  T.au = P.tab + P.o_au;
  T.scp = P.tab + P.o_scp;
  T.mlc = P.tab[P.o_ml];
  T.mli = P.tab[P.o_ml + 1];
  const double* scp = T.scp;
  const bool ngu = P.no_gu != 0, ncg = P.no_closing_gu != 0;
  const uint8_t* __restrict__ lp = P.lp ? P.lp + sq.lp_off : nullptr;
  auto ptype = [&](int i, int j) {
    const int t = pair_raw(c[i], c[j]);
    if (lp && !lp[(size_t)i * n + j]) return 0;  // --noLonelyPairs (host table)
    return (ngu && is_gu(t)) ? 0 : t;
  };

  // ---------------------------------------------------------------- inside
  for (int d = 4; d < n; ++d) {
    for (int i = tid; i + d < n; i += nt) {
      const int j = i + d;
      const int t = ptype(i, j);
      double qb = 0.0;
      if (t) {
        if (!(ncg && is_gu(t))) qb = T.hp[d - 1] * T.au[t] * scp[d + 1];  // hairpin, n = d-1 >= 3
        for (int p = i + 1; p <= j - 5 && p - i - 1 <= 30; ++p) {
          const int n1 = p - i - 1;
          const int qmin = max(p + 4, j - 1 - (30 - n1));
          const double* __restrict__ row = Qb + (size_t)p * n;
          for (int q = j - 1; q >= qmin; --q) {
            const double v = row[q];
            if (v != 0.0) {
              const int n2 = j - q - 1;
              qb += v * fold_interior(T, t, pair_raw(c[q], c[p]), n1, n2, ncg) * scp[n1 + n2 + 2];
            }
          }
        }
        if (!(ncg && is_gu(t))) {
          double ml = 0.0;
          const double* __restrict__ a = Qm + (size_t)(i + 1) * n;
          const double* __restrict__ b = Qm1T + (size_t)(j - 1) * n;
          for (int u = i + 5; u + 5 <= j - 1; ++u) ml += a[u] * b[u + 1];
          qb += ml * T.mlc * T.au[t] * scp[2];
        }
      }
      Qb[(size_t)i * n + j] = qb;
      double m1 = 0.0;
      for (int l = i + 4; l <= j; ++l) {
        const double v = Qb[(size_t)i * n + l];
        if (v != 0.0) m1 += v * T.mli * T.au[pair_raw(c[i], c[l])] * scp[j - l];
      }
      Qm1[(size_t)i * n + j] = m1;
      Qm1T[(size_t)j * n + i] = m1;
      double m = 0.0;
      for (int u = i; u + 4 <= j; ++u)
        m += (scp[u - i] + (u - 1 >= i ? Qm[(size_t)i * n + u - 1] : 0.0)) * Qm1T[(size_t)j * n + u];
      Qm[(size_t)i * n + j] = m;
      QmT[(size_t)j * n + i] = m;
    }
    __syncthreads();
  }

  // ---------------------------------------------------------------- exterior
  if (tid == 0) Q5[0] = 1.0;
  __syncthreads();
  for (int j = 0; j < n; ++j) {
    double s = 0.0;
    for (int k = tid; k + 4 <= j; k += nt) {
      const double v = Qb[(size_t)k * n + j];
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
      const double v = Qb[(size_t)k * n + j];
      if (v != 0.0) s += H5[j + 1] * v * T.au[pair_raw(c[k], c[j])];
    }
    s = block_sum(s, red);
    if (tid == 0) H5[k] = H5[k + 1] * scp[1] + s;
    __syncthreads();
  }

  // ---------------------------------------------------------------- outside
  double* __restrict__ out = P.out + sq.out_off;
  for (int d = n - 1; d >= 4; --d) {
    for (int i = tid; i + d < n; i += nt) {
      const int j = i + d;
      // Hm(i,j): Qm(i,j2) += Qm(i,j) Qm1(j+1,j2);  Qb(i-1,j') ML rule with u = j
      double hm = 0.0;
      {
        const double* __restrict__ h = Hm + (size_t)i * n;
        const double* __restrict__ q1 = Qm1 + (size_t)(j + 1) * n;
        for (int j2 = j + 5; j2 < n; ++j2) hm += h[j2] * q1[j2];
        if (i >= 1) {
          const double* __restrict__ hb = Hb + (size_t)(i - 1) * n;
          for (int jp = j + 6; jp < n; ++jp) {
            const double v = hb[jp];
            if (v == 0.0) continue;
            const int t1 = ptype(i - 1, jp);
            if (!t1 || (ncg && is_gu(t1))) continue;
            hm += v * T.mlc * T.au[t1] * scp[2] * q1[jp - 1];
          }
        }
      }
      Hm[(size_t)i * n + j] = hm;
      HmT[(size_t)j * n + i] = hm;
      // Hm1(i,j): Qm(ii,j) += (sc^(i-ii) + Qm(ii,i-1)) Qm1(i,j), ii <= i;
      //           Qb(i',j+1) ML rule with u + 1 = i
      double hm1 = 0.0;
      {
        const double* __restrict__ hmt = HmT + (size_t)j * n;
        const double* __restrict__ qmt = i >= 1 ? QmT + (size_t)(i - 1) * n : nullptr;
        for (int ii = 0; ii <= i; ++ii) {
          const double v = hmt[ii];
          if (v != 0.0) hm1 += v * (scp[i - ii] + (ii <= i - 1 ? qmt[ii] : 0.0));
        }
        if (j + 1 < n) {
          const double* __restrict__ hbt = HbT + (size_t)(j + 1) * n;
          for (int ip = 0; ip <= i - 6; ++ip) {
            const double v = hbt[ip];
            if (v == 0.0) continue;
            const int t1 = ptype(ip, j + 1);
            if (!t1 || (ncg && is_gu(t1))) continue;
            hm1 += v * T.mlc * T.au[t1] * scp[2] * qmt[ip + 1];
          }
        }
      }
      Hm1[(size_t)i * n + j] = hm1;
      // Hb(i,j): exterior branch, Qm1(i,jj) += Qb(i,j) (branch) sc^(jj-j),
      //          enclosing interior loops
      const int t = ptype(i, j);
      double hb = 0.0;
      const double qbij = Qb[(size_t)i * n + j];
      if (t) {
        hb = H5[j + 1] * Q5[i] * T.au[t];
        const double* __restrict__ h1 = Hm1 + (size_t)i * n;
        double s = 0.0;
        for (int jj = j; jj < n; ++jj) s += h1[jj] * scp[jj - j];
        hb += s * T.mli * T.au[t];
        const int t2 = pair_raw(c[j], c[i]);
        for (int ip = i - 1; ip >= 0 && i - ip - 1 <= 30; --ip) {
          const int n1 = i - ip - 1;
          const double* __restrict__ row = Hb + (size_t)ip * n;
          for (int jp = j + 1; jp < n && n1 + (jp - j - 1) <= 30; ++jp) {
            const double v = row[jp];
            if (v == 0.0) continue;
            const int t1 = ptype(ip, jp);
            if (!t1) continue;
            const int n2 = jp - j - 1;
            hb += v * fold_interior(T, t1, t2, n1, n2, ncg) * scp[n1 + n2 + 2];
          }
        }
      }
      Hb[(size_t)i * n + j] = hb;
      HbT[(size_t)j * n + i] = hb;
      out[(size_t)i * n - (size_t)i * (i + 1) / 2 + (size_t)(j - i - 1)] = qbij != 0.0 ? qbij * hb / Z : 0.0;
    }
    __syncthreads();
  }
}

hipError_t launch_fold(const FoldLaunch& P, int n_seqs, hipStream_t st) {
  if (n_seqs <= 0) return hipSuccess;
  hipLaunchKernelGGL(sk_fold_kernel, dim3(n_seqs), dim3(256), 0, st, P);
  return hipGetLastError();
}

}  // namespace sk
