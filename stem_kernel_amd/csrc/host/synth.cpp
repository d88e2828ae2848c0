// Synthetic inputs for the stem-kernel engine.
//
// * Sequences: a splitmix64 stream -- base = "ACGU"[x >> 62].
// * Base-pairing probabilities: a Boltzmann-weighted Nussinov partition
//   function (GC/CG e^1.5, AU/UA e^1.0, GU/UG e^0.5, hairpin >= 3 unpaired),
//   inside + outside in O(L^3).  This stands in for ViennaRNA's pf_fold
//   (common/bpmatrix.cpp:151-177, common/pf_wrapper.cpp:15-36), which is not
//   available in this image; it is NOT Vienna's energy model.  Its output is
//   the same packed strict-upper-triangle layout the engine consumes, so any
//   real folding engine's matrix can be passed in its place.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "sk_internal.h"

namespace sk {

uint64_t splitmix64_next(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static double pair_weight(char a, char b, bool no_gu) {
  auto lc = [](char c) { return (c >= 'A' && c <= 'Z') ? char(c - 'A' + 'a') : c; };
  a = lc(a);
  b = lc(b);
  if (a == 't') a = 'u';
  if (b == 't') b = 'u';
  if ((a == 'g' && b == 'c') || (a == 'c' && b == 'g')) return std::exp(1.5);
  if ((a == 'a' && b == 'u') || (a == 'u' && b == 'a')) return std::exp(1.0);
  if (!no_gu && ((a == 'g' && b == 'u') || (a == 'u' && b == 'g'))) return std::exp(0.5);
  return 0.0;
}

// Inside/outside over the grammar  S(i,j) -> S(i,j-1) | S(i,k-1) (k S(k+1,j-1) j)
// with spans scaled by s^-(len) to stay in range.  Output: p(i,j), i<j, 0-based,
// packed strict upper triangle.
void fold_nussinov(const char* seq, int n, bool no_gu, double* out) {
  if (n < 2) return;
  const double s = 2.0, inv_s = 1.0 / s, inv_s2 = inv_s * inv_s;
  const int hp = 3;
  // Q(i,j) for 0<=i<=j<n; empty spans (j=i-1) are 1.  Q is kept in both
  // layouts (QT[j][i] = Q[i][j]) and B, P transposed, so every k loop below
  // walks memory contiguously; each value is formed by the same operations
  // in the same order as the row-major loops (bit-identical output).
  auto at = [n](int i, int j) { return (size_t)i * n + j; };
  // per-thread workspace: repeated folds reuse already-faulted pages
  thread_local std::vector<double> Q, QT, O, BT, PT;
  Q.assign((size_t)n * n, 0.0);
  QT.assign((size_t)n * n, 0.0);
  O.assign((size_t)n * n, 0.0);
  BT.assign((size_t)n * n, 0.0);  // BT[j][k] = B(k, j)
  auto q = [&](int i, int j) -> double { return j < i ? 1.0 : Q[at(i, j)]; };
  for (int i = 0; i < n; ++i)
    for (int j = i + hp + 1; j < n; ++j) BT[at(j, i)] = pair_weight(seq[i], seq[j], no_gu) * inv_s2;
  for (int d = 0; d < n; ++d) {
    for (int i = 0; i + d < n; ++i) {
      const int j = i + d;
      double v = q(i, j - 1) * inv_s;
      const double* __restrict__ bj = &BT[at(j, 0)];
      const double* __restrict__ qi = &Q[at(i, 0)];
      const double* __restrict__ qtj = &QT[at(j - 1 >= 0 ? j - 1 : 0, 0)];
      // k = i (left span empty), then the rest; a pair that cannot form
      // adds an exact +0 (v > 0), so no branch is needed on b
      // (inner = q(k+1, j-1) always has k+1 <= j-3)
      if (i <= j - hp - 1) v += 1.0 * bj[i] * qtj[i + 1];
      for (int k = i + 1; k <= j - hp - 1; ++k) v += qi[k - 1] * bj[k] * qtj[k + 1];
      Q[at(i, j)] = v;
      QT[at(j, i)] = v;
    }
  }
  const double Z = Q[at(0, n - 1)];
  O[at(0, n - 1)] = 1.0;
  PT.assign((size_t)n * n, 0.0);  // PT[j][k] = P(k, j)
  for (int d = n - 1; d >= 0; --d) {
    for (int i = 0; i + d < n; ++i) {
      const int j = i + d;
      const double o = O[at(i, j)];
      if (o == 0.0) continue;
      if (j - 1 >= i) O[at(i, j - 1)] += o * inv_s;
      const double* __restrict__ bj = &BT[at(j, 0)];
      const double* __restrict__ qi = &Q[at(i, 0)];
      const double* __restrict__ qtj = &QT[at(j - 1 >= 0 ? j - 1 : 0, 0)];
      double* __restrict__ pj = &PT[at(j, 0)];
      // (every term of a pair that cannot form is an exact +0: no branch;
      // inner = q(k+1, j-1) always has k+1 <= j-3)
      double* __restrict__ oi = &O[at(i, 0)];
      for (int k = i; k <= j - hp - 1; ++k) {
        const double b = bj[k];
        const double left = k - 1 >= i ? qi[k - 1] : 1.0;
        const double inner = qtj[k + 1];
        if (k - 1 >= i) oi[k - 1] += o * b * inner;
        O[at(k + 1, j - 1)] += o * b * left;
        pj[k] += o * left * b * inner;
      }
    }
  }
  size_t t = 0;
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j) out[t++] = PT[at(j, i)] / Z;
}

void random_sequence(uint64_t& state, int len, char* out) {
  static const char kBases[4] = {'A', 'C', 'G', 'U'};
  for (int i = 0; i < len; ++i) out[i] = kBases[splitmix64_next(state) >> 62];
  out[len] = 0;
}

}  // namespace sk
