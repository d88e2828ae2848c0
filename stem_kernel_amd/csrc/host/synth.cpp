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
//
// Layout: every table is stored by diagonal, X(i, i+e) at D[e+1][i] (e = -1
// holds the empty spans, Q = 1), so for four neighbouring cells (i..i+3, j =
// i + d) each term of the k loop -- Q(i, k-1), B(k, j), Q(k+1, j-1), and in
// the outside pass the updates of O(i, k-1), O(k+1, j-1), P(k, j) -- is one
// contiguous 4-wide access.  Four cells of a diagonal run side by side: each
// cell's value is formed by the same operations in the same order as the
// scalar loop (bit-identical output; fp contraction off), four independent
// add chains instead of one.  In the outside pass the four cells' updates
// never hit one element (two cells i < i' of a diagonal share a target only
// when i' - i >= hp + 1 = 4), so updating them side by side keeps the
// scalar loop's order per element.
// (an unaligned 4-double vector: plain dereferences, no vector-valued
// functions, so the AVX2 clone and the baseline one share one source)
typedef double sk_v4d __attribute__((vector_size(32), aligned(8)));
#define v4_ld(p) (*reinterpret_cast<const sk_v4d*>(p))
#define v4_st(p, v) (*reinterpret_cast<sk_v4d*>(p) = (v))

// AVX2 where the host has it (no FMA: the products and sums stay separate)
__attribute__((target_clones("avx2", "default"))) void fold_nussinov(const char* seq, int n, bool no_gu, double* out) {
#pragma STDC FP_CONTRACT OFF
  if (n < 2) return;
  const double s = 2.0, inv_s = 1.0 / s, inv_s2 = inv_s * inv_s;
  const int hp = 3;
  // diagonal e (-1 .. n-1) starts at off[e + 1]; n - e cells (n + 1 for e = -1)
  thread_local std::vector<size_t> off;
  off.assign((size_t)n + 2, 0);
  for (int e = -1; e < n; ++e) off[e + 2] = off[e + 1] + (size_t)(e < 0 ? n + 1 : n - e) + 4;  // +4: vector tails
  const size_t tot = off[n + 1];
  thread_local std::vector<double> Q, O, B, P;
  Q.assign(tot, 0.0);
  O.assign(tot, 0.0);
  B.assign(tot, 0.0);
  P.assign(tot, 0.0);
  auto D = [&](std::vector<double>& X, int e) { return X.data() + off[e + 1]; };
  for (int i = 0; i <= n; ++i) D(Q, -1)[i] = 1.0;
  for (int e = hp + 1; e < n; ++e)
    for (int i = 0; i + e < n; ++i) D(B, e)[i] = pair_weight(seq[i], seq[i + e], no_gu) * inv_s2;
  for (int d = 0; d < n; ++d) {
    const int m = n - d;  // cells of diagonal d
    const double* qd1 = D(Q, d - 1);
    double* qd = D(Q, d);
    int i = 0;
    for (; i + 4 <= m; i += 4) {
      sk_v4d v = v4_ld(qd1 + i) * inv_s;
      for (int t = 0; t <= d - hp - 1; ++t) v += v4_ld(D(Q, t - 1) + i) * v4_ld(D(B, d - t) + i + t) * v4_ld(D(Q, d - t - 2) + i + t + 1);
      v4_st(qd + i, v);
    }
    for (; i < m; ++i) {
      double v = qd1[i] * inv_s;
      for (int t = 0; t <= d - hp - 1; ++t) v += D(Q, t - 1)[i] * D(B, d - t)[i + t] * D(Q, d - t - 2)[i + t + 1];
      qd[i] = v;
    }
  }
  const double Z = D(Q, n - 1)[0];
  D(O, n - 1)[0] = 1.0;
  for (int d = n - 1; d >= 0; --d) {
    const int m = n - d;
    const double* od = D(O, d);
    double* od1 = D(O, d - 1);  // (d = 0: the e = -1 row, written and never read)
    int i = 0;
    for (; i + 4 <= m; i += 4) {
      const sk_v4d o = v4_ld(od + i);
      if (o[0] == 0.0 && o[1] == 0.0 && o[2] == 0.0 && o[3] == 0.0) continue;
      if (d >= 1) v4_st(od1 + i, v4_ld(od1 + i) + o * inv_s);
      for (int t = 0; t <= d - hp - 1; ++t) {
        const sk_v4d b = v4_ld(D(B, d - t) + i + t);
        const sk_v4d left = v4_ld(D(Q, t - 1) + i);
        const sk_v4d inner = v4_ld(D(Q, d - t - 2) + i + t + 1);
        if (t >= 1) {
          double* orow = D(O, t - 1) + i;
          v4_st(orow, v4_ld(orow) + o * b * inner);
        }
        double* ocol = D(O, d - t - 2) + i + t + 1;
        v4_st(ocol, v4_ld(ocol) + o * b * left);
        double* pp = D(P, d - t) + i + t;
        v4_st(pp, v4_ld(pp) + o * left * b * inner);
      }
    }
    for (; i < m; ++i) {
      const double o = od[i];
      if (o == 0.0) continue;
      if (d >= 1) od1[i] += o * inv_s;
      for (int t = 0; t <= d - hp - 1; ++t) {
        const double b = D(B, d - t)[i + t];
        const double left = D(Q, t - 1)[i];
        const double inner = D(Q, d - t - 2)[i + t + 1];
        if (t >= 1) D(O, t - 1)[i] += o * b * inner;
        D(O, d - t - 2)[i + t + 1] += o * b * left;
        D(P, d - t)[i + t] += o * left * b * inner;
      }
    }
  }
  size_t t = 0;
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j) out[t++] = D(P, j - i)[i] / Z;
}

void random_sequence(uint64_t& state, int len, char* out) {
  static const char kBases[4] = {'A', 'C', 'G', 'U'};
  for (int i = 0; i < len; ++i) out[i] = kBases[splitmix64_next(state) >> 62];
  out[len] = 0;
}

}  // namespace sk
