/* ORACLE (test infrastructure only): CPU restatement of the engine's
 * McCaskill base-pairing-probability fold (sk_fold_mccaskill), and an
 * exhaustive enumeration that pins the restatement's recursions.
 *
 * Only tests/ (and nothing in the product) load this.
 *
 * The reference folds with ViennaRNA's pf_fold (common/bpmatrix.cpp:151-177,
 * common/pf_wrapper.cpp:15-36; ViennaRNA >= 1.6, legacy API, not vendored).
 * Its energy parameter files are not in this image, so this model keeps the
 * loop decomposition and the Turner-1999 tables the legacy library compiles
 * in for stacks, hairpin / bulge / interior initiation, Ninio asymmetry,
 * terminal AU / GU penalties and the linear multiloop, and leaves out the
 * terminal-mismatch, dangle, special-hairpin and 1x1/1x2/2x2 tables:
 * parity against ViennaRNA is UNPINNED.  What is pinned: the DP equals the
 * Boltzmann sum over every secondary structure (orc_fold_enum) under the
 * loop energies orc_fold_loop_energy defines.
 *
 * Model (energies in dcal/mol at 37 C, positions 0-based, pair types CG=1,
 * GC=2, GU=3, UG=4, AU=5, UA=6; kT = (37+273.15)*1.98717/10 dcal/mol):
 *   hairpin (i,j), n = j-i-1 >= 3:   H[min(n,30)] + (n>30 ? lxc ln(n/30)) + AU(ij)
 *   stack (i,j)/(p,q):               S[t(i,j)][t(q,p)]
 *   bulge, n = n1+n2 (one side 0):   B[n] + (n==1 ? S[..][..] : AU(ij)+AU(qp))
 *   interior, n1,n2 > 0:             I[n] + min(300, 50|n1-n2|) + AU(ij) + AU(qp)
 *   (interior and bulge loops with n1+n2 > 30 are not formed)
 *   multiloop closed by (i,j):       a + b + AU(ij), each branch b + AU, unpaired 0
 *   exterior branch:                 AU
 *   AU(t) = 50 for t in {GU, UG, AU, UA}, else 0.
 *   noGU: GU/UG never pair; noClosingGU: GU/UG close no hairpin, bulge,
 *   interior or multiloop (a GU may still stack).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define ORC_INF 1e300
#define MAXLOOP 30

static const double kT = (37.0 + 273.15) * 1.98717 / 10.0;
static const double lxc = 107.856;
static const int stack37[7][7] = {
    {0, 0, 0, 0, 0, 0, 0},
    {0, -240, -330, -210, -140, -210, -210},
    {0, -330, -340, -250, -150, -220, -240},
    {0, -210, -250, 130, -50, -140, -130},
    {0, -140, -150, -50, 30, -60, -100},
    {0, -210, -220, -140, -60, -110, -90},
    {0, -210, -240, -130, -100, -90, -130}};
static const int hairpin37[31] = {0,   0,   0,   570, 560, 560, 540, 590, 560, 640, 650,
                                  660, 670, 678, 686, 694, 701, 707, 713, 719, 725, 730,
                                  735, 740, 744, 749, 753, 757, 761, 765, 769};
static const int bulge37[31] = {0,   380, 280, 320, 360, 400, 440, 459, 470, 480, 490,
                                500, 510, 519, 527, 534, 541, 548, 554, 560, 565, 571,
                                576, 580, 585, 589, 594, 598, 602, 605, 609};
static const int interior37[31] = {0,   0,   410, 510, 170, 180, 200, 220, 230, 240, 250,
                                   260, 270, 278, 286, 294, 301, 307, 313, 319, 325, 330,
                                   335, 340, 345, 349, 353, 357, 361, 365, 369};
static const int ML_closing = 340, ML_intern = 40, TerminalAU = 50, ninio = 50, max_ninio = 300;

static int base_code(char c) {
  switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'U': case 'u': case 'T': case 't': return 3;
    default: return -1;
  }
}

static int pair_type(int a, int b) {
  static const int t[4][4] = {{0, 0, 0, 5}, {0, 0, 1, 0}, {0, 2, 0, 4}, {6, 0, 3, 0}};
  return (a < 0 || b < 0) ? 0 : t[a][b];
}

typedef struct {
  int n;
  int *s;  /* base codes */
  int no_gu, no_closing_gu;
  unsigned char *lp;  /* --noLonelyPairs: lp[i*n+j] = the pair survives the filter (NULL: off) */
} fold_in;

static int ptype_raw(const fold_in *F, int i, int j) {
  int t = pair_type(F->s[i], F->s[j]);
  if (F->no_gu && (t == 3 || t == 4)) return 0;
  return t;
}
static int ptype(const fold_in *F, int i, int j) {
  int t = ptype_raw(F, i, j);
  if (t && F->lp && !F->lp[(size_t)i * F->n + j]) return 0;
  return t;
}

/* --noLonelyPairs (common/bpmatrix.cpp:56-58, 149: Vienna::noLonelyPairs
 * before pf_fold).  The legacy ViennaRNA partition function (1.8,
 * part_func.c make_ptypes; not vendored, restated from its published
 * source) applies it only through the pair-type table: walking each chain of
 * pairs (i, j), (i-1, j+1), ... outward from its innermost pair, a pair
 * whose inner neighbour was removed or cannot pair, and whose outer
 * neighbour cannot pair, is removed (it "can only form isolated pairs").  As
 * written there the outer-neighbour type is only re-read while i > 1 and
 * j < n (1-based), so at a chain's outermost pair it still holds that
 * pair's own type: such a pair is kept whenever it can pair (unless it is
 * also the chain's innermost pair).  Chains start at j - i = 4 and 5
 * (0-based: hairpins of 3 and 4). */
static void lonely_filter(fold_in *F) {
  int n = F->n;
  F->lp = (unsigned char *)calloc((size_t)(n ? n : 1) * (n ? n : 1), 1);
  for (int k = 0; k < n; ++k)
    for (int l = 1; l <= 2; ++l) {
      int i = k, j = k + 3 + l, otype = 0, ntype = 0, type;
      if (j >= n) continue;
      type = ptype_raw(F, i, j);
      while (i >= 0 && j < n) {
        if (i > 0 && j < n - 1) ntype = ptype_raw(F, i - 1, j + 1);
        if (!otype && !ntype) type = 0;
        F->lp[(size_t)i * n + j] = type != 0;
        otype = type;
        type = ntype;
        --i;
        ++j;
      }
    }
}
static int is_gu(int t) { return t == 3 || t == 4; }
static double au(int t) { return t > 2 ? (double)TerminalAU : 0.0; }

/* loop energies (dcal/mol); ORC_INF = loop not formed */
static double e_hairpin(const fold_in *F, int i, int j) {
  int t = ptype(F, i, j), n = j - i - 1;
  if (!t || n < 3) return ORC_INF;
  if (F->no_closing_gu && is_gu(t)) return ORC_INF;
  double e = hairpin37[n <= 30 ? n : 30];
  if (n > 30) e += lxc * log((double)n / 30.0);
  return e + au(t);
}

static double e_interior(const fold_in *F, int i, int j, int p, int q) {
  int t1 = ptype(F, i, j), t2 = pair_type(F->s[q], F->s[p]);  /* inner pair, reversed */
  int n1 = p - i - 1, n2 = j - q - 1, n = n1 + n2;
  if (!t1 || !ptype(F, p, q) || n > MAXLOOP) return ORC_INF;
  if (n == 0) return stack37[t1][t2];
  if (F->no_closing_gu && (is_gu(t1) || is_gu(t2))) return ORC_INF;
  if (n1 == 0 || n2 == 0) return bulge37[n] + (n == 1 ? stack37[t1][t2] : au(t1) + au(t2));
  double asym = ninio * (double)abs(n1 - n2);
  if (asym > max_ninio) asym = max_ninio;
  return interior37[n] + asym + au(t1) + au(t2);
}

static double e_ml_closing(const fold_in *F, int i, int j) {
  int t = ptype(F, i, j);
  if (!t || (F->no_closing_gu && is_gu(t))) return ORC_INF;
  return ML_closing + ML_intern + au(t);
}
static double e_ml_branch(const fold_in *F, int p, int q) { return ML_intern + au(ptype(F, p, q)); }
static double e_ext_branch(const fold_in *F, int p, int q) { return au(ptype(F, p, q)); }

static double boltz(double e) { return e >= ORC_INF ? 0.0 : exp(-e / kT); }

/* flags bit 0 no_gu, 1 no_closing_gu, 2 no_lonely_pairs (the library's
 * SK_FOLD_* bits); the older two-flag entry points pass no_closing_gu alone */
static int setup(fold_in *F, const char *seq, int no_gu, int no_closing_gu) {
  F->n = (int)strlen(seq);
  F->s = (int *)malloc(sizeof(int) * (F->n ? F->n : 1));
  for (int k = 0; k < F->n; ++k) F->s[k] = base_code(seq[k]);
  F->no_gu = no_gu;
  F->no_closing_gu = no_closing_gu & 1;
  F->lp = NULL;
  if (no_closing_gu & 2) lonely_filter(F);
  return F->n;
}
static void teardown(fold_in *F) {
  free(F->s);
  free(F->lp);
}

static size_t tri(int n, int i, int j) { return (size_t)i * n - (size_t)i * (i + 1) / 2 + (size_t)(j - i - 1); }

/* ------------------------------------------------------------------ DP */
/* McCaskill inside / outside over Qb (pair i.j closes a loop), Qm1 (one
 * multiloop branch starting at i, unpaired to j), Qm (>= 1 branch), Q5
 * (exterior prefix); outside values as adjoints of the inside rules.
 * bpp (packed strict upper triangle, optional); returns ln Z. */
double orc_fold_mccaskill(const char *seq, int no_gu, int no_closing_gu, double *bpp) {
  fold_in F;
  int n = setup(&F, seq, no_gu, no_closing_gu);
  if (n == 0) {
    teardown(&F);
    return 0.0;
  }
  size_t N2 = (size_t)n * n;
  double *Qb = calloc(N2, sizeof(double)), *Qm = calloc(N2, sizeof(double)),
         *Qm1 = calloc(N2, sizeof(double));
  double *Hb = calloc(N2, sizeof(double)), *Hm = calloc(N2, sizeof(double)),
         *Hm1 = calloc(N2, sizeof(double));
  double *Q5 = calloc(n + 1, sizeof(double)), *H5 = calloc(n + 1, sizeof(double));
#define A(M, i, j) M[(size_t)(i) * n + (j)]
  for (int d = 4; d < n; ++d) {
    for (int i = 0; i + d < n; ++i) {
      int j = i + d;
      double qb = 0.0;
      if (ptype(&F, i, j)) {
        qb = boltz(e_hairpin(&F, i, j));
        for (int p = i + 1; p <= j - 5 && p - i - 1 <= MAXLOOP; ++p)
          for (int q = j - 1; q >= p + 4 && (p - i - 1) + (j - q - 1) <= MAXLOOP; --q)
            if (A(Qb, p, q) != 0.0) qb += A(Qb, p, q) * boltz(e_interior(&F, i, j, p, q));
        double ml = 0.0;
        for (int u = i + 5; u + 5 <= j - 1; ++u) ml += A(Qm, i + 1, u) * A(Qm1, u + 1, j - 1);
        qb += ml * boltz(e_ml_closing(&F, i, j));
      }
      A(Qb, i, j) = qb;
      double m1 = 0.0;
      for (int l = i + 4; l <= j; ++l)
        if (A(Qb, i, l) != 0.0) m1 += A(Qb, i, l) * boltz(e_ml_branch(&F, i, l));
      A(Qm1, i, j) = m1;
      double m = 0.0;
      for (int u = i; u + 4 <= j; ++u) m += (1.0 + (u - 1 >= i ? A(Qm, i, u - 1) : 0.0)) * A(Qm1, u, j);
      A(Qm, i, j) = m;
    }
  }
  Q5[0] = 1.0;
  for (int j = 0; j < n; ++j) {
    double q = Q5[j];
    for (int k = 0; k + 4 <= j; ++k)
      if (A(Qb, k, j) != 0.0) q += Q5[k] * A(Qb, k, j) * boltz(e_ext_branch(&F, k, j));
    Q5[j + 1] = q;
  }
  double Z = Q5[n];
  if (bpp) {
    memset(bpp, 0, sizeof(double) * (size_t)n * (n - 1) / 2);
    H5[n] = 1.0;
    for (int j = n - 1; j >= 0; --j) {  /* Q5[j+1] = Q5[j] + sum_k Q5[k] Qb(k,j) ext */
      H5[j] += H5[j + 1];
      for (int k = 0; k + 4 <= j; ++k) {
        double w = boltz(e_ext_branch(&F, k, j));
        H5[k] += H5[j + 1] * A(Qb, k, j) * w;
        A(Hb, k, j) += H5[j + 1] * Q5[k] * w;
      }
    }
    for (int d = n - 1; d >= 4; --d) {
      for (int i = 0; i + d < n; ++i) {
        int j = i + d;
        /* Qm(i,j): final (larger spans only).  Propagate its rule. */
        double hm = A(Hm, i, j);
        for (int u = i; u + 4 <= j; ++u) {
          A(Hm1, u, j) += hm * (1.0 + (u - 1 >= i ? A(Qm, i, u - 1) : 0.0));
          if (u - 1 >= i) A(Hm, i, u - 1) += hm * A(Qm1, u, j);
        }
        /* Qm1(i,j): final now (the u = i term above was this cell's own). */
        double hm1 = A(Hm1, i, j);
        for (int l = i + 4; l <= j; ++l) A(Hb, i, l) += hm1 * boltz(e_ml_branch(&F, i, l));
        /* Qb(i,j): final now. */
        double hb = A(Hb, i, j);
        if (ptype(&F, i, j) && hb != 0.0) {
          for (int p = i + 1; p <= j - 5 && p - i - 1 <= MAXLOOP; ++p)
            for (int q = j - 1; q >= p + 4 && (p - i - 1) + (j - q - 1) <= MAXLOOP; --q)
              A(Hb, p, q) += hb * boltz(e_interior(&F, i, j, p, q));
          double c = hb * boltz(e_ml_closing(&F, i, j));
          for (int u = i + 5; u + 5 <= j - 1; ++u) {
            A(Hm, i + 1, u) += c * A(Qm1, u + 1, j - 1);
            A(Hm1, u + 1, j - 1) += c * A(Qm, i + 1, u);
          }
        }
        if (A(Qb, i, j) != 0.0) bpp[tri(n, i, j)] = A(Qb, i, j) * hb / Z;
      }
    }
  }
#undef A
  free(Qb); free(Qm); free(Qm1); free(Hb); free(Hm); free(Hm1); free(Q5); free(H5); teardown(&F);
  return log(Z);
}

/* ------------------------------------------------------------------ energy of a structure */
/* pt[i] = partner of i or -1.  Loop decomposition; ORC_INF if a loop is not
 * formed by the model (e.g. an interior loop over MAXLOOP). */
static double struct_energy(const fold_in *F, const int *pt) {
  double e = 0.0;
  int n = F->n;
  for (int i = 0; i < n; ++i) {
    if (pt[i] > i) {  /* loop closed by (i, pt[i]) */
      int j = pt[i];
      int nb = 0, bp_ = -1, bq_ = -1;
      for (int k = i + 1; k < j; ++k) {
        if (pt[k] > k) {
          ++nb;
          if (nb == 1) { bp_ = k; bq_ = pt[k]; }
          k = pt[k];
        }
      }
      double le;
      if (nb == 0) le = e_hairpin(F, i, j);
      else if (nb == 1) le = e_interior(F, i, j, bp_, bq_);
      else {
        le = e_ml_closing(F, i, j);
        for (int k = i + 1; k < j; ++k)
          if (pt[k] > k) {
            le += e_ml_branch(F, k, pt[k]);
            k = pt[k];
          }
      }
      if (le >= ORC_INF) return ORC_INF;
      e += le;
    }
  }
  for (int k = 0; k < n; ++k)
    if (pt[k] > k) {
      e += e_ext_branch(F, k, pt[k]);
      k = pt[k];
    }
  return e;
}

double orc_fold_structure_energy(const char *seq, const int *pt, int no_gu, int no_closing_gu) {
  fold_in F;
  setup(&F, seq, no_gu, no_closing_gu);
  for (int i = 0; i < F.n; ++i)
    if (pt[i] > i && !ptype(&F, i, pt[i])) {
      teardown(&F);
      return ORC_INF;
    }
  double e = struct_energy(&F, pt);
  teardown(&F);
  return e;
}

/* ------------------------------------------------------------------ enumeration */
typedef struct {
  fold_in *F;
  int *pt;
  double Z;
  double *bpp;
  long count;
} enum_st;

static void enum_rec(enum_st *E, int i) {
  int n = E->F->n;
  while (i < n && E->pt[i] >= 0) ++i;  /* already paired (as a right partner) */
  if (i >= n) {
    double e = struct_energy(E->F, E->pt);
    if (e < ORC_INF) {
      double w = exp(-e / kT);
      E->Z += w;
      ++E->count;
      if (E->bpp)
        for (int a = 0; a < n; ++a)
          if (E->pt[a] > a) E->bpp[tri(n, a, E->pt[a])] += w;
    }
    return;
  }
  /* i unpaired */
  enum_rec(E, i + 1);
  /* i paired with j: past i's minimal hairpin and inside the innermost pair
   * enclosing i (every position between is still free) */
  int lim = n;
  for (int k = i - 1; k >= 0; --k)
    if (E->pt[k] > i) {
      lim = E->pt[k];
      break;
    }
  for (int j = i + 4; j < lim; ++j) {
    if (!ptype(E->F, i, j)) continue;
    E->pt[i] = j;
    E->pt[j] = i;
    enum_rec(E, i + 1);
    E->pt[i] = E->pt[j] = -1;
  }
}

/* Boltzmann sum over every secondary structure (exponential: short
 * sequences only); bpp as in orc_fold_mccaskill; returns ln Z. */
double orc_fold_enum(const char *seq, int no_gu, int no_closing_gu, double *bpp, long *n_struct) {
  fold_in F;
  int n = setup(&F, seq, no_gu, no_closing_gu);
  enum_st E;
  E.F = &F;
  E.pt = (int *)malloc(sizeof(int) * (n ? n : 1));
  for (int k = 0; k < n; ++k) E.pt[k] = -1;
  E.Z = 0.0;
  E.bpp = bpp;
  E.count = 0;
  if (bpp && n > 1) memset(bpp, 0, sizeof(double) * (size_t)n * (n - 1) / 2);
  enum_rec(&E, 0);
  if (bpp && n > 1)
    for (size_t k = 0; k < (size_t)n * (n - 1) / 2; ++k) bpp[k] /= E.Z;
  if (n_struct) *n_struct = E.count;
  free(E.pt);
  teardown(&F);
  return log(E.Z);
}
