/*
 * sk_oracle.h -- CPU ORACLE for the stem-kernel hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * This is a plain-C restatement of the reference algorithms
 * (keio-bioinformatics/stem_kernel rev 296), written from the reference
 * sources read as text.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it, and only as the checker; the product library
 * (stem_kernel_amd) never links or calls it.
 *
 * Pinning status:
 *   - alphabet (char2rna), IUPAC profile columns and the RIBOSUM85-60 tables
 *     are PINNED against the reference's own translation units
 *     (common/rna.cpp, common/profile.cpp, stem_kernel_lite/ribosum.cpp),
 *     compiled unmodified from /root/reference into oracle/_ref/ by
 *     oracle/Makefile and compared in tests/test_oracle_pinning.py;
 *   - the DAG builder and every kernel DP are "parity unpinned": the
 *     reference TUs that hold them need Boost, ViennaRNA and the
 *     configure-generated config.h, none of which exist in this image, and
 *     the reference ships no tests, fixtures or golden values.
 */
#ifndef SK_ORACLE_H
#define SK_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_mdata orc_mdata;

/* MData ctor (stem_kernel_lite/data.cpp:324-345) for one example of n_rows
 * aligned rows (equal length).  bpp_rows[r] is the base-pairing-probability
 * matrix of row r AFTER erase_gap (length n_r = #non-gap chars), packed as the
 * strict upper triangle, row-major: p(i,j), 0<=i<j<n_r at
 * index i*n_r - i*(i+1)/2 + (j-i-1).  (Stands for Vienna pf_fold output,
 * common/bpmatrix.cpp:166-173.)  th = --basepair threshold.
 * use_bp=0 gives MData(ma) (no DAG, empty weight; data.cpp:347-352). */
orc_mdata *orc_mdata_new(int n_rows, const char *const *rows,
                         const double *const *bpp_rows, float th, int use_bp);
void orc_mdata_free(orc_mdata *d);

/* DAG introspection (dag.h, data.h:33-37) for packer parity tests. */
int orc_mdata_n_nodes(const orc_mdata *d);
int orc_mdata_n_edges(const orc_mdata *d);
int orc_mdata_n_bpfreq(const orc_mdata *d);
int orc_mdata_seq_len(const orc_mdata *d);
/* node arrays (length n_nodes): first,last,n_edges,n_bpfreq,weight,max_pa */
void orc_mdata_nodes(const orc_mdata *d, uint32_t *first, uint32_t *last,
                     uint32_t *n_edges, uint32_t *n_bpfreq, float *weight,
                     uint32_t *max_pa);
/* edge arrays (length n_edges, node-major, list order): to, gaps */
void orc_mdata_edges(const orc_mdata *d, uint32_t *to, uint32_t *gaps);
/* bp_freq arrays (length n_bpfreq): code=a*4+b, p */
void orc_mdata_bpfreq(const orc_mdata *d, uint32_t *code, float *p);
int orc_mdata_n_roots(const orc_mdata *d);
void orc_mdata_roots(const orc_mdata *d, uint32_t *roots);
/* per-position weight (fill_weight, data.cpp:437-453) and profile columns
 * (ProfileSequence, common/profile.cpp) float[L][5], n_seqs */
void orc_mdata_weight(const orc_mdata *d, float *w);
void orc_mdata_profile(const orc_mdata *d, float *prof5, float *n_seqs);

/* Averaged bp matrix (common/bpmatrix.cpp:306-342), packed as above over the
 * aligned length. */
void orc_mdata_bpp(const orc_mdata *d, double *packed);

/* ---- kernels: each returns K(x,y) with x = row example, y = column ---- */
/* StemKernel<SubstScoreTable> (stem_kernel_lite/stem_kernel.cpp:14-95,
 * score_table.cpp:118-201) == SuStemKernel(loop_gap, beta, band) */
double orc_su_stem(const orc_mdata *x, const orc_mdata *y, double loop_gap,
                   double beta, unsigned band);
/* StemKernel<SimpleScoreTable> == SiStemKernel(loop_gap, stack, covar, band)
 * (def_kernel.h:11-33, score_table.cpp:14-53) */
double orc_si_stem(const orc_mdata *x, const orc_mdata *y, double loop_gap,
                   double stack, double covar, unsigned band);
/* StringKernel<double,MData> (stem_kernel_lite/string_kernel.cpp:10-132):
 * ribosum=1 -> ctor(gap, alpha); ribosum=0 -> ctor(gap, match, mismatch) */
double orc_profile_string(const orc_mdata *x, const orc_mdata *y, double gap,
                          int ribosum, double alpha, double match,
                          double mismatch);

/* RIBOSUM tables as restated (stem_kernel_lite/ribosum.cpp:6-120) */
void orc_ribosum_tables(float *s16, float *p256);
/* char2rna restated (common/rna.cpp:201-231) */
int orc_char2rna(int c);

/* Naive gapped string kernel (string_kernel/string_kernel.cpp:14-85) */
double orc_naive_string(const char *x, const char *y, double gap);

/* BPLA kernel (bpla_kernel/bpla_kernel.cpp:159-174): local-alignment
 * partition function (sw=0, :64-115) or Smith-Waterman score (sw=1,
 * :117-157) over profile columns, with the base-pairing score of BPLAScore
 * (no_bp=0, :48-62) or LAScore alone (no_bp=1, :24-43).  table16 is the 4x4
 * score table (row = x residue).  The CLI parses gap/ext/alpha/beta as float
 * (bpla_kernel/main.cpp:52-76): pass float-rounded values for CLI parity. */
double orc_bpla(const orc_mdata *x, const orc_mdata *y, int no_bp, int sw, double gap, double ext,
                double alpha, double beta, const double *table16);
/* fill_weight of bpla_kernel/data.cpp:19-45 (sqrt of left / right / unpaired
 * probabilities per aligned position); example built with use_bp. */
void orc_bpla_weights(const orc_mdata *d, float *p_left, float *p_right, float *p_unpair);

/* BPLAKernel::compute_gradients (bpla_kernel/bpla_kernel.cpp:178-401): the
 * forward value and d4[0..3] = d/d(alpha, beta, gap, ext); d4[4] = the
 * backward pass's total (equal to the value up to rounding).  Examples need
 * base pairs. */
double orc_bpla_gradients(const orc_mdata *x, const orc_mdata *y, double alpha, double beta,
                          double gap, double ext, const double *table16, double *d4);

/* 4-D stem kernel full_dp (stem_kernel/stem_kernel.cpp:282-351) of two
 * single sequences.  model 0: bpx/bpy are the strict-upper packed bpp of x
 * and y (PFWrapper pr; prob(i,i)=0); 1/2: NormalBasePair / WobbleBasePair
 * (:354-396, bpx/bpy unused).  Returns K0(0,|x|,0,|y|). */
double orc_stem4d(const char *x, const double *bpx, const char *y, const double *bpy,
                  double gap, double stack, double subst, float bp_bound, int model,
                  unsigned loop);
/* Banded variant: partial_dp (stem_kernel.cpp:113-280) with the -b band
 * constraints of alignment_constraints (ali_bound == 0, :66-72). */
double orc_stem4d_banded(const char *x, const double *bpx, const char *y, const double *bpy,
                         double gap, double stack, double subst, float bp_bound, int model,
                         unsigned loop, unsigned band);
void orc_stem4d_band(int n, int m, unsigned band, unsigned *c_low, unsigned *c_high);
/* partial_dp with the constraints of alignment_constraints(ali_bound, band)
 * (stem_kernel.cpp:14-81, the -a option); zerop_fixed selects LogValue's
 * zerop semantics (see sk_oracle.c).  NaN on a non-ACGU residue when
 * ali_bound > 0 (the reference asserts). */
double orc_stem4d_partial(const char *x, const double *bpx, const char *y, const double *bpy,
                          double gap, double stack, double subst, float bp_bound, int model,
                          unsigned loop, unsigned band, float ali_bound, int zerop_fixed);
/* PairHMM posteriors fw*bk/w (phmm.cpp:10-115): fb[s][i][j], s = M, IX, IY,
 * 3*(|x|+1)*(|y|+1) doubles.  -1 on a non-ACGU residue. */
int orc_phmm_posterior(const char *x, const char *y, int zerop_fixed, double *fb);
/* alignment_constraints (stem_kernel.cpp:14-81): c_low/c_high, |x|+1 each. */
int orc_alignment_constraints(const char *x, const char *y, float ali_bound, unsigned band,
                              int zerop_fixed, unsigned *c_low, unsigned *c_high);

#ifdef __cplusplus
}
#endif
#endif
