/*
 * stem_kernel.h -- C ABI of the MI355X stem-kernel Gram engine.
 *
 * Drop-in boundary for the reference's hot path (keio-bioinformatics/stem_kernel
 * rev 296): the per-pair kernel DP evaluated for every (i,j) cell of the Gram
 * matrix by KernelMatrix::calculate (common/kernel_matrix.h:67-105,
 * common/kernel_matrix.cpp:485-575).  Each entry point below names the
 * reference interface it replaces.  Plain pointers and sizes only; every call
 * returns SK_OK (0) or a negative sk_status and never throws.  Host buffers are
 * caller-owned; device buffers (sk_*_device) are addresses in the context's HIP
 * device.
 *
 * Semantics kept from the reference:
 *   - K(x,y) is evaluated with x = row example, y = column example, only for
 *     i <= j, and mirrored (kernel_matrix.cpp:44-55): the DAG kernel is not
 *     symmetric;
 *   - normalisation K_ij / sqrt(K_ii K_jj), diagonal := 1, only when asked
 *     (kernel_matrix.cpp:560-571); NaN from non-positive diagonals propagates;
 *   - libsvm precomputed-kernel text layout (kernel_matrix.cpp:756-770).
 */
#ifndef STEM_KERNEL_H
#define STEM_KERNEL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SK_ABI_VERSION 2

typedef enum {
  SK_OK = 0,
  SK_ERR_INVALID = -1,    /* bad argument (the reference threw const char*) */
  SK_ERR_HIP = -2,        /* HIP runtime error */
  SK_ERR_NO_DEVICE = -3,  /* no gfx950 device / HIP unavailable */
  SK_ERR_ALLOC = -4,      /* host or device allocation failed */
  SK_ERR_RANGE = -5,      /* index out of range */
  SK_ERR_UNSUPPORTED = -6 /* kernel kind / size not supported */
} sk_status;

/* Kernel kinds: the instantiations stem_kernel_lite/main.cpp:180-215 dispatches
 * to, plus their components (stem_kernel_lite/def_kernel.h, ss_kernel.h). */
typedef enum {
  SK_SU_STEM = 0,      /* SuStemKernel(loop_gap, beta, band)        --no-string     */
  SK_SI_STEM = 1,      /* SiStemKernel(loop_gap, stack, covar, band) --no-string --no-ribosum */
  SK_SU_STR = 2,       /* StringKernel(gap, alpha)                                  */
  SK_SI_STR = 3,       /* StringKernel(gap, match, mismatch)                        */
  SK_SU_STEM_STR = 4,  /* SuStemStrKernel == StemStrKernel (ss_kernel.h)  default   */
  SK_SI_STEM_STR = 5,  /* SiStemStrKernel                                --no-ribosum */
  SK_LSU_STEM = 6,     /* LSuStemKernel: beta*log(K_stem)                --log --no-string */
  SK_LSU_STEM_STR = 7, /* LSuStemStrKernel: beta*log K_stem + alpha*log K_str  --log */
  SK_NAIVE_STR = 8,    /* StringKernel<double>(gap) of string_kernel/ (exact character
                          match of row 0, weight gap^2, string_kernel.cpp:11-50) */
  /* BPLAKernel<double,MData> of bpla_kernel/ (bpla_kernel.cpp:159-174) */
  SK_BPLA = 9,         /* local_alignment_exp with BPLAScore            (default)    */
  SK_LA = 10,          /* local_alignment_exp with LAScore               --noBP      */
  SK_BPLA_SW = 11,     /* local_alignment_max with BPLAScore             --SW        */
  SK_LA_SW = 12,       /* local_alignment_max with LAScore               --noBP --SW */
  /* StemKernel<double,BPMat>::full_dp of stem_kernel/ (stem_kernel.cpp:282-351)
   * over single sequences (row 0, lowercased as the loader does) */
  SK_STEM4D = 13
} sk_kernel_kind;

/* Kernel parameters; defaults are stem_kernel_lite/main.cpp:103-149
 * (sk_kernel_params_default).  BPLA kinds use alpha, beta, gap, ext and
 * score_table with the defaults of bpla_kernel/main.cpp:20-26, 68-76; that
 * CLI parses them as float, so the defaults are float-rounded. */
typedef struct {
  int32_t kind;       /* sk_kernel_kind */
  uint32_t len_band;  /* --length-band (0 = off), default 10 */
  double beta;        /* -b   0.3 */
  double loop_gap;    /* -g   0.2 */
  double stack;       /* -s   1.3 */
  double covar;       /* -v   0.8 */
  double alpha;       /* -a   0.2 */
  double gap;         /* -G   0.8 */
  double match;       /* --match 1.0 */
  double mismatch;    /* --mismatch 0.8 */
  double ext;         /* BPLA -e (gap extension), -0.75 */
  double score_table[16]; /* BPLA --score table, [x residue][y residue] ACGU */
  /* 4-D stem kernel (stem_kernel/main.cpp:40-60; float options): gap -g 0.8,
   * stack -s 1.0 (fields above), and: */
  double subst;       /* -v substitution weight for base pairs, 0.5 */
  double bp_bound;    /* -p pairs count when prob > bp_bound (float compare), 0.0 */
  int32_t bp_model;   /* 0: dataset bpp (BPMatrix/PFWrapper, the -p path),
                         1: NormalBasePair, 2: WobbleBasePair (-w) */
  uint32_t loop;      /* -l minimum loop (Normal/Wobble models), 3 */
  /* -a alignment constraints (stem_kernel.cpp:14-81): when > 0, partial_dp
   * restricted to the PairHMM MAP path's match positions whose posterior is
   * >= ali_bound (PairHMM<Ribosum>, stem_kernel/phmm.cpp), widened by
   * len_band; 0.0 = off.  Sequences must then be ACGU only (the reference
   * asserts in char2rna, phmm.cpp:247-258). */
  double ali_bound;   /* float option, compared as float */
  /* LogValue zerop semantics (log_value.h:374-378).  0: as the reference
   * builds with a C++11 <cmath> (std::isinf returns bool, `<0` is never true,
   * posteriors are NaN and no position is anchored); 1: the intended -inf
   * test (anchored constraints). */
  int32_t ali_zerop_fixed;
} sk_kernel_params;

void sk_kernel_params_default(sk_kernel_params *p, int32_t kind);

/* ---------------------------------------------------------------- context */
typedef struct sk_context sk_context;

/* One context per GPU (HIP device ordinal).  hip_stream may be NULL (the
 * context creates its own) or a hipStream_t owned by the caller. */
int sk_open(int device, void *hip_stream, sk_context **ctx);
int sk_close(sk_context *ctx);
const char *sk_strerror(int status);
/* Last error message recorded on this context (static storage). */
const char *sk_last_error(const sk_context *ctx);

/* ---------------------------------------------------------------- examples */
/* An example set: the reference's ExampleSet of (label, MData)
 * (common/framework.h:308-353), built host-side and uploaded once. */
typedef struct sk_dataset sk_dataset;

int sk_dataset_create(sk_dataset **ds);
int sk_dataset_free(sk_dataset *ds);

/* Append one example = one alignment of n_rows rows of equal length.
 * bpp_rows[r]: base-pairing probabilities of row r after erase_gap (length
 * n_r = number of non-'-' characters), strict upper triangle packed row-major:
 * p(i,j), 0<=i<j<n_r, at i*n_r - i*(i+1)/2 + (j-i-1).  This is the matrix
 * Vienna pf_fold would give the reference (common/bpmatrix.cpp:151-177).
 * th = --basepair.  use_bp = 0 builds MData(ma) (no DAG; string kernels only).
 * Replaces: new MData(ma, th, pf_scale, opts)  stem_kernel_lite/data.cpp:324-345
 * and DataLoader<MData>::get()  stem_kernel_lite/data.cpp:548-586. */
int sk_dataset_add(sk_dataset *ds, const char *label, int n_rows,
                   const char *const *rows, const double *const *bpp_rows,
                   float th, int use_bp);
/* Append n single-sequence examples, folding each with sk_fold_synthetic and
 * building its DAG on n_threads host threads (0 = hardware concurrency).
 * labels may be NULL ("+1").  Parallel form of the reference's load loop
 * (common/framework.h:308-353 + DataLoader<MData>::get). */
int sk_dataset_add_synthetic(sk_dataset *ds, int32_t n, const char *const *seqs,
                             const char *const *labels, float th, int32_t n_threads);
/* Same for alignments: n examples of n_rows equal-length rows each, rows
 * [i*n_rows + r]; every row is folded gap-erased and lowercased, then the
 * per-row matrices are averaged (common/bpmatrix.cpp:306-342, 399-417). */
int sk_dataset_add_synthetic_rows(sk_dataset *ds, int32_t n, int32_t n_rows,
                                  const char *const *rows, const char *const *labels,
                                  float th, int32_t n_threads);
/* Append a copy of example i of src (its built DAG, profile and weights: no
 * rebuild) to dst, e.g. to assemble the pair a per-pair Kernel::operator()
 * call evaluates from examples built once.  dst must not be uploaded yet. */
int sk_dataset_add_copy(sk_dataset *dst, const sk_dataset *src, int32_t i);
int sk_dataset_size(const sk_dataset *ds);
/* Examples [first, first + count) as bytes -- their labels, built DAGs,
 * profiles, weights and averaged bp matrices, every field as the dataset
 * holds it -- into buf (cap bytes); *size = the bytes needed (buf NULL: query
 * only; SK_ERR_RANGE when cap is short).  sk_dataset_import appends such a
 * buffer's examples to ds (not uploaded; a malformed buffer appends nothing):
 * ranks that each build a share of the examples and gather the shares in
 * rank order hold a dataset that packs bit for bit as one built whole
 * (stem_kernel_amd/shard.py build_split).  Host-side counterpart of the
 * reference's MPI Gram, where every rank reads and builds every example
 * (common/kernel_matrix.cpp:186-261, common/framework.h:308-353). */
int sk_dataset_export(const sk_dataset *ds, int32_t first, int32_t count, uint8_t *buf,
                      size_t cap, size_t *size);
int sk_dataset_import(sk_dataset *ds, const uint8_t *buf, size_t size);
/* Diagnostic: pack ds on the host (ds not uploaded) and return FNV-1a hashes
 * of every packed array, y-role records and x-role / per-example arrays (the
 * lists of tools/pack_compare.cpp). */
int sk_dataset_pack_digest(sk_dataset *ds, uint64_t *y_hash, uint64_t *x_hash);
/* label of example i (pointer valid while ds lives) */
const char *sk_dataset_label(const sk_dataset *ds, int i);
/* DAG shape of example i: nodes, edges, bp_freq entries, roots, length */
int sk_dataset_shape(const sk_dataset *ds, int i, int32_t *n_nodes,
                     int32_t *n_edges, int32_t *n_bpfreq, int32_t *n_roots,
                     int32_t *seq_len);
/* Row traffic of example i in the x role of the DAG stem kernel's gamma
 * schedule (dag_stem.hip): its rows (the x nodes the schedule
 * computes per pair), the rows it stores in the HBM slab, and the child-row
 * reads of its rows from the slab, the y's Gamma and Phi tables and
 * registers; y_slots = its non-leaf node count, the length of every row a
 * pair (x', example i as y) moves.  Per pair (x, y) the engine moves each of
 * x's row transfers as 8 * y_slots(y) bytes.  Replaces nothing in the
 * reference (its DP keeps K0/G0 tables per pair in host memory,
 * stem_kernel_lite/stem_kernel.cpp:14-95): a roofline input of bench.py.
 * The dataset must be uploaded (packed). */
int sk_dataset_row_traffic(const sk_dataset *ds, int i, int32_t *rows, int32_t *stored,
                           int32_t *slab_reads, int32_t *gamma_reads, int32_t *phi_reads,
                           int32_t *reg_reads, int32_t *y_slots);
/* DAG arrays of example i (packer-parity introspection; any pointer may be
 * NULL).  Node arrays have n_nodes entries, edge arrays n_edges (node-major,
 * reference list order), bp arrays n_bpfreq. */
int sk_dataset_dag(const sk_dataset *ds, int i, uint32_t *first, uint32_t *last,
                   uint32_t *n_edges, uint32_t *n_bpfreq, float *weight,
                   uint32_t *max_pa, uint32_t *edge_to, uint32_t *edge_gaps,
                   uint32_t *bp_code, float *bp_p, uint32_t *roots,
                   float *pos_weight);

/* ProfileSequence of example i (common/profile.cpp): prof5 gets len*5 floats
 * (A,C,G,U,gap), *n_seqs the row count. */
int sk_dataset_profile(const sk_dataset *ds, int i, float *prof5, float *n_seqs);

/* BPLA position weights of example i (bpla_kernel/data.cpp:19-45: sqrt of
 * the left, right and unpaired probabilities; 0,0,1 without base pairs),
 * len floats each (packer-parity introspection). */
int sk_dataset_bpla_weights(const sk_dataset *ds, int i, float *p_left,
                            float *p_right, float *p_unpair);

/* Upload the packed example set to the context's device (idempotent).
 * Must be called after the last sk_dataset_add and before any compute. */
int sk_dataset_upload(sk_context *ctx, sk_dataset *ds);

/* ---------------------------------------------------------------- compute */
/* Train Gram matrix: K(train[i], train[j]) for i<=j, mirrored, optional
 * normalisation.  out: n*n doubles, row-major, host memory.
 * Replaces: KernelMatrix<double>::calculate(train, kernel, normalize, n_th)
 *           common/kernel_matrix.cpp:485-575. */
int sk_gram(sk_context *ctx, sk_dataset *ds, const sk_kernel_params *kp,
            int normalize, double *out);

/* Arbitrary (x,y) pair list, results to a DEVICE buffer out_dev[k] =
 * K(ds[x[k]], ds[y[k]]).  No normalisation.  Asynchronous on the context's
 * stream; host arrays are read before return.  Used by row-block shards
 * (multi-GPU) and by the benchmark.
 * Replaces: the inner loop CalcTrainMatrix::operator() kernel_matrix.cpp:42-56
 * (and the MPI variant's per-rank share, kernel_matrix.cpp:186-261). */
int sk_pairs_device(sk_context *ctx, sk_dataset *ds, const sk_kernel_params *kp,
                    const int32_t *x, const int32_t *y, int64_t n_pairs,
                    double *out_dev);
/* Same, host output (synchronous). */
int sk_pairs(sk_context *ctx, sk_dataset *ds, const sk_kernel_params *kp,
             const int32_t *x, const int32_t *y, int64_t n_pairs, double *out);

/* Test row: out[i] = K(train[i], test[t]) for i in sv_index[0..n_sv) (all i
 * when sv_index == NULL); out has n_train entries and entries outside
 * sv_index are left untouched (the reference indexes by train position).
 * *self = K(test[t], test[t]) when self != NULL.  test and train may be the
 * same dataset.
 * Replaces: KernelMatrix::calculate(vec, data, train, sv_index, kernel, n_th,
 * data_self)  common/kernel_matrix.cpp:112-182, 635-697. */
int sk_test_row(sk_context *ctx, sk_dataset *test, int t, sk_dataset *train,
                const int32_t *sv_index, int32_t n_sv,
                const sk_kernel_params *kp, double *out, double *self);

/* Diagonal: out[i] = K(train[i], train[i]) for i in sv_index (or all i);
 * out has n_train entries.
 * Replaces: KernelMatrix::diagonal  common/kernel_matrix.cpp:59-110, 577-633. */
int sk_diagonal(sk_context *ctx, sk_dataset *ds, const int32_t *sv_index,
                int32_t n_sv, const sk_kernel_params *kp, double *out);

/* Test x train matrix: out[i*n_train + j] = K(train[j], test[i]).  When
 * norm_test || normalize, self_out[i] = K(test[i], test[i]) (self_out may be
 * NULL otherwise); when normalize, out[i][j] /= sqrt(self[i] * diag[j]).
 * Replaces: KernelMatrix::calculate(test, train, kernel, norm_test,
 * normalize, n_th)  common/kernel_matrix.cpp:699-754. */
int sk_test_matrix(sk_context *ctx, sk_dataset *test, sk_dataset *train,
                   const sk_kernel_params *kp, int norm_test, int normalize,
                   double *out, double *self_out);

/* ---------------------------------------------------------------- multi-GPU
 * One process (or host thread) per GPU, one context each.  The plan is the
 * reference MPI Gram's: upper-triangle cell k (i <= j, row-major) belongs to
 * rank k % world (CalcTrainMatrix::operator(), common/kernel_matrix.cpp:
 * 210-224).  Each rank computes its cells into a device buffer of
 * sk_shard_count(n, 0, world) doubles, one RCCL all-gather over xGMI joins
 * them on every rank, and every rank assembles the mirrored (normalised)
 * matrix -- the reference's Ssend/Recv to rank 0 and its scatter
 * (:225-261, 495-527).  The result is bit-identical to sk_gram. */
/* Cells of `rank` (host only, no GPU): count, and their (x, y) lists. */
int64_t sk_shard_count(int32_t n, int32_t rank, int32_t world);
int sk_shard_cells(int32_t n, int32_t rank, int32_t world, int32_t *x, int32_t *y);
/* Host assembly: gathered = world buffers of per_rank doubles (rank-major,
 * rank r's values in sk_shard_cells order); out = n*n, mirrored, normalised
 * as kernel_matrix.cpp:560-571 when normalize. */
int sk_shard_assemble(int32_t n, int32_t world, const double *gathered, int64_t per_rank,
                      int normalize, double *out);
/* RCCL communicator of the context: rank 0 calls sk_comm_unique_id and
 * hands the 128 bytes to every rank (any channel: MPI_Bcast, a file, a
 * socket); each rank calls sk_comm_init on its own context. */
int sk_comm_unique_id(uint8_t *id, size_t id_bytes);
int sk_comm_init(sk_context *ctx, const uint8_t *id, size_t id_bytes, int32_t rank, int32_t world);
/* ncclAllGather of count doubles per rank on the context's stream
 * (asynchronous; device buffers, recv_dev holds world*count). */
int sk_comm_allgather(sk_context *ctx, const double *send_dev, int64_t count, double *recv_dev);
/* The Gram over the communicator's ranks: every rank passes the same dataset
 * and parameters and receives the whole n*n matrix in out (host).
 * Replaces: KernelMatrix<double>::calculate under HAVE_MPI,
 * common/kernel_matrix.cpp:186-261, 495-527. */
int sk_gram_sharded(sk_context *ctx, sk_dataset *ds, const sk_kernel_params *kp, int normalize,
                    double *out);

/* ---------------------------------------------------------------- output */
/* libsvm precomputed-kernel text: "label 0:(i+1) 1:K_i1 ... n:K_in \n" with
 * ostream default formatting (6 significant digits).  Writes into buf (NUL
 * terminated) if buf_size is large enough; *needed receives the byte count
 * including the NUL.  Replaces: KernelMatrix::print common/kernel_matrix.cpp:756-770. */
int sk_format_libsvm(const double *matrix, int32_t rows, int32_t cols,
                     const char *const *labels, char *buf, size_t buf_size,
                     size_t *needed);

/* ---------------------------------------------------------------- inputs */
/* Synthetic base-pairing probabilities: Boltzmann-weighted Nussinov partition
 * function (GC 1.5, AU 1.0, GU 0.5 in kT units, hairpin >= 3).  Stand-in for
 * Vienna pf_fold; out gets n*(n-1)/2 doubles in the packed layout above. */
int sk_fold_synthetic(const char *seq, int32_t n, int32_t no_gu, double *out);

/* McCaskill base-pairing probabilities on the GPU, one workgroup per
 * sequence (csrc/kernels/fold.hip).  Replaces ViennaRNA pf_fold as the
 * reference calls it: BPMatrix FOLD, common/bpmatrix.cpp:151-177 (per row of
 * an alignment, :404-414), PFWrapper::fold, common/pf_wrapper.cpp:15-36.
 * Loop model: the Turner-1999 core ViennaRNA 1.x compiles in (stacks,
 * hairpin / bulge / interior initiation, Ninio asymmetry, terminal AU/GU,
 * linear multiloop; no mismatch, dangle or special-loop tables: its
 * parameter files are not available, so parity against ViennaRNA is
 * unpinned -- DESIGN.md §9).  seqs[k]: any case, T as U, other characters
 * never pair.  out: for each k in order, n_k(n_k-1)/2 doubles in the packed
 * layout of sk_dataset_add, concatenated.  log_z (optional): ln Z per
 * sequence.  flags: SK_FOLD_NO_GU (--noGU), SK_FOLD_NO_CLOSING_GU
 * (--noClosingGU), SK_FOLD_NO_LONELY_PAIRS (--noLonelyPairs: the legacy
 * ViennaRNA pair-type filter, pairs that can only be isolated removed).  Sequences up to ~1,400 nt (SK_ERR_UNSUPPORTED when Z
 * leaves the double range). */
#define SK_FOLD_NO_GU 1
#define SK_FOLD_NO_CLOSING_GU 2
#define SK_FOLD_NO_LONELY_PAIRS 4
int sk_fold_mccaskill(sk_context *ctx, int32_t n, const char *const *seqs, int32_t flags,
                      double *out, double *log_z);
/* n examples of n_rows equal-length rows (rows[i*n_rows + r]), built on
 * n_threads host threads (0 = hardware concurrency) from the caller's
 * per-row bpp (bpp_rows[i*n_rows + r], layout of sk_dataset_add; ignored
 * when use_bp = 0).  Parallel form of the reference's load loop
 * (common/framework.h:308-353 + DataLoader<MData>::get,
 * stem_kernel_lite/data.cpp:548-586). */
int sk_dataset_add_batch(sk_dataset *ds, int32_t n, int32_t n_rows, const char *const *rows,
                         const double *const *bpp_rows, const char *const *labels, float th,
                         int32_t use_bp, int32_t n_threads);
/* Same, folding every gap-erased row with sk_fold_mccaskill on ctx's GPU
 * first: the engine's whole input path (MData(ma, th, pf_scale, opts),
 * data.cpp:324-345, with BPMatrix FOLD) without ViennaRNA. */
int sk_dataset_add_folded(sk_context *ctx, sk_dataset *ds, int32_t n, int32_t n_rows,
                          const char *const *rows, const char *const *labels, float th,
                          int32_t fold_flags, int32_t n_threads);

/* BPLA gradients, the bpla_optimizer's per-pair step: for k < n_pairs,
 * value[k] = BPLAKernel::compute_gradients(xs[x[k]], ys[y[k]], score_table,
 * {alpha, beta, gap, ext}, d) and grad[4k..4k+3] = d (d/d alpha, beta, gap,
 * ext).  Replaces bpla_kernel/bpla_kernel.cpp:385-401 (BPLA_Forward :178-243,
 * BPLA_Backward :245-305, BPLA_ForwardBackword :325-383) as called from
 * bpla_kernel/bpla_optimizer.cpp:52-255.  Uses kp->alpha/beta/gap/ext and
 * kp->score_table; examples need base pairs.  Host buffers; synchronous. */
int sk_bpla_gradients(sk_context *ctx, sk_dataset *xs, sk_dataset *ys, const sk_kernel_params *kp,
                      const int32_t *x, const int32_t *y, int64_t n_pairs, double *value,
                      double *grad);

/* ---------------------------------------------------------------- example files
 * The readers DataLoader<MData>::get (stem_kernel_lite/data.cpp:547-586) pulls
 * examples from, with the reference grammars' exact acceptance (Boost.Spirit
 * classic semantics, csrc/host/readers.cpp):
 *   SK_FMT_FASTA    load_fa   common/fa.cpp:13-55    one sequence per example
 *   SK_FMT_CLUSTAL  load_aln  common/aln.cpp:16-107  one alignment per example
 *   SK_FMT_MAF      load_maf  common/maf.cpp:15-49   one alignment block per example
 * Reading stops at the first example that does not parse.  SK_ERR_INVALID on a
 * missing file, aln's format_error or rows of unequal length ("wrong
 * alignment", data.cpp:574-578); sk_seqfile_last_error() (thread-local) says
 * which.  Rows are returned as written (gaps kept, case kept). */
typedef enum { SK_FMT_FASTA = 0, SK_FMT_CLUSTAL = 1, SK_FMT_MAF = 2 } sk_file_format;
typedef struct sk_seqfile sk_seqfile;
int sk_seqfile_read(const char *path, int32_t format, sk_seqfile **out);
int sk_seqfile_parse(const char *text, size_t len, int32_t format, sk_seqfile **out);
int sk_seqfile_free(sk_seqfile *f);
int64_t sk_seqfile_count(const sk_seqfile *f);                        /* examples */
int32_t sk_seqfile_rows(const sk_seqfile *f, int64_t i);              /* rows of example i */
const char *sk_seqfile_row(const sk_seqfile *f, int64_t i, int32_t r); /* NUL-terminated */
const char *sk_seqfile_last_error(void);
/* splitmix64 sequences over ACGU: n_seqs strings of length len written to
 * out (n_seqs*(len+1) bytes, NUL separated); *state advances. */
int sk_random_sequences(uint64_t *state, int32_t n_seqs, int32_t len, char *out);

/* ---------------------------------------------------------------- SVM prediction
 * Predict mode's Output (f3) feeds every test row through the libsvm models
 * of --model / --predict: SVMPredict (libsvm/svm_util.cpp:11-95) over the
 * reference's vendored libsvm 2.8x, restated in csrc/host/svm_predict.cpp.
 *   sk_svm_model_load   svm_load_model (libsvm/svm.cpp:1288-1475): text
 *                       model, any svm_type / kernel_type (precomputed:
 *                       an SV's value is its 1-based training index);
 *                       SK_ERR_INVALID with sk_svm_last_error() on failure.
 *   sk_svm_model_info   svm_get_svm_type / svm_get_nr_class / svm_get_labels
 *                       (svm.cpp:1024-1039; labels untouched when the model
 *                       has none), and whether probA/probB are present.
 *   sk_svm_predict      SVMPredict::do_svm_predict's arithmetic
 *                       (svm_util.cpp:41-80) on the test vector
 *                       make_svm_node(cnt, row) builds (x[0] = cnt,
 *                       x[i+1] = row[i], row = the test row over the training
 *                       examples): with probability != 0 and a C-SVC / nu-SVC
 *                       model, *label = svm_predict_probability
 *                       (svm.cpp:1152-1189) and values[0..nr_class) = the
 *                       class probabilities (zeros if the model has no
 *                       probA/probB: svm_predict's label); otherwise *label =
 *                       svm_predict (svm.cpp:1108-1150) and
 *                       values[0..max(nr_class(nr_class-1)/2, 1)) = the
 *                       decision values (svm_predict_values, svm.cpp:1053-1106). */
typedef struct sk_svm_model sk_svm_model;
int sk_svm_model_load(const char *path, sk_svm_model **out);
void sk_svm_model_free(sk_svm_model *m);
int sk_svm_model_info(const sk_svm_model *m, int32_t *svm_type, int32_t *nr_class, int32_t *labels,
                      int32_t *has_probability);
int sk_svm_predict(const sk_svm_model *m, int32_t cnt, const double *row, int32_t n, int32_t probability,
                   double *label, double *values);
const char *sk_svm_last_error(void);

/* ---------------------------------------------------------------- diagnostics */
/* Milliseconds spent in the last compute call's dominant kernel (DAG stem
 * DP), measured with HIP events on the context's stream, and its launch
 * count.  Algorithmic work of that launch: *cells = sum |Vx|*|Vy| over the
 * pairs (non-leaf nodes). */
int sk_last_timing(const sk_context *ctx, double *stem_ms, double *string_ms,
                   double *cells, int32_t *launches);
/* Summed durations of the last compute call's dominant-kernel launches (DAG
 * stem, 4-D stem or BPLA), each timed by HIP events around it on its own
 * stream, and their count: *ms_sum / *n_launches is the average launch
 * duration a kernel-trace profiler reports.  Launches on several streams
 * overlap, so the sum can exceed sk_last_timing's span. */
int sk_last_launch_ms(const sk_context *ctx, double *ms_sum, int32_t *n_launches);
/* Asynchronous compute calls (default off).  With on != 0, sk_pairs_device
 * (and every call that returns its results on the device) returns once its
 * work is enqueued on the context's stream, so the host plans call t+1
 * while the GPU runs call t; host inputs are staged through pinned buffers,
 * so they may be freed when the call returns.  Results are ready after a
 * stream synchronisation.  The timing queries above then report totals:
 * sk_sync_timing waits for every call since the previous sk_sync_timing and
 * makes their summed timings (spans, launches, cells) what sk_last_timing and
 * sk_last_launch_ms return.  Turning async off resolves what is pending. */
int sk_set_async(sk_context *ctx, int32_t on);
int sk_sync_timing(sk_context *ctx);
/* Kernel instantiations launched by the last compute call (parity-coverage
 * diagnostic): *stem_maxk_mask has bit MAXK/4 set for every DAG stem register
 * class run (MAXK = 4, 8, ..., 32 64-node slots per lane; bit 17 for the MAXK 17
 * class, y examples of 1,025-1,088 non-leaf nodes) and bit 0 when the
 * big-y kernel ran (y examples of 2,048 non-leaf nodes or more, or with a stem edge
 * gap over 1,023, which the register classes cannot hold); *stem4d_mask has
 * bit log2(CPL) set for every 4-D stem class run (CPL = 1, 2, 4, 8 cells per
 * lane), shifted by 4 for the banded (partial_dp) variant and by 8 for the
 * column-pipelined full_dp kernel. */
int sk_last_classes(const sk_context *ctx, uint32_t *stem_maxk_mask, uint32_t *stem4d_mask);
/* Shape the column-pipelined 4-D kernel takes for a full_dp Gram batch whose
 * x and y examples have lengths [min_len, max_len]: *nb chained columns per
 * group, *waves waves per pair, *pf rows fetched ahead per wave (diagnostic;
 * bench roofline).  *waves = 0 when that batch does not run on the column
 * kernel: max_len >= 512 (k-tiled span kernel), max_len over the column
 * kernel's x limit (2,048), or min_len too short for the column schedule. */
int sk_stem4d_col_shape(int32_t min_len, int32_t max_len, int32_t *nb, int32_t *waves, int32_t *pf);
/* RIBOSUM85-60 tables as compiled into the library (pinning tests). */
void sk_ribosum_tables(float *s16, float *p256);
int sk_char2rna(int c);
/* 1 in the experiments build (make exp: build/libstem_kernel_amd_exp.so, which
 * reads the A/B switches INTEGRATION.md lists from the environment), 0 in the
 * shipped library (no switches compiled in). */
int sk_experiments(void);

#ifdef __cplusplus
}
#endif
#endif /* STEM_KERNEL_H */
