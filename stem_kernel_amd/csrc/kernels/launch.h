// Launch descriptors shared by the host runtime (sk_api.cpp) and the kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "device_set.h"

namespace sk {

struct StemLaunch {
  DevSet xset;        // row examples (x role)
  DevSet yset;        // column examples (y role); may equal xset
  DevParamNodes pn;   // parameter-dependent node values of xset
  const double* co_subst = nullptr;  // 256: node-score table (pair x pair)
  const double* gpow = nullptr;      // loop_gap^k, k < n_gpow
  int32_t n_gpow = 0, n_gpow_pad = 0;
  double gap2 = 0.0;                 // loop_gap^2
  uint32_t band = 0;                 // --length-band (0 = off)
  // LDS sizing (maxima over the y examples of this launch)
  int32_t lds_max_nl = 0, lds_max_edges = 0, lds_max_bpf = 0, lds_max_nch = 0;
  int32_t lds_max_len_pad = 0;  // length -> first node table (max node length + 2, padded)
  // work: items {y, base, count, 0}; pair t of an item is x = xs[base+t],
  // result -> out[oidx[base+t]]
  const int4* items = nullptr;
  int32_t n_items = 0;
  const int32_t* xs = nullptr;
  const int64_t* oidx = nullptr;
  double* out = nullptr;
  int* item_counter = nullptr;
  double* scratch = nullptr;   // per-wave G0 slabs
  int64_t slab_doubles = 0;
  // Gamma rows (gam_on: the x set has gamma keys): per-workgroup table of
  // xset.n_gam rows of 64*MAXK doubles, Gamma_g(y) of the current item's y
  double* gam = nullptr;
  int64_t gam_doubles = 0;  // per workgroup
  int32_t gam_on = 0;
  // Phi rows (phi_on: the x set has phi keys): per-workgroup table of
  // xset.n_phi rows of 64*MAXK doubles and their n_phi sums; the item's phi
  // keys item_phi[item_phi_off[it] .. item_phi_off[it + 1])
  double* phi = nullptr;
  int64_t phi_doubles = 0;  // per workgroup
  const int32_t* item_phi_off = nullptr;
  const int32_t* item_phi = nullptr;
  int32_t phi_on = 0;
  unsigned long long* stamps = nullptr;  // diagnostic builds (SK_STAMPS) only
};

// DAG stem kernel for y examples the register classes cannot hold
// (dag_stem_big.hip): one wavefront per pair, the y DAG in level order from
// HBM (L2-resident), rows S and G1 in per-wave scratch next to the G0 slab.
struct StemBigLaunch {
  DevSet xset, yset;
  DevParamNodes pn;
  const double* co_subst = nullptr;
  const double* gpow = nullptr;
  int32_t n_gpow = 0;
  double gap2 = 0.0;
  uint32_t band = 0;
  const int32_t* xs = nullptr;   // pair k: K(x = xs[k], y = ys[k]) -> out[oidx[k]]
  const int32_t* ys = nullptr;
  const int64_t* oidx = nullptr;
  int64_t n_pairs = 0;
  double* out = nullptr;
  double* scratch = nullptr;     // per wave: (slots + 1) G0 rows, S, G1 (stride doubles each)
  int64_t stride = 0;            // >= max y non-leaf nodes, multiple of 64
  int64_t wave_doubles = 0;      // (slots + 3) * stride
};
hipError_t launch_stem_big(const StemBigLaunch& P, int grid, hipStream_t st);
constexpr int kStemBigWaves = 4;  // waves per workgroup (independent pairs)

struct StrLaunch {
  DevSet xset, yset;
  const double* st = nullptr;    // 16: exp(alpha*ribosum_s) or match/mismatch
  const double* gpow = nullptr;  // gap^k, k <= max_len
  double gap = 0.0;
  int32_t naive = 0;  // StringKernel<double> of string_kernel/: exact char match, g^2, no weights
  const int32_t* xs = nullptr;
  const int32_t* ys = nullptr;
  int64_t n_pairs = 0;
  double* out = nullptr;
  const int64_t* oidx = nullptr;  // out[oidx[k]] (nullptr: out[k])
  unsigned long long* pair_counter = nullptr;
  int32_t lds_max_len = 0;
};

// Profile string kernel, fast path (dyadic profiles without empty columns,
// both examples weighted or neither; profile_string.hip): per-position
// operands x role v_l = (sum_k st[k][l] x_k) / xs * w, y role v_l = y_l / ys
// * w, so a cell's weighted subst_score is sum_l vx_l vy_l.
struct StrPos {
  double v[4];
};
// one-hot columns (single sequences): the residue code and the weight
struct StrCode {
  float w;
  int32_t code;
};
struct StrFastLaunch {
  DevSet xset, yset;
  const StrPos* xtab = nullptr;  // by x-set position (onehot: StrCode)
  const StrPos* ytab = nullptr;  // by y-set position (onehot: StrCode)
  const double* st = nullptr;    // 16: the substitution table (onehot)
  int32_t onehot = 0;
  const double* gpow = nullptr;  // gap^k (the reference's repeated products), k <= max_len
  double gap = 0.0;
  const int32_t* xs = nullptr;   // pair k: x = xs[k], y = ys[k] -> out[oidx ? oidx[k] : k]
  const int32_t* ys = nullptr;
  const int64_t* oidx = nullptr;
  int64_t n_pairs = 0;
  double* out = nullptr;
  unsigned long long* pair_counter = nullptr;
  int32_t lds_max_len = 0;  // >= 64
};
__host__ __device__ inline size_t str_fast_wave_lds_bytes(int maxlen, bool onehot) {
  return ((size_t)maxlen * (onehot ? sizeof(StrCode) : sizeof(StrPos)) + (size_t)2 * (maxlen + 2) * 8 + 15) &
         ~(size_t)15;
}
constexpr size_t kStrFastLds0 = 16 * 8;  // the substitution table
hipError_t launch_str_tab(const float4* prof, const float* pos_w, int64_t n, const double* st, StrPos* xrole,
                          StrPos* yrole, hipStream_t stream);
hipError_t launch_str_code_tab(const float4* prof, const float* pos_w, int64_t n, StrCode* tab,
                               hipStream_t stream);
hipError_t launch_str_fast(const StrFastLaunch& P, int grid, int nwaves, hipStream_t stream);

// Per-position BPLA score operands, computed per call by sk_bpla_tab_kernel
// (dyadic profile columns only, see bpla.hip): x role v = u_l / xs with
// u_l = sum_k table[k][l] x_k, y role v = y_l / ys, so LAScore = sum_l
// v_x[l] v_y[l]; pr, pl, pu: sqrt p_right, p_left, p_unpair.
struct alignas(16) BplaPos {  // 16-B aligned: three ds_read_b128 with immediate offsets
  double v[4];
  float pr, pl, pu, dyadic;
};
static_assert(sizeof(BplaPos) == 48, "BplaPos is three 16-B loads");

struct BplaLaunch {
  DevSet xset, yset;
  const BplaPos* xtab = nullptr;  // fast kernel: x-role operands by x position
  const BplaPos* ytab = nullptr;  // fast kernel: y-role operands by y position
  const int64_t* oidx = nullptr;  // out[oidx[k]] = K(pair k) (nullptr: out[k])
  // fast kernel, grouped by y: items {first pair, count} of pairs sharing y
  const int2* items = nullptr;
  int32_t n_items = 0;
  const double* table = nullptr;  // 16: score table (x residue major)
  double alpha = 0.0, beta = 0.0, gap = 0.0, ext = 0.0;
  double beta_gap = 0.0, beta_ext = 0.0;  // exp(beta*gap), exp(beta*ext)
  int32_t sw = 0;  // local_alignment_max instead of local_alignment_exp
  int32_t bp = 0;  // BPLAScore (base-pairing terms) instead of LAScore
  const int32_t* xs = nullptr;
  const int32_t* ys = nullptr;
  int64_t n_pairs = 0;
  double* out = nullptr;
  unsigned long long* pair_counter = nullptr;
  int32_t lds_max_len = 0;  // even, >= 64 (streamed strips)
  int32_t chunk = 1;        // grouped fast kernel: pairs a wave streams back to back (<= kBplaChunkMax)
};

// BPLA gradients (bpla_kernel.cpp:178-401): one thread per pair, forward and
// backward tables interleaved in scratch (n_pairs * bpla_grad_pair_bytes)
struct BplaGradLaunch {
  DevSet xset, yset;
  const double* table = nullptr;  // 16, x residue major
  double alpha = 0.0, beta = 0.0, gap = 0.0, ext = 0.0;
  double beta_gap = 0.0, beta_ext = 0.0;
  const int32_t* xs = nullptr;
  const int32_t* ys = nullptr;
  int64_t n_pairs = 0;
  int32_t n1 = 1, m1 = 1;  // max |x|+1, |y|+1 of the launch
  double* scratch = nullptr;
  double* value = nullptr;  // n_pairs
  double* grad = nullptr;   // 4 * n_pairs: d/d(alpha, beta, gap, ext)
  // wave-per-pair kernel (dyadic profiles, bpla_grad.hip): operand tables of
  // sk_bpla_tab_kernel, pairs pulled by waves, result of pair k at oidx[k]
  const BplaPos* xtab = nullptr;
  const BplaPos* ytab = nullptr;
  unsigned long long* pair_counter = nullptr;
  const int64_t* oidx = nullptr;
  int32_t lds_max_len = 0;  // even, >= 64
  int64_t bt_doubles = 0;   // per-wave backward table: 3 states x steps x 64 lanes
};
size_t bpla_grad_pair_bytes(int n1, int m1);
hipError_t launch_bpla_grad(const BplaGradLaunch& P, hipStream_t st);
// steps of the streamed-strip systolic schedule of one (|x|, |y|) pair
__host__ __device__ inline int bpla_steps(int lx, int ly) {
  const int lys = ly > 64 ? ly : 64;
  return lx <= 0 || ly <= 0 ? 0 : ((lx + 63) / 64 - 1) * lys + ((lx - 1) & 63) + ly;
}
// per-wave LDS of the wave gradient kernel: y columns | boundary row
__host__ __device__ inline size_t bpla_grad_wave_lds_bytes(int maxlen) {
  const size_t b = (size_t)maxlen * sizeof(BplaPos) + (size_t)3 * (maxlen + 2) * 8;
  return (b + 15) & ~(size_t)15;
}
hipError_t launch_bpla_grad_wave(const BplaGradLaunch& P, int grid, int nwaves, hipStream_t st);

// per-wave LDS of the BPLA kernel: 4 boundary rows + y columns (16-B aligned)
__host__ __device__ inline size_t bpla_wave_lds_bytes(int maxlen) {
  const size_t b = (size_t)4 * (maxlen + 2) * 8 + (size_t)maxlen * 32;
  return (b + 15) & ~(size_t)15;
}

// 4-D stem kernel (stem4d.hip): one pair of a batch
struct Stem4dPair {
  int32_t n = 0, m = 0;          // |x|, |y|
  int64_t plane_doubles = 0;     // per state, padded rows
  int64_t scratch_off = 0;       // ring of 3 spans x (n+1) planes x 4 states (2 + acc: gsum)
  int64_t x_bp = 0, y_bp = 0;    // into bpdiag
  int64_t x_chr = 0, y_chr = 0;  // into chars
  int64_t out_index = 0;
  int64_t band_off = 0;          // into band_lo/band_hi (n+1 entries)
};

struct Stem4dLaunch {
  const Stem4dPair* pairs = nullptr;
  const int2* items = nullptr;  // {pair slot, i} of this launch's span d1
  int64_t n_items = 0;
  int32_t d1 = 0;
  double* scratch = nullptr;
  const float* bpdiag = nullptr;  // per x example: prob(a, a+e) by diagonal e
  const uint8_t* chars = nullptr;  // lowercased x sequences
  const float* bpdiag_y = nullptr;  // the same of the y examples (their
  const uint8_t* chars_y = nullptr;  // dataset's resident tables)
  const double* gpow = nullptr;   // gap^k
  double gap = 0.0, stack = 0.0, subst = 0.0;
  float bp_bound = 0.0f;
  double* out = nullptr;
  const int32_t* band_lo = nullptr;  // partial_dp band (nullptr: full_dp)
  const int32_t* band_hi = nullptr;
  // |y| >= 512: per work item 2 x 2 boundary columns of kbound_stride / 4
  // doubles each (stem4d.hip k tiles)
  double* kbound = nullptr;
  int64_t kbound_stride = 0;
  // full_dp with the K chain summed (stem4d.hip sk_stem4d_gsum_kernel): planes
  // of two states (G0, G1) and a per-pair accumulator of n+1 doubles after
  // the ring; 0 = the four-state planes; 2 = the same planes with each plane's
  // G1 pre-combined by the plane (i+1, j) (sk_stem4d_pre_kernel, one k tile)
  int32_t gsum = 0;
  // column kernel: steps between full (global-memory) barriers (stem4d.hip)
  int32_t col_f = 1;
};

int stem4d_cpl(int m);
hipError_t launch_stem4d(const Stem4dLaunch& P, int cpl, hipStream_t st);
// full_dp, column groups (stem4d.hip sk_stem4d_col_kernel): one workgroup of
// `waves` waves per pair (pairs[0..n_pairs)); per pair n planes of
// plane_doubles (G0) and stem4d_col_nb(cpl) B' planes (the round wrap) at
// scratch_off; |y| < 512, |x| <= stem4d_col_max_n(), and waves <=
// stem4d_col_w_max(m) for every pair with m >= 2 (pairs with m <= 1 have K = 1
// and take any waves); the LDS holds the batch's longest y and x
int stem4d_col_w_max(int m);
int stem4d_col_max_n();
int stem4d_col_pf();  // rows fetched ahead per wave (SK4C_PF)
int stem4d_col_nb(int cpl);
size_t stem4d_col_lds_bytes(int cpl, int waves, int max_m, int max_n);
int stem4d_col_max_waves(int cpl);
hipError_t launch_stem4d_col(const Stem4dLaunch& P, int64_t n_pairs, int cpl, int waves, int max_m,
                             int max_n, hipStream_t st);

// PairHMM alignment constraints of a 4-D batch (-a, stem_kernel.cpp:14-81):
// one wavefront per pair writes c_low/c_high (n+1 each at pair.band_off).
struct PhmmLaunch {
  const Stem4dPair* pairs = nullptr;
  int64_t n_pairs = 0;
  const uint8_t* chars = nullptr;  // x sequences, ACGU only (checked on the host)
  const uint8_t* chars_y = nullptr;  // y sequences
  char* scratch = nullptr;         // n_pairs * pair_bytes
  size_t pair_bytes = 0;           // phmm_pair_bytes(n1, m1)
  int32_t n1 = 1, m1 = 1;          // max |x|+1, max |y|+1 of the launch
  float ali_bound = 0.0f;
  uint32_t band = 0;
  int32_t zerop_fixed = 0;
  int32_t* band_lo = nullptr;
  int32_t* band_hi = nullptr;
};
size_t phmm_pair_bytes(int n1, int m1);
hipError_t launch_phmm(const PhmmLaunch& P, hipStream_t st);

// McCaskill fold (fold.hip): one workgroup per sequence
struct FoldSeq {
  int64_t seq_off = 0;   // into codes
  int64_t work_off = 0;  // into work: 10 n^2 + 2 (n + 1) doubles
  int64_t out_off = 0;   // into out: n (n - 1) / 2 packed probabilities
  int64_t lp_off = 0;    // into lp (--noLonelyPairs): n x n pair filter
  int32_t n = 0, pad = 0;
};
struct FoldLaunch {
  const FoldSeq* seqs = nullptr;
  const int8_t* codes = nullptr;  // A C G U = 0..3, anything else -1
  const double* tab = nullptr;    // Boltzmann factors, offsets below (host: fold_tables)
  int32_t o_st = 0, o_hp = 0, o_bu = 0, o_in = 0, o_ni = 0, o_au = 0, o_ml = 0, o_scp = 0;
  double log_sc = 0.0;            // ln of the per-nucleotide scale
  int32_t no_gu = 0, no_closing_gu = 0;
  const uint8_t* lp = nullptr;    // --noLonelyPairs pair filter (nullptr: off)
  int32_t n_tab = 0, n_tab_pad = 0;  // table length (doubles), rounded up to 2 (LDS copy)
  int32_t n_small = 0;              // the fixed-size head of the tables (o_st .. o_ml)
  int32_t ring_n = 0;               // set by launch_fold: ring row length (0: no ring)
  double* work = nullptr;           // per sequence 6 n^2 + 2 (n + 1) doubles (fold_work_doubles)
  double* out = nullptr;
  double* log_z = nullptr;        // per sequence of the launch (nullptr: not wanted)
};
// the fold kernel keeps the interior-loop window of the inside / outside
// tables in LDS for sequences up to this length (33 n doubles)
constexpr int kFoldRingMaxN = 248;
// dynamic LDS a fold launch may take (160 KB less the kernel's static block sums)
constexpr size_t kFoldLdsMax = 163840 - 256;
bool fold_ring(int max_n);
// whether a launch keeps the hairpin / scale tables in HBM (they and the ring
// and codes would not fit the LDS)
bool fold_gtab(const FoldLaunch& P, int max_n);
size_t fold_lds_bytes(const FoldLaunch& P, int max_n);
inline size_t fold_work_doubles(size_t n) { return 6 * n * n + 2 * (n + 1); }
hipError_t launch_fold(const FoldLaunch& P, int n_seqs, int max_n, hipStream_t st);

enum CombineMode : int32_t {
  kCombineStem = 0,      // K = stem
  kCombineStr = 1,       // K = str
  kCombineAdd = 2,       // K = stem + str                 (AddKernel)
  kCombineLogStem = 3,   // K = beta*log(stem) + 0         (LTKernel(LogKernel))
  kCombineLogAdd = 4     // K = (beta*log stem + 0) + (alpha*log str + 0)
};

hipError_t launch_prep(const DevSet& s, const DevParamNodes& pn, const double* gpow, double gap2,
                       hipStream_t st);
size_t stem_lds_bytes(const StemLaunch& P, int nwaves);
hipError_t launch_stem(const StemLaunch& P, int grid, int nwaves, hipStream_t st);
hipError_t stem_kernel_attr(int max_nl, int* max_dyn_lds, int* vgprs, int* max_waves);
int stem_maxk(int max_nl);

size_t str_lds_bytes(const StrLaunch& P, int nwaves);
hipError_t launch_str(const StrLaunch& P, int grid, int nwaves, hipStream_t st);

// fast kernels: a workgroup's LDS starts with the exp table 2^(j/1024), j < 1024
constexpr size_t kBplaExpLds = 1024 * 8;
// a wave's chunk of pairs streamed back to back: per pair {xtab base,
// length, first row, -} and its K sum
constexpr int kBplaChunkMax = 16;
// y-grouped fast kernel: at most 12 waves per workgroup, 3 per SIMD (the
// two-row exp path holds two rows' operands and state: up to 168 VGPRs)
#ifndef SK_BPLA_ITEMS_WAVES
#define SK_BPLA_ITEMS_WAVES 12
#endif
constexpr int kBplaItemsWavesMax = SK_BPLA_ITEMS_WAVES;
constexpr size_t kBplaChunkLds = kBplaChunkMax * (16 + 8);
// grouped fast kernel: exp table | shared y columns | per wave boundary row
// and chunk
__host__ __device__ inline size_t bpla_items_lds_bytes(int maxlen, int nwaves) {
  return kBplaExpLds + 16 + (size_t)maxlen * sizeof(BplaPos) +
         (size_t)nwaves * (3 * (maxlen + 2) * 8 + kBplaChunkLds);
}
size_t bpla_lds_bytes(const BplaLaunch& P, int nwaves);
hipError_t launch_bpla(const BplaLaunch& P, int grid, int nwaves, hipStream_t st);
// dyadic-profile fast path: per-call operand tables, then the DP
// xscale multiplies the x-role factors v[l] (beta for the exp path, whose
// exponent is then formed without a multiply; 1 elsewhere)
hipError_t launch_bpla_tab(const float4* prof, const float4* lru, int64_t n, const double* table,
                           double xscale, BplaPos* xrole, BplaPos* yrole, hipStream_t st);
// per-wave LDS of the fast kernel: y columns (BplaPos, maxlen) | boundary
// row {M, X, Y} [maxlen + 2] | chunk
__host__ __device__ inline size_t bpla_fast_wave_lds_bytes(int maxlen) {
  const size_t b = (size_t)maxlen * sizeof(BplaPos) + (size_t)3 * (maxlen + 2) * 8 + kBplaChunkLds;
  return (b + 15) & ~(size_t)15;
}
hipError_t launch_bpla_fast(const BplaLaunch& P, int grid, int nwaves, hipStream_t st);

hipError_t launch_combine(const double* stem, const double* str, double* out, int64_t n,
                          int32_t mode, double alpha, double beta, hipStream_t st);

}  // namespace sk
