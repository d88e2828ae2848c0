// stem_kernel_compat.hpp -- the stem_kernel_lite tool's own host types over
// the MI355X engine, so that App<K,LDF> (common/framework.h:100-306) and its
// callers compile unchanged: replacing
//     #include "../common/kernel_matrix.h"   // KernelMatrix<V>
//     #include "def_kernel.h" / "data.h"       // kernels, MData, loaders
// by
//     #include "stem_kernel_compat.hpp"
// is the only edit.  The names below are the reference's, with the
// reference's template parameters, constructor arguments and member
// signatures:
//
//   KernelMatrix<V>            common/kernel_matrix.h:13-108
//     calculate(train, kernel, normalize, n_th)                 :67-70
//     calculate(test, train, kernel, norm_test, normalize, n_th) :72-75
//     calculate(vec, data, train, [sv_index,] kernel, n_th, self) :77-93
//     diagonal(diag, train, [sv_index,] kernel, n_th)          :95-106
//     operator()(x, y), operator()(x), self(), resize(), print(ostream)
//   SuStemKernel / SiStemKernel / SuStemStrKernel / SiStemStrKernel /
//   LSuStemKernel / LSuStemStrKernel <V, D>     stem_kernel_lite/def_kernel.h
//   StringKernel<V, D>                          stem_kernel_lite/string_kernel.h:16-17
//   BPLAKernel<V, D>                            bpla_kernel/bpla_kernel.h:21-26
//   MData, DataLoader<MData>, DataLoaderFactory<LD>   stem_kernel_lite/data.h:26-133
//   BPMatrix::Options                           common/bpmatrix.h:17-38
//
// The other tools have their own headers (their names clash with these:
// string_kernel.h and bpla_kernel.h even share one include guard):
//   stem_kernel/   (4-D, pair<string,string>)  stem_kernel_ref_compat.hpp
//   string_kernel/ (naive, pair<string,string>) string_kernel_compat.hpp
//   bpla_kernel/   (bpla's MData)               bpla_kernel_compat.hpp
//
// Every Gram cell is computed by the HIP engine through the C ABI
// (stem_kernel.h); there is no CPU fallback.  The engine is one process-wide
// context on device $SK_DEVICE (default 0).  Under MPI the caller gives each
// rank its GPU and the RCCL id once -- skc::Engine::init_rank(...), before
// any load or fold -- and KernelMatrix::calculate then runs the reference MPI
// Gram's cyclic plan over RCCL (sk_gram_sharded), every rank receiving the
// whole matrix.
//
// What differs, by necessity:
//   - base-pairing probabilities: ViennaRNA's pf_fold is replaced by the
//     engine's GPU McCaskill (sk_fold_mccaskill, SURVEY.md §8 f1: the
//     Turner-1999 core loop model, parity against ViennaRNA unpinned; a
//     one-line notice goes to stderr the first time it folds); MData folds
//     each gap-erased, lowercased row with it (honouring --noGU and
//     --noClosingGU, --noLonelyPairs; --use-alifold is refused) and
//     averages alignment rows as the reference does
//     (common/bpmatrix.cpp:306-342).  BPMatrix::Options::fold plugs in any
//     other folder (e.g. ViennaRNA itself, or skc::synthetic_fold);
//   - elapsed times are wall-clock seconds (the reference sums boost::timer
//     CPU seconds);
//   - errors are thrown as const char* like the reference, carrying the
//     engine's message.
#ifndef STEM_KERNEL_COMPAT_HPP
#define STEM_KERNEL_COMPAT_HPP

#include "skc/core.hpp"

namespace skc {

struct BPMatrix {
  typedef BPMatrixOptions Options;  // common/bpmatrix.h:17-38 (+ the fold hook)
};

// The reference's MData (stem_kernel_lite/data.h:26-55) as the engine
// consumes it: the alignment rows and each row's folded matrix; the DAG is
// built by the engine (sk_dataset_add) when a KernelMatrix needs it.
struct MData : RowsData {
  MData() {}
  // MData(ma, th, pf_scale, opts)  stem_kernel_lite/data.cpp:324-345
  MData(const std::list<std::string>& ma, float th_, float /*pf_scale*/, const BPMatrix::Options& opts) {
    rows.assign(ma.begin(), ma.end());
    th = th_;
    use_bp = true;
    fold_rows(*this, opts);
  }
  // MData(ma): no base-pairing information (string kernels only)
  explicit MData(const std::list<std::string>& ma) { rows.assign(ma.begin(), ma.end()); }
};

template <>
struct ExampleTraits<MData> {
  static void add(sk_dataset* ds, const std::string& label, const MData& d, const BuildSpec&) {
    add_rows(ds, label, d, d.th);
  }
  static void mix(Fnv& f, const MData& d) { mix_rows(f, d); }
};

// DataLoader<MData> (stem_kernel_lite/data.h:79-102, data.cpp:482-586)
template <class D>
class DataLoader;

template <>
class DataLoader<MData> {
 public:
  typedef MData Data;

  DataLoader(const char* filename, float th, const BPMatrix::Options& bp_opts, bool use_bp)
      : file_(filename), th_(th), opts_(bp_opts), use_bp_(use_bp) {}
  DataLoader(const char* filename, float th, const char* /*pf_scales*/,
             const BPMatrix::Options& bp_opts, bool use_bp)
      : file_(filename), th_(th), opts_(bp_opts), use_bp_(use_bp) {}

  // next example, or NULL at the end (caller deletes)
  Data* get() {
    std::list<std::string> ma;
    if (!file_.next(ma)) return nullptr;
    return use_bp_ ? new MData(ma, th_, -1.0f, opts_) : new MData(ma);
  }

 private:
  SeqFile file_;
  float th_;
  BPMatrix::Options opts_;
  bool use_bp_;
};

// DataLoaderFactory<LD>  stem_kernel_lite/data.h:104-133
template <class LD>
class DataLoaderFactory {
 public:
  typedef LD Loader;
  typedef typename Loader::Data Data;

  DataLoaderFactory(float th, const BPMatrix::Options& bp_opts)
      : th_(th), bp_opts_(bp_opts), use_bp_(true) {}
  DataLoaderFactory() : th_(0.0f), use_bp_(false) {}
  Loader* get_loader(const char* filename) const {
    return new Loader(filename, th_, bp_opts_, use_bp_);
  }
  Loader* get_loader(const char* filename, const char* pf_scales) const {
    return new Loader(filename, th_, pf_scales, bp_opts_, use_bp_);
  }

 private:
  float th_;
  BPMatrix::Options bp_opts_;
  bool use_bp_;
};

// ------------------------------------------------------------------ kernels
template <class V, class D>
class SuStemKernel : public KernelBase<V, D> {  // def_kernel.h:35-59
 public:
  SuStemKernel(V loop_gap, V beta, uint len_band) : KernelBase<V, D>(SK_SU_STEM) {
    this->p_.loop_gap = loop_gap;
    this->p_.beta = beta;
    this->p_.len_band = len_band;
  }
};

template <class V, class D>
class SiStemKernel : public KernelBase<V, D> {  // def_kernel.h:10-33
 public:
  SiStemKernel(V loop_gap, V stack, V covar, uint len_band) : KernelBase<V, D>(SK_SI_STEM) {
    this->p_.loop_gap = loop_gap;
    this->p_.stack = stack;
    this->p_.covar = covar;
    this->p_.len_band = len_band;
  }
};

template <class V, class D>
class StringKernel : public KernelBase<V, D> {  // string_kernel.h:16-17
 public:
  StringKernel(V gap, V alpha) : KernelBase<V, D>(SK_SU_STR) {
    this->p_.gap = gap;
    this->p_.alpha = alpha;
  }
  StringKernel(V gap, V match, V mismatch) : KernelBase<V, D>(SK_SI_STR) {
    this->p_.gap = gap;
    this->p_.match = match;
    this->p_.mismatch = mismatch;
  }
};

template <class V, class D>
class SuStemStrKernel : public KernelBase<V, D> {  // def_kernel.h:86-111
 public:
  SuStemStrKernel(V alpha, V beta, V loop_gap, V gap, uint len_band)
      : KernelBase<V, D>(SK_SU_STEM_STR) {
    this->p_.alpha = alpha;
    this->p_.beta = beta;
    this->p_.loop_gap = loop_gap;
    this->p_.gap = gap;
    this->p_.len_band = len_band;
  }
};

template <class V, class D>
class SiStemStrKernel : public KernelBase<V, D> {  // def_kernel.h:61-84
 public:
  SiStemStrKernel(V loop_gap, V stack, V covar, V gap, V match, V mismatch, uint len_band)
      : KernelBase<V, D>(SK_SI_STEM_STR) {
    this->p_.loop_gap = loop_gap;
    this->p_.stack = stack;
    this->p_.covar = covar;
    this->p_.gap = gap;
    this->p_.match = match;
    this->p_.mismatch = mismatch;
    this->p_.len_band = len_band;
  }
};

template <class V, class D>
class LSuStemKernel : public KernelBase<V, D> {  // def_kernel.h:113-138
 public:
  LSuStemKernel(V loop_gap, V beta, uint len_band) : KernelBase<V, D>(SK_LSU_STEM) {
    this->p_.loop_gap = loop_gap;
    this->p_.beta = beta;
    this->p_.len_band = len_band;
  }
};

template <class V, class D>
class LSuStemStrKernel : public KernelBase<V, D> {  // def_kernel.h:165-190
 public:
  LSuStemStrKernel(V alpha, V beta, V loop_gap, V gap, uint len_band)
      : KernelBase<V, D>(SK_LSU_STEM_STR) {
    this->p_.alpha = alpha;
    this->p_.beta = beta;
    this->p_.loop_gap = loop_gap;
    this->p_.gap = gap;
    this->p_.len_band = len_band;
  }
};

// BPLAKernel(score_table, noBP, SW, gap, ext, alpha, beta)
// bpla_kernel/bpla_kernel.h:21-26; score_table is any 4x4 [x][y] indexable
// (the reference passes boost::multi_array<value_type,2>).
template <class V, class D>
class BPLAKernel : public KernelBase<V, D> {
 public:
  template <class Table>
  BPLAKernel(const Table& score_table, bool noBP, bool SW = false, V gap = 1, V ext = 1,
             V alpha = 1, V beta = 1)
      : KernelBase<V, D>(noBP ? (SW ? SK_LA_SW : SK_LA) : (SW ? SK_BPLA_SW : SK_BPLA)) {
    for (int a = 0; a < 4; ++a)
      for (int b = 0; b < 4; ++b) this->p_.score_table[4 * a + b] = score_table[a][b];
    this->p_.gap = gap;
    this->p_.ext = ext;
    this->p_.alpha = alpha;
    this->p_.beta = beta;
  }
};

}  // namespace skc

// the reference's unqualified names (common/kernel_matrix.h,
// stem_kernel_lite/def_kernel.h, data.h, common/bpmatrix.h)
#ifndef SKC_NO_REFERENCE_NAMES
using skc::BPLAKernel;
using skc::BPMatrix;
using skc::DataLoader;
using skc::DataLoaderFactory;
using skc::KernelMatrix;
using skc::LSuStemKernel;
using skc::LSuStemStrKernel;
using skc::MData;
using skc::SiStemKernel;
using skc::SiStemStrKernel;
using skc::StringKernel;
using skc::SuStemKernel;
using skc::SuStemStrKernel;
typedef unsigned int uint;
#endif

#endif  // STEM_KERNEL_COMPAT_HPP
