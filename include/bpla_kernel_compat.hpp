// bpla_kernel_compat.hpp -- drop-in for the BPLA kernel tool (bpla_kernel/):
// replacing
//     #include "data.h"            // bpla's Data<S,IS>, MData, loaders
//     #include "bpla_kernel.h"     // BPLAKernel
// and common/framework.h's  #include "../common/kernel_matrix.h"
// by
//     #include "bpla_kernel_compat.hpp"
// is the only edit; main's code (bpla_kernel/main.cpp:100-127: the score
// table, `LDF ldf;` / `LDF ldf(bp_opts);`, BPLAKernel<double,MData>,
// App<BPLAKernel<double,MData>, LDF>) compiles unchanged and every cell runs
// on the GPU (csrc/kernels/bpla.hip).
//
//   Data<S, IS> / MData = Data<ProfileSequence, list<string>>
//     Data(ma, pf_scale, opts), Data(ma), size()    bpla_kernel/data.h:22-48,
//                                                    data.cpp:19-63
//   DataLoader<MData>(filename, bp_opts, use_bp) / (filename, pf_scales, ...)
//     get()                                          data.h:84-104, data.cpp:181-230
//   DataLoaderFactory<LD>() / (bp_opts)              data.h:136-160
//   BPLAKernel<V, D>(score_table, noBP, SW, gap, ext, alpha, beta)
//     operator()(x, y)                               bpla_kernel.h:13-45
//     static compute_gradients(x, y, score_table, param, d)
//                                                    bpla_kernel.cpp:385-401
//   BPMatrix::Options                                common/bpmatrix.h:17-38
//   KernelMatrix<V>                                  common/kernel_matrix.h:13-108
//
// Folding is the engine's McCaskill (notice on stderr; parity against
// ViennaRNA unpinned) unless BPMatrix::Options::fold supplies the bpp.
// `LDF ldf;` (--noBP) builds examples without base pairs: the engine then
// weights every position unpaired (p_left = p_right = 0, p_unpair = 1),
// which the LAScore path never reads.
#ifndef BPLA_KERNEL_COMPAT_HPP
#define BPLA_KERNEL_COMPAT_HPP

#include "skc/core.hpp"

namespace skc {
namespace bpla {

struct BPMatrix {
  typedef BPMatrixOptions Options;
};

struct ProfileSequence {};  // the profile is built by the engine (common/profile.cpp)

// Data<S, IS> (bpla_kernel/data.h:22-48): rows and per-row folded matrices;
// the engine derives the profile and sqrt(p_left / p_right / p_unpair)
// (fill_weight, data.cpp:19-45) when a KernelMatrix needs them.
template <class S, class IS>
struct Data : RowsData {
  typedef S Seq;
  Data() {}
  Data(const IS& ma, float /*pf_scale*/, const BPMatrix::Options& opts) {
    rows.assign(ma.begin(), ma.end());
    use_bp = true;
    fold_rows(*this, opts);
  }
  explicit Data(const IS& ma) { rows.assign(ma.begin(), ma.end()); }
  uint size() const { return rows.empty() ? 0u : (uint)rows.front().size(); }
};

typedef Data<ProfileSequence, std::list<std::string>> MData;

template <class D>
class DataLoader;

template <>
class DataLoader<MData> {
 public:
  typedef MData Data;
  DataLoader(const char* filename, const BPMatrix::Options& bp_opts, bool use_bp)
      : file_(filename), opts_(bp_opts), use_bp_(use_bp) {}
  DataLoader(const char* filename, const char* /*pf_scales*/, const BPMatrix::Options& bp_opts, bool use_bp)
      : file_(filename), opts_(bp_opts), use_bp_(use_bp) {}
  Data* get() {
    std::list<std::string> ma;
    if (!file_.next(ma)) return nullptr;
    return use_bp_ ? new MData(ma, -1.0f, opts_) : new MData(ma);
  }

 private:
  SeqFile file_;
  BPMatrix::Options opts_;
  bool use_bp_;
};

template <class LD>
class DataLoaderFactory {
 public:
  typedef LD Loader;
  typedef typename Loader::Data Data;
  explicit DataLoaderFactory(const BPMatrix::Options& bp_opts) : bp_opts_(bp_opts), use_bp_(true) {}
  DataLoaderFactory() : use_bp_(false) {}
  Loader* get_loader(const char* filename) const { return new Loader(filename, bp_opts_, use_bp_); }
  Loader* get_loader(const char* filename, const char* pf_scales) const {
    return new Loader(filename, pf_scales, bp_opts_, use_bp_);
  }

 private:
  BPMatrix::Options bp_opts_;
  bool use_bp_;
};

template <class ValueType, class DataT>
class BPLAKernel : public KernelBase<ValueType, DataT> {
 public:
  typedef ValueType value_type;
  typedef DataT Data;

  // score_table: any [4][4]-indexable table (the reference passes
  // boost::multi_array<value_type,2>)
  template <class Table>
  BPLAKernel(const Table& score_table, bool noBP, bool SW = false, value_type gap = 1, value_type ext = 1,
             value_type alpha = 1, value_type beta = 1)
      : KernelBase<ValueType, DataT>(noBP ? (SW ? SK_LA_SW : SK_LA) : (SW ? SK_BPLA_SW : SK_BPLA)) {
    for (int a = 0; a < 4; ++a)
      for (int b = 0; b < 4; ++b) this->p_.score_table[4 * a + b] = score_table[a][b];
    this->p_.gap = gap;
    this->p_.ext = ext;
    this->p_.alpha = alpha;
    this->p_.beta = beta;
  }

  // the bpla_optimizer's per-pair step: value, d = d/d(alpha, beta, gap,
  // ext) for param = {alpha, beta, gap, ext} (sk_bpla_gradients)
  template <class Table>
  static value_type compute_gradients(const Data& x, const Data& y, const Table& score_table,
                                      const std::vector<double>& param, std::vector<double>& d) {
    sk_kernel_params p;
    sk_kernel_params_default(&p, SK_BPLA);
    for (int a = 0; a < 4; ++a)
      for (int b = 0; b < 4; ++b) p.score_table[4 * a + b] = score_table[a][b];
    p.alpha = param.at(0);
    p.beta = param.at(1);
    p.gap = param.at(2);
    p.ext = param.at(3);
    std::vector<std::pair<std::string, Data>> ex{{"+1", x}, {"+1", y}};
    Engine& E = Engine::get();
    const Engine::DsPtr hold = E.dataset(ex, BuildSpec());
    sk_dataset* ds = hold.get();
    const int32_t a = 0, b = 1;
    double v = 0.0, g[4];
    check(sk_bpla_gradients(E.ctx(), ds, ds, &p, &a, &b, 1, &v, g), E.ctx());
    d.assign(g, g + 4);
    return (value_type)v;
  }
};

}  // namespace bpla

template <class S, class IS>
struct ExampleTraits<bpla::Data<S, IS>> {
  static void add(sk_dataset* ds, const std::string& label, const bpla::Data<S, IS>& d, const BuildSpec&) {
    add_rows(ds, label, d, 1.0f);  // th = 1: no DAG (BPLA reads profiles and weights only)
  }
  static void mix(Fnv& f, const bpla::Data<S, IS>& d) { mix_rows(f, d); }
};

}  // namespace skc

#ifndef SKC_NO_REFERENCE_NAMES
using skc::KernelMatrix;
using skc::bpla::BPLAKernel;
using skc::bpla::BPMatrix;
using skc::bpla::Data;
using skc::bpla::DataLoader;
using skc::bpla::DataLoaderFactory;
using skc::bpla::MData;
using skc::bpla::ProfileSequence;
typedef unsigned int uint;
#endif

#endif  // BPLA_KERNEL_COMPAT_HPP
