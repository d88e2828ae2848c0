// stem_kernel_compat.hpp -- the reference's own host types over the MI355X
// engine, so that App<K,LDF> (common/framework.h:100-306) and its callers
// compile unchanged: replacing
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
// Every Gram cell is computed by the HIP engine through the C ABI
// (stem_kernel.h); there is no CPU fallback.  The engine is one process-wide
// context on device $SK_DEVICE (default 0).  Under MPI the caller gives each
// rank its GPU and the RCCL id once -- skc::Engine::init_rank(...) -- and
// KernelMatrix::calculate then runs the reference MPI Gram's cyclic plan
// over RCCL (sk_gram_sharded), every rank receiving the whole matrix.
//
// What differs, by necessity:
//   - base-pairing probabilities: ViennaRNA's pf_fold is replaced by the
//     engine's GPU McCaskill (sk_fold_mccaskill, SURVEY.md §8 f1: the
//     Turner-1999 core loop model, parity against ViennaRNA unpinned); MData
//     folds each gap-erased, lowercased row with it (honouring --noGU and
//     --noClosingGU; --noLonelyPairs and --use-alifold are refused) and
//     averages alignment rows as the reference does
//     (common/bpmatrix.cpp:306-342).  BPMatrix::Options::fold plugs in any
//     other folder (skc::synthetic_fold: the Nussinov-Boltzmann stand-in);
//   - elapsed times are wall-clock seconds (the reference sums boost::timer
//     CPU seconds);
//   - errors are thrown as const char* like the reference, carrying the
//     engine's message.
#ifndef STEM_KERNEL_COMPAT_HPP
#define STEM_KERNEL_COMPAT_HPP

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <ostream>
#include <string>
#include <utility>
#include <vector>

#include "stem_kernel.h"

namespace skc {

typedef unsigned int uint;

inline void check(int st, const sk_context* ctx = nullptr) {
  if (st != SK_OK) throw ctx ? sk_last_error(ctx) : sk_strerror(st);
}

// ------------------------------------------------------------------ inputs
// gap-erased, lowercased row -> packed strict upper triangle p(i,j)
// (stem_kernel.h sk_dataset_add layout)
typedef std::function<void(const std::string&, bool /*no_GU*/, std::vector<double>&)> FoldFn;

inline void synthetic_fold(const std::string& s, bool no_gu, std::vector<double>& out) {
  const int32_t n = (int32_t)s.size();
  out.assign(std::max<size_t>((size_t)n * (n > 0 ? n - 1 : 0) / 2, 1), 0.0);
  check(sk_fold_synthetic(s.c_str(), n, no_gu ? 1 : 0, out.data()));
}

struct BPMatrix {
  // common/bpmatrix.h:17-38 (+ the fold hook)
  struct Options {
    bool alifold = false, contrafold = false, no_GU = false, no_closingGU = false,
         no_LonelyPairs = false;
    uint n_samples = 0;
    bool use_pf_scale_mfe = false;
    FoldFn fold;  // empty: the engine's GPU McCaskill (engine_fold)
  };
};

// the engine's GPU McCaskill fold of one example's rows (defined after Engine)
inline void engine_fold(const std::vector<std::string>& rows, const BPMatrix::Options& opts,
                        std::vector<std::vector<double>>& out);

// The reference's MData (stem_kernel_lite/data.h:26-55) as the engine
// consumes it: the alignment rows and each row's folded matrix; the DAG is
// built by the engine (sk_dataset_add) when a KernelMatrix needs it.
struct MData {
  std::vector<std::string> rows;
  std::vector<std::vector<double>> bpp;  // per row, gap-erased
  float th = 0.0f;
  bool use_bp = false;

  MData() {}
  // MData(ma, th, pf_scale, opts)  stem_kernel_lite/data.cpp:324-345
  MData(const std::list<std::string>& ma, float th_, float /*pf_scale*/,
        const BPMatrix::Options& opts)
      : rows(ma.begin(), ma.end()), th(th_), use_bp(true) {
    std::vector<std::string> erased;
    for (const std::string& r : rows) {
      std::string s;
      for (char c : r)
        if (c != '-') s.push_back((char)std::tolower((unsigned char)c));
      erased.push_back(s);
    }
    if (opts.fold) {
      for (const std::string& s : erased) {
        bpp.emplace_back();
        opts.fold(s, opts.no_GU, bpp.back());
      }
    } else {
      engine_fold(erased, opts, bpp);
    }
  }
  // MData(ma): no base-pairing information (string kernels only)
  explicit MData(const std::list<std::string>& ma) : rows(ma.begin(), ma.end()) {}
};

// DataLoader<MData> (stem_kernel_lite/data.h:79-102, data.cpp:482-586): the
// file type is sniffed like check_filetype (data.cpp:460-480) and read by
// the engine's FASTA / CLUSTAL / MAF readers (sk_seqfile_*).
template <class D>
class DataLoader;

template <>
class DataLoader<MData> {
 public:
  typedef MData Data;

  DataLoader(const char* filename, float th, const BPMatrix::Options& bp_opts, bool use_bp)
      : th_(th), opts_(bp_opts), use_bp_(use_bp) {
    open(filename);
  }
  DataLoader(const char* filename, float th, const char* /*pf_scales*/,
             const BPMatrix::Options& bp_opts, bool use_bp)
      : th_(th), opts_(bp_opts), use_bp_(use_bp) {
    open(filename);
  }
  ~DataLoader() {
    if (f_) sk_seqfile_free(f_);
  }
  DataLoader(const DataLoader&) = delete;
  DataLoader& operator=(const DataLoader&) = delete;

  // next example, or NULL at the end (caller deletes)
  Data* get() {
    if (!f_ || next_ >= sk_seqfile_count(f_)) return nullptr;
    std::list<std::string> ma;
    const int32_t nr = sk_seqfile_rows(f_, next_);
    for (int32_t r = 0; r < nr; ++r) ma.push_back(sk_seqfile_row(f_, next_, r));
    ++next_;
    return use_bp_ ? new MData(ma, th_, -1.0f, opts_) : new MData(ma);
  }

 private:
  void open(const char* filename) {
    int fmt = -1;
    std::ifstream in(filename);
    std::string l;
    while (fmt < 0 && std::getline(in, l)) {
      if (!l.empty() && l[0] == '>') fmt = SK_FMT_FASTA;
      else if (l.compare(0, 7, "CLUSTAL") == 0) fmt = SK_FMT_CLUSTAL;
      else if (l.compare(0, 2, "a ") == 0) fmt = SK_FMT_MAF;
    }
    if (fmt < 0 || sk_seqfile_read(filename, fmt, &f_) != SK_OK) {
      // the message outlives this (never constructed) loader
      static thread_local std::string msg;
      msg = std::string(filename) + ": no such file";
      throw msg.c_str();
    }
  }
  float th_;
  BPMatrix::Options opts_;
  bool use_bp_;
  sk_seqfile* f_ = nullptr;
  int64_t next_ = 0;
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

// ------------------------------------------------------------------ engine
// One context per process; example sets are packed and uploaded once and
// cached by content (App::predict hands the same train set to every test
// row).
class Engine {
 public:
  static Engine& get() {
    static Engine e;
    return e;
  }
  sk_context* ctx() {
    std::lock_guard<std::mutex> g(mu_);
    open_locked();
    return ctx_;
  }
  // Multi-GPU (the reference's HAVE_MPI build): this rank's GPU and the RCCL
  // id rank 0 drew with sk_comm_unique_id (broadcast by the caller, e.g.
  // MPI_Bcast of 128 bytes).
  void init_rank(int device, int rank, int world, const uint8_t* uid, size_t uid_bytes) {
    std::lock_guard<std::mutex> g(mu_);
    device_ = device;
    open_locked();
    check(sk_comm_init(ctx_, uid, uid_bytes, rank, world), ctx_);
    world_ = world;
  }
  int world() const { return world_; }

  // Packed, uploaded dataset of an ExampleSet of (label, MData).
  template <class ExampleSet>
  sk_dataset* dataset(const ExampleSet& ex) {
    std::lock_guard<std::mutex> g(mu_);
    open_locked();
    const uint64_t key = fingerprint(ex);
    auto it = cache_.find(key);
    if (it != cache_.end()) return it->second.get();
    if (cache_.size() >= 8) cache_.clear();
    std::unique_ptr<sk_dataset, int (*)(sk_dataset*)> ds(nullptr, sk_dataset_free);
    sk_dataset* raw = nullptr;
    check(sk_dataset_create(&raw));
    ds.reset(raw);
    for (const auto& e : ex) add(raw, e.first, e.second);
    check(sk_dataset_upload(ctx_, raw), ctx_);
    sk_dataset* p = ds.get();
    cache_.emplace(key, std::move(ds));
    return p;
  }

  static void add(sk_dataset* ds, const std::string& label, const MData& d) {
    std::vector<const char*> r;
    std::vector<const double*> b;
    for (const auto& s : d.rows) r.push_back(s.c_str());
    for (const auto& v : d.bpp) b.push_back(v.data());
    check(sk_dataset_add(ds, label.c_str(), (int)r.size(), r.data(),
                         d.use_bp ? b.data() : nullptr, d.th, d.use_bp ? 1 : 0));
  }

 private:
  Engine() {
    const char* e = std::getenv("SK_DEVICE");
    device_ = e ? std::atoi(e) : 0;
  }
  ~Engine() {
    cache_.clear();
    if (ctx_) sk_close(ctx_);
  }
  void open_locked() {
    if (!ctx_) check(sk_open(device_, nullptr, &ctx_));
  }
  template <class ExampleSet>
  static uint64_t fingerprint(const ExampleSet& ex) {
    uint64_t h = 1469598103934665603ull;  // FNV-1a over labels, rows and bpp
    auto mix = [&h](const void* p, size_t n) {
      const unsigned char* c = static_cast<const unsigned char*>(p);
      for (size_t i = 0; i < n; ++i) h = (h ^ c[i]) * 1099511628211ull;
    };
    for (const auto& e : ex) {
      mix(e.first.data(), e.first.size());
      for (const auto& r : e.second.rows) mix(r.data(), r.size() + 1);
      for (const auto& b : e.second.bpp) mix(b.data(), b.size() * sizeof(double));
      mix(&e.second.th, sizeof(float));
      mix(&e.second.use_bp, sizeof(bool));
    }
    return h;
  }
  std::mutex mu_;
  int device_ = 0, world_ = 1;
  sk_context* ctx_ = nullptr;
  std::map<uint64_t, std::unique_ptr<sk_dataset, int (*)(sk_dataset*)>> cache_;
};

inline void engine_fold(const std::vector<std::string>& rows, const BPMatrix::Options& opts,
                        std::vector<std::vector<double>>& out) {
  if (opts.no_LonelyPairs) throw "--noLonelyPairs is not supported by the engine's fold";
  if (opts.alifold || opts.contrafold || opts.n_samples > 0)
    throw "only the FOLD method (McCaskill per row) is supported by the engine";
  std::vector<const char*> p;
  size_t total = 0;
  for (const std::string& s : rows) {
    p.push_back(s.c_str());
    total += s.size() > 1 ? s.size() * (s.size() - 1) / 2 : 0;
  }
  std::vector<double> all(std::max<size_t>(total, 1));
  sk_context* ctx = Engine::get().ctx();
  check(sk_fold_mccaskill(ctx, (int32_t)p.size(), p.data(),
                          (opts.no_GU ? SK_FOLD_NO_GU : 0) | (opts.no_closingGU ? SK_FOLD_NO_CLOSING_GU : 0),
                          all.data(), nullptr),
        ctx);
  out.clear();
  size_t o = 0;
  for (const std::string& s : rows) {
    const size_t z = s.size() > 1 ? s.size() * (s.size() - 1) / 2 : 0;
    out.emplace_back(all.begin() + o, all.begin() + o + z);
    if (out.back().empty()) out.back().assign(1, 0.0);
    o += z;
  }
}

// ------------------------------------------------------------------ kernels
// Each kernel carries its sk_kernel_params; operator() evaluates one pair on
// the GPU (the Kernel concept, stem_kernel_lite/def_kernel.h:43-51) --
// KernelMatrix batches whole Grams instead.
template <class V, class D>
class KernelBase {
 public:
  typedef V value_type;
  typedef D Data;
  const sk_kernel_params& sk_params() const { return p_; }
  value_type operator()(const Data& x, const Data& y) const {
    std::vector<std::pair<std::string, Data>> ex{{"+1", x}, {"+1", y}};
    Engine& E = Engine::get();
    sk_dataset* ds = E.dataset(ex);
    const int32_t a = 0, b = 1;
    double v = 0.0;
    check(sk_pairs(E.ctx(), ds, &p_, &a, &b, 1, &v), E.ctx());
    return (value_type)v;
  }

 protected:
  explicit KernelBase(sk_kernel_kind k) { sk_kernel_params_default(&p_, k); }
  sk_kernel_params p_;
};

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

// ------------------------------------------------------------------ matrix
template <class ValueType>
class KernelMatrix {
 public:
  typedef ValueType value_type;

  KernelMatrix() : row_(0), col_(0) {}
  KernelMatrix(uint row, uint col)
      : row_(row), col_(col), matrix_((size_t)row * col), self_(row), label_(row) {}

  void resize(uint row, uint col) {
    row_ = row;
    col_ = col;
    matrix_.resize((size_t)row * col);
    label_.resize(row);
  }
  value_type& operator()(uint x, uint y) { return matrix_[(size_t)x * col_ + y]; }
  const value_type& operator()(uint x, uint y) const { return matrix_[(size_t)x * col_ + y]; }
  value_type& operator()(uint x) { return self_[x]; }
  const value_type& operator()(uint x) const { return self_[x]; }
  const std::vector<value_type>& self() const { return self_; }

  // train Gram: kernel_matrix.cpp:485-575 (HAVE_MPI: :186-261, 495-527)
  template <class Kernel, class ExampleSet>
  double calculate(const ExampleSet& train, const Kernel& kernel, bool normalize = false,
                   uint /*n_th*/ = 1) {
    const auto t0 = std::chrono::steady_clock::now();
    Engine& E = Engine::get();
    sk_dataset* ds = E.dataset(train);
    const uint n = (uint)train.size();
    resize(n, n);
    self_.assign(n, value_type());
    for (uint i = 0; i != n; ++i) label_[i] = train[i].first;
    std::vector<double> m((size_t)n * n);
    if (E.world() > 1)
      check(sk_gram_sharded(E.ctx(), ds, &kernel.sk_params(), normalize ? 1 : 0, m.data()),
            E.ctx());
    else
      check(sk_gram(E.ctx(), ds, &kernel.sk_params(), normalize ? 1 : 0, m.data()), E.ctx());
    matrix_.assign(m.begin(), m.end());
    return seconds_since(t0);
  }

  // test x train: kernel_matrix.cpp:699-754
  template <class Kernel, class ExampleSet>
  double calculate(const ExampleSet& test, const ExampleSet& train, const Kernel& kernel,
                   bool norm_test = false, bool normalize = false, uint /*n_th*/ = 1) {
    const auto t0 = std::chrono::steady_clock::now();
    Engine& E = Engine::get();
    sk_dataset* dtr = E.dataset(train);
    sk_dataset* dte = E.dataset(test);
    const uint nt = (uint)test.size(), ntr = (uint)train.size();
    resize(nt, ntr);
    for (uint i = 0; i != nt; ++i) label_[i] = test[i].first;
    std::vector<double> m((size_t)nt * ntr), s(nt);
    check(sk_test_matrix(E.ctx(), dte, dtr, &kernel.sk_params(), norm_test ? 1 : 0,
                         normalize ? 1 : 0, m.data(), s.data()),
          E.ctx());
    matrix_.assign(m.begin(), m.end());
    self_.assign(s.begin(), s.end());
    return seconds_since(t0);
  }

  // predict-mode row: kernel_matrix.cpp:112-182, 635-697
  template <class Kernel, class ExampleSet>
  static double calculate(std::vector<value_type>& matrix,
                          const typename ExampleSet::value_type& data, const ExampleSet& train,
                          const std::vector<uint>& sv_index, const Kernel& kernel,
                          uint /*n_th*/ = 1, value_type* data_self = NULL) {
    const auto t0 = std::chrono::steady_clock::now();
    Engine& E = Engine::get();
    sk_dataset* dtr = E.dataset(train);
    const ExampleSet one(1, data);
    sk_dataset* dte = E.dataset(one);
    std::vector<double> v(train.size());
    for (size_t i = 0; i < v.size() && i < matrix.size(); ++i) v[i] = (double)matrix[i];
    std::vector<int32_t> idx(sv_index.begin(), sv_index.end());
    double self = 0.0;
    check(sk_test_row(E.ctx(), dte, 0, dtr, idx.empty() ? nullptr : idx.data(),
                      (int32_t)idx.size(), &kernel.sk_params(), v.data(),
                      data_self ? &self : nullptr),
          E.ctx());
    matrix.assign(v.begin(), v.end());
    if (data_self) *data_self = (value_type)self;
    return seconds_since(t0);
  }

  template <class Kernel, class ExampleSet>
  static double calculate(std::vector<value_type>& matrix,
                          const typename ExampleSet::value_type& data, const ExampleSet& train,
                          const Kernel& kernel, uint n_th = 1, value_type* data_self = NULL) {
    std::vector<uint> idx;
    return calculate(matrix, data, train, idx, kernel, n_th, data_self);
  }

  // kernel_matrix.cpp:59-110, 577-633
  template <class Kernel, class ExampleSet>
  static double diagonal(std::vector<value_type>& diag, const ExampleSet& train,
                         const std::vector<uint>& sv_index, const Kernel& kernel,
                         uint /*n_th*/ = 1) {
    const auto t0 = std::chrono::steady_clock::now();
    Engine& E = Engine::get();
    sk_dataset* ds = E.dataset(train);
    std::vector<double> d(train.size());
    for (size_t i = 0; i < d.size() && i < diag.size(); ++i) d[i] = (double)diag[i];
    std::vector<int32_t> idx(sv_index.begin(), sv_index.end());
    check(sk_diagonal(E.ctx(), ds, idx.empty() ? nullptr : idx.data(), (int32_t)idx.size(),
                      &kernel.sk_params(), d.data()),
          E.ctx());
    diag.assign(d.begin(), d.end());
    return seconds_since(t0);
  }

  template <class Kernel, class ExampleSet>
  static double diagonal(std::vector<value_type>& diag, const ExampleSet& train,
                         const Kernel& kernel, uint n_th = 1) {
    std::vector<uint> idx;
    return diagonal(diag, train, idx, kernel, n_th);
  }

  // libsvm precomputed-kernel text: kernel_matrix.cpp:756-770
  void print(std::ostream& out) const {
    std::vector<double> m(matrix_.begin(), matrix_.end());
    std::vector<const char*> lab;
    for (const auto& s : label_) lab.push_back(s.c_str());
    size_t need = 0;
    check(sk_format_libsvm(m.data(), (int32_t)row_, (int32_t)col_, lab.data(), nullptr, 0,
                           &need));
    std::string buf(need, '\0');
    check(sk_format_libsvm(m.data(), (int32_t)row_, (int32_t)col_, lab.data(), &buf[0], need,
                           &need));
    out << buf.c_str();
  }

 private:
  static double seconds_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  uint row_, col_;
  std::vector<value_type> matrix_;
  std::vector<value_type> self_;
  std::vector<std::string> label_;
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
