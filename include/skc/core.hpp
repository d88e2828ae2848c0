// skc/core.hpp -- shared machinery of the drop-in headers (not included
// directly by reference code): the process-wide engine context, the dataset
// cache, the Kernel-concept base class and KernelMatrix<V>.
//
// The reference ships four tools with four data types, all consumed by the
// same KernelMatrix<V> (common/kernel_matrix.h:13-108):
//   stem_kernel_lite  pair<string, MData>   (DAG + profile)      stem_kernel_compat.hpp
//   bpla_kernel       pair<string, MData>   (bpla's Data<...>)   bpla_kernel_compat.hpp
//   stem_kernel       pair<string, string>  (Example, 4-D)       stem_kernel_ref_compat.hpp
//   string_kernel     pair<string, string>  (Example, naive)     string_kernel_compat.hpp
// Each tool header specialises ExampleTraits<D> for its data type (how one
// example becomes an engine example, and its fingerprint) and defines its
// kernels over KernelBase; KernelMatrix batches every Gram through the C
// ABI (stem_kernel.h).  There is no CPU fallback.
#ifndef SKC_CORE_HPP
#define SKC_CORE_HPP

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

// gap-erased, lowercased row -> packed strict upper triangle p(i,j)
// (stem_kernel.h sk_dataset_add layout)
typedef std::function<void(const std::string&, bool /*no_GU*/, std::vector<double>&)> FoldFn;

// the Nussinov-Boltzmann stand-in (sk_fold_synthetic)
inline void synthetic_fold(const std::string& s, bool no_gu, std::vector<double>& out) {
  const int32_t n = (int32_t)s.size();
  out.assign(std::max<size_t>((size_t)n * (n > 0 ? n - 1 : 0) / 2, 1), 0.0);
  check(sk_fold_synthetic(s.c_str(), n, no_gu ? 1 : 0, out.data()));
}

// How a kernel wants raw-string examples built (the 4-D tool folds each
// sequence for its BPMatrix model; the naive string kernel does not).
struct BuildSpec {
  bool fold = false;   // fold each sequence (engine McCaskill, or fold_fn)
  int fold_flags = 0;  // SK_FOLD_NO_GU ...
  FoldFn fold_fn;      // empty: the engine's GPU McCaskill
  uint64_t tag() const { return (fold ? 1u : 0u) | (uint64_t)fold_flags << 1 | (fold_fn ? 1u << 8 : 0u); }
};

struct Fnv {
  uint64_t h = 1469598103934665603ull;
  void operator()(const void* p, size_t n) {
    const unsigned char* c = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ c[i]) * 1099511628211ull;
  }
};

// Specialised per data type by the tool headers:
//   static void add(sk_dataset*, const std::string& label, const D&, const BuildSpec&);
//   static void mix(Fnv&, const D&);
template <class D>
struct ExampleTraits;

// ------------------------------------------------------------------ engine
// One context per process on device $SK_DEVICE (default 0), or the rank's
// device under init_rank; example sets are packed and uploaded once and
// cached by content (App::predict hands the same train set to every test
// row).
class Engine {
 public:
  typedef std::shared_ptr<sk_dataset> DsPtr;
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
  // MPI_Bcast of 128 bytes).  Must come before anything opens the context
  // (a load that folds, a Gram): a context already open on another device
  // is refused rather than silently keeping every rank on one GPU.
  void init_rank(int device, int rank, int world, const uint8_t* uid, size_t uid_bytes) {
    std::lock_guard<std::mutex> g(mu_);
    if (ctx_ && device != device_)
      throw "Engine::init_rank must come before any load, fold or kernel call "
            "(the context is already open on another device)";
    device_ = device;
    open_locked();
    check(sk_comm_init(ctx_, uid, uid_bytes, rank, world), ctx_);
    world_ = world;
  }
  int world() const { return world_; }

  // Packed, uploaded dataset of an ExampleSet of (label, D).  The handle is
  // shared: the cache keeps at most 8 sets and evicts the least recently used
  // one, but a set stays alive while any caller still holds its handle (the
  // predict loop adds one single-example test set per row beside one train
  // set, so eviction must never free a set a call is still using).
  template <class ExampleSet>
  DsPtr dataset(const ExampleSet& ex, const BuildSpec& spec) {
    typedef typename ExampleSet::value_type::second_type D;
    const uint64_t key = fingerprint(ex, spec);
    {
      std::lock_guard<std::mutex> g(mu_);
      open_locked();
      auto it = cache_.find(key);
      if (it != cache_.end()) {
        it->second.used = ++tick_;
        return it->second.ds;
      }
    }
    DsPtr ds = make_ds();
    for (const auto& e : ex) ExampleTraits<D>::add(ds.get(), e.first, e.second, spec);
    std::lock_guard<std::mutex> g(mu_);
    check(sk_dataset_upload(ctx_, ds.get()), ctx_);
    return insert_lru(cache_, key, std::move(ds), 8);  // (a racing build of the same set is dropped)
  }

  // One pair through the Kernel concept (Kernel::operator()(x, y)): each
  // example is built once (DAG, profile, weights) and kept; the pair's
  // 2-example set is assembled from the built examples (sk_dataset_add_copy),
  // uploaded and evaluated in one launch.
  template <class D>
  double pair(const D& x, const D& y, const BuildSpec& spec, const sk_kernel_params& p) {
    const DsPtr bx = single(x, spec);
    const DsPtr by = single(y, spec);  // may evict bx from the cache: bx is still held
    DsPtr ds = make_ds();
    check(sk_dataset_add_copy(ds.get(), bx.get(), 0));
    check(sk_dataset_add_copy(ds.get(), by.get(), 0));
    std::lock_guard<std::mutex> g(mu_);
    open_locked();
    check(sk_dataset_upload(ctx_, ds.get()), ctx_);
    const int32_t a = 0, b = 1;
    double v = 0.0;
    check(sk_pairs(ctx_, ds.get(), &p, &a, &b, 1, &v), ctx_);
    return v;
  }

  // The engine's GPU McCaskill fold of gap-erased rows (BPMatrix FOLD without
  // ViennaRNA).  Prints a one-line notice the first time: values built from
  // it are not comparable with the reference's ViennaRNA-based outputs.
  void fold(const std::vector<std::string>& rows, int flags, std::vector<std::vector<double>>& out) {
    std::vector<const char*> p;
    size_t total = 0;
    for (const std::string& s : rows) {
      p.push_back(s.c_str());
      total += s.size() > 1 ? s.size() * (s.size() - 1) / 2 : 0;
    }
    std::vector<double> all(std::max<size_t>(total, 1));
    {
      std::lock_guard<std::mutex> g(mu_);
      open_locked();
      if (!fold_notice_ && !std::getenv("SK_QUIET_FOLD")) {
        std::fprintf(stderr,
                     "stem_kernel_amd: base-pairing probabilities from the engine's McCaskill fold "
                     "(Turner-1999 core loop model, not ViennaRNA): kernel values are not comparable "
                     "with ViennaRNA-based reference outputs (pass bpp through BPMatrix::Options::fold "
                     "for that)\n");
        fold_notice_ = true;
      }
      check(sk_fold_mccaskill(ctx_, (int32_t)p.size(), p.data(), flags, all.data(), nullptr), ctx_);
    }
    out.clear();
    size_t o = 0;
    for (const std::string& s : rows) {
      const size_t z = s.size() > 1 ? s.size() * (s.size() - 1) / 2 : 0;
      out.emplace_back(all.begin() + o, all.begin() + o + z);
      if (out.back().empty()) out.back().assign(1, 0.0);
      o += z;
    }
  }

 private:
  struct Entry {
    DsPtr ds;
    uint64_t used;
  };
  static DsPtr make_ds() {
    sk_dataset* raw = nullptr;
    check(sk_dataset_create(&raw));
    return DsPtr(raw, sk_dataset_free);
  }
  // caller holds mu_; evicts the least recently used entry when full (its
  // set is freed when the last holder drops its handle)
  DsPtr insert_lru(std::map<uint64_t, Entry>& m, uint64_t key, DsPtr ds, size_t cap) {
    auto it = m.find(key);
    if (it != m.end()) {
      it->second.used = ++tick_;
      return it->second.ds;
    }
    if (m.size() >= cap) {
      auto old = m.begin();
      for (auto j = m.begin(); j != m.end(); ++j)
        if (j->second.used < old->second.used) old = j;
      m.erase(old);
    }
    return m.emplace(key, Entry{std::move(ds), ++tick_}).first->second.ds;
  }
  Engine() {
    const char* e = std::getenv("SK_DEVICE");
    device_ = e ? std::atoi(e) : 0;
  }
  ~Engine() {
    cache_.clear();
    singles_.clear();
    if (ctx_) sk_close(ctx_);
  }
  void open_locked() {
    if (!ctx_) check(sk_open(device_, nullptr, &ctx_));
  }
  template <class D>
  DsPtr single(const D& d, const BuildSpec& spec) {
    Fnv f;
    ExampleTraits<D>::mix(f, d);
    const uint64_t t = spec.tag();
    f(&t, sizeof t);
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = singles_.find(f.h);
      if (it != singles_.end()) {
        it->second.used = ++tick_;
        return it->second.ds;
      }
    }
    DsPtr ds = make_ds();
    ExampleTraits<D>::add(ds.get(), "+1", d, spec);
    std::lock_guard<std::mutex> g(mu_);
    return insert_lru(singles_, f.h, std::move(ds), 16384);
  }
  template <class ExampleSet>
  static uint64_t fingerprint(const ExampleSet& ex, const BuildSpec& spec) {
    typedef typename ExampleSet::value_type::second_type D;
    Fnv f;  // FNV-1a over labels and examples
    for (const auto& e : ex) {
      f(e.first.data(), e.first.size() + 1);
      ExampleTraits<D>::mix(f, e.second);
    }
    const uint64_t t = spec.tag();
    f(&t, sizeof t);
    return f.h;
  }
  std::mutex mu_;
  int device_ = 0, world_ = 1;
  bool fold_notice_ = false;
  sk_context* ctx_ = nullptr;
  uint64_t tick_ = 0;
  std::map<uint64_t, Entry> cache_;
  std::map<uint64_t, Entry> singles_;
};

// ------------------------------------------------------------------ kernels
// Each kernel carries its sk_kernel_params and how its examples are built;
// operator() evaluates one pair on the GPU (the Kernel concept,
// stem_kernel_lite/def_kernel.h:43-51) -- KernelMatrix batches whole Grams.
template <class V, class D>
class KernelBase {
 public:
  typedef V value_type;
  typedef D Data;
  const sk_kernel_params& sk_params() const { return p_; }
  const BuildSpec& build_spec() const { return spec_; }
  value_type operator()(const Data& x, const Data& y) const {
    return (value_type)Engine::get().pair(x, y, spec_, p_);
  }

 protected:
  explicit KernelBase(sk_kernel_kind k) { sk_kernel_params_default(&p_, k); }
  sk_kernel_params p_;
  BuildSpec spec_;
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
    const Engine::DsPtr hold = E.dataset(train, kernel.build_spec());
    sk_dataset* ds = hold.get();
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
    const Engine::DsPtr htr = E.dataset(train, kernel.build_spec());
    const Engine::DsPtr hte = E.dataset(test, kernel.build_spec());  // may evict train: htr holds it
    sk_dataset* dtr = htr.get();
    sk_dataset* dte = hte.get();
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
    const Engine::DsPtr htr = E.dataset(train, kernel.build_spec());
    const ExampleSet one(1, data);
    const Engine::DsPtr hte = E.dataset(one, kernel.build_spec());  // may evict train: htr holds it
    sk_dataset* dtr = htr.get();
    sk_dataset* dte = hte.get();
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
    const Engine::DsPtr hold = E.dataset(train, kernel.build_spec());
    sk_dataset* ds = hold.get();
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

// ------------------------------------------------------------------ MData
// The alignment rows of one example and each row's folded matrix, as the
// lite (stem_kernel_lite/data.h:26-55) and BPLA (bpla_kernel/data.h:22-48)
// tools' MData consume them; the engine builds the DAG / profile / BPLA
// weights (sk_dataset_add) when a KernelMatrix needs them.
struct RowsData {
  std::vector<std::string> rows;
  std::vector<std::vector<double>> bpp;  // per row, gap-erased
  float th = 0.0f;
  bool use_bp = false;
};

// BPMatrix(list<string>, pf_scale, opts) (common/bpmatrix.cpp:122-128,
// 345-426): lowercase, erase gaps, fold every row (the caller's fold hook,
// else the engine's McCaskill honouring --noGU / --noClosingGU).
struct BPMatrixOptions {
  // common/bpmatrix.h:17-38 (+ the fold hook)
  bool alifold = false, contrafold = false, no_GU = false, no_closingGU = false,
       no_LonelyPairs = false;
  uint n_samples = 0;
  bool use_pf_scale_mfe = false;
  FoldFn fold;  // empty: the engine's GPU McCaskill
};

inline void fold_rows(RowsData& d, const BPMatrixOptions& opts) {
  std::vector<std::string> erased;
  for (const std::string& r : d.rows) {
    std::string s;
    for (char c : r)
      if (c != '-') s.push_back((char)std::tolower((unsigned char)c));
    erased.push_back(s);
  }
  if (opts.fold) {
    for (const std::string& s : erased) {
      d.bpp.emplace_back();
      opts.fold(s, opts.no_GU, d.bpp.back());
    }
    return;
  }
  if (opts.alifold || opts.contrafold || opts.n_samples > 0)
    throw "only the FOLD method (McCaskill per row) is supported by the engine";
  Engine::get().fold(erased,
                     (opts.no_GU ? SK_FOLD_NO_GU : 0) | (opts.no_closingGU ? SK_FOLD_NO_CLOSING_GU : 0) |
                         (opts.no_LonelyPairs ? SK_FOLD_NO_LONELY_PAIRS : 0),
                     d.bpp);
}

inline void add_rows(sk_dataset* ds, const std::string& label, const RowsData& d, float th) {
  std::vector<const char*> r;
  std::vector<const double*> b;
  for (const auto& s : d.rows) r.push_back(s.c_str());
  for (const auto& v : d.bpp) b.push_back(v.data());
  check(sk_dataset_add(ds, label.c_str(), (int)r.size(), r.data(), d.use_bp ? b.data() : nullptr, th,
                       d.use_bp ? 1 : 0));
}

inline void mix_rows(Fnv& f, const RowsData& d) {
  for (const auto& r : d.rows) f(r.data(), r.size() + 1);
  for (const auto& b : d.bpp) f(b.data(), b.size() * sizeof(double));
  f(&d.th, sizeof(float));
  f(&d.use_bp, sizeof(bool));
}

// Example files (stem_kernel_lite/data.cpp:460-586, bpla_kernel/data.cpp:
// 68-230): the type is sniffed like check_filetype and read by the engine's
// FASTA / CLUSTAL / MAF readers (sk_seqfile_*).
class SeqFile {
 public:
  explicit SeqFile(const char* filename) {
    int fmt = -1;
    std::FILE* fp = std::fopen(filename, "r");
    if (fp) {
      char line[4096];
      while (fmt < 0 && std::fgets(line, sizeof line, fp)) {
        if (line[0] == '>') fmt = SK_FMT_FASTA;
        else if (std::strncmp(line, "CLUSTAL", 7) == 0) fmt = SK_FMT_CLUSTAL;
        else if (std::strncmp(line, "a ", 2) == 0) fmt = SK_FMT_MAF;
      }
      std::fclose(fp);
    }
    if (fmt < 0 || sk_seqfile_read(filename, fmt, &f_) != SK_OK) {
      // the message outlives this (never constructed) loader
      static thread_local std::string msg;
      msg = std::string(filename) + ": no such file";
      throw msg.c_str();
    }
  }
  ~SeqFile() {
    if (f_) sk_seqfile_free(f_);
  }
  SeqFile(const SeqFile&) = delete;
  SeqFile& operator=(const SeqFile&) = delete;
  bool next(std::list<std::string>& ma) {
    if (!f_ || next_ >= sk_seqfile_count(f_)) return false;
    ma.clear();
    const int32_t nr = sk_seqfile_rows(f_, next_);
    for (int32_t r = 0; r < nr; ++r) ma.push_back(sk_seqfile_row(f_, next_, r));
    ++next_;
    return true;
  }

 private:
  sk_seqfile* f_ = nullptr;
  int64_t next_ = 0;
};

}  // namespace skc

#endif  // SKC_CORE_HPP
