// stem_kernel.hpp -- header-only C++ facade over the C ABI (stem_kernel.h).
//
// Mirrors the reference's host API so that App<K,LDF> code
// (common/framework.h:100-306) can switch by changing types, not call sites:
//   KernelMatrix<double>::calculate(train, kernel, normalize, n_th)
//                                              common/kernel_matrix.h:67-70
//   KernelMatrix::calculate(test, train, kernel, norm_test, normalize, n_th)
//                                              common/kernel_matrix.h:72-75
//   KernelMatrix::calculate(vec, data, train, sv_index, kernel, n_th, self)
//                                              common/kernel_matrix.h:77-83
//   KernelMatrix::diagonal(diag, train, sv_index, kernel, n_th)
//                                              common/kernel_matrix.h:95-98
//   KernelMatrix::print(ostream)               common/kernel_matrix.h:104
// Errors are thrown as `const char*` like the reference (framework.cpp
// catches `const char*`), carrying sk_last_error().  n_th is accepted and
// ignored: the device is the parallelism.
#ifndef STEM_KERNEL_HPP
#define STEM_KERNEL_HPP

#include <cmath>
#include <ostream>
#include <string>
#include <utility>
#include <vector>

#include "stem_kernel.h"

namespace sk {

inline void check(int st, const sk_context* ctx = nullptr) {
  if (st != SK_OK) throw ctx ? sk_last_error(ctx) : sk_strerror(st);
}

// A kernel object of the reference's Kernel concept: kind + parameters
// (stem_kernel_lite/def_kernel.h, ss_kernel.h).  Evaluation goes through a
// Context; there is no per-pair operator() on the host.
struct Kernel {
  sk_kernel_params p;
  explicit Kernel(sk_kernel_kind kind = SK_SU_STEM_STR) { sk_kernel_params_default(&p, kind); }
};

// ExampleSet of (label, MData): examples built host-side, uploaded once.
class Dataset {
 public:
  Dataset() { check(sk_dataset_create(&ds_)); }
  ~Dataset() { if (ds_) sk_dataset_free(ds_); }
  Dataset(const Dataset&) = delete;
  Dataset& operator=(const Dataset&) = delete;

  // One alignment (n_rows rows) with its per-row bpp (strict upper triangle,
  // see stem_kernel.h); th = --basepair.
  void add(const std::string& label, const std::vector<std::string>& rows,
           const std::vector<std::vector<double>>& bpp, float th = 0.01f, bool use_bp = true) {
    std::vector<const char*> r;
    std::vector<const double*> b;
    for (auto& s : rows) r.push_back(s.c_str());
    for (auto& v : bpp) b.push_back(v.data());
    check(sk_dataset_add(ds_, label.c_str(), (int)rows.size(), r.data(),
                         use_bp ? b.data() : nullptr, th, use_bp ? 1 : 0));
  }
  int size() const { return sk_dataset_size(ds_); }
  std::string label(int i) const { return sk_dataset_label(ds_, i); }
  sk_dataset* get() const { return ds_; }

 private:
  sk_dataset* ds_ = nullptr;
};

class Context {
 public:
  explicit Context(int device = 0, void* hip_stream = nullptr) {
    check(sk_open(device, hip_stream, &ctx_));
  }
  ~Context() { if (ctx_) sk_close(ctx_); }
  Context(const Context&) = delete;
  Context& operator=(const Context&) = delete;
  sk_context* get() const { return ctx_; }
  void upload(Dataset& d) const { check(sk_dataset_upload(ctx_, d.get()), ctx_); }

 private:
  sk_context* ctx_ = nullptr;
};

// KernelMatrix<double> with the reference's member functions.
class KernelMatrix {
 public:
  typedef double value_type;
  explicit KernelMatrix(Context& ctx) : ctx_(ctx) {}

  // Train Gram (kernel_matrix.cpp:485-575); returns 0.0 (the reference
  // returns summed CPU seconds).
  double calculate(Dataset& train, const Kernel& k, bool normalize = false, unsigned = 1) {
    ctx_.upload(train);
    const int n = train.size();
    rows_ = cols_ = n;
    m_.assign((size_t)n * n, 0.0);
    labels_.clear();
    for (int i = 0; i < n; ++i) labels_.push_back(train.label(i));
    check(sk_gram(ctx_.get(), train.get(), &k.p, normalize ? 1 : 0, m_.data()), ctx_.get());
    return 0.0;
  }

  // Test x train (kernel_matrix.cpp:699-754): row i = K(train[j], test[i]).
  double calculate(Dataset& test, Dataset& train, const Kernel& k, bool norm_test = false,
                   bool normalize = false, unsigned = 1) {
    ctx_.upload(test);
    ctx_.upload(train);
    rows_ = test.size();
    cols_ = train.size();
    m_.assign((size_t)rows_ * cols_, 0.0);
    self_.assign(rows_, 0.0);
    labels_.clear();
    for (int i = 0; i < rows_; ++i) labels_.push_back(test.label(i));
    check(sk_test_matrix(ctx_.get(), test.get(), train.get(), &k.p, norm_test, normalize,
                         m_.data(), self_.data()),
          ctx_.get());
    return 0.0;
  }

  // Predict-mode row (kernel_matrix.cpp:635-697): vec[i] = K(train[i], test[t])
  // for i in sv_index (all i if empty); vec is indexed by train position.
  static double calculate(Context& ctx, std::vector<value_type>& vec, Dataset& test, int t,
                          Dataset& train, const std::vector<unsigned>& sv_index, const Kernel& k,
                          unsigned = 1, value_type* data_self = nullptr) {
    ctx.upload(test);
    ctx.upload(train);
    vec.resize(train.size());
    std::vector<int32_t> idx(sv_index.begin(), sv_index.end());
    check(sk_test_row(ctx.get(), test.get(), t, train.get(), idx.empty() ? nullptr : idx.data(),
                      (int32_t)idx.size(), &k.p, vec.data(), data_self),
          ctx.get());
    return 0.0;
  }

  // kernel_matrix.cpp:577-633
  static double diagonal(Context& ctx, std::vector<value_type>& diag, Dataset& train,
                         const std::vector<unsigned>& sv_index, const Kernel& k, unsigned = 1) {
    ctx.upload(train);
    diag.resize(train.size());
    std::vector<int32_t> idx(sv_index.begin(), sv_index.end());
    check(sk_diagonal(ctx.get(), train.get(), idx.empty() ? nullptr : idx.data(),
                      (int32_t)idx.size(), &k.p, diag.data()),
          ctx.get());
    return 0.0;
  }

  value_type operator()(int i, int j) const { return m_[(size_t)i * cols_ + j]; }
  const std::vector<value_type>& self() const { return self_; }
  int rows() const { return rows_; }
  int cols() const { return cols_; }

  // libsvm precomputed-kernel text (kernel_matrix.cpp:756-770)
  void print(std::ostream& out) const {
    std::vector<const char*> lab;
    for (auto& s : labels_) lab.push_back(s.c_str());
    size_t need = 0;
    check(sk_format_libsvm(m_.data(), rows_, cols_, lab.data(), nullptr, 0, &need));
    std::string buf(need, '\0');
    check(sk_format_libsvm(m_.data(), rows_, cols_, lab.data(), &buf[0], need, &need));
    out << buf.c_str();
  }

 private:
  Context& ctx_;
  int rows_ = 0, cols_ = 0;
  std::vector<value_type> m_, self_;
  std::vector<std::string> labels_;
};

}  // namespace sk

#endif  // STEM_KERNEL_HPP
