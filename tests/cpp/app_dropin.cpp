// A reference-shaped App (the shape of App<K,LDF>::train / predict,
// common/framework.h:100-306) written against the reference's own names --
// KernelMatrix<value_type>, SuStemStrKernel<double,MData>,
// DataLoaderFactory<DataLoader<MData> >, BPMatrix::Options -- with one
// include changed: stem_kernel_compat.hpp in place of kernel_matrix.h,
// def_kernel.h and data.h.  Nothing below names the engine.
//
// argv: train.fa test.fa libsvm_out [normalize]
// stdout: the train Gram (%.17g), then one line per test example:
//         self and the test row against the train set.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <string>
#include <utility>
#include <vector>

#include "stem_kernel_compat.hpp"

template <class K, class LDF>
class App {
 public:
  typedef typename LDF::Data Data;
  typedef std::pair<std::string, Data> Example;
  typedef std::vector<Example> ExampleSet;
  typedef double value_type;

  App(const K& kernel, const LDF& ldf, bool normalize)
      : kernel_(kernel), ldf_(ldf), normalize_(normalize) {}

  bool train(const char* file, const char* out_file, KernelMatrix<value_type>& matrix) const {
    ExampleSet ex;
    if (!load_examples(ex, file)) return false;
    matrix.calculate(ex, kernel_, normalize_, 4);
    std::ofstream out(out_file);
    if (!out) throw out_file;
    matrix.print(out);
    return true;
  }

  bool predict(const char* train_file, const char* test_file,
               std::vector<std::vector<value_type> >& rows,
               std::vector<value_type>& selfs) const {
    ExampleSet ex;
    if (!load_examples(ex, train_file)) return false;
    std::vector<value_type> diag(ex.size()), vec(ex.size());
    std::vector<uint> sv_index;
    if (normalize_) KernelMatrix<value_type>::diagonal(diag, ex, sv_index, kernel_, 4);
    typename LDF::Loader* loader = ldf_.get_loader(test_file);
    if (loader == NULL) return false;
    while (true) {
      Data* data = loader->get();
      if (data == NULL) break;
      value_type self;
      KernelMatrix<value_type>::calculate(vec, std::make_pair(std::string("+1"), *data), ex,
                                          sv_index, kernel_, 4, &self);
      delete data;
      if (normalize_)
        for (uint j = 0; j != vec.size(); ++j) vec[j] /= std::sqrt(diag[j] * self);
      rows.push_back(vec);
      selfs.push_back(self);
    }
    delete loader;
    return true;
  }

 private:
  bool load_examples(ExampleSet& ex, const char* file) const {
    typename LDF::Loader* loader = ldf_.get_loader(file);
    if (loader == NULL) return false;
    while (true) {
      Data* d = loader->get();
      if (d == NULL) break;
      ex.push_back(std::make_pair(std::string(ex.size() % 2 ? "-1" : "+1"), *d));
      delete d;
    }
    delete loader;
    return true;
  }

  K kernel_;
  LDF ldf_;
  bool normalize_;
};

int main(int argc, char** argv) {
  if (argc < 4) return 2;
  const bool normalize = argc > 4 && std::atoi(argv[4]) != 0;
  try {
    // stem_kernel_lite/main.cpp defaults: th 0.01, alpha 0.2, beta 0.3,
    // loop_gap 0.2, gap 0.8, len_band 10
    BPMatrix::Options bp_opts;
    typedef DataLoaderFactory<DataLoader<MData> > LDF;
    LDF ldf(0.01f, bp_opts);
    SuStemStrKernel<double, MData> kernel(0.2, 0.3, 0.2, 0.8, 10);
    App<SuStemStrKernel<double, MData>, LDF> app(kernel, ldf, normalize);
    KernelMatrix<double> matrix;
    if (!app.train(argv[1], argv[3], matrix)) return 1;
    std::vector<std::vector<double> > rows;
    std::vector<double> selfs;
    if (!app.predict(argv[1], argv[2], rows, selfs)) return 1;
    for (uint i = 0; i != matrix.self().size(); ++i) {
      for (uint j = 0; j != matrix.self().size(); ++j) std::printf("%.17g ", matrix(i, j));
      std::printf("\n");
    }
    for (size_t t = 0; t != rows.size(); ++t) {
      std::printf("%.17g", selfs[t]);
      for (double v : rows[t]) std::printf(" %.17g", v);
      std::printf("\n");
    }
  } catch (const char* e) {
    std::fprintf(stderr, "error: %s\n", e);
    return 1;
  }
  return 0;
}
