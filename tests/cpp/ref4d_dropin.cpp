// A reference-shaped main of the 4-D stem kernel tool (the shape of
// stem_kernel/main.cpp:88-160 after option parsing): examples through Fasta +
// load_examples, the kernel type picked by bp_bound / use_GU, a train Gram or
// a test x train matrix through KernelMatrix<value_type>, printed with
// print() plus the test norms matrix(i).  The only engine-specific line is
// the include.
//
// argv: out norms bp_bound use_GU band ali_bound normalize train.fa [test.fa]
// stdout: the matrix (%.17g), then the norms when a test set is given.
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <string>

#include "stem_kernel_ref_compat.hpp"

template <class Kernel>
static void run(const Kernel& kernel, const ExampleSet& train, const ExampleSet& test, bool normalize,
                bool norms, KernelMatrix<double>& matrix) {
  if (test.empty())
    matrix.calculate(train, kernel, normalize, 1);
  else
    matrix.calculate(test, train, kernel, norms, normalize, 1);
}

int main(int argc, char** argv) {
  if (argc < 9) return 2;
  typedef double value_type;
  const float gap = 0.8f, stack = 1.0f, subst = 0.5f;  // stem_kernel/main.cpp defaults
  const uint loop = 3;
  const float bp_bound = (float)std::atof(argv[3]);
  const bool use_GU = std::atoi(argv[4]) != 0;
  const uint band = (uint)std::atoi(argv[5]);
  const float ali_bound = (float)std::atof(argv[6]);
  const bool normalize = std::atoi(argv[7]) != 0;
  const std::string norm_out = argv[2];
  ExampleSet train, test;
  for (int a = 8; a < argc; ++a) {
    std::ifstream in(argv[a]);
    if (!in.is_open()) return 1;
    Fasta fasta(in);
    load_examples(a == 8 ? "+1" : "-1", fasta, a == 8 ? train : test);
  }
  try {
    KernelMatrix<value_type> matrix;
    if (bp_bound < 1.0) {
      StemKernel<value_type, BPMatrix> kernel(use_GU, loop, gap, stack, subst, band, ali_bound, bp_bound);
      run(kernel, train, test, normalize, !norm_out.empty(), matrix);
    } else if (use_GU) {
      StemKernel<value_type, WobbleBasePair> kernel(use_GU, loop, gap, stack, subst, band, ali_bound);
      run(kernel, train, test, normalize, !norm_out.empty(), matrix);
    } else {
      StemKernel<value_type, NormalBasePair> kernel(use_GU, loop, gap, stack, subst, band, ali_bound);
      run(kernel, train, test, normalize, !norm_out.empty(), matrix);
    }
    std::ofstream out(argv[1]);
    matrix.print(out);
    const size_t rows = test.empty() ? train.size() : test.size();
    for (size_t i = 0; i != rows; ++i) {
      for (size_t j = 0; j != train.size(); ++j) std::printf("%.17g ", matrix((uint)i, (uint)j));
      std::printf("\n");
    }
    for (size_t i = 0; i != test.size(); ++i) std::printf("%.17g\n", matrix((uint)i));
    // the Kernel concept itself: one pair through operator()
    if (bp_bound < 1.0 && train.size() > 1) {
      StemKernel<value_type, BPMatrix> kernel(use_GU, loop, gap, stack, subst, band, ali_bound, bp_bound);
      std::printf("pair %.17g\n", kernel(train[0].second, train[1].second));
    }
  } catch (const char* e) {
    std::fprintf(stderr, "error: %s\n", e);
    return 1;
  }
  return 0;
}
