// A reference-shaped main of the naive string kernel tool (the shape of
// string_kernel/main.cpp:73-112 after option parsing): Fasta +
// load_examples, StringKernel<value_type>(gap), KernelMatrix::calculate and
// print.  The only engine-specific line is the include.
//
// argv: out gap normalize train.fa [test.fa]
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>

#include "string_kernel_compat.hpp"

int main(int argc, char** argv) {
  if (argc < 5) return 2;
  typedef double value_type;
  const float gap = (float)std::atof(argv[2]);
  const bool normalize = std::atoi(argv[3]) != 0;
  ExampleSet train, test;
  for (int a = 4; a < argc; ++a) {
    std::ifstream in(argv[a]);
    if (!in.is_open()) return 1;
    Fasta fasta(in);
    load_examples(a == 4 ? "+1" : "-1", fasta, a == 4 ? train : test);
  }
  try {
    StringKernel<value_type> kernel(gap);
    KernelMatrix<value_type> matrix;
    if (test.empty())
      matrix.calculate(train, kernel, normalize, 1);
    else
      matrix.calculate(test, train, kernel, false, normalize, 1);
    std::ofstream out(argv[1]);
    matrix.print(out);
    const size_t rows = test.empty() ? train.size() : test.size();
    for (size_t i = 0; i != rows; ++i) {
      for (size_t j = 0; j != train.size(); ++j) std::printf("%.17g ", matrix((uint)i, (uint)j));
      std::printf("\n");
    }
    if (train.size() > 1) std::printf("pair %.17g\n", kernel(train[0].second, train[1].second));
  } catch (const char* e) {
    std::fprintf(stderr, "error: %s\n", e);
    return 1;
  }
  return 0;
}
