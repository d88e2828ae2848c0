// Exercises include/stem_kernel.hpp the way App<K,LDF>::train would
// (common/framework.h:121-165): load examples, KernelMatrix::calculate,
// print in libsvm layout.  argv: n_seqs length seed [kind]
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <string>
#include <vector>

#include "stem_kernel.hpp"

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 6;
  const int len = argc > 2 ? std::atoi(argv[2]) : 60;
  uint64_t state = argc > 3 ? std::strtoull(argv[3], nullptr, 0) : 0x5EED0001ull;
  const int kind = argc > 4 ? std::atoi(argv[4]) : SK_SU_STEM_STR;
  try {
    std::vector<char> buf((size_t)n * (len + 1));
    sk::check(sk_random_sequences(&state, n, len, buf.data()));
    sk::Dataset train;
    for (int i = 0; i < n; ++i) {
      std::string s(&buf[(size_t)i * (len + 1)], len);
      std::vector<double> bpp((size_t)len * (len - 1) / 2);
      sk::check(sk_fold_synthetic(s.c_str(), len, 0, bpp.data()));
      train.add(i % 2 ? "-1" : "+1", {s}, {bpp});
    }
    sk::Context ctx(0);
    sk::KernelMatrix km(ctx);
    km.calculate(train, sk::Kernel((sk_kernel_kind)kind), false);
    km.print(std::cout);
  } catch (const char* e) {
    std::fprintf(stderr, "error: %s\n", e);
    return 1;
  }
  return 0;
}
