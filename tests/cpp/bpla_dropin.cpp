// A reference-shaped BPLA tool (the shape of bpla_kernel/main.cpp:100-127
// and App<K,LDF>::train, common/framework.h:121-165): the score table, the
// loader factory built as `LDF ldf;` (--noBP) or `LDF ldf(bp_opts);`,
// BPLAKernel<double,MData>, examples read through the factory's loader and a
// train Gram through KernelMatrix.  The only engine-specific line is the
// include.
//
// argv: out noBP SW normalize train(.fa|.aln|.maf)
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <utility>
#include <vector>

#include "bpla_kernel_compat.hpp"

static const float kScore[4][4] = {  // bpla_kernel/main.cpp default table (ACGU)
    {5.846613f, -1.860000f, -1.460000f, -1.390000f},
    {-1.860000f, 4.786613f, -2.480000f, -1.050000f},
    {-1.460000f, -2.480000f, 4.656613f, -1.740000f},
    {-1.390000f, -1.050000f, -1.740000f, 5.276613f}};

template <class LDF>
static int train(const LDF& ldf, bool noBP, bool SW, bool normalize, const char* file, const char* out_file) {
  typedef typename LDF::Data Data;
  std::vector<std::vector<double> > score_table(4, std::vector<double>(4));
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) score_table[i][j] = kScore[i][j];
  const float gap = -8.0f, ext = -0.75f, alpha = 4.5f, beta = 0.11f;
  BPLAKernel<double, Data> kernel(score_table, noBP, SW, gap, ext, alpha, beta);
  std::vector<std::pair<std::string, Data> > ex;
  typename LDF::Loader* loader = ldf.get_loader(file);
  while (Data* d = loader->get()) {
    ex.push_back(std::make_pair(std::string(ex.size() % 2 ? "-1" : "+1"), *d));
    delete d;
  }
  delete loader;
  KernelMatrix<double> matrix;
  matrix.calculate(ex, kernel, normalize, 1);
  std::ofstream out(out_file);
  matrix.print(out);
  for (size_t i = 0; i != ex.size(); ++i) {
    for (size_t j = 0; j != ex.size(); ++j) std::printf("%.17g ", matrix((uint)i, (uint)j));
    std::printf("\n");
  }
  if (ex.size() > 1) {
    std::printf("pair %.17g\n", kernel(ex[0].second, ex[1].second));
    if (!noBP && !SW) {
      std::vector<double> param = {alpha, beta, gap, ext}, d;
      const double v = BPLAKernel<double, Data>::compute_gradients(ex[0].second, ex[1].second, score_table,
                                                                     param, d);
      std::printf("grad %.17g %.17g %.17g %.17g %.17g\n", v, d[0], d[1], d[2], d[3]);
    }
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 6) return 2;
  const bool noBP = std::atoi(argv[2]) != 0, SW = std::atoi(argv[3]) != 0;
  const bool normalize = std::atoi(argv[4]) != 0;
  try {
    typedef DataLoaderFactory<DataLoader<MData> > LDF;
    if (noBP) {
      LDF ldf;
      return train(ldf, noBP, SW, normalize, argv[5], argv[1]);
    }
    BPMatrix::Options bp_opts;
    LDF ldf(bp_opts);
    return train(ldf, noBP, SW, normalize, argv[5], argv[1]);
  } catch (const char* e) {
    std::fprintf(stderr, "error: %s\n", e);
    return 1;
  }
}
