// Harness for the PARTIAL reference build (oracle/_ref/libskref.so).
// Links the reference's own, unmodified translation units
//   common/rna.cpp, common/profile.cpp, stem_kernel_lite/ribosum.cpp
// (compiled in place from /root/reference by oracle/Makefile) and exposes the
// pieces of the stem-kernel input path they define through a C ABI, so that
// tests/test_oracle_pinning.py can pin the oracle's alphabet, IUPAC profile
// and RIBOSUM85-60 restatements against the reference itself.
// These are the only hot-path TUs that build with nothing but the C++
// standard library; everything else needs Boost/ViennaRNA/config.h.
#include <cstring>
#include <list>
#include <string>
#include "rna.h"
#include "profile.h"
#include "ribosum.h"

extern "C" {

int skref_char2rna(int c) { return (int)char2rna((char)c); }

// ProfileSequence(list<string>) (common/profile.h:555-562): out float[L][5]
int skref_profile(int n_rows, const char* const* rows, float* out5, float* n_seqs) {
  std::list<std::string> ma;
  for (int r = 0; r != n_rows; ++r) ma.push_back(std::string(rows[r]));
  ProfileSequence ps(ma);
  for (unsigned i = 0; i != ps.size(); ++i)
    for (unsigned k = 0; k != N_RNA + 1; ++k) out5[i * 5 + k] = ps[i][k];
  *n_seqs = ps.n_seqs();
  return (int)ps.size();
}

void skref_ribosum(float* s16, float* p256) {
  std::memcpy(s16, &ribosum_s[0][0], sizeof(float) * 16);
  std::memcpy(p256, &ribosum_p[0][0][0][0], sizeof(float) * 256);
}
}
