// Internal host-side structures of the stem-kernel engine (not part of the ABI).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

// Experiment switches (A/B variants of equal results, tuning knobs): read
// from the environment only in the experiments build (make exp ->
// build/libstem_kernel_amd_exp.so, -DSK_EXPERIMENTS); the shipped library
// compiles them out -- SK_KNOB is a null pointer and the switch's name is not
// in the binary -- so it reads only diagnostics and thread-count variables.
#ifdef SK_EXPERIMENTS
#include <cstdlib>
#define SK_KNOB(name) (std::getenv(name))
#else
#define SK_KNOB(name) ((const char*)nullptr)
#endif

namespace sk {

// ---------------------------------------------------------------------------
// One example (the reference's MData, stem_kernel_lite/data.h:26-55), held as
// flat CSR arrays.  Node numbering is the reference's post-order numbering
// (children before parents), edges keep the reference's candidate-list order.
struct Example {
  int len = 0;          // aligned length
  int n_rows = 0;       // alignment rows
  bool has_bp = false;  // built with folding (DAG + weights) or MData(ma)
  std::vector<std::string> rows;
  // ProfileSequence of all rows (common/profile.cpp): [len][5], n_seqs
  std::vector<float> prof5;
  float n_seqs = 0.f;
  // fill_weight (data.cpp:437-453)
  std::vector<float> pos_weight;
  // averaged bp matrix over the aligned length (packed strict upper)
  std::vector<double> bpp;
  // DAG (dag.h): nodes
  std::vector<uint32_t> first, last;
  std::vector<float> weight;
  std::vector<uint32_t> edge_off;  // n_nodes+1
  std::vector<uint32_t> edge_to, edge_gaps;
  std::vector<uint32_t> bpf_off;   // n_nodes+1
  std::vector<uint8_t> bpf_code;   // a*4+b
  std::vector<float> bpf_p;
  std::vector<uint32_t> roots;
  std::vector<uint32_t> max_pa;
  int n_nodes() const { return (int)first.size(); }
  int n_edges() const { return (int)edge_to.size(); }
};

// Builds an Example from aligned rows and per-row (gap-erased) bpp matrices.
// Restates MData(ma, th, ...) (stem_kernel_lite/data.cpp:324-345).
void build_example(Example& ex, int n_rows, const char* const* rows,
                   const double* const* bpp_rows, float th, bool use_bp);

// synth.cpp
uint64_t splitmix64_next(uint64_t& s);
void fold_nussinov(const char* seq, int n, bool no_gu, double* out);
void random_sequence(uint64_t& state, int len, char* out);

inline size_t tri_index(int n, int i, int j) {  // 0-based i<j
  return (size_t)i * n - (size_t)i * (i + 1) / 2 + (size_t)(j - i - 1);
}

int char2rna(int c);
extern const float kIupac[16][4];

}  // namespace sk
