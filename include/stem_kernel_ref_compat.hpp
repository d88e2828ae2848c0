// stem_kernel_ref_compat.hpp -- drop-in for the reference implementation's
// 4-D stem kernel tool (stem_kernel/, --enable-ref-impl): replacing
//     #include "stem_kernel.h"
//     #include "../common/kernel_matrix.h"
//     #include "../common/example.h"
//     #include "../common/fasta.h"
// in stem_kernel/main.cpp by
//     #include "stem_kernel_ref_compat.hpp"
// is the only edit; main's code (stem_kernel/main.cpp:88-160: Fasta,
// load_examples, StemKernel<value_type, BPMatrix | WobbleBasePair |
// NormalBasePair>, KernelMatrix::calculate / print / operator()(i)) compiles
// unchanged and every Gram cell is computed on the GPU (sk_gram /
// sk_test_matrix over SK_STEM4D, csrc/kernels/stem4d.hip).
//
//   StemKernel<V, BPMat>(use_GU, loop, gap, stack, subst, band, ali_bound,
//                        bp_bound = 1.0)          stem_kernel/stem_kernel.h:25-54
//     operator()(x, y): full_dp, or partial_dp when ali_bound > 0 || band > 0
//   NormalBasePair, WobbleBasePair, BPMatrix      stem_kernel/stem_kernel.cpp:353-421
//   Example, ExampleSet, Fasta, load_examples      common/example.h, common/fasta.h
//   KernelMatrix<V>                                common/kernel_matrix.h:13-108
//
// Kept exactly: the BPMatrix model's probabilities come from folding each
// sequence with noGU = use_GU (the reference constructs PFWrapper(seq,
// useGU), whose second parameter is noGU: stem_kernel.cpp:405 against
// common/pf_wrapper.h:17-18); Normal/Wobble models with the CLI's default
// bp_bound 1.0 give K = 1 (prob <= 1 is never > bp_bound); the -a
// constraints follow the reference as built (LogValue zerop never true:
// stem_kernel.h's sk_kernel_params.ali_zerop_fixed = 0).
// Differs: the reference folds x and y with ViennaRNA for every pair; here
// each sequence is folded once, by the engine's McCaskill (notice on stderr;
// parity against ViennaRNA unpinned) or by skc::stem4d_fold() when set.
#ifndef STEM_KERNEL_REF_COMPAT_HPP
#define STEM_KERNEL_REF_COMPAT_HPP

#include "skc/core.hpp"
#include "skc/example.hpp"

namespace skc {

// base-pair models (tags; the engine evaluates them)
class NormalBasePair {};
class WobbleBasePair {};
class BPMatrix {};

template <class BPMat>
struct BpModel;
template <>
struct BpModel<BPMatrix> {
  static const int value = 0;
};
template <>
struct BpModel<NormalBasePair> {
  static const int value = 1;
};
template <>
struct BpModel<WobbleBasePair> {
  static const int value = 2;
};

// fold used for the BPMatrix model (empty: the engine's GPU McCaskill)
inline FoldFn& stem4d_fold() {
  static FoldFn f;
  return f;
}

template <class ValueType, class BPMat>
class StemKernel : public KernelBase<ValueType, std::string> {
 public:
  typedef ValueType value_type;

  StemKernel(bool use_GU, uint loop, value_type gap, value_type stack, value_type subst, uint band,
             float ali_bound, float bp_bound = 1.0)
      : KernelBase<ValueType, std::string>(SK_STEM4D) {
    sk_kernel_params& p = this->p_;
    p.gap = gap;
    p.stack = stack;
    p.subst = subst;
    p.loop = loop;
    p.len_band = band;
    p.ali_bound = ali_bound;
    p.ali_zerop_fixed = 0;
    p.bp_bound = bp_bound;
    p.bp_model = BpModel<BPMat>::value;
    if (BpModel<BPMat>::value == 0) {
      this->spec_.fold = true;
      this->spec_.fold_flags = use_GU ? SK_FOLD_NO_GU : 0;  // PFWrapper(seq, useGU): noGU = useGU
      this->spec_.fold_fn = stem4d_fold();
    }
  }
};

}  // namespace skc

#ifndef SKC_NO_REFERENCE_NAMES
using skc::BPMatrix;
using skc::Example;
using skc::ExampleSet;
using skc::Fasta;
using skc::KernelMatrix;
using skc::load_examples;
using skc::NormalBasePair;
using skc::StemKernel;
using skc::WobbleBasePair;
typedef unsigned int uint;
#endif

#endif  // STEM_KERNEL_REF_COMPAT_HPP
