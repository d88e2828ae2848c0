// string_kernel_compat.hpp -- drop-in for the naive string kernel tool
// (string_kernel/, --enable-string-kernel): replacing
//     #include "string_kernel.h"
//     #include "../common/kernel_matrix.h"
//     #include "../common/example.h"
//     #include "../common/fasta.h"
// in string_kernel/main.cpp by
//     #include "string_kernel_compat.hpp"
// is the only edit; main's code (string_kernel/main.cpp:73-112) compiles
// unchanged and the Gram runs on the GPU (SK_NAIVE_STR of
// csrc/kernels/profile_string.hip).
//
//   StringKernel<V>(gap = 1)          string_kernel/string_kernel.h:10-22,
//                                     string_kernel.cpp:14-85 (exact match of
//                                     the lowercased characters, weight gap^2)
//   Example, ExampleSet, Fasta, load_examples, KernelMatrix<V>
#ifndef STRING_KERNEL_COMPAT_HPP
#define STRING_KERNEL_COMPAT_HPP

#include "skc/core.hpp"
#include "skc/example.hpp"

namespace skc {

template <class ValueType>
class StringKernel : public KernelBase<ValueType, std::string> {
 public:
  typedef ValueType value_type;
  explicit StringKernel(value_type gap = 1) : KernelBase<ValueType, std::string>(SK_NAIVE_STR) {
    this->p_.gap = gap;
  }
};

}  // namespace skc

#ifndef SKC_NO_REFERENCE_NAMES
using skc::Example;
using skc::ExampleSet;
using skc::Fasta;
using skc::KernelMatrix;
using skc::load_examples;
using skc::StringKernel;
typedef unsigned int uint;
#endif

#endif  // STRING_KERNEL_COMPAT_HPP
