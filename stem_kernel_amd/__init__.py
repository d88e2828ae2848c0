"""MI355X-native stem-kernel Gram engine (gfx950 HIP kernels behind a C ABI).

See include/stem_kernel.h for the ABI and DESIGN.md for the design.
"""
from ._lib import StemKernelError, lib, default_params  # noqa: F401
from .kernel_matrix import (  # noqa: F401
    BPLAKernel, Context, Dataset, KernelMatrix, SVMModel, LSuStemKernel, LSuStemStrKernel, NaiveStringKernel, SiStemKernel,
    SiStemStrKernel, StemKernel4D, StemStrKernel, StringKernel, SuStemKernel, SuStemStrKernel, fold,
    format_libsvm, parse_examples, random_sequences, read_examples,
)

__version__ = "0.1.0"
