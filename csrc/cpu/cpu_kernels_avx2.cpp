// The CPU stencils compiled for AVX2 + FMA (Makefile / CMake add -mavx2 -mfma for this file only);
// cpu_kernels.cpp selects them at run time when the host CPU supports both.
#include <cstring>

#include "mdfx/kernels.hpp"
#include "mdfx/stencil_math.hpp"

#define MDFX_CPU_NS cpu_avx2
#include "cpu_stencils.inc"
