// GEMM instantiation unit: 64x64 tile, single-level k maps, fp32 (see gemm_kern.hpp)
#include "gemm_kern.hpp"

namespace dsgemm {
DS_GEMM_UNIT(gemm_c0_k0, 2, 2, 1, 1, false, false)
}  // namespace dsgemm
