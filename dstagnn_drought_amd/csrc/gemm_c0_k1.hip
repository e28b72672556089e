// GEMM instantiation unit: 64x64 tile, two-level k maps, fp32 (see gemm_kern.hpp)
#include "gemm_kern.hpp"

namespace dsgemm {
DS_GEMM_UNIT(gemm_c0_k1, 2, 2, 1, 1, true, false)
}  // namespace dsgemm
