// GEMM instantiation unit: 128x32 tile, single-level k maps, fp32 (see gemm_kern.hpp)
#include "gemm_kern.hpp"

namespace dsgemm {
DS_GEMM_UNIT(gemm_c2_k0, 4, 1, 1, 1, false, false)
}  // namespace dsgemm
