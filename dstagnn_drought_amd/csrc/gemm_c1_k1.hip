// GEMM instantiation unit: 128x128 tile, two-level k maps, fp32 (see gemm_kern.hpp)
#include "gemm_kern.hpp"

namespace dsgemm {
DS_GEMM_UNIT(gemm_c1_k1, 2, 2, 2, 2, true, false)
}  // namespace dsgemm
