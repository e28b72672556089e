// GEMM instantiation unit: 128x32 tile, single-level k maps, fp32 with two-level accumulation
// (long reductions; see gemm_kern.hpp)
#include "gemm_kern.hpp"

namespace dsgemm {
DS_GEMM_UNIT_ACC2(gemm_c2_k0_a2, 4, 1, 1, 1, false)
}  // namespace dsgemm
