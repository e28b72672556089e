// GEMM instantiation unit: 64x64 tile, two-level k maps, fp32 with two-level accumulation
// (long reductions; see gemm_kern.hpp)
#include "gemm_kern.hpp"

namespace dsgemm {
DS_GEMM_UNIT_ACC2(gemm_c0_k1_a2, 2, 2, 1, 1, true)
}  // namespace dsgemm
