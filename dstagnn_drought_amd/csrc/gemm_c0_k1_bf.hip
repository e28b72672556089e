// GEMM instantiation unit: 64x64 tile, two-level k maps, bf16 operands (fp32 accumulate) (see gemm_kern.hpp)
#include "gemm_kern.hpp"

namespace dsgemm {
DS_GEMM_UNIT(gemm_c0_k1_bf, 2, 2, 1, 1, true, true)
}  // namespace dsgemm
