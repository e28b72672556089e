// GEMM instantiation unit: 128x128 tile, single-level k maps, bf16 operands (fp32 accumulate) (see gemm_kern.hpp)
#include "gemm_kern.hpp"

namespace dsgemm {
DS_GEMM_UNIT(gemm_c1_k0_bf, 2, 2, 2, 2, false, true)
}  // namespace dsgemm
