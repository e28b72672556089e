// GEMM instantiation unit: 128x32 tile, single-level k maps, bf16 operands (fp32 accumulate) (see gemm_kern.hpp)
#include "gemm_kern.hpp"

namespace dsgemm {
DS_GEMM_UNIT(gemm_c2_k0_bf, 4, 1, 1, 1, false, true)
}  // namespace dsgemm
