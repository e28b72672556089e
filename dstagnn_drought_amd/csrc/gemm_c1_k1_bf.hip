// GEMM instantiation unit: 128x128 tile, two-level k maps, bf16 operands (fp32 accumulate) (see gemm_kern.hpp)
#include "gemm_kern.hpp"

namespace dsgemm {
DS_GEMM_UNIT(gemm_c1_k1_bf, 2, 2, 2, 2, true, true)
}  // namespace dsgemm
