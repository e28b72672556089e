// GEMM instantiation unit: the persistent tile loop, 64x64 tile, two-level k maps, fp32 (see gemm_kern.hpp)
#include "gemm_kern.hpp"

namespace dsgemm {
DS_GEMM_PUNIT(gemm_p0_k1, 2, 2, 1, 1, true)
}  // namespace dsgemm
