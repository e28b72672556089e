// GEMM instantiation unit: the persistent tile loop, 64x64 tile, single-level k maps, fp32 (see gemm_kern.hpp)
#include "gemm_kern.hpp"

namespace dsgemm {
DS_GEMM_PUNIT(gemm_p0_k0, 2, 2, 1, 1, false)
}  // namespace dsgemm
