// GEMM instantiation unit: the persistent tile loop, 128x32 tile, single-level k maps (+ K-concatenated), fp32 (see gemm_kern.hpp)
#include "gemm_kern.hpp"

namespace dsgemm {
DS_GEMM_PUNIT(gemm_p2_k0, 4, 1, 1, 1, false)
}  // namespace dsgemm
