// GEMM instantiation unit: the persistent tile loop, 128x32 tile, two-level k maps, fp32 (see gemm_kern.hpp)
#include "gemm_kern.hpp"

namespace dsgemm {
DS_GEMM_PUNIT(gemm_p2_k1, 4, 1, 1, 1, true)
}  // namespace dsgemm
