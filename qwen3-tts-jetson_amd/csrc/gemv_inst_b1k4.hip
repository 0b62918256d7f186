// gemv_inst_b1k4.hip — explicit instantiations of the GEMV launch templates (gemv_kernel.h)
#include "gemv_kernel.h"

namespace q3t {
template void launch_pro<1, 1, 4>(const GemvParams &p, int nl, dim3 grid, size_t lds, hipStream_t s);
template void launch_pro<2, 1, 4>(const GemvParams &p, int nl, dim3 grid, size_t lds, hipStream_t s);
}  // namespace q3t
