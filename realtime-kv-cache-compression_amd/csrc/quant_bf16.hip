// quant_bf16.hip — K4 instantiation for RTKV_BF16 (see quant_impl.h).
#include "quant_impl.h"

namespace rtkv {
template int launch_quant_dt<RTKV_BF16>(const QuantArgs&, hipStream_t);
}  // namespace rtkv
