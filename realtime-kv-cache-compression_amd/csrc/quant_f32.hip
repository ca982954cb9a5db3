// quant_f32.hip — K4 instantiation for RTKV_F32 (see quant_impl.h).
#include "quant_impl.h"

namespace rtkv {
template int launch_quant_dt<RTKV_F32>(const QuantArgs&, hipStream_t);
}  // namespace rtkv
