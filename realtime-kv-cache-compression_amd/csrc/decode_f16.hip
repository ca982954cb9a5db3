// decode_f16.hip — the fp16 instantiations of the decode split kernel (decode_kernel.h), compiled
// without SLP vectorisation (Makefile): the value accumulation then stays one v_fma_mix_f32 per
// element instead of a widening plus v_pk_fma_f32 (7-9 % faster); bf16/fp32 (decode.hip) keep SLP,
// which their packed bf16 / fp32 arithmetic gains from.
#include "decode_kernel.h"

namespace rtkv {

int launch_decode_split_f16(const DecodeArgs& a, int nch, int gq, int D, dim3 grid, size_t lds, hipStream_t st) {
  return launch_decode_split<RTKV_F16>(a, nch, gq, D, grid, lds, st);
}

}  // namespace rtkv
