// fused_f32.hip — the fused K2 + K4 launch (fused.h) for F32 K/V rows (its own translation unit so the
// per-dtype instantiations compile in parallel).
#include "fused.h"

namespace rtkv {

int launch_fused_f32(const FinalizeArgs& f, void* sel_ws, const QuantArgs& q, hipStream_t st) {
  FusedArgs x;
  x.g = make_fast_args(f, sel_ws);
  x.g.fused = 1;
  x.q = q;
  return launch_fused_kv<RTKV_F32>(x, (int)((q.kv.H * q.kv.D) / 8), st);
}

}  // namespace rtkv
