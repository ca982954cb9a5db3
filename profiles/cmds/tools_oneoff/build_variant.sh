#!/usr/bin/env bash
# Build an experimental variant of librtkv.so with extra defines for some objects (default: the K4
# units; VARIANT_OBJS="importance" for K1), for A/B runs on the GPU box through RTKV_LIB (not part of
# the product build):
#   bash tools/build_variant.sh sc1 -DRTKV_K4_SC1    ->  realtime-kv-cache-compression_amd/librtkv_sc1.so
set -euo pipefail
name=$1; shift
cd "$(dirname "$0")/../realtime-kv-cache-compression_amd"
make -s -j8 librtkv.so
mkdir -p build_$name
objs=""
for f in build/*.o; do
  b=$(basename "$f" .o)
  if [[ " ${VARIANT_OBJS:-quant_f32 quant_f16 quant_bf16} " == *" $b "* ]]; then
      /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math \
        -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -I../include -Icsrc "$@" \
        -c csrc/$b.hip -o build_$name/$b.o
      objs="$objs build_$name/$b.o"
  else
    objs="$objs $f"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o librtkv_$name.so $objs -ldl
echo "built librtkv_$name.so"
