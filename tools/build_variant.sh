#!/bin/bash
# Build an experimental libadlbq variant with extra compile flags (measurement only; the product is
# adlb_amd/libadlbq.so):  tools/build_variant.sh seg128 -DADLBQ_CHAIN_SEG=128
# -> adlb_amd/variants/libadlbq_seg128.so, loaded with ADLBQ_LIB=<that path>
set -e
name=$1; shift
D=$(cd "$(dirname "$0")/.." && pwd)
O=$D/adlb_amd/variants/$name
mkdir -p $O
for f in adlbq_store adlbq_reserve adlbq_steal adlbq_rsx adlbq_wide adlbq_keyrank; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$D/include "$@" -c $D/adlb_amd/csrc/$f.hip -o $O/$f.o &
done
wait
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared $O/*.o -o $D/adlb_amd/variants/libadlbq_$name.so
rm -rf $O
