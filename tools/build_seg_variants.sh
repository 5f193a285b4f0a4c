#!/bin/bash
# experiment builds of libadlbq with other chain segment / warm-up sizes (ADLBQ_LIB=... to load one)
set -e
cd "$(dirname "$0")/../adlb_amd/csrc"
for v in "128 512" "64 512"; do
  set -- $v
  out=../libadlbq_s$1.so
  objs=""
  for f in adlbq_store adlbq_reserve adlbq_steal; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -DADLBQ_CHAIN_SEG=$1 -DADLBQ_CHAIN_WARM=$2 -c $f.hip -o /tmp/${f}_s$1.o &
    objs="$objs /tmp/${f}_s$1.o"
  done
  wait
  /opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared $objs -o $out
  echo built $out
done
