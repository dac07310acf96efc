#!/bin/bash
# tools/build_variant.sh NAME "-DFLAG ..." -> ringpop_amd/variants/libringpop_hip_NAME.so (experiments only)
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p ringpop_amd/variants/$NAME
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function $*"
for s in rp_capi rp_ring rp_sim; do /opt/rocm/bin/hipcc $F -c ringpop_amd/csrc/$s.hip -o ringpop_amd/variants/$NAME/$s.o & done; wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ringpop_amd/variants/libringpop_hip_$NAME.so ringpop_amd/variants/$NAME/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
