#!/bin/bash
# tools/build_variant.sh NAME "-DFLAG ..." -> ringpop_amd/variants/libringpop_hip_NAME.so (experiments only)
# SRC=<dir>: take the .hip sources from <dir> (e.g. a git-exported older tree) instead of ringpop_amd/csrc
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p ringpop_amd/variants/$NAME
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function $*"
SRC=${SRC:-ringpop_amd/csrc}
pids=()
for s in rp_capi rp_ring rp_sim rp_node rp_calib; do /opt/rocm/bin/hipcc $F -I$SRC -c $SRC/$s.hip -o ringpop_amd/variants/$NAME/$s.o & pids+=($!); done
for p in "${pids[@]}"; do wait $p || { echo "variant $NAME: compile failed" >&2; exit 1; }; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ringpop_amd/variants/libringpop_hip_$NAME.so ringpop_amd/variants/$NAME/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
