#!/bin/bash
# Variant of libavdb_hip.so with ONE translation unit rebuilt with extra flags
# (the others from the in-tree objects), for on-device A/B:
#   tools/build_variant_one.sh NAME SOURCE.hip [-DFOO=1 ...] -> annotatedvdb_amd/_lib/var/libavdb_NAME.so
cd "$(dirname "$0")/.."
name=$1; src=$2; shift 2
mkdir -p annotatedvdb_amd/_lib/var
obj=/tmp/var_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I include "$@" -c "annotatedvdb_amd/csrc/$src" -o "$obj" || exit 1
others=$(ls annotatedvdb_amd/_lib/obj/*.o | grep -v "/${src%.hip}.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o annotatedvdb_amd/_lib/var/libavdb_$name.so $others "$obj"
