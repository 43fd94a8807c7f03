#!/bin/bash
# Builds libort.so with extra compile flags into build/ab/lib<NAME>.so (own object dir), for
# tools/ab_stream.py.  usage: tools/build_variant.sh NAME [extra hipcc/g++ flags...]
set -e
NAME=$1; shift
cd "$(dirname "$0")/.."
BASE="-O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fno-slp-vectorize -fPIC -Wall -Wno-unused-parameter"
make -s lib OBJ=build/obj_$NAME LIB=build/ab/lib$NAME.so HIPFLAGS="$BASE $*" -j8
