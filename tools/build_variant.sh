#!/bin/bash
# Builds libort.so with extra compile flags into build/ab/lib<NAME>.so (own object dir), for
# tools/ab_stream.py.  usage: tools/build_variant.sh NAME [extra hipcc/g++ flags...]
# A/B and timeline variants are analysis builds (-DORT_ANALYSIS=1: ORT_OPT_DEBUG_FLAGS, the
# ort_debug_* hooks, ORT_TILE_CLOCK / ORT_PERSIST_CLOCK / ORT_PERSIST_STATS).
set -e
NAME=$1; shift
cd "$(dirname "$0")/.."
BASE="-DORT_ANALYSIS=1 -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fno-slp-vectorize -fPIC -Wall -Wno-unused-parameter"
make -s lib OBJ=build/obj_$NAME LIB=build/ab/lib$NAME.so HIPFLAGS="$BASE $*" -j8
