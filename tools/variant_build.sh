#!/bin/bash
# Build a compile-time variant of the library for A/B timing on the GPU box:
#   tools/variant_build.sh NAME "-DFLAG=1 ..."  ->  entropy_coders_amd/libfsehip_NAME.so
# (load it with FSEHIP_LIB=libfsehip_NAME.so).  Never the product.
set -e
NAME=$1; shift
cd "$(dirname "$0")/../entropy_coders_amd"
make -s -j8 BUILD=build_$NAME LIB=libfsehip_$NAME.so EXTRA="$*"
