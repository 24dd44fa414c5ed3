#!/bin/bash
# Build librgpu.so with extra defines into abtest/librgpu_<tag>.so (A/B experiments; see ab_lib.sh).
#   tools/build_variant.sh <tag> [-DFOO ...]
set -e
cd "$(dirname "$0")/.."
tag=$1; shift
d=raphtory_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result "$@" -shared \
  -o "abtest/librgpu_$tag.so" $d/kernels.hip $d/xchg.hip $d/tslots.hip $d/check.hip $d/merge.hip $d/diffusion.hip $d/vp.hip $d/rgpu.cpp $d/packer.cpp \
  $d/exchange.cpp $d/rgev.cpp -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
