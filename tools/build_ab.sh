#!/bin/bash
# variant library for A/B runs: tools/build_ab.sh <tag> "<extra hipcc flags>" [files]
#   -> rs-bann_amd/ab/librsbann_amd_<tag>.so
# files (default: every .hip source) are compiled with the flags; the other objects are
# taken from the in-tree build (make -C rs-bann_amd/csrc first)
set -e
TAG=$1; FLAGS=$2; FILES=${3:-"bann_api bann_dist bann_residual bann_io_dev kernels_data kernels_gx kernels_fx kernels_wx kernels_update kernels_feed kernels_fi"}
R=$(cd "$(dirname "$0")/.." && pwd); C=$R/rs-bann_amd/csrc; O=/tmp/ab_$TAG; rm -rf $O; mkdir -p $O $R/rs-bann_amd/ab
for f in $FILES; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -munsafe-fp-atomics $FLAGS -c $C/$f.hip -o $O/$f.o 2>/dev/null &
done
wait
for f in bann_api bann_dist bann_residual bann_io_dev kernels_data kernels_gx kernels_fx kernels_wx kernels_update kernels_feed kernels_fi; do
  [ -f $O/$f.o ] || cp $C/$f.o $O/$f.o
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $R/rs-bann_amd/ab/librsbann_amd_$TAG.so $O/*.o $C/bann_net.o $C/bann_io.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built $R/rs-bann_amd/ab/librsbann_amd_$TAG.so
