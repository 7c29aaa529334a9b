#!/bin/bash
# build the committed (HEAD) library as rs-bann_amd/abl/librsbann_amd_abl0.so for an A/B
# against the working tree (tools/gpu_ab.sh / gpu_abwx.sh with VARIANTS=0); CPU only
set -e
cd "$(dirname "$0")/.."
git stash -q
trap 'git stash pop -q' EXIT
make -C rs-bann_amd/csrc -j8 >/dev/null
mkdir -p rs-bann_amd/abl
cp rs-bann_amd/librsbann_amd.so rs-bann_amd/abl/librsbann_amd_abl0.so
