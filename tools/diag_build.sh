#!/bin/bash
# Build diagnostic variants of libsurfhip.so (kernel sections compiled out via
# SURF_DIAG_* macros) into cuda-surf_amd/diag/<name>/; select one at run time
# with SURFHIP_LIB_DIR=cuda-surf_amd/diag/<name>.
#   bash tools/diag_build.sh NAME:FLAG[,FLAG] ...     e.g. nored:SURF_DIAG_NORED
set -eu
cd "$(dirname "$0")/../cuda-surf_amd"
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -I../include -Icsrc -mllvm -amdgpu-atomic-optimizer-strategy=None"
make -s build/surfhip_api.o build/surfhip_match.o build/surfhip_double.o build/surfhip_stream.o
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  D=""; IFS=, read -ra FL <<< "$flags"; for f in "${FL[@]}"; do [ -n "$f" ] && D="$D -D$f"; done
  mkdir -p diag/$name
  $H $D -c csrc/surfhip_kernels.hip -o diag/$name/k.o &
done
wait
for spec in "$@"; do
  name=${spec%%:*}
  $H -shared -fPIC -o diag/$name/libsurfhip.so diag/$name/k.o build/surfhip_api.o build/surfhip_match.o build/surfhip_double.o build/surfhip_stream.o
  rm -f diag/$name/k.o
done
echo built "$@"
