#!/bin/bash
# Build timing variants of the library in parallel: tools/build_variants.sh NAME=FLAGS ...
#   e.g. tools/build_variants.sh d1=-DSIREN_FREG_DBG=1 d7=-DSIREN_FREG_DBG=7
# -> siren_mri_amd/libsiren_mri_amd_NAME.so (load with SIREN_MRI_AMD_LIB=...)
set -e
cd "$(dirname "$0")/../siren_mri_amd/csrc"
pids=()
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared $flags -o ../libsiren_mri_amd_$name.so siren_runtime.hip &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
