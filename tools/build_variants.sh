#!/bin/bash
# Build timing variants of the library in parallel: tools/build_variants.sh NAME=FLAGS ...
#   e.g. tools/build_variants.sh d1=-DSIREN_FREG_DBG=1 d7=-DSIREN_FREG_DBG=7
# -> siren_mri_amd/libsiren_mri_amd_NAME.so (load with SIREN_MRI_AMD_LIB=...); every translation
# unit of __graft_entry__.TUS, each with the variant's flags
set -e
cd "$(dirname "$0")/.."
pids=()
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  python -c "import sys, __graft_entry__ as g; g.build(extra_flags=sys.argv[2].split(), lib=sys.argv[1])" \
    "$(pwd)/siren_mri_amd/libsiren_mri_amd_$name.so" "$flags" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
