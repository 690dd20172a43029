#!/bin/bash
# Backward pair-kernel times of each library variant: tools/pair_variants.sh name1 name2 ...
for n in "$@"; do
  if [ "$n" = base ]; then lib=$PWD/siren_mri_amd/libsiren_mri_amd.so; else lib=$PWD/siren_mri_amd/libsiren_mri_amd_$n.so; fi
  printf "%s: " "$n"
  SIREN_MRI_AMD_LIB=$lib timeout -k 10 100 python -u tools/pair_roles.py --roles 3 2>/dev/null | tail -1 || exit 1
done
