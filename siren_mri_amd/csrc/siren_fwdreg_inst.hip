// siren_fwdreg_inst.hip — the register-resident forward's kernels (siren_fwdreg.hip) as a
// translation unit of their own, compiled beside siren_runtime.hip (which declares them) and linked
// into libsiren_mri_amd.so: 20 instantiations of the largest kernel build in parallel with the rest.
#include "siren_fwdreg.hip"

namespace siren {

#define SIREN_FREG_INST(CC, OC)                                                        \
  template __global__ void fused_fwd_reg_kernel<CC, OC, 0>(FwdRegArgs);               \
  template __global__ void fused_fwd_reg_kernel<CC, OC, 1>(FwdRegArgs);
#ifndef SIREN_FREG_INST_OC
SIREN_FREG_INST(1, 0)
SIREN_FREG_INST(2, 0)
SIREN_FREG_INST(3, 0)
SIREN_FREG_INST(4, 0)
SIREN_FREG_INST(16, 0)
SIREN_FREG_INST(1, 1)
SIREN_FREG_INST(2, 1)
SIREN_FREG_INST(3, 1)
SIREN_FREG_INST(4, 1)
SIREN_FREG_INST(16, 1)
SIREN_FREG_INST(17, 0)
SIREN_FREG_INST(17, 1)
// the fused-loss forms (fract epilogue only): the coordinate fits (1..4 inputs, one output) and the
// hypernetwork's wide form (Fourier features, one or more outputs)
template __global__ void fused_fwd_reg_kernel<1, 1, 0, true>(FwdRegArgs);
template __global__ void fused_fwd_reg_kernel<2, 1, 0, true>(FwdRegArgs);
template __global__ void fused_fwd_reg_kernel<3, 1, 0, true>(FwdRegArgs);
template __global__ void fused_fwd_reg_kernel<4, 1, 0, true>(FwdRegArgs);
template __global__ void fused_fwd_reg_kernel<16, 0, 0, true>(FwdRegArgs);
template __global__ void fused_fwd_reg_kernel<16, 1, 0, true>(FwdRegArgs);
template __global__ void fused_fwd_reg_kernel<17, 0, 0, true>(FwdRegArgs);
template __global__ void fused_fwd_reg_kernel<17, 1, 0, true>(FwdRegArgs);
#endif
#undef SIREN_FREG_INST

}  // namespace siren
