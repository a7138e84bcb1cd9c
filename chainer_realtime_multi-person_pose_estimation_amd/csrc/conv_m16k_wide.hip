// conv_m16k_bf16x3<false, 3, 6> (the 92- and 46-wide 3x3 layers, 4 x 48 tiles: 20 % of the step)
// in its own translation unit, built with the Makefile's FLAGS_conv_m16k_wide: LLVM's iterative-ilp
// scheduler runs it 0.6-2 % faster per launch (two boxes), while the 8 x 32 instantiations in
// conv_big.hip lose with it (profiles/r02/ab_r02ai_3x3_sched_per_kernel.log).
#include "conv_big.hpp"
#include "conv_m16k.hpp"

namespace op {

int launch_m16k_wide(dim3 grid, int lds, hipStream_t st, const SplitConvShape& s, const SplitConvGroup& g0,
                     const SplitConvGroup& g1, const BigTiling& tl) {
  static bool attr = false;
  if (!attr) {
    OP_HIP_CHECK(hipFuncSetAttribute((const void*)conv_m16k_bf16x3<false, 3, 6>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024));
    attr = true;
  }
  hipLaunchKernelGGL((conv_m16k_bf16x3<false, 3, 6>), grid, dim3(256), lds, st, s, g0, g1, tl);
  return OP_OK;
}

}  // namespace op
