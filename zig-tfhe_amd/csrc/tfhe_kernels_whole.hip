// tfhe_kernels_whole.hip — the default whole-form blind-rotation kernels
// (k_blind_rotate<L, true, true>: loader waves, slot counters, fused arithmetic)
// in their own compilation unit, built with hipcc's max-memory-clause machine
// scheduler (Makefile).  That scheduler groups the kernel's LDS operations into
// clauses: 6.37-6.41 vs 6.48-6.55 ms per 1,024 gates, alternating on two boxes,
// the same words (profiles/r03r_ab_sched_strategy.txt).  Applied to the whole
// library it cost the latency form 2 % (16-bit adder 101.5 vs 99.7 ms), hence
// the separate unit.
#include "tfhe_device.hpp"

namespace tfhe {

hipError_t launch_whole_default(int L, dim3 grid, dim3 block, hipStream_t s, const KParams &P, const DevTables &T,
                                const uint8_t *ops, const uint32_t *in_a, const uint32_t *in_b, const uint32_t *idx,
                                const uint32_t *testvec, const double2 *bk2, uint32_t *out, int out_mode, size_t B) {
    switch (L) {
    case 1: hipLaunchKernelGGL((k_blind_rotate<1, true, true>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec, bk2, out, out_mode, B); break;
    case 2: hipLaunchKernelGGL((k_blind_rotate<2, true, true>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec, bk2, out, out_mode, B); break;
    case 3: hipLaunchKernelGGL((k_blind_rotate<3, true, true>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec, bk2, out, out_mode, B); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace tfhe
