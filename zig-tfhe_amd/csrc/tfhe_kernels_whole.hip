// The default whole-form blind-rotation kernels, compiled in their own unit
// with the max-memory-clause machine scheduler (Makefile; see
// launch_whole_default in tfhe_kernels.hip).
#define TFHE_WHOLE_TU
#include "tfhe_kernels.hip"
