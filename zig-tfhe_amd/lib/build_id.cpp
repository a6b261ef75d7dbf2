extern "C" const char *tfhe_gpu_build_id(void) { return "5b1f3d172f15b25d"; }
