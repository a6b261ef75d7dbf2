extern "C" const char *tfhe_gpu_build_id(void) { return "fbb4a7979347ae33"; }
