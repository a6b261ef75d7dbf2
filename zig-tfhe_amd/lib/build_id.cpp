extern "C" const char *tfhe_gpu_build_id(void) { return "8f9a288a25ac410a"; }
