extern "C" const char *tfhe_gpu_build_id(void) { return "e2b3a4ec3adbd578"; }
