extern "C" const char *tfhe_gpu_build_id(void) { return "429fac9a75b08927"; }
