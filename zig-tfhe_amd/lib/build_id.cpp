extern "C" const char *tfhe_gpu_build_id(void) { return "401bf4ef5abd48e7"; }
