extern "C" const char *tfhe_gpu_build_id(void) { return "b9b3cb35de6e928c"; }
