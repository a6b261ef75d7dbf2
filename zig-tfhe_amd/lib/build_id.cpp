extern "C" const char *tfhe_gpu_build_id(void) { return "9eb2c2abe875f7dc"; }
