extern "C" const char *tfhe_gpu_build_id(void) { return "7c526deca9178542"; }
