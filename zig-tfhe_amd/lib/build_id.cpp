extern "C" const char *tfhe_gpu_build_id(void) { return "a40108a8a968a632"; }
