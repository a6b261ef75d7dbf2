extern "C" const char *tfhe_gpu_build_id(void) { return "91c5540e9fe579c9"; }
