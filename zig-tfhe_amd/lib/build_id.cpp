extern "C" const char *tfhe_gpu_build_id(void) { return "57925cd354d0f201"; }
