extern "C" const char *tfhe_gpu_build_id(void) { return "6f42bccc38c84f34"; }
