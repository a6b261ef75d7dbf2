extern "C" const char *tfhe_gpu_build_id(void) { return "9b5b5487d60d1094"; }
