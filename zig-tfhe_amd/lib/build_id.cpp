extern "C" const char *tfhe_gpu_build_id(void) { return "69aa5d53b89e97a8"; }
