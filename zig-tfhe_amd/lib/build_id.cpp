extern "C" const char *tfhe_gpu_build_id(void) { return "bd07b1dca5d094c5"; }
