extern "C" const char *tfhe_gpu_build_id(void) { return "029107cca9f90f89"; }
