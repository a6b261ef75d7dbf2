extern "C" const char *tfhe_gpu_build_id(void) { return "8f1f211af6f4c756"; }
