extern "C" const char *tfhe_gpu_build_id(void) { return "09fac45f4eb4400b"; }
