extern "C" const char *tfhe_gpu_build_id(void) { return "ff7ea4a196060eeb"; }
