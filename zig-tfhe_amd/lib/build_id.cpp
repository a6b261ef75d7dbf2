extern "C" const char *tfhe_gpu_build_id(void) { return "af1aa8960787e960"; }
