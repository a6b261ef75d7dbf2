extern "C" const char *tfhe_gpu_build_id(void) { return "1ad45ef93f0c22b2"; }
