extern "C" const char *tfhe_gpu_build_id(void) { return "f329aee4351f8cfd"; }
