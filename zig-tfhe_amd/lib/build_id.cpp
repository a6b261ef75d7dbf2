extern "C" const char *tfhe_gpu_build_id(void) { return "94fc3d60340ab112"; }
