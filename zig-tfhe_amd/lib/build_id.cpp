extern "C" const char *tfhe_gpu_build_id(void) { return "3176deede320ec19"; }
