extern "C" const char *tfhe_gpu_build_id(void) { return "4e48b30123fddc13"; }
