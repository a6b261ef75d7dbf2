extern "C" const char *tfhe_gpu_build_id(void) { return "75924c6b6990778d"; }
