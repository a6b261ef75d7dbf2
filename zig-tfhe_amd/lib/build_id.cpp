extern "C" const char *tfhe_gpu_build_id(void) { return "b797a328ef5233b6"; }
