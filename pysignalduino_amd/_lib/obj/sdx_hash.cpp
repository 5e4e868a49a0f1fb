extern "C" const char* sdx_source_hash(void) { return "50ccc9b81f9b3643"; }
