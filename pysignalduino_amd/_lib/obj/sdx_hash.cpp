extern "C" const char* sdx_source_hash(void) { return "0724b5b4aebf6e57"; }
