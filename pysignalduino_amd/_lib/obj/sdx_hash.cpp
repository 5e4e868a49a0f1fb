extern "C" const char* sdx_source_hash(void) { return "0c4dcfe1ddfcfa81"; }
