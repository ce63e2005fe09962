// sl_build_id(): the hash of the library's sources, headers and Makefile, compiled in
// at every link (the Makefile passes SL_BUILD_ID); bench.py matches committed PMC
// records against it.
#ifndef SL_BUILD_ID
#define SL_BUILD_ID "unknown"
#endif
extern "C" const char *sl_build_id(void) { return SL_BUILD_ID; }
