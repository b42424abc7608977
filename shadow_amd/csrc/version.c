/* shdr_version(): the library's identity. SHDR_SRC_SHA is the first 16 hex digits
 * of the SHA-256 of every source the library is built from (routes.hip,
 * topology.cpp, graph.cpp, ...: the list is LIB_SRCS in shadow_amd/Makefile and
 * LIB_SOURCES in shadow_amd/routes.py), so a number measured with this library
 * names the exact kernel AND host code it ran (bench.py lib_sha). */
#include "../../include/shdr.h"

#ifndef SHDR_SRC_SHA
#define SHDR_SRC_SHA "unknown"
#endif

const char* shdr_version(void) { return "shadow-amd routes 0.3 (gfx950) kernel " SHDR_SRC_SHA; }
