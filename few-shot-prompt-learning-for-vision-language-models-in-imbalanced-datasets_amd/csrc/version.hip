// Library identity: the version string and the digest of the sources it was built from
// (include/clipk.h clipk_source_digest; the Makefile generates ../build/clipk_digest.h from
// fsp_amd/_native.py source_digest, and the loader refuses a library whose digest differs from
// the tree it ships with).
#include "clipk_digest.h"
#include "../../include/clipk.h"

extern "C" const char* clipk_version(void) { return "clipk 0.2.0 gfx950"; }

extern "C" const char* clipk_source_digest(void) { return CLIPK_SOURCE_DIGEST; }
