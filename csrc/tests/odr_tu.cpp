// ODR / multiple-definition check for the shared native headers
// (tools/odr_check.py): this file is compiled twice, as two translation
// units with different ODR_TU values, and the two objects are linked into
// one program.  A non-inline function or variable defined in a header shows
// up as a "multiple definition" link error.
#include "../hash/hash_core.h"
#include "../hash/sha256_mb.h"
#include "../hash/sha1_mb.h"
#include "../hash/sha_ni.h"
#include "../relay/relay_core.h"
#include "../relay/stream.h"
#include "../utp/utp_engine.h"
#include "../btwire/btwire_core.h"

#if ODR_TU == 1
int odr_tu_two();
int main() { return odr_tu_two(); }
#else
int odr_tu_two() { return 0; }
#endif
