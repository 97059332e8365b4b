// oracle/_ref recipe (test infrastructure only): exports the reference's own scalar
// fast-math helpers, compiled from the headers where they lie under /root/reference
// (include/utils/fastlog.h:75-85, include/utils/fastgamma.h:58-60).  Nothing from the
// reference is copied into this repository; the build writes only to oracle/_ref/.
#include "fastgamma.h"

extern "C" float ref_fasterlog(float x) { return fasterlog(x); }
extern "C" float ref_fasterlgamma(float x) { return fasterlgamma(x); }
