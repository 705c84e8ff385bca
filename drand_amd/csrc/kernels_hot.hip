// The throughput-bound kernels of the verify path (hash-to-G2, signature decode + subgroup check),
// compiled in their own translation unit with the mid-level field/curve routines inlined (DG_FLAT=1):
// ~1.5x faster G2 doubling chains than the out-of-line build, at a compile cost the rest of the library
// does not pay (DESIGN.md §code generation).  Launched from drand_gpu.hip through their declarations.
#define DG_TU_HOT 1
#define DG_SEQ_DIG 1  // serialised Fp2 products in digit form (field.h fp2_mul_dig; k_rs_sac -5% measured)
#include "kernels.h"
