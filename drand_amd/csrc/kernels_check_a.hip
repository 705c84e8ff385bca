// Part 1 of Recover's pairing-check pipeline (checks.h), compiled in its own translation unit with every field
// product inlined and serialised (DG_FP_CALL=3) and the Fp12 routines inlined (DG_INLINE12=1): each kernel of the
// pipeline is short, so its formula fits the register file without calls or scratch.  The parts build in parallel.
#define DG_TU_CHECK 1
#define DG_FP_CALL 3
#define DG_INLINE12 1
#define DG_CYC_SQR 1
#define DG_FP2_ILV 1
#define DG_FP2_DIG 2  // Fp2 products in digit form, each operand unpacked once, two Montgomery reductions (field.h fp2_mul_dig2)
#define DG_SEQ_DIG 1  // ... and the serialised forms (subgroup checks, column loops, compressed squarings: -1% C5)
#include "kernels.h"
