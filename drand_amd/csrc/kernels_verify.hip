// The per-item pairing kernels (k_verify_items, k_verify_groups: kyber's bls.Verify of single shares and the
// group tests of Recover's examined prefix), compiled in their own translation unit with the Fp2/Fp6
// routines inlined into the out-of-line Fp12 / pairing routines (DG_FLAT=1).  In the library TU every Fp2
// and Fp6 product is a call whose operands are marshalled through the call ABI (moves, AGPR and scratch
// spills): about half of the instructions of a per-item pairing check.
#define DG_TU_VERIFY 1
#include "kernels.h"
