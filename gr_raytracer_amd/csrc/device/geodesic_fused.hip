// geodesic_fused.hip — the light charts' trace kernels (integrate, shade, raymarch) built a
// second time with FMA contraction, for grt_set_arithmetic(1) (include/grt_api.h).
//
// The exact build (geodesic.hip, -ffp-contract=off) keeps the reference's separately
// rounded multiply and add everywhere, which is what makes its pixels bit-identical to the
// reference's; here the compiler may fuse a*b + c into one FMA (one rounding instead of
// two).  The algorithm, its operation order and every exact skip are the same code; only
// the rounding of the fused pairs differs, so pixels stay within the north-star 1e-4
// relative per channel of the reference on every robust pixel (tests/test_fused.py;
// DESIGN.md section 4), while the FP64 issue slots per step drop (C2 -17%, C3 -13%,
// profiles/r06c).  Kerr-Schild is not built here: its finite-difference metric turns the
// changed roundings into different step sequences on robust pixels of C4, so it always
// runs the exact kernels.
#define GRT_FUSED 1
#include "geodesic.hip"
