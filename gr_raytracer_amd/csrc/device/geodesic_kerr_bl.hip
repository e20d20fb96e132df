// geodesic_kerr_bl.hip — the exact KerrBL trace kernels (integrate, shade, raymarch),
// compiled apart from geodesic.hip with the machine-level loop-invariant code motion off
// (-mllvm -disable-machine-licm, Makefile).  Same source, same arithmetic and operation
// order (-ffp-contract=off as in the exact build), so every pixel is bit-identical; what
// changes is register allocation: with the motion on, the compiler hoists the 64-bit
// polynomial constants of the glibc restatements and of atan2 out of the sample and step
// loops into ~100 VGPRs, and the 3-wave KerrBL integrate kernel spilled 22 VGPRs to
// scratch.  Without it: no spills, C3 162-170 against 165-173 ms, the KerrBL raymarch
// 1,391-1,416 against 1,484-1,561 ms (profiles/r06p).  The Schwarzschild kernel is 1.4%
// slower built this way (its constants are then rematerialised in the step loop), so it
// stays in geodesic.hip.
#define GRT_KERR_BL_TU 1
#include "geodesic.hip"
