// ba_cluster.hip — the window-BA cluster route's persistent kernel (ph_cluster_kernel, ba_phases.inc) and its
// host launch in a translation unit of their own, so that this kernel alone is compiled without machine-level
// loop-invariant hoisting (Makefile CLFLAGS): hoisted f64 constants and per-thread addresses otherwise stay
// live across its persistent loops and spill to scratch, while the phase kernels (ph_prep) lose time without
// the hoisting.  Everything else of ba_kernel.hip is compiled out here (VIO_BA_CLUSTER_TU).
#define VIO_BA_CLUSTER_TU 1
#include "ba_kernel.hip"
