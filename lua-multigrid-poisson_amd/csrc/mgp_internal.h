// mgp_internal.h — shared declarations between the C-ABI layer (mgp_api.cpp) and the CDNA4
// kernels (mgp_kernels.hip).  Not part of the public ABI (include/mgpoisson.h is).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace mgp {

// Geometry of one level as seen by this rank.  Arrays are x fastest; a 3D level carries one
// ghost plane below and above its nz local planes (zeros at the physical boundary, the
// neighbour rank's plane on a slab boundary).  Kernels receive the INTERIOR pointer (plane 0).
struct Geo {
    int nx, ny;     // in-plane cells (powers of two)
    int lx, ly;     // log2(nx), log2(ny)
    int64_t nz;     // local planes (1 in 2D)
    int64_t plane;  // nx * ny
    int64_t z0;     // global index of local plane 0
    int64_t gnz;    // global planes of this level
};

// All launchers enqueue on `s` and return hipGetLastError() of the launch.
// rb = sizeof(real) (4 or 8), dim = 2 or 3.  `fine` selects the finest-level instantiation
// (a distinct symbol, so that rocprofv3 reports the finest smoother separately).
hipError_t launch_init_point_charge(int rb, int dim, void* u, void* f, Geo g, int64_t cx,
                                    int64_t cy, int64_t cz, hipStream_t s);
hipError_t launch_jacobi(int rb, int dim, bool fine, const void* u, const void* f, void* out,
                         Geo g, double h, double cl, hipStream_t s);
hipError_t launch_rb_half(int rb, int dim, bool fine, void* u, const void* f, Geo g, int color,
                          double h, double cl, hipStream_t s);
// R points at the coarse cell that corresponds to this rank's local fine plane 0.
hipError_t launch_residual_restrict(int rb, int dim, const void* u, const void* f, void* R, Geo g,
                                    double h, double cl, hipStream_t s);
// V points at the coarse interior plane that corresponds to global coarse index gc.z0; its
// planes -1 and gc.nz must be readable (ghosts / neighbours' planes) for the linear kind.
hipError_t launch_prolong_correct(int rb, int dim, int linear, void* u, const void* V, Geo g,
                                  Geo gc, double clc, hipStream_t s);
// Deterministic two-pass sum of (a - b)^2 in double into *out (overwrites).
hipError_t launch_sqdiff_sum(int rb, const void* a, const void* b, int64_t n, double* partials,
                             double* out, hipStream_t s);

constexpr int kSumBlocks = 1024;

}  // namespace mgp
