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

// Fused out-of-place red/black sweeps of a 3D level (mgp_rbgs3d.hip): nh half-sweeps (2 or 4)
// per launch; needs nh ghost planes of u and f (zeros at a physical boundary).
// ty = tile height (8 or 16 rows of 64 cells).  With old != nullptr the launch also writes one fp64
// partial of sum (uout - old)^2 per workgroup to partials[0 .. fused3d_blocks()).
int fused3d_blocks(Geo g, int ty, int kc);
bool rbgs_fused3d_supported(int rb, int nh, int ty, Geo g);
hipError_t launch_rbgs_fused3d(int rb, bool fine, int nh, int ty, const void* uin, const void* f, void* uout,
                               const void* old, double* partials, Geo g, int kc, double h, double cl, hipStream_t s);
// LDS-tiled fused residual + 2x2x2 restriction of a 3D level (nx % 64 == 0, ny % 16 == 0, even nz).
bool residual_restrict3d_supported(Geo g);
hipError_t launch_residual_restrict3d(int rb, const void* u, const void* f, void* R, Geo g, double h, double cl,
                                      hipStream_t s);
// Vectorised 3D prolongation + correction (4 fine x-cells per thread; nx >= 4).
bool prolong3d_x4_supported(Geo g);
hipError_t launch_prolong3d_x4(int rb, int linear, void* u, const void* V, Geo g, Geo gc, double clc, hipStream_t s);
// Fixed-order fp64 sum of n partials into *out (one workgroup).
hipError_t launch_sum_partials(const double* partials, int n, double* out, hipStream_t s);

constexpr int kSumBlocks = 1024;
constexpr int kGhost3D = 4;  // ghost planes per side of every 3D level (= max nh)

}  // namespace mgp
