// mgp_internal.h — shared declarations between the C-ABI layer (mgp_api.cpp) and the CDNA4
// kernels (mgp_kernels.hip).  Not part of the public ABI (include/mgpoisson.h is).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace mgp {

constexpr int kGhost3D = 1;  // ghost planes per side of every 3D level
// ... when a slab-distributed level runs the temporally blocked phases (k_zs): PRE reads 5 planes
// of u and f beyond its slab, POST 4 of u and f and 3 coarse planes of V
constexpr int kGhostZs = 5;
constexpr int kZsHaloPre = 5, kZsHaloPost = 4, kZsHaloCoarse = 3;

// Device layout of one level ("red/black packed").  A level is a stack of planes (one plane in
// 2D).  Each plane holds its red cells ((i + j + gk) even) in the first half and its black cells
// in the second half; a half is ny rows of hw = max(1, nx/2) cells and cell (i, j) sits at
// m = i >> 1 of its row.  Every stencil neighbour of a cell has the other colour, at
// m - 1 + (i & 1) and m + (i & 1) for x-1 / x+1 and at m for y +- 1, z +- 1, so a half-sweep is a
// plain streaming stencil over one half reading the other half.  3D levels carry one ghost plane
// below and above (zeros at the physical boundary, the neighbour rank's plane across a slab
// edge); kernels receive pointers to interior plane 0.
struct Geo {
    int nx, ny;     // cells per row / rows per plane (powers of two)
    int lx, ly;     // log2(nx), log2(ny)
    int hw, lhw;    // cells per half row = max(1, nx / 2), log2(hw)
    int64_t nz;     // local planes (1 in 2D)
    int64_t H;      // cells per half plane = hw * ny
    int64_t P;      // plane stride = 2 H
    int64_t z0;     // global index of local plane 0
    int64_t gnz;    // global planes of this level (1 in 2D)
};

// Launchers enqueue on `s` and return the launch's hipGetLastError().  rb = sizeof(real),
// dim = 2 or 3.  `fine` selects the finest-level instantiation (a distinct symbol, so rocprofv3
// reports the finest smoother on its own line).
//
// The launchers of the per-piece cycle (half-sweep, residual + restriction, full weighting, prolongation +
// correction, err sum, the residual / errorBuf views and the residual norm) also take rb = kRealF32D:
// float buffers with every expression evaluated in double and rounded once at the store — cpu-raw.lua
// under real = 'float' (cpu-raw.lua:142-153: LuaJIT numbers are doubles; mgp_opts.arith =
// MGP_ARITH_DOUBLE).  Those run the scalar kernels templated on the compute type (C = double).
constexpr int kRealF32D = 12;

// f = -1e6 at global (cx, cy, cz), 0 elsewhere; u = -f (cpu.lua:180-193).
hipError_t launch_init_point_charge(int rb, int dim, void* u, void* f, Geo g, int64_t cx, int64_t cy,
                                    int64_t cz, hipStream_t s);
// lexicographic (x fastest, this rank's planes) <-> packed
hipError_t launch_pack(int rb, const void* lex, void* packed, Geo g, hipStream_t s);
hipError_t launch_unpack(int rb, const void* packed, void* lex, Geo g, hipStream_t s);
// Fingerprint of a packed field (this rank's planes): out_h = sum mod 2^64 of a per-cell mix of the
// bits and the global lexicographic index; out_d = {sum, sum of squares, max |x|} in fp64.
// hpart / dpart: kSumBlocks / 3 * kSumBlocks scratch.
hipError_t launch_field_stats(int rb, const void* packed, Geo g, uint64_t* hpart, double* dpart, uint64_t* out_h,
                              double* out_d, hipStream_t s);

// Computed views for mgp_get_field (cpu-raw.lua's rs / errorBuf): r = f - A u at every packed slot, and
// out = (a - b)^2 elementwise over n packed reals.
hipError_t launch_residual_field(int rb, int dim, const void* u, const void* f, void* r, Geo g, double h, double cl,
                                 hipStream_t s);
hipError_t launch_sqdiff_field(int rb, const void* a, const void* b, void* out, int64_t n, hipStream_t s);

// One colour of a red/black sweep: dst(colour c) = relax(other(1-c), f) (cpu.lua:40-54 update).
// other and dst may be the same buffer (in place) or different (out of place: Jacobi, the first
// sweep of a cycle).  With old != nullptr, sum (dst - old)^2 over colour c goes to one fp64
// partial per workgroup in partials[0 .. half_blocks()).
// gs: large levels use the grid-stride form (kGsBlocks workgroups, XCD-banded)
int half_blocks(int rb, Geo g, bool gs);
hipError_t launch_half_sweep(int rb, int dim, bool fine, int color, const void* other, const void* f, void* dst,
                             const void* old, double* partials, Geo g, double h, double cl, bool gs, hipStream_t s);
// The first red/black sweep of a fresh zero guess (cpu.lua:138) in one pass: u (both colours) from f
// alone, bit-identical to the red and black half-sweeps reading u = 0.  Levels with hw >= 16 / rb.
bool fresh_supported(int rb, const Geo& g);
// store_red = false: the red cells are left as they are (a later sweep's red half-sweep replaces them unread).
hipError_t launch_fresh_sweep(int rb, int dim, const void* f, void* u, Geo g, double h, double cl, hipStream_t s,
                              bool store_red = true);
// prolong_correct + the red half of the first post-smoothing sweep in one pass: red cells of u from black u
// + P V (never stored: the black half-sweep that follows replaces the black cells without reading
// them).  Vector levels of one rank's box with coarse nx >= 16 / rb.
bool post1_supported(int rb, const Geo& g, const Geo& gc);
hipError_t launch_post_first(int rb, int dim, int linear, void* u, const void* V, const void* f, Geo g, Geo gc,
                             double h, double cl, double clc, hipStream_t s);
// Fused residual + restriction (calcResidual + reduceResidual): R (coarse packed, pointing at the
// coarse plane of this rank's fine plane 0; its Geo is gc) from u, f of the fine level.
hipError_t launch_residual_restrict(int rb, int dim, const void* u, const void* f, void* R, Geo g, Geo gc, double h,
                                    double cl, hipStream_t s);
// The last black half-sweep of a red/black pre-smoothing + residual + restriction in one pass (k_bres): u's black
// cells relaxed in place from its (final) red cells and f, R as launch_residual_restrict would compute it from the
// swept u.  Bit-identical to launch_half_sweep(colour 1, in place) + launch_residual_restrict.  Real arithmetic
// (rb 4 / 8), a replicated level (planes -1 and nz are not read) with nx, ny (and nz) >= 2.
bool bres_supported(int rb, const Geo& g);
hipError_t launch_black_residual_restrict(int rb, int dim, void* u, const void* f, void* R, Geo g, Geo gc, double h,
                                          double cl, hipStream_t s);
// One whole red/black sweep in one pass (k_rbsweep): dst's black cells (and with store_red its red ones) = the sweep
// of src, read from src's black cells and f only (src != dst; same shapes as launch_black_residual_restrict).
// Bit-identical to the red and black launch_half_sweep pair.
hipError_t launch_rb_sweep(int rb, int dim, const void* src, const void* f, void* dst, Geo g, double h, double cl,
                           bool store_red, hipStream_t s);
// Full-weighting restriction (mgp_opts.restriction, build-defined): r = f - A u of the level's own planes
// into the scratch r (same packed layout and ghost planes as the level), then R (coarse packed, Geo gc)
// from r, which must have current planes -1 and g.nz (zero at the physical boundary, the neighbours'
// planes across a slab edge).  clc: the coarse level's boundary coefficient (face weight 3 - clc).
hipError_t launch_residual_field_v(int rb, int dim, const void* u, const void* f, void* r, Geo g, double h, double cl,
                                   hipStream_t s);
hipError_t launch_fw_restrict(int rb, int dim, const void* r, void* R, Geo g, Geo gc, double clc, hipStream_t s);
// calcResidual + the full weighting in one z-streamed pass from u and f (k_resfw, mgp_fw.hip): R of the coarse
// level (gc) bit-identical to launch_residual_field_v + launch_fw_restrict, without the level-sized residual.
// gz: readable ghost planes of u / f per side (a slab level needs u two and f one plane deep: resfw_supported).
bool resfw_supported(int rb, int dim, const Geo& g, int gz, bool dist);
hipError_t launch_resfw(int rb, int dim, const void* u, const void* f, void* R, Geo g, Geo gc, double h, double cl,
                        double clc, int gz, hipStream_t s);
// u += P V (expandResidual + addTo); V points at the coarse plane gc.z0, which must correspond to
// this rank's fine plane 0; planes -1 and gc.nz of V must be readable for the linear kind.
// black_only: the black cells only (before a red/black post-smoothing: its red half-sweep replaces
// every red cell without reading it).
hipError_t launch_prolong_correct(int rb, int dim, int linear, void* u, const void* V, Geo g, Geo gc, double clc,
                                  hipStream_t s, bool black_only = false);
// Deterministic two-pass fp64 sum of (a - b)^2 over n elements into *out (ctr != nullptr: into
// out[*ctr], then ++*ctr on the device).
hipError_t launch_sqdiff_sum(int rb, const void* a, const void* b, int64_t n, double* partials, double* out,
                             hipStream_t s, int* ctr = nullptr);
// out[0..2] = {sum |1 - psi/psiOld| over nonzero entries, their count, sum (psi - psiOld)^2}
// over n elements; partials needs 3 * kSumBlocks doubles.
// Debugging check (cpu-raw.lua:126-140, gpu.lua:269-284): *first = min(*first, id) if p[0, n) holds a NaN or inf.
hipError_t launch_nonfinite_check(int rb, const void* p, int64_t n, int id, int* first, hipStream_t s);
hipError_t launch_metrics(int rb, const void* psi, const void* old, int64_t n, double* partials, double* out,
                          hipStream_t s);
// out[0] = sum (f - A u)^2, out[1] = sum f^2 over the level's cells (fp64, wave-level then fixed-order
// reductions).  partials: 2 * (resnorm_blocks() + sum_scratch(resnorm_blocks())) doubles.
int resnorm_blocks(int rb, Geo g);
hipError_t launch_residual_norm(int rb, int dim, const void* u, const void* f, Geo g, double h, double cl,
                                double* partials, double* out, hipStream_t s);
// Fixed-order fp64 sum of n partials into *out.  Needs sum_scratch(n) doubles of scratch right
// after partials[n - 1].
int sum_scratch(int n);
hipError_t launch_sum_partials(const double* partials, int n, double* out, hipStream_t s, int* ctr = nullptr);

// Temporally blocked smoothing phases of a replicated 3D red/black level (ns = 2 sweeps):
//   pre : dst = nu1 sweeps of src; R (coarse packed, Geo gc) = restrict(residual(dst))
//   post: dst = nu2 sweeps of (src + P V); with partials, sum (dst - dst_before)^2 per workgroup
// src and dst are different buffers (tiles read each other's halos of src).
// Tile settings of the temporally blocked phases (k_zs / k_ys), read from the environment ONCE, when a context is
// created, and kept in it: the sizes planned then (z-chunks, the err partials buffer, mgp_plan's engines) are the
// ones every later launch uses (they used to be re-read per launch).
struct FusedTuning {
    bool wide = true;    // MGP_ZS_WIDE=0: POST on the narrow 64 x 32 tile
    int ys_half = -1;    // MGP_YS_HALF: 2D segment width rule (-1 auto, 0 full, 1 half)
    int ys_rows = 32;    // MGP_YS_ROWS: 2D rows per workgroup chunk
    int64_t wgs = 256;   // MGP_ZS_WGS: z-chunks are halved until a launch has this many workgroups
    // tile order of launches of > 512 workgroups: px | py << 8 patches of tiles per XCD band, 0 = tile rows
    // (MGP_ZS_PATCH=px,py sets both phases, MGP_ZS_PATCH_PRE / MGP_ZS_PATCH_POST one; "0" off; -1: POST's default,
    // 4 x 8 on planes of >= 4096 tiles)
    int patch_pre = 0, patch_post = -1;
    bool fwf = true;     // MGP_ZS_FWF=0: the full weighting after the fused PRE instead of inside it
    int post_zc = 256;   // MGP_ZS_POST_ZC: POST's z-chunks hold at most this many planes (0: no limit)
    bool stamp_r = false;  // MGP_STAMP_R=1 (ZS_STAMP timing builds only): POST's wall-clock stamps go to level l+1's f
};
FusedTuning fused_tuning_from_env();

// What a launcher actually launched: the kernel's symbol as rocprofv3 prints it (template arguments included)
// and its grid in work-items (rocprofv3's Grid_Size), so measured PMC traffic can be matched to this launch
// (bench.py) instead of being re-derived from the options.
struct LaunchInfo {
    char name[96];
    int64_t grid;
};

struct FusedArgs {
    FusedTuning tu;
    LaunchInfo* info;  // optional out: the launched kernel
    bool pre;
    int linear;  // POST: linear prolongation; PRE: 1 = no restriction (both colours stored, full weighting after),
                 // 2 = the full-weighting restriction fused (fused_fwf_supported)
    const void* src;
    const void* f;
    void* dst;
    const void* old;  // POST + err: psiOld (nullptr: dst, overwritten plane by plane as the output is stored)
    void* R;
    const void* V;
    double* partials;
    Geo g, gc;
    double h, cl, clc;
    int zc;
    int ghost;  // readable ghost planes per side of src / f / dst
};
bool fused_supported(int rb, int dim, int ns, const Geo& g, const FusedTuning& tu);
// Raise the dynamic-LDS limit of the fused and tail kernels (once per context, before any capture).
hipError_t prepare_kernels(int rb);
// clz: the level's operator has no boundary modification (cl == 0): PRE's tile may differ otherwise
int fused_zc(int rb, const Geo& g, bool pre, bool clz, const FusedTuning& tu);
int fused_blocks(int rb, const Geo& g, int zc, bool clz, const FusedTuning& tu);
hipError_t launch_fused(int rb, const FusedArgs& a, hipStream_t s);
// PRE with the full weighting fused (FusedArgs::linear = 2): fp32, cl = 0, a replicated level (MGP_ZS_FWF=0: off)
bool fused_fwf_supported(int rb, int dim, bool clz, bool dist, const FusedTuning& tu);

// Tiled smoothing phases of a small replicated red/black level (k_blk: one launch per phase, the 3D
// or 2D tile and its halo in LDS):
//   pre : dst = ns sweeps of src; R (coarse packed, Geo gc) = restrict(residual(dst))
//   post: dst = ns sweeps of (src + P V)
// src == nullptr reads u = 0 (a fresh coarse guess).  src != dst.
constexpr int kBlkMaxSweeps = 2;
constexpr int kBlkTile = 8;     // 3D owned tile edge (every axis of a tiled level is a multiple)
constexpr int kBlkTile2D = 32;  // 2D owned tile edge
struct BlockArgs {
    bool pre;
    int linear;  // POST: linear prolongation; PRE: 1 = full-weighting restriction (face weight 3 - clc)
    int ns;
    const void* src;
    const void* f;
    void* dst;
    void* R;
    const void* V;
    Geo g, gc;
    double h, cl, clc;
};
bool block_supported(int rb, int dim, int ns, const Geo& g);
hipError_t launch_block(int rb, int dim, const BlockArgs& a, hipStream_t s);

// PRE (POST) of two consecutive small 2D levels in one launch (mgp_blk2.hip): level l (g) smoothed and restricted, then
// level l + 1 (g1) smoothed from its guess and restricted onto level l + 2 (g2); POST: level l + 1 corrected from
// level l + 2 and smoothed, then level l corrected from it and smoothed
struct Block2Args {
    bool pre;          // false: POST of level l + 1 then of level l (k_blk2_post)
    int ns;
    int linear;        // POST: linear prolongation
    const void* src;   // level l's u (PRE: nullptr = a fresh zero guess)
    const void* f;
    void* dst;         // level l's smoothed u (PRE: black cells; POST: both colours)
    void* f1;          // level l + 1's f (PRE: written, both colours; POST: read)
    const void* src1;  // level l + 1's u (PRE: the warm guess, nullptr = a fresh zero guess)
    void* dst1;        // level l + 1's smoothed u
    void* R;           // level l + 2's f
    const void* V2;    // POST: level l + 2's u (the correction prolongated into level l + 1)
    Geo g, g1, g2;
    double h, cl, cl1, cl2;  // h of level l (level l + 1: 2 h); the coarse-boundary coefficients of levels l .. l + 2
};
bool block2_supported(int rb, int dim, int ns, const Geo& g, const Geo& g1, const Geo& g2);
hipError_t launch_block2(int rb, int dim, const Block2Args& a, hipStream_t s);
hipError_t blk2_attr(int rb);

// Coarse-level tail: the sub-cycle below one level as a single one-workgroup launch with every
// level in LDS.  ops[] = (op | level << 4 | arg << 8), levels relative to the tail's first level.
constexpr int kTailMaxLevels = 8;
constexpr int kTailMaxOps = 192;
constexpr size_t kTailMaxLds = 160 * 1024;  // gfx950 LDS per workgroup
enum TailOp { TAIL_SMOOTH = 1, TAIL_RR = 2, TAIL_ZERO = 3, TAIL_PROLONG = 4 };
struct TailSpec {
    int nlev, nops, jacobi, linear;
    int zero_first;  // the first level's u is logically 0 (a fresh guess): loaded as zeros
    int fw;          // TAIL_RR restricts by full weighting (mgp_opts.restriction)
    void* u[kTailMaxLevels];  // interior plane 0 of each level's u / f (global)
    void* f[kTailMaxLevels];
    Geo g[kTailMaxLevels];
    double h[kTailMaxLevels];
    double cl[kTailMaxLevels];
    uint32_t ops[kTailMaxOps];
};
size_t tail_lds_bytes(int rb, int dim, int jacobi, const Geo* g, int nlev);
hipError_t launch_tail(int rb, int dim, const TailSpec& t, hipStream_t s);

// Conjugate gradients on a level's operator (mgp_krylov.hip; converge-multigrid-vs-krylov.lua:38-69).
// Packed level vectors x (in/out), b, and scratch r, p, q; scratch holds cg_scratch_doubles() doubles.
struct CgArgs {
    Geo g;
    double h, cl;
    void *x, *r, *p, *q;
    const void* b;
    double* scratch;
    bool x0_neg_b;    // x0 = -b (the reference's start) instead of x's content
    int maxiter;
    double epsilon;   // stop when rSq / bSq < epsilon
    double* linf;     // optional: |x|_inf after each iteration (maxiter entries)
    int iters;        // out
    double err;       // out: final rSq / bSq
};
int cg_scratch_doubles();
hipError_t launch_cg(int rb, int dim, CgArgs& a, hipStream_t s);

// 16-byte streaming copy of `bytes` (a multiple of 16) for the copy-bandwidth probe; kind 0..2 (kCopyKinds):
// grid-stride / one pass / one pass non-temporal; kinds 3 and 4 (calibration only): 8- and 4-byte lanes
constexpr int kCopyKinds = 3, kCopyCalibKinds = 5;
hipError_t launch_copy16(int kind, const void* src, void* dst, int64_t bytes, hipStream_t s);

// One in-place lexicographic Gauss-Seidel sweep (cpu.lua:24-37) of a whole replicated level, bit-identical to the
// sequential ascending-order sweep: tiles in tile-hyperplane order, one launch per tile-hyperplane (k_gslex).
hipError_t launch_gslex_sweep(int rb, int dim, void* u, const void* f, Geo g, double h, double cl, hipStream_t s);

// Test hook of the communication deadline (MGP_TEST_STALL): one wave that holds stream s until *flag (host-pinned,
// mapped) is non-zero, and in any case at most max_s seconds of wall clock (every wave reaches that exit).
hipError_t launch_stall(const int* flag, double max_s, hipStream_t s);

constexpr int kSumBlocks = 1024;

}  // namespace mgp
