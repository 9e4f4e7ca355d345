/*
 * mgpoisson.h — C ABI of libmgpoisson.so, the MI355X (gfx950) multigrid Poisson hot path.
 *
 * This is the drop-in boundary for the reference's solver classes.  The reference has no
 * native FFI (it is Lua): its boundary is the Lua class protocol of cpu.lua / cpu-raw.lua /
 * gpu.lua.  Each entry point below names the reference interface it replaces;
 * the Lua-side binding (LuaJIT ffi.cdef of this header) is in INTEGRATION.md and
 * lua-multigrid-poisson_amd/lua/multigrid-poisson/hip.lua, the Python mirror in
 * lua-multigrid-poisson_amd/mgpoisson/.
 *
 * Conventions
 *  - Every function returning int returns MGP_OK (0) or a negative mgp_status; the message is
 *    in mgp_last_error(ctx) (or mgp_last_error(NULL) when mgp_create itself failed).  No C++
 *    exception or longjmp crosses this ABI.
 *  - A context owns one HIP stream and all device memory; it is not thread-safe.  Calls are
 *    synchronous at return except where stated.  Host buffers are borrowed for the call.
 *  - Layout is the reference's: x fastest, index = i + nx*(j + ny*k) (cpu-raw.lua:9, gpu.lua:72),
 *    0-based, real = float or double (gpu.lua:32).  With world > 1 a rank owns the z-slab
 *    [z0, z0 + nz_local) of every distributed level (mgp_level_info).
 */
#ifndef MGPOISSON_H
#define MGPOISSON_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MGP_API_VERSION 3  /* 2: mgp_opts.restriction; 3: mgp_opts.arith and .api_version appended (232 bytes) */
#define MGP_COMM_ID_BYTES 128 /* == NCCL_UNIQUE_ID_BYTES */

typedef enum mgp_status {
    MGP_OK = 0,
    MGP_ERR_ARG = -1,   /* invalid argument / unsupported configuration */
    MGP_ERR_HIP = -2,   /* HIP runtime error (no device, launch failure, ...) */
    MGP_ERR_RCCL = -3,  /* RCCL error (communicator init, send/recv, collective) */
    MGP_ERR_OOM = -4,   /* device allocation failed */
    MGP_ERR_STATE = -5  /* call not valid in the context's current state */
} mgp_status;

/* cpu.lua:56-57 inPlaceIterativeSolver: Jacobi (cpu.lua:40-54), red/black GS (build-defined, the temporally blocked
 * engines), lexicographic in-place GS (cpu.lua:24-37 GaussSeidel, bit-identical hyperplane-ordered sweeps; one
 * rank's whole box; with MGP_ARITH_DOUBLE cpu-raw.lua:22-32's GaussSeidel over float images) */
enum { MGP_JACOBI = 0, MGP_RBGS = 1, MGP_GS_LEX = 2 };
enum { MGP_CYCLE_V = 0, MGP_CYCLE_F = 1 };             /* twoGrid recursion (gamma 1) / F-cycle */
enum { MGP_PROLONG_PC = 0, MGP_PROLONG_LINEAR = 1 };   /* cpu.lua:142-150 injection / (tri)linear */
enum { MGP_COARSE_FRESH = 0, MGP_COARSE_WARM = 1 };    /* cpu.lua:138 zeros / cpu-raw.lua:221 Vs */
enum { MGP_BC_ZERO = 0, MGP_BC_CONSISTENT = 1 };       /* coarse ghost: 0 (ref) / extrapolated */
/* restriction: the 2^dim cell average of cpu.lua:127-135 (reduceResidual) or the cell-centred full
 * weighting (north_star "full-weighting restriction"): the adjoint of the linear prolongation, per axis
 * (1, 3, 3, 1) / 8 over fine cells 2I-1 .. 2I+2, face weight (3 - c) next to the box boundary */
enum { MGP_RESTRICT_AVERAGE = 0, MGP_RESTRICT_FULL_WEIGHTING = 1 };
/* arith: the arithmetic of real = float (no effect on double).  The reference's two float paths disagree:
 *   MGP_ARITH_REAL   every operation rounded to float, gpu.lua's OpenCL `real` (gpu.lua:32) — the default,
 *                    and the arithmetic of the north-star configurations
 *   MGP_ARITH_DOUBLE float buffers, every expression evaluated in double and rounded once where the
 *                    reference stores into a buffer: cpu-raw.lua under real = 'float' (cpu-raw.lua:142-153,
 *                    LuaJIT numbers are doubles; Jacobi :34-44, calcResidual :46-57, reduceResidual :59-63,
 *                    addTo :83-85), err from the float errorBuf (calcFrobErr :96-100, summed in double
 *                    :249-254).  Every level then runs one launch per piece (no fused / tiled / tail engines). */
enum { MGP_ARITH_REAL = 0, MGP_ARITH_DOUBLE = 1 };
/* Fields of a level, by cpu-raw.lua's names (cpu-raw.lua:148-171).  U and F are the stored, writable
 * state; the others are read-only views computed on request from it:
 *   MGP_FIELD_U          psi on level 0, Vs[L] below (the coarse correction)
 *   MGP_FIELD_F          f on level 0, Rs[L] below (the restricted residual)
 *   MGP_FIELD_RESIDUAL   rs[L] = f - A u (calcResidual, cpu.lua:108-123)
 *   MGP_FIELD_CORRECTION vs[L] = P Vs[L/2] (expandResidual, cpu.lua:142-150), the prolonged correction
 *   MGP_FIELD_PSI_OLD    psiOld (level 0): the iterate before the last outer iteration (cpu.lua:200)
 *   MGP_FIELD_ERROR      errorBuf (level 0) = (psi - psiOld)^2 per cell (calcFrobErr, gpu.lua:189-200)
 *   MGP_FIELD_TMP        tmpU: the Jacobi target buffer (cpu-raw.lua:153, 176-184)
 * PSI_OLD / ERROR need err_mode 1 (MGP_ERR_STATE otherwise; a temporally blocked finest level keeps psiOld
 * in a buffer of its own, unless the environment sets MGP_KEEP_PSI_OLD=0).  TMP: MGP_ERR_STATE when the
 * level has no second buffer (red/black Gauss-Seidel works in place). */
enum { MGP_FIELD_U = 0, MGP_FIELD_F = 1, MGP_FIELD_RESIDUAL = 2, MGP_FIELD_CORRECTION = 3, MGP_FIELD_PSI_OLD = 4,
       MGP_FIELD_ERROR = 5, MGP_FIELD_TMP = 6, MGP_FIELD_KINDS = 7 };
enum { MGP_MEM_HOST = 0, MGP_MEM_DEVICE = 1 };         /* where a caller buffer lives */

typedef struct mgp_opts {
    int32_t struct_size;   /* sizeof(mgp_opts), checked by mgp_create */
    int32_t dim;           /* 2 or 3 */
    int64_t n[3];          /* GLOBAL cells per axis, powers of two (n[2] = 1 in 2D) */
    int32_t real_bytes;    /* 4 = float, 8 = double (gpu.lua:32 "real") */
    int32_t nu1, nu2;      /* pre/post sweeps (cpu.lua:20 smooth = 7) */
    int32_t smoother;      /* MGP_JACOBI | MGP_RBGS | MGP_GS_LEX */
    int32_t cycle;         /* MGP_CYCLE_V | MGP_CYCLE_F */
    int32_t prolong;       /* MGP_PROLONG_PC | MGP_PROLONG_LINEAR */
    int32_t coarse_init;   /* MGP_COARSE_FRESH | MGP_COARSE_WARM */
    int32_t coarse_bc;     /* MGP_BC_ZERO | MGP_BC_CONSISTENT */
    int32_t coarse_sweeps; /* sweeps on a coarsest level with more than one cell */
    int32_t err_mode;      /* 1: psiOld snapshot + RMS update per cycle (cpu.lua:200-203); 0: off */
    int32_t device;        /* HIP device ordinal; -1 = current device */
    int32_t rank, world;   /* slab-z domain decomposition over `world` GPUs (3D only) */
    int32_t restriction;   /* MGP_RESTRICT_AVERAGE (reference) | MGP_RESTRICT_FULL_WEIGHTING */
    int64_t gather_cells;  /* a level with <= this many cells is replicated on every rank */
    uint8_t comm_id[MGP_COMM_ID_BYTES]; /* from mgp_comm_unique_id() on rank 0 (world > 1) */
    int32_t arith;         /* MGP_ARITH_REAL (gpu.lua) | MGP_ARITH_DOUBLE (cpu-raw.lua's real = 'float') */
    int32_t api_version;   /* MGP_API_VERSION of the header the caller was built with (mgp_opts_default sets it) */
} mgp_opts;
/* The layout is part of the ABI (LuaJIT cdef, ctypes mirror): a change must bump MGP_API_VERSION and append
 * fields, so that struct_size changes with it.  mgp_create rejects a struct_size or api_version that is not
 * this library's: fill the struct with the library's own mgp_opts_default before setting fields. */
#ifdef __cplusplus
static_assert(sizeof(mgp_opts) == 232, "mgp_opts layout changed");
#else
_Static_assert(sizeof(mgp_opts) == 232, "mgp_opts layout changed");
#endif

typedef struct mgp_ctx mgp_ctx;

int         mgp_version(void);
/* Defaults = the reference cpu.lua configuration: 2D, double, Jacobi 7+7, V, PC, fresh, zero. */
void        mgp_opts_default(mgp_opts* o);
/* RCCL unique id for a world > 1 context (call on rank 0, broadcast the bytes).  With the environment variable
 * MGP_TRANSPORT=rccl when it is created, a world-1 context (or a one-device group) takes the multi-GPU code
 * path on a one-rank RCCL communicator of its own (3D: its levels are "distributed" slabs without neighbours),
 * so that every RCCL call of a cycle executes on a one-GPU machine; results equal the plain world-1 run.
 * A context on its own RCCL communicator (one process per GPU, or MGP_TRANSPORT=rccl) waits for its streams under
 * a deadline, MGP_COMM_TIMEOUT_S seconds at creation (default 600, 0 = block): when it expires the call prints and
 * returns MGP_ERR_RCCL naming the rank and the first exchange / collective that has not completed (its level and
 * stream), after ncclCommAbort of the context's communicators; the context then refuses every exchange (destroy
 * it).  MGP_TEST_STALL=k (tests): the context's k-th halo exchange first holds its stream like an absent peer. */
int         mgp_comm_unique_id(void* out, int64_t nbytes);

/* Replaces MultigridCPU:init{size,...} (cpu.lua:173-194) / MultigridCPURaw:init(size, real)
 * (cpu-raw.lua:142-174) / MultigridGPU:init (gpu.lua:26-245): allocates the level hierarchy. */
int         mgp_create(mgp_ctx** out, const mgp_opts* o);
void        mgp_destroy(mgp_ctx* c);
const char* mgp_last_error(const mgp_ctx* c);

/* Level hierarchy.  info[0..7] = {nx, ny, nz_global, nz_local, z0, distributed, engine, exchanges}; engine =
 * how a cycle runs the level's smoothing phases: 0 one launch per piece, 1 inside the single-launch coarse
 * tail (LDS-resident levels), 2 temporally blocked z-streamed phases, 3 3D-tiled one-launch phases, 4 PRE one
 * launch per piece and POST temporally blocked; exchanges =
 * halo exchanges (grouped send/recv with the z-neighbours) of this level so far on this rank. */
int         mgp_num_levels(const mgp_ctx* c);
int         mgp_level_info(const mgp_ctx* c, int level, int64_t info[8]);
/* The same plan without a device (host logic only): fills up to max_levels rows of 8 int64s. */
int         mgp_plan(const mgp_opts* o, int64_t* rows, int max_levels);

/* f = -1e6 at 0-based (n/2, n/2[, n/2]), psi = -f (cpu.lua:180-193, cpu-raw.lua:8-20, gpu.lua:41-59). */
int         mgp_init_point_charge(mgp_ctx* c);
/* Copy a level's field in/out (this rank's slab on distributed levels; count in elements).
 * Replaces direct access to mg.psi / mg.f (cpu.lua) and .psi.buffer / .f.buffer (cpu-raw.lua). */
int         mgp_set_field(mgp_ctx* c, int level, int which, const void* src, int64_t count, int mem);
int         mgp_get_field(const mgp_ctx* c, int level, int which, void* dst, int64_t count, int mem);

/* Plane ranges of a level's field: local planes [z_begin, z_begin + nz) of this rank's slab, nz * ny * nx
 * reals, x fastest.  Host transfers stream through a bounded staging buffer (~256 MiB), so fields
 * far larger than host-convenient (a 4096 x 4096 x 512 fp32 slab is 34 GB) can be read piecewise. */
int         mgp_set_planes(mgp_ctx* c, int level, int which, int64_t z_begin, int64_t nz, const void* src, int mem);
int         mgp_get_planes(const mgp_ctx* c, int level, int which, int64_t z_begin, int64_t nz, void* dst, int mem);
/* Device-side fingerprint of this rank's part of a field, for comparing runs that cannot come to the
 * host: *hash = sum mod 2^64 over cells of mix64(bits(x) ^ mix64(global lexicographic index)) (order-
 * and decomposition-independent: the ranks' hashes add up to the global one, and two fields hash
 * equal when they are bit-identical), stats = {sum x, sum x^2, max |x|} in fp64. */
int         mgp_field_stats(const mgp_ctx* c, int level, int which, uint64_t* hash, double stats[3]);

/* One outer iteration = MultigridCPU:step() (cpu.lua:196-206): psiOld = psi; one V/F-cycle from
 * the finest level with h = 1/n; *err_out = sqrt(sum (psi - psiOld)^2 / N) (NaN if err_mode 0). */
int         mgp_cycle(mgp_ctx* c, double* err_out);
/* k outer iterations back to back with one host synchronisation at the end (the loop of
 * MultigridCPURaw:run, cpu-raw.lua:245, without early exit); errs[k] may be NULL. */
int         mgp_cycles(mgp_ctx* c, int32_t k, double* errs);

/* MultigridCPURaw:twoGrid(h, u, f, L) (cpu-raw.lua:186; gpu.lua:296): one cycle from the level of
 * size L with spacing h on caller buffers of L^dim reals (mem = MGP_MEM_HOST | MGP_MEM_DEVICE);
 * u is updated in place, f is read only.  Single-GPU contexts only. */
int         mgp_two_grid(mgp_ctx* c, double h, void* u, const void* f, int64_t L, int mem);

/* Level-granular pieces of twoGrid (cpu-raw.lua:198-236), for hybrid hand-off (cpu-gpu.lua:17-52)
 * and kernel-level tests.  h of level l is 2^l / n[0]. */
int         mgp_smooth(mgp_ctx* c, int level, int sweeps);          /* inPlaceIterativeSolver x sweeps */
int         mgp_residual_restrict(mgp_ctx* c, int level);           /* calcResidual + reduceResidual -> f of level+1 */
int         mgp_prolong_correct(mgp_ctx* c, int level);             /* expandResidual + addTo from level+1 */
int         mgp_coarse_solve(mgp_ctx* c);                           /* L == 1 branch of twoGrid */

int         mgp_sync(mgp_ctx* c);

/* Coarse-engine switch, the MI355X form of cpu-gpu.lua's cpuDepth (cpu-gpu.lua:61): the levels of
 * nx <= size run as ONE launch of the LDS-resident coarse engine (levels of <= 4096 cells by
 * default).  size 0 turns the engine off.  MGP_ERR_ARG if that sub-hierarchy does not fit one
 * workgroup's LDS. */
int         mgp_set_coarse_level(mgp_ctx* c, int64_t size);
/* Hybrid hand-off (cpu-gpu.lua:17-52).  When the cycle reaches the level of nx = size it copies
 * that level's u and f to host buffers (lexicographic, size^dim reals), calls fn(user, h, u, f,
 * size), which runs the coarse cycle in place on u (e.g. the reference's MultigridCPURaw:twoGrid),
 * and copies u and f back.  fn returns 0 on success.  fn == NULL removes the hand-off.  Replicated
 * levels >= 1 only; hipGraph replay is off while a hand-off is set. */
typedef int (*mgp_coarse_fn)(void* user, double h, void* u, const void* f, int64_t size);
int         mgp_set_coarse_handoff(mgp_ctx* c, int64_t size, mgp_coarse_fn fn, void* user);

/* The reference's convergence metrics of the last outer iteration, on the device
 * (gpu.lua:173-200 calcRelErr / calcFrobErr, test-gpu-obj.lua:216-247 relErr / count / frobErr):
 * rel_err = mean of |1 - psi/psiOld| over the cells where it is nonzero, count = their number,
 * frob = sqrt(sum (psi - psiOld)^2 / N).  Needs err_mode 1. */
int         mgp_metrics(mgp_ctx* c, double* rel_err, int64_t* count, double* frob);

/* Residual norm of a level (north star: "wavefront-level reductions for the residual norm"):
 * *rnorm = ||f - A u||_2 with the level's operator (calcResidual, cpu.lua:108-123, never materialised),
 * *fnorm = ||f||_2; squares summed in fp64 per wave (butterfly), per workgroup and then in a fixed
 * order, all-reduced over the ranks on a distributed level.  Level 0 after a cycle gives the
 * converged relative residual ||r|| / ||f||. */
int         mgp_residual_norm(mgp_ctx* c, int level, double* rnorm, double* fnorm);

/* The reference's Krylov cross-check (test/converge-multigrid-vs-krylov.lua:38-69, solver.conjgrad) on
 * the device, as an independent second oracle for the converged multigrid answer: matrix-free
 * conjugate gradients on the finest level's operator (same 5-/7-point stencil, ghost 0) from
 * x0 = -f with b = f, fp64 dot products, stopping when rSq / bSq < epsilon or after maxiter
 * iterations.  The solution goes to x_out (level-0 cells, x fastest; may be NULL); linf_hist (maxiter
 * doubles, may be NULL) gets |x|_inf after every iteration, the quantity the reference plots.  The
 * solver's own psi / f are not changed.  Single-GPU contexts only. */
int         mgp_cg_solve(mgp_ctx* c, double epsilon, int32_t maxiter, void* x_out, int mem, int32_t* iters,
                         double* err, double* linf_hist);

/* Loopback transport (tests only): the `world` ranks of a slab decomposition as contexts of ONE
 * process on one GPU, each driven by its own host thread.  Halo exchanges, the all-gather and the
 * err all-reduce become device copies ordered by events and a host barrier instead of RCCL calls;
 * everything else runs the multi-GPU code path unchanged.  A rank that stops calling makes the
 * others fail with MGP_ERR_STATE after 120 s instead of hanging. */
typedef struct mgp_loopback mgp_loopback;
int         mgp_loopback_create(mgp_loopback** out, int world);
void        mgp_loopback_destroy(mgp_loopback* lb);
int         mgp_create_loopback(mgp_ctx** out, const mgp_opts* o, mgp_loopback* lb);
/* Single-process multi-GPU group (the form of cpu-gpu.lua:55-72's one host object
 * owning several engines): ONE host process drives `ngpu` GPUs of the node.  The library creates
 * the RCCL communicators with ncclCommInitAll over devices[0..ngpu) (NULL = 0..ngpu-1) and one
 * context per rank (rank r = z-slab r of the box, opts->rank / opts->world / opts->device are set
 * by the group); every group call runs the ranks' work in one host thread per device inside the
 * library and returns when all are done.  When all devices[] are equal the ranks share that GPU
 * through the loopback transport (tests).  Field I/O is in the global x-fastest layout. */
typedef struct mgp_group mgp_group;
int         mgp_group_create(mgp_group** out, const mgp_opts* o, int ngpu, const int* devices);
void        mgp_group_destroy(mgp_group* g);
const char* mgp_group_last_error(const mgp_group* g);
int         mgp_group_size(const mgp_group* g);
mgp_ctx*    mgp_group_rank(mgp_group* g, int rank);   /* per-rank context (its slab, its stream) */
int         mgp_group_init_point_charge(mgp_group* g);
int         mgp_group_cycle(mgp_group* g, double* err_out);
int         mgp_group_cycles(mgp_group* g, int32_t k, double* errs);
int         mgp_group_set_field(mgp_group* g, int level, int which, const void* src, int64_t count, int mem);
int         mgp_group_get_field(mgp_group* g, int level, int which, void* dst, int64_t count, int mem);
int         mgp_group_residual_norm(mgp_group* g, int level, double* rnorm, double* fnorm);
int         mgp_group_field_stats(mgp_group* g, int level, int which, uint64_t* hash, double stats[3]);

/* The reference's debugging check (MultigridCPURaw.debugging / MultigridGPU.debugging: show / showAndCheck after
 * every sweep and piece of twoGrid, error "found a nan" on a non-finite cell; cpu-raw.lua:126-140,
 * gpu.lua:269-284).  mode 1: every phase of every cycle (pre-smoothing, the restricted residual, the coarse solve
 * or tail, prolongation + post-smoothing, per level) is followed by a device-side scan of its output; mgp_cycle /
 * mgp_cycles then return MGP_ERR_STATE naming the FIRST phase whose output holds a NaN or inf ("found a nan: cycle
 * c, level l (nx x ny x nz), <phase>").  Cycles run eagerly while it is on.  mode 0: off (the default). */
int         mgp_set_debug(mgp_ctx* c, int mode);

/* Kernel and communication timing with HIP events on the stream the work runs on.  mgp_timing(c, 1) resets
 * and enables (cycles then run eagerly, without hipGraph replay, so each launch can be bracketed).
 * Timed kinds; the first three on level 0 only:
 *   MGP_TIMING_HALF_SWEEP  plain red/black (or Jacobi) half-sweeps (not the err-fused last ones);
 *                          1.5 reals per cell per launch
 *   MGP_TIMING_FUSED_PRE   temporally blocked nu1 sweeps + residual + restriction: ALGORITHMIC bytes
 *                          (2 + 2^-dim) reals per cell (read black u and f, write black u and R / 2^dim;
 *                          2.5 with the full weighting, which restricts after the phase)
 *   MGP_TIMING_FUSED_POST  temporally blocked prolongation + correction + nu2 sweeps (+ err): (2.5 + 2^-dim
 *                          [+ 1 psiOld]) reals per cell
 *   MGP_TIMING_EXCHANGE    every halo exchange of any level (grouped send/recv with the z-neighbours, on the
 *                          compute or the side stream); bytes = what this rank sends
 *   MGP_TIMING_COLLECTIVE  the agglomeration all-gather and the err all-reduce; bytes = what this rank sends
 * mgp_timing_read returns, for one kind, the summed milliseconds, the number of timed launches / calls and
 * their bytes (algorithmic for the kernels: SURVEY.md §8d, not measured traffic). */
enum { MGP_TIMING_HALF_SWEEP = 0, MGP_TIMING_FUSED_PRE = 1, MGP_TIMING_FUSED_POST = 2, MGP_TIMING_EXCHANGE = 3,
       MGP_TIMING_COLLECTIVE = 4, MGP_TIMING_KINDS = 5 };
int         mgp_timing(mgp_ctx* c, int enable);
int         mgp_timing_read(mgp_ctx* c, int kind, double* ms_total, int64_t* launches, double* bytes);
/* The kernel the last timed launch of a kind ran (MGP_TIMING_FUSED_PRE / _POST; level 0): its symbol with the
 * template arguments as rocprofv3 prints it (NUL-terminated, truncated to cap bytes) and its grid in work-items
 * (rocprofv3's Grid_Size), so that PMC counters measured separately can be matched to exactly this launch.
 * MGP_ERR_STATE when no launch of that kind was timed since mgp_timing(c, 1).  No reference counterpart
 * (measurement only). */
int         mgp_timing_kernel(mgp_ctx* c, int kind, char* name, int cap, int64_t* grid);

/* The exchanges and collectives this rank has issued since creation or the last reset (reset != 0 clears after
 * reading), in issue order: up to max_rows rows of 5 int64 {op, side, level, msgs, bytes}, op 0 = halo exchange
 * (msgs per neighbour and direction, bytes sent per neighbour), 1 = agglomeration all-gather (bytes of this
 * rank's part), 2 = err all-reduce (8 bytes); side 1 = issued on the side stream (under RCCL on its own communicator, split off
 * the context's at creation).  Returns the
 * number of rows recorded (which may exceed max_rows).  Every rank of a decomposition must issue the same
 * sequence per communicator (RCCL matches calls in order); tests compare the ranks' logs. */
int         mgp_comm_log(mgp_ctx* c, int64_t* rows, int max_rows, int reset);
/* The same log for `cycles` outer iterations of a context mgp_create(o) would build, computed on the host
 * without a device (the cycle's host logic runs with every device and RCCL call skipped): what each rank of a
 * world > 1 decomposition will issue per cycle.  GPU tests check it against the executed mgp_comm_log. */
int         mgp_plan_comm(const mgp_opts* o, int32_t cycles, int64_t* rows, int max_rows);

/* Measurement helper (BASELINE.md "a measured copy-kernel peak"): the best of `reps` 16-byte streaming copies
 * of `bytes` between two fresh device buffers on `device` (-1: current), over three copy-kernel shapes
 * (grid-stride, one pass, one pass non-temporal), in GB/s of read + write bytes. */
int         mgp_copy_bandwidth(int device, int64_t bytes, int32_t reps, double* gbps);

#ifdef __cplusplus
}
#endif
#endif /* MGPOISSON_H */
