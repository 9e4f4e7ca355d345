/*
 * mgp_oracle.c — CPU restatement of the reference V/F-cycle (TEST INFRASTRUCTURE ONLY).
 * See mgp_oracle.h for the reference lines each piece follows and for the parity status.
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp).
 */
#include "mgp_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* gpu.lua's real = float (every operation in float) and real = double */
#define MGO_T float
#define MGO_C float
#define MGO_S f
#define MGO_ROUND_ERR 0
#include "mgp_oracle_impl.h"
#undef MGO_T
#undef MGO_C
#undef MGO_S
#define MGO_T double
#define MGO_C double
#define MGO_S d
#include "mgp_oracle_impl.h"
#undef MGO_T
#undef MGO_C
#undef MGO_S
#undef MGO_ROUND_ERR
/* cpu-raw.lua's real = 'float': float buffers, double expressions, float errorBuf */
#define MGO_T float
#define MGO_C double
#define MGO_S fd
#define MGO_ROUND_ERR 1
#include "mgp_oracle_impl.h"
#undef MGO_T
#undef MGO_C
#undef MGO_S
#undef MGO_ROUND_ERR

#define MGO_MAX_LEVELS 40

static int kind_of(int real_bytes, int arith)
{
    return real_bytes == 4 && arith == MGO_ARITH_DOUBLE ? MGO_REAL_F32_ARITH_F64 : real_bytes;
}
static size_t kind_bytes(int kind) { return kind == 8 ? 8 : 4; }

#define MGO_DISPATCH(kind, CALL_D, CALL_F, CALL_FD) \
    do {                                            \
        if ((kind) == 8)                            \
            CALL_D;                                 \
        else if ((kind) == MGO_REAL_F32_ARITH_F64)  \
            CALL_FD;                                \
        else                                        \
            CALL_F;                                 \
    } while (0)


typedef struct {
    int64_t nx, ny, nz;
    void* u;   /* current guess (psi on level 0, V on coarser levels) */
    void* f;   /* right-hand side (f on level 0, R on coarser levels) */
    void* r;   /* residual scratch */
    void* tmp; /* Jacobi lastU scratch */
} mgo_level;

struct mgo_ctx {
    mgo_opts o;
    int kind; /* kind_of(real_bytes, arith) */
    int nlev;
    mgo_level lev[MGO_MAX_LEVELS];
    void* psi_old;
};

void mgo_opts_default(mgo_opts* o)
{
    memset(o, 0, sizeof(*o));
    o->dim = 2;
    o->nx = o->ny = 8;
    o->nz = 1;
    o->real_bytes = 8;
    o->nu1 = o->nu2 = 7;              /* cpu.lua:20 */
    o->smoother = MGO_JACOBI;         /* cpu.lua:57 */
    o->cycle = MGO_CYCLE_V;           /* twoGrid recursion, gamma = 1 */
    o->prolong = MGO_PROLONG_PC;      /* cpu.lua:142-150 */
    o->coarse_init = MGO_COARSE_FRESH;/* cpu.lua:138 */
    o->coarse_sweeps = 48;
    o->coarse_bc = MGO_BC_ZERO;       /* ghost 0 on every level, cpu.lua:28-31 */
    o->threads = 1;
    o->restriction = MGO_RESTRICT_AVERAGE; /* cpu.lua:127-135 */
    o->arith = MGO_ARITH_REAL;
}

static int64_t ncell(const mgo_level* L) { return L->nx * L->ny * L->nz; }

static int is_pow2(int64_t v) { return v > 0 && (v & (v - 1)) == 0; }

mgo_ctx* mgo_create(const mgo_opts* o)
{
    if (!o || (o->dim != 2 && o->dim != 3) || (o->real_bytes != 4 && o->real_bytes != 8) ||
        (o->arith != MGO_ARITH_REAL && o->arith != MGO_ARITH_DOUBLE))
        return NULL;
    int64_t nz = o->dim == 2 ? 1 : o->nz;
    if (!is_pow2(o->nx) || !is_pow2(o->ny) || !is_pow2(nz)) return NULL;
    mgo_ctx* c = (mgo_ctx*)calloc(1, sizeof(mgo_ctx));
    c->o = *o;
    c->o.nz = nz;
    if (c->o.threads < 1) c->o.threads = 1;
    c->kind = kind_of(o->real_bytes, o->arith);
    int64_t nx = o->nx, ny = o->ny;
    const size_t rb = (size_t)o->real_bytes;
    for (;;) {
        mgo_level* L = &c->lev[c->nlev++];
        L->nx = nx;
        L->ny = ny;
        L->nz = nz;
        size_t bytes = (size_t)(nx * ny * nz) * rb;
        L->u = calloc(1, bytes);
        L->f = calloc(1, bytes);
        L->r = calloc(1, bytes);
        L->tmp = calloc(1, bytes);
        /* coarsen while every active axis has >= 2 cells (cpu.lua recursion to width 1) */
        int more = nx >= 2 && ny >= 2 && (o->dim == 2 || nz >= 2);
        if (!more || c->nlev == MGO_MAX_LEVELS) break;
        nx /= 2;
        ny /= 2;
        if (o->dim == 3) nz /= 2;
    }
    c->psi_old = calloc(1, (size_t)ncell(&c->lev[0]) * rb);
    return c;
}

void mgo_destroy(mgo_ctx* c)
{
    if (!c) return;
    for (int l = 0; l < c->nlev; ++l) {
        free(c->lev[l].u);
        free(c->lev[l].f);
        free(c->lev[l].r);
        free(c->lev[l].tmp);
    }
    free(c->psi_old);
    free(c);
}

int mgo_num_levels(const mgo_ctx* c) { return c->nlev; }

void mgo_level_dims(const mgo_ctx* c, int level, int64_t out[3])
{
    out[0] = c->lev[level].nx;
    out[1] = c->lev[level].ny;
    out[2] = c->lev[level].nz;
}

/* f = -1e6 at 0-based (n/2, n/2[, n/2]), 0 elsewhere; psi = -f
 * (cpu.lua:182-193, cpu-raw.lua:8-20: center = floor(L/2)). */
void mgo_init_point_charge(mgo_ctx* c)
{
    mgo_level* L = &c->lev[0];
    int64_t n = ncell(L);
    int64_t ci = L->nx / 2, cj = L->ny / 2, ck = c->o.dim == 3 ? L->nz / 2 : 0;
    int64_t center = ci + L->nx * cj + L->nx * L->ny * ck;
    const double charge = 1e+6, epsilon0 = 1;
    const double Q = -charge / epsilon0;
    if (c->o.real_bytes == 8) {
        double *f = (double*)L->f, *u = (double*)L->u;
        for (int64_t i = 0; i < n; ++i) f[i] = 0.0;
        f[center] = Q;
        for (int64_t i = 0; i < n; ++i) u[i] = -f[i];
    } else {
        float *f = (float*)L->f, *u = (float*)L->u;
        for (int64_t i = 0; i < n; ++i) f[i] = 0.0f;
        f[center] = (float)Q;
        for (int64_t i = 0; i < n; ++i) u[i] = -f[i];
    }
}

int mgo_set_field(mgo_ctx* c, int which, const void* src, int64_t count)
{
    mgo_level* L = &c->lev[0];
    if (count != ncell(L) || (which != 0 && which != 1)) return -1;
    memcpy(which == 0 ? L->u : L->f, src, (size_t)count * (size_t)c->o.real_bytes);
    return 0;
}

int mgo_get_field(const mgo_ctx* c, int which, void* dst, int64_t count)
{
    const mgo_level* L = &c->lev[0];
    if (count != ncell(L) || (which != 0 && which != 1)) return -1;
    memcpy(dst, which == 0 ? L->u : L->f, (size_t)count * (size_t)c->o.real_bytes);
    return 0;
}

/* ---- dispatch helpers on (dims, kind) ----
 * kind = 8 (double), 4 (float, gpu.lua's float arithmetic) or MGO_REAL_F32_ARITH_F64 (float buffers,
 * double arithmetic: cpu-raw.lua's real = 'float'); buffers are float for both float kinds. */

static void smooth_any(int dim, int64_t nx, int64_t ny, int64_t nz, int kind, int smoother, int sweeps,
                       double h, double cl, void* u, const void* f, void* tmp, int threads)
{
    MGO_DISPATCH(kind,
                 smooth_d(dim, nx, ny, nz, smoother, sweeps, h, cl, (double*)u, (const double*)f, (double*)tmp, threads),
                 smooth_f(dim, nx, ny, nz, smoother, sweeps, h, cl, (float*)u, (const float*)f, (float*)tmp, threads),
                 smooth_fd(dim, nx, ny, nz, smoother, sweeps, h, cl, (float*)u, (const float*)f, (float*)tmp, threads));
}

static void residual_any(int dim, int64_t nx, int64_t ny, int64_t nz, int kind, double h, double cl,
                         const void* u, const void* f, void* r, int threads)
{
    MGO_DISPATCH(kind, residual_d(dim, nx, ny, nz, h, cl, (const double*)u, (const double*)f, (double*)r, threads),
                 residual_f(dim, nx, ny, nz, h, cl, (const float*)u, (const float*)f, (float*)r, threads),
                 residual_fd(dim, nx, ny, nz, h, cl, (const float*)u, (const float*)f, (float*)r, threads));
}

static void restrict_any(int dim, int64_t nx, int64_t ny, int64_t nz, int kind, const void* r, void* R,
                         int threads)
{
    MGO_DISPATCH(kind, restrict__d(dim, nx, ny, nz, (const double*)r, (double*)R, threads),
                 restrict__f(dim, nx, ny, nz, (const float*)r, (float*)R, threads),
                 restrict__fd(dim, nx, ny, nz, (const float*)r, (float*)R, threads));
}

static void restrict_fw_any(int dim, int64_t nx, int64_t ny, int64_t nz, int kind, double clc, const void* r,
                            void* R, int threads)
{
    MGO_DISPATCH(kind, restrict_fw_d(dim, nx, ny, nz, clc, (const double*)r, (double*)R, threads),
                 restrict_fw_f(dim, nx, ny, nz, clc, (const float*)r, (float*)R, threads),
                 restrict_fw_fd(dim, nx, ny, nz, clc, (const float*)r, (float*)R, threads));
}

static void prolong_any(int dim, int64_t nx, int64_t ny, int64_t nz, int kind, int prolong, double clc,
                        void* u, const void* V, int threads)
{
    MGO_DISPATCH(kind, prolong_correct_d(dim, nx, ny, nz, prolong, clc, (double*)u, (const double*)V, threads),
                 prolong_correct_f(dim, nx, ny, nz, prolong, clc, (float*)u, (const float*)V, threads),
                 prolong_correct_fd(dim, nx, ny, nz, prolong, clc, (float*)u, (const float*)V, threads));
}

double mgo_coarse_coef(int coarse_bc, int level)
{
    if (coarse_bc != MGO_BC_CONSISTENT || level <= 0) return 0.0;
    double p = ldexp(1.0, level);
    return (p - 1.0) / (p + 1.0);
}

/* ---- the cycle (cpu.lua:70-165) ---- */

static void cycle_rec(mgo_ctx* c, int l, double h, int fcycle);

static void coarse_solve(mgo_ctx* c, int l, double h)
{
    mgo_level* L = &c->lev[l];
    /* 1 cell: one sweep == u = (f - 0)/adiag exactly (cpu.lua:76-93, cpu-raw.lua:190-196).
     * A coarsest line/plane (non-cubic boxes, build-defined) gets coarse_sweeps sweeps. */
    int sweeps = ncell(L) == 1 ? 1 : c->o.coarse_sweeps;
    smooth_any(c->o.dim, L->nx, L->ny, L->nz, c->kind, c->o.smoother, sweeps, h,
               mgo_coarse_coef(c->o.coarse_bc, l), L->u, L->f, L->tmp, c->o.threads);
}

static void cycle_rec(mgo_ctx* c, int l, double h, int fcycle)
{
    const mgo_opts* o = &c->o;
    mgo_level* L = &c->lev[l];
    if (l == c->nlev - 1) {
        coarse_solve(c, l, h);
        return;
    }
    mgo_level* C = &c->lev[l + 1];
    const double cl = mgo_coarse_coef(o->coarse_bc, l), clc = mgo_coarse_coef(o->coarse_bc, l + 1);
    smooth_any(o->dim, L->nx, L->ny, L->nz, c->kind, o->smoother, o->nu1, h, cl, L->u, L->f,
               L->tmp, o->threads);
    residual_any(o->dim, L->nx, L->ny, L->nz, c->kind, h, cl, L->u, L->f, L->r, o->threads);
    if (o->restriction == MGO_RESTRICT_FULL_WEIGHTING)
        restrict_fw_any(o->dim, L->nx, L->ny, L->nz, c->kind, clc, L->r, C->f, o->threads);
    else
        restrict_any(o->dim, L->nx, L->ny, L->nz, c->kind, L->r, C->f, o->threads);
    if (o->coarse_init == MGO_COARSE_FRESH) /* V = matrix.zeros (cpu.lua:138) */
        memset(C->u, 0, (size_t)ncell(C) * (size_t)o->real_bytes);
    if (fcycle) {
        cycle_rec(c, l + 1, 2 * h, 1);
        cycle_rec(c, l + 1, 2 * h, 0);
    } else {
        cycle_rec(c, l + 1, 2 * h, 0); /* twoGrid(2*h, V, R) (cpu.lua:139) */
    }
    prolong_any(o->dim, L->nx, L->ny, L->nz, c->kind, o->prolong, clc, L->u, C->u, o->threads);
    smooth_any(o->dim, L->nx, L->ny, L->nz, c->kind, o->smoother, o->nu2, h, cl, L->u, L->f,
               L->tmp, o->threads);
}

double mgo_err_arr(int64_t n, int real_bytes, const void* psi, const void* psi_old)
{
    double s = 0.0;
    MGO_DISPATCH(real_bytes, s = sqdiff_d(n, (const double*)psi, (const double*)psi_old),
                 s = sqdiff_f(n, (const float*)psi, (const float*)psi_old),
                 s = sqdiff_fd(n, (const float*)psi, (const float*)psi_old));
    return sqrt(s / (double)n);
}

double mgo_step(mgo_ctx* c)
{
    mgo_level* L = &c->lev[0];
    const double h = 1.0 / (double)L->nx; /* cpu.lua:197-198 */
    const size_t bytes = (size_t)ncell(L) * (size_t)c->o.real_bytes;
    memcpy(c->psi_old, L->u, bytes); /* psiOld = matrix(self.psi) (cpu.lua:200) */
    cycle_rec(c, 0, h, c->o.cycle == MGO_CYCLE_F);
    return mgo_err_arr(ncell(L), c->kind, L->u, c->psi_old); /* cpu.lua:203, cpu-raw.lua:249-254 */
}

int mgo_solve(mgo_ctx* c, int maxiter, double epsilon, double* errs)
{
    int it = 0;
    for (int iter = 1; iter <= maxiter; ++iter) { /* cpu.lua:211-215 */
        double err = mgo_step(c);
        if (errs) errs[iter - 1] = err;
        it = iter;
        if (err < epsilon || !isfinite(err)) break;
    }
    return it;
}

int mgo_two_grid(mgo_ctx* c, double h, void* u, const void* f, int64_t L)
{
    for (int l = 0; l < c->nlev; ++l) {
        mgo_level* Lv = &c->lev[l];
        if (Lv->nx != L) continue;
        size_t bytes = (size_t)ncell(Lv) * (size_t)c->o.real_bytes;
        memcpy(Lv->u, u, bytes);
        memcpy(Lv->f, f, bytes);
        cycle_rec(c, l, h, c->o.cycle == MGO_CYCLE_F);
        memcpy(u, Lv->u, bytes);
        return 0;
    }
    return -1;
}

/* ---- stateless per-level kernels for the unit tests ---- */

void mgo_smooth_arr(int dim, int64_t nx, int64_t ny, int64_t nz, int real_bytes, int smoother,
                    int sweeps, double h, double cl, void* u, const void* f)
{
    if (dim == 2) nz = 1;
    void* tmp = malloc((size_t)(nx * ny * nz) * kind_bytes(real_bytes));
    smooth_any(dim, nx, ny, nz, real_bytes, smoother, sweeps, h, cl, u, f, tmp, 1);
    free(tmp);
}

void mgo_residual_arr(int dim, int64_t nx, int64_t ny, int64_t nz, int real_bytes, double h,
                      double cl, const void* u, const void* f, void* r)
{
    residual_any(dim, nx, ny, dim == 2 ? 1 : nz, real_bytes, h, cl, u, f, r, 1);
}

void mgo_restrict_arr(int dim, int64_t nx, int64_t ny, int64_t nz, int real_bytes, const void* r,
                      void* R)
{
    restrict_any(dim, nx, ny, dim == 2 ? 1 : nz, real_bytes, r, R, 1);
}

double mgo_residual_sumsq_arr(int dim, int64_t nx, int64_t ny, int64_t nz, int real_bytes, double h, double cl,
                              const void* u, const void* f, int64_t z_lo, int64_t z_hi, int threads)
{
    if (dim == 2) nz = 1;
    double s = 0.0;
    MGO_DISPATCH(real_bytes, s = residual_sumsq_d(dim, nx, ny, nz, h, cl, (const double*)u, (const double*)f, z_lo, z_hi, threads),
                 s = residual_sumsq_f(dim, nx, ny, nz, h, cl, (const float*)u, (const float*)f, z_lo, z_hi, threads),
                 s = residual_sumsq_fd(dim, nx, ny, nz, h, cl, (const float*)u, (const float*)f, z_lo, z_hi, threads));
    return s;
}

void mgo_restrict_fw_arr(int dim, int64_t nx, int64_t ny, int64_t nz, int real_bytes, double cl_coarse,
                         const void* r, void* R)
{
    restrict_fw_any(dim, nx, ny, dim == 2 ? 1 : nz, real_bytes, cl_coarse, r, R, 1);
}

void mgo_prolong_correct_arr(int dim, int64_t nx, int64_t ny, int64_t nz, int real_bytes,
                             int prolong, double cl_coarse, void* u, const void* V)
{
    prolong_any(dim, nx, ny, dim == 2 ? 1 : nz, real_bytes, prolong, cl_coarse, u, V, 1);
}
