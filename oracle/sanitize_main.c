/*
 * sanitize_main.c — drives the C oracle under AddressSanitizer + UndefinedBehaviorSanitizer
 * (TEST INFRASTRUCTURE ONLY; `make -C oracle sanitize`, run by tests/test_oracle_sanitize.py).
 *
 * Every option of mgo_opts on small boxes (2D / 3D, cubic and non-cubic, fp32 / fp64, Jacobi / red-black /
 * lexicographic GS, V / F, injection / linear prolongation, fresh / warm coarse guess, both coarse boundary
 * conditions, both restrictions, 1 and 2 OpenMP threads, fp32 with cpu-raw.lua's double arithmetic) for a few outer iterations, plus the stateless
 * per-level functions and cpu-raw's twoGrid entry (mgo_two_grid).  Any out-of-bounds access, leak-free
 * misuse or undefined arithmetic aborts the run with a sanitizer report; success prints "sanitize ok".
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mgp_oracle.h"

static int run_case(int dim, int64_t nx, int64_t ny, int64_t nz, int rb, int smoother, int cycle, int prolong,
                    int init, int bc, int restriction, int threads)
{
    mgo_opts o;
    mgo_opts_default(&o);
    o.dim = dim;
    o.nx = nx;
    o.ny = ny;
    o.nz = dim == 3 ? nz : 1;
    o.real_bytes = rb == MGO_REAL_F32_ARITH_F64 ? 4 : rb;
    o.arith = rb == MGO_REAL_F32_ARITH_F64 ? MGO_ARITH_DOUBLE : MGO_ARITH_REAL;
    o.nu1 = o.nu2 = 2;
    o.smoother = smoother;
    o.cycle = cycle;
    o.prolong = prolong;
    o.coarse_init = init;
    o.coarse_bc = bc;
    o.restriction = restriction;
    o.threads = threads;
    mgo_ctx* c = mgo_create(&o);
    if (!c) {
        fprintf(stderr, "mgo_create failed: dim %d n %ld %ld %ld\n", dim, (long)nx, (long)ny, (long)nz);
        return 1;
    }
    mgo_init_point_charge(c);
    double errs[3];
    mgo_solve(c, 3, 0.0, errs);
    const int64_t n = nx * ny * o.nz;
    void* psi = malloc((size_t)n * o.real_bytes);
    mgo_get_field(c, 0, psi, n);
    mgo_set_field(c, 0, psi, n);
    const double e = mgo_step(c);
    free(psi);
    mgo_destroy(c);
    return isfinite(e) && isfinite(errs[0]) ? 0 : 2;
}

static int run_arrays(int dim, int64_t n, int rb)
{
    const int64_t nz = dim == 3 ? n : 1, cells = n * n * nz, coarse = cells >> dim;
    const size_t eb = rb == 8 ? 8 : 4;
    void* u = calloc((size_t)cells, eb);
    void* f = calloc((size_t)cells, eb);
    void* r = calloc((size_t)cells, eb);
    void* R = calloc((size_t)coarse, eb);
    for (int64_t i = 0; i < cells; ++i) {
        const double v = sin(0.37 * (double)i);
        if (rb == 8) ((double*)f)[i] = v, ((double*)u)[i] = 0.5 * v;
        else ((float*)f)[i] = (float)v, ((float*)u)[i] = (float)(0.5 * v);
    }
    const double h = 1.0 / (double)n;
    for (int sm = 0; sm < 3; ++sm) mgo_smooth_arr(dim, n, n, nz, rb, sm, 2, h, mgo_coarse_coef(1, 1), u, f);
    mgo_residual_arr(dim, n, n, nz, rb, h, 0.0, u, f, r);
    mgo_restrict_arr(dim, n, n, nz, rb, r, R);
    mgo_restrict_fw_arr(dim, n, n, nz, rb, mgo_coarse_coef(1, 1), r, R);
    for (int p = 0; p < 2; ++p) mgo_prolong_correct_arr(dim, n, n, nz, rb, p, mgo_coarse_coef(1, 1), u, R);
    const double s = mgo_residual_sumsq_arr(dim, n, n, nz, rb, h, 0.0, u, f, 0, nz, 2);
    const double e = mgo_err_arr(cells, rb, u, f);
    free(u), free(f), free(r), free(R);
    return isfinite(s) && isfinite(e) ? 0 : 3;
}

static int run_two_grid(int rb)
{
    mgo_opts o;
    mgo_opts_default(&o);
    o.dim = 2;
    o.nx = o.ny = 32;
    o.nz = 1;
    o.real_bytes = rb == 8 ? 8 : 4;
    o.arith = rb == MGO_REAL_F32_ARITH_F64 ? MGO_ARITH_DOUBLE : MGO_ARITH_REAL;
    mgo_ctx* c = mgo_create(&o);
    if (!c) return 4;
    const int64_t L = 16, n = L * L;
    void* u = calloc((size_t)n, o.real_bytes);
    void* f = calloc((size_t)n, o.real_bytes);
    if (rb == 8) ((double*)f)[n / 2 + L / 2] = -1e6;
    else ((float*)f)[n / 2 + L / 2] = -1e6f;
    const int rc = mgo_two_grid(c, 1.0 / (double)L, u, f, L);
    free(u), free(f);
    mgo_destroy(c);
    return rc == 0 ? 0 : 5;
}

int main(void)
{
    static const int64_t boxes[][4] = {
        {2, 16, 16, 1}, {2, 32, 8, 1}, {2, 8, 32, 1}, {3, 8, 8, 8}, {3, 16, 8, 4}, {3, 4, 8, 16}, {3, 16, 16, 16},
    };
    int fails = 0, cases = 0;
    for (size_t b = 0; b < sizeof(boxes) / sizeof(boxes[0]); ++b)
        for (int rb = 4; rb <= MGO_REAL_F32_ARITH_F64; rb += 4)
            for (int sm = 0; sm < 3; ++sm)
                for (int v = 0; v < 16; ++v) {
                    const int cycle = v & 1, prolong = (v >> 1) & 1, init = (v >> 2) & 1, bc = (v >> 3) & 1;
                    const int restriction = (b + (size_t)v) & 1, threads = 1 + (int)(v & 1);
                    const int rc = run_case((int)boxes[b][0], boxes[b][1], boxes[b][2], boxes[b][3], rb, sm, cycle,
                                            prolong, init, bc, restriction, threads);
                    if (rc) fprintf(stderr, "case failed (%d): box %zu rb %d smoother %d variant %d\n", rc, b, rb, sm, v);
                    fails += rc != 0;
                    ++cases;
                }
    for (int rb = 4; rb <= MGO_REAL_F32_ARITH_F64; rb += 4) {
        fails += run_arrays(2, 16, rb) != 0;
        fails += run_arrays(3, 8, rb) != 0;
        fails += run_two_grid(rb) != 0;
    }
    if (fails) {
        fprintf(stderr, "%d failures\n", fails);
        return 1;
    }
    printf("sanitize ok: %d cycle configurations, per-level functions, twoGrid\n", cases);
    return 0;
}
