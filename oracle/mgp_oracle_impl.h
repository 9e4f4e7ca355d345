/*
 * mgp_oracle_impl.h — type-generic body of the CPU oracle (TEST INFRASTRUCTURE ONLY).
 * Included three times by mgp_oracle.c: MGO_T is the storage type (the buffers), MGO_C the type every
 * expression is evaluated in, MGO_S the name suffix:
 *   f  (float, float)   gpu.lua's OpenCL real = float (gpu.lua:32): every operation rounded to float
 *   d  (double, double) real = double, the reference default (cpu-raw.lua:143)
 *   fd (float, double)  cpu-raw.lua under real = 'float' (cpu-raw.lua:142-153): float images read into
 *                       LuaJIT numbers, so every expression is double and only the store into the
 *                       float buffer rounds (Jacobi :34-44, calcResidual :46-57, reduceResidual :59-63,
 *                       addTo :83-85, and calcFrobErr :96-100 into the float errorBuf: MGO_ROUND_ERR)
 * With MGO_C == MGO_T every cast below is the identity.  Every arithmetic expression keeps the
 * reference's operation order; the file is compiled with -ffp-contract=off so no multiply-add is fused.
 */
#define MGO_CAT2(a, b) a##_##b
#define MGO_CAT(a, b) MGO_CAT2(a, b)
#define FN(name) MGO_CAT(name, MGO_S)

typedef MGO_T FN(real);
#if !defined(MGO_C) || !defined(MGO_ROUND_ERR)
#error "mgp_oracle.c defines MGO_T, MGO_C, MGO_S and MGO_ROUND_ERR per instantiation"
#endif

/* Sum of the 2*dim neighbours, ghost value 0 outside the array.
 * Order ((xl + xr) + yl) + yr [+ zl + zr] as written in cpu.lua:45-49 / cpu-raw.lua:36-41. */
static inline MGO_C FN(nbsum)(const MGO_T* u, int dim, int64_t nx, int64_t ny, int64_t nz,
                              int64_t i, int64_t j, int64_t k)
{
    const int64_t pl = nx * ny;
    const MGO_T* c = u + i + nx * j + pl * k;
    MGO_C xl = i > 0 ? (MGO_C)c[-1] : (MGO_C)0;
    MGO_C xr = i < nx - 1 ? (MGO_C)c[1] : (MGO_C)0;
    MGO_C yl = j > 0 ? (MGO_C)c[-nx] : (MGO_C)0;
    MGO_C yr = j < ny - 1 ? (MGO_C)c[nx] : (MGO_C)0;
    MGO_C s = xl + xr;
    s = s + yl;
    s = s + yr;
    if (dim == 3) {
        MGO_C zl = k > 0 ? (MGO_C)c[-pl] : (MGO_C)0;
        MGO_C zr = k < nz - 1 ? (MGO_C)c[pl] : (MGO_C)0;
        s = s + zl;
        s = s + zr;
    }
    return s;
}

/* One smoother update of one cell: (f - askew_u) / adiag with askew_u = sum / h^2,
 * adiag = -2*dim / h^2 (cpu.lua:49-51, cpu-raw.lua:40-43). */
static inline MGO_C FN(relax)(MGO_C sum, MGO_C fc, MGO_C hSq, MGO_C adiag)
{
    MGO_C askew = sum / hSq;
    return (fc - askew) / adiag;
}

/* Number of the cell's faces on the box boundary (a 1-cell axis counts 2). */
static inline int FN(nfaces)(int dim, int64_t nx, int64_t ny, int64_t nz, int64_t i, int64_t j,
                             int64_t k)
{
    int nb = (i == 0) + (i == nx - 1) + (j == 0) + (j == ny - 1);
    if (dim == 3) nb += (k == 0) + (k == nz - 1);
    return nb;
}

/* Diagonal of the level operator.  cl = 0 gives the reference's adiag = -2*dim/h^2 exactly;
 * cl > 0 (MGO_BC_CONSISTENT) folds the extrapolated ghost -cl*u into the diagonal:
 * diag = ((T)(-2*dim) - (T)nb * cl) / h^2. */
static inline MGO_C FN(diag)(int dim, int nb, MGO_C cl, MGO_C hSq, MGO_C adiag)
{
    if (cl == (MGO_C)0 || nb == 0) return adiag;
    MGO_C dg = (MGO_C)(-2 * dim) - (MGO_C)nb * cl;
    return dg / hSq;
}

static void FN(jacobi)(int dim, int64_t nx, int64_t ny, int64_t nz, double h, MGO_C cl, MGO_T* u,
                       const MGO_T* f, MGO_T* last, int threads)
{
    const MGO_C hh = (MGO_C)h, hSq = hh * hh, adiag = (MGO_C)(-2 * dim) / hSq;
    const int64_t pl = nx * ny;
    memcpy(last, u, (size_t)(pl * nz) * sizeof(MGO_T)); /* lastU = matrix(u), cpu.lua:42 */
#pragma omp parallel for num_threads(threads) schedule(static) if (threads > 1 && pl * nz > 65536)
    for (int64_t k = 0; k < nz; ++k)
        for (int64_t j = 0; j < ny; ++j)
            for (int64_t i = 0; i < nx; ++i) {
                int64_t c = i + nx * j + pl * k;
                MGO_C dg = FN(diag)(dim, FN(nfaces)(dim, nx, ny, nz, i, j, k), cl, hSq, adiag);
                u[c] = (MGO_T)FN(relax)(FN(nbsum)(last, dim, nx, ny, nz, i, j, k), (MGO_C)f[c], hSq, dg);
            }
}

/* Red/black Gauss-Seidel (build-defined; red = (i + j + k + z0) even, red first). */
static void FN(rbgs)(int dim, int64_t nx, int64_t ny, int64_t nz, double h, MGO_C cl, MGO_T* u,
                     const MGO_T* f, int threads)
{
    const MGO_C hh = (MGO_C)h, hSq = hh * hh, adiag = (MGO_C)(-2 * dim) / hSq;
    const int64_t pl = nx * ny;
    for (int color = 0; color < 2; ++color) {
#pragma omp parallel for num_threads(threads) schedule(static) if (threads > 1 && pl * nz > 65536)
        for (int64_t k = 0; k < nz; ++k)
            for (int64_t j = 0; j < ny; ++j) {
                int64_t i0 = (int64_t)((color + j + k) & 1);
                for (int64_t i = i0; i < nx; i += 2) {
                    int64_t c = i + nx * j + pl * k;
                    MGO_C dg = FN(diag)(dim, FN(nfaces)(dim, nx, ny, nz, i, j, k), cl, hSq, adiag);
                    u[c] = (MGO_T)FN(relax)(FN(nbsum)(u, dim, nx, ny, nz, i, j, k), (MGO_C)f[c], hSq, dg);
                }
            }
    }
}

/* Lexicographic GS in cpu.lua:26-27 loop order (x outer, then y, then z). */
static void FN(gslex)(int dim, int64_t nx, int64_t ny, int64_t nz, double h, MGO_C cl, MGO_T* u,
                      const MGO_T* f)
{
    const MGO_C hh = (MGO_C)h, hSq = hh * hh, adiag = (MGO_C)(-2 * dim) / hSq;
    const int64_t pl = nx * ny;
    for (int64_t i = 0; i < nx; ++i)
        for (int64_t j = 0; j < ny; ++j)
            for (int64_t k = 0; k < nz; ++k) {
                int64_t c = i + nx * j + pl * k;
                MGO_C dg = FN(diag)(dim, FN(nfaces)(dim, nx, ny, nz, i, j, k), cl, hSq, adiag);
                u[c] = (MGO_T)FN(relax)(FN(nbsum)(u, dim, nx, ny, nz, i, j, k), (MGO_C)f[c], hSq, dg);
            }
}

static void FN(smooth)(int dim, int64_t nx, int64_t ny, int64_t nz, int smoother, int sweeps,
                       double h, double cl, MGO_T* u, const MGO_T* f, MGO_T* tmp, int threads)
{
    const MGO_C c = (MGO_C)cl;
    for (int s = 0; s < sweeps; ++s) {
        if (smoother == MGO_JACOBI)
            FN(jacobi)(dim, nx, ny, nz, h, c, u, f, tmp, threads);
        else if (smoother == MGO_RBGS)
            FN(rbgs)(dim, nx, ny, nz, h, c, u, f, threads);
        else
            FN(gslex)(dim, nx, ny, nz, h, c, u, f);
    }
}

/* r = f - A u, A u = askew_u + adiag * u (cpu.lua:112-123, cpu-raw.lua:46-57). */
static void FN(residual)(int dim, int64_t nx, int64_t ny, int64_t nz, double h, double cl,
                         const MGO_T* u, const MGO_T* f, MGO_T* r, int threads)
{
    const MGO_C hh = (MGO_C)h, hSq = hh * hh, adiag = (MGO_C)(-2 * dim) / hSq, c = (MGO_C)cl;
    const int64_t pl = nx * ny;
#pragma omp parallel for num_threads(threads) schedule(static) if (threads > 1 && pl * nz > 65536)
    for (int64_t k = 0; k < nz; ++k)
        for (int64_t j = 0; j < ny; ++j)
            for (int64_t i = 0; i < nx; ++i) {
                int64_t cc = i + nx * j + pl * k;
                MGO_C askew = FN(nbsum)(u, dim, nx, ny, nz, i, j, k) / hSq;
                MGO_C dg = FN(diag)(dim, FN(nfaces)(dim, nx, ny, nz, i, j, k), c, hSq, adiag);
                MGO_C a_u = askew + dg * (MGO_C)u[cc];
                r[cc] = (MGO_T)((MGO_C)f[cc] - a_u);
            }
}

/* R = 1/4 (r00 + r10 + r01 + r11), x-first (cpu-raw.lua:59-63); 3D: 1/8 of 8 children,
 * x fastest, then y, then z, summed left to right. */
static void FN(restrict_)(int dim, int64_t nx, int64_t ny, int64_t nz, const MGO_T* r, MGO_T* R,
                          int threads)
{
    const int64_t cx = nx / 2, cy = ny / 2, cz = dim == 3 ? nz / 2 : 1;
    const int64_t pl = nx * ny, cpl = cx * cy;
#pragma omp parallel for num_threads(threads) schedule(static) if (threads > 1 && pl * nz > 65536)
    for (int64_t K = 0; K < cz; ++K)
        for (int64_t J = 0; J < cy; ++J)
            for (int64_t I = 0; I < cx; ++I) {
                if (dim == 2) {
                    const MGO_T* s = r + 2 * I + nx * (2 * J);
                    MGO_C sum = (MGO_C)s[0] + (MGO_C)s[1];
                    sum = sum + (MGO_C)s[nx];
                    sum = sum + (MGO_C)s[nx + 1];
                    R[I + cx * J] = (MGO_T)((MGO_C)0.25 * sum);
                } else {
                    const MGO_T* s = r + 2 * I + nx * (2 * J) + pl * (2 * K);
                    MGO_C sum = (MGO_C)s[0] + (MGO_C)s[1];
                    sum = sum + (MGO_C)s[nx];
                    sum = sum + (MGO_C)s[nx + 1];
                    sum = sum + (MGO_C)s[pl];
                    sum = sum + (MGO_C)s[pl + 1];
                    sum = sum + (MGO_C)s[pl + nx];
                    sum = sum + (MGO_C)s[pl + nx + 1];
                    R[I + cx * J + cpl * K] = (MGO_T)((MGO_C)0.125 * sum);
                }
            }
}

/* Full-weighting restriction (build-defined option, BASELINE north_star "full-weighting restriction"):
 * the cell-centred adjoint of the linear prolongation below, R = 2^-d P^T r.  Per axis a coarse cell I
 * takes fine cells 2I-1, 2I, 2I+1, 2I+2 with weights 1, w_lo, w_hi, 1 (then / 8), where w = 3, and at
 * the box faces (I = 0 for 2I, I = m-1 for 2I+1) w = 3 - clc: the -clc ghost factor of cval() (clc =
 * the coarse level's coefficient, 0 for MGO_BC_ZERO).  Fine cells outside the box count as r = +0.
 * Separable, x first, then y, then z, each axis summed ((r_a + w_b r_b) + w_c r_c) + r_d, and the
 * result scaled by 1/8^d (exact).  The 2x2x2 average above stays the default (cpu.lua:127-135). */
static inline MGO_C FN(fw_axis)(MGO_C a, MGO_C b, MGO_C c, MGO_C d, MGO_C wb, MGO_C wc)
{
    MGO_C s = a + wb * b;
    s = s + wc * c;
    s = s + d;
    return s;
}

static void FN(restrict_fw)(int dim, int64_t nx, int64_t ny, int64_t nz, double clc, const MGO_T* r,
                            MGO_T* R, int threads)
{
    const int64_t cx = nx / 2, cy = ny / 2, cz = dim == 3 ? nz / 2 : 1;
    const int64_t pl = nx * ny, cpl = cx * cy;
    const MGO_C w3 = (MGO_C)3, wf = (MGO_C)3 - (MGO_C)clc;
    const MGO_C scale = dim == 3 ? (MGO_C)(1.0 / 512.0) : (MGO_C)(1.0 / 64.0);
#pragma omp parallel for num_threads(threads) schedule(static) if (threads > 1 && pl * nz > 65536)
    for (int64_t K = 0; K < cz; ++K)
        for (int64_t J = 0; J < cy; ++J)
            for (int64_t I = 0; I < cx; ++I) {
                MGO_C az[4];
                const int nzz = dim == 3 ? 4 : 1;
                for (int dz = 0; dz < nzz; ++dz) {
                    const int64_t k = dim == 3 ? 2 * K - 1 + dz : 0;
                    MGO_C ay[4];
                    for (int dy = 0; dy < 4; ++dy) {
                        const int64_t j = 2 * J - 1 + dy;
                        MGO_C x[4];
                        for (int dx = 0; dx < 4; ++dx) {
                            const int64_t i = 2 * I - 1 + dx;
                            const int in = i >= 0 && i < nx && j >= 0 && j < ny && k >= 0 && k < nz;
                            x[dx] = in ? (MGO_C)r[i + nx * j + pl * k] : (MGO_C)0;
                        }
                        ay[dy] = FN(fw_axis)(x[0], x[1], x[2], x[3], I == 0 ? wf : w3, I == cx - 1 ? wf : w3);
                    }
                    az[dz] = FN(fw_axis)(ay[0], ay[1], ay[2], ay[3], J == 0 ? wf : w3, J == cy - 1 ? wf : w3);
                }
                const MGO_C s = dim == 3 ? FN(fw_axis)(az[0], az[1], az[2], az[3], K == 0 ? wf : w3, K == cz - 1 ? wf : w3)
                                         : az[0];
                R[I + cx * J + cpl * K] = (MGO_T)(scale * s);
            }
}

/* Coarse value for the linear prolongation.  Outside the box the ghost is -cl times the
 * value of the nearest cell inside (cl = 0: the reference's ghost 0).  Only one axis can be
 * outside at a time for the separable weights used below, but the clamp is applied per axis. */
static inline MGO_C FN(cval)(const MGO_T* V, int64_t cx, int64_t cy, int64_t cz, int64_t I,
                             int64_t J, int64_t K, MGO_C cl)
{
    MGO_C s = (MGO_C)1;
    if (I < 0) { I = 0; s = -cl * s; } else if (I >= cx) { I = cx - 1; s = -cl * s; }
    if (J < 0) { J = 0; s = -cl * s; } else if (J >= cy) { J = cy - 1; s = -cl * s; }
    if (K < 0) { K = 0; s = -cl * s; } else if (K >= cz) { K = cz - 1; s = -cl * s; }
    MGO_C v = (MGO_C)V[I + cx * J + cx * cy * K];
    return s == (MGO_C)1 ? v : s * v;
}

/* u += P V.  PC: v = V[parent] (cpu.lua:142-158, cpu-raw.lua:65-85).
 * LINEAR (build-defined): cell-centred, separable 3/4-1/4 weights, x then y then z.
 * v is rounded to the storage type (cpu-raw.lua:226 writes it into the real buffer vs[L]) before
 * addTo's u + v (cpu-raw.lua:83-85). */
static void FN(prolong_correct)(int dim, int64_t nx, int64_t ny, int64_t nz, int prolong,
                                double clc, MGO_T* u, const MGO_T* V, int threads)
{
    const int64_t cx = nx / 2, cy = ny / 2, cz = dim == 3 ? nz / 2 : 1;
    const int64_t pl = nx * ny;
    const MGO_C w0 = (MGO_C)0.75, w1 = (MGO_C)0.25, cl = (MGO_C)clc;
#pragma omp parallel for num_threads(threads) schedule(static) if (threads > 1 && pl * nz > 65536)
    for (int64_t k = 0; k < nz; ++k)
        for (int64_t j = 0; j < ny; ++j)
            for (int64_t i = 0; i < nx; ++i) {
                int64_t c = i + nx * j + pl * k;
                int64_t I = i >> 1, J = j >> 1, K = dim == 3 ? (k >> 1) : 0;
                MGO_C v;
                if (prolong == MGO_PROLONG_PC) {
                    v = (MGO_C)V[I + cx * J + cx * cy * K];
                } else {
                    int64_t In = (i & 1) ? I + 1 : I - 1;
                    int64_t Jn = (j & 1) ? J + 1 : J - 1;
                    if (dim == 2) {
                        MGO_C a0 = w0 * FN(cval)(V, cx, cy, 1, I, J, 0, cl) + w1 * FN(cval)(V, cx, cy, 1, In, J, 0, cl);
                        MGO_C a1 = w0 * FN(cval)(V, cx, cy, 1, I, Jn, 0, cl) + w1 * FN(cval)(V, cx, cy, 1, In, Jn, 0, cl);
                        v = w0 * a0 + w1 * a1;
                    } else {
                        int64_t Kn = (k & 1) ? K + 1 : K - 1;
                        MGO_C a00 = w0 * FN(cval)(V, cx, cy, cz, I, J, K, cl) + w1 * FN(cval)(V, cx, cy, cz, In, J, K, cl);
                        MGO_C a10 = w0 * FN(cval)(V, cx, cy, cz, I, Jn, K, cl) + w1 * FN(cval)(V, cx, cy, cz, In, Jn, K, cl);
                        MGO_C a01 = w0 * FN(cval)(V, cx, cy, cz, I, J, Kn, cl) + w1 * FN(cval)(V, cx, cy, cz, In, J, Kn, cl);
                        MGO_C a11 = w0 * FN(cval)(V, cx, cy, cz, I, Jn, Kn, cl) + w1 * FN(cval)(V, cx, cy, cz, In, Jn, Kn, cl);
                        MGO_C b0 = w0 * a00 + w1 * a10;
                        MGO_C b1 = w0 * a01 + w1 * a11;
                        v = w0 * b0 + w1 * b1;
                    }
                }
                const MGO_T vs = (MGO_T)v;
                u[c] = (MGO_T)((MGO_C)u[c] + (MGO_C)vs);
            }
}

/* sum of r^2 (r = f - A u in the real type, residual()'s expressions) over planes [z_lo, z_hi) of an
 * nx x ny x nz array whose ends are the Dirichlet ghost (a caller that passes a chunk of a larger field
 * with one halo plane per side gets that field's residual on the chunk's inner planes); per-plane fp64
 * partials, then summed in plane order. */
static double FN(residual_sumsq)(int dim, int64_t nx, int64_t ny, int64_t nz, double h, double cl, const MGO_T* u,
                                 const MGO_T* f, int64_t z_lo, int64_t z_hi, int threads)
{
    const MGO_C hh = (MGO_C)h, hSq = hh * hh, adiag = (MGO_C)(-2 * dim) / hSq, c = (MGO_C)cl;
    const int64_t pl = nx * ny, np_ = z_hi - z_lo;
    double* part = (double*)calloc((size_t)(np_ > 0 ? np_ : 1), sizeof(double));
#pragma omp parallel for num_threads(threads) schedule(static) if (threads > 1)
    for (int64_t q = 0; q < np_; ++q) {
        const int64_t k = z_lo + q;
        double s = 0.0;
        for (int64_t j = 0; j < ny; ++j)
            for (int64_t i = 0; i < nx; ++i) {
                const int64_t cc = i + nx * j + pl * k;
                const MGO_C askew = FN(nbsum)(u, dim, nx, ny, nz, i, j, k) / hSq;
                const MGO_C dg = FN(diag)(dim, FN(nfaces)(dim, nx, ny, nz, i, j, k), c, hSq, adiag);
                const MGO_T r = (MGO_T)((MGO_C)f[cc] - (askew + dg * (MGO_C)u[cc])); /* as rs[L] holds it */
                s += (double)r * (double)r;
            }
        part[q] = s;
    }
    double t = 0.0;
    for (int64_t q = 0; q < np_; ++q) t += part[q];
    free(part);
    return t;
}

/* sum over cells of (psi - psiOld)^2 in double, in cell order.  MGO_ROUND_ERR: each square is first
 * stored into the real errorBuf (cpu-raw.lua:96-100, 249-253), i.e. rounded to MGO_T. */
static double FN(sqdiff)(int64_t n, const MGO_T* a, const MGO_T* b)
{
    double s = 0.0;
    for (int64_t c = 0; c < n; ++c) {
        double d = (double)a[c] - (double)b[c];
        s += MGO_ROUND_ERR ? (double)(MGO_T)(d * d) : d * d;
    }
    return s;
}

#undef FN
#undef MGO_CAT
#undef MGO_CAT2
