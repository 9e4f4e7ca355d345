// mgp_krylov.hip — matrix-free conjugate gradients on a level's operator: the reference's
// independent cross-check of the multigrid answer (test/converge-multigrid-vs-krylov.lua:38-69,
// solver.conjgrad with x0 = -f, b = f and the 5-point A of :48-58), on the device as a second
// oracle for the hot path's converged solution.
//
// Vectors live in the red/black packed layout of the level (mgp_internal.h Geo), so A p reuses the
// hot path's neighbour addressing; empty slots (nx = 1 rows) stay 0 and add nothing to a dot.
// Dot products and max |x| are reduced in fp64 per workgroup, then summed in a fixed order.
#include "mgp_internal.h"

namespace mgp {
namespace {

constexpr int kB = 256;
constexpr unsigned kCgBlocks = 1024;  // grid-stride; == kSumBlocks partials per reduction

__device__ __forceinline__ int64_t nb_other(const Geo& g, int64_t own, int64_t k)
{
    return own + ((own - k * g.P) >= g.H ? -g.H : g.H);
}

// q = A p on every cell of the level (A: (sum of the 2 dim neighbours + diag' p) / h^2, ghost 0;
// diag' = -2 dim - nb cl on faces touching the box with a consistent coarse boundary)
template <typename T, int DIM>
__global__ __launch_bounds__(kB) void k_cg_apply(const T* __restrict__ p, T* __restrict__ q, Geo g, T inv_hSq, T cl)
{
    const int64_t n = g.P * g.nz;
    for (int64_t s = (int64_t)blockIdx.x * kB + threadIdx.x; s < n; s += (int64_t)gridDim.x * kB) {
        const int m = (int)(s & (g.hw - 1));
        const int j = (int)((s >> g.lhw) & (g.ny - 1));
        const int c = (int)((s >> (g.lhw + g.ly)) & 1);
        const int64_t k = s >> (g.lhw + g.ly + 1);
        const int64_t gk = g.z0 + k;
        const int i = 2 * m + (c ^ (int)((j + gk) & 1));
        if (i >= g.nx) {
            q[s] = (T)0;
            continue;
        }
        const int o = i & 1;
        const int64_t oth = nb_other(g, s, k);
        T sum = (i > 0 ? p[oth - 1 + o] : (T)0) + (i < g.nx - 1 ? p[oth + o] : (T)0);
        sum = sum + (j > 0 ? p[oth - g.hw] : (T)0);
        sum = sum + (j < g.ny - 1 ? p[oth + g.hw] : (T)0);
        if (DIM == 3) {
            sum = sum + p[oth - g.P];  // ghost planes are 0 at the box faces
            sum = sum + p[oth + g.P];
        }
        const int nb = (i == 0) + (i == g.nx - 1) + (j == 0) + (j == g.ny - 1) +
                       (DIM == 3 ? (gk == 0) + (gk == g.gnz - 1) : 0);
        const T diag = (T)(-2 * DIM) - (T)nb * cl;
        q[s] = (sum + diag * p[s]) * inv_hSq;
    }
}

__device__ __forceinline__ void block_sum2(double a, double b, double* pa, double* pb, bool mx)
{
    __shared__ double sa[kB], sb[kB];
    sa[threadIdx.x] = a;
    sb[threadIdx.x] = b;
    __syncthreads();
    for (int w = kB / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            sa[threadIdx.x] += sa[threadIdx.x + w];
            sb[threadIdx.x] = mx ? fmax(sb[threadIdx.x], sb[threadIdx.x + w]) : sb[threadIdx.x] + sb[threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        pa[blockIdx.x] = sa[0];
        pb[blockIdx.x] = sb[0];
    }
}

// partials: {a . b, c . d} (mx = false) or {a . b, max |c|} (mx = true), kCgBlocks each
template <typename T>
__global__ __launch_bounds__(kB) void k_cg_dots(const T* __restrict__ a, const T* __restrict__ b,
                                                const T* __restrict__ c, const T* __restrict__ d, int64_t n, bool mx,
                                                double* __restrict__ partials)
{
    double s0 = 0.0, s1 = 0.0;
    for (int64_t x = (int64_t)blockIdx.x * kB + threadIdx.x; x < n; x += (int64_t)gridDim.x * kB) {
        s0 += (double)a[x] * (double)b[x];
        if (mx) s1 = fmax(s1, fabs((double)c[x]));
        else s1 += (double)c[x] * (double)d[x];
    }
    block_sum2(s0, s1, partials, partials + gridDim.x, mx);
}

__global__ __launch_bounds__(kB) void k_cg_final(const double* __restrict__ partials, int nb, bool mx,
                                                 double* __restrict__ out)
{
    double s0 = 0.0, s1 = 0.0;
    for (int x = threadIdx.x; x < nb; x += kB) {
        s0 += partials[x];
        s1 = mx ? fmax(s1, partials[nb + x]) : s1 + partials[nb + x];
    }
    __shared__ double sa[kB], sb[kB];
    sa[threadIdx.x] = s0;
    sb[threadIdx.x] = s1;
    __syncthreads();
    for (int w = kB / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            sa[threadIdx.x] += sa[threadIdx.x + w];
            sb[threadIdx.x] = mx ? fmax(sb[threadIdx.x], sb[threadIdx.x + w]) : sb[threadIdx.x] + sb[threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out[0] = sa[0];
        out[1] = sb[0];
    }
}

// x += alpha p; r -= alpha q   (alpha = rSq / pAp, read on the device)
template <typename T>
__global__ __launch_bounds__(kB) void k_cg_update(T* __restrict__ x, T* __restrict__ r, const T* __restrict__ p,
                                                  const T* __restrict__ q, int64_t n, const double* __restrict__ num,
                                                  const double* __restrict__ den)
{
    const T alpha = (T)(*num / *den);
    for (int64_t s = (int64_t)blockIdx.x * kB + threadIdx.x; s < n; s += (int64_t)gridDim.x * kB) {
        x[s] = x[s] + alpha * p[s];
        r[s] = r[s] - alpha * q[s];
    }
}

// p = r + beta p   (beta = rSq_new / rSq, read on the device); then rSq = rSq_new (one thread, after
// every workgroup has read the old value: a separate launch)
template <typename T>
__global__ __launch_bounds__(kB) void k_cg_dir(T* __restrict__ p, const T* __restrict__ r, int64_t n,
                                               const double* __restrict__ num, const double* __restrict__ den)
{
    const T beta = (T)(*num / *den);
    for (int64_t s = (int64_t)blockIdx.x * kB + threadIdx.x; s < n; s += (int64_t)gridDim.x * kB)
        p[s] = r[s] + beta * p[s];
}

// r = b - q, p = r, x = x0 (already set)
template <typename T>
__global__ __launch_bounds__(kB) void k_cg_init(T* __restrict__ r, T* __restrict__ p, const T* __restrict__ b,
                                                const T* __restrict__ q, int64_t n)
{
    for (int64_t s = (int64_t)blockIdx.x * kB + threadIdx.x; s < n; s += (int64_t)gridDim.x * kB) {
        const T v = b[s] - q[s];
        r[s] = v;
        p[s] = v;
    }
}

__global__ void k_cg_copy1(double* __restrict__ dst, const double* __restrict__ src) { *dst = *src; }

template <typename T>
__global__ __launch_bounds__(kB) void k_cg_neg(T* __restrict__ x, const T* __restrict__ b, int64_t n)
{
    for (int64_t s = (int64_t)blockIdx.x * kB + threadIdx.x; s < n; s += (int64_t)gridDim.x * kB) x[s] = -b[s];
}

inline unsigned grid(int64_t n)
{
    const int64_t b = (n + kB - 1) / kB;
    return (unsigned)(b < (int64_t)kCgBlocks ? (b > 0 ? b : 1) : kCgBlocks);
}

template <typename T, int DIM>
hipError_t cg_t(CgArgs& a, hipStream_t s)
{
    const Geo& g = a.g;
    const int64_t n = g.P * g.nz;
    T* x = (T*)a.x;
    T* r = (T*)a.r;
    T* p = (T*)a.p;
    T* q = (T*)a.q;
    const T* b = (const T*)a.b;
    const T hh = (T)a.h;
    const T inv_hSq = (T)1 / (hh * hh);
    const T cl = (T)a.cl;
    double* part = a.scratch;                  // 2 * kCgBlocks
    double* d_rr = a.scratch + 2 * kCgBlocks;  // {rSq, bSq}
    double* d_pq = d_rr + 2;                   // {pAp, .}
    double* d_lx = d_pq + 2;                   // {rSq_new, max |x|}
    const unsigned gb = grid(n);
    auto dots = [&](const T* a0, const T* b0, const T* c0, const T* d0, bool mx, double* out) {
        k_cg_dots<T><<<gb, kB, 0, s>>>(a0, b0, c0, d0, n, mx, part);
        k_cg_final<<<1, kB, 0, s>>>(part, (int)gb, mx, out);
    };
    auto host2 = [&](const double* dev, double* h) -> hipError_t {
        hipError_t e = hipMemcpyAsync(h, dev, 2 * sizeof(double), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        return e;
    };
    if (a.x0_neg_b) k_cg_neg<T><<<gb, kB, 0, s>>>(x, b, n);
    k_cg_apply<T, DIM><<<gb, kB, 0, s>>>(x, q, g, inv_hSq, cl);
    k_cg_init<T><<<gb, kB, 0, s>>>(r, p, b, q, n);
    dots(r, r, b, b, false, d_rr);
    double h[2];
    hipError_t e = host2(d_rr, h);
    if (e != hipSuccess) return e;
    const double bsq = h[1];
    a.iters = 0;
    a.err = bsq > 0 ? h[0] / bsq : 0.0;
    // solver.conjgrad: stop when rSq / bSq < epsilon (the reference's errorCallback, converge...lua:60-67)
    while (a.iters < a.maxiter && !(a.err < a.epsilon)) {
        k_cg_apply<T, DIM><<<gb, kB, 0, s>>>(p, q, g, inv_hSq, cl);
        dots(p, q, p, q, false, d_pq);
        k_cg_update<T><<<gb, kB, 0, s>>>(x, r, p, q, n, d_rr, d_pq);
        dots(r, r, x, x, true, d_lx);
        e = host2(d_lx, h);
        if (e != hipSuccess) return e;
        ++a.iters;
        if (a.linf) a.linf[a.iters - 1] = h[1];  // |x|_inf per iteration, as the reference records
        a.err = h[0] / bsq;
        k_cg_dir<T><<<gb, kB, 0, s>>>(p, r, n, d_lx, d_rr);
        k_cg_copy1<<<1, 1, 0, s>>>(d_rr, d_lx);
    }
    return hipGetLastError();
}

}  // namespace

int cg_scratch_doubles() { return 2 * (int)kCgBlocks + 8; }

hipError_t launch_cg(int rb, int dim, CgArgs& a, hipStream_t s)
{
    if (rb == 8) return dim == 3 ? cg_t<double, 3>(a, s) : cg_t<double, 2>(a, s);
    return dim == 3 ? cg_t<float, 3>(a, s) : cg_t<float, 2>(a, s);
}

}  // namespace mgp
