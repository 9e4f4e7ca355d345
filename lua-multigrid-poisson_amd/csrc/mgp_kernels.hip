// mgp_kernels.hip — CDNA4 (gfx950) kernels of the multigrid cycle.
//
// One kernel per piece of the reference's twoGrid (cpu-raw.lua:186-237, gpu.lua:83-200),
// re-cut for HBM traffic:
//   k_jacobi            Jacobi sweep, out-of-place into a ping-pong buffer (gpu.lua:83-102 plus
//                       the enqueueCopyBuffer of gpu.lua:292, which the pointer swap removes)
//   k_rb_half           one colour of a red/black Gauss-Seidel sweep, in place (build-defined;
//                       the deterministic replacement of the racy gpu.lua:61-81 kernel)
//   k_residual_restrict calcResidual + reduceResidual fused (gpu.lua:104-137): the fine
//                       residual is never written to HBM
//   k_prolong_correct   expandResidual + addTo fused (gpu.lua:139-171); PC or (tri)linear
//   k_sqdiff_*          calcFrobErr + host sum (gpu.lua:189-200, 361-369) as a two-pass
//                       deterministic fp64 reduction on the device
//
// Arithmetic follows the reference operation by operation (sum ((xl+xr)+yl)+yr[+zl+zr],
// askew = sum/h^2, (f - askew)/adiag, r = f - (askew + adiag*u), 1/4 (r00+r10+r01+r11)); the
// library is compiled with -ffp-contract=off so no multiply-add is fused, and division is
// IEEE correctly rounded, so results are bit-identical to the C oracle in fp32 and fp64.
#include "mgp_internal.h"

namespace mgp {
namespace {

constexpr int kBlock = 256;

template <typename T>
struct Consts {
    T hSq, adiag, cl;
};

template <typename T, int DIM>
__device__ __forceinline__ Consts<T> make_consts(double h, double cl)
{
    Consts<T> c;
    T hh = (T)h;
    c.hSq = hh * hh;
    c.adiag = (T)(-2 * DIM) / c.hSq;
    c.cl = (T)cl;
    return c;
}

// Neighbour sum with ghost value 0 outside the box in x/y (cpu-raw.lua:36-39) and the ghost
// planes in z (zero at the physical boundary, the neighbour's plane across a slab boundary).
template <typename T, int DIM>
__device__ __forceinline__ T nbsum(const T* __restrict__ u, int64_t c, int i, int j, const Geo& g)
{
    T xl = i > 0 ? u[c - 1] : (T)0;
    T xr = i < g.nx - 1 ? u[c + 1] : (T)0;
    T yl = j > 0 ? u[c - g.nx] : (T)0;
    T yr = j < g.ny - 1 ? u[c + g.nx] : (T)0;
    T s = xl + xr;
    s = s + yl;
    s = s + yr;
    if (DIM == 3) {
        T zl = u[c - g.plane];
        T zr = u[c + g.plane];
        s = s + zl;
        s = s + zr;
    }
    return s;
}

// Level diagonal: the reference adiag, or with MGP_BC_CONSISTENT the extrapolated ghost
// folded in at boundary cells (oracle/mgp_oracle_impl.h diag()).
template <typename T, int DIM>
__device__ __forceinline__ T diag(int i, int j, int64_t gk, const Geo& g, const Consts<T>& k)
{
    if (k.cl == (T)0) return k.adiag;
    int nb = (i == 0) + (i == g.nx - 1) + (j == 0) + (j == g.ny - 1);
    if (DIM == 3) nb += (gk == 0) + (gk == g.gnz - 1);
    if (nb == 0) return k.adiag;
    T dg = (T)(-2 * DIM) - (T)nb * k.cl;
    return dg / k.hSq;
}

__device__ __forceinline__ void split(int64_t idx, const Geo& g, int& i, int& j, int64_t& k)
{
    i = (int)(idx & (g.nx - 1));
    j = (int)((idx >> g.lx) & (g.ny - 1));
    k = idx >> (g.lx + g.ly);
}

template <typename T, int DIM>
__global__ __launch_bounds__(kBlock) void k_init_point_charge(T* __restrict__ u, T* __restrict__ f,
                                                              Geo g, int64_t cx, int64_t cy, int64_t cz)
{
    int64_t idx = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (idx >= g.plane * g.nz) return;
    int i, j;
    int64_t k;
    split(idx, g, i, j, k);
    const double charge = 1e+6, epsilon0 = 1;
    bool hit = i == cx && j == cy && (DIM == 2 || g.z0 + k == cz);
    T v = hit ? (T)(-charge / epsilon0) : (T)0;
    f[idx] = v;
    u[idx] = -v;
}

// TAG distinguishes the finest-level instantiation (same code, separate symbol).
template <typename T, int DIM, int TAG>
__global__ __launch_bounds__(kBlock) void k_jacobi(const T* __restrict__ u, const T* __restrict__ f,
                                                   T* __restrict__ out, Geo g, double h, double cl)
{
    int64_t idx = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (idx >= g.plane * g.nz) return;
    int i, j;
    int64_t k;
    split(idx, g, i, j, k);
    const Consts<T> kc = make_consts<T, DIM>(h, cl);
    T askew = nbsum<T, DIM>(u, idx, i, j, g) / kc.hSq;
    out[idx] = (f[idx] - askew) / diag<T, DIM>(i, j, g.z0 + k, g, kc);
}

template <typename T, int DIM, int TAG>
__global__ __launch_bounds__(kBlock) void k_rb_half(T* __restrict__ u, const T* __restrict__ f,
                                                    Geo g, int color, double h, double cl)
{
    int64_t idx = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (idx >= g.plane * g.nz) return;
    int i, j;
    int64_t k;
    split(idx, g, i, j, k);
    if (((i + j + g.z0 + k) & 1) != color) return;
    const Consts<T> kc = make_consts<T, DIM>(h, cl);
    T askew = nbsum<T, DIM>(u, idx, i, j, g) / kc.hSq;
    u[idx] = (f[idx] - askew) / diag<T, DIM>(i, j, g.z0 + k, g, kc);
}

template <typename T, int DIM>
__device__ __forceinline__ T residual_at(const T* __restrict__ u, const T* __restrict__ f, int i,
                                         int j, int64_t k, const Geo& g, const Consts<T>& kc)
{
    int64_t c = (int64_t)i + (int64_t)g.nx * j + g.plane * k;
    T askew = nbsum<T, DIM>(u, c, i, j, g) / kc.hSq;
    T a_u = askew + diag<T, DIM>(i, j, g.z0 + k, g, kc) * u[c];
    return f[c] - a_u;
}

template <typename T, int DIM>
__global__ __launch_bounds__(kBlock) void k_residual_restrict(const T* __restrict__ u,
                                                              const T* __restrict__ f,
                                                              T* __restrict__ R, Geo g, double h,
                                                              double cl)
{
    const int cx = g.nx >> 1, cy = g.ny >> 1;
    const int64_t cz = DIM == 3 ? (g.nz >> 1) : 1;
    const int64_t cplane = (int64_t)cx * cy;
    int64_t idx = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (idx >= cplane * cz) return;
    const int I = (int)(idx & (cx - 1));
    const int J = (int)((idx >> (g.lx - 1)) & (cy - 1));
    const int64_t K = idx >> (g.lx - 1 + g.ly - 1);
    const Consts<T> kc = make_consts<T, DIM>(h, cl);
    const int i = 2 * I, j = 2 * J;
    const int64_t k = DIM == 3 ? 2 * K : 0;
    T s = residual_at<T, DIM>(u, f, i, j, k, g, kc) + residual_at<T, DIM>(u, f, i + 1, j, k, g, kc);
    s = s + residual_at<T, DIM>(u, f, i, j + 1, k, g, kc);
    s = s + residual_at<T, DIM>(u, f, i + 1, j + 1, k, g, kc);
    if (DIM == 3) {
        s = s + residual_at<T, DIM>(u, f, i, j, k + 1, g, kc);
        s = s + residual_at<T, DIM>(u, f, i + 1, j, k + 1, g, kc);
        s = s + residual_at<T, DIM>(u, f, i, j + 1, k + 1, g, kc);
        s = s + residual_at<T, DIM>(u, f, i + 1, j + 1, k + 1, g, kc);
        R[idx] = (T)0.125 * s;
    } else {
        R[idx] = (T)0.25 * s;
    }
}

// Coarse sample for the linear prolongation: an out-of-box neighbour is replaced by the parent
// times -cl per out-of-box axis (oracle cval()).
template <typename T>
__device__ __forceinline__ T cval(const T* __restrict__ V, int I, int J, int64_t K, bool ox, bool oy,
                                  bool oz, int cx, int64_t cplane, T cl)
{
    T s = (T)1;
    if (ox) s = -cl * s;
    if (oy) s = -cl * s;
    if (oz) s = -cl * s;
    T v = V[(int64_t)I + (int64_t)cx * J + cplane * K];
    return s == (T)1 ? v : s * v;
}

template <typename T, int DIM, int LINEAR>
__global__ __launch_bounds__(kBlock) void k_prolong_correct(T* __restrict__ u, const T* __restrict__ V,
                                                            Geo g, Geo gc, double clc)
{
    int64_t idx = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (idx >= g.plane * g.nz) return;
    int i, j;
    int64_t k;
    split(idx, g, i, j, k);
    const int cx = gc.nx;
    const int64_t cplane = gc.plane;
    const int I = i >> 1, J = j >> 1;
    const int64_t K = DIM == 3 ? (k >> 1) : 0;
    T v;
    if (!LINEAR) {
        v = V[(int64_t)I + (int64_t)cx * J + cplane * K];
    } else {
        const T w0 = (T)0.75, w1 = (T)0.25, cl = (T)clc;
        int In = (i & 1) ? I + 1 : I - 1;
        int Jn = (j & 1) ? J + 1 : J - 1;
        bool ox = In < 0 || In >= cx;
        bool oy = Jn < 0 || Jn >= gc.ny;
        if (ox) In = I;
        if (oy) Jn = J;
        if (DIM == 2) {
            T a0 = w0 * cval(V, I, J, 0, false, false, false, cx, cplane, cl) +
                   w1 * cval(V, In, J, 0, ox, false, false, cx, cplane, cl);
            T a1 = w0 * cval(V, I, Jn, 0, false, oy, false, cx, cplane, cl) +
                   w1 * cval(V, In, Jn, 0, ox, oy, false, cx, cplane, cl);
            v = w0 * a0 + w1 * a1;
        } else {
            int64_t Kn = (k & 1) ? K + 1 : K - 1;
            int64_t Kng = gc.z0 + Kn;
            bool oz = Kng < 0 || Kng >= gc.gnz;
            if (oz) Kn = K;
            T a00 = w0 * cval(V, I, J, K, false, false, false, cx, cplane, cl) +
                    w1 * cval(V, In, J, K, ox, false, false, cx, cplane, cl);
            T a10 = w0 * cval(V, I, Jn, K, false, oy, false, cx, cplane, cl) +
                    w1 * cval(V, In, Jn, K, ox, oy, false, cx, cplane, cl);
            T a01 = w0 * cval(V, I, J, Kn, false, false, oz, cx, cplane, cl) +
                    w1 * cval(V, In, J, Kn, ox, false, oz, cx, cplane, cl);
            T a11 = w0 * cval(V, I, Jn, Kn, false, oy, oz, cx, cplane, cl) +
                    w1 * cval(V, In, Jn, Kn, ox, oy, oz, cx, cplane, cl);
            T b0 = w0 * a00 + w1 * a10;
            T b1 = w0 * a01 + w1 * a11;
            v = w0 * b0 + w1 * b1;
        }
    }
    u[idx] = u[idx] + v;
}

// Pass 1: kSumBlocks fixed blocks, grid-stride, fp64 partial per block (fixed tree order).
template <typename T>
__global__ __launch_bounds__(kBlock) void k_sqdiff_partial(const T* __restrict__ a, const T* __restrict__ b,
                                                           int64_t n, double* __restrict__ partials)
{
    __shared__ double sh[kBlock];
    double acc = 0.0;
    for (int64_t c = (int64_t)blockIdx.x * kBlock + threadIdx.x; c < n; c += (int64_t)gridDim.x * kBlock) {
        double d = (double)a[c] - (double)b[c];
        acc += d * d;
    }
    sh[threadIdx.x] = acc;
    __syncthreads();
    for (int w = kBlock / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) partials[blockIdx.x] = sh[0];
}

// Pass 2: one block sums the kSumBlocks partials in a fixed order.
__global__ __launch_bounds__(1024) void k_sum_partials(const double* __restrict__ partials, double* __restrict__ out)
{
    __shared__ double sh[kSumBlocks];
    sh[threadIdx.x] = partials[threadIdx.x];
    __syncthreads();
    for (int w = kSumBlocks / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) *out = sh[0];
}

// Fixed-order sum of n fp64 partials (n arbitrary) by one workgroup.
__global__ __launch_bounds__(1024) void k_sum_n(const double* __restrict__ partials, int n, double* __restrict__ out)
{
    __shared__ double sh[1024];
    double a = 0.0;
    for (int i = threadIdx.x; i < n; i += 1024) a += partials[i];
    sh[threadIdx.x] = a;
    __syncthreads();
    for (int w = 512; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) *out = sh[0];
}

inline unsigned blocks_for(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

}  // namespace

#define MGP_DISPATCH(rb, dim, BODY)                                 \
    do {                                                            \
        if (rb == 8 && dim == 3) { using T = double; constexpr int D = 3; BODY; } \
        else if (rb == 8) { using T = double; constexpr int D = 2; BODY; }        \
        else if (dim == 3) { using T = float; constexpr int D = 3; BODY; }        \
        else { using T = float; constexpr int D = 2; BODY; }                      \
    } while (0)

hipError_t launch_init_point_charge(int rb, int dim, void* u, void* f, Geo g, int64_t cx, int64_t cy,
                                    int64_t cz, hipStream_t s)
{
    int64_t n = g.plane * g.nz;
    if (n == 0) return hipSuccess;
    MGP_DISPATCH(rb, dim, (k_init_point_charge<T, D><<<blocks_for(n), kBlock, 0, s>>>((T*)u, (T*)f, g, cx, cy, cz)));
    return hipGetLastError();
}

hipError_t launch_jacobi(int rb, int dim, bool fine, const void* u, const void* f, void* out, Geo g,
                         double h, double cl, hipStream_t s)
{
    int64_t n = g.plane * g.nz;
    if (fine)
        MGP_DISPATCH(rb, dim, (k_jacobi<T, D, 1><<<blocks_for(n), kBlock, 0, s>>>((const T*)u, (const T*)f, (T*)out, g, h, cl)));
    else
        MGP_DISPATCH(rb, dim, (k_jacobi<T, D, 0><<<blocks_for(n), kBlock, 0, s>>>((const T*)u, (const T*)f, (T*)out, g, h, cl)));
    return hipGetLastError();
}

hipError_t launch_rb_half(int rb, int dim, bool fine, void* u, const void* f, Geo g, int color, double h,
                          double cl, hipStream_t s)
{
    int64_t n = g.plane * g.nz;
    if (fine)
        MGP_DISPATCH(rb, dim, (k_rb_half<T, D, 1><<<blocks_for(n), kBlock, 0, s>>>((T*)u, (const T*)f, g, color, h, cl)));
    else
        MGP_DISPATCH(rb, dim, (k_rb_half<T, D, 0><<<blocks_for(n), kBlock, 0, s>>>((T*)u, (const T*)f, g, color, h, cl)));
    return hipGetLastError();
}

hipError_t launch_residual_restrict(int rb, int dim, const void* u, const void* f, void* R, Geo g,
                                    double h, double cl, hipStream_t s)
{
    int64_t n = (int64_t)(g.nx / 2) * (g.ny / 2) * (dim == 3 ? g.nz / 2 : 1);
    if (n == 0) return hipSuccess;
    MGP_DISPATCH(rb, dim, (k_residual_restrict<T, D><<<blocks_for(n), kBlock, 0, s>>>((const T*)u, (const T*)f, (T*)R, g, h, cl)));
    return hipGetLastError();
}

hipError_t launch_prolong_correct(int rb, int dim, int linear, void* u, const void* V, Geo g, Geo gc,
                                  double clc, hipStream_t s)
{
    int64_t n = g.plane * g.nz;
    if (linear)
        MGP_DISPATCH(rb, dim, (k_prolong_correct<T, D, 1><<<blocks_for(n), kBlock, 0, s>>>((T*)u, (const T*)V, g, gc, clc)));
    else
        MGP_DISPATCH(rb, dim, (k_prolong_correct<T, D, 0><<<blocks_for(n), kBlock, 0, s>>>((T*)u, (const T*)V, g, gc, clc)));
    return hipGetLastError();
}

hipError_t launch_sqdiff_sum(int rb, const void* a, const void* b, int64_t n, double* partials, double* out,
                             hipStream_t s)
{
    if (rb == 8)
        k_sqdiff_partial<double><<<kSumBlocks, kBlock, 0, s>>>((const double*)a, (const double*)b, n, partials);
    else
        k_sqdiff_partial<float><<<kSumBlocks, kBlock, 0, s>>>((const float*)a, (const float*)b, n, partials);
    k_sum_partials<<<1, kSumBlocks, 0, s>>>(partials, out);
    return hipGetLastError();
}

hipError_t launch_sum_partials(const double* partials, int n, double* out, hipStream_t s)
{
    k_sum_n<<<1, 1024, 0, s>>>(partials, n, out);
    return hipGetLastError();
}

}  // namespace mgp
