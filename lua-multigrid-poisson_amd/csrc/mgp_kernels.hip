// mgp_kernels.hip — CDNA4 (gfx950) kernels of the multigrid cycle on the red/black packed layout
// (see Geo in mgp_internal.h).
//
// One kernel per piece of the reference's twoGrid (cpu-raw.lua:186-237, gpu.lua:83-200),
// re-cut for HBM traffic:
//   k_half            one colour of a red/black sweep (build-defined smoother; the deterministic
//                     replacement of the racy gpu.lua:61-81 GaussSeidel kernel).  Run on both
//                     colours out of place it is the reference Jacobi sweep (gpu.lua:83-102) without
//                     the enqueueCopyBuffer of gpu.lua:292.  Per cell it moves 1.5 reals (read the
//                     other colour, read f, write this colour): 3 reals per full sweep.
//   k_resrestrict     calcResidual + reduceResidual fused (gpu.lua:104-137): the fine residual
//                     never reaches HBM.
//   k_prolong         expandResidual + addTo fused (gpu.lua:139-171); injection or (tri)linear.
//   k_sqdiff / k_sum  calcFrobErr + the host sum of gpu.lua:189-200, 361-369 as a deterministic
//                     two-pass fp64 reduction on the device (also fused into the last half-sweep).
//
// Arithmetic follows the reference operation by operation: neighbour sum ((xl+xr)+yl)+yr[+zl+zr],
// askew = sum/h^2, (f - askew)/adiag, r = f - (askew + adiag*u), 1/4 (r00+r10+r01+r11) and
// 1/8 of the 8 children in x-fastest order.  The library is compiled with -ffp-contract=off.
// Two rewrites are exact: x / h^2 == x * 2^(2k) (h is a power of two), and the division by the
// interior diagonal uses y = RN(1/adiag) plus one FMA correction (q = RN(a y),
// q' = RN(q + RN(a - q d) y)), which equals the IEEE quotient for operands away from
// over/underflow (Markstein); boundary cells with a modified diagonal divide directly.  The GPU
// parity tests check every piece bit for bit against the C oracle's plain divisions.
#include "mgp_internal.h"

namespace mgp {
namespace {

constexpr int kBlock = 256;

// ---- small helpers --------------------------------------------------------------------------

template <typename T>
struct VN {
    static constexpr int n = 16 / sizeof(T);  // reals per 16-byte access
};

template <typename T, int N>
struct alignas(16) Vec {
    T v[N];
};

template <typename T, int N>
__device__ __forceinline__ Vec<T, N> vload(const T* p)
{
    return *reinterpret_cast<const Vec<T, N>*>(p);
}
template <typename T, int N>
__device__ __forceinline__ void vstore(T* p, const Vec<T, N>& a)
{
    *reinterpret_cast<Vec<T, N>*>(p) = a;
}
template <typename T, int N>
__device__ __forceinline__ Vec<T, N> vzero()
{
    Vec<T, N> a;
#pragma unroll
    for (int e = 0; e < N; ++e) a.v[e] = (T)0;
    return a;
}

__device__ __forceinline__ float fmaT(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ double fmaT(double a, double b, double c) { return __builtin_fma(a, b, c); }

// RN(a / d) from y = RN(1 / d): one Markstein correction step.
template <typename T>
__device__ __forceinline__ T div_rn(T a, T d, T y)
{
    T q = a * y;
    T r = fmaT(-q, d, a);
    return fmaT(r, y, q);
}

// Level operator constants (oracle: relax(), diag(), residual()).
template <typename T, int DIM>
struct Op {
    T hSq, inv_hSq, adiag, yadiag, cl;
    __device__ __forceinline__ Op(double h, double cld)
    {
        const T hh = (T)h;
        hSq = hh * hh;
        inv_hSq = (T)1 / hSq;       // exact: h is a power of two
        adiag = (T)(-2 * DIM) / hSq;
        yadiag = (T)1 / adiag;      // RN(1/adiag)
        cl = (T)cld;
    }
    // diagonal of a cell with nb faces on the box boundary (cl = 0: the reference adiag)
    __device__ __forceinline__ T diag(int nb) const
    {
        if (cl == (T)0 || nb == 0) return adiag;
        return ((T)(-2 * DIM) - (T)nb * cl) / hSq;
    }
    // (f - sum/h^2) / diag
    __device__ __forceinline__ T relax(T sum, T fc, int nb) const
    {
        const T a = fc - sum * inv_hSq;
        if (cl != (T)0 && nb != 0) return a / (((T)(-2 * DIM) - (T)nb * cl) / hSq);
        return div_rn(a, adiag, yadiag);
    }
    // f - (sum/h^2 + diag*u)
    __device__ __forceinline__ T residual(T sum, T fc, T uc, int nb) const
    {
        const T askew = sum * inv_hSq;
        const T a_u = askew + diag(nb) * uc;
        return fc - a_u;
    }
};

// packed offset of cell (i, j, local plane k) (any level size, nx = 1 included)
__device__ __forceinline__ int64_t pidx(const Geo& g, int i, int j, int64_t k)
{
    const int c = (int)((i + j + g.z0 + k) & 1);
    return k * g.P + c * g.H + (int64_t)j * g.hw + (i >> 1);
}

__device__ __forceinline__ int xcd_remap(int b, int nblocks)
{
    // blocks b and b + 8 share an XCD: hand each XCD a contiguous band of the grid (z-neighbour
    // planes of a stencil then meet in that XCD's L2)
    if ((nblocks & 7) != 0) return b;
    return (b & 7) * (nblocks >> 3) + (b >> 3);
}

inline unsigned nblk(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

template <typename T>
__device__ __forceinline__ void block_partial(double acc, double* partials)
{
    __shared__ double red[kBlock];
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int w = kBlock / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) partials[blockIdx.x] = red[0];
}

// ---- init / pack / unpack -------------------------------------------------------------------

// thread per packed slot: slot -> (k, c, j, m) -> i = 2m + (c ^ parity); i >= nx only when nx = 1
__device__ __forceinline__ bool slot_cell(int64_t s, const Geo& g, int& i, int& j, int64_t& k)
{
    const int m = (int)(s & (g.hw - 1));
    j = (int)((s >> g.lhw) & (g.ny - 1));
    const int c = (int)((s >> (g.lhw + g.ly)) & 1);
    k = s >> (g.lhw + g.ly + 1);
    const int p = (int)((j + g.z0 + k) & 1);
    i = 2 * m + (c ^ p);
    return i < g.nx;
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_init(T* __restrict__ u, T* __restrict__ f, Geo g, int64_t cx, int64_t cy,
                                                 int64_t cz, int dim3)
{
    const int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (s >= g.P * g.nz) return;
    int i, j;
    int64_t k;
    const bool cell = slot_cell(s, g, i, j, k);
    const double charge = 1e+6, epsilon0 = 1;
    const bool hit = cell && i == cx && j == cy && (!dim3 || g.z0 + k == cz);
    const T v = hit ? (T)(-charge / epsilon0) : (T)0;
    f[s] = v;
    u[s] = -v;  // psi = -f (cpu.lua:193): -0.0 off the charge, as in the oracle
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_pack(const T* __restrict__ lex, T* __restrict__ out, Geo g)
{
    const int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (s >= g.P * g.nz) return;
    int i, j;
    int64_t k;
    out[s] = slot_cell(s, g, i, j, k) ? lex[(k * g.ny + j) * (int64_t)g.nx + i] : (T)0;
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_unpack(const T* __restrict__ in, T* __restrict__ lex, Geo g)
{
    const int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (s >= g.P * g.nz) return;
    int i, j;
    int64_t k;
    if (slot_cell(s, g, i, j, k)) lex[(k * g.ny + j) * (int64_t)g.nx + i] = in[s];
}

// ---- red/black half-sweep -------------------------------------------------------------------

// Vector form: a thread owns N consecutive cells of colour `color` in one row (hw % N == 0).
template <typename T, int DIM, int TAG, bool ERR>
__global__ __launch_bounds__(kBlock) void k_half(const T* __restrict__ other, const T* __restrict__ f,
                                                 T* __restrict__ dst, const T* __restrict__ old,
                                                 double* __restrict__ partials, Geo g, int color, double h,
                                                 double cld)
{
    constexpr int N = VN<T>::n;
    constexpr int LN = N == 4 ? 2 : 1;
    const int b = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t it = (int64_t)b * kBlock + threadIdx.x;
    const int lgpr = g.lhw - LN;  // log2 groups per row
    const int grp = (int)(it & ((1 << lgpr) - 1));
    const int j = (int)((it >> lgpr) & (g.ny - 1));
    const int64_t k = it >> (lgpr + g.ly);
    double acc = 0.0;
    if (k < g.nz) {
        const Op<T, DIM> op(h, cld);
        const int m0 = grp * N;
        const int64_t gk = g.z0 + k;
        const int o = color ^ (int)((j + gk) & 1);  // x parity of this row's colour-c cells
        const int64_t own = k * g.P + color * g.H + (int64_t)j * g.hw + m0;
        const int64_t oth = k * g.P + (color ^ 1) * g.H + (int64_t)j * g.hw + m0;
        const Vec<T, N> cen = vload<T, N>(other + oth);
        T edge;
        if (o == 0)
            edge = m0 > 0 ? other[oth - 1] : (T)0;      // x-1 of the first cell
        else
            edge = m0 + N < g.hw ? other[oth + N] : (T)0;  // x+1 of the last cell
        const Vec<T, N> yl = j > 0 ? vload<T, N>(other + oth - g.hw) : vzero<T, N>();
        const Vec<T, N> yr = j < g.ny - 1 ? vload<T, N>(other + oth + g.hw) : vzero<T, N>();
        Vec<T, N> zl, zr;
        if (DIM == 3) {
            zl = vload<T, N>(other + oth - g.P);
            zr = vload<T, N>(other + oth + g.P);
        }
        const Vec<T, N> fv = vload<T, N>(f + own);
        const int nbyz = (j == 0) + (j == g.ny - 1) + (DIM == 3 ? (gk == 0) + (gk == g.gnz - 1) : 0);
        Vec<T, N> out;
#pragma unroll
        for (int e = 0; e < N; ++e) {
            const int i = 2 * (m0 + e) + o;
            const T xl = o == 0 ? (e == 0 ? edge : cen.v[e - 1]) : cen.v[e];
            const T xr = o == 0 ? cen.v[e] : (e == N - 1 ? edge : cen.v[e + 1]);
            T s = xl + xr;
            s = s + yl.v[e];
            s = s + yr.v[e];
            if (DIM == 3) {
                s = s + zl.v[e];
                s = s + zr.v[e];
            }
            const int nb = nbyz + (i == 0) + (i == g.nx - 1);
            out.v[e] = op.relax(s, fv.v[e], nb);
        }
        vstore<T, N>(dst + own, out);
        if (ERR) {
            const Vec<T, N> w = vload<T, N>(old + own);
#pragma unroll
            for (int e = 0; e < N; ++e) {
                const double d = (double)out.v[e] - (double)w.v[e];
                acc += d * d;
            }
        }
    }
    if (ERR) block_partial<T>(acc, partials);
}

// Scalar form for small levels (hw < N, nx = 1 included): a thread per colour-c slot.
template <typename T, int DIM, bool ERR>
__global__ __launch_bounds__(kBlock) void k_half_s(const T* __restrict__ other, const T* __restrict__ f,
                                                   T* __restrict__ dst, const T* __restrict__ old,
                                                   double* __restrict__ partials, Geo g, int color, double h,
                                                   double cld)
{
    const int64_t it = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int m = (int)(it & (g.hw - 1));
    const int j = (int)((it >> g.lhw) & (g.ny - 1));
    const int64_t k = it >> (g.lhw + g.ly);
    double acc = 0.0;
    if (k < g.nz) {
        const int64_t gk = g.z0 + k;
        const int o = color ^ (int)((j + gk) & 1);
        const int i = 2 * m + o;
        if (i < g.nx) {
            const Op<T, DIM> op(h, cld);
            const int64_t own = k * g.P + color * g.H + (int64_t)j * g.hw + m;
            const int64_t oth = k * g.P + (color ^ 1) * g.H + (int64_t)j * g.hw + m;
            const T xl = i > 0 ? other[oth - 1 + o] : (T)0;
            const T xr = i < g.nx - 1 ? other[oth + o] : (T)0;
            T s = xl + xr;
            s = s + (j > 0 ? other[oth - g.hw] : (T)0);
            s = s + (j < g.ny - 1 ? other[oth + g.hw] : (T)0);
            if (DIM == 3) {
                s = s + other[oth - g.P];
                s = s + other[oth + g.P];
            }
            const int nb = (i == 0) + (i == g.nx - 1) + (j == 0) + (j == g.ny - 1) +
                           (DIM == 3 ? (gk == 0) + (gk == g.gnz - 1) : 0);
            const T v = op.relax(s, f[own], nb);
            dst[own] = v;
            if (ERR) {
                const double d = (double)v - (double)old[own];
                acc += d * d;
            }
        }
    }
    if (ERR) block_partial<T>(acc, partials);
}

// ---- fused residual + restriction -----------------------------------------------------------

// Residual of one fine cell from packed u (generic, scalar loads).
template <typename T, int DIM>
__device__ __forceinline__ T residual_at(const T* __restrict__ u, const T* __restrict__ f, const Geo& g,
                                         const Op<T, DIM>& op, int i, int j, int64_t k)
{
    const int64_t c = pidx(g, i, j, k);
    const int o = i & 1;
    // neighbours: other colour, same row at m-1+o / m+o; rows j+-1 and planes k+-1 at m
    const int64_t oth = c + ((c - k * g.P) >= g.H ? -g.H : g.H);
    const T xl = i > 0 ? u[oth - 1 + o] : (T)0;
    const T xr = i < g.nx - 1 ? u[oth + o] : (T)0;
    T s = xl + xr;
    s = s + (j > 0 ? u[oth - g.hw] : (T)0);
    s = s + (j < g.ny - 1 ? u[oth + g.hw] : (T)0);
    const int64_t gk = g.z0 + k;
    if (DIM == 3) {
        s = s + u[oth - g.P];
        s = s + u[oth + g.P];
    }
    const int nb = (i == 0) + (i == g.nx - 1) + (j == 0) + (j == g.ny - 1) + (DIM == 3 ? (gk == 0) + (gk == g.gnz - 1) : 0);
    return op.residual(s, f[c], u[c], nb);
}

// Scalar form: a thread per coarse cell (any sizes).
template <typename T, int DIM>
__global__ __launch_bounds__(kBlock) void k_resrestrict_s(const T* __restrict__ u, const T* __restrict__ f,
                                                          T* __restrict__ R, Geo g, Geo gc, double h, double cld)
{
    const int cx = g.nx >> 1, cy = g.ny >> 1;
    const int lcx = g.lx - 1, lcy = g.ly - 1;
    const int64_t ncz = DIM == 3 ? (g.nz >> 1) : 1;
    const int64_t it = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (it >= ((int64_t)cx * cy) * ncz) return;
    const int I = (int)(it & (cx - 1));
    const int J = (int)((it >> lcx) & (cy - 1));
    const int64_t K = it >> (lcx + lcy);
    const Op<T, DIM> op(h, cld);
    const int i = 2 * I, j = 2 * J;
    const int64_t k = DIM == 3 ? 2 * K : 0;
    T s = residual_at<T, DIM>(u, f, g, op, i, j, k) + residual_at<T, DIM>(u, f, g, op, i + 1, j, k);
    s = s + residual_at<T, DIM>(u, f, g, op, i, j + 1, k);
    s = s + residual_at<T, DIM>(u, f, g, op, i + 1, j + 1, k);
    if (DIM == 3) {
        s = s + residual_at<T, DIM>(u, f, g, op, i, j, k + 1);
        s = s + residual_at<T, DIM>(u, f, g, op, i + 1, j, k + 1);
        s = s + residual_at<T, DIM>(u, f, g, op, i, j + 1, k + 1);
        s = s + residual_at<T, DIM>(u, f, g, op, i + 1, j + 1, k + 1);
        R[pidx(gc, I, J, K)] = (T)0.125 * s;
    } else {
        R[pidx(gc, I, J, 0)] = (T)0.25 * s;
    }
}

// Vector form: a thread owns N consecutive coarse cells I0 .. I0+N-1 of one coarse row.  Their
// fine children are, in every fine row, the N cells m = I0 .. of BOTH colours; the thread loads
// each fine row / colour it needs once (N reals per access) and keeps the reference order
//   R = 1/8 (((((((r000 + r100) + r010) + r110) + r001) + r101) + r011) + r111).
template <typename T, int DIM>
__global__ __launch_bounds__(kBlock) void k_resrestrict(const T* __restrict__ u, const T* __restrict__ f,
                                                        T* __restrict__ R, Geo g, Geo gc, double h, double cld)
{
    constexpr int N = VN<T>::n;
    constexpr int LN = N == 4 ? 2 : 1;
    const int cy = g.ny >> 1;
    const int lgpr = (g.lx - 1) - LN;  // log2 groups of N per coarse row
    const int64_t ncz = DIM == 3 ? (g.nz >> 1) : 1;
    const int b = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t it = (int64_t)b * kBlock + threadIdx.x;
    const int grp = (int)(it & ((1 << lgpr) - 1));
    const int J = (int)((it >> lgpr) & (cy - 1));
    const int64_t K = it >> (lgpr + g.ly - 1);
    if (K >= ncz) return;
    const Op<T, DIM> op(h, cld);
    const int m0 = grp * N;  // = I0
    const int j0 = 2 * J;
    const int64_t k0 = DIM == 3 ? 2 * K : 0;
    constexpr int NZ = DIM == 3 ? 2 : 1;
    // r[dz][dy][x parity][e]
    T r[NZ][2][2][N];
#pragma unroll
    for (int dz = 0; dz < NZ; ++dz) {
        const int64_t k = k0 + dz;
        const int64_t gk = g.z0 + k;
#pragma unroll
        for (int dy = 0; dy < 2; ++dy) {
            const int j = j0 + dy;
            const int p = (int)((j + gk) & 1);
            const int nbyz = (j == 0) + (j == g.ny - 1) + (DIM == 3 ? (gk == 0) + (gk == g.gnz - 1) : 0);
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const int o = c ^ p;
                const int64_t own = k * g.P + c * g.H + (int64_t)j * g.hw + m0;
                const int64_t oth = k * g.P + (c ^ 1) * g.H + (int64_t)j * g.hw + m0;
                const Vec<T, N> cen = vload<T, N>(u + oth);
                const T edge = o == 0 ? (m0 > 0 ? u[oth - 1] : (T)0) : (m0 + N < g.hw ? u[oth + N] : (T)0);
                const Vec<T, N> yl = j > 0 ? vload<T, N>(u + oth - g.hw) : vzero<T, N>();
                const Vec<T, N> yr = j < g.ny - 1 ? vload<T, N>(u + oth + g.hw) : vzero<T, N>();
                Vec<T, N> zl, zr;
                if (DIM == 3) {
                    zl = vload<T, N>(u + oth - g.P);
                    zr = vload<T, N>(u + oth + g.P);
                }
                const Vec<T, N> uc = vload<T, N>(u + own);
                const Vec<T, N> fv = vload<T, N>(f + own);
#pragma unroll
                for (int e = 0; e < N; ++e) {
                    const int i = 2 * (m0 + e) + o;
                    const T xl = o == 0 ? (e == 0 ? edge : cen.v[e - 1]) : cen.v[e];
                    const T xr = o == 0 ? cen.v[e] : (e == N - 1 ? edge : cen.v[e + 1]);
                    T s = xl + xr;
                    s = s + yl.v[e];
                    s = s + yr.v[e];
                    if (DIM == 3) {
                        s = s + zl.v[e];
                        s = s + zr.v[e];
                    }
                    const int nb = nbyz + (i == 0) + (i == g.nx - 1);
                    r[dz][dy][o][e] = op.residual(s, fv.v[e], uc.v[e], nb);
                }
            }
        }
    }
    // coarse cells I0 + e: colour (I0 + e + J + gK) & 1, packed position (I0 + e) >> 1
    const int64_t gK = gc.z0 + K;
    const int pc = (int)((J + gK) & 1);
#pragma unroll
    for (int e = 0; e < N; ++e) {
        T s = r[0][0][0][e] + r[0][0][1][e];
        s = s + r[0][1][0][e];
        s = s + r[0][1][1][e];
        T val;
        if (DIM == 3) {
            s = s + r[1][0][0][e];
            s = s + r[1][0][1][e];
            s = s + r[1][1][0][e];
            s = s + r[1][1][1][e];
            val = (T)0.125 * s;
        } else {
            val = (T)0.25 * s;
        }
        const int I = m0 + e;
        const int cc = (I + pc) & 1;
        R[K * gc.P + cc * gc.H + (int64_t)J * gc.hw + (I >> 1)] = val;
    }
}

// ---- prolongation + correction --------------------------------------------------------------

// coarse value at (I, J, K) (K relative to the V pointer), times the ghost factor of the
// linear kind (oracle cval(): -cl per out-of-box axis, in x, y, z order)
template <typename T>
__device__ __forceinline__ T cval(const T* __restrict__ V, const Geo& gc, int I, int J, int64_t K, bool ox, bool oy,
                                  bool oz, T cl)
{
    T s = (T)1;
    if (ox) s = -cl * s;
    if (oy) s = -cl * s;
    if (oz) s = -cl * s;
    const T v = V[pidx(gc, I, J, K)];
    return s == (T)1 ? v : s * v;
}

// a thread per fine slot of colour `color` (any sizes)
template <typename T, int DIM, int LINEAR>
__global__ __launch_bounds__(kBlock) void k_prolong(T* __restrict__ u, const T* __restrict__ V, Geo g, Geo gc,
                                                    double clc, int color)
{
    const int64_t it = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int m = (int)(it & (g.hw - 1));
    const int j = (int)((it >> g.lhw) & (g.ny - 1));
    const int64_t k = it >> (g.lhw + g.ly);
    if (k >= g.nz) return;
    const int o = color ^ (int)((j + g.z0 + k) & 1);
    const int i = 2 * m + o;
    if (i >= g.nx) return;
    const int64_t own = k * g.P + color * g.H + (int64_t)j * g.hw + m;
    const int I = i >> 1, J = j >> 1;
    const int64_t K = DIM == 3 ? (k >> 1) : 0;
    T v;
    if (!LINEAR) {
        v = V[pidx(gc, I, J, K)];
    } else {
        const T w0 = (T)0.75, w1 = (T)0.25, cl = (T)clc;
        int In = (i & 1) ? I + 1 : I - 1;
        int Jn = (j & 1) ? J + 1 : J - 1;
        const bool ox = In < 0 || In >= gc.nx;
        const bool oy = Jn < 0 || Jn >= gc.ny;
        if (ox) In = I;
        if (oy) Jn = J;
        if (DIM == 2) {
            const T a0 = w0 * cval(V, gc, I, J, 0, false, false, false, cl) + w1 * cval(V, gc, In, J, 0, ox, false, false, cl);
            const T a1 = w0 * cval(V, gc, I, Jn, 0, false, oy, false, cl) + w1 * cval(V, gc, In, Jn, 0, ox, oy, false, cl);
            v = w0 * a0 + w1 * a1;
        } else {
            int64_t Kn = (k & 1) ? K + 1 : K - 1;
            const int64_t Kng = gc.z0 + Kn;
            const bool oz = Kng < 0 || Kng >= gc.gnz;
            if (oz) Kn = K;
            const T a00 = w0 * cval(V, gc, I, J, K, false, false, false, cl) + w1 * cval(V, gc, In, J, K, ox, false, false, cl);
            const T a10 = w0 * cval(V, gc, I, Jn, K, false, oy, false, cl) + w1 * cval(V, gc, In, Jn, K, ox, oy, false, cl);
            const T a01 = w0 * cval(V, gc, I, J, Kn, false, false, oz, cl) + w1 * cval(V, gc, In, J, Kn, ox, false, oz, cl);
            const T a11 = w0 * cval(V, gc, I, Jn, Kn, false, oy, oz, cl) + w1 * cval(V, gc, In, Jn, Kn, ox, oy, oz, cl);
            const T b0 = w0 * a00 + w1 * a10;
            const T b1 = w0 * a01 + w1 * a11;
            v = w0 * b0 + w1 * b1;
        }
    }
    u[own] = u[own] + v;
}

// Vector form (fine hw % N == 0, coarse nx >= N): a thread owns N consecutive fine cells of one
// colour in one row; their parents are the N consecutive coarse cells I = m0 .. m0+N-1 of coarse
// row (J, K), whose packed positions alternate colour, and the linear neighbours In = I - 1 + 2o.
template <typename T, int DIM, int LINEAR>
__global__ __launch_bounds__(kBlock) void k_prolong_v(T* __restrict__ u, const T* __restrict__ V, Geo g, Geo gc,
                                                      double clc, int color)
{
    constexpr int N = VN<T>::n;
    constexpr int LN = N == 4 ? 2 : 1;
    const int b = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t it = (int64_t)b * kBlock + threadIdx.x;
    const int lgpr = g.lhw - LN;
    const int grp = (int)(it & ((1 << lgpr) - 1));
    const int j = (int)((it >> lgpr) & (g.ny - 1));
    const int64_t k = it >> (lgpr + g.ly);
    if (k >= g.nz) return;
    const int m0 = grp * N;
    const int o = color ^ (int)((j + g.z0 + k) & 1);
    const int64_t own = k * g.P + color * g.H + (int64_t)j * g.hw + m0;
    const int J = j >> 1;
    const int64_t K = DIM == 3 ? (k >> 1) : 0;
    // coarse row (Jr, Kr): values at I = m0 - 1 + e for e = 0 .. N + 1 (out-of-row entries 0)
    auto crow = [&](int Jr, int64_t Kr, T (&c)[N + 2]) {
        const int pc = (int)((Jr + gc.z0 + Kr) & 1);
        const int64_t base = Kr * gc.P + (int64_t)Jr * gc.hw;
#pragma unroll
        for (int e = 0; e < N + 2; ++e) {
            const int I = m0 - 1 + e;
            if (I < 0 || I >= gc.nx) {
                c[e] = (T)0;
            } else {
                const int cc = (I + pc) & 1;
                c[e] = V[base + cc * gc.H + (I >> 1)];
            }
        }
    };
    Vec<T, N> uv = vload<T, N>(u + own);
    if (!LINEAR) {
        T c[N + 2];
        crow(J, K, c);
#pragma unroll
        for (int e = 0; e < N; ++e) uv.v[e] = uv.v[e] + c[e + 1];
    } else {
        const T w0 = (T)0.75, w1 = (T)0.25, cl = (T)clc;
        int Jn = (j & 1) ? J + 1 : J - 1;
        const bool oy = Jn < 0 || Jn >= gc.ny;
        if (oy) Jn = J;
        int64_t Kn = K;
        bool oz = false;
        if (DIM == 3) {
            Kn = (k & 1) ? K + 1 : K - 1;
            const int64_t Kng = gc.z0 + Kn;
            oz = Kng < 0 || Kng >= gc.gnz;
            if (oz) Kn = K;
        }
        T c00[N + 2], c10[N + 2], c01[N + 2], c11[N + 2];
        crow(J, K, c00);
        crow(Jn, K, c10);
        if (DIM == 3) {
            crow(J, Kn, c01);
            crow(Jn, Kn, c11);
        }
        auto sv = [&](T v, bool ox, bool yy, bool zz) {
            T s = (T)1;
            if (ox) s = -cl * s;
            if (yy) s = -cl * s;
            if (zz) s = -cl * s;
            return s == (T)1 ? v : s * v;
        };
#pragma unroll
        for (int e = 0; e < N; ++e) {
            const int I = m0 + e;
            const int In = I - 1 + 2 * o;
            const bool ox = In < 0 || In >= gc.nx;
            const int pe = e + 1;                    // parent column in c[]
            const int ne = ox ? pe : e + 2 * o;      // neighbour column (clamped to the parent)
            T v;
            if (DIM == 2) {
                const T a0 = w0 * sv(c00[pe], false, false, false) + w1 * sv(c00[ne], ox, false, false);
                const T a1 = w0 * sv(c10[pe], false, oy, false) + w1 * sv(c10[ne], ox, oy, false);
                v = w0 * a0 + w1 * a1;
            } else {
                const T a00 = w0 * sv(c00[pe], false, false, false) + w1 * sv(c00[ne], ox, false, false);
                const T a10 = w0 * sv(c10[pe], false, oy, false) + w1 * sv(c10[ne], ox, oy, false);
                const T a01 = w0 * sv(c01[pe], false, false, oz) + w1 * sv(c01[ne], ox, false, oz);
                const T a11 = w0 * sv(c11[pe], false, oy, oz) + w1 * sv(c11[ne], ox, oy, oz);
                const T b0 = w0 * a00 + w1 * a10;
                const T b1 = w0 * a01 + w1 * a11;
                v = w0 * b0 + w1 * b1;
            }
            uv.v[e] = uv.v[e] + v;
        }
    }
    vstore<T, N>(u + own, uv);
}

// ---- reductions -----------------------------------------------------------------------------

template <typename T>
__global__ __launch_bounds__(kBlock) void k_sqdiff_partial(const T* __restrict__ a, const T* __restrict__ b,
                                                           int64_t n, double* __restrict__ partials)
{
    double acc = 0.0;
    for (int64_t c = (int64_t)blockIdx.x * kBlock + threadIdx.x; c < n; c += (int64_t)gridDim.x * kBlock) {
        const double d = (double)a[c] - (double)b[c];
        acc += d * d;
    }
    block_partial<T>(acc, partials);
}

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

template <typename T>
constexpr int lnv() { return VN<T>::n == 4 ? 2 : 1; }

}  // namespace

// =============================================================================================
// launchers
// =============================================================================================

#define MGP_REAL(rb, BODY)             \
    do {                               \
        if (rb == 8) {                 \
            using T = double;          \
            BODY;                      \
        } else {                       \
            using T = float;           \
            BODY;                      \
        }                              \
    } while (0)

hipError_t launch_init_point_charge(int rb, int dim, void* u, void* f, Geo g, int64_t cx, int64_t cy, int64_t cz,
                                    hipStream_t s)
{
    const int64_t n = g.P * g.nz;
    MGP_REAL(rb, (k_init<T><<<nblk(n), kBlock, 0, s>>>((T*)u, (T*)f, g, cx, cy, cz, dim == 3)));
    return hipGetLastError();
}

hipError_t launch_pack(int rb, const void* lex, void* packed, Geo g, hipStream_t s)
{
    const int64_t n = g.P * g.nz;
    MGP_REAL(rb, (k_pack<T><<<nblk(n), kBlock, 0, s>>>((const T*)lex, (T*)packed, g)));
    return hipGetLastError();
}

hipError_t launch_unpack(int rb, const void* packed, void* lex, Geo g, hipStream_t s)
{
    const int64_t n = g.P * g.nz;
    MGP_REAL(rb, (k_unpack<T><<<nblk(n), kBlock, 0, s>>>((const T*)packed, (T*)lex, g)));
    return hipGetLastError();
}

static bool half_vector(int rb, const Geo& g) { return g.hw >= 16 / rb && g.nx >= 2; }

int half_blocks(int rb, Geo g)
{
    const int n = 16 / rb;
    const int64_t items = half_vector(rb, g) ? (g.H / n) * g.nz : g.H * g.nz;
    return (int)nblk(items);
}

hipError_t launch_half_sweep(int rb, int dim, bool fine, int color, const void* other, const void* f, void* dst,
                             const void* old, double* partials, Geo g, double h, double cl, hipStream_t s)
{
    const unsigned nb = (unsigned)half_blocks(rb, g);
    const bool err = old != nullptr;
    if (half_vector(rb, g)) {
#define HALF(D, TAG, E)                                                                                      \
    MGP_REAL(rb, (k_half<T, D, TAG, E><<<nb, kBlock, 0, s>>>((const T*)other, (const T*)f, (T*)dst, (const T*)old, \
                                                             partials, g, color, h, cl)))
        if (dim == 3) {
            if (fine) { if (err) HALF(3, 1, true); else HALF(3, 1, false); }
            else { if (err) HALF(3, 0, true); else HALF(3, 0, false); }
        } else {
            if (fine) { if (err) HALF(2, 1, true); else HALF(2, 1, false); }
            else { if (err) HALF(2, 0, true); else HALF(2, 0, false); }
        }
#undef HALF
    } else {
#define HALFS(D, E)                                                                                          \
    MGP_REAL(rb, (k_half_s<T, D, E><<<nb, kBlock, 0, s>>>((const T*)other, (const T*)f, (T*)dst, (const T*)old, \
                                                          partials, g, color, h, cl)))
        if (dim == 3) { if (err) HALFS(3, true); else HALFS(3, false); }
        else { if (err) HALFS(2, true); else HALFS(2, false); }
#undef HALFS
    }
    return hipGetLastError();
}

hipError_t launch_residual_restrict(int rb, int dim, const void* u, const void* f, void* R, Geo g, Geo gc, double h,
                                    double cl, hipStream_t s)
{
    const int n = 16 / rb;
    const int cx = g.nx / 2;
    const int64_t ncz = dim == 3 ? g.nz / 2 : 1;
    if (cx >= n && g.nx >= 2 * n) {
        const int64_t items = (int64_t)(cx / n) * (g.ny / 2) * ncz;
        if (dim == 3)
            MGP_REAL(rb, (k_resrestrict<T, 3><<<nblk(items), kBlock, 0, s>>>((const T*)u, (const T*)f, (T*)R, g, gc, h, cl)));
        else
            MGP_REAL(rb, (k_resrestrict<T, 2><<<nblk(items), kBlock, 0, s>>>((const T*)u, (const T*)f, (T*)R, g, gc, h, cl)));
    } else {
        const int64_t items = (int64_t)cx * (g.ny / 2) * ncz;
        if (dim == 3)
            MGP_REAL(rb, (k_resrestrict_s<T, 3><<<nblk(items), kBlock, 0, s>>>((const T*)u, (const T*)f, (T*)R, g, gc, h, cl)));
        else
            MGP_REAL(rb, (k_resrestrict_s<T, 2><<<nblk(items), kBlock, 0, s>>>((const T*)u, (const T*)f, (T*)R, g, gc, h, cl)));
    }
    return hipGetLastError();
}

hipError_t launch_prolong_correct(int rb, int dim, int linear, void* u, const void* V, Geo g, Geo gc, double clc,
                                  hipStream_t s)
{
    const int n = 16 / rb;
    const bool vec = g.hw >= n && g.nx >= 2;
    for (int color = 0; color < 2; ++color) {
        if (vec) {
            const unsigned nb = nblk((g.H / n) * g.nz);
#define PV(D, L) MGP_REAL(rb, (k_prolong_v<T, D, L><<<nb, kBlock, 0, s>>>((T*)u, (const T*)V, g, gc, clc, color)))
            if (dim == 3) { if (linear) PV(3, 1); else PV(3, 0); }
            else { if (linear) PV(2, 1); else PV(2, 0); }
#undef PV
        } else {
            const unsigned nb = nblk(g.H * g.nz);
#define PS(D, L) MGP_REAL(rb, (k_prolong<T, D, L><<<nb, kBlock, 0, s>>>((T*)u, (const T*)V, g, gc, clc, color)))
            if (dim == 3) { if (linear) PS(3, 1); else PS(3, 0); }
            else { if (linear) PS(2, 1); else PS(2, 0); }
#undef PS
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_sqdiff_sum(int rb, const void* a, const void* b, int64_t n, double* partials, double* out,
                             hipStream_t s)
{
    MGP_REAL(rb, (k_sqdiff_partial<T><<<kSumBlocks, kBlock, 0, s>>>((const T*)a, (const T*)b, n, partials)));
    k_sum_n<<<1, 1024, 0, s>>>(partials, kSumBlocks, out);
    return hipGetLastError();
}

hipError_t launch_sum_partials(const double* partials, int n, double* out, hipStream_t s)
{
    k_sum_n<<<1, 1024, 0, s>>>(partials, n, out);
    return hipGetLastError();
}

}  // namespace mgp
