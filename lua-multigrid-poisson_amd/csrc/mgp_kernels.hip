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

// Level operator constants (oracle: relax(), diag(), residual()), computed once on the host in
// the real type (IEEE host arithmetic gives the same values the oracle computes) and passed by
// value to every kernel.
template <typename T, int DIM>
struct Op {
    T hSq, inv_hSq, adiag, yadiag, cl;
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

template <typename T, int DIM>
Op<T, DIM> make_op(double h, double cl)
{
    Op<T, DIM> op;
    const T hh = (T)h;
    op.hSq = hh * hh;
    op.inv_hSq = (T)1 / op.hSq;  // exact: h is a power of two
    op.adiag = (T)(-2 * DIM) / op.hSq;
    op.yadiag = (T)1 / op.adiag;  // RN(1/adiag)
    op.cl = (T)cl;
    return op;
}

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
                                                 double* __restrict__ partials, Geo g, int color,
                                                 Op<T, DIM> op)
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
                                                   double* __restrict__ partials, Geo g, int color,
                                                   Op<T, DIM> op)
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
                                                          T* __restrict__ R, Geo g, Geo gc, Op<T, DIM> op)
{
    const int cx = g.nx >> 1, cy = g.ny >> 1;
    const int lcx = g.lx - 1, lcy = g.ly - 1;
    const int64_t ncz = DIM == 3 ? (g.nz >> 1) : 1;
    const int64_t it = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (it >= ((int64_t)cx * cy) * ncz) return;
    const int I = (int)(it & (cx - 1));
    const int J = (int)((it >> lcx) & (cy - 1));
    const int64_t K = it >> (lcx + lcy);
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
// fine children are, in every fine row, the N cells m = I0 .. of BOTH colours.  The thread loads
// each fine (plane, row, colour) vector it needs exactly once into registers — planes 2K, 2K+1
// with rows 2J-1 .. 2J+2, planes 2K-1, 2K+2 with rows 2J, 2J+1 — and keeps the reference order
//   R = 1/8 (((((((r000 + r100) + r010) + r110) + r001) + r101) + r011) + r111).
template <typename T, int DIM>
__global__ __launch_bounds__(kBlock) void k_resrestrict(const T* __restrict__ u, const T* __restrict__ f,
                                                        T* __restrict__ R, Geo g, Geo gc, Op<T, DIM> op)
{
    constexpr int N = VN<T>::n;
    constexpr int LN = N == 4 ? 2 : 1;
    constexpr int NZ = DIM == 3 ? 2 : 1;  // fine planes per coarse plane
    const int cy = g.ny >> 1;
    const int lgpr = (g.lx - 1) - LN;  // log2 groups of N per coarse row
    const int64_t ncz = DIM == 3 ? (g.nz >> 1) : 1;
    const int b = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t it = (int64_t)b * kBlock + threadIdx.x;
    const int grp = (int)(it & ((1 << lgpr) - 1));
    const int J = (int)((it >> lgpr) & (cy - 1));
    const int64_t K = it >> (lgpr + g.ly - 1);
    if (K >= ncz) return;
    const int m0 = grp * N;
    const int j0 = 2 * J;
    const int64_t k0 = DIM == 3 ? 2 * K : 0;

    const bool xlo = m0 == 0, xhi = m0 + N == g.hw;
    auto row = [&](int64_t k, int j, int c) {
        return (j >= 0 && j < g.ny) ? vload<T, N>(u + k * g.P + c * g.H + (int64_t)j * g.hw + m0) : vzero<T, N>();
    };
    // running sum in the reference order: the children of fine plane 2K, then of 2K+1
    T acc[N];
#pragma unroll
    for (int dz = 0; dz < NZ; ++dz) {
        const int64_t k = k0 + dz;
        const int64_t gk = g.z0 + k;
        // this plane's rows j0-1 .. j0+2 (both colours) and, in 3D, rows j0, j0+1 of planes k-1, k+1
        Vec<T, N> M[4][2], Z[2][2][2];
#pragma unroll
        for (int yi = 0; yi < 4; ++yi)
#pragma unroll
            for (int c = 0; c < 2; ++c) M[yi][c] = row(k, j0 - 1 + yi, c);
        if (DIM == 3) {
#pragma unroll
            for (int zz = 0; zz < 2; ++zz)
#pragma unroll
                for (int yi = 0; yi < 2; ++yi)
#pragma unroll
                    for (int c = 0; c < 2; ++c) Z[zz][yi][c] = row(k - 1 + 2 * zz, j0 + yi, c);
        }
#pragma unroll
        for (int dy = 0; dy < 2; ++dy) {
            const int j = j0 + dy;
            const int p = (int)((j + gk) & 1);
            const int nbyz = (j == 0) + (j == g.ny - 1) + (DIM == 3 ? (gk == 0) + (gk == g.gnz - 1) : 0);
            const bool fast = op.cl == (T)0 || (nbyz == 0 && !xlo && !xhi);
            T rr[2][N];  // [x parity][e]
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const int o = c ^ p;
                const int oc = c ^ 1;
                const Vec<T, N>& cen = M[dy + 1][oc];
                const Vec<T, N>& uc = M[dy + 1][c];
                const int64_t own = k * g.P + c * g.H + (int64_t)j * g.hw + m0;
                const int64_t oth = k * g.P + oc * g.H + (int64_t)j * g.hw + m0;
                const Vec<T, N> fv = vload<T, N>(f + own);
                const T edge = o == 0 ? (xlo ? (T)0 : u[oth - 1]) : (xhi ? (T)0 : u[oth + N]);
#pragma unroll
                for (int e = 0; e < N; ++e) {
                    const T xl = o == 0 ? (e == 0 ? edge : cen.v[e - 1]) : cen.v[e];
                    const T xr = o == 0 ? cen.v[e] : (e == N - 1 ? edge : cen.v[e + 1]);
                    T s = xl + xr;
                    s = s + M[dy][oc].v[e];
                    s = s + M[dy + 2][oc].v[e];
                    if (DIM == 3) {
                        s = s + Z[0][dy][oc].v[e];
                        s = s + Z[1][dy][oc].v[e];
                    }
                    T res;
                    if (fast) {
                        const T askew = s * op.inv_hSq;
                        const T a_u = askew + op.adiag * uc.v[e];
                        res = fv.v[e] - a_u;
                    } else {
                        const int i = 2 * (m0 + e) + o;
                        res = op.residual(s, fv.v[e], uc.v[e], nbyz + (i == 0) + (i == g.nx - 1));
                    }
                    rr[o][e] = res;
                }
            }
#pragma unroll
            for (int e = 0; e < N; ++e) {
                if (dz == 0 && dy == 0) {
                    acc[e] = rr[0][e] + rr[1][e];
                } else {
                    acc[e] = acc[e] + rr[0][e];
                    acc[e] = acc[e] + rr[1][e];
                }
            }
        }
    }
    // coarse cells I0 + e: colour (I0 + e + J + gK) & 1, packed position (I0 + e) >> 1
    const int64_t gK = gc.z0 + K;
    const int pc = (int)((J + gK) & 1);
    T val[N];
#pragma unroll
    for (int e = 0; e < N; ++e) val[e] = (DIM == 3 ? (T)0.125 : (T)0.25) * acc[e];
    const int64_t rowc = K * gc.P + (int64_t)J * gc.hw;
#pragma unroll
    for (int e = 0; e < N; ++e) {
        const int I = m0 + e;
        R[rowc + ((I + pc) & 1) * gc.H + (I >> 1)] = val[e];
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

// Coarse samples x = I0-1 .. I0+N of coarse row (Jr, Kr) (Kr relative to the V pointer) into
// c[0 .. N+1]; samples outside the row are 0 (never used: the caller clamps to the parent).
// In the packed layout I0 .. I0+N-1 sit pairwise in the two halves at (I0 >> 1) ..: two 2-wide
// loads for fp32, plus the two edge samples.
template <typename T, int N>
__device__ __forceinline__ void coarse_row(const T* __restrict__ V, const Geo& gc, int Jr, int64_t Kr, int I0,
                                           T (&c)[N + 2])
{
    const int pc = (int)((Jr + gc.z0 + Kr) & 1);  // colour of even x in this row
    const int64_t row = Kr * gc.P + (int64_t)Jr * gc.hw;
    const T* hp = V + row + pc * gc.H;        // colour of I0, I0+2, ...
    const T* hq = V + row + (pc ^ 1) * gc.H;  // colour of I0+1, I0+3, ...
    const int cm = I0 >> 1;
    if (N == 4) {
        const Vec<T, 2> a = vload<T, 2>(hp + cm);
        const Vec<T, 2> b = vload<T, 2>(hq + cm);
        c[1] = a.v[0];
        c[2] = b.v[0];
        c[3] = a.v[1];
        c[4] = b.v[1];
    } else {
#pragma unroll
        for (int e = 0; e < N; ++e) c[e + 1] = ((e & 1) ? hq : hp)[cm + (e >> 1)];
    }
    c[0] = I0 > 0 ? hq[cm - 1] : (T)0;
    c[N + 1] = I0 + N < gc.nx ? hp[cm + N / 2] : (T)0;
}

// Vector form (coarse nx >= N): a thread owns the fine cells of one fine row (j, k) above N
// consecutive coarse cells I0 .. — fine m = I0 .. in BOTH colours (one N-wide access of u each).
// It needs the coarse rows J, Jn and planes K, Kn only (Jn, Kn clamped to the parent row/plane
// outside the box, where the oracle's cval() factor applies) and evaluates exactly the oracle's
// per-cell expression.
template <typename T, int DIM, int LINEAR>
__global__ __launch_bounds__(kBlock) void k_prolong_v(T* __restrict__ u, const T* __restrict__ V, Geo g, Geo gc,
                                                      T cl)
{
    constexpr int N = VN<T>::n;
    constexpr int LN = N == 4 ? 2 : 1;
    const int cx = gc.nx, cy = gc.ny;
    const int lgpr = gc.lx - LN;
    const int b = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t it = (int64_t)b * kBlock + threadIdx.x;
    const int grp = (int)(it & ((1 << lgpr) - 1));
    const int j = (int)((it >> lgpr) & (g.ny - 1));
    const int64_t k = DIM == 3 ? it >> (lgpr + g.ly) : 0;
    if (k >= g.nz) return;
    const int I0 = grp * N;
    const int J = j >> 1;
    const int64_t K = DIM == 3 ? (k >> 1) : 0;
    int Jn = (j & 1) ? J + 1 : J - 1;
    const bool oy = Jn < 0 || Jn >= cy;
    if (oy) Jn = J;
    int64_t Kn = K;
    bool oz = false;
    if (DIM == 3) {
        Kn = (k & 1) ? K + 1 : K - 1;
        oz = gc.z0 + Kn < 0 || gc.z0 + Kn >= gc.gnz;
        if (oz) Kn = K;
    }
    T c00[N + 2], c10[N + 2], c01[N + 2], c11[N + 2];  // [z: K / Kn][y: J / Jn]
    coarse_row<T, N>(V, gc, J, K, I0, c00);
    if (LINEAR) {
        coarse_row<T, N>(V, gc, Jn, K, I0, c10);
        if (DIM == 3) {
            coarse_row<T, N>(V, gc, J, Kn, I0, c01);
            coarse_row<T, N>(V, gc, Jn, Kn, I0, c11);
        }
    }
    const T w0 = (T)0.75, w1 = (T)0.25;
    auto sv = [&](T val, bool fx, bool fy, bool fz) {
        T s = (T)1;
        if (fx) s = -cl * s;
        if (fy) s = -cl * s;
        if (fz) s = -cl * s;
        return s == (T)1 ? val : s * val;
    };
    const int p = (int)((j + g.z0 + k) & 1);
    const bool interior = !oy && !oz && I0 > 0 && I0 + N < cx;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const int o = c ^ p;  // x parity of this colour's cells in row j
        const int64_t own = k * g.P + c * g.H + (int64_t)j * g.hw + I0;
        Vec<T, N> uv = vload<T, N>(u + own);
#pragma unroll
        for (int e = 0; e < N; ++e) {
            const int pe = e + 1;  // parent I0 + e
            T v;
            if (!LINEAR) {
                v = c00[pe];
            } else if (interior) {  // no neighbour leaves the box: every factor is 1
                const T nb00 = o ? c00[e + 2] : c00[e];
                const T nb10 = o ? c10[e + 2] : c10[e];
                const T a00 = w0 * c00[pe] + w1 * nb00;
                const T a10 = w0 * c10[pe] + w1 * nb10;
                if (DIM == 2) {
                    v = w0 * a00 + w1 * a10;
                } else {
                    const T nb01 = o ? c01[e + 2] : c01[e];
                    const T nb11 = o ? c11[e + 2] : c11[e];
                    const T a01 = w0 * c01[pe] + w1 * nb01;
                    const T a11 = w0 * c11[pe] + w1 * nb11;
                    const T b0 = w0 * a00 + w1 * a10;
                    const T b1 = w0 * a01 + w1 * a11;
                    v = w0 * b0 + w1 * b1;
                }
            } else {
                const bool ox = (o == 0 && I0 + e == 0) || (o == 1 && I0 + e == cx - 1);
                // neighbour column: e (o = 0) or e + 2 (o = 1); the parent when out of the box
                auto col = [&](const T (&cc)[N + 2]) { return ox ? cc[pe] : (o ? cc[e + 2] : cc[e]); };
                const T a00 = w0 * c00[pe] + w1 * sv(col(c00), ox, false, false);
                const T a10 = w0 * sv(c10[pe], false, oy, false) + w1 * sv(col(c10), ox, oy, false);
                if (DIM == 2) {
                    v = w0 * a00 + w1 * a10;
                } else {
                    const T a01 = w0 * sv(c01[pe], false, false, oz) + w1 * sv(col(c01), ox, false, oz);
                    const T a11 = w0 * sv(c11[pe], false, oy, oz) + w1 * sv(col(c11), ox, oy, oz);
                    const T b0 = w0 * a00 + w1 * a10;
                    const T b1 = w0 * a01 + w1 * a11;
                    v = w0 * b0 + w1 * b1;
                }
            }
            uv.v[e] = uv.v[e] + v;
        }
        vstore<T, N>(u + own, uv);
    }
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

// First level of a two-level fixed-order sum: block b sums partials [b*chunk, (b+1)*chunk).
__global__ __launch_bounds__(1024) void k_sum_chunks(const double* __restrict__ partials, int n, int chunk,
                                                     double* __restrict__ out)
{
    __shared__ double sh[1024];
    const int lo = blockIdx.x * chunk, hi = lo + chunk < n ? lo + chunk : n;
    double a = 0.0;
    for (int i = lo + threadIdx.x; i < hi; i += 1024) a += partials[i];
    sh[threadIdx.x] = a;
    __syncthreads();
    for (int w = 512; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[blockIdx.x] = sh[0];
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

template <typename T, int D>
static void half_t(bool fine, bool err, bool vec, unsigned nb, int color, const void* other, const void* f, void* dst,
                   const void* old, double* partials, Geo g, double h, double cl, hipStream_t s)
{
    const Op<T, D> op = make_op<T, D>(h, cl);
    const T* o_ = (const T*)other;
    const T* f_ = (const T*)f;
    T* d_ = (T*)dst;
    const T* w_ = (const T*)old;
    if (vec) {
        if (fine) {
            if (err) k_half<T, D, 1, true><<<nb, kBlock, 0, s>>>(o_, f_, d_, w_, partials, g, color, op);
            else k_half<T, D, 1, false><<<nb, kBlock, 0, s>>>(o_, f_, d_, w_, partials, g, color, op);
        } else {
            if (err) k_half<T, D, 0, true><<<nb, kBlock, 0, s>>>(o_, f_, d_, w_, partials, g, color, op);
            else k_half<T, D, 0, false><<<nb, kBlock, 0, s>>>(o_, f_, d_, w_, partials, g, color, op);
        }
    } else {
        if (err) k_half_s<T, D, true><<<nb, kBlock, 0, s>>>(o_, f_, d_, w_, partials, g, color, op);
        else k_half_s<T, D, false><<<nb, kBlock, 0, s>>>(o_, f_, d_, w_, partials, g, color, op);
    }
}

hipError_t launch_half_sweep(int rb, int dim, bool fine, int color, const void* other, const void* f, void* dst,
                             const void* old, double* partials, Geo g, double h, double cl, hipStream_t s)
{
    const unsigned nb = (unsigned)half_blocks(rb, g);
    const bool err = old != nullptr, vec = half_vector(rb, g);
    if (rb == 8) {
        if (dim == 3) half_t<double, 3>(fine, err, vec, nb, color, other, f, dst, old, partials, g, h, cl, s);
        else half_t<double, 2>(fine, err, vec, nb, color, other, f, dst, old, partials, g, h, cl, s);
    } else {
        if (dim == 3) half_t<float, 3>(fine, err, vec, nb, color, other, f, dst, old, partials, g, h, cl, s);
        else half_t<float, 2>(fine, err, vec, nb, color, other, f, dst, old, partials, g, h, cl, s);
    }
    return hipGetLastError();
}

template <typename T, int D>
static void rr_t(const void* u, const void* f, void* R, Geo g, Geo gc, double h, double cl, hipStream_t s)
{
    const Op<T, D> op = make_op<T, D>(h, cl);
    constexpr int n = VN<T>::n;
    const int cx = g.nx / 2;
    const int64_t ncz = D == 3 ? g.nz / 2 : 1;
    if (cx >= n) {
        const int64_t items = (int64_t)(cx / n) * (g.ny / 2) * ncz;
        k_resrestrict<T, D><<<nblk(items), kBlock, 0, s>>>((const T*)u, (const T*)f, (T*)R, g, gc, op);
    } else {
        const int64_t items = (int64_t)cx * (g.ny / 2) * ncz;
        k_resrestrict_s<T, D><<<nblk(items), kBlock, 0, s>>>((const T*)u, (const T*)f, (T*)R, g, gc, op);
    }
}

hipError_t launch_residual_restrict(int rb, int dim, const void* u, const void* f, void* R, Geo g, Geo gc, double h,
                                    double cl, hipStream_t s)
{
    if (rb == 8) {
        if (dim == 3) rr_t<double, 3>(u, f, R, g, gc, h, cl, s);
        else rr_t<double, 2>(u, f, R, g, gc, h, cl, s);
    } else {
        if (dim == 3) rr_t<float, 3>(u, f, R, g, gc, h, cl, s);
        else rr_t<float, 2>(u, f, R, g, gc, h, cl, s);
    }
    return hipGetLastError();
}

template <typename T, int D>
static hipError_t pr_t(int linear, void* u, const void* V, Geo g, Geo gc, double clc, hipStream_t s)
{
    constexpr int n = VN<T>::n;
    if (gc.nx >= n) {
        const int64_t items = (int64_t)(gc.nx / n) * g.ny * g.nz;
        if (linear) k_prolong_v<T, D, 1><<<nblk(items), kBlock, 0, s>>>((T*)u, (const T*)V, g, gc, (T)clc);
        else k_prolong_v<T, D, 0><<<nblk(items), kBlock, 0, s>>>((T*)u, (const T*)V, g, gc, (T)clc);
        return hipGetLastError();
    }
    for (int color = 0; color < 2; ++color) {
        const unsigned nb = nblk(g.H * g.nz);
        if (linear) k_prolong<T, D, 1><<<nb, kBlock, 0, s>>>((T*)u, (const T*)V, g, gc, clc, color);
        else k_prolong<T, D, 0><<<nb, kBlock, 0, s>>>((T*)u, (const T*)V, g, gc, clc, color);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_prolong_correct(int rb, int dim, int linear, void* u, const void* V, Geo g, Geo gc, double clc,
                                  hipStream_t s)
{
    if (rb == 8) return dim == 3 ? pr_t<double, 3>(linear, u, V, g, gc, clc, s) : pr_t<double, 2>(linear, u, V, g, gc, clc, s);
    return dim == 3 ? pr_t<float, 3>(linear, u, V, g, gc, clc, s) : pr_t<float, 2>(linear, u, V, g, gc, clc, s);
}

hipError_t launch_sqdiff_sum(int rb, const void* a, const void* b, int64_t n, double* partials, double* out,
                             hipStream_t s)
{
    MGP_REAL(rb, (k_sqdiff_partial<T><<<kSumBlocks, kBlock, 0, s>>>((const T*)a, (const T*)b, n, partials)));
    k_sum_n<<<1, 1024, 0, s>>>(partials, kSumBlocks, out);
    return hipGetLastError();
}

int sum_scratch(int n) { return n <= 8192 ? 0 : (n + 8191) / 8192; }

hipError_t launch_sum_partials(const double* partials, int n, double* out, hipStream_t s)
{
    const int nb = sum_scratch(n);
    if (nb == 0) {
        k_sum_n<<<1, 1024, 0, s>>>(partials, n, out);
    } else {
        // two fixed-order levels; the first level's sums go right after the partials
        double* mid = const_cast<double*>(partials) + n;
        k_sum_chunks<<<nb, 1024, 0, s>>>(partials, n, 8192, mid);
        k_sum_n<<<1, 1024, 0, s>>>(mid, nb, out);
    }
    return hipGetLastError();
}

}  // namespace mgp
