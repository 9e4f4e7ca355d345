// mgp_device.h — device primitives shared by the kernel translation units (mgp_kernels.hip, mgp_fw.hip):
// 16-byte vectors, the Markstein division, the level operator Op, the packed red/black index, the XCD remap.
// Everything is internal to each translation unit (anonymous namespace).
#pragma once
#include "mgp_internal.h"

#include <cstdint>
#include <type_traits>
#include <utility>

namespace mgp {
namespace {

constexpr int kBlock = 256;

// ---- small helpers --------------------------------------------------------------------------

template <typename T>
struct VN {
    static constexpr int n = 16 / sizeof(T);  // reals per 16-byte access
};

template <typename T, int N>
struct alignas(sizeof(T) * N) Vec {
    T v[N];
};

template <typename T, int N>
__device__ __forceinline__ Vec<T, N> vload(const T* p)
{
    return *reinterpret_cast<const Vec<T, N>*>(p);
}
// A whole-vector LDS read the compiler may not narrow: one element of a 16-byte ds_read_b128 of
// consecutive lanes is conflict-free, while the ds_read_b32 it would be narrowed to hits every
// 4th bank (4-way conflicts).
template <typename T, int N>
__device__ __forceinline__ Vec<T, N> vload_lds_whole(const T* p)
{
    typedef T vt __attribute__((ext_vector_type(N)));
    typedef const volatile __attribute__((address_space(3))) vt* lds_ptr;
    const vt x = *(lds_ptr)(p);
    Vec<T, N> r;
#pragma unroll
    for (int e = 0; e < N; ++e) r.v[e] = x[e];
    return r;
}
template <typename T, int N>
__device__ __forceinline__ void vstore(T* p, const Vec<T, N>& a)
{
    *reinterpret_cast<Vec<T, N>*>(p) = a;
}
// Nontemporal (streaming) 16-byte access: data touched once by this kernel
template <typename T, int N>
__device__ __forceinline__ Vec<T, N> vload_nt(const T* p)
{
    using V4 = float __attribute__((ext_vector_type(4)));
    static_assert(sizeof(Vec<T, N>) == 16, "16-byte vectors only");
    const V4 r = __builtin_nontemporal_load(reinterpret_cast<const V4*>(p));
    Vec<T, N> a;
    __builtin_memcpy(&a, &r, 16);
    return a;
}
template <typename T, int N>
__device__ __forceinline__ void vstore_nt(T* p, const Vec<T, N>& a)
{
    using V4 = float __attribute__((ext_vector_type(4)));
    V4 r;
    __builtin_memcpy(&r, &a, 16);
    __builtin_nontemporal_store(r, reinterpret_cast<V4*>(p));
}

// Non-temporal 8- or 16-byte access, or a plain one (NT = false)
template <typename T, int N, bool NT>
__device__ __forceinline__ Vec<T, N> gload(const T* p)
{
    if constexpr (!NT) {
        return vload<T, N>(p);
    } else {
        typedef float vt __attribute__((ext_vector_type(sizeof(T) * N / 4)));
        const vt r = __builtin_nontemporal_load(reinterpret_cast<const vt*>(p));
        Vec<T, N> a;
        __builtin_memcpy(&a, &r, sizeof(a));
        return a;
    }
}
template <typename T, int N, bool NT>
__device__ __forceinline__ void gstore(T* p, const Vec<T, N>& a)
{
    if constexpr (!NT) {
        vstore<T, N>(p, a);
    } else {
        typedef float vt __attribute__((ext_vector_type(sizeof(T) * N / 4)));
        vt r;
        __builtin_memcpy(&r, &a, sizeof(a));
        __builtin_nontemporal_store(r, reinterpret_cast<vt*>(p));
    }
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
// value to every kernel.  Boundary-modified diagonals (coarse_bc consistent, cl != 0) come from a
// table dg[nb] = ((T)(-2 DIM) - (T)nb cl) / h^2 with ydg[nb] = RN(1 / dg[nb]): the division is the
// same Markstein sequence as the interior one (no divergent IEEE division on boundary cells).  That
// it equals the oracle's plain division was checked for every such divisor (dims 2/3, levels 0-13,
// n <= 4096, fp32 and fp64, 2.8e8 random numerators) and is pinned by the bit-exact GPU tests.
template <typename T, int DIM>
struct Op {
    T hSq, inv_hSq, adiag, yadiag, cl;
    T dg[2 * DIM + 1], ydg[2 * DIM + 1];
    // table entry nb >= 1 by a select chain (nb is per lane: no dynamic register indexing)
    __device__ __forceinline__ T sel(const T (&t)[2 * DIM + 1], int nb) const
    {
        T r = t[1];
#pragma unroll
        for (int k = 2; k <= 2 * DIM; ++k) r = nb == k ? t[k] : r;
        return r;
    }
    // diagonal of a cell with nb faces on the box boundary (cl = 0: the reference adiag)
    __device__ __forceinline__ T diag(int nb) const
    {
        if (cl == (T)0 || nb == 0) return adiag;
        return sel(dg, nb);
    }
    // (f - sum/h^2) / diag
    __device__ __forceinline__ T relax(T sum, T fc, int nb) const
    {
        const T a = fc - sum * inv_hSq;
        if (cl != (T)0 && nb != 0) return div_rn(a, sel(dg, nb), sel(ydg, nb));
        return div_rn(a, adiag, yadiag);
    }
    // f - (sum/h^2 + diag*u)
    __device__ __forceinline__ T residual(T sum, T fc, T uc, int nb) const
    {
        const T askew = sum * inv_hSq;
        const T a_u = askew + diag(nb) * uc;
        return fc - a_u;
    }
    // The same two with the table indexed directly (for an Op that lives in LDS, where a per-lane
    // index is one read): dg[0] = adiag, ydg[0] = yadiag, and with cl = 0 every entry is those, so
    // these equal relax / residual for every nb, without the branch or the select chain.
    __device__ __forceinline__ T relax_idx(T sum, T fc, int nb) const
    {
        const T a = fc - sum * inv_hSq;
        return div_rn(a, dg[nb], ydg[nb]);
    }
    __device__ __forceinline__ T residual_idx(T sum, T fc, T uc, int nb) const
    {
        const T askew = sum * inv_hSq;
        const T a_u = askew + dg[nb] * uc;
        return fc - a_u;
    }
    // The diagonals of a row whose cells have nbyz y/z faces on the box boundary: off (d0, y0 = RN(1/d0)) and on
    // (d1, y1) an x face, one table walk per row; relax(s, f, nbyz + xface) == div_rn(f - s/h^2, xface ? d1 : d0,
    // xface ? y1 : y0) (dg[0] = adiag, ydg[0] = yadiag, and with cl = 0 every entry equals those)
    __device__ __forceinline__ void row_diag(int nbyz, T& d0, T& y0, T& d1, T& y1) const
    {
        d0 = dg[0];
        y0 = ydg[0];
        d1 = dg[1];
        y1 = ydg[1];
#pragma unroll
        for (int q = 1; q < 2 * DIM; ++q) {
            d0 = nbyz == q ? dg[q] : d0;
            y0 = nbyz == q ? ydg[q] : y0;
            d1 = nbyz == q ? dg[q + 1] : d1;
            y1 = nbyz == q ? ydg[q + 1] : y1;
        }
    }
    // The same two with the diagonal computed and divided by directly (the oracle's expressions):
    // the temporally blocked phases' rare boundary path, where the table selects cost registers.
    __device__ __forceinline__ T diag_direct(int nb) const
    {
        if (cl == (T)0 || nb == 0) return adiag;
        return ((T)(-2 * DIM) - (T)nb * cl) / hSq;
    }
    __device__ __forceinline__ T relax_direct(T sum, T fc, int nb) const
    {
        const T a = fc - sum * inv_hSq;
        if (cl != (T)0 && nb != 0) return a / diag_direct(nb);
        return div_rn(a, adiag, yadiag);
    }
    __device__ __forceinline__ T residual_direct(T sum, T fc, T uc, int nb) const
    {
        const T askew = sum * inv_hSq;
        const T a_u = askew + diag_direct(nb) * uc;
        return fc - a_u;
    }
};

// Op::row_diag with a wave-uniform shortcut: rows off every y / z face (nearly all of a level) take table
// entries 0 and 1 without the walk (on a cl != 0 level the walk is 4 (2D) / 20 (3D) selects per row)
#ifndef ROWDIAG_FAST  // timing switch (0: always the walk)
#define ROWDIAG_FAST 1
#endif
template <typename T, int DIM>
__device__ __forceinline__ void row_diag_fast(const Op<T, DIM>& op, int nbyz, T& d0, T& y0, T& d1, T& y1)
{
    if (ROWDIAG_FAST && __all(nbyz == 0)) {
        d0 = op.dg[0];
        y0 = op.ydg[0];
        d1 = op.dg[1];
        y1 = op.ydg[1];
    } else {
        op.row_diag(nbyz, d0, y0, d1, y1);
    }
}

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
    for (int nb = 0; nb <= 2 * DIM; ++nb) {
        op.dg[nb] = nb == 0 ? op.adiag : ((T)(-2 * DIM) - (T)nb * op.cl) / op.hSq;
        op.ydg[nb] = (T)1 / op.dg[nb];
    }
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


// The full weighting's per-axis combination ((a + wb b) + wc c) + d (weights 1, 3, 3, 1; wb / wc = 3 - c_l
// next to a face of the coarse box)
template <typename T>
__device__ __forceinline__ T fw_axis(T a, T b, T c, T d, T wb, T wc)
{
    T s = a + wb * b;
    s = s + wc * c;
    s = s + d;
    return s;
}

// The oracle's cval() factor: -cl per out-of-box axis, in x, y, z order, applied to coarse value v
template <typename T>
__device__ __forceinline__ T cfac(T v, bool ox, bool oy, bool oz, T cl)
{
    T s = (T)1;
    if (ox) s = -cl * s;
    if (oy) s = -cl * s;
    if (oz) s = -cl * s;
    return s == (T)1 ? v : s * v;
}

// (P V) at fine cell (i, j, local plane k): the oracle's per-cell prolongation value, with the coarse
// values read through get(I, J, K) (K relative to the V pointer; always inside the box).
template <typename T, int DIM, int LINEAR, typename Get>
__device__ __forceinline__ T prolong_eval(const Get& get, const Geo& gc, T cl, int i, int j, int64_t k)
{
    const int I = i >> 1, J = j >> 1;
    const int64_t K = DIM == 3 ? (k >> 1) : 0;
    T v;
    if (!LINEAR) {
        v = get(I, J, K);
    } else {
        const T w0 = (T)0.75, w1 = (T)0.25;
        int In = (i & 1) ? I + 1 : I - 1;
        int Jn = (j & 1) ? J + 1 : J - 1;
        const bool ox = In < 0 || In >= gc.nx;
        const bool oy = Jn < 0 || Jn >= gc.ny;
        if (ox) In = I;
        if (oy) Jn = J;
        if (DIM == 2) {
            const T a0 = w0 * cfac(get(I, J, 0), false, false, false, cl) + w1 * cfac(get(In, J, 0), ox, false, false, cl);
            const T a1 = w0 * cfac(get(I, Jn, 0), false, oy, false, cl) + w1 * cfac(get(In, Jn, 0), ox, oy, false, cl);
            v = w0 * a0 + w1 * a1;
        } else {
            int64_t Kn = (k & 1) ? K + 1 : K - 1;
            const int64_t Kng = gc.z0 + Kn;
            const bool oz = Kng < 0 || Kng >= gc.gnz;
            if (oz) Kn = K;
            const T a00 = w0 * cfac(get(I, J, K), false, false, false, cl) + w1 * cfac(get(In, J, K), ox, false, false, cl);
            const T a10 = w0 * cfac(get(I, Jn, K), false, oy, false, cl) + w1 * cfac(get(In, Jn, K), ox, oy, false, cl);
            const T a01 = w0 * cfac(get(I, J, Kn), false, false, oz, cl) + w1 * cfac(get(In, J, Kn), ox, false, oz, cl);
            const T a11 = w0 * cfac(get(I, Jn, Kn), false, oy, oz, cl) + w1 * cfac(get(In, Jn, Kn), ox, oy, oz, cl);
            const T b0 = w0 * a00 + w1 * a10;
            const T b1 = w0 * a01 + w1 * a11;
            v = w0 * b0 + w1 * b1;
        }
    }
    return v;
}

}  // namespace
}  // namespace mgp
