// mgp_rbgs3d.hip — fused red/black Gauss-Seidel sweeps for 3D levels (the finest-level hot path).
//
// One launch performs NH/2 complete RB-GS sweeps (NH half-sweeps: red, black, red, ...) of a 3D
// level OUT OF PLACE: uin is only read, uout only written, so any tiling is race-free and the
// result is bit-identical to NH/2 in-place sweeps of the reference-order update
//     u = (f - ((((xl + xr) + yl) + yr) + zl) + zr) / h^2) / diag
// (cpu.lua:40-54 generalised to 3D; oracle/mgp_oracle_impl.h rbgs()).
//
// Structure (2.5D blocking, CDNA4):
//  * a 256-thread workgroup owns a TX x TY column of the level and marches a chunk of z-planes;
//  * every loaded plane keeps an NH-cell halo in x/y in LDS; stage s of the pipeline (colour
//    s & 1) updates plane t-1-s on the tile grown by NH-1-s cells, so after NH stages the tile
//    interior of plane t-NH is final and is written back once: HBM traffic per launch is one
//    read of u, one read of f and one write of u (3 s per cell) for NH/2 sweeps;
//  * LDS rows are stored split by x parity (even x | odd x), so every stage reads stride-1
//    across lanes for the centre colour and for all six neighbours (no bank conflicts);
//  * the next plane's global loads (16 B per lane) are issued before the stages of the current
//    plane and written to LDS after them (register double-buffering); the finished plane is
//    stored during the next plane's first stage;
//  * division: x / h^2 is an exact multiply by 2^(2k); (f - askew) / diag uses the correctly
//    rounded reciprocal y = RN(1/diag) and one FMA correction, q = RN(a y), q' = RN(q + RN(a - q d) y),
//    which equals the IEEE quotient RN(a / d) for operands away from over/underflow
//    (Markstein); the GPU parity tests check it bit for bit against the oracle's division;
//  * blockIdx is remapped so that each XCD works on a contiguous band of tiles (halo reuse in
//    that XCD's L2).
// Requirements (checked by the launcher): nx % TX == 0, ny % TY == 0, NH ghost planes below and
// above the interior of u and f (zeros at a physical boundary, the neighbour's planes across a
// slab edge).
#include "mgp_internal.h"

namespace mgp {
namespace {

constexpr int kThreads = 256;
constexpr int kTX = 64;

template <typename T>
struct Vec;
template <>
struct Vec<float> {
    using type = float4;
    static constexpr int n = 4;
};
template <>
struct Vec<double> {
    using type = double2;
    static constexpr int n = 2;
};

template <typename T, int NH, int TY>
struct Cfg {
    static constexpr int TX = kTX;
    static constexpr int VN = Vec<T>::n;                 // elements per 16-byte vector
    static constexpr int E = NH;                         // halo (cells) needed by stage 0
    static constexpr int XE = ((E + VN - 1) / VN) * VN;  // x halo rounded to a vector (even)
    static constexpr int PW = TX + 2 * XE;               // LDS row length (elements)
    static constexpr int HW = PW / 2;                    // half row (one x parity)
    static constexpr int PH = TY + 2 * E;                // LDS rows
    static constexpr int PS = PW * PH;                   // plane size in LDS
    static constexpr int NU = NH + 2;                    // u plane ring
    static constexpr int NF = NH + 1;                    // f plane ring
    static constexpr int VR = PW / VN;                   // vectors per row
    static constexpr int NV = VR * PH;                   // vectors per plane
    static constexpr int VPT = (NV + kThreads - 1) / kThreads;  // vectors per thread
    static constexpr size_t lds_bytes = sizeof(T) * (size_t)PS * (NU + NF);
};

template <typename T>
__device__ __forceinline__ void split_store(T* __restrict__ row, int a, const typename Vec<T>::type& v, int HW);
template <>
__device__ __forceinline__ void split_store<float>(float* __restrict__ row, int a, const float4& v, int HW)
{
    *reinterpret_cast<float2*>(row + (a >> 1)) = make_float2(v.x, v.z);
    *reinterpret_cast<float2*>(row + HW + (a >> 1)) = make_float2(v.y, v.w);
}
template <>
__device__ __forceinline__ void split_store<double>(double* __restrict__ row, int a, const double2& v, int HW)
{
    row[a >> 1] = v.x;
    row[HW + (a >> 1)] = v.y;
}

template <typename T>
__device__ __forceinline__ typename Vec<T>::type split_load(const T* __restrict__ row, int a, int HW);
template <>
__device__ __forceinline__ float4 split_load<float>(const float* __restrict__ row, int a, int HW)
{
    float2 e = *reinterpret_cast<const float2*>(row + (a >> 1));
    float2 o = *reinterpret_cast<const float2*>(row + HW + (a >> 1));
    return make_float4(e.x, o.x, e.y, o.y);
}
template <>
__device__ __forceinline__ double2 split_load<double>(const double* __restrict__ row, int a, int HW)
{
    return make_double2(row[a >> 1], row[HW + (a >> 1)]);
}

template <typename T>
__device__ __forceinline__ typename Vec<T>::type vzero();
template <>
__device__ __forceinline__ float4 vzero<float>() { return make_float4(0.f, 0.f, 0.f, 0.f); }
template <>
__device__ __forceinline__ double2 vzero<double>() { return make_double2(0.0, 0.0); }

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

struct Tile {
    int x0, y0;
    int64_t k0, k1;  // local planes [k0, k1) written by this workgroup
    bool inner;      // tile + halo strictly inside the box in x and y (no per-cell checks)
};

template <typename T, int NH, int TY>
struct Plane {
    using C = Cfg<T, NH, TY>;
    using V = typename Vec<T>::type;
    // Global loads of local plane q into registers; zeros outside the box.
    __device__ __forceinline__ static void fetch(const T* __restrict__ src, int64_t q, const Geo& g, const Tile& tl, bool valid,
                                 V (&r)[C::VPT])
    {
        const T* __restrict__ base = src + q * g.plane;
#pragma unroll
        for (int k = 0; k < C::VPT; ++k) {
            const int e = threadIdx.x + k * kThreads;
            V v = vzero<T>();
            if ((C::NV % kThreads == 0 || e < C::NV) && valid) {
                const int b = e / C::VR;
                const int a = (e - b * C::VR) * C::VN;
                const int x = tl.x0 - C::XE + a;
                const int y = tl.y0 - C::E + b;
                if (tl.inner || (x >= 0 && x < g.nx && y >= 0 && y < g.ny))
                    v = *reinterpret_cast<const V*>(base + (int64_t)y * g.nx + x);
            }
            r[k] = v;
        }
    }
    __device__ __forceinline__ static void stash(T* __restrict__ slot, const V (&r)[C::VPT])
    {
#pragma unroll
        for (int k = 0; k < C::VPT; ++k) {
            const int e = threadIdx.x + k * kThreads;
            if (C::NV % kThreads == 0 || e < C::NV) {
                const int b = e / C::VR;
                const int a = (e - b * C::VR) * C::VN;
                split_store<T>(slot + b * C::PW, a, r[k], C::HW);
            }
        }
    }
    // Tile interior of a finished plane back to HBM (16 B per lane, whole rows).  With ERR the
    // squared update against `old` (the cycle-start psi) is accumulated in fp64 (cpu.lua:203).
    template <bool ERR>
    __device__ __forceinline__ static void writeback(T* __restrict__ dst, const T* __restrict__ slot, int64_t q, const Geo& g,
                                     const Tile& tl, const T* __restrict__ old, double& acc)
    {
        constexpr int VROW = C::TX / C::VN;
        for (int e = threadIdx.x; e < VROW * TY; e += kThreads) {
            const int r = e / VROW;
            const int a = C::XE + (e - r * VROW) * C::VN;
            V v = split_load<T>(slot + (r + C::E) * C::PW, a, C::HW);
            const int64_t o = q * g.plane + (int64_t)(tl.y0 + r) * g.nx + tl.x0 + (a - C::XE);
            *reinterpret_cast<V*>(dst + o) = v;
            if (ERR) {
                V w = *reinterpret_cast<const V*>(old + o);
                const T* pv = reinterpret_cast<const T*>(&v);
                const T* pw = reinterpret_cast<const T*>(&w);
#pragma unroll
                for (int i = 0; i < C::VN; ++i) {
                    double d = (double)pv[i] - (double)pw[i];
                    acc += d * d;
                }
            }
        }
    }
};

template <int N>
__device__ __forceinline__ int slot_of(int64_t q)
{
    int s = (int)(q % N);
    return s < 0 ? s + N : s;
}

// Per-thread item table of every pipeline stage, built once per workgroup: for each unrolled
// iteration and each row-parity phase (the colour pattern flips from plane to plane) the LDS
// offset of the cell, its x parity and its count of box faces in x/y; -1 = no cell (past the
// region or outside the box).  The inner loop then does no index arithmetic at all.
template <int NH, int TY>
struct Items {
    static constexpr int MAXIT = ((TY + 2 * (NH - 1)) * (kTX / 2 + NH - 1) + kThreads - 1) / kThreads;
    int tab[NH][MAXIT][2];

    template <typename T, int S>
    __device__ __forceinline__ void build_stage(const Geo& g, const Tile& tl)
    {
        using C = Cfg<T, NH, TY>;
        constexpr int e = NH - 1 - S;
        constexpr int IR = kTX / 2 + e;
        constexpr int ITEMS = (TY + 2 * e) * IR;
#pragma unroll
        for (int k = 0; k < MAXIT; ++k) {
            const int it = threadIdx.x + k * kThreads;
            const int r = it / IR;
            const int m = it - r * IR;
            const int y = r - e;
#pragma unroll
            for (int par = 0; par < 2; ++par) {
                const int px = (par + y) & 1;
                const int x = -e + ((px + e) & 1) + 2 * m;
                const int gx = tl.x0 + x, gy = tl.y0 + y;
                int v = -1;
                if (it < ITEMS && gx >= 0 && gx < g.nx && gy >= 0 && gy < g.ny) {
                    const int same = (y + C::E) * C::PW + px * C::HW + ((x + C::XE) >> 1);
                    const int nb = (gx == 0) + (gx == g.nx - 1) + (gy == 0) + (gy == g.ny - 1);
                    v = same | (px << 16) | (nb << 17);
                }
                tab[S][k][par] = v;
            }
        }
        if constexpr (S + 1 < NH) build_stage<T, S + 1>(g, tl);
    }
    template <typename T>
    __device__ __forceinline__ void build(const Geo& g, const Tile& tl)
    {
        build_stage<T, 0>(g, tl);
    }
};

// One pipeline stage: colour c = S & 1 on plane q (neighbour planes q-1, q+1).
template <typename T, int NH, int TY, int S>
__device__ __forceinline__ void stage(T* __restrict__ lds_u, const T* __restrict__ lds_f, int64_t q, const Geo& g,
                                      const Tile& tl, const Items<NH, TY>& items, T hSq, T inv_hSq, T adiag, T yadiag,
                                      T cl)
{
    using C = Cfg<T, NH, TY>;
    constexpr int c = S & 1;  // 0 = red (first), 1 = black
    const int64_t gq = g.z0 + q;
    T* __restrict__ cur = lds_u + slot_of<C::NU>(q) * C::PS;
    const T* __restrict__ lo = lds_u + slot_of<C::NU>(q - 1) * C::PS;
    const T* __restrict__ hi = lds_u + slot_of<C::NU>(q + 1) * C::PS;
    const T* __restrict__ ff = lds_f + slot_of<C::NF>(q) * C::PS;
    const int zb = (gq == 0) + (gq == g.gnz - 1);
    const int par = (c + tl.y0 + (int)(gq & 1)) & 1;
#pragma unroll
    for (int k = 0; k < Items<NH, TY>::MAXIT; ++k) {
        int p0 = items.tab[S][k][0], p1 = items.tab[S][k][1];
        asm volatile("" : "+v"(p0), "+v"(p1));  // keep the table in registers (no load-of-select)
        const int p = par ? p1 : p0;
        if (p < 0) continue;
        const int same = p & 0xFFFF;
        const int px = (p >> 16) & 1;
        const int oth = same + (px ? 1 - C::HW : C::HW);  // x+1 neighbour; x-1 is oth - 1
        const T xl = cur[oth - 1];
        const T xr = cur[oth];
        const T yl = cur[same - C::PW];
        const T yr = cur[same + C::PW];
        const T zl = lo[same];
        const T zr = hi[same];
        const T fc = ff[same];
        T s = xl + xr;
        s = s + yl;
        s = s + yr;
        s = s + zl;
        s = s + zr;
        const T a = fc - s * inv_hSq;  // = fc - s / h^2 exactly (h^2 is a power of two)
        const int nb = (p >> 17) + zb;
        T res;
        if (cl != (T)0 && nb) {
            const T dg = ((T)(-6) - (T)nb * cl) / hSq;  // boundary cell: IEEE division as the oracle
            res = a / dg;
        } else {
            res = div_rn(a, adiag, yadiag);
        }
        cur[same] = res;
    }
}

template <typename T, int NH, int TY, int S>
struct Stages {
    __device__ __forceinline__ static void run(T* lds_u, const T* lds_f, int64_t t, const Geo& g, const Tile& tl,
                               const Items<NH, TY>& items, T hSq, T inv_hSq, T adiag, T yadiag, T cl)
    {
        const int64_t q = t - 1 - S;
        constexpr int e = NH - 1 - S;
        if (q >= tl.k0 - e && q <= tl.k1 - 1 + e && g.z0 + q >= 0 && g.z0 + q < g.gnz)
            stage<T, NH, TY, S>(lds_u, lds_f, q, g, tl, items, hSq, inv_hSq, adiag, yadiag, cl);
        __syncthreads();
        Stages<T, NH, TY, S + 1>::run(lds_u, lds_f, t, g, tl, items, hSq, inv_hSq, adiag, yadiag, cl);
    }
};
template <typename T, int NH, int TY>
struct Stages<T, NH, TY, NH> {
    __device__ static void run(T*, const T*, int64_t, const Geo&, const Tile&, const Items<NH, TY>&, T, T, T, T, T) {}
};

template <typename T, int NH, int TY, bool ERR>
struct Marcher {
    using C = Cfg<T, NH, TY>;
    using V = typename Vec<T>::type;
    using P = Plane<T, NH, TY>;
    const T* __restrict__ uin;
    const T* __restrict__ f;
    T* __restrict__ uout;
    const T* __restrict__ old;
    const Geo& g;
    const Tile& tl;
    T* lds_u;
    T* lds_f;
    T hSq, inv_hSq, adiag, yadiag, cl;
    int64_t tfirst, tlast;
    Items<NH, TY> items;
    double acc = 0.0;

    __device__ __forceinline__ bool planeok(int64_t q) const { return g.z0 + q >= 0 && g.z0 + q < g.gnz; }

    // One z-step: plane t enters LDS (registers ru/rf are then refilled with plane t + 2),
    // plane t-1-NH leaves to HBM, and the NH stages advance the pipeline.
    __device__ __forceinline__ void step(int64_t t, V (&ru)[C::VPT], V (&rf)[C::VPT])
    {
        P::stash(lds_u + slot_of<C::NU>(t) * C::PS, ru);
        P::stash(lds_f + slot_of<C::NF>(t) * C::PS, rf);
        if (t + 2 <= tlast) {  // prefetch depth 2: two planes of loads in flight per workgroup
            P::fetch(uin, t + 2, g, tl, planeok(t + 2), ru);
            P::fetch(f, t + 2, g, tl, planeok(t + 2), rf);
        }
        __syncthreads();
        const int64_t qo = t - 1 - NH;
        if (qo >= tl.k0 && qo < tl.k1)
            P::template writeback<ERR>(uout, lds_u + slot_of<C::NU>(qo) * C::PS, qo, g, tl, old, acc);
        Stages<T, NH, TY, 0>::run(lds_u, lds_f, t, g, tl, items, hSq, inv_hSq, adiag, yadiag, cl);
    }

    __device__ __forceinline__ void run()
    {
        items.template build<T>(g, tl);
        V ru0[C::VPT], rf0[C::VPT], ru1[C::VPT], rf1[C::VPT];
        P::fetch(uin, tfirst, g, tl, planeok(tfirst), ru0);
        P::fetch(f, tfirst, g, tl, planeok(tfirst), rf0);
        P::fetch(uin, tfirst + 1, g, tl, planeok(tfirst + 1), ru1);  // tlast >= tfirst + 2 NH
        P::fetch(f, tfirst + 1, g, tl, planeok(tfirst + 1), rf1);
        for (int64_t t = tfirst; t <= tlast; t += 2) {
            step(t, ru0, rf0);
            if (t + 1 <= tlast) step(t + 1, ru1, rf1);
        }
        const int64_t qo = tlast - NH;
        if (qo >= tl.k0 && qo < tl.k1)
            P::template writeback<ERR>(uout, lds_u + slot_of<C::NU>(qo) * C::PS, qo, g, tl, old, acc);
    }
};

template <typename T, int NH, int TY, bool ERR>
__device__ __forceinline__ double march(const T* __restrict__ uin, const T* __restrict__ f, T* __restrict__ uout,
                                        const T* __restrict__ old, const Geo& g, const Tile& tl, T* lds_u, T* lds_f,
                                        double h, double cld)
{
    Marcher<T, NH, TY, ERR> m{uin, f, uout, old, g, tl, lds_u, lds_f};
    const T hh = (T)h;
    m.hSq = hh * hh;
    m.inv_hSq = (T)1 / m.hSq;  // exact: h is a power of two
    m.adiag = (T)(-6) / m.hSq;
    m.yadiag = (T)1 / m.adiag;  // RN(1/adiag)
    m.cl = (T)cld;
    m.tfirst = tl.k0 - NH;
    m.tlast = tl.k1 - 1 + NH;
    m.run();
    return m.acc;
}

template <typename T, int NH, int TY, int TAG, bool ERR>
__global__ __launch_bounds__(kThreads) void k_rbgs_fused3d(const T* __restrict__ uin, const T* __restrict__ f,
                                                           T* __restrict__ uout, const T* __restrict__ old,
                                                           double* __restrict__ partials, Geo g, int kc,
                                                           int xcd_chunk, double h, double cld)
{
    using C = Cfg<T, NH, TY>;
    extern __shared__ __align__(16) unsigned char smem[];
    T* lds_u = reinterpret_cast<T*>(smem);
    T* lds_f = lds_u + C::NU * C::PS;

    // XCD-aware remap: blocks b and b+8 share an XCD; give each XCD a contiguous band of tiles.
    int b = blockIdx.x;
    if (xcd_chunk > 0) b = (b & 7) * xcd_chunk + (b >> 3);
    const int ntx = g.nx / kTX, nty = g.ny / TY;
    const int tx = b % ntx;
    const int rest = b / ntx;
    const int ty = rest % nty;
    const int kch = rest / nty;
    Tile tl;
    tl.x0 = tx * kTX;
    tl.y0 = ty * TY;
    tl.k0 = (int64_t)kch * kc;
    tl.k1 = tl.k0 + kc < g.nz ? tl.k0 + kc : g.nz;
    tl.inner = tl.x0 - C::XE >= 0 && tl.x0 + kTX + C::XE <= g.nx && tl.y0 - C::E >= 0 && tl.y0 + TY + C::E <= g.ny;
    const double acc = march<T, NH, TY, ERR>(uin, f, uout, old, g, tl, lds_u, lds_f, h, cld);
    if (ERR) {  // fixed-order block reduction -> one fp64 partial per workgroup
        __syncthreads();
        double* red = reinterpret_cast<double*>(smem);
        red[threadIdx.x] = acc;
        __syncthreads();
        for (int w = kThreads / 2; w > 0; w >>= 1) {
            if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
            __syncthreads();
        }
        if (threadIdx.x == 0) partials[blockIdx.x] = red[0];
    }
}

template <typename T, int NH, int TY, int TAG, bool ERR>
hipError_t launch_cfg(const void* uin, const void* f, void* uout, const void* old, double* partials, Geo g, int kc,
                      double h, double cl, hipStream_t s)
{
    using C = Cfg<T, NH, TY>;
    const int nblocks = fused3d_blocks(g, TY, kc);
    const int xcd_chunk = (nblocks % 8 == 0) ? nblocks / 8 : 0;
    static bool attr_done = false;
    if (!attr_done) {
        hipError_t e = hipFuncSetAttribute((const void*)k_rbgs_fused3d<T, NH, TY, TAG, ERR>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)C::lds_bytes);
        if (e != hipSuccess) return e;
        attr_done = true;
    }
    k_rbgs_fused3d<T, NH, TY, TAG, ERR><<<nblocks, kThreads, C::lds_bytes, s>>>(
        (const T*)uin, (const T*)f, (T*)uout, (const T*)old, partials, g, kc, xcd_chunk, h, cl);
    return hipGetLastError();
}

template <typename T, int TAG, bool ERR>
hipError_t launch_t(int nh, int ty, const void* uin, const void* f, void* uout, const void* old, double* partials,
                    Geo g, int kc, double h, double cl, hipStream_t s)
{
    if (nh == 4) {
        if (ty == 16) return launch_cfg<T, 4, 16, TAG, ERR>(uin, f, uout, old, partials, g, kc, h, cl, s);
        return launch_cfg<T, 4, 8, TAG, ERR>(uin, f, uout, old, partials, g, kc, h, cl, s);
    }
    if (ty == 16) return launch_cfg<T, 2, 16, TAG, ERR>(uin, f, uout, old, partials, g, kc, h, cl, s);
    return launch_cfg<T, 2, 8, TAG, ERR>(uin, f, uout, old, partials, g, kc, h, cl, s);
}

template <typename T, int TAG>
hipError_t launch_e(int nh, int ty, const void* uin, const void* f, void* uout, const void* old, double* partials,
                    Geo g, int kc, double h, double cl, hipStream_t s)
{
    if (old) return launch_t<T, TAG, true>(nh, ty, uin, f, uout, old, partials, g, kc, h, cl, s);
    return launch_t<T, TAG, false>(nh, ty, uin, f, uout, old, partials, g, kc, h, cl, s);
}

// ---------------------------------------------------------------------------------------------
// Fused residual + restriction for 3D levels (calcResidual + reduceResidual, gpu.lua:104-137):
// a workgroup owns a 64 x 16 fine tile (32 x 8 coarse cells, one per thread) and marches pairs
// of fine planes; u planes carry a 1-cell halo in LDS (x-parity split rows, conflict-free), the
// fine residual never touches HBM.  Per coarse cell:
//   r = f - (askew + diag * u),  R = 1/8 (((((((r000 + r100) + r010) + r110) + r001) + r101) + r011) + r111)
// exactly as oracle/mgp_oracle_impl.h residual() + restrict_().
template <typename T, int TY>
struct RCfg {
    static constexpr int TX = kTX;
    static constexpr int VN = Vec<T>::n;
    static constexpr int E = 1;
    static constexpr int XE = VN;                 // 1-cell halo rounded to a vector
    static constexpr int PW = TX + 2 * XE;
    static constexpr int HW = PW / 2;
    static constexpr int PH = TY + 2 * E;
    static constexpr int PS = PW * PH;
    static constexpr int VR = PW / VN;
    static constexpr int NV = VR * PH;
    static constexpr int VPT = (NV + kThreads - 1) / kThreads;
    static constexpr size_t lds_bytes = sizeof(T) * (size_t)PS * 6;  // 4 u planes + 2 f planes
};

template <typename T, int TY>
struct RPlane {
    using C = RCfg<T, TY>;
    using V = typename Vec<T>::type;
    __device__ __forceinline__ static void fetch(const T* __restrict__ src, int64_t q, const Geo& g, int x0, int y0, bool inner,
                                 bool valid, V (&r)[C::VPT])
    {
        const T* __restrict__ base = src + q * g.plane;
#pragma unroll
        for (int k = 0; k < C::VPT; ++k) {
            const int e = threadIdx.x + k * kThreads;
            V v = vzero<T>();
            if ((C::NV % kThreads == 0 || e < C::NV) && valid) {
                const int b = e / C::VR;
                const int a = (e - b * C::VR) * C::VN;
                const int x = x0 - C::XE + a;
                const int y = y0 - C::E + b;
                if (inner || (x >= 0 && x < g.nx && y >= 0 && y < g.ny))
                    v = *reinterpret_cast<const V*>(base + (int64_t)y * g.nx + x);
            }
            r[k] = v;
        }
    }
    __device__ __forceinline__ static void stash(T* __restrict__ slot, const V (&r)[C::VPT])
    {
#pragma unroll
        for (int k = 0; k < C::VPT; ++k) {
            const int e = threadIdx.x + k * kThreads;
            if (C::NV % kThreads == 0 || e < C::NV) {
                const int b = e / C::VR;
                const int a = (e - b * C::VR) * C::VN;
                split_store<T>(slot + b * C::PW, a, r[k], C::HW);
            }
        }
    }
};

template <typename T, int TY>
__global__ __launch_bounds__(kThreads) void k_residual_restrict3d(const T* __restrict__ u, const T* __restrict__ f,
                                                                  T* __restrict__ R, Geo g, int kcc, int xcd_chunk,
                                                                  double h, double cld)
{
    using C = RCfg<T, TY>;
    using V = typename Vec<T>::type;
    using P = RPlane<T, TY>;
    extern __shared__ __align__(16) unsigned char smem[];
    T* lds_u = reinterpret_cast<T*>(smem);  // 4 slots: fine plane q in slot q & 3
    T* lds_f = lds_u + 4 * C::PS;           // 2 slots: fine plane q in slot q & 1

    int b = blockIdx.x;
    if (xcd_chunk > 0) b = (b & 7) * xcd_chunk + (b >> 3);
    const int ntx = g.nx / kTX, nty = g.ny / TY;
    const int tx = b % ntx;
    const int rest = b / ntx;
    const int ty = rest % nty;
    const int kch = rest / nty;
    const int x0 = tx * kTX, y0 = ty * TY;
    const int64_t ncz = g.nz >> 1;
    const int64_t K0 = (int64_t)kch * kcc;
    const int64_t K1 = K0 + kcc < ncz ? K0 + kcc : ncz;
    const bool inner = x0 - C::XE >= 0 && x0 + kTX + C::XE <= g.nx && y0 - 1 >= 0 && y0 + TY + 1 <= g.ny;

    const T hh = (T)h;
    const T hSq = hh * hh;
    const T inv_hSq = (T)1 / hSq;
    const T adiag = (T)(-6) / hSq;
    const T cl = (T)cld;
    const int cx = g.nx >> 1, cy = g.ny >> 1;
    const int64_t cplane = (int64_t)cx * cy;
    auto planeok = [&](int64_t q) { return g.z0 + q >= 0 && g.z0 + q < g.gnz; };

    // thread -> coarse cell (I, J) of the 32 x (TY/2) coarse tile
    const int I = threadIdx.x & 31;
    const int J = threadIdx.x >> 5;  // 0 .. 7 for TY = 16
    V ru0[C::VPT], ru1[C::VPT], rf0[C::VPT], rf1[C::VPT];
    // prologue: u planes 2K0-1 .. 2K0+2, f planes 2K0, 2K0+1
    {
        V t0[C::VPT], t1[C::VPT];
        P::fetch(u, 2 * K0 - 1, g, x0, y0, inner, planeok(2 * K0 - 1), t0);
        P::fetch(u, 2 * K0, g, x0, y0, inner, planeok(2 * K0), t1);
        P::stash(lds_u + ((2 * K0 - 1) & 3) * C::PS, t0);
        P::stash(lds_u + ((2 * K0) & 3) * C::PS, t1);
    }
    P::fetch(u, 2 * K0 + 1, g, x0, y0, inner, planeok(2 * K0 + 1), ru0);
    P::fetch(u, 2 * K0 + 2, g, x0, y0, inner, planeok(2 * K0 + 2), ru1);
    P::fetch(f, 2 * K0, g, x0, y0, inner, true, rf0);
    P::fetch(f, 2 * K0 + 1, g, x0, y0, inner, true, rf1);
    for (int64_t K = K0; K < K1; ++K) {
        const int64_t q0 = 2 * K;
        P::stash(lds_u + ((q0 + 1) & 3) * C::PS, ru0);
        P::stash(lds_u + ((q0 + 2) & 3) * C::PS, ru1);
        P::stash(lds_f + (q0 & 1) * C::PS, rf0);
        P::stash(lds_f + ((q0 + 1) & 1) * C::PS, rf1);
        if (K + 1 < K1) {
            P::fetch(u, q0 + 3, g, x0, y0, inner, planeok(q0 + 3), ru0);
            P::fetch(u, q0 + 4, g, x0, y0, inner, planeok(q0 + 4), ru1);
            P::fetch(f, q0 + 2, g, x0, y0, inner, true, rf0);
            P::fetch(f, q0 + 3, g, x0, y0, inner, true, rf1);
        }
        __syncthreads();
        T r[8];
#pragma unroll
        for (int dz = 0; dz < 2; ++dz) {
            const int64_t q = q0 + dz;
            const T* cur = lds_u + (q & 3) * C::PS;
            const T* lo = lds_u + ((q - 1) & 3) * C::PS;
            const T* hi = lds_u + ((q + 1) & 3) * C::PS;
            const T* ff = lds_f + (q & 1) * C::PS;
            const int64_t gq = g.z0 + q;
            const int zb = (gq == 0) + (gq == g.gnz - 1);
#pragma unroll
            for (int dy = 0; dy < 2; ++dy) {
                const int y = 2 * J + dy;
                const int rowo = (y + 1) * C::PW;
#pragma unroll
                for (int dx = 0; dx < 2; ++dx) {
                    const int x = 2 * I + dx;
                    const int px = dx;  // x0 even
                    const int same = rowo + px * C::HW + ((x + C::XE) >> 1);
                    const int oth = same + (1 - 2 * px) * C::HW + px;
                    T s = cur[oth - 1] + cur[oth];
                    s = s + cur[same - C::PW];
                    s = s + cur[same + C::PW];
                    s = s + lo[same];
                    s = s + hi[same];
                    T dg = adiag;
                    if (cl != (T)0) {
                        const int gx = x0 + x, gy = y0 + y;
                        const int nb = (gx == 0) + (gx == g.nx - 1) + (gy == 0) + (gy == g.ny - 1) + zb;
                        if (nb) dg = ((T)(-6) - (T)nb * cl) / hSq;
                    }
                    const T askew = s * inv_hSq;
                    const T a_u = askew + dg * cur[same];
                    r[dz * 4 + dy * 2 + dx] = ff[same] - a_u;
                }
            }
        }
        T acc = r[0] + r[1];
#pragma unroll
        for (int i = 2; i < 8; ++i) acc = acc + r[i];
        R[K * cplane + (int64_t)((y0 >> 1) + J) * cx + (x0 >> 1) + I] = (T)0.125 * acc;
        __syncthreads();
    }
}

// Vectorised u += P V for 3D levels: a thread owns 4 consecutive fine x-cells (one 16-B access
// of u for fp32) and gathers the coarse samples they share.  Same per-cell expression as
// k_prolong_correct / oracle prolong_correct().
template <typename T, int LINEAR>
__global__ __launch_bounds__(kThreads) void k_prolong3d_x4(T* __restrict__ u, const T* __restrict__ V, Geo g,
                                                           Geo gc, double clc)
{
    const int64_t n4 = (g.plane * g.nz) >> 2;
    const int64_t idx = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (idx >= n4) return;
    const int64_t c0 = idx << 2;
    const int i0 = (int)(c0 & (g.nx - 1));
    const int j = (int)((c0 >> g.lx) & (g.ny - 1));
    const int64_t k = c0 >> (g.lx + g.ly);
    const int cx = gc.nx;
    const int64_t cplane = gc.plane;
    const int I0 = i0 >> 1;  // parents I0 (cells i0, i0+1) and I0 + 1 (cells i0+2, i0+3)
    const int J = j >> 1;
    const int64_t K = k >> 1;
    T out[4];
    if (!LINEAR) {
        const T* row = V + (int64_t)cx * J + cplane * K;
        const T va = row[I0], vb = row[I0 + 1];
        out[0] = va;
        out[1] = va;
        out[2] = vb;
        out[3] = vb;
    } else {
        const T w0 = (T)0.75, w1 = (T)0.25, cl = (T)clc;
        int Jn = (j & 1) ? J + 1 : J - 1;
        const bool oy = Jn < 0 || Jn >= gc.ny;
        if (oy) Jn = J;
        int64_t Kn = (k & 1) ? K + 1 : K - 1;
        const int64_t Kng = gc.z0 + Kn;
        const bool oz = Kng < 0 || Kng >= gc.gnz;
        if (oz) Kn = K;
        const bool oxl = I0 - 1 < 0, oxr = I0 + 2 >= cx;
        const int il = oxl ? I0 : I0 - 1, ir = oxr ? I0 + 1 : I0 + 2;
        // coarse x samples il, I0, I0+1, ir on the four (J', K') rows; the oracle's per-cell factor
        // s multiplies by -cl once per out-of-box axis in x, y, z order (cval())
        T c[4][4];
        const int64_t rows[4] = {(int64_t)cx * J + cplane * K, (int64_t)cx * Jn + cplane * K,
                                 (int64_t)cx * J + cplane * Kn, (int64_t)cx * Jn + cplane * Kn};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const T* row = V + rows[r];
            c[r][0] = row[il];
            c[r][1] = row[I0];
            c[r][2] = row[I0 + 1];
            c[r][3] = row[ir];
        }
        auto sv = [&](T v, bool ox, bool yy, bool zz) {
            T s = (T)1;
            if (ox) s = -cl * s;
            if (yy) s = -cl * s;
            if (zz) s = -cl * s;
            return s == (T)1 ? v : s * v;
        };
        // fine cell e: parent column pc, neighbour column nc (indices into c[r][.])
        const int pcol[4] = {1, 1, 2, 2};
        const int ncol[4] = {0, 2, 1, 3};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const bool ox = (e == 0 && oxl) || (e == 3 && oxr);
            const int p = pcol[e], q = ncol[e];
            T a00 = w0 * sv(c[0][p], false, false, false) + w1 * sv(c[0][q], ox, false, false);
            T a10 = w0 * sv(c[1][p], false, oy, false) + w1 * sv(c[1][q], ox, oy, false);
            T a01 = w0 * sv(c[2][p], false, false, oz) + w1 * sv(c[2][q], ox, false, oz);
            T a11 = w0 * sv(c[3][p], false, oy, oz) + w1 * sv(c[3][q], ox, oy, oz);
            T b0 = w0 * a00 + w1 * a10;
            T b1 = w0 * a01 + w1 * a11;
            out[e] = w0 * b0 + w1 * b1;
        }
    }
    T* p = u + c0;
    if (sizeof(T) == 4) {
        float4 v = *reinterpret_cast<float4*>(p);
        v.x = v.x + (float)out[0];
        v.y = v.y + (float)out[1];
        v.z = v.z + (float)out[2];
        v.w = v.w + (float)out[3];
        *reinterpret_cast<float4*>(p) = v;
    } else {
        double2 a = *reinterpret_cast<double2*>(p);
        double2 b = *reinterpret_cast<double2*>(p + 2);
        a.x = a.x + (double)out[0];
        a.y = a.y + (double)out[1];
        b.x = b.x + (double)out[2];
        b.y = b.y + (double)out[3];
        *reinterpret_cast<double2*>(p) = a;
        *reinterpret_cast<double2*>(p + 2) = b;
    }
}

template <typename T>
hipError_t launch_rr(const void* u, const void* f, void* R, Geo g, int kcc, double h, double cl, hipStream_t s)
{
    constexpr int TY = 16;
    using C = RCfg<T, TY>;
    const int nblocks = (g.nx / kTX) * (g.ny / TY) * (int)(((g.nz >> 1) + kcc - 1) / kcc);
    const int xcd_chunk = (nblocks % 8 == 0) ? nblocks / 8 : 0;
    k_residual_restrict3d<T, TY><<<nblocks, kThreads, C::lds_bytes, s>>>((const T*)u, (const T*)f, (T*)R, g, kcc,
                                                                        xcd_chunk, h, cl);
    return hipGetLastError();
}

}  // namespace

int fused3d_blocks(Geo g, int ty, int kc)
{
    return (g.nx / kTX) * (g.ny / ty) * (int)((g.nz + kc - 1) / kc);
}

bool rbgs_fused3d_supported(int rb, int nh, int ty, Geo g)
{
    (void)rb;
    if (nh != 2 && nh != 4) return false;
    if (ty != 8 && ty != 16) return false;
    return g.nx % kTX == 0 && g.ny % ty == 0 && g.nz >= 1;
}

bool residual_restrict3d_supported(Geo g) { return g.nx % kTX == 0 && g.ny % 16 == 0 && g.nz >= 2 && (g.nz & 1) == 0; }

hipError_t launch_residual_restrict3d(int rb, const void* u, const void* f, void* R, Geo g, double h, double cl,
                                      hipStream_t s)
{
    const int kcc = 16;
    return rb == 4 ? launch_rr<float>(u, f, R, g, kcc, h, cl, s) : launch_rr<double>(u, f, R, g, kcc, h, cl, s);
}

bool prolong3d_x4_supported(Geo g) { return g.nx >= 4; }

hipError_t launch_prolong3d_x4(int rb, int linear, void* u, const void* V, Geo g, Geo gc, double clc, hipStream_t s)
{
    const int64_t n4 = (g.plane * g.nz) >> 2;
    const unsigned blocks = (unsigned)((n4 + kThreads - 1) / kThreads);
    if (rb == 4) {
        if (linear) k_prolong3d_x4<float, 1><<<blocks, kThreads, 0, s>>>((float*)u, (const float*)V, g, gc, clc);
        else k_prolong3d_x4<float, 0><<<blocks, kThreads, 0, s>>>((float*)u, (const float*)V, g, gc, clc);
    } else {
        if (linear) k_prolong3d_x4<double, 1><<<blocks, kThreads, 0, s>>>((double*)u, (const double*)V, g, gc, clc);
        else k_prolong3d_x4<double, 0><<<blocks, kThreads, 0, s>>>((double*)u, (const double*)V, g, gc, clc);
    }
    return hipGetLastError();
}

hipError_t launch_rbgs_fused3d(int rb, bool fine, int nh, int ty, const void* uin, const void* f, void* uout,
                               const void* old, double* partials, Geo g, int kc, double h, double cl, hipStream_t s)
{
    if (kc <= 0) kc = 32;
    if (rb == 4)
        return fine ? launch_e<float, 1>(nh, ty, uin, f, uout, old, partials, g, kc, h, cl, s)
                    : launch_e<float, 0>(nh, ty, uin, f, uout, old, partials, g, kc, h, cl, s);
    return fine ? launch_e<double, 1>(nh, ty, uin, f, uout, old, partials, g, kc, h, cl, s)
                : launch_e<double, 0>(nh, ty, uin, f, uout, old, partials, g, kc, h, cl, s);
}

}  // namespace mgp
