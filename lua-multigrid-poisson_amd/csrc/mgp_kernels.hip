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
#include "mgp_device.h"

#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <utility>

namespace mgp {
namespace {

// (kBlock, vectors, div_rn, Op, pidx, xcd_remap, block_partial, fw_axis: mgp_device.h)

// ---- init / pack / unpack -------------------------------------------------------------------

// thread per packed slot: slot -> (k, c, j, m) -> i = 2m + (c ^ parity); i >= nx only when nx = 1.  A plane stride
// beyond 2 H (MGP_PLANE_PAD) leaves pad slots after each plane's two halves: no cell (they stay 0)
__device__ __forceinline__ bool slot_cell(int64_t s, const Geo& g, int& i, int& j, int64_t& k)
{
    int64_t r = s;
    bool pad = false;
    if (g.P == 2 * g.H) {
        k = s >> (g.lhw + g.ly + 1);
    } else {
        k = s / g.P;
        r = s - k * g.P;
        pad = r >= 2 * g.H;
    }
    const int m = (int)(r & (g.hw - 1));
    j = (int)((r >> g.lhw) & (g.ny - 1));
    const int c = (int)((r >> (g.lhw + g.ly)) & 1);
    const int p = (int)((j + g.z0 + k) & 1);
    i = 2 * m + (c ^ p);
    return i < g.nx && !pad;
}

// Element-wise kernels over every packed slot of a level run grid-stride over at most kMaxBlocks
// workgroups: a 4096 x 4096 x 512 slab has 8.6e9 slots, past the 2^32 work-items one launch allows.
constexpr unsigned kMaxBlocks = 1u << 20;
inline unsigned nblk_gs(int64_t n)
{
    const int64_t b = (n + kBlock - 1) / kBlock;
    return (unsigned)(b < (int64_t)kMaxBlocks ? (b > 0 ? b : 1) : kMaxBlocks);
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_init(T* __restrict__ u, T* __restrict__ f, Geo g, int64_t cx, int64_t cy,
                                                 int64_t cz, int dim3)
{
    const int64_t n = g.P * g.nz;
    for (int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x; s < n; s += (int64_t)gridDim.x * kBlock) {
        int i, j;
        int64_t k;
        const bool cell = slot_cell(s, g, i, j, k);
        const double charge = 1e+6, epsilon0 = 1;
        const bool hit = cell && i == cx && j == cy && (!dim3 || g.z0 + k == cz);
        const T v = hit ? (T)(-charge / epsilon0) : (T)0;
        f[s] = v;
        u[s] = -v;  // psi = -f (cpu.lua:193): -0.0 off the charge, as in the oracle
    }
}

// lex: planes 0 .. g.nz-1 of the (sub)slab described by g (g.z0 = global index of its plane 0)
template <typename T>
__global__ __launch_bounds__(kBlock) void k_pack(const T* __restrict__ lex, T* __restrict__ out, Geo g)
{
    const int64_t n = g.P * g.nz;
    for (int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x; s < n; s += (int64_t)gridDim.x * kBlock) {
        int i, j;
        int64_t k;
        out[s] = slot_cell(s, g, i, j, k) ? lex[(k * g.ny + j) * (int64_t)g.nx + i] : (T)0;
    }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_unpack(const T* __restrict__ in, T* __restrict__ lex, Geo g)
{
    const int64_t n = g.P * g.nz;
    for (int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x; s < n; s += (int64_t)gridDim.x * kBlock) {
        int i, j;
        int64_t k;
        if (slot_cell(s, g, i, j, k)) lex[(k * g.ny + j) * (int64_t)g.nx + i] = in[s];
    }
}

// Order-independent fingerprint of a field (mgp_field_stats): per cell a 64-bit mix of its bit
// pattern and its global lexicographic index, summed modulo 2^64, so two fields have the same
// hash exactly when (with overwhelming probability) every cell is bit-identical, whatever the
// slab decomposition or reduction order.  Alongside: fp64 sum, sum of squares and max |x|.
__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

template <typename T>
__device__ __forceinline__ uint64_t real_bits(T v)
{
    if constexpr (sizeof(T) == 8) {
        uint64_t b;
        __builtin_memcpy(&b, &v, 8);
        return b;
    } else {
        uint32_t b;
        __builtin_memcpy(&b, &v, 4);
        return b;
    }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_field_stats(const T* __restrict__ in, Geo g, uint64_t* __restrict__ hpart,
                                                        double* __restrict__ dpart)
{
    const int64_t n = g.P * g.nz;
    uint64_t h = 0;
    double s = 0.0, q = 0.0, mx = 0.0;
    for (int64_t x = (int64_t)blockIdx.x * kBlock + threadIdx.x; x < n; x += (int64_t)gridDim.x * kBlock) {
        int i, j;
        int64_t k;
        if (!slot_cell(x, g, i, j, k)) continue;
        const T v = in[x];
        const uint64_t gi = ((uint64_t)(g.z0 + k) * (uint64_t)g.ny + (uint64_t)j) * (uint64_t)g.nx + (uint64_t)i;
        h += mix64(real_bits(v) ^ mix64(gi));
        const double d = (double)v;
        s += d;
        q += d * d;
        mx = fmax(mx, fabs(d));
    }
    __shared__ uint64_t sh[kBlock];
    __shared__ double sd[3][kBlock];
    sh[threadIdx.x] = h;
    sd[0][threadIdx.x] = s;
    sd[1][threadIdx.x] = q;
    sd[2][threadIdx.x] = mx;
    __syncthreads();
    for (int w = kBlock / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            sh[threadIdx.x] += sh[threadIdx.x + w];
            sd[0][threadIdx.x] += sd[0][threadIdx.x + w];
            sd[1][threadIdx.x] += sd[1][threadIdx.x + w];
            sd[2][threadIdx.x] = fmax(sd[2][threadIdx.x], sd[2][threadIdx.x + w]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        hpart[blockIdx.x] = sh[0];
        for (int c = 0; c < 3; ++c) dpart[c * gridDim.x + blockIdx.x] = sd[c][0];
    }
}

// one workgroup: the nb partials of k_field_stats -> out_h[0], out_d[0..2]
__global__ __launch_bounds__(kBlock) void k_field_stats_final(const uint64_t* __restrict__ hpart,
                                                              const double* __restrict__ dpart, int nb,
                                                              uint64_t* __restrict__ out_h, double* __restrict__ out_d)
{
    uint64_t h = 0;
    double s = 0.0, q = 0.0, mx = 0.0;
    for (int b = threadIdx.x; b < nb; b += kBlock) {
        h += hpart[b];
        s += dpart[b];
        q += dpart[nb + b];
        mx = fmax(mx, dpart[2 * nb + b]);
    }
    __shared__ uint64_t sh[kBlock];
    __shared__ double sd[3][kBlock];
    sh[threadIdx.x] = h;
    sd[0][threadIdx.x] = s;
    sd[1][threadIdx.x] = q;
    sd[2][threadIdx.x] = mx;
    __syncthreads();
    for (int w = kBlock / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            sh[threadIdx.x] += sh[threadIdx.x + w];
            sd[0][threadIdx.x] += sd[0][threadIdx.x + w];
            sd[1][threadIdx.x] += sd[1][threadIdx.x + w];
            sd[2][threadIdx.x] = fmax(sd[2][threadIdx.x], sd[2][threadIdx.x + w]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out_h[0] = sh[0];
        out_d[0] = sd[0][0];
        out_d[1] = sd[1][0];
        out_d[2] = sd[2][0];
    }
}

// ---- red/black half-sweep -------------------------------------------------------------------

// Vector form: a thread owns N consecutive cells of colour `color` in one row (hw % N == 0).
// half_load gathers an item's operands (all loads issued), half_store computes and stores it, so
// a thread can keep several items' loads in flight.
template <typename T, int N>
struct HalfIn {
    Vec<T, N> cen, yl, yr, zl, zr, fv;
    T edge;
    int64_t own;
    int o, j, nbyz, m0;
    int64_t gk;
};

template <typename T, int DIM, bool NT = false>
__device__ __forceinline__ void half_load(HalfIn<T, VN<T>::n>& in, const T* __restrict__ other, const T* __restrict__ f,
                                          const Geo& g, int color, int64_t it)
{
    constexpr int N = VN<T>::n;
    constexpr int LN = N == 4 ? 2 : 1;
    const int lgpr = g.lhw - LN;  // log2 groups per row
    const int grp = (int)(it & ((1 << lgpr) - 1));
    const int j = (int)((it >> lgpr) & (g.ny - 1));
    const int64_t k = it >> (lgpr + g.ly);
    const int m0 = grp * N;
    const int64_t gk = g.z0 + k;
    const int o = color ^ (int)((j + gk) & 1);  // x parity of this row's colour-c cells
    const int64_t own = k * g.P + color * g.H + (int64_t)j * g.hw + m0;
    const int64_t oth = k * g.P + (color ^ 1) * g.H + (int64_t)j * g.hw + m0;
    in.cen = vload<T, N>(other + oth);
    if (o == 0)
        in.edge = m0 > 0 ? other[oth - 1] : (T)0;      // x-1 of the first cell
    else
        in.edge = m0 + N < g.hw ? other[oth + N] : (T)0;  // x+1 of the last cell
    in.yl = j > 0 ? vload<T, N>(other + oth - g.hw) : vzero<T, N>();
    in.yr = j < g.ny - 1 ? vload<T, N>(other + oth + g.hw) : vzero<T, N>();
    if (DIM == 3) {
        in.zl = vload<T, N>(other + oth - g.P);
        in.zr = vload<T, N>(other + oth + g.P);
    }
    in.fv = NT ? vload_nt<T, N>(f + own) : vload<T, N>(f + own);
    in.own = own;
    in.o = o;
    in.j = j;
    in.m0 = m0;
    in.gk = gk;
    in.nbyz = (j == 0) + (j == g.ny - 1) + (DIM == 3 ? (gk == 0) + (gk == g.gnz - 1) : 0);
}

template <typename T, int DIM, bool ERR, bool NT = false>
__device__ __forceinline__ void half_store(const HalfIn<T, VN<T>::n>& in, T* __restrict__ dst, const T* __restrict__ old,
                                           const Geo& g, const Op<T, DIM>& op, double& acc)
{
    constexpr int N = VN<T>::n;
    const int o = in.o;
    T d0, y0, d1, y1;
    row_diag_fast(op, in.nbyz, d0, y0, d1, y1);
    Vec<T, N> out;
#pragma unroll
    for (int e = 0; e < N; ++e) {
        const int i = 2 * (in.m0 + e) + o;
        const T xl = o == 0 ? (e == 0 ? in.edge : in.cen.v[e - 1]) : in.cen.v[e];
        const T xr = o == 0 ? in.cen.v[e] : (e == N - 1 ? in.edge : in.cen.v[e + 1]);
        T s = xl + xr;
        s = s + in.yl.v[e];
        s = s + in.yr.v[e];
        if (DIM == 3) {
            s = s + in.zl.v[e];
            s = s + in.zr.v[e];
        }
        const bool xf = i == 0 || i == g.nx - 1;
        out.v[e] = div_rn(in.fv.v[e] - s * op.inv_hSq, xf ? d1 : d0, xf ? y1 : y0);  // op.relax(s, f, nbyz + xf)
    }
    if (NT)
        vstore_nt<T, N>(dst + in.own, out);
    else
        vstore<T, N>(dst + in.own, out);
    if (ERR) {
        const Vec<T, N> w = NT ? vload_nt<T, N>(old + in.own) : vload<T, N>(old + in.own);
#pragma unroll
        for (int e = 0; e < N; ++e) {
            const double d = (double)out.v[e] - (double)w.v[e];
            acc += d * d;
        }
    }
}

template <typename T, int DIM, int TAG, bool ERR>
__global__ __launch_bounds__(kBlock) void k_half(const T* __restrict__ other, const T* __restrict__ f,
                                                 T* __restrict__ dst, const T* __restrict__ old,
                                                 double* __restrict__ partials, Geo g, int color,
                                                 Op<T, DIM> op)
{
    const int b = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t it = (int64_t)b * kBlock + threadIdx.x;
    double acc = 0.0;
    if ((it >> (g.lhw - (VN<T>::n == 4 ? 2 : 1) + g.ly)) < g.nz) {
        HalfIn<T, VN<T>::n> in;
        half_load<T, DIM, TAG == 2>(in, other, f, g, color, it);
        half_store<T, DIM, ERR, TAG == 2>(in, dst, old, g, op, acc);
    }
    if (ERR) block_partial<T>(acc, partials);
}

// Grid-stride form for large levels (kGsBlocks workgroups): the workgroups of XCD x (b % 8 == x)
// sweep the contiguous band x of the items, so y/z neighbours meet in that XCD's L2, and each
// thread keeps two items' loads in flight.
constexpr int kGsBlocks = 2048;

template <typename T, int DIM, int TAG, bool ERR>
__global__ __launch_bounds__(kBlock) void k_half_gs(const T* __restrict__ other, const T* __restrict__ f,
                                                    T* __restrict__ dst, const T* __restrict__ old,
                                                    double* __restrict__ partials, Geo g, int color,
                                                    Op<T, DIM> op, int64_t items)
{
    const int nlb = gridDim.x >> 3;
    const int64_t band = (items + 7) >> 3;
    const int64_t base = (int64_t)(blockIdx.x & 7) * band;
    const int64_t end = base + band < items ? base + band : items;
    const int64_t step = (int64_t)nlb * kBlock;
    double acc = 0.0;
    for (int64_t i0 = base + (int64_t)(blockIdx.x >> 3) * kBlock + threadIdx.x; i0 < end; i0 += 2 * step) {
        const int64_t i1 = i0 + step;
        HalfIn<T, VN<T>::n> a, c;
        half_load<T, DIM>(a, other, f, g, color, i0);
        if (i1 < end) half_load<T, DIM>(c, other, f, g, color, i1);
        half_store<T, DIM, ERR>(a, dst, old, g, op, acc);
        if (i1 < end) half_store<T, DIM, ERR>(c, dst, old, g, op, acc);
    }
    if (ERR) block_partial<T>(acc, partials);
}

// One colour-c slot of a half-sweep (scalar; any level size, nx = 1 included).  Returns the
// packed index written, or -1 for the empty slot of an nx = 1 row; *v = the new value.
// C: the type the expression is evaluated in (C = double with T = float: cpu-raw.lua's real = 'float',
// LuaJIT doubles rounded once at the store, cpu-raw.lua:34-44); with C = T every cast is the identity.
template <typename T, int DIM, typename C = T>
__device__ __forceinline__ int64_t half_item(const T* other, const T* __restrict__ f, T* dst, const Geo& g,
                                             int color, const Op<C, DIM>& op, int64_t it, T* v)
{
    const int m = (int)(it & (g.hw - 1));
    const int j = (int)((it >> g.lhw) & (g.ny - 1));
    const int64_t k = it >> (g.lhw + g.ly);
    const int64_t gk = g.z0 + k;
    const int o = color ^ (int)((j + gk) & 1);
    const int i = 2 * m + o;
    if (i >= g.nx) return -1;
    const int64_t own = k * g.P + color * g.H + (int64_t)j * g.hw + m;
    const int64_t oth = k * g.P + (color ^ 1) * g.H + (int64_t)j * g.hw + m;
    const C xl = i > 0 ? (C)other[oth - 1 + o] : (C)0;
    const C xr = i < g.nx - 1 ? (C)other[oth + o] : (C)0;
    C s = xl + xr;
    s = s + (j > 0 ? (C)other[oth - g.hw] : (C)0);
    s = s + (j < g.ny - 1 ? (C)other[oth + g.hw] : (C)0);
    if (DIM == 3) {
        s = s + (C)other[oth - g.P];
        s = s + (C)other[oth + g.P];
    }
    const int nb = (i == 0) + (i == g.nx - 1) + (j == 0) + (j == g.ny - 1) +
                   (DIM == 3 ? (gk == 0) + (gk == g.gnz - 1) : 0);
    *v = (T)op.relax(s, (C)f[own], nb);
    dst[own] = *v;
    return own;
}

// Scalar form for small levels (hw < N, nx = 1 included) and for the cpu-raw float arithmetic
// (C = double, every level): a thread per colour-c slot.
template <typename T, int DIM, bool ERR, typename C = T>
__global__ __launch_bounds__(kBlock) void k_half_s(const T* __restrict__ other, const T* __restrict__ f,
                                                   T* __restrict__ dst, const T* __restrict__ old,
                                                   double* __restrict__ partials, Geo g, int color,
                                                   Op<C, DIM> op)
{
    const int64_t it = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    double acc = 0.0;
    if (it < g.H * g.nz) {
        T v;
        const int64_t own = half_item<T, DIM, C>(other, f, dst, g, color, op, it, &v);
        if (ERR && own >= 0) {
            const double d = (double)v - (double)old[own];
            acc += d * d;
        }
    }
    if (ERR) block_partial<T>(acc, partials);
}

// First RB-GS sweep from a fresh zero guess (cpu.lua:138), both colours in one pass over f.
// With u = 0 the red half-sweep's neighbour sum is +0, so red = relax(0, f_red, nb): a pointwise
// function of f.  The black half-sweep then needs the red values of its six neighbours, which
// this thread recomputes from f (red rows j-1, j, j+1 and planes k-1, k+1 of its N-cell segment,
// plus one edge cell) with the same expression, so u after the sweep is bit-identical to the two
// half-sweeps reading a zero black input.  A thread owns the N red and N black cells at half
// positions m0 .. m0+N-1 of one row.  HBM: read f, write u (the per-piece pair also reads the
// zero input and re-reads the red cells).
// RED = false: the red cells are not stored (a later sweep's red half-sweep replaces them unread)
template <typename T, int DIM, bool RED = true>
__global__ __launch_bounds__(kBlock) void k_fresh(const T* __restrict__ f, T* __restrict__ u, Geo g, Op<T, DIM> op)
{
    constexpr int N = VN<T>::n;
    constexpr int LN = N == 4 ? 2 : 1;
    const int lgpr = g.lhw - LN;
    const int b = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t it = (int64_t)b * kBlock + threadIdx.x;
    const int grp = (int)(it & ((1 << lgpr) - 1));
    const int j = (int)((it >> lgpr) & (g.ny - 1));
    const int64_t k = it >> (lgpr + g.ly);
    if (k >= g.nz) return;
    const int m0 = grp * N;
    const int64_t gk = g.z0 + k;
    const int ob = 1 ^ (int)((j + gk) & 1);  // x parity of this row's black cells (red: ob ^ 1)
    // A row's diagonals are looked up once per row (Op::row_diag), so a cell's relax is div_rn with a select
    // between two of them.  relax(+0, f, nb) = div_rn(f - (+0), ..) = div_rn(f, ..) exactly (f - (+0) == f).
    struct RowDiag {
        T d0, y0, d1, y1;
    };
    auto row_diag = [&](int nbyz) {
        RowDiag r;
        row_diag_fast(op, nbyz, r.d0, r.y0, r.d1, r.y1);  // five rows per thread
        return r;
    };
    // Every load is issued before any arithmetic (round 4: with a load per red-row evaluation behind its box
    // test, each thread waited for five memory latencies one after another; 256^3 31.8 us)
    const int64_t own = k * g.P + (int64_t)j * g.hw + m0;
    const bool vyl = j > 0, vyr = j < g.ny - 1;
    const bool vzl = DIM == 3 && gk > 0, vzr = DIM == 3 && gk < g.gnz - 1;
    const Vec<T, N> fc = vload<T, N>(f + own);  // red half of the row (colour 0)
    const Vec<T, N> fyl = vload<T, N>(f + own - (vyl ? g.hw : 0));
    const Vec<T, N> fyr = vload<T, N>(f + own + (vyr ? g.hw : 0));
    Vec<T, N> fzl = fc, fzr = fc;
    if (DIM == 3) {
        fzl = vload<T, N>(f + own - (vzl ? g.P : 0));
        fzr = vload<T, N>(f + own + (vzr ? g.P : 0));
    }
    // the red x-neighbour outside the segment: m0 - 1 (black cells at even x) or m0 + N (odd x)
    const int me = ob == 0 ? m0 - 1 : m0 + N;
    const bool ve = me >= 0 && me < g.hw;
    const T fe = f[own + (ve ? me - m0 : 0)];
    const Vec<T, N> fb = vload<T, N>(f + own + g.H);
    // red values of row (jj, gkk) at m0 .. m0+N-1 from its f (0 outside the box)
    auto red_row = [&](const Vec<T, N>& fv, bool valid, int jj, int64_t gkk, Vec<T, N>& r) {
        if (!valid) {
            r = vzero<T, N>();
            return;
        }
        const int orr = (int)((jj + gkk) & 1);  // x parity of red cells in that row
        const int nbyz = (jj == 0) + (jj == g.ny - 1) + (DIM == 3 ? (gkk == 0) + (gkk == g.gnz - 1) : 0);
        const RowDiag rd = row_diag(nbyz);
#pragma unroll
        for (int e = 0; e < N; ++e) {
            const int i = 2 * (m0 + e) + orr;
            const bool xf = i == 0 || i == g.nx - 1;
            r.v[e] = div_rn(fv.v[e], xf ? rd.d1 : rd.d0, xf ? rd.y1 : rd.y0);
        }
    };
    Vec<T, N> rc, ryl, ryr, rzl, rzr;
    red_row(fc, true, j, gk, rc);
    red_row(fyl, vyl, j - 1, gk, ryl);
    red_row(fyr, vyr, j + 1, gk, ryr);
    if (DIM == 3) {
        red_row(fzl, vzl, j, gk - 1, rzl);
        red_row(fzr, vzr, j, gk + 1, rzr);
    }
    const int nbyz = (j == 0) + (j == g.ny - 1) + (DIM == 3 ? (gk == 0) + (gk == g.gnz - 1) : 0);
    T edge = (T)0;
    if (ve) {
        const int i = 2 * me + (ob ^ 1);
        edge = op.relax((T)0, fe, nbyz + (i == 0) + (i == g.nx - 1));
    }
    const RowDiag bd = row_diag(nbyz);
    Vec<T, N> out;
#pragma unroll
    for (int e = 0; e < N; ++e) {
        const int i = 2 * (m0 + e) + ob;
        const T xl = ob == 0 ? (e == 0 ? edge : rc.v[e - 1]) : rc.v[e];
        const T xr = ob == 0 ? rc.v[e] : (e == N - 1 ? edge : rc.v[e + 1]);
        T s = xl + xr;
        s = s + ryl.v[e];
        s = s + ryr.v[e];
        if (DIM == 3) {
            s = s + rzl.v[e];
            s = s + rzr.v[e];
        }
        const bool xf = i == 0 || i == g.nx - 1;
        out.v[e] = div_rn(fb.v[e] - s * op.inv_hSq, xf ? bd.d1 : bd.d0, xf ? bd.y1 : bd.y0);  // Op::relax
    }
    if (RED) vstore<T, N>(u + own, rc);
    vstore<T, N>(u + own + g.H, out);
}

// ---- fused residual + restriction -----------------------------------------------------------

// Residual of one fine cell from packed u (generic, scalar loads), evaluated in C (half_item's C).
template <typename T, int DIM, typename C = T>
__device__ __forceinline__ C residual_at(const T* __restrict__ u, const T* __restrict__ f, const Geo& g,
                                         const Op<C, DIM>& op, int i, int j, int64_t k)
{
    const int64_t c = pidx(g, i, j, k);
    const int o = i & 1;
    // neighbours: other colour, same row at m-1+o / m+o; rows j+-1 and planes k+-1 at m
    const int64_t oth = c + ((c - k * g.P) >= g.H ? -g.H : g.H);
    const C xl = i > 0 ? (C)u[oth - 1 + o] : (C)0;
    const C xr = i < g.nx - 1 ? (C)u[oth + o] : (C)0;
    C s = xl + xr;
    s = s + (j > 0 ? (C)u[oth - g.hw] : (C)0);
    s = s + (j < g.ny - 1 ? (C)u[oth + g.hw] : (C)0);
    const int64_t gk = g.z0 + k;
    if (DIM == 3) {
        s = s + (C)u[oth - g.P];
        s = s + (C)u[oth + g.P];
    }
    const int nb = (i == 0) + (i == g.nx - 1) + (j == 0) + (j == g.ny - 1) + (DIM == 3 ? (gk == 0) + (gk == g.gnz - 1) : 0);
    return op.residual(s, (C)f[c], (C)u[c], nb);
}

// ---- residual norm (north star: wavefront-level reductions for the residual norm) -------------

// Fixed-order fp64 sum across the 64 lanes of a wave (butterfly over lane distances 32 .. 1; every
// lane ends with the same value, the same on every run).
__device__ __forceinline__ double wave_sum(double v)
{
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// sum (f - A u)^2 and sum f^2 over both colours of a level (calcResidual, cpu.lua:108-123, squared
// and reduced on the device instead of materialising r).  Vector form: a thread owns N cells of one
// colour in one row (k_half's item; colour = the item's half of the grid), loads the other colour's
// neighbours with half_load and its own cells with one vector load.  Per wave a butterfly sum, per
// workgroup the 4 wave sums in fixed order, one fp64 pair per workgroup into partials[b] and
// partials[fofs + b] (fofs leaves room for the first row's sum_partials scratch).
template <typename T, int DIM>
__global__ __launch_bounds__(kBlock) void k_resnorm(const T* __restrict__ u, const T* __restrict__ f, Geo g,
                                                    Op<T, DIM> op, int64_t items, double* __restrict__ partials,
                                                    int fofs)
{
    constexpr int N = VN<T>::n;
    const int64_t it = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    double rr = 0.0, ff = 0.0;
    if (it < 2 * items) {
        const int color = it >= items;
        HalfIn<T, N> in;
        half_load<T, DIM>(in, u, f, g, color, it - color * items);
        const Vec<T, N> uc = vload<T, N>(u + in.own);
#pragma unroll
        for (int e = 0; e < N; ++e) {
            const int o = in.o;
            const int i = 2 * (in.m0 + e) + o;
            const T xl = o == 0 ? (e == 0 ? in.edge : in.cen.v[e - 1]) : in.cen.v[e];
            const T xr = o == 0 ? in.cen.v[e] : (e == N - 1 ? in.edge : in.cen.v[e + 1]);
            T sm = xl + xr;
            sm = sm + in.yl.v[e];
            sm = sm + in.yr.v[e];
            if (DIM == 3) {
                sm = sm + in.zl.v[e];
                sm = sm + in.zr.v[e];
            }
            const T r = op.residual(sm, in.fv.v[e], uc.v[e], in.nbyz + (i == 0) + (i == g.nx - 1));
            rr = __builtin_fma((double)r, (double)r, rr);
            ff = __builtin_fma((double)in.fv.v[e], (double)in.fv.v[e], ff);
        }
    }
    rr = wave_sum(rr);
    ff = wave_sum(ff);
    __shared__ double ws[2][kBlock / 64];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        ws[0][w] = rr;
        ws[1][w] = ff;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = 0.0, b = 0.0;
        for (int k = 0; k < kBlock / 64; ++k) {
            a += ws[0][k];
            b += ws[1][k];
        }
        partials[blockIdx.x] = a;
        partials[fofs + blockIdx.x] = b;
    }
}

// 3D levels streamed through z: a thread owns N cells of each colour in one row (j, packed m0 .. m0 + N - 1)
// and walks kResZ planes, holding both colours of the row in planes k - 1, k, k + 1 in registers, so each
// plane of u and f is read once (rows j +- 1 come from L2, where the neighbouring rows' threads read them as
// their own).  The per-cell expressions are k_resnorm's; only the partial sums' grouping differs.
constexpr int kResZ = 16;
template <typename T>
__global__ __launch_bounds__(kBlock) void k_resnorm_z(const T* __restrict__ u, const T* __restrict__ f, Geo g,
                                                      Op<T, 3> op, double* __restrict__ partials, int fofs)
{
    constexpr int N = VN<T>::n;
    const int groups = g.hw / N;
    const int64_t cols = (int64_t)groups * g.ny;
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    double rr = 0.0, ff = 0.0;
    if (t < cols * (g.nz / kResZ)) {
        const int64_t col = t % cols;
        const int64_t k0 = (t / cols) * kResZ;
        const int grp = (int)(col % groups), j = (int)(col / groups), m0 = grp * N;
        const int64_t roff = (int64_t)j * g.hw + m0;
        Vec<T, N> A[2], B[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            A[c] = vload<T, N>(u + (k0 - 1) * g.P + c * g.H + roff);  // a ghost plane at the slab's ends
            B[c] = vload<T, N>(u + k0 * g.P + c * g.H + roff);
        }
        for (int64_t k = k0; k < k0 + kResZ; ++k) {
            const int64_t gk = g.z0 + k;
            const T* const pk = u + k * g.P + roff;
            Vec<T, N> C[2], YL[2], YR[2], F[2];
            T edge[2];
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                C[c] = vload<T, N>(pk + g.P + c * g.H);
                YL[c] = j > 0 ? vload<T, N>(pk + c * g.H - g.hw) : vzero<T, N>();
                YR[c] = j < g.ny - 1 ? vload<T, N>(pk + c * g.H + g.hw) : vzero<T, N>();
                F[c] = vload<T, N>(f + k * g.P + c * g.H + roff);
                // x edge of colour c's cells, from the other colour's row: x - 1 of the first cell (x parity 0)
                // or x + 1 of the last (parity 1)
                const int o = c ^ (int)((j + gk) & 1);
                const T* const oth = pk + (c ^ 1) * g.H;
                if (o == 0)
                    edge[c] = m0 > 0 ? oth[-1] : (T)0;
                else
                    edge[c] = m0 + N < g.hw ? oth[N] : (T)0;
            }
            const int nbyz = (j == 0) + (j == g.ny - 1) + (gk == 0) + (gk == g.gnz - 1);
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const int oc = c ^ 1, o = c ^ (int)((j + gk) & 1);
                const Vec<T, N>& cen = B[oc];
#pragma unroll
                for (int e = 0; e < N; ++e) {
                    const int i = 2 * (m0 + e) + o;
                    const T xl = o == 0 ? (e == 0 ? edge[c] : cen.v[e - 1]) : cen.v[e];
                    const T xr = o == 0 ? cen.v[e] : (e == N - 1 ? edge[c] : cen.v[e + 1]);
                    T sm = xl + xr;
                    sm = sm + YL[oc].v[e];
                    sm = sm + YR[oc].v[e];
                    sm = sm + A[oc].v[e];
                    sm = sm + C[oc].v[e];
                    const T r = op.residual(sm, F[c].v[e], B[c].v[e], nbyz + (i == 0) + (i == g.nx - 1));
                    rr = __builtin_fma((double)r, (double)r, rr);
                    ff = __builtin_fma((double)F[c].v[e], (double)F[c].v[e], ff);
                }
            }
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                A[c] = B[c];
                B[c] = C[c];
            }
        }
    }
    rr = wave_sum(rr);
    ff = wave_sum(ff);
    __shared__ double ws[2][kBlock / 64];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        ws[0][w] = rr;
        ws[1][w] = ff;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = 0.0, b = 0.0;
        for (int q = 0; q < kBlock / 64; ++q) {
            a += ws[0][q];
            b += ws[1][q];
        }
        partials[blockIdx.x] = a;
        partials[fofs + blockIdx.x] = b;
    }
}

// Scalar form for small levels (hw < N, nx = 1 included), and for the cpu-raw float arithmetic (C = double:
// r evaluated in double and rounded to the real type, as rs[L] would hold it): a thread per packed slot.
template <typename T, int DIM, typename C = T>
__global__ __launch_bounds__(kBlock) void k_resnorm_s(const T* __restrict__ u, const T* __restrict__ f, Geo g,
                                                      Op<C, DIM> op, double* __restrict__ partials, int fofs)
{
    const int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    double rr = 0.0, ff = 0.0;
    if (s < g.P * g.nz) {
        int i, j;
        int64_t k;
        if (slot_cell(s, g, i, j, k)) {
            const T r = (T)residual_at<T, DIM, C>(u, f, g, op, i, j, k);
            rr = (double)r * (double)r;
            ff = (double)f[s] * (double)f[s];
        }
    }
    rr = wave_sum(rr);
    ff = wave_sum(ff);
    __shared__ double ws[2][kBlock / 64];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        ws[0][w] = rr;
        ws[1][w] = ff;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = 0.0, b = 0.0;
        for (int k = 0; k < kBlock / 64; ++k) {
            a += ws[0][k];
            b += ws[1][k];
        }
        partials[blockIdx.x] = a;
        partials[fofs + blockIdx.x] = b;
    }
}

// rs[L] of cpu-raw.lua:155-171 (calcResidual, cpu.lua:108-123) materialised on request (mgp_get_field
// MGP_FIELD_RESIDUAL): r at every packed slot, grid-stride.
template <typename T, int DIM, typename C = T>
__global__ __launch_bounds__(kBlock) void k_residual_field(const T* __restrict__ u, const T* __restrict__ f,
                                                           T* __restrict__ r, Geo g, Op<C, DIM> op)
{
    const int64_t n = g.P * g.nz;
    for (int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x; s < n; s += (int64_t)gridDim.x * kBlock) {
        int i, j;
        int64_t k;
        r[s] = slot_cell(s, g, i, j, k) ? (T)residual_at<T, DIM, C>(u, f, g, op, i, j, k) : (T)0;
    }
}

// errorBuf of cpu-raw.lua:96-100 / gpu.lua:189-200 (calcFrobErr): (psi - psiOld)^2 per cell, evaluated in C
// (gpu.lua: real; cpu-raw.lua: LuaJIT double) and stored in real.
template <typename T, typename C = T>
__global__ __launch_bounds__(kBlock) void k_sqdiff_field(const T* __restrict__ a, const T* __restrict__ b,
                                                         T* __restrict__ out, int64_t n)
{
    for (int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x; s < n; s += (int64_t)gridDim.x * kBlock) {
        const C d = (C)a[s] - (C)b[s];
        out[s] = (T)(d * d);
    }
}

// One coarse cell of the fused residual + restriction (scalar; any sizes).  C = double (cpu-raw.lua's float):
// each child residual is rounded to the real type first (calcResidual stores it in rs[L], cpu-raw.lua:211),
// then summed and scaled in double and rounded once (reduceResidual, cpu-raw.lua:59-63).
template <typename T, int DIM, typename C = T>
__device__ __forceinline__ void resrestrict_item(const T* u, const T* f, T* R, const Geo& g, const Geo& gc,
                                                 const Op<C, DIM>& op, int64_t it)
{
    const int cx = g.nx >> 1, cy = g.ny >> 1;
    const int lcx = g.lx - 1, lcy = g.ly - 1;
    const int I = (int)(it & (cx - 1));
    const int J = (int)((it >> lcx) & (cy - 1));
    const int64_t K = it >> (lcx + lcy);
    const int i = 2 * I, j = 2 * J;
    const int64_t k = DIM == 3 ? 2 * K : 0;
    auto r = [&](int a, int b, int64_t c) { return (C)(T)residual_at<T, DIM, C>(u, f, g, op, a, b, c); };
    C s = r(i, j, k) + r(i + 1, j, k);
    s = s + r(i, j + 1, k);
    s = s + r(i + 1, j + 1, k);
    if (DIM == 3) {
        s = s + r(i, j, k + 1);
        s = s + r(i + 1, j, k + 1);
        s = s + r(i, j + 1, k + 1);
        s = s + r(i + 1, j + 1, k + 1);
        R[pidx(gc, I, J, K)] = (T)((C)0.125 * s);
    } else {
        R[pidx(gc, I, J, 0)] = (T)((C)0.25 * s);
    }
}

template <typename T, int DIM>
__device__ __forceinline__ int64_t resrestrict_items(const Geo& g)
{
    return (int64_t)(g.nx >> 1) * (g.ny >> 1) * (DIM == 3 ? (g.nz >> 1) : 1);
}

// Scalar form: a thread per coarse cell (any sizes; every level under the cpu-raw float arithmetic).
template <typename T, int DIM, typename C = T>
__global__ __launch_bounds__(kBlock) void k_resrestrict_s(const T* __restrict__ u, const T* __restrict__ f,
                                                          T* __restrict__ R, Geo g, Geo gc, Op<C, DIM> op)
{
    const int64_t it = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (it >= resrestrict_items<T, DIM>(g)) return;
    resrestrict_item<T, DIM, C>(u, f, R, g, gc, op, it);
}

// Vector form: a thread owns N consecutive coarse cells I0 .. I0+N-1 of one coarse row.  Their
// fine children are, in every fine row, the N cells m = I0 .. of BOTH colours.  The thread loads
// each fine (plane, row, colour) vector it needs exactly once into registers — planes 2K, 2K+1
// with rows 2J-1 .. 2J+2, planes 2K-1, 2K+2 with rows 2J, 2J+1 — and keeps the reference order
//   R = 1/8 (((((((r000 + r100) + r010) + r110) + r001) + r101) + r011) + r111).
// NV: coarse cells per thread (default: one 16-byte vector; 2 gives mid-size levels more threads)
template <typename T, int DIM, int NV = VN<T>::n>
__global__ __launch_bounds__(kBlock) void k_resrestrict(const T* __restrict__ u, const T* __restrict__ f,
                                                        T* __restrict__ R, Geo g, Geo gc, Op<T, DIM> op)
{
    constexpr int N = NV;
    constexpr int LN = N == 4 ? 2 : (N == 2 ? 1 : 0);
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

// ---- full-weighting restriction (build-defined option, north_star) ------------------------------
//
// The cell-centred adjoint of the linear prolongation (oracle: restrict_fw in mgp_oracle_impl.h): per
// axis coarse I takes fine 2I-1 .. 2I+2 as ((r_a + w_b r_b) + w_c r_c) + r_d, w = 3 or, next to a box
// face, 3 - clc; fine cells outside the box are +0; x, then y, then z; times 1/8^DIM.  The residual is
// materialised first (k_resfield_v / k_residual_field into the level-sized scratch), because each fine
// residual feeds 2^DIM coarse cells; on a slab level one ghost plane of r is exchanged in between.


// Coarse cell (I, J, local plane K) from fine residuals get(i, j, k) (k local; called only for cells
// inside the box).  gc.z0 = g.z0 / 2 (the coarse plane of this rank's fine plane 0).
template <typename T, int DIM, typename Get>
__device__ __forceinline__ T fw_eval(const Get& get, const Geo& g, const Geo& gc, T wf, int I, int J, int64_t K)
{
    const T w3 = (T)3;
    T az = (T)0;
#pragma unroll
    for (int dz = 0; dz < (DIM == 3 ? 4 : 1); ++dz) {
        const int64_t k = DIM == 3 ? 2 * K - 1 + dz : 0;
        const bool kin = DIM == 2 || (g.z0 + k >= 0 && g.z0 + k < g.gnz);
        T ay = (T)0;
#pragma unroll
        for (int dy = 0; dy < 4; ++dy) {
            const int j = 2 * J - 1 + dy;
            const bool jin = kin && j >= 0 && j < g.ny;
            T x[4];
#pragma unroll
            for (int dx = 0; dx < 4; ++dx) {
                const int i = 2 * I - 1 + dx;
                x[dx] = (jin && i >= 0 && i < g.nx) ? get(i, j, k) : (T)0;
            }
            const T ax = fw_axis(x[0], x[1], x[2], x[3], I == 0 ? wf : w3, I == gc.nx - 1 ? wf : w3);
            // ay = ((ax0 + wb ax1) + wc ax2) + ax3, accumulated row by row
            if (dy == 0) ay = ax;
            else if (dy == 1) ay = ay + (J == 0 ? wf : w3) * ax;
            else if (dy == 2) ay = ay + (J == gc.ny - 1 ? wf : w3) * ax;
            else ay = ay + ax;
        }
        if (DIM == 2) {
            az = ay;
        } else {
            const int64_t gK = gc.z0 + K;
            if (dz == 0) az = ay;
            else if (dz == 1) az = az + (gK == 0 ? wf : w3) * ay;
            else if (dz == 2) az = az + (gK == gc.gnz - 1 ? wf : w3) * ay;
            else az = az + ay;
        }
    }
    return (DIM == 3 ? (T)(1.0 / 512.0) : (T)(1.0 / 64.0)) * az;
}

// r = f - A u at both colours of a level (vector form, k_half's item): the scratch of the full weighting
template <typename T, int DIM>
__global__ __launch_bounds__(kBlock) void k_resfield_v(const T* __restrict__ u, const T* __restrict__ f,
                                                       T* __restrict__ r, Geo g, Op<T, DIM> op, int64_t items)
{
    constexpr int N = VN<T>::n;
    const int b = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t it = (int64_t)b * kBlock + threadIdx.x;
    if (it >= 2 * items) return;
    const int color = it >= items;
    HalfIn<T, N> in;
    half_load<T, DIM>(in, u, f, g, color, it - color * items);
    const Vec<T, N> uc = vload<T, N>(u + in.own);
    const bool fast = op.cl == (T)0;
    Vec<T, N> out;
#pragma unroll
    for (int e = 0; e < N; ++e) {
        const int o = in.o;
        const int i = 2 * (in.m0 + e) + o;
        const T xl = o == 0 ? (e == 0 ? in.edge : in.cen.v[e - 1]) : in.cen.v[e];
        const T xr = o == 0 ? in.cen.v[e] : (e == N - 1 ? in.edge : in.cen.v[e + 1]);
        T sm = xl + xr;
        sm = sm + in.yl.v[e];
        sm = sm + in.yr.v[e];
        if (DIM == 3) {
            sm = sm + in.zl.v[e];
            sm = sm + in.zr.v[e];
        }
        out.v[e] = fast ? op.residual(sm, in.fv.v[e], uc.v[e], 0)
                        : op.residual(sm, in.fv.v[e], uc.v[e], in.nbyz + (i == 0) + (i == g.nx - 1));
    }
    vstore<T, N>(r + in.own, out);
}

// Scalar form: a thread per coarse cell (any sizes), r packed with readable planes -1 and g.nz; evaluated in
// C (double under the cpu-raw float arithmetic) and rounded once
template <typename T, int DIM, typename C = T>
__global__ __launch_bounds__(kBlock) void k_fw_s(const T* __restrict__ r, T* __restrict__ R, Geo g, Geo gc, C wf)
{
    const int64_t it = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (it >= resrestrict_items<T, DIM>(g)) return;
    const int cx = g.nx >> 1, cy = g.ny >> 1;
    const int I = (int)(it % cx), J = (int)((it / cx) % cy);
    const int64_t K = it / ((int64_t)cx * cy);
    auto get = [&](int i, int j, int64_t k) { return (C)r[pidx(g, i, j, k)]; };
    R[pidx(gc, I, J, K)] = (T)fw_eval<C, DIM>(get, g, gc, wf, I, J, K);
}

// Vector form (coarse nx >= N): a thread owns N consecutive coarse cells I0 .. of one coarse row; each
// of its 4 (2D) / 16 (3D) fine rows is two N-wide loads (even and odd x of fine cells 2 I0 .. 2 I0 + 2N - 1)
// plus the two edge cells, reduced along x at once and accumulated in fw_eval's order.
template <typename T, int DIM>
__global__ __launch_bounds__(kBlock) void k_fw_v(const T* __restrict__ r, T* __restrict__ R, Geo g, Geo gc, T wf)
{
    constexpr int N = VN<T>::n;
    constexpr int LN = N == 4 ? 2 : 1;
    const int cx = g.nx >> 1, cy = g.ny >> 1;
    const int lgpr = (g.lx - 1) - LN;
    const int64_t ncz = DIM == 3 ? (g.nz >> 1) : 1;
    const int b = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t it = (int64_t)b * kBlock + threadIdx.x;
    const int grp = (int)(it & ((1 << lgpr) - 1));
    const int J = (int)((it >> lgpr) & (cy - 1));
    const int64_t K = it >> (lgpr + g.ly - 1);
    if (K >= ncz) return;
    const int I0 = grp * N;
    const T w3 = (T)3;
    T az[N], ay[N];
#pragma unroll
    for (int e = 0; e < N; ++e) az[e] = (T)0;
#pragma unroll
    for (int dz = 0; dz < (DIM == 3 ? 4 : 1); ++dz) {
        const int64_t k = DIM == 3 ? 2 * K - 1 + dz : 0;
        const int64_t gk = g.z0 + k;
        const bool kin = DIM == 2 || (gk >= 0 && gk < g.gnz);
#pragma unroll
        for (int dy = 0; dy < 4; ++dy) {
            const int j = 2 * J - 1 + dy;
            Vec<T, N> ev = vzero<T, N>(), od = vzero<T, N>();
            T left = (T)0, right = (T)0;
            if (kin && j >= 0 && j < g.ny) {
                const int pe = (int)((j + gk) & 1);  // colour of the row's even x
                const T* row = r + k * g.P + (int64_t)j * g.hw;
                ev = vload<T, N>(row + pe * g.H + I0);
                od = vload<T, N>(row + (pe ^ 1) * g.H + I0);
                if (I0 > 0) left = row[(pe ^ 1) * g.H + I0 - 1];  // fine 2 I0 - 1
                if (I0 + N < cx) right = row[pe * g.H + I0 + N];  // fine 2 I0 + 2N
            }
#pragma unroll
            for (int e = 0; e < N; ++e) {
                const int I = I0 + e;
                const T a = e == 0 ? left : od.v[e - 1];
                const T d = e == N - 1 ? right : ev.v[e + 1];
                const T ax = fw_axis(a, ev.v[e], od.v[e], d, I == 0 ? wf : w3, I == cx - 1 ? wf : w3);
                if (dy == 0) ay[e] = ax;
                else if (dy == 1) ay[e] = ay[e] + (J == 0 ? wf : w3) * ax;
                else if (dy == 2) ay[e] = ay[e] + (J == cy - 1 ? wf : w3) * ax;
                else ay[e] = ay[e] + ax;
            }
        }
#pragma unroll
        for (int e = 0; e < N; ++e) {
            if (DIM == 2) {
                az[e] = ay[e];
            } else {
                const int64_t gK = gc.z0 + K;
                if (dz == 0) az[e] = ay[e];
                else if (dz == 1) az[e] = az[e] + (gK == 0 ? wf : w3) * ay[e];
                else if (dz == 2) az[e] = az[e] + (gK == gc.gnz - 1 ? wf : w3) * ay[e];
                else az[e] = az[e] + ay[e];
            }
        }
    }
    const int64_t gK = gc.z0 + K;
    const int pc = (int)((J + gK) & 1);
    const int64_t rowc = K * gc.P + (int64_t)J * gc.hw;
#pragma unroll
    for (int e = 0; e < N; ++e) {
        const int I = I0 + e;
        R[rowc + ((I + pc) & 1) * gc.H + (I >> 1)] = (DIM == 3 ? (T)(1.0 / 512.0) : (T)(1.0 / 64.0)) * az[e];
    }
}

// ---- prolongation + correction --------------------------------------------------------------

// (P V) at fine cell (i, j, local plane k) from the packed coarse level V
template <typename T, int DIM, int LINEAR>
__device__ __forceinline__ T prolong_value(const T* V, const Geo& g, const Geo& gc, T cl, int i, int j, int64_t k)
{
    auto get = [&](int I, int J, int64_t K) { return V[pidx(gc, I, J, K)]; };
    return prolong_eval<T, DIM, LINEAR>(get, gc, cl, i, j, k);
}

// One fine slot of colour `color` of the prolongation + correction (scalar; any sizes).  C = double
// (cpu-raw.lua's float): P V evaluated in double and rounded into the real type (the vs[L] buffer,
// cpu-raw.lua:226), then addTo's u + v in double, rounded once (cpu-raw.lua:83-85).
template <typename T, int DIM, int LINEAR, typename C = T>
__device__ __forceinline__ void prolong_item(T* u, const T* V, const Geo& g, const Geo& gc, C cl, int color,
                                             int64_t it)
{
    const int m = (int)(it & (g.hw - 1));
    const int j = (int)((it >> g.lhw) & (g.ny - 1));
    const int64_t k = it >> (g.lhw + g.ly);
    const int o = color ^ (int)((j + g.z0 + k) & 1);
    const int i = 2 * m + o;
    if (i >= g.nx) return;
    const int64_t own = k * g.P + color * g.H + (int64_t)j * g.hw + m;
    auto get = [&](int I, int J, int64_t K) { return (C)V[pidx(gc, I, J, K)]; };
    const T v = (T)prolong_eval<C, DIM, LINEAR>(get, gc, cl, i, j, k);
    u[own] = (T)((C)u[own] + (C)v);
}

// a thread per fine slot of colour `color` (any sizes)
template <typename T, int DIM, int LINEAR, typename C = T>
__global__ __launch_bounds__(kBlock) void k_prolong(T* __restrict__ u, const T* __restrict__ V, Geo g, Geo gc,
                                                    double clc, int color)
{
    const int64_t it = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (it >= g.H * g.nz) return;
    prolong_item<T, DIM, LINEAR, C>(u, V, g, gc, (C)clc, color, it);
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
    if constexpr (N == 4) {
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

// The coarse neighbourhood of fine row (j, k) above coarse cells I0 .. I0+N-1 (coarse rows J, Jn and
// planes K, Kn; Jn, Kn clamped to the parent row / plane outside the box, where the oracle's cval()
// factor applies) and the oracle's per-cell prolongation value of its cells.
template <typename T, int N, int DIM, int LINEAR>
struct PvRow {
    T c00[N + 2], c10[N + 2], c01[N + 2], c11[N + 2];  // [z: K / Kn][y: J / Jn]
    bool oy, oz, interior;
    int I0, cx;
    // load()'s flags with rows J / Jn (2D, or plane K with oz = false) already in registers
    __device__ __forceinline__ void set_rows(const Geo& gc, int j, int64_t k, int i0, const T (&r0)[N + 2],
                                             const T (&r1)[N + 2])
    {
        static_assert(DIM == 2, "set_rows: 2D rows");
        I0 = i0;
        cx = gc.nx;
        const int J = j >> 1;
        const int Jn = (j & 1) ? J + 1 : J - 1;
        oy = Jn < 0 || Jn >= gc.ny;
        oz = false;
        (void)k;
#pragma unroll
        for (int e = 0; e < N + 2; ++e) {
            c00[e] = r0[e];
            if (LINEAR) c10[e] = r1[e];
        }
        interior = !oy && I0 > 0 && I0 + N < cx;
    }
    __device__ __forceinline__ void load(const T* __restrict__ V, const Geo& gc, int j, int64_t k, int i0)
    {
        I0 = i0;
        cx = gc.nx;
        const int J = j >> 1;
        const int64_t K = DIM == 3 ? (k >> 1) : 0;
        int Jn = (j & 1) ? J + 1 : J - 1;
        oy = Jn < 0 || Jn >= gc.ny;
        if (oy) Jn = J;
        int64_t Kn = K;
        oz = false;
        if (DIM == 3) {
            Kn = (k & 1) ? K + 1 : K - 1;
            oz = gc.z0 + Kn < 0 || gc.z0 + Kn >= gc.gnz;
            if (oz) Kn = K;
        }
        coarse_row<T, N>(V, gc, J, K, I0, c00);
        if (LINEAR) {
            coarse_row<T, N>(V, gc, Jn, K, I0, c10);
            if (DIM == 3) {
                coarse_row<T, N>(V, gc, J, Kn, I0, c01);
                coarse_row<T, N>(V, gc, Jn, Kn, I0, c11);
            }
        }
        interior = !oy && !oz && I0 > 0 && I0 + N < cx;
    }
    // P V at the cell above coarse I0 + e with x parity o
    __device__ __forceinline__ T value(int e, int o, T cl) const
    {
        const T w0 = (T)0.75, w1 = (T)0.25;
        const int pe = e + 1;  // parent I0 + e
        if (!LINEAR) return c00[pe];
        if (interior) {  // no neighbour leaves the box: every factor is 1
            const T nb00 = o ? c00[e + 2] : c00[e];
            const T nb10 = o ? c10[e + 2] : c10[e];
            const T a00 = w0 * c00[pe] + w1 * nb00;
            const T a10 = w0 * c10[pe] + w1 * nb10;
            if (DIM == 2) return w0 * a00 + w1 * a10;
            const T nb01 = o ? c01[e + 2] : c01[e];
            const T nb11 = o ? c11[e + 2] : c11[e];
            const T a01 = w0 * c01[pe] + w1 * nb01;
            const T a11 = w0 * c11[pe] + w1 * nb11;
            const T b0 = w0 * a00 + w1 * a10;
            const T b1 = w0 * a01 + w1 * a11;
            return w0 * b0 + w1 * b1;
        }
        const bool ox = (o == 0 && I0 + e == 0) || (o == 1 && I0 + e == cx - 1);
        if (!oy && !oz) {
            // only the x neighbour can leave the box: the general form below with fy = fz = false, i.e. the
            // neighbour column replaced by the parent times the factor -cl (sv's s == 1 test kept)
            const T sx = -cl;
            auto nx_ = [&](const T (&cc)[N + 2]) {
                return ox ? (sx == (T)1 ? cc[pe] : sx * cc[pe]) : (o ? cc[e + 2] : cc[e]);
            };
            const T a00 = w0 * c00[pe] + w1 * nx_(c00);
            const T a10 = w0 * c10[pe] + w1 * nx_(c10);
            if (DIM == 2) return w0 * a00 + w1 * a10;
            const T a01 = w0 * c01[pe] + w1 * nx_(c01);
            const T a11 = w0 * c11[pe] + w1 * nx_(c11);
            const T b0 = w0 * a00 + w1 * a10;
            const T b1 = w0 * a01 + w1 * a11;
            return w0 * b0 + w1 * b1;
        }
        auto sv = [&](T val, bool fx, bool fy, bool fz) {
            T s = (T)1;
            if (fx) s = -cl * s;
            if (fy) s = -cl * s;
            if (fz) s = -cl * s;
            return s == (T)1 ? val : s * val;
        };
        // neighbour column: e (o = 0) or e + 2 (o = 1); the parent when out of the box
        auto col = [&](const T (&cc)[N + 2]) { return ox ? cc[pe] : (o ? cc[e + 2] : cc[e]); };
        const T a00 = w0 * c00[pe] + w1 * sv(col(c00), ox, false, false);
        const T a10 = w0 * sv(c10[pe], false, oy, false) + w1 * sv(col(c10), ox, oy, false);
        if (DIM == 2) return w0 * a00 + w1 * a10;
        const T a01 = w0 * sv(c01[pe], false, false, oz) + w1 * sv(col(c01), ox, false, oz);
        const T a11 = w0 * sv(c11[pe], false, oy, oz) + w1 * sv(col(c11), ox, oy, oz);
        const T b0 = w0 * a00 + w1 * a10;
        const T b1 = w0 * a01 + w1 * a11;
        return w0 * b0 + w1 * b1;
    }
};

// Vector form (coarse nx >= N): a thread owns the fine cells of one fine row (j, k) above N
// consecutive coarse cells I0 .. — fine m = I0 .. in BOTH colours (one N-wide access of u each) —
// and evaluates exactly the oracle's per-cell expression (PvRow).
// BLACK: only the black cells (the cycle's prolongation before a red/black post-smoothing, whose red
// half-sweep replaces every red cell without reading it)
template <typename T, int DIM, int LINEAR, bool BLACK = false>
__global__ __launch_bounds__(kBlock) void k_prolong_v(T* __restrict__ u, const T* __restrict__ V, Geo g, Geo gc,
                                                      T cl)
{
    constexpr int N = VN<T>::n;
    constexpr int LN = N == 4 ? 2 : 1;
    const int lgpr = gc.lx - LN;
    const int b = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t it = (int64_t)b * kBlock + threadIdx.x;
    const int grp = (int)(it & ((1 << lgpr) - 1));
    const int j = (int)((it >> lgpr) & (g.ny - 1));
    // the threads past the last item (the grid is whole workgroups) leave here in 2D as well: their j would
    // wrap onto rows that other threads update (u += P V twice, a cross-wave race)
    const int64_t k = it >> (lgpr + g.ly);
    if (k >= (DIM == 3 ? (int64_t)g.nz : 1)) return;
    const int I0 = grp * N;
    PvRow<T, N, DIM, LINEAR> pv;
    pv.load(V, gc, j, k, I0);
    const int p = (int)((j + g.z0 + k) & 1);
#pragma unroll
    for (int c = BLACK ? 1 : 0; c < 2; ++c) {
        const int o = c ^ p;  // x parity of this colour's cells in row j
        const int64_t own = k * g.P + c * g.H + (int64_t)j * g.hw + I0;
        Vec<T, N> uv = vload<T, N>(u + own);
#pragma unroll
        for (int e = 0; e < N; ++e) uv.v[e] = uv.v[e] + pv.value(e, o, cl);
        vstore<T, N>(u + own, uv);
    }
}

// Prolongation + correction fused with the first (red) half-sweep of the post-smoothing
// (prolong_correct + the red half of smooth's first sweep).  The red half-sweep replaces every red
// cell without reading it, and the black half-sweep after it replaces every black cell without
// reading it, so u + P V is only ever read on black cells by this red half-sweep: each thread
// evaluates it (PvRow, k_prolong_v's expressions) for the black neighbours of its N red cells —
// its own row, rows j +- 1 and planes k +- 1, plus one edge cell — and writes only the red cells.
// The black cells keep u without P V until the black half-sweep overwrites them.  HBM: read black u,
// red f and V, write red u (the per-piece pair also writes and re-reads both colours of u).
template <typename T, int DIM, int LINEAR>
__global__ __launch_bounds__(kBlock) void k_post1(T* __restrict__ u, const T* __restrict__ V,
                                                  const T* __restrict__ f, Geo g, Geo gc, Op<T, DIM> op, T clc)
{
    constexpr int N = VN<T>::n;
    constexpr int LN = N == 4 ? 2 : 1;
    const int lgpr = g.lhw - LN;
    const int b = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t it = (int64_t)b * kBlock + threadIdx.x;
    const int grp = (int)(it & ((1 << lgpr) - 1));
    const int j = (int)((it >> lgpr) & (g.ny - 1));
    const int64_t k = it >> (lgpr + g.ly);
    if (k >= g.nz) return;
    const int m0 = grp * N;
    const int64_t gk = g.z0 + k;
    const int orr = (int)((j + gk) & 1);  // x parity of this row's red cells (black: orr ^ 1)
    // u + P V of black row (jj, kk) at m0 .. m0+N-1 (0 outside the box)
    auto black_row = [&](int jj, int64_t kk, Vec<T, N>& r) {
        const int64_t gkk = g.z0 + kk;
        if (jj < 0 || jj >= g.ny || (DIM == 3 && (gkk < 0 || gkk >= g.gnz))) {
            r = vzero<T, N>();
            return;
        }
        const int ob = 1 ^ (int)((jj + gkk) & 1);
        r = vload<T, N>(u + kk * g.P + g.H + (int64_t)jj * g.hw + m0);
        PvRow<T, N, DIM, LINEAR> pv;
        pv.load(V, gc, jj, kk, m0);
#pragma unroll
        for (int e = 0; e < N; ++e) r.v[e] = r.v[e] + pv.value(e, ob, clc);
    };
    Vec<T, N> bc, byl, byr, bzl, bzr;
    black_row(j, k, bc);
    black_row(j - 1, k, byl);
    black_row(j + 1, k, byr);
    if (DIM == 3) {
        black_row(j, k - 1, bzl);
        black_row(j, k + 1, bzr);
    }
    // the black x-neighbour outside the segment: m0 - 1 (red cells at even x) or m0 + N (odd x)
    const int me = orr == 0 ? m0 - 1 : m0 + N;
    T edge = (T)0;
    if (me >= 0 && me < g.hw) {
        const int i = 2 * me + (orr ^ 1);
        edge = u[k * g.P + g.H + (int64_t)j * g.hw + me] + prolong_value<T, DIM, LINEAR>(V, g, gc, clc, i, j, k);
    }
    const int64_t own = k * g.P + (int64_t)j * g.hw + m0;
    const Vec<T, N> fr = vload<T, N>(f + own);
    const int nbyz = (j == 0) + (j == g.ny - 1) + (DIM == 3 ? (gk == 0) + (gk == g.gnz - 1) : 0);
    Vec<T, N> out;
#pragma unroll
    for (int e = 0; e < N; ++e) {
        const int i = 2 * (m0 + e) + orr;
        const T xl = orr == 0 ? (e == 0 ? edge : bc.v[e - 1]) : bc.v[e];
        const T xr = orr == 0 ? bc.v[e] : (e == N - 1 ? edge : bc.v[e + 1]);
        T s = xl + xr;
        s = s + byl.v[e];
        s = s + byr.v[e];
        if (DIM == 3) {
            s = s + bzl.v[e];
            s = s + bzr.v[e];
        }
        out.v[e] = op.relax(s, fr.v[e], nbyz + (i == 0) + (i == g.nx - 1));
    }
    vstore<T, N>(u + own, out);
}

// ---- z-streamed temporally blocked smoothing (3D, red/black 2+2) -------------------------------
//
// k_zs applies a whole smoothing phase of a level in ONE pass over HBM:
//   PRE : 2 RB-GS sweeps, then residual + restriction (smooth(l, 2) + residual_restrict(l))
//   POST: prolongation + correction, then 2 RB-GS sweeps (+ err) (prolong_correct + smooth(l, 2))
// A workgroup owns an x-y tile (plus a halo of H rows and S::HX >= H cells per side) and a chunk of zc
// planes and streams through z.  Every thread owns one column of the extended tile: N consecutive
// cells of each colour of one row.  At step p:
//   stage 0   plane p of the input's BLACK cells (POST: plus the prolongation, k_prolong_v's
//             expressions).  Red cells are never loaded: half-sweep 1 overwrites them, and a
//             Gauss-Seidel update does not read the value it replaces.
//   stage k   half-sweep k (k = 1..4, red first) on plane p - k.
//   last      the smoothed plane p - 4 is stored; PRE: residual + restriction of plane p - 5
//             (k_resrestrict's expressions, children summed in the reference order, the odd row's
//             residuals handed to the even row through LDS); POST: (psi - psiOld)^2 partials.
// The z-neighbours of stage k's inputs are the thread's own registers (a window of 3-4 planes per
// stage).  The in-plane neighbours (rows above / below, the neighbouring groups of the row) come
// from LDS, where every stage leaves the plane it computed; stage k reads the plane stage k-1
// wrote one step earlier, so a step issues its LDS reads up front and needs one barrier.  Cells
// outside the box are never written to LDS (they read as 0 there: the Dirichlet ghost) and
// planes outside it are forced to 0; halo cells are recomputed by every tile that needs them (the
// trapezoid shrinks by one cell per stage).  Plane indices are clamped to the readable planes, so
// the loads need no branches.  On a slab-distributed level the z-halo comes from H ghost planes per
// side (u: black cells, f).  HBM traffic per cell: PRE reads black u and f and writes u and R/8
// (2.625 reals), POST reads black u, V/8, f and psiOld and writes u (3.625 reals), against 8.125
// and 9.125 for the launch-per-piece path.

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its
// outstanding global loads (the next step's prefetch stays in flight across the barrier).
__device__ __forceinline__ void lds_barrier()
{
#ifdef ZS_NOBAR  // timing experiment only: results are wrong
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#else
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#endif
}
#ifdef ZS_NOCHAIN  // timing experiment only: each stage's newest z-neighbour is an older ring entry,
#define ZS_NC 1    // so the stages of a step do not depend on each other (results are wrong)
#else
#define ZS_NC 0
#endif
#ifdef ZS_NOLOAD  // timing experiment only: every plane reads plane 0 (cache-resident)
#define ZS_PLANE(q) 0
#else
#define ZS_PLANE(q) (q)
#endif

// Tile and column width: N cells of each colour per thread.  fp32 PRE uses 16-byte columns (7 waves,
// fewest instructions per cell: 576 us against 762 us with 8-byte columns at 512^3); fp32 POST,
// whose prolongation and err make it VALU-bound, uses 8-byte columns (14 waves: 642 against
// 756 us).  exp/run.sh A/B; ZS_NPRE_F32 / ZS_NPOST_F32 override.
#ifndef ZS_NPRE_F32
#define ZS_NPRE_F32 4
#endif
// Row-parity-uniform waves (ZS_PSPLIT, see ZsShape) and x-edge operands read raw at the extended tile's
// outer groups (ZS_XRAW: those cells lie in the halo that every stage shrinks by one cell, so their
// values never reach an owned cell and need no zeroing select)
#ifndef ZS_PSPLIT
#define ZS_PSPLIT 0
#endif
#ifndef ZS_PSPLIT_PRE
#define ZS_PSPLIT_PRE ZS_PSPLIT
#endif
#ifndef ZS_PSPLIT_POST
#define ZS_PSPLIT_POST ZS_PSPLIT
#endif
#ifndef ZS_XRAW
#define ZS_XRAW 1
#endif
#ifndef ZS_YROLE
#define ZS_YROLE 1
#endif
#ifndef ZS_XROLE  // (with ZS_YROLE: the tile rows' x-halo column groups in waves of their own)
#define ZS_XROLE 1
#endif
#ifndef ZS_XPAIR  // (with ZS_XROLE: tile rows r and r + 4 in each 16-lane pass of a tile wave)
#define ZS_XPAIR 1
#endif
#ifndef ZS_FHALO
#define ZS_FHALO 1
#endif
#ifndef ZS_NPOST_F32
#define ZS_NPOST_F32 2
#endif
// PRE tile height: 64 (less y halo, 12 waves) spills at the 168-VGPR cap and measured slower
// (640 against 578 us).  fp64 PRE: 32 x 32 tiles (8 waves, 216 VGPRs) instead of 64 x 16 (9 waves,
// spilling at the 168-VGPR cap): 1111 -> 800 us at 512^3; fp64 POST stays 64 x 16 (890 us against
// 999 / 1536 us for 32 x 32 / 32 x 16).
#ifndef ZS_TYPRE_F32
#define ZS_TYPRE_F32 32
#endif
#ifndef ZS_TYPOST_F32
#define ZS_TYPOST_F32 32
#endif
#ifndef ZS_TXPRE_F32
#define ZS_TXPRE_F32 64
#endif
#ifndef ZS_TXPOST_F32
#define ZS_TXPOST_F32 64
#endif
// PRE on a level with a boundary-modified operator (cl != 0): its own tile (the boundary diagonals cost
// registers: at the level-0 shape the variant spills)
#ifndef ZS_TXPRE_CL_F32
#define ZS_TXPRE_CL_F32 ZS_TXPRE_F32
#endif
#ifndef ZS_TYPRE_CL_F32
#define ZS_TYPRE_CL_F32 ZS_TYPRE_F32
#endif
#ifndef ZS_NPRE_CL_F32
#define ZS_NPRE_CL_F32 ZS_NPRE_F32
#endif
// POST's wide tile (levels with cl = 0 whose box it divides; MGP_ZS_WIDE=0 turns it off): a 64-wide tile's row
// of one colour is one 128-byte line, and its x halo (2 packed cells per side) touches the two neighbouring
// lines, so every row costs 3 line requests per field for 1 line of data; 128 x 16 tiles cost 4 for 2.
// 512^3 POST 480 -> 436 us (round 4).  Its 14 waves leave 128 VGPRs (a few spill).
#ifndef ZS_TXPOST_W_F32
#define ZS_TXPOST_W_F32 128
#endif
#ifndef ZS_TYPOST_W_F32
#define ZS_TYPOST_W_F32 16
#endif
#ifndef ZS_NPOST_W_F32  // (4: 128 x 16 POST at 18 x 24 threads measured 439 against 434 us)
#define ZS_NPOST_W_F32 ZS_NPOST_F32
#endif
template <typename T>
struct ZsTile;
template <>
struct ZsTile<float> {
    static constexpr int TXPRE = ZS_TXPRE_F32, TXPOST = ZS_TXPOST_F32, TYPRE = ZS_TYPRE_F32, TYPOST = ZS_TYPOST_F32,
                         NPRE = ZS_NPRE_F32, NPOST = ZS_NPOST_F32;
    static constexpr int TXPRE_CL = ZS_TXPRE_CL_F32, TYPRE_CL = ZS_TYPRE_CL_F32, NPRE_CL = ZS_NPRE_CL_F32;
    static constexpr int TXPOST_W = ZS_TXPOST_W_F32, TYPOST_W = ZS_TYPOST_W_F32, NPOST_W = ZS_NPOST_W_F32;
};
#ifndef ZS_TXPRE_F64
#define ZS_TXPRE_F64 32
#endif
#ifndef ZS_TXPOST_F64
#define ZS_TXPOST_F64 64
#endif
#ifndef ZS_TYPRE_F64
#define ZS_TYPRE_F64 32
#endif
#ifndef ZS_TYPOST_F64
#define ZS_TYPOST_F64 16
#endif
template <>
struct ZsTile<double> {
    static constexpr int TXPRE = ZS_TXPRE_F64, TXPOST = ZS_TXPOST_F64, TYPRE = ZS_TYPRE_F64, TYPOST = ZS_TYPOST_F64,
                         NPRE = 2, NPOST = 2;
    static constexpr int TXPRE_CL = TXPRE, TYPRE_CL = TYPRE, NPRE_CL = NPRE;
    static constexpr int TXPOST_W = TXPOST, TYPOST_W = TYPOST, NPOST_W = NPOST;  // (no wide fp64 variant is instantiated)
};
// Streaming (non-temporal) level-0 loads / stores of the phases: timing experiments (ZS_NT bit 0:
// loads, bit 1: stores), so that the level-0 stream does not evict the coarse level it writes
#ifndef ZS_NT
#define ZS_NT 0
#endif
// bit 2: psiOld loads only (read once per launch: nothing else in the launch reads them)
constexpr bool kZsNTL = (ZS_NT & 1) != 0, kZsNTS = (ZS_NT & 2) != 0, kZsNTO = (ZS_NT & 5) != 0;
#ifndef ZS_PRE_RED_STORE  // timing experiment: PRE stores its (unread) red cells too
#define ZS_PRE_RED_STORE 0
#endif
constexpr bool kZsPreRed = ZS_PRE_RED_STORE != 0;

// FWF (PRE only): the full-weighting restriction fused into the phase (k_zs LINEAR = 2): the residual is needed one
// cell beyond the tile (the full weighting's 4-cell stencil), so the trapezoid is one stage deeper (H = 6)
template <typename T, bool PRE, bool CLZ = true, bool WIDE = false, bool FWF = false>
struct ZsShape {
    static constexpr int N = PRE ? (CLZ ? ZsTile<T>::NPRE : ZsTile<T>::NPRE_CL)
                                 : (WIDE ? ZsTile<T>::NPOST_W : ZsTile<T>::NPOST);
    static constexpr int TX = PRE ? (CLZ ? ZsTile<T>::TXPRE : ZsTile<T>::TXPRE_CL)
                                  : (WIDE ? ZsTile<T>::TXPOST_W : ZsTile<T>::TXPOST);
    static constexpr int TY = PRE ? (CLZ ? ZsTile<T>::TYPRE : ZsTile<T>::TYPRE_CL)
                                  : (WIDE ? ZsTile<T>::TYPOST_W : ZsTile<T>::TYPOST);
    static constexpr int H = PRE ? (FWF ? 6 : 5) : 4;  // y/z halo = stages that read neighbours
    // x halo cells per side: the trapezoid depth H in whole column groups (2 N cells of x each)
#ifdef ZS_HX_FIXED  // timing experiment: the round-1 fixed 8-cell x halo
    static constexpr int HX = ZS_HX_FIXED;
#else
    static constexpr int HX = 2 * N * ((H + 2 * N - 1) / (2 * N));
#endif
    static constexpr int HWE = (TX + 2 * HX) / 2;      // reals per LDS half-row
    static constexpr int G = HWE / N;                  // column groups per row
    static constexpr int HXG = HX / 2 / N;             // halo groups per side
    static constexpr int YE = TY + 2 * H;
    static constexpr int NT = G * YE;                  // threads with a column
    // ZS_PSPLIT: the even extended rows in waves [0, NPAR / 64), the odd ones in the waves after them, so
    // that a wave's row parity is uniform and steady steps know every cell's colour at compile time
    static constexpr int YEV = (YE + 1) / 2;           // even extended rows
    static constexpr int NPAR = (G * YEV + 63) / 64 * 64;
    static constexpr bool PS = PRE ? ZS_PSPLIT_PRE != 0 : ZS_PSPLIT_POST != 0;
    static constexpr int NTL = PS ? 2 * NPAR : (NT + 63) / 64 * 64;  // launched threads
    // PRE, ZS_YROLE: threads ordered by their row's distance d from the tile in y (tile rows first, then d = 1..3,
    // then d = 4..5 from a wave boundary), so that whole waves hold only halo rows: stage k (half-sweep k) is needed
    // on rows d <= H - k and the residual on d = 0, so a wave of rows d >= 4 runs stage 1 only and a wave of rows
    // d in 1..3 skips the residual (a third of the step's VALU for the halo waves; only where it costs no wave)
    static constexpr int YT0 = TY * G, YT1 = YT0 + 6 * G, YT2S = (YT1 + 63) / 64 * 64, YT2 = YT2S + 4 * G;
    static constexpr bool YROLE = ZS_YROLE && PRE && !PS && H == 5 && (YT2 + 63) / 64 * 64 <= NTL;
    // ZS_XROLE: the tile rows' own columns (TC threads, whole waves) first, then their x-halo column groups (HXG per
    // side; those need stages 1..4 but no residual, role 1), so that the waves that run everything are TC / 64 (4 of
    // 7 at 64 x 32: one per SIMD, where 5 put two on one SIMD)
    static constexpr int GC = G - 2 * HXG, TC = TY * GC;
    static constexpr bool XROLE = YROLE && ZS_XROLE && TC % 64 == 0;
    // ZS_XPAIR (XROLE with 8 column groups per tile row and HWE = 40): a tile wave's 64 lanes hold 8 rows x 8
    // groups so that every 16-byte LDS access is conflict-free (MI355X_MICROARCH.md §LDS: ds_read_b128 serves the
    // lane groups {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31} (+32) with banks (a/4) mod 64, ds_write_b128 8
    // contiguous lanes with banks (a/4) mod 32).  Rows r and r + 4 start 160 words apart (32 mod 64), so each read
    // group holds two whole rows (lanes 0-31: rows 0, 4 and 1, 5; lanes 32-63: 2, 6 and 3, 7), and each write block
    // of 8 lanes holds 4 cells of each of two rows whose slots (mod 8) do not meet; row order / neighbour offsets
    // move every lane alike, so the x and y neighbour reads stay conflict-free.  (Row-major 8 x 8 lanes: 2-way.)
    static constexpr bool XPAIR = XROLE && ZS_XPAIR && GC == 8 && TY % 8 == 0 && HWE == 40;
    // lane l of a tile wave: quad q = (l & 31) >> 2 -> row xp_row(q) + 2 (l >> 5), group (xp_gx(q) + (l & 3)) & 7
    static __device__ __forceinline__ int xp_row(int q) { return (0x54450110 >> (4 * q)) & 15; }  // 0 1 1 0 5 4 4 5
    static __device__ __forceinline__ int xp_gx(int q) { return (0x64024620 >> (4 * q)) & 15; }   // 0 2 6 4 2 0 4 6
    // extended row (0 .. YE - 1) of thread t (-1: no row) and the role of wave w (0: tile rows, every stage and the
    // residual; 1: rows d <= 3 (XROLE: and the tile rows' x-halo groups), stages 1..4; 2: rows d >= 4, stage 1)
    static __device__ __forceinline__ int yrow(int t)
    {
        if (!YROLE) return t < NT ? t / G : -1;
        if (XPAIR && t < TC) return H + 8 * (t >> 6) + xp_row((t & 31) >> 2) + 2 * ((t >> 5) & 1);
        if (t < YT0) return H + (XROLE ? (t < TC ? t / GC : (t - TC) / (2 * HXG)) : t / G);
        // rows d = 1..3 (role 1) and d = 4, 5 (role 2): the ones above the tile, then the ones below, each in LDS row
        // order (conflict-free 16-byte accesses, where alternating above / below rows overlapped banks)
        if (t < YT1) {
            const int r = (t - YT0) / G;
            return r < 3 ? H - 3 + r : H + TY + r - 3;
        }
        if (t >= YT2S && t < YT2) {
            const int r = (t - YT2S) / G;
            return r < 2 ? H - 5 + r : H + TY + r + 1;
        }
        return -1;
    }
    static __device__ __forceinline__ int ycol(int t)
    {
        if (XROLE && t < YT0) {
            if (t < TC) return HXG + (XPAIR ? ((xp_gx((t & 31) >> 2) + (t & 3)) & 7) : t % GC);
            const int k = (t - TC) % (2 * HXG);
            return k < HXG ? k : GC + k;
        }
        return YROLE && t >= YT2S ? (t - YT2S) % G : t % G;
    }
    static constexpr int wave_role(int w)
    {
        return !YROLE || 64 * w < (XROLE ? TC : YT0) ? 0 : (64 * w < YT1 ? 1 : 2);
    }
    static constexpr int SLOT = YE * HWE;              // reals per LDS slot (one colour of a plane)
    // stage-3 slots: PRE's residual reads 2 back (3 needed; 4 while LDS allows: power-of-2 ring)
    static constexpr int NS3 = PRE ? (TY > 32 ? 3 : 4) : 2;
    static constexpr int OFF1 = 2 * SLOT, OFF2 = 4 * SLOT, OFF3 = 6 * SLOT, OFF4 = OFF3 + NS3 * SLOT;
    static constexpr int OFFX = OFF4 + (PRE ? 2 * SLOT : 0);
    static constexpr int XPAIRS = YE / 2 + 1;          // row pairs of the residual hand-off
    static constexpr int XSLOT = PRE ? XPAIRS * G * 2 * N : 0;
    // POST: coarse rows J in [Y0/2 - 3, Y0/2 + TY/2 + 3) and cells I in [X0/2 - 8, X0/2 + TX/2 + 8)
    // of 4 coarse planes around the stream position, unpacked (x order, both colours)
    static constexpr int CJ = PRE ? 0 : TY / 2 + 6, CI = PRE ? N : TX / 2 + 16;
    static constexpr int CSLOT = CJ * CI, CPAIRS = CSLOT / 2;
    static constexpr int OFFC = OFFX + 2 * XSLOT;
    // FWF: the residual rows in x order (RXSLOT per step parity), their x-combinations (AXSLOT per step parity) and a
    // ring of the y-combinations of 4 fine planes per coarse cell of the tile (AYSLOT per plane)
    static constexpr int RXSLOT = FWF ? YE * G * 2 * N : 0, AXSLOT = FWF ? YE * G * N : 0,
                         AYSLOT = FWF ? (TY / 2) * (TX / 2) : 0;  // (item i's N cells at i N)
    static constexpr int OFFRX = OFFC + 4 * CSLOT, OFFAX = OFFRX + 2 * RXSLOT, OFFAY = OFFAX + 2 * AXSLOT;
    // FWF: the wave running the y-combinations (the 4th when the workgroup has 7 waves: alone on its SIMD) and its
    // items per lane
    static constexpr int FWY = NTL >= 4 * 64 ? 3 : 0;
    static constexpr int FWYI = FWF ? (TY / 2) * (TX / (2 * N)) / 64 : 0;
    static_assert(!FWF || ((TY / 2) * (TX / (2 * N)) % 64 == 0 && FWY * 64 + 64 <= NTL), "FWF: whole waves of y items");
    static constexpr size_t lds_bytes = (size_t)(OFFAY + 4 * AYSLOT) * sizeof(T);
    static_assert(CPAIRS <= 2 * NTL, "coarse staging: two pairs per thread");
    static_assert(CI % N == 0 && OFFC % N == 0, "coarse rows must hold aligned groups");
    static_assert(NTL <= 1024, "too many threads");
    static_assert(2 * N * HXG >= H, "x halo too small");
    static_assert(HWE % N == 0, "LDS row must hold whole groups");
};

template <typename T, int N>
struct ZsPrefetch {
    Vec<T, N> u;                                       // stage 0: black cells of the input at plane p
    Vec<T, 2> cv[2];                                   // POST: this thread's coarse pairs for the ring
    Vec<T, N> f1, f2;  // f of half-sweeps 1 (red, plane p - 1) and 2 (black, plane p - 2); sweeps 3
                       // and 4 reuse them two steps later
    Vec<T, N> o0, o1;  // POST + ERR: psiOld (red, black) of plane p - 4, the plane step p finalizes
};

// Pin a prefetched vector: the compiler must have waited for its load before this point, and no
// memory access is moved across it.  Used at the top of a step so that the wait for plane p's loads
// (a vmcnt(0) once stores are pending: gfx9 counts loads and stores together) comes before plane
// p + 1's prefetch is issued, not after it.
template <typename T, int N>
__device__ __forceinline__ void zs_hold(const Vec<T, N>& a)
{
#pragma unroll
    for (int e = 0; e < N; ++e) asm volatile("" ::"v"(a.v[e]));
}

struct ZsCol {
    int lrow, lym, lyp, lxm, lxp, gm;
    bool x_first, x_last;
    bool xin;  // no cell of the group touches the x faces of the box (or the column is outside it)
};

// In-plane operands of one stage's cells: the other colour in the rows above / below and the x
// neighbours beyond my group (last cell of the left group, first of the right group).  Stage k
// reads them from the LDS slot stage k-1 filled one step earlier.
template <typename T, int N>
struct ZsNb {
    Vec<T, N> yl, yr;
    T ep, en;
};

template <typename T, int N>
__device__ __forceinline__ void zs_nb_load(ZsNb<T, N>& nb, const T* s_in, const ZsCol& c)
{
#ifdef ZS_NOLDSREAD  // timing experiment only: results are wrong
    nb.yl = nb.yr = vzero<T, N>();
    nb.ep = nb.en = (T)c.lrow;
    return;
#endif
    nb.yl = vload<T, N>(s_in + c.lym);
    nb.yr = vload<T, N>(s_in + c.lyp);
    // whole neighbouring groups (conflict-free), of which one cell each is used
    const Vec<T, N> l = vload_lds_whole<T, N>(s_in + c.lxm), r = vload_lds_whole<T, N>(s_in + c.lxp);
    nb.ep = (c.x_first && !ZS_XRAW) ? (T)0 : l.v[N - 1];
    nb.en = (c.x_last && !ZS_XRAW) ? (T)0 : r.v[0];
}

// xl + xr of my N cells of x parity o (IEEE addition commutes, so the pair sums are shared
// between the two parities)
template <typename T, int N>
__device__ __forceinline__ void zs_xsum(const Vec<T, N>& cen, const ZsNb<T, N>& nb, int o, T (&s)[N])
{
    const T edge = o == 0 ? nb.ep : nb.en;
    T m[N + 1];
    m[0] = edge + cen.v[0];
#pragma unroll
    for (int e = 0; e + 1 < N; ++e) m[e + 1] = cen.v[e] + cen.v[e + 1];
    m[N] = cen.v[N - 1] + edge;
#pragma unroll
    for (int e = 0; e < N; ++e) s[e] = o == 0 ? m[e] : m[e + 1];
}

// ((((xl + xr) + yl) + yr) + zl) + zr of my N cells
template <typename T, int N>
__device__ __forceinline__ void zs_nbsum(const Vec<T, N>& zl, const Vec<T, N>& cen, const Vec<T, N>& zr,
                                         const ZsNb<T, N>& nb, int o, T (&t)[N])
{
    zs_xsum<T, N>(cen, nb, o, t);
#pragma unroll
    for (int e = 0; e < N; ++e) {
        t[e] = t[e] + nb.yl.v[e];
        t[e] = t[e] + nb.yr.v[e];
        t[e] = t[e] + zl.v[e];
        t[e] = t[e] + zr.v[e];
    }
}

// Steady-step diagonals of a level with a boundary-modified operator (cl != 0): inside the z-range
// of the steady steps a cell's face count is nby (its row on a y face) plus 1 for the x-face cell,
// which can only be the first cell of a group at the left edge (x parity 0) or the last at the right
// edge (x parity 1).  db / yb = dg[nby] / RN(1/dg[nby]), de / ye = dg[nby + 1] / RN(1/dg[nby + 1]):
// the table Markstein division of Op::relax without selects over the whole table.
template <typename T>
struct ZsDiag {
    T db, yb, de, ye;
    bool left, right;
};

// dz's diagonals as register values.  Without the opaque copy the compiler turns `edge ? dz.de : dz.db`
// into a select of the two members' addresses and keeps dz in private memory: six scratch loads per
// step on every cl != 0 PRE step (5x the launch's vector memory reads, 670 against 407 us for the
// same launch with the cl = 0 code at 1024^2 x 128).
template <typename T>
__device__ __forceinline__ void zs_dvals(const ZsDiag<T>& dz, T& db, T& yb, T& de, T& ye)
{
    db = dz.db;
    yb = dz.yb;
    de = dz.de;
    ye = dz.ye;
    asm("" : "+v"(db), "+v"(yb), "+v"(de), "+v"(ye));
}

// One half-sweep of my N cells of one colour (x parity o) from the other colour's window
// (zl, cen, zr) and its in-plane operands: k_half's expressions.  Waves whose cells all have the
// interior diagonal (every wave of a level with cl = 0) take the reciprocal form, which is what
// Op::relax computes there.
// ask: the cells' neighbour sums times 1/h^2 (the askew of k_resrestrict's expression, same operands and
// order): a PRE black cell's residual one step later sees exactly these neighbours (zs_residual_a)
template <typename T, int N, bool CLZ, bool ST = false>
__device__ __forceinline__ Vec<T, N> zs_relax_a(const Vec<T, N>& zl, const Vec<T, N>& cen, const Vec<T, N>& zr,
                                                const ZsNb<T, N>& nb, const Vec<T, N>& fv, const ZsCol& c, int o,
                                                int nbyz, int nx, const Op<T, 3>& op, const ZsDiag<T>& dz,
                                                T (&ask)[N])
{
    Vec<T, N> out;
    T t[N];
    zs_nbsum<T, N>(zl, cen, zr, nb, o, t);
#pragma unroll
    for (int e = 0; e < N; ++e) ask[e] = t[e] * op.inv_hSq;
    if (!CLZ && ST) {
        T db, yb, de, ye;
        zs_dvals(dz, db, yb, de, ye);
#pragma unroll
        for (int e = 0; e < N; ++e) {
            const bool edge = (e == 0 && o == 0 && dz.left) || (e == N - 1 && o == 1 && dz.right);
            out.v[e] = div_rn(fv.v[e] - ask[e], edge ? de : db, edge ? ye : yb);
        }
    } else if (CLZ || __all(nbyz == 0 && c.xin)) {
#pragma unroll
        for (int e = 0; e < N; ++e) out.v[e] = div_rn(fv.v[e] - ask[e], op.adiag, op.yadiag);
    } else {
#pragma unroll
        for (int e = 0; e < N; ++e) {
            const int i = 2 * (c.gm + e) + o;
            out.v[e] = op.relax_direct(t[e], fv.v[e], nbyz + (i == 0) + (i == nx - 1));
        }
    }
    return out;
}

template <typename T, int N, bool CLZ, bool ST = false>
__device__ __forceinline__ Vec<T, N> zs_relax(const Vec<T, N>& zl, const Vec<T, N>& cen, const Vec<T, N>& zr,
                                              const ZsNb<T, N>& nb, const Vec<T, N>& fv, const ZsCol& c, int o,
                                              int nbyz, int nx, const Op<T, 3>& op, const ZsDiag<T>& dz)
{
    T ask[N];
    return zs_relax_a<T, N, CLZ, ST>(zl, cen, zr, nb, fv, c, o, nbyz, nx, op, dz, ask);
}

// Residual of my N cells of one colour (x parity o) at one plane: k_resrestrict's expressions.
template <typename T, int N, bool CLZ, bool ST = false>
__device__ __forceinline__ void zs_residual(const Vec<T, N>& zl, const Vec<T, N>& cen, const Vec<T, N>& zr,
                                            const ZsNb<T, N>& nb, const Vec<T, N>& uc, const Vec<T, N>& fv,
                                            const ZsCol& c, int o, int nbyz, int nx, const Op<T, 3>& op,
                                            const ZsDiag<T>& dz, T (&rr)[N])
{
    T t[N];
    zs_nbsum<T, N>(zl, cen, zr, nb, o, t);
    if (!CLZ && ST) {
        T db, yb, de, ye;
        zs_dvals(dz, db, yb, de, ye);
#pragma unroll
        for (int e = 0; e < N; ++e) {
            const bool edge = (e == 0 && o == 0 && dz.left) || (e == N - 1 && o == 1 && dz.right);
            const T askew = t[e] * op.inv_hSq;
            const T a_u = askew + (edge ? de : db) * uc.v[e];
            rr[e] = fv.v[e] - a_u;
        }
    } else if (CLZ || __all(nbyz == 0 && c.xin)) {
#pragma unroll
        for (int e = 0; e < N; ++e) {
            const T askew = t[e] * op.inv_hSq;
            const T a_u = askew + op.adiag * uc.v[e];
            rr[e] = fv.v[e] - a_u;
        }
    } else {
#pragma unroll
        for (int e = 0; e < N; ++e) {
            const int i = 2 * (c.gm + e) + o;
            rr[e] = op.residual_direct(t[e], fv.v[e], uc.v[e], nbyz + (i == 0) + (i == nx - 1));
        }
    }
}

// The same residual from the cells' askew (zs_relax_a of the half-sweep that last saw these neighbours)
template <typename T, int N, bool CLZ, bool ST = false>
__device__ __forceinline__ void zs_residual_a(const T (&ask)[N], const Vec<T, N>& uc, const Vec<T, N>& fv,
                                              const ZsCol& c, int o, int nbyz, int nx, const Op<T, 3>& op,
                                              const ZsDiag<T>& dz, T (&rr)[N])
{
    if (!CLZ && ST) {
        T db, yb, de, ye;
        zs_dvals(dz, db, yb, de, ye);
#pragma unroll
        for (int e = 0; e < N; ++e) {
            const bool edge = (e == 0 && o == 0 && dz.left) || (e == N - 1 && o == 1 && dz.right);
            const T a_u = ask[e] + (edge ? de : db) * uc.v[e];
            rr[e] = fv.v[e] - a_u;
        }
    } else if (CLZ || __all(nbyz == 0 && c.xin)) {
#pragma unroll
        for (int e = 0; e < N; ++e) {
            const T a_u = ask[e] + op.adiag * uc.v[e];
            rr[e] = fv.v[e] - a_u;
        }
    } else {
#pragma unroll
        for (int e = 0; e < N; ++e) {
            const int i = 2 * (c.gm + e) + o;
            const T a_u = ask[e] + op.diag_direct(nbyz + (i == 0) + (i == nx - 1)) * uc.v[e];
            rr[e] = fv.v[e] - a_u;
        }
    }
}

// uv += P V for my N cells of x parity o in one fine row (k_prolong_v's expressions).  Waves with
// no cell next to a face of the coarse box take the interior form (every factor is 1 there).
template <typename T, int N>
struct ZsCoarse {
    T c00[N + 2], c10[N + 2], c01[N + 2], c11[N + 2];  // [z: K / Kn][y: J / Jn], cells I0-1 .. I0+N
};

template <typename T, int N, int LINEAR>
__device__ __forceinline__ void zs_correct(Vec<T, N>& uv, const ZsCoarse<T, N>& cur, int o, int I0, int cx, bool oy,
                                           bool oz, T cl, bool fast)
{
    const T w0 = (T)0.75, w1 = (T)0.25;
    if (!LINEAR) {
#pragma unroll
        for (int e = 0; e < N; ++e) uv.v[e] = uv.v[e] + cur.c00[e + 1];
        return;
    }
    if (fast) {  // __all(!oy && !oz && I0 > 0 && I0 + N < cx), from the caller
#pragma unroll
        for (int e = 0; e < N; ++e) {
            const int pe = e + 1;
            const T nb00 = o ? cur.c00[e + 2] : cur.c00[e];
            const T nb10 = o ? cur.c10[e + 2] : cur.c10[e];
            const T nb01 = o ? cur.c01[e + 2] : cur.c01[e];
            const T nb11 = o ? cur.c11[e + 2] : cur.c11[e];
            const T a00 = w0 * cur.c00[pe] + w1 * nb00;
            const T a10 = w0 * cur.c10[pe] + w1 * nb10;
            const T a01 = w0 * cur.c01[pe] + w1 * nb01;
            const T a11 = w0 * cur.c11[pe] + w1 * nb11;
            const T b0 = w0 * a00 + w1 * a10;
            const T b1 = w0 * a01 + w1 * a11;
            uv.v[e] = uv.v[e] + (w0 * b0 + w1 * b1);
        }
        return;
    }
    auto sv = [&](T val, bool fx, bool fy, bool fz) {
        T s = (T)1;
        if (fx) s = -cl * s;
        if (fy) s = -cl * s;
        if (fz) s = -cl * s;
        return s == (T)1 ? val : s * val;
    };
#pragma unroll
    for (int e = 0; e < N; ++e) {
        const int pe = e + 1;
        const bool ox = (o == 0 && I0 + e == 0) || (o == 1 && I0 + e == cx - 1);
        auto col = [&](const T (&cc)[N + 2]) { return ox ? cc[pe] : (o ? cc[e + 2] : cc[e]); };
        const T a00 = w0 * cur.c00[pe] + w1 * sv(col(cur.c00), ox, false, false);
        const T a10 = w0 * sv(cur.c10[pe], false, oy, false) + w1 * sv(col(cur.c10), ox, oy, false);
        const T a01 = w0 * sv(cur.c01[pe], false, false, oz) + w1 * sv(col(cur.c01), ox, false, oz);
        const T a11 = w0 * sv(cur.c11[pe], false, oy, oz) + w1 * sv(col(cur.c11), ox, oy, oz);
        const T b0 = w0 * a00 + w1 * a10;
        const T b1 = w0 * a01 + w1 * a11;
        uv.v[e] = uv.v[e] + (w0 * b0 + w1 * b1);
    }
}

// The y-interpolated half of zs_correct for one coarse plane: b[e] = w0 a(J) + w1 a(Jn) with a = the
// x-interpolation of coarse row c0 (J) / c1 (Jn) (zs_correct's b0, or b1 with oz = false: the same
// expressions over the other plane).  A thread's rows J, Jn and its columns never change, so k_zs
// evaluates it once per coarse plane and x parity and keeps it in registers for the four fine planes
// that read the plane.
template <typename T, int N>
__device__ __forceinline__ void zs_bq(T (&b)[N], const T (&c0)[N + 2], const T (&c1)[N + 2], int o, int I0, int cx,
                                      bool oy, T cl, bool fast)
{
    const T w0 = (T)0.75, w1 = (T)0.25;
    if (fast) {
#pragma unroll
        for (int e = 0; e < N; ++e) {
            const T nb0 = o ? c0[e + 2] : c0[e];
            const T nb1 = o ? c1[e + 2] : c1[e];
            const T a0 = w0 * c0[e + 1] + w1 * nb0;
            const T a1 = w0 * c1[e + 1] + w1 * nb1;
            b[e] = w0 * a0 + w1 * a1;
        }
        return;
    }
    auto sv = [&](T val, bool fx, bool fy) {
        T s = (T)1;
        if (fx) s = -cl * s;
        if (fy) s = -cl * s;
        return s == (T)1 ? val : s * val;
    };
#pragma unroll
    for (int e = 0; e < N; ++e) {
        const int pe = e + 1;
        const bool ox = (o == 0 && I0 + e == 0) || (o == 1 && I0 + e == cx - 1);
        auto col = [&](const T (&cc)[N + 2]) { return ox ? cc[pe] : (o ? cc[e + 2] : cc[e]); };
        const T a0 = w0 * c0[pe] + w1 * sv(col(c0), ox, false);
        const T a1 = w0 * sv(c1[pe], false, oy) + w1 * sv(col(c1), ox, oy);
        b[e] = w0 * a0 + w1 * a1;
    }
}

// Fixed-order workgroup sum of one double per thread (NTL threads, any count <= 1024).
template <int NTL>
__device__ __forceinline__ void block_partial_t(double acc, double* partials)
{
    __shared__ double red[NTL];
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int w = 512; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w && (int)threadIdx.x + w < NTL) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) partials[blockIdx.x] = red[0];
}

// src: the level's u before the phase; dst: the phase's output; old (POST with ERR): psiOld, either dst
// itself (read plane by plane just before the output overwrites it) or a buffer of its own (kept for the
// reference's metrics, mgp_metrics / psiOld / errorBuf).  V/gc: coarse correction (POST); R/gc: restricted residual (PRE); both point at the
// coarse plane of local fine plane 0 (gc.z0 = g.z0 / 2).  zc: planes per z-chunk.  gz: readable
// ghost planes per side of src / f / dst (on a distributed level they must hold the neighbours'
// current H planes).  CLZ: the level operator has no boundary modification (cl == 0, level 0).
#ifndef ZS_WPE_PRE
#define ZS_WPE_PRE 2
#endif
// Prefetch distance in planes: step p issues the loads of plane p + PFD into one of PFD + 1 register
// buffers (the loop unrolls lcm(PFD + 1, 4) steps, so every buffer and ring index is static)
#ifndef ZS_PFD_PRE
#define ZS_PFD_PRE 2
#endif
#ifndef ZS_PFD_POST
#define ZS_PFD_POST 1
#endif
// PRE on a level with a boundary-modified operator (cl != 0, the coarser fused levels): distance 1 — at 2 the
// variant needed 54 (fp64: 33) VGPRs beyond the 256 of two waves per SIMD and spilled to scratch
#ifndef ZS_PFD_PRE_CL
#define ZS_PFD_PRE_CL 1
#endif
template <typename F, int... K>
__device__ __forceinline__ void zs_unroll_impl(F& f, std::integer_sequence<int, K...>)
{
    (f(std::integral_constant<int, K>()), ...);
}
// f(integral_constant<int, k>) for k = 0 .. U - 1, in order
template <int U, typename F>
__device__ __forceinline__ void zs_unroll(F&& f)
{
    zs_unroll_impl(f, std::make_integer_sequence<int, U>());
}
#ifndef ZS_BQ
#define ZS_BQ 1  // POST: per-thread cache of the coarse planes' y-interpolation (zs_bq)
#endif
// PRE: the black cells' residual reuses the askew of the stage-4 half-sweep that relaxed them one step earlier
// (the same red neighbours, sum order and scaling) instead of re-reading and re-summing those neighbours
#ifndef ZS_RASK
#define ZS_RASK 1
#endif
constexpr bool kZsRask = ZS_RASK != 0;
#ifndef ZS_WPE_POST
#define ZS_WPE_POST 4
#endif
template <typename T, bool PRE, int LINEAR, bool ERR, bool CLZ, bool WIDE = false>
__global__ __launch_bounds__((ZsShape<T, PRE, CLZ, WIDE, PRE && LINEAR == 2>::NTL))
__attribute__((amdgpu_waves_per_eu(1, PRE ? ZS_WPE_PRE : ZS_WPE_POST))) void k_zs(const T* __restrict__ src, const T* __restrict__ f,
                                                                T* __restrict__ dst, const T* old, T* __restrict__ R,
                                                                const T* __restrict__ V, double* __restrict__ partials,
                                                                Geo g, Geo gc, Op<T, 3> op, T clc, int zc, int gz,
                                                                int patch)
{
    // PRE: LINEAR selects the restriction: 0 = residual + 2^3 average here; 1 = none (both colours of the
    // smoothed level stored; the host runs the full-weighting restriction after the phase); 2 = residual + the full
    // weighting here (FWF)
    constexpr bool FWF = PRE && LINEAR == 2;
    using S = ZsShape<T, PRE, CLZ, WIDE, FWF>;
    constexpr int N = S::N, H = S::H, HWE = S::HWE, G = S::G, YE = S::YE, SLOT = S::SLOT, TX = S::TX,
                  TY = S::TY, NS3 = S::NS3, NTL = S::NTL;
    constexpr bool RR = PRE && LINEAR == 0;
    // PRE with ERR (which only POST uses): the input is a fresh zero guess, never loaded (src may be null); this
    // replaces the memset of a fused coarse level's u before its PRE
    constexpr bool ZSRC = PRE && ERR;
    using VT = Vec<T, N>;
    using PF = ZsPrefetch<T, N>;
    constexpr int PFD = PRE ? (CLZ ? ZS_PFD_PRE : ZS_PFD_PRE_CL) : ZS_PFD_POST, NPF = PFD + 1, UNR = NPF == 3 ? 12 : 4;
    static_assert(PFD >= 1 && PFD <= 3, "prefetch distance 1..3");
    extern __shared__ __align__(16) unsigned char zs_smem[];
    T* const lds = reinterpret_cast<T*>(zs_smem);
    const int tid = threadIdx.x;

    const int tiles_x = g.nx / TX, tiles_y = g.ny / TY;
    const int b = xcd_remap(blockIdx.x, gridDim.x);
    const int tile = b % (tiles_x * tiles_y);
    const int Z0 = (b / (tiles_x * tiles_y)) * zc;
    int tx_ = tile % tiles_x, ty_ = tile / tiles_x;
    if (patch) {  // the tiles an XCD runs at once form px x py patches (host: px | tiles_x, py | tiles_y)
        const int px = patch & 255, py = patch >> 8, per = px * py, prow = tiles_x / px;
        const int pi = tile / per, q = tile % per;
        tx_ = (pi % prow) * px + q % px;
        ty_ = (pi / prow) * py + q / px;
    }
    const int X0 = tx_ * TX, Y0 = ty_ * TY;
    const int hw = g.hw, Hh = (int)g.H;
    const int z0 = (int)g.z0, gnz = (int)g.gnz, cz0 = (int)gc.z0;
    const int64_t P = g.P;
    const int qlo = -gz, qhi = (int)g.nz - 1 + gz;  // readable local planes

    // my column of the extended tile; ZS_PSPLIT: wcls = my wave's row parity (even / odd extended rows)
    const int wcls = S::PS ? __builtin_amdgcn_readfirstlane(tid >= S::NPAR ? 1 : 0) : 0;
    const int rt_ = S::PS ? tid - wcls * S::NPAR : tid;
    const int yr_ = S::PS ? 0 : S::yrow(tid);
    const bool on = S::PS ? rt_ < G * (wcls ? YE / 2 : S::YEV) : yr_ >= 0;
    const int gx = on ? (S::PS ? rt_ % G : S::ycol(tid)) : 0, ye = S::PS ? (on ? 2 * (rt_ / G) + wcls : wcls) : (on ? yr_ : 0);
    const int gy = Y0 - H + ye;
    const int m0 = gx * N;
    ZsCol col;
    // LDS row of extended row y: ZS_PSPLIT stores the even rows first, then the odd ones, so that the rows
    // of one wave stay contiguous in LDS (conflict-free vector reads)
    auto lr = [&](int y) { return S::PS ? (y & 1) * S::YEV + (y >> 1) : y; };
    col.lrow = lr(ye) * HWE + m0;
    col.lym = lr(ye > 0 ? ye - 1 : ye) * HWE + m0;
    col.lyp = lr(ye < YE - 1 ? ye + 1 : ye) * HWE + m0;
    col.gm = (X0 - S::HX) / 2 + m0;  // global packed m of my first cell
    col.x_first = gx == 0;
    col.x_last = gx == G - 1;
    col.lxm = col.x_first ? col.lrow : col.lrow - N;
    col.lxp = col.x_last ? col.lrow : col.lrow + N;
    const bool in_xy = on && gy >= 0 && gy < g.ny && col.gm >= 0 && col.gm < hw;
    col.xin = !in_xy || (col.gm > 0 && 2 * (col.gm + N) < g.nx);
    // columns outside the box load from a clamped in-plane position; their results never reach
    // LDS or HBM
    const int cgy = gy < 0 ? 0 : (gy >= g.ny ? g.ny - 1 : gy);
    const int cgm = col.gm < 0 ? 0 : (col.gm > hw - N ? hw - N : col.gm);
#if defined(ZS_HALO_ALIAS)  // timing experiment only (wrong results): the halo's loads read the tile's own lines
    // bit 0: x-halo column groups load from owned columns; bit 1: y-halo rows load from owned rows
    const int agm = (ZS_HALO_ALIAS & 1) ? (gx < S::HXG ? cgm + S::HXG * N : (gx >= G - S::HXG ? cgm - S::HXG * N : cgm)) : cgm;
    const int agy = (ZS_HALO_ALIAS & 2) ? (ye < H ? cgy + H : (ye >= H + TY ? cgy - H : cgy)) : cgy;
    const int goff = agy * hw + agm;
#else
    const int goff = cgy * hw + cgm;  // in-plane offset (nx * ny < 2^31)
#endif
    const bool tile_xy = on && ye >= H && ye < H + TY && gx >= S::HXG && gx < G - S::HXG;
    // ZS_FHALO: the y-halo rows load only the f their stages can use: stage k is needed on rows d <= H - k from the
    // tile, so f1 (red f: stages 1 and 3) only on d <= H - 1 and f2 (black f: stages 2, 4, the residual) only on
    // d <= H - 2; the others keep zeros (their outputs lie outside every later stage's region)
    const int ydist = ye < H ? H - ye : (ye >= H + TY ? ye - (H + TY) + 1 : 0);
    // (POST only: in PRE it measured slower, 335.5 -> 341 us, against POST 435 -> 432 us at 512^3)
    const bool need_f1 = !ZS_FHALO || PRE || ydist <= H - 1, need_f2 = !ZS_FHALO || PRE || ydist <= H - 2;
    const int zlo = Z0 - H;
    ZsDiag<T> dz;
    {
        const int nby = (gy == 0) + (gy == g.ny - 1);  // 0 .. 2 (ny >= 2)
        dz.db = nby == 0 ? op.dg[0] : (nby == 1 ? op.dg[1] : op.dg[2]);
        dz.yb = nby == 0 ? op.ydg[0] : (nby == 1 ? op.ydg[1] : op.ydg[2]);
        dz.de = nby == 0 ? op.dg[1] : (nby == 1 ? op.dg[2] : op.dg[3]);
        dz.ye = nby == 0 ? op.ydg[1] : (nby == 1 ? op.ydg[2] : op.ydg[3]);
        dz.left = col.gm == 0;
        dz.right = col.gm + N == hw;
    }
    // (FWF: the x- and y-combinations of the full weighting follow the residual of plane p - 5 one and two steps later)
    const int p_end = Z0 + zc + (PRE ? (FWF ? 7 : 5) : 3);
    auto inz = [&](int q) { return z0 + q >= 0 && z0 + q < gnz; };  // inside the global box
    auto pcl = [&](int q) { return q < qlo ? qlo : (q > qhi ? qhi : q); };
    // ring slot of plane q (q may be negative; ns = 3 as q mod 3)
    auto slot = [&](int off, int ns, int q) {
        const int r = ns == 3 ? ((q % 3) + 3) % 3 : (q & (ns - 1));
        return lds + off + r * SLOT;
    };
    auto nbyz = [&](int q) {
        return CLZ ? 0 : (gy == 0) + (gy == g.ny - 1) + (z0 + q == 0) + (z0 + q == gnz - 1);
    };
    const int rowpar = (gy + z0) & 1;
    const int wrole = S::YROLE ? __builtin_amdgcn_readfirstlane(S::wave_role(tid >> 6)) : 0;  // (ZS_YROLE)
    const T* const src_black = ZSRC ? nullptr : src + Hh;

    for (int i = tid; i < (int)(S::lds_bytes / sizeof(T)); i += NTL) lds[i] = (T)0;
    __syncthreads();

    // ---- POST: coarse staging ring, plane K in slot K & 3 (planes clamped to the box) ----
    const int Ia = X0 / 2 - 8, Ja = Y0 / 2 - 3;
    auto ckl = [&](int K) { return K < 0 ? 0 : (K >= gc.gnz ? gc.gnz - 1 : K); };
    auto cslot = [&](int K) { return lds + S::OFFC + (K & 3) * S::CSLOT; };
    auto cload = [&](PF& r, int K) {
        K = ckl(K);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int t = tid + i * NTL;
            const int J = Ja + t / (S::CI / 2), I = Ia + 2 * (t % (S::CI / 2));
            r.cv[i].v[0] = r.cv[i].v[1] = (T)0;
            if (t < S::CPAIRS && J >= 0 && J < gc.ny && I >= 0 && I < gc.nx) {
                // I even: cells I and I + 1 sit at m = I / 2 of the two colour halves
                const T* row = V + (int64_t)(K - cz0) * gc.P + (int64_t)J * gc.hw + (I >> 1);
                const int ce = (I + J + K) & 1;
                r.cv[i].v[0] = row[ce * gc.H];
                r.cv[i].v[1] = row[(ce ^ 1) * gc.H];
            }
        }
    };
    auto cstore = [&](const PF& r, int K) {
        T* const sl = cslot(ckl(K));
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int t = tid + i * NTL;
            if (t < S::CPAIRS) vstore<T, 2>(sl + 2 * t, r.cv[i]);  // pair t: cells 2t, 2t + 1 of the region
        }
    };
    auto crow = [&](int K, int J, T (&c)[N + 2]) {  // cells cgm - 1 .. cgm + N of coarse row J, plane K
        const T* const sl = cslot(ckl(K)) + (J - Ja) * S::CI + (cgm - Ia);
        const Vec<T, N> mid = vload<T, N>(sl);
        c[0] = vload_lds_whole<T, N>(sl - N).v[N - 1];
#pragma unroll
        for (int e = 0; e < N; ++e) c[e + 1] = mid.v[e];
        c[N + 1] = vload_lds_whole<T, N>(sl + N).v[0];
    };

    // ST (steady): every plane the step touches lies inside the box, the readable planes and the
    // chunk, so the plane clamps and the box / chunk tests drop out and a step is one basic block
    // the scheduler can interleave (LDS reads of all stages up front).
    // In steady steps z0, Z0 and zc are even (checked before the steady loop), so the parity of p
    // is static within a step pair: zz0 / the caller's p carry it as known low bits and the parity
    // tests below fold away.
    auto prefetch = [&](auto st, PF& r, int p) {
        constexpr bool ST = decltype(st)::value;
        const int zz0 = ST ? (z0 & ~1) : z0;
        // POST: fine plane 2m + 1 is the first to need coarse plane m + 1; it is loaded with the
        // prefetch of plane 2m and put in the ring at the top of step 2m
        if (!PRE && ((zz0 + p) & 1) == 0) cload(r, ((zz0 + p) >> 1) + 1);
        if (ST) {  // one 64-bit plane offset, the others by subtraction
#ifdef ZS_NOLOAD
            const int64_t pP = 0, Pz = 0;  // every plane reads plane 0
#else
            const int64_t pP = (int64_t)p * P, Pz = P;
#endif
            if constexpr (ZSRC)
                r.u = vzero<T, N>();
            else
                r.u = gload<T, N, kZsNTL>(src_black + pP + goff);
            if (need_f1) r.f1 = gload<T, N, kZsNTL>(f + (pP - Pz) + goff);
            if (need_f2) r.f2 = gload<T, N, kZsNTL>(f + (pP - 2 * Pz) + Hh + goff);
            if (!PRE && ERR && tile_xy) {  // psiOld of plane p - 4, for the tile's own columns only
                const T* dp = old + (pP - 4 * Pz);
                r.o0 = gload<T, N, kZsNTO>(dp + goff);
                r.o1 = gload<T, N, kZsNTO>(dp + Hh + goff);
            }
        } else {
            if constexpr (ZSRC)
                r.u = vzero<T, N>();
            else
                r.u = gload<T, N, kZsNTL>(src_black + (int64_t)ZS_PLANE(pcl(p)) * P + goff);
            if (need_f1) r.f1 = gload<T, N, kZsNTL>(f + (int64_t)ZS_PLANE(pcl(p - 1)) * P + goff);
            if (need_f2) r.f2 = gload<T, N, kZsNTL>(f + (int64_t)ZS_PLANE(pcl(p - 2)) * P + Hh + goff);
            if (!PRE && ERR && tile_xy) {
                const T* dp = old + (int64_t)pcl(p - 4) * P;
                r.o0 = gload<T, N, kZsNTO>(dp + goff);
                r.o1 = gload<T, N, kZsNTO>(dp + Hh + goff);
            }
        }
    };

    const VT vz = vzero<T, N>();
    // Register rings of four planes: plane q lives in slot (q - zlo) & 3.  Every loop runs whole
    // groups of four steps, so each step knows its slot offset R = (p - zlo) & 3 at compile time and
    // the rings never move (no register rotation).
    VT W0[4], W1[4], W2[4], W3[4], W4[4], FR[4], FB[4];
    T AS[2][N];  // PRE (ZS_RASK): stage 4's askew of the last two steps (plane p - 4 at slot RS & 1)
#pragma unroll
    for (int e = 0; e < N; ++e) AS[0][e] = AS[1][e] = (T)0;
#pragma unroll
    for (int i = 0; i < 4; ++i) W0[i] = W1[i] = W2[i] = W3[i] = W4[i] = FR[i] = FB[i] = vz;
    // W0: A0 black at p-2 .. p; W1: A1 red at p-3 .. p-1; W2: A2 black at p-4 .. p-2;
    // W3: A3 red at p-6 .. p-3; W4: A4 black at p-6 .. p-4; FR: red f (cur.f1) of planes p-5 .. p-2;
    // FB: black f (cur.f2) of planes p-5 .. p-3
    T acc[N];
#pragma unroll
    for (int e = 0; e < N; ++e) acc[e] = (T)0;
    double err = 0.0, err1 = 0.0;
    const bool even_row_l = (gy & 1) == 0;
    T* const xbase = lds + S::OFFX + (((ye + (H & 1)) >> 1) * G + gx) * 2 * N;
    auto xs = [&](int q) { return xbase + (q & 1) * (S::XPAIRS * G * 2 * N); };

    // cur: plane p (loaded one step earlier); nxt: the buffer plane p + 1 is loaded into
    // POST: the per-lane half of the interior test of the coarse correction (loop invariant)
    const bool corr_lane = !PRE && (cgy >> 1) + ((cgy & 1) ? 1 : -1) >= 0 && (cgy >> 1) + ((cgy & 1) ? 1 : -1) < gc.ny &&
                           cgm > 0 && cgm + N < gc.nx;
    const bool corr_fast = __all(corr_lane);
    // POST, linear P, steady steps: BQ[K & 1][q][e] = zs_bq of coarse plane K for the black cells of the
    // fine planes of parity 1 ^ q (x parity q ^ (cgy & 1)).  Plane K + 1 is evaluated at odd step 2K + 1,
    // its first reader; fine plane p reads planes K and Kn = K +- 1, the two slots.
    T BQ[2][2][N];
#pragma unroll
    for (int i = 0; i < 2 * 2 * N; ++i) (&BQ[0][0][0])[i] = (T)0;
    const int bq_J = cgy >> 1;
    int bq_Jn = (cgy & 1) ? bq_J + 1 : bq_J - 1;
    const bool bq_oy = !PRE && (bq_Jn < 0 || bq_Jn >= gc.ny);
    if (bq_oy) bq_Jn = bq_J;
    auto bq_fill = [&](auto rp, T (&bq)[2][N], int K) {
        constexpr int RP = decltype(rp)::value;  // static row parity (>= 0) or runtime (-1)
        const int cp = RP >= 0 ? RP : (cgy & 1);
        T c0[N + 2], c1[N + 2];
        crow(K, bq_J, c0);
        crow(K, bq_Jn, c1);
#pragma unroll
        for (int q = 0; q < 2; ++q)
            zs_bq<T, N>(bq[q], c0, c1, q ^ cp, cgm, gc.nx, bq_oy, clc, corr_fast);
    };
    auto step = [&](auto st, auto rt, auto rp, auto ro, const PF& cur, PF& nxt, int p) __attribute__((always_inline)) {
        constexpr bool ST = decltype(st)::value;
        constexpr int RS = decltype(rt)::value;  // (p - zlo) & 3
        (void)ro;
        // my wave's role (ZsShape::wave_role, wave-uniform; every generic step runs the full work)
        const int RO = ST ? wrole : 0;
        // RP >= 0: my wave's row parity rowpar, known statically (ZS_PSPLIT steady steps: z0 and Y0 even, so
        // it is also the parity of gy); -1: per lane
        constexpr int RP = decltype(rp)::value;
        static_assert(RP < 0 || ST, "static row parity in steady steps only");
        auto par = [&](int q) { return RP >= 0 ? ((RP ^ q) & 1) : (rowpar ^ (q & 1)); };
        const bool even_row = RP >= 0 ? RP == 0 : even_row_l;
        // ring slot of plane p - k
        auto sl = [](int k) constexpr { return (RS - k) & 3; };
        // steady: Z0 even, so p's parity is zlo's plus RS
        if (ST) p = (p & ~1) | ((H + RS) & 1);
        const int zz0 = ST ? (z0 & ~1) : z0;
        zs_hold<T, N>(cur.u);
        zs_hold<T, N>(cur.f1);
        zs_hold<T, N>(cur.f2);
        if (!PRE && ERR) {
            zs_hold<T, N>(cur.o0);
            zs_hold<T, N>(cur.o1);
        }
        if (!PRE) {
            zs_hold<T, 2>(cur.cv[0]);
            zs_hold<T, 2>(cur.cv[1]);
        }
        asm volatile("" ::: "memory");
        // POST: the coarse plane cur's prefetch loaded (first read one step on; the slot it replaces
        // was last read three steps back)
        if (!PRE && ((zz0 + p) & 1) == 0) cstore(cur, ((zz0 + p) >> 1) + 1);
        if (ST || p + PFD <= p_end) prefetch(st, nxt, p + PFD);

        // Every LDS read of a step hits a slot filled in the previous step (the writes come after
        // the stages), so the compiler may schedule them as early as registers allow.
        ZsNb<T, N> n1, n2, n3, n4, nr, nk;

        // ---- stage 0: black cells of plane p ----
        VT a0 = cur.u;
        if constexpr (!PRE && ST && LINEAR == 1 && ZS_BQ) {
            // (z0 + Z0) % 4 == 0 in steady steps: K & 1 and p & 1 are static
            constexpr int KS = (RS >> 1) & 1, Q = 1 ^ (RS & 1);
            if constexpr ((RS & 1) != 0) bq_fill(rp, BQ[KS ^ 1], ((zz0 + p) >> 1) + 1);
            const T w0 = (T)0.75, w1 = (T)0.25;
#pragma unroll
            for (int e = 0; e < N; ++e) a0.v[e] = a0.v[e] + (w0 * BQ[KS][Q][e] + w1 * BQ[KS ^ 1][Q][e]);
        } else if (!PRE && (ST || inz(p))) {
            const int J = cgy >> 1, K = (zz0 + p) >> 1;
            int Jn = (cgy & 1) ? J + 1 : J - 1;
            int Kn = ((zz0 + p) & 1) ? K + 1 : K - 1;
            const bool oy = Jn < 0 || Jn >= gc.ny, oz = !ST && (Kn < 0 || Kn >= gc.gnz);
            if (oy) Jn = J;
            if (oz) Kn = K;
            ZsCoarse<T, N> cc;
            crow(K, J, cc.c00);
            if (LINEAR) {
                crow(K, Jn, cc.c10);
                crow(Kn, J, cc.c01);
                crow(Kn, Jn, cc.c11);
            }
            zs_correct<T, N, LINEAR>(a0, cc, 1 ^ ((cgy + zz0 + p) & 1), cgm, gc.nx, oy, oz, clc,
                                     ST ? corr_fast : __all(!oy && !oz && cgm > 0 && cgm + N < gc.nx));
        }
        if (!ST && !inz(p)) a0 = vz;
        W0[sl(0)] = a0;

        // ---- stages 1..4: half-sweep k on plane p - k (red, black, red, black) ----
        zs_nb_load<T, N>(n1, slot(0, 2, p - 1), col);
        VT o1 = zs_relax<T, N, CLZ, ST>(W0[sl(2)], W0[sl(1)], W0[sl(ZS_NC ? 3 : 0)], n1, cur.f1, col, par(p - 1), nbyz(p - 1), g.nx, op, dz);
        if (!ST && !inz(p - 1)) o1 = vz;
        W1[sl(1)] = o1;
        // (a wave of halo rows d >= 4, role 2, needs stage 1 only: its stages 2..4 would feed no needed cell)
        VT o2 = vz, o3 = vz, o4 = vz;
        if (RO < 2) {
            zs_nb_load<T, N>(n2, slot(S::OFF1, 2, p - 2), col);
            o2 = zs_relax<T, N, CLZ, ST>(W1[sl(3)], W1[sl(2)], W1[sl(ZS_NC ? 0 : 1)], n2, cur.f2, col, 1 ^ par(p - 2), nbyz(p - 2),
                                         g.nx, op, dz);
            if (!ST && !inz(p - 2)) o2 = vz;
            W2[sl(2)] = o2;
            zs_nb_load<T, N>(n3, slot(S::OFF2, 2, p - 3), col);
            o3 = zs_relax<T, N, CLZ, ST>(W2[sl(4)], W2[sl(3)], W2[sl(ZS_NC ? 1 : 2)], n3, FR[sl(3)], col, par(p - 3), nbyz(p - 3),
                                         g.nx, op, dz);
            if (!ST && !inz(p - 3)) o3 = vz;
            W3[sl(3)] = o3;
            zs_nb_load<T, N>(n4, slot(S::OFF3, NS3, p - 4), col);
            o4 = zs_relax_a<T, N, CLZ, ST>(W3[sl(5)], W3[sl(4)], W3[sl(ZS_NC ? 2 : 3)], n4, FB[sl(4)], col, 1 ^ par(p - 4),
                                           nbyz(p - 4), g.nx, op, dz, AS[RS & 1]);
            if (!ST && !inz(p - 4)) o4 = vz;
            W4[sl(4)] = o4;
        }

        // ---- LDS writes (slots no stage of this step reads); columns outside the box stay 0 ----
        if (in_xy) {
            vstore<T, N>(slot(0, 2, p) + col.lrow, a0);
            vstore<T, N>(slot(S::OFF1, 2, p - 1) + col.lrow, o1);
            if (RO < 2) {
                vstore<T, N>(slot(S::OFF2, 2, p - 2) + col.lrow, o2);
                vstore<T, N>(slot(S::OFF3, NS3, p - 3) + col.lrow, o3);
                if (RR || FWF) vstore<T, N>(slot(S::OFF4, 2, p - 4) + col.lrow, o4);
            }
        }

        // ---- the smoothed plane p - 4: red final after stage 3, black after stage 4 ----
        // (the chunk test is wave-uniform: steady steps also run the trapezoid's warm-up before the chunk and
        // its drain after it, which store nothing)
        if (RO == 0) {
            const int q = p - 4;
            if (q >= Z0 && q < Z0 + zc && tile_xy) {
                if (!PRE && ERR) {
#pragma unroll
                    for (int e = 0; e < N; ++e) {
                        // (psi - psiOld)^2 in fp64, fused multiply-add into two accumulators (err
                        // matches the oracle's sum to summation order, not bit for bit)
                        const double d0 = (double)W3[sl(4)].v[e] - (double)cur.o0.v[e];
                        const double d1 = (double)o4.v[e] - (double)cur.o1.v[e];
                        err = __builtin_fma(d0, d0, err);
                        err1 = __builtin_fma(d1, d1, err1);
                    }
                }
                T* dp = dst + (int64_t)q * P;
                // PRE: the red cells are not stored.  Its output is read only by POST, whose stage 0
                // loads the black cells (the first post half-sweep replaces the red ones unread).
                if (!(RR || FWF) || kZsPreRed) gstore<T, N, kZsNTS>(dp + goff, W3[sl(4)]);
                gstore<T, N, kZsNTS>(dp + Hh + goff, o4);
            }
        }

        // ---- PRE: residual + restriction of plane p - 5 (tile rows only: role 0) ----
        if (RR && RO == 0) {
            const int q = p - 5;
            const int pq = par(q);
            if (!kZsRask) zs_nb_load<T, N>(nr, slot(S::OFF3, NS3, q), col);  // red of A4 at q
            zs_nb_load<T, N>(nk, slot(S::OFF4, 2, q), col);                  // black of A4 at q
            T xr[2 * N];
            {
                const T* x = xs(q - 1);  // the odd row's residuals of plane q - 1 (even rows read them)
#pragma unroll
                for (int e = 0; e < 2 * N; ++e) xr[e] = x[e];
            }
            // red cells (x parity pq) see black neighbours, black cells (x parity 1 - pq) red ones
            T rred[N], rblk[N], rr[2][N];  // rr: [x parity][e]
            zs_residual<T, N, CLZ, ST>(W4[sl(6)], W4[sl(5)], W4[sl(ZS_NC ? 3 : 4)], nk, W3[sl(5)], FR[sl(5)], col, pq, nbyz(q), g.nx, op,
                                   dz, rred);
            // the black cells' neighbours are the red cells of the last step's stage 4 (its askew, ZS_RASK)
            if (kZsRask)
                zs_residual_a<T, N, CLZ, ST>(AS[(RS & 1) ^ 1], W4[sl(5)], FB[sl(5)], col, 1 ^ pq, nbyz(q), g.nx, op, dz,
                                             rblk);
            else
                zs_residual<T, N, CLZ, ST>(W3[sl(6)], W3[sl(5)], W3[sl(4)], nr, W4[sl(5)], FB[sl(5)], col, 1 ^ pq, nbyz(q),
                                           g.nx, op, dz, rblk);
#pragma unroll
            for (int e = 0; e < N; ++e) {
                rr[0][e] = pq == 0 ? rred[e] : rblk[e];
                rr[1][e] = pq == 0 ? rblk[e] : rred[e];
            }
            const int dq = q - (ST ? (Z0 & ~1) : Z0);
            if (dq >= 0 && dq <= zc && tile_xy) {
                if (!even_row) {
                    if (dq < zc) {
                        T* x = xs(q);
#pragma unroll
                        for (int e = 0; e < N; ++e) {
                            x[e] = rr[0][e];
                            x[N + e] = rr[1][e];
                        }
                    }
                } else {
                    if (dq >= 1) {  // the odd row's children of plane q - 1
#pragma unroll
                        for (int e = 0; e < N; ++e) {
                            acc[e] = acc[e] + xr[e];
                            acc[e] = acc[e] + xr[N + e];
                        }
                        if ((dq & 1) == 0) {  // coarse plane (q - 1) / 2 complete
                            const int K = (zz0 + q - 1) >> 1, J = gy >> 1;  // global
                            T* rowc = R + (int64_t)(K - cz0) * gc.P + (int64_t)J * gc.hw;
#pragma unroll
                            for (int e = 0; e < N; ++e) {
                                const int I = col.gm + e;
                                rowc[((I + J + K) & 1) * gc.H + (I >> 1)] = (T)0.125 * acc[e];
                            }
                        }
                    }
                    if (dq < zc) {
#pragma unroll
                        for (int e = 0; e < N; ++e) {
                            if ((dq & 1) == 0) {
                                acc[e] = rr[0][e] + rr[1][e];
                            } else {
                                acc[e] = acc[e] + rr[0][e];
                                acc[e] = acc[e] + rr[1][e];
                            }
                        }
                    }
                }
            }
        }
        // ---- PRE, FWF: residual of plane p - 5 into RX, the x-combination of plane p - 6, the y-combination and the
        // coarse planes of plane p - 7 (fw_eval's order; cells outside the box weigh 0) ----
        if constexpr (FWF) {
            const int q = p - 5;
            const int pq = par(q);
            if (!kZsRask) zs_nb_load<T, N>(nr, slot(S::OFF3, NS3, q), col);
            zs_nb_load<T, N>(nk, slot(S::OFF4, 2, q), col);
            T rred[N], rblk[N];
            zs_residual<T, N, CLZ, ST>(W4[sl(6)], W4[sl(5)], W4[sl(ZS_NC ? 3 : 4)], nk, W3[sl(5)], FR[sl(5)], col, pq, nbyz(q), g.nx, op,
                                   dz, rred);
            if (kZsRask)
                zs_residual_a<T, N, CLZ, ST>(AS[(RS & 1) ^ 1], W4[sl(5)], FB[sl(5)], col, 1 ^ pq, nbyz(q), g.nx, op, dz,
                                             rblk);
            else
                zs_residual<T, N, CLZ, ST>(W3[sl(6)], W3[sl(5)], W3[sl(4)], nr, W4[sl(5)], FB[sl(5)], col, 1 ^ pq, nbyz(q),
                                           g.nx, op, dz, rblk);
            const bool rin = in_xy && (ST || inz(q));  // (the residuals of cells outside the box weigh 0)
            // RX: the group's 2N cells in x order, the low N at t N and the high N at RXH + t N (t = ye G + gx), so
            // that every access is one conflict-free 16-byte vector per lane
            constexpr int RXH = S::RXSLOT / 2;
            const int t = ye * G + gx;
            if (ydist <= 1) {  // (rows within one of the tile: the only ones the x-combination reads)
                VT x[2];  // x order: cell 2 (gm + e) + parity
#pragma unroll
                for (int e = 0; e < N; ++e) {
                    x[(2 * e) / N].v[(2 * e) % N] = rin ? (pq ? rblk[e] : rred[e]) : (T)0;
                    x[(2 * e + 1) / N].v[(2 * e + 1) % N] = rin ? (pq ? rred[e] : rblk[e]) : (T)0;
                }
                T* const rxw = lds + S::OFFRX + (p & 1) * S::RXSLOT + t * N;
                vstore<T, N>(rxw, x[0]);
                vstore<T, N>(rxw + RXH, x[1]);
            }
            const T wfv = (T)3 - clc, w3 = (T)3;
            // the x-combination of plane p - 6 (written to RX one step ago) for the tile's coarse columns, rows within
            // one of the tile: fine cells 2I - 1 .. 2I + 2 of coarse I = gm + e
            const bool tile_x = gx >= S::HXG && gx < G - S::HXG;
            if (tile_x && ydist <= 1) {
                const T* rxr = lds + S::OFFRX + ((p - 1) & 1) * S::RXSLOT;
                T x[2 * N + 2];
                const VT lo = vload_lds_whole<T, N>(rxr + t * N), hi = vload_lds_whole<T, N>(rxr + RXH + t * N);
                x[0] = vload_lds_whole<T, N>(rxr + RXH + (t - 1) * N).v[N - 1];
                x[2 * N + 1] = vload_lds_whole<T, N>(rxr + (t + 1) * N).v[0];
#pragma unroll
                for (int e = 0; e < N; ++e) {
                    x[1 + e] = lo.v[e];
                    x[1 + N + e] = hi.v[e];
                }
                const int cxn = g.nx >> 1;
                VT ax;
#pragma unroll
                for (int e = 0; e < N; ++e) {
                    const int I = col.gm + e;
                    ax.v[e] = fw_axis(x[2 * e], x[2 * e + 1], x[2 * e + 2], x[2 * e + 3], I == 0 ? wfv : w3,
                                      I == cxn - 1 ? wfv : w3);
                }
                vstore<T, N>(lds + S::OFFAX + (p & 1) * S::AXSLOT + t * N, ax);
            }
            // the y-combination of plane p - 7 (its x-combinations were written one step ago) for every coarse cell
            // group of the tile (coarse row J: fine rows 2J - 1 .. 2J + 2), then coarse plane K when p - 7 = 2K + 2.
            // The TY / 2 x TX / (2 N) items run in wave FWY (ZsShape: the wave that shares no SIMD when the
            // workgroup has 4 k + 3 waves), each item on the same lane every step (the AY ring is lane-private)
            if (tid >= S::FWY * 64 && tid < S::FWY * 64 + 64) {
                const T* axr = lds + S::OFFAX + ((p - 1) & 1) * S::AXSLOT;
                const int cyn = g.ny >> 1, q2 = p - 7;
                const int dq2 = q2 - 2 - (ST ? (Z0 & ~1) : Z0);  // 2K - z0 - Z0 for the coarse plane K ending at q2
                const bool emit = dq2 >= 0 && dq2 < zc && (dq2 & 1) == 0;
                const int K = (z0 + q2 - 2) >> 1;  // global coarse plane
                const T wk0 = K == 0 ? wfv : w3, wk1 = K == gc.gnz - 1 ? wfv : w3;
                constexpr int CG = TX / (2 * N);  // coarse groups per coarse row
#pragma unroll
                for (int k = 0; k < S::FWYI; ++k) {
                    const int i = tid - S::FWY * 64 + 64 * k;
                    const int jl = i / CG, cg = i % CG;
                    const int J = (Y0 >> 1) + jl, ty = (H + 2 * jl) * G + S::HXG + cg;
                    const VT a0 = vload_lds_whole<T, N>(axr + (ty - G) * N), a1 = vload_lds_whole<T, N>(axr + ty * N),
                             a2 = vload_lds_whole<T, N>(axr + (ty + G) * N), a3 = vload_lds_whole<T, N>(axr + (ty + 2 * G) * N);
                    const T wj0 = J == 0 ? wfv : w3, wj1 = J == cyn - 1 ? wfv : w3;
                    VT ay;
#pragma unroll
                    for (int e = 0; e < N; ++e) ay.v[e] = ((a0.v[e] + wj0 * a1.v[e]) + wj1 * a2.v[e]) + a3.v[e];
                    T* const ayb = lds + S::OFFAY + i * N;
                    vstore<T, N>(ayb + (q2 & 3) * S::AYSLOT, ay);
                    if (emit) {
                        const VT b0 = vload_lds_whole<T, N>(ayb + ((q2 - 3) & 3) * S::AYSLOT),
                                 b1 = vload_lds_whole<T, N>(ayb + ((q2 - 2) & 3) * S::AYSLOT),
                                 b2 = vload_lds_whole<T, N>(ayb + ((q2 - 1) & 3) * S::AYSLOT);
                        // coarse cells I = gm .. gm + N - 1 (gm even): the even ones at m = gm / 2 .. of one colour
                        // half, the odd ones of the other
                        const int gm = X0 / 2 + cg * N;
                        T* rowc = R + (int64_t)(K - cz0) * gc.P + (int64_t)J * gc.hw + (gm >> 1);
                        Vec<T, N / 2> ev, od;
#pragma unroll
                        for (int e = 0; e < N; ++e) {
                            const T az = ((b0.v[e] + wk0 * b1.v[e]) + wk1 * b2.v[e]) + ay.v[e];
                            if (e & 1)
                                od.v[e >> 1] = (T)(1.0 / 512.0) * az;
                            else
                                ev.v[e >> 1] = (T)(1.0 / 512.0) * az;
                        }
                        const int ce = (gm + J + K) & 1;
                        vstore<T, N / 2>(rowc + ce * gc.H, ev);
                        vstore<T, N / 2>(rowc + (ce ^ 1) * gc.H, od);
                    }
                }
            }
        }
        FR[sl(1)] = cur.f1;  // red f of plane p - 1 (replaces p - 5, read above)
        FB[sl(2)] = cur.f2;  // black f of plane p - 2
        lds_barrier();
    };

    const std::false_type GEN;
    const std::true_type STY;
    PF pb[NPF];
#pragma unroll
    for (int k = 0; k < NPF; ++k) pb[k].f1 = pb[k].f2 = vz;  // (the halo rows that skip f loads keep zeros)
    if (!PRE) {  // the coarse planes the first fine plane needs
        const int K = (z0 + zlo) >> 1;
        for (int k = K - 1; k <= K + 1; ++k) {
            cload(pb[0], k);
            cstore(pb[0], k);
        }
        __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < PFD; ++k) prefetch(GEN, pb[k], zlo + k);
    // steady steps [ps, pe]: stages inside the box (z0 + p - 5 >= 1, z0 + p < gnz) and the prefetched planes
    // (p + PFD .. p - 4) readable; the chunk's warm-up and drain steps are steady too (their stores are skipped
    // by the uniform chunk test), so a chunk away from the box faces runs no generic step at all (the short
    // chunks of the coarser fused levels were ~45 % generic steps before)
    int ps = zlo, pe = p_end;
    ps = ps > 6 - z0 ? ps : 6 - z0;  // PRE's residual plane p - 5 off the z face (steady diagonals have no z face)
    ps = ps > qlo + 4 ? ps : qlo + 4;
    pe = pe < gnz - (PRE ? 1 : 2) - z0 ? pe : gnz - (PRE ? 1 : 2) - z0;  // POST: Kn inside the coarse box
    pe = pe < qhi - PFD ? pe : qhi - PFD;
    ps += (UNR - (ps - zlo) % UNR) % UNR;  // whole groups of UNR steps in the prologue
    pe -= (pe - ps + 1) % UNR;             // and in the steady part
    // no steady part (the epilogue takes all) without a whole group or with odd z0 / Z0 (static parity)
    // POST with the BQ cache: (z0 + Z0) % 4 == 0 as well (static parity of the coarse plane)
#ifndef ZS_ALL_GENERIC  // timing experiment: every step generic (the price of the box-face steps)
#define ZS_ALL_GENERIC 0
#endif
    if (ZS_ALL_GENERIC || pe < ps || ((z0 | Z0) & 1) || (!PRE && LINEAR == 1 && ZS_BQ && ((z0 + Z0) & 3))) ps = pe = zlo - 1;
    int p = zlo;
    const std::integral_constant<int, -1> RPL;
    // UNR steps from p0 (p0 - zlo a multiple of UNR): ring slot k & 3, buffers k % NPF and (k + PFD) % NPF;
    // steps past plim are skipped (epilogue)
    const std::integral_constant<int, 0> RO0;
    auto group = [&](auto st, auto rp, auto ro, int p0, int plim) __attribute__((always_inline)) {
        zs_unroll<UNR>([&](auto kk) __attribute__((always_inline)) {
            constexpr int k = decltype(kk)::value;
            if (k == 0 || p0 + k <= plim)
                step(st, std::integral_constant<int, (k & 3)>(), rp, ro, pb[k % NPF], pb[(k + PFD) % NPF], p0 + k);
        });
    };
    for (; p < ps; p += UNR) group(GEN, RPL, RO0, p, p + UNR);
    auto steady = [&](auto rp, auto ro) __attribute__((always_inline)) {
        if constexpr (!PRE && LINEAR == 1 && ZS_BQ) {
            if (p <= pe) {  // the first steady step (even, K & 1 == 0) reads coarse planes K and K - 1
                const int K = (z0 + p) >> 1;
                bq_fill(rp, BQ[0], K);
                bq_fill(rp, BQ[1], K - 1);
            }
        }
        for (; p <= pe; p += UNR) {
#ifdef ZS_STAMP  // timing experiment (wrong results): POST's wall clock every 16 steps into R (level 1's f)
            if (!PRE && tid == 0 && ((p - zlo) & 15) == 0 && (p - zlo) / 16 < 32) {
                const unsigned long long w = wall_clock64();
                float* out = reinterpret_cast<float*>(R) + 64 * (int)blockIdx.x + 2 * ((p - zlo) / 16);
                out[0] = __uint_as_float((unsigned)(w & 0xffffffffu));
                out[1] = __uint_as_float((unsigned)(w >> 32));
            }
#endif
            group(STY, rp, ro, p, p + UNR);
        }
    };
    if constexpr (S::PS) {  // wave-uniform: one copy of the steady loop per row parity
        if (((H + wcls) & 1) == 0)
            steady(std::integral_constant<int, 0>(), RO0);
        else
            steady(std::integral_constant<int, 1>(), RO0);
    } else {
        steady(RPL, RO0);
    }
    for (; p <= p_end; p += UNR) group(GEN, RPL, RO0, p, p_end);
    if constexpr (ERR && !PRE) block_partial_t<NTL>(err + err1, partials);  // (PRE: ERR is ZSRC, no partials)
}

// ---- y-streamed temporally blocked smoothing (2D, red/black 2+2) -------------------------------
//
// k_ys is k_zs for a 2D level: rows take the place of planes.  A workgroup owns an x-segment of TX cells
// (plus HX halo cells per side) and a chunk of yc rows, and streams through y; every thread owns one
// column group of the segment: N consecutive cells of each colour (packed m0 .. m0 + N - 1).  At step p:
//   stage 0   black cells of row p (POST: plus the prolongation, PvRow: k_prolong_v's expressions)
//   stage k   half-sweep k (k = 1..4, red first) on row p - k
//   last      row p - 4 is final and stored; PRE: residual of row p - 5 and the restriction (both fine rows
//             of a coarse row belong to the same thread, so the children are summed in registers in the
//             reference order); POST: (psi - psiOld)^2 partials.
// The y-neighbours of stage k are the thread's own register windows of stage k - 1; the only operands
// from other threads are the two x-edge cells, which every stage leaves in LDS (first and last cell of
// its group) for the next stage one step later: one barrier per step.  Halo cells are recomputed by the
// neighbouring segments (the trapezoid shrinks by one cell per stage); rows outside the box are 0.  With
// yc even, Y0 is even and the parity of row p is a compile-time function of the ring slot.  Arithmetic is
// k_half's / k_resrestrict's / k_prolong_v's, so results are bit-identical to the per-piece path.
#ifndef YS_TX_F32
#define YS_TX_F32 1024
#endif
#ifndef YS_TX_F64
#define YS_TX_F64 512
#endif
template <typename T>
constexpr int ys_tx_full() { return sizeof(T) == 4 ? YS_TX_F32 : YS_TX_F64; }
// TXV: segment width (ys_tx_full, or half of it on levels whose full-width segments make too few workgroups)
template <typename T, bool PRE, int TXV = ys_tx_full<T>()>
struct YsShape {
    static constexpr int N = 16 / sizeof(T);
    static constexpr int TX = TXV;
    static constexpr int H = PRE ? 5 : 4;
    static constexpr int HX = 2 * N * ((H + 2 * N - 1) / (2 * N));  // whole column groups
    static constexpr int HWE = TX / 2 + HX;                          // packed cells per colour of a row
    static constexpr int G = HWE / N;                                // column groups (threads with work)
    static constexpr int HXG = HX / 2 / N;
    static constexpr int NTL = (G + 63) / 64 * 64;
    // edge slots (first, last cell of every group): stages 0..2 two rows each, stage 3 four (PRE reads
    // its row p - 5 at step p), stage 4 two (PRE)
    static constexpr int ES = 2 * G;
    static constexpr int OFF1 = 2 * ES, OFF2 = 4 * ES, OFF3 = 6 * ES, OFF4 = 10 * ES;
    // POST: ring of 4 coarse rows (cells I in [X0/2 - 8, X0/2 + TX/2 + 8), x order, both colours)
    static constexpr int CI = PRE ? 0 : TX / 2 + 16, CPAIRS = CI / 2, OFFC = 12 * ES;
    static constexpr size_t lds_floats = 12 * ES + 4 * CI;
    static_assert(CPAIRS <= 2 * NTL, "coarse staging: two pairs per thread");
    static_assert(NTL <= 1024, "too many threads");
    static_assert(2 * N * HXG >= H, "x halo too small");
};

// Rows prefetched YS_PF steps ahead (a ring of 4 buffers, so every index stays static in the 4-step loop).
#ifndef YS_PF
#define YS_PF 2
#endif
static_assert(YS_PF >= 1 && YS_PF <= 3, "prefetch distance 1..3");
template <typename T>
struct YsPrefetch {
    static constexpr int N = 16 / sizeof(T);
    Vec<T, N> u, f1, f2, o0, o1;  // black u of row p; red f of p - 1; black f of p - 2; psiOld of p - 4
    Vec<T, 2> cv[2];              // POST, even p: this thread's coarse pairs of coarse row p / 2 + 1
};

// relax of my N cells of x parity o: rows ym / yp above and below (other colour), cen my row's other
// colour, ep / en the x-edge cells beyond my group; nby = y faces of the row (0 with CLZ).  ask: the cells'
// neighbour sums times 1/h^2, written (AIN = false) or, for a residual whose neighbours a half-sweep of the
// previous step saw (PRE's black cells, as k_zs's ZS_RASK), read instead of re-summing them
template <typename T, int N, bool CLZ, bool RES, bool AIN = false>
__device__ __forceinline__ void ys_cells(const Vec<T, N>& ym, const Vec<T, N>& cen, const Vec<T, N>& yp, T ep, T en,
                                         const Vec<T, N>& fv, const Vec<T, N>& uc, int o, int nby, int gm, int nx,
                                         bool xin, const Op<T, 2>& op, T (&out)[N], T (&ask)[N])
{
    if (!AIN) {
        ZsNb<T, N> nb;
        nb.yl = ym;
        nb.yr = yp;
        nb.ep = ep;
        nb.en = en;
        T t[N];
        zs_xsum<T, N>(cen, nb, o, t);
#pragma unroll
        for (int e = 0; e < N; ++e) {
            t[e] = t[e] + ym.v[e];
            t[e] = t[e] + yp.v[e];
            ask[e] = t[e] * op.inv_hSq;
        }
    }
    // cl != 0: nby is the row's (uniform across the workgroup), so the row's two diagonals (off / on an x
    // face) are one uniform table walk and a cell selects between them: no divergent boundary path (a
    // segment at an x face would otherwise hold its whole workgroup at every step's barrier)
    T d0 = op.adiag, y0 = op.yadiag, d1 = op.adiag, y1 = op.yadiag;
    if (!CLZ) row_diag_fast(op, nby, d0, y0, d1, y1);
#pragma unroll
    for (int e = 0; e < N; ++e) {
        const int i = 2 * (gm + e) + o;
        const bool xf = !CLZ && (i == 0 || i == nx - 1);
        const T d = xf ? d1 : d0;
        if (RES) {
            const T a_u = ask[e] + d * uc.v[e];
            out[e] = fv.v[e] - a_u;
        } else {
            out[e] = div_rn(fv.v[e] - ask[e], d, xf ? y1 : y0);
        }
    }
    (void)xin;
}

// PRE: LINEAR selects the restriction (0: residual + 2x2 average here; 1: none, both colours stored)
template <typename T, bool PRE, int LINEAR, bool ERR, bool CLZ, int TXV>
__global__ __launch_bounds__((YsShape<T, PRE, TXV>::NTL)) void k_ys(const T* __restrict__ src, const T* __restrict__ f,
                                                               T* __restrict__ dst, const T* old, T* __restrict__ R,
                                                               const T* __restrict__ V, double* __restrict__ partials,
                                                               Geo g, Geo gc, Op<T, 2> op, T clc, int yc)
{
    using S = YsShape<T, PRE, TXV>;
    constexpr int N = S::N, H = S::H, G = S::G, TX = S::TX, NTL = S::NTL, ES = S::ES;
    constexpr bool RR = PRE && LINEAR == 0;
    using VT = Vec<T, N>;
    using PF = YsPrefetch<T>;
    __shared__ __align__(16) T lds[S::lds_floats];
    const int tid = threadIdx.x;
    const int tiles_x = g.nx / TX;
    const int b = xcd_remap(blockIdx.x, gridDim.x);
    const int X0 = (b % tiles_x) * TX, Y0 = (b / tiles_x) * yc;
    const int hw = g.hw, Hh = (int)g.H, ny = g.ny;
    const bool on = tid < G;
    const int gx = on ? tid : 0;
    const int gm = (X0 - S::HX) / 2 + gx * N;  // global packed m of my first cell
    const bool inx = on && gm >= 0 && gm < hw;
    const bool xin = !inx || (gm > 0 && 2 * (gm + N) < g.nx);  // no cell of the group on an x face
    const int cgm = gm < 0 ? 0 : (gm > hw - N ? hw - N : gm);
    const bool tile_x = on && gx >= S::HXG && gx < G - S::HXG;
    const int zlo = Y0 - H;
    const int p_end = Y0 + yc + (PRE ? 4 : 3);
    auto iny = [&](int q) { return q >= 0 && q < ny; };
    auto rcl = [&](int q) { return q < 0 ? 0 : (q >= ny ? ny - 1 : q); };
    auto nby = [&](int q) { return CLZ ? 0 : (q == 0) + (q == ny - 1); };
    for (int i = tid; i < (int)S::lds_floats; i += NTL) lds[i] = (T)0;
    __syncthreads();
    // edge slot of stage base `off` with `ns` rows, row q
    auto eslot = [&](int off, int ns, int q) { return lds + off + (q & (ns - 1)) * ES; };
    auto put = [&](T* sl, const VT& v) {
        if (inx) {
            sl[2 * gx] = v.v[0];
            sl[2 * gx + 1] = v.v[N - 1];
        }
    };
    auto edges = [&](const T* sl, T& ep, T& en) {  // left group's last cell, right group's first
        ep = gx > 0 ? sl[2 * gx - 1] : (T)0;
        en = gx < G - 1 ? sl[2 * gx + 2] : (T)0;
    };
    // ---- POST: coarse staging ring, row J in slot J & 3 (rows clamped to the box) ----
    const int Ia = X0 / 2 - 8;
    auto cjl = [&](int J) { return J < 0 ? 0 : (J >= gc.ny ? gc.ny - 1 : J); };
    auto cslot = [&](int J) { return lds + S::OFFC + (J & 3) * S::CI; };
    auto cload = [&](PF& r, int J) {
        J = cjl(J);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int t = tid + i * NTL;
            const int I = Ia + 2 * t;
            r.cv[i].v[0] = r.cv[i].v[1] = (T)0;
            if (t < S::CPAIRS && I >= 0 && I < gc.nx) {  // I even: cells I, I + 1 at m = I / 2 of the two halves
                const T* row = V + (int64_t)J * gc.hw + (I >> 1);
                const int ce = (I + J) & 1;
                r.cv[i].v[0] = row[ce * gc.H];
                r.cv[i].v[1] = row[(ce ^ 1) * gc.H];
            }
        }
    };
    auto cstore = [&](const PF& r, int J) {
        T* const sl = cslot(cjl(J));
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int t = tid + i * NTL;
            if (t < S::CPAIRS) vstore<T, 2>(sl + 2 * t, r.cv[i]);
        }
    };
    auto crow = [&](int J, T (&c)[N + 2]) {  // cells cgm - 1 .. cgm + N of coarse row J
        const T* const sl = cslot(cjl(J)) + (cgm - Ia);
        const Vec<T, N> mid = vload<T, N>(sl);
        c[0] = vload_lds_whole<T, N>(sl - N).v[N - 1];
#pragma unroll
        for (int e = 0; e < N; ++e) c[e + 1] = mid.v[e];
        c[N + 1] = vload_lds_whole<T, N>(sl + N).v[0];
    };
    auto prefetch = [&](PF& r, int p) {
        r.u = vload<T, N>(src + Hh + (int64_t)rcl(p) * hw + cgm);
        r.f1 = vload<T, N>(f + (int64_t)rcl(p - 1) * hw + cgm);
        r.f2 = vload<T, N>(f + Hh + (int64_t)rcl(p - 2) * hw + cgm);
        if (!PRE && ERR && tile_x) {
            const int64_t ro = (int64_t)rcl(p - 4) * hw + cgm;
            r.o0 = vload<T, N>(old + ro);
            r.o1 = vload<T, N>(old + Hh + ro);
        }
        // POST: fine row 2m + 1 is the first to need coarse row m + 1; it is loaded with the prefetch of row
        // 2m and put in the ring at the top of step 2m
        if (!PRE && (p & 1) == 0) cload(r, (p >> 1) + 1);
    };
    const VT vz = vzero<T, N>();
    VT W0[4], W1[4], W2[4], W3[4], W4[4], FR[4], FB[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) W0[i] = W1[i] = W2[i] = W3[i] = W4[i] = FR[i] = FB[i] = vz;
    T AS[2][N], askd[N];  // PRE: stage 4's askew of the last two steps (row p - 4 at slot RS & 1); scratch
#pragma unroll
    for (int e = 0; e < N; ++e) AS[0][e] = AS[1][e] = askd[e] = (T)0;
    T acc[N];
#pragma unroll
    for (int e = 0; e < N; ++e) acc[e] = (T)0;
    double err = 0.0, err1 = 0.0;

    PF pf[4];
    auto step = [&](auto rt, int p) {
        constexpr int RS = decltype(rt)::value;  // (p - zlo) & 3
        const PF& cur = pf[RS];
        auto sl = [](int k) constexpr { return (RS - k) & 3; };
        constexpr int PP = (H + RS) & 1;  // parity of p (Y0 even)
        auto par = [](int k) constexpr { return (PP + k) & 1; };  // parity of row p - k (mod 2)
        zs_hold<T, N>(cur.u);
        zs_hold<T, N>(cur.f1);
        zs_hold<T, N>(cur.f2);
        if (!PRE && ERR) {
            zs_hold<T, N>(cur.o0);
            zs_hold<T, N>(cur.o1);
        }
        if (!PRE && PP == 0) {
            zs_hold<T, 2>(cur.cv[0]);
            zs_hold<T, 2>(cur.cv[1]);
        }
        asm volatile("" ::: "memory");
        // POST: the coarse row this row's prefetch loaded (first read one step on; the slot it replaces was
        // last read three steps back)
        if (!PRE && PP == 0) cstore(cur, (p >> 1) + 1);
        if (p + YS_PF <= p_end) prefetch(pf[(RS + YS_PF) & 3], p + YS_PF);

        // ---- stage 0: black cells of row p (POST: + P V) ----
        VT a0 = cur.u;
        if (!iny(p) || !inx) {
            a0 = vz;
        } else if (!PRE) {
            PvRow<T, N, 2, LINEAR> pv;
            T c0[N + 2], c1[N + 2];
            const int J = p >> 1;
            crow(J, c0);
            if (LINEAR) crow((p & 1) ? J + 1 : J - 1, c1);  // Jn (clamped: PvRow's oy factor applies)
            pv.set_rows(gc, p, 0, cgm, c0, c1);
            const int ob = 1 ^ par(0);  // x parity of row p's black cells
#pragma unroll
            for (int e = 0; e < N; ++e) a0.v[e] = a0.v[e] + pv.value(e, ob, clc);
        }
        W0[sl(0)] = a0;
        // ---- stages 1..4: half-sweep k on row p - k (red, black, red, black) ----
        T ep, en;
        VT o1, o2, o3, o4;
        edges(eslot(0, 2, p - 1), ep, en);
        ys_cells<T, N, CLZ, false>(W0[sl(2)], W0[sl(1)], W0[sl(0)], ep, en, cur.f1, vz, par(1), nby(p - 1), gm, g.nx, xin,
                                   op, o1.v, askd);
        if (!iny(p - 1) || !inx) o1 = vz;
        W1[sl(1)] = o1;
        edges(eslot(S::OFF1, 2, p - 2), ep, en);
        ys_cells<T, N, CLZ, false>(W1[sl(3)], W1[sl(2)], W1[sl(1)], ep, en, cur.f2, vz, 1 ^ par(2), nby(p - 2), gm, g.nx,
                                   xin, op, o2.v, askd);
        if (!iny(p - 2) || !inx) o2 = vz;
        W2[sl(2)] = o2;
        edges(eslot(S::OFF2, 2, p - 3), ep, en);
        ys_cells<T, N, CLZ, false>(W2[sl(4)], W2[sl(3)], W2[sl(2)], ep, en, FR[sl(3)], vz, par(3), nby(p - 3), gm, g.nx,
                                   xin, op, o3.v, askd);
        if (!iny(p - 3) || !inx) o3 = vz;
        W3[sl(3)] = o3;
        edges(eslot(S::OFF3, 4, p - 4), ep, en);
        ys_cells<T, N, CLZ, false>(W3[sl(5)], W3[sl(4)], W3[sl(3)], ep, en, FB[sl(4)], vz, 1 ^ par(4), nby(p - 4), gm,
                                   g.nx, xin, op, o4.v, AS[RS & 1]);
        if (!iny(p - 4) || !inx) o4 = vz;
        W4[sl(4)] = o4;
        // ---- edge writes (slots no stage of this step reads) ----
        put(eslot(0, 2, p), a0);
        put(eslot(S::OFF1, 2, p - 1), o1);
        put(eslot(S::OFF2, 2, p - 2), o2);
        put(eslot(S::OFF3, 4, p - 3), o3);
        if (RR) put(eslot(S::OFF4, 2, p - 4), o4);
        // ---- the smoothed row p - 4: red final after stage 3, black after stage 4 ----
        {
            const int q = p - 4;
            if (q >= Y0 && q < Y0 + yc && tile_x) {
                if (!PRE && ERR) {
#pragma unroll
                    for (int e = 0; e < N; ++e) {
                        const double d0 = (double)W3[sl(4)].v[e] - (double)cur.o0.v[e];
                        const double d1 = (double)o4.v[e] - (double)cur.o1.v[e];
                        err = __builtin_fma(d0, d0, err);
                        err1 = __builtin_fma(d1, d1, err1);
                    }
                }
                T* dp = dst + (int64_t)q * hw + gm;
                if (!RR) vstore<T, N>(dp, W3[sl(4)]);  // PRE's red cells are read by no one (POST loads black)
                vstore<T, N>(dp + Hh, o4);
            }
        }
        // ---- PRE: residual of row p - 5 and the 2 x 2 restriction ----
        if (RR) {
            const int q = p - 5;
            T rred[N], rblk[N];
            T bep, ben, rep = (T)0, ren = (T)0;
            edges(eslot(S::OFF4, 2, q), bep, ben);  // black (stage 4) cells of row q
            ys_cells<T, N, CLZ, true>(W4[sl(6)], W4[sl(5)], W4[sl(4)], bep, ben, FR[sl(5)], W3[sl(5)], par(5), nby(q), gm,
                                      g.nx, xin, op, rred, askd);
            // the black cells' neighbours are the red cells the last step's stage 4 summed (its askew)
            if (kZsRask) {
                ys_cells<T, N, CLZ, true, true>(W3[sl(6)], W3[sl(5)], W3[sl(4)], rep, ren, FB[sl(5)], W4[sl(5)], 1 ^ par(5),
                                                nby(q), gm, g.nx, xin, op, rblk, AS[(RS & 1) ^ 1]);
            } else {
                edges(eslot(S::OFF3, 4, q), rep, ren);  // red (stage 3) cells of row q
                ys_cells<T, N, CLZ, true>(W3[sl(6)], W3[sl(5)], W3[sl(4)], rep, ren, FB[sl(5)], W4[sl(5)], 1 ^ par(5), nby(q),
                                          gm, g.nx, xin, op, rblk, askd);
            }
            if (q >= Y0 && q < Y0 + yc && tile_x) {
#pragma unroll
                for (int e = 0; e < N; ++e) {
                    const T r0 = par(5) == 0 ? rred[e] : rblk[e];  // x parity 0 (cell 2I) and 1 (2I + 1)
                    const T r1 = par(5) == 0 ? rblk[e] : rred[e];
                    if (par(5) == 0) {
                        acc[e] = r0 + r1;
                    } else {
                        acc[e] = acc[e] + r0;
                        acc[e] = acc[e] + r1;
                    }
                }
                if (par(5) == 1) {  // coarse row q >> 1 complete
                    const int J = q >> 1;
                    T* rowc = R + (int64_t)J * gc.hw;
#pragma unroll
                    for (int e = 0; e < N; ++e) {
                        const int I = gm + e;
                        rowc[((I + J) & 1) * gc.H + (I >> 1)] = (T)0.25 * acc[e];
                    }
                }
            }
        }
        FR[sl(1)] = cur.f1;
        FB[sl(2)] = cur.f2;
        lds_barrier();
    };

    const std::integral_constant<int, 0> R0;
    const std::integral_constant<int, 1> R1;
    const std::integral_constant<int, 2> R2;
    const std::integral_constant<int, 3> R3;
    if (!PRE) {  // the coarse rows the first fine row needs
        const int J = zlo >> 1;
        for (int k = J - 1; k <= J + 1; ++k) {
            cload(pf[0], k);
            cstore(pf[0], k);
        }
        __syncthreads();
    }
#pragma unroll
    for (int d = 0; d < YS_PF; ++d) prefetch(pf[d], zlo + d);
    for (int p = zlo; p <= p_end; p += 4) {
        step(R0, p);
        if (p + 1 <= p_end) step(R1, p + 1);
        if (p + 2 <= p_end) step(R2, p + 2);
        if (p + 3 <= p_end) step(R3, p + 3);
    }
    if (ERR) block_partial_t<NTL>(err + err1, partials);
}

// ---- coarse-level tail ----------------------------------------------------------------------
//
// The levels at and below ~16^3 cost one launch (3-5 us) per piece while their work is a few
// thousand cells.  k_tail runs the whole sub-cycle below level T — the ops of cycle_rec(T, ...)
// that the host recorded into TailSpec::ops — in ONE workgroup with every level resident in LDS
// (same packed layout, ghost planes zero), a __syncthreads() between dependent phases.  The
// per-cell arithmetic is the scalar kernels' (half_item / resrestrict_item / prolong_item), so
// results are bit-identical to the launch-per-piece path.

// 1024 threads = 16 waves on the CU; fp64 gets 512 so the kernel keeps 256 VGPRs without spills
template <typename T>
#ifndef TAIL_THREADS_F32
#define TAIL_THREADS_F32 1024
#endif
constexpr int tail_threads() { return sizeof(T) == 4 ? TAIL_THREADS_F32 : 512; }

template <typename T, int DIM>
struct TailArgs {
    int nlev, nops, jacobi, zero0;  // zero0: level 0's u is a fresh zero guess (not read)
    int fw;                          // full-weighting restriction (TAIL_RR)
    // bit l: the program reads level l's u / f before it writes them (copied in; the others start as 0), and writes
    // level l's f (copied out; u is always copied out)  (tail_io_masks)
    uint32_t in_u, in_f, out_f;
    int64_t off[kTailMaxLevels];     // element offset of the level's LDS region
    int64_t region[kTailMaxLevels];  // elements of one LDS array of the level (ghost planes included)
    T* u[kTailMaxLevels];            // global interior plane 0 of u / f
    T* f[kTailMaxLevels];
    Geo g[kTailMaxLevels];
    Op<T, DIM> op[kTailMaxLevels];
    uint32_t ops[kTailMaxOps];
};

template <typename T, int DIM, int LINEAR>
__global__ __launch_bounds__(tail_threads<T>()) void k_tail(const TailArgs<T, DIM> a)
{
    constexpr int kTailThreads = tail_threads<T>();
    extern __shared__ __align__(16) unsigned char tail_smem[];
    T* const lds = reinterpret_cast<T*>(tail_smem);
    constexpr int G = DIM == 3 ? kGhost3D : 0;
    const int tid = threadIdx.x;
    // level l: u at off, f at off + region, Jacobi target at off + 2 region
#ifndef TAIL_NOCOPYIN  // timing experiment only: results are wrong
    for (int l = 0; l < a.nlev; ++l) {
        const Geo& g = a.g[l];
        T* U = lds + a.off[l];
        T* F = U + a.region[l];
        const int64_t lo = G * g.P, n = g.nz * g.P;
        for (int64_t e = tid; e < a.region[l]; e += kTailThreads) {
            const int64_t ie = e - lo;
            const bool in = ie >= 0 && ie < n;
            U[e] = in && ((a.in_u >> l) & 1) ? a.u[l][ie] : (T)0;
            F[e] = in && ((a.in_f >> l) & 1) ? a.f[l][ie] : (T)0;
            if (a.jacobi) U[e + 2 * a.region[l]] = (T)0;
        }
    }
#endif
    __syncthreads();
#ifdef TAIL_PROF  // timing experiment: shader cycles per op into f of the first level (tools/tail_prof.py)
    __shared__ float tprof[128];
    __shared__ long long tlast;
#endif
    unsigned alt = 0;  // Jacobi: bit l = level l's iterate currently lives in its second array
    auto cur = [&](int l) { return lds + a.off[l] + G * a.g[l].P + (((alt >> l) & 1) ? 2 * a.region[l] : 0); };
    auto rhs = [&](int l) { return lds + a.off[l] + a.region[l] + G * a.g[l].P; };
#ifdef TAIL_NOOPS  // timing experiment only: results are wrong
    for (int pc = 0; pc < 0; ++pc) {
#else
    for (int pc = 0; pc < a.nops; ++pc) {
#endif
#ifdef TAIL_PROF
        if (tid == 0) {
            const long long now = (long long)__builtin_amdgcn_s_memtime();
            if (pc > 0 && pc <= 128) tprof[pc - 1] = (float)(now - tlast);
            tlast = now;
        }
#endif
        const uint32_t w = a.ops[pc];
        const int op = (int)(w & 15), l = (int)((w >> 4) & 15), arg = (int)(w >> 8);
        const Geo g = a.g[l];
        const int64_t half = g.H * g.nz;
        if (op == TAIL_SMOOTH) {
            for (int sw = 0; sw < arg; ++sw) {
                T* U = cur(l);
                const T* F = rhs(l);
                T v;
                if (a.jacobi) {  // both colours from the old iterate into the other array
                    T* D = lds + a.off[l] + G * g.P + (((alt >> l) & 1) ? 0 : 2 * a.region[l]);
                    for (int64_t it = tid; it < 2 * half; it += kTailThreads) {
                        const int c = it >= half;
                        half_item<T, DIM>(U, F, D, g, c, a.op[l], it - c * half, &v);
                    }
                    alt ^= 1u << l;
                    __syncthreads();
                } else {
                    for (int c = 0; c < 2; ++c) {
                        for (int64_t it = tid; it < half; it += kTailThreads) half_item<T, DIM>(U, F, U, g, c, a.op[l], it, &v);
                        __syncthreads();
                    }
                }
            }
        } else if (op == TAIL_RR) {
            const int64_t n = resrestrict_items<T, DIM>(g);
            if (a.fw) {  // full weighting: every fine residual evaluated where a coarse cell reads it
                const Geo gc = a.g[l + 1];
                const T* U = cur(l);
                const T* F = rhs(l);
                const T wf = (T)3 - a.op[l + 1].cl;
                auto get = [&](int i, int j, int64_t k) { return residual_at<T, DIM>(U, F, g, a.op[l], i, j, k); };
                for (int64_t it = tid; it < n; it += kTailThreads) {
                    const int cx = g.nx >> 1, cy = g.ny >> 1;
                    const int I = (int)(it % cx), J = (int)((it / cx) % cy);
                    const int64_t K = it / ((int64_t)cx * cy);
                    rhs(l + 1)[pidx(gc, I, J, K)] = fw_eval<T, DIM>(get, g, gc, wf, I, J, K);
                }
            } else {
                for (int64_t it = tid; it < n; it += kTailThreads)
                    resrestrict_item<T, DIM>(cur(l), rhs(l), rhs(l + 1), g, a.g[l + 1], a.op[l], it);
            }
            __syncthreads();
        } else if (op == TAIL_ZERO) {
            T* U = cur(l);
            for (int64_t e = tid; e < g.nz * g.P; e += kTailThreads) U[e] = (T)0;
            __syncthreads();
        } else if (op == TAIL_PROLONG) {
            for (int64_t it = tid; it < 2 * half; it += kTailThreads) {
                const int c = it >= half;
                prolong_item<T, DIM, LINEAR>(cur(l), cur(l + 1), g, a.g[l + 1], a.op[l + 1].cl, c, it - c * half);
            }
            __syncthreads();
        }
    }
#ifdef TAIL_PROF
    if (tid == 0) {
        const long long now = (long long)__builtin_amdgcn_s_memtime();
        if (a.nops <= 128) tprof[a.nops - 1] = (float)(now - tlast);
        for (int i = 0; i < 128 && i < a.nops; ++i) rhs(0)[i] = (T)tprof[i];
    }
    __syncthreads();
#endif
    for (int l = 0; l < a.nlev; ++l) {
        const T* U = cur(l);
        const T* F = rhs(l);
        const int64_t n = a.g[l].nz * a.g[l].P;
        const bool st_f = (a.out_f >> l) & 1;
        for (int64_t e = tid; e < n; e += kTailThreads) {
            a.u[l][e] = U[e];
            if (st_f) a.f[l][e] = F[e];
        }
    }
}

// ---- coarse tail with compile-time level shapes (k_tail_c) -------------------------------------
//
// The same op program as k_tail for a red/black tail whose first level has one of the compile-time shapes of
// TcTops below (the cubic / square tails of cubic / square boxes, and the tails of the slab-shaped boxes: one
// rank's slab of configs[3] / configs[4] ends in 32 x 32 x 4 -> 16 x 16 x 2 -> 8 x 8 x 1, the weak-scaling box
// 512 x 512 x 512 N in 8 x 8 x 8 N ... 1 x 1 x N).  Level l is (TX >> l, TY >> l, TZ >> l), down to the first
// level with an axis of one cell.  Each level lives in LDS as an unpacked (nx+2)(ny+2)(nz+2) array with a zero
// halo (the Dirichlet ghost), so a cell's neighbours are fixed offsets, every loop bound and index is a
// compile-time constant and no box test is needed.  The per-cell arithmetic is half_item's / residual_at +
// resrestrict_item's / prolong_value's, so results are bit-identical to k_tail and to the launch-per-piece path.
template <int DIM, int NX, int NY, int NZ>
struct TcLev {
    static constexpr int W = NX + 2, WY = NY + 2, WZ = NZ + 2, P = DIM == 3 ? W * WY * WZ : W * WY;
    static constexpr int CELLS = DIM == 3 ? NX * NY * NZ : NX * NY;
    static constexpr int SZ = W * WY;  // z stride
    static __device__ __forceinline__ int idx(int i, int j, int k)
    {
        return DIM == 3 ? ((k + 1) * WY + (j + 1)) * W + (i + 1) : (j + 1) * W + (i + 1);
    }
    static __device__ __forceinline__ int nb(int i, int j, int k)  // faces on the box boundary
    {
        return (i == 0) + (i == NX - 1) + (j == 0) + (j == NY - 1) + (DIM == 3 ? (k == 0) + (k == NZ - 1) : 0);
    }
};
template <int T0, int L>
constexpr int tc_dim_at() { return (T0 >> L) > 0 ? (T0 >> L) : 1; }
// level count of a top shape: the levels down to the first one with an axis of one cell
template <int DIM, int TX, int TY, int TZ>
constexpr int tc_levels()
{
    int m = TX < TY ? TX : TY;
    if (DIM == 3 && TZ < m) m = TZ;
    int n = 1;
    for (int t = m; t > 1; t >>= 1) ++n;
    return n;
}
template <int DIM, int TX, int TY, int TZ>
constexpr int tc_off(int l)  // element offset of level l's (u, f) pair
{
    int o = 0;
    for (int q = 0; q < l; ++q) {
        const int wx = (TX >> q > 0 ? TX >> q : 1) + 2, wy = (TY >> q > 0 ? TY >> q : 1) + 2,
                  wz = (TZ >> q > 0 ? TZ >> q : 1) + 2;
        o += 2 * (DIM == 3 ? wx * wy * wz : wx * wy);
    }
    return o;
}
// the full weighting's residual scratch (one array of the first level's layout after the levels): where the levels
// and it fit the LDS with 4 KB to spare for the static part (all fp32 shapes, fp64 16^3)
template <typename T, int DIM, int TX, int TY, int TZ>
constexpr bool tc_fw_scratch()
{
    const int p0 = DIM == 3 ? (TX + 2) * (TY + 2) * (TZ + 2) : (TX + 2) * (TY + 2);
    int n = 1, m = TX < TY ? TX : TY;
    if (DIM == 3 && TZ < m) m = TZ;
    for (int t = m; t > 1; t >>= 1) ++n;
    return (size_t)(tc_off<DIM, TX, TY, TZ>(n) + p0) * sizeof(T) + 4096 <= 160 * 1024;
}
// 16 waves in fp32; fp64 takes 8, so that the kernel keeps 256 VGPRs (at 16 waves it spilled 100-240 VGPRs)
#ifndef TC_THREADS_2D_F32  // (build knob: threads of the 2D fp32 tail)
#define TC_THREADS_2D_F32 1024
#endif
template <typename T, int DIM>
constexpr int tc_threads() { return sizeof(T) == 4 ? (DIM == 2 ? TC_THREADS_2D_F32 : 1024) : 512; }
#ifndef TC_MAXL  // timing experiment: skip the ops of levels >= TC_MAXL (wrong results)
#define TC_MAXL 16
#endif
// Levels of at most this many cells run on wave 0 alone, without workgroup barriers (build knob, 0: every level on the
// workgroup).  Measured slower (round 6, interleaved A/B): 3D 512 / 64 cells +6 / +3 us per 512^3 cycle, 2D 1024 cells
// +8 us, 256 cells neutral; a 16-wave barrier costs less than one wave walking a small level's cells alone.
#ifndef TC_WAVE_CELLS_3D
#define TC_WAVE_CELLS_3D 0
#endif
#ifndef TC_WAVE_CELLS_2D
#define TC_WAVE_CELLS_2D 0
#endif
template <int DIM, int NX, int NY, int NZ>
constexpr bool tc_wave_level()
{
    return TcLev<DIM, NX, NY, NZ>::CELLS <= (DIM == 3 ? TC_WAVE_CELLS_3D : TC_WAVE_CELLS_2D);
}
// The tail's phase boundary: a workgroup barrier, or on a level run by wave 0 alone its own ordering (the LDS accesses
// of one wave are performed in issue order; the wavefront-scope fences keep the compiler from moving them across)
template <bool WV>
__device__ __forceinline__ void tc_sync()
{
    if constexpr (WV) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
        __syncthreads();
    }
}

template <typename T, int DIM, int NX, int NY, int NZ, int NTH = tc_threads<T, DIM>()>
__device__ __forceinline__ void tc_half(T* U, const T* F, const Op<T, DIM>& op, int c, int tid)
{
    using L = TcLev<DIM, NX, NY, NZ>;
    if constexpr (NX >= 2) {
        constexpr int HN = NX / 2, CNT = L::CELLS / 2;
#pragma unroll
        for (int q0 = 0; q0 < CNT; q0 += NTH) {
            const int q = q0 + tid;
            if (q < CNT) {
                const int i2 = q % HN, j = (q / HN) % NY, k = DIM == 3 ? q / (HN * NY) : 0;
                const int i = 2 * i2 + ((j + k + c) & 1);
                const int x = L::idx(i, j, k);
                T sm = U[x - 1] + U[x + 1];
                sm = sm + U[x - L::W];
                sm = sm + U[x + L::W];
                if (DIM == 3) {
                    sm = sm + U[x - L::SZ];
                    sm = sm + U[x + L::SZ];
                }
                U[x] = op.relax_idx(sm, F[x], L::nb(i, j, k));
            }
        }
    } else {  // one cell per row: cell (0, j, k) has colour (j + k) & 1 (half_item's empty slot is skipped)
        constexpr int CNT = L::CELLS;
        for (int q = tid; q < CNT; q += NTH) {
            const int j = q % NY, k = DIM == 3 ? q / NY : 0;
            if (((j + k) & 1) != c) continue;
            const int x = L::idx(0, j, k);
            T sm = U[x - 1] + U[x + 1];
            sm = sm + U[x - L::W];
            sm = sm + U[x + L::W];
            if (DIM == 3) {
                sm = sm + U[x - L::SZ];
                sm = sm + U[x + L::SZ];
            }
            U[x] = op.relax_idx(sm, F[x], L::nb(0, j, k));
        }
    }
}

template <typename T, int DIM, int NX, int NY, int NZ>
__device__ __forceinline__ T tc_res(const T* U, const T* F, const Op<T, DIM>& op, int i, int j, int k)
{
    using L = TcLev<DIM, NX, NY, NZ>;
    const int x = L::idx(i, j, k);
    T sm = U[x - 1] + U[x + 1];
    sm = sm + U[x - L::W];
    sm = sm + U[x + L::W];
    if (DIM == 3) {
        sm = sm + U[x - L::SZ];
        sm = sm + U[x + L::SZ];
    }
    return op.residual_idx(sm, F[x], U[x], L::nb(i, j, k));
}

template <typename T, int DIM, int NX, int NY, int NZ, int NTH = tc_threads<T, DIM>()>
__device__ __forceinline__ void tc_rr(const T* U, const T* F, T* Fc, const Op<T, DIM>& op, int tid)
{
    constexpr int MX = NX / 2, MY = NY / 2, MZ = DIM == 3 ? NZ / 2 : 1;
    using C = TcLev<DIM, MX, MY, MZ>;
    constexpr int CNT = C::CELLS;
    auto res = [&](int i, int j, int k) { return tc_res<T, DIM, NX, NY, NZ>(U, F, op, i, j, k); };
    for (int q = tid; q < CNT; q += NTH) {
        const int I = q % MX, J = (q / MX) % MY, K = DIM == 3 ? q / (MX * MY) : 0;
        const int i = 2 * I, j = 2 * J, k = 2 * K;
        T sm = res(i, j, k) + res(i + 1, j, k);
        sm = sm + res(i, j + 1, k);
        sm = sm + res(i + 1, j + 1, k);
        if (DIM == 3) {
            sm = sm + res(i, j, k + 1);
            sm = sm + res(i + 1, j, k + 1);
            sm = sm + res(i, j + 1, k + 1);
            sm = sm + res(i + 1, j + 1, k + 1);
        }
        Fc[C::idx(I, J, K)] = (DIM == 3 ? (T)0.125 : (T)0.25) * sm;
    }
}

// tc_rr with the full-weighting restriction (fw_eval over the residuals of the 4^DIM fine cells)
template <typename T, int DIM, int NX, int NY, int NZ, int NTH = tc_threads<T, DIM>()>
__device__ __forceinline__ void tc_rr_fw(const T* U, const T* F, T* Fc, const Op<T, DIM>& op, T wf, int tid)
{
    constexpr int MX = NX / 2, MY = NY / 2, MZ = DIM == 3 ? NZ / 2 : 1;
    using C = TcLev<DIM, MX, MY, MZ>;
    constexpr int CNT = C::CELLS;
    Geo g{}, gc{};
    g.nx = NX;
    g.ny = NY;
    g.gnz = DIM == 3 ? NZ : 1;
    gc.nx = MX;
    gc.ny = MY;
    gc.gnz = MZ;
    auto res = [&](int i, int j, int64_t k64) { return tc_res<T, DIM, NX, NY, NZ>(U, F, op, i, j, (int)k64); };
    for (int q = tid; q < CNT; q += NTH) {
        const int I = q % MX, J = (q / MX) % MY, K = DIM == 3 ? q / (MX * MY) : 0;
        Fc[C::idx(I, J, K)] = fw_eval<T, DIM>(res, g, gc, wf, I, J, (int64_t)K);
    }
}

// tc_rr_fw through a residual scratch: r of every cell of the level into RS (the level's unpacked layout) once, then
// the full weighting of each coarse cell from RS (tc_rr_fw evaluates each fine residual for all 8 coarse cells that
// weight it: 64 residuals per coarse cell, the FW tail's extra 27 us per 512^3 cycle)
template <typename T, int DIM, int NX, int NY, int NZ, int NTH = tc_threads<T, DIM>()>
__device__ __forceinline__ void tc_rr_fw_s(const T* U, const T* F, T* Fc, const Op<T, DIM>& op, T wf, int tid, T* RS)
{
    using L = TcLev<DIM, NX, NY, NZ>;
    constexpr int MX = NX / 2, MY = NY / 2, MZ = DIM == 3 ? NZ / 2 : 1;
    using C = TcLev<DIM, MX, MY, MZ>;
    for (int q = tid; q < L::CELLS; q += NTH) {
        const int i = q % NX, j = (q / NX) % NY, k = DIM == 3 ? q / (NX * NY) : 0;
        RS[L::idx(i, j, k)] = tc_res<T, DIM, NX, NY, NZ>(U, F, op, i, j, k);
    }
    tc_sync<(NTH < tc_threads<T, DIM>())>();
    Geo g{}, gc{};
    g.nx = NX;
    g.ny = NY;
    g.gnz = DIM == 3 ? NZ : 1;
    gc.nx = MX;
    gc.ny = MY;
    gc.gnz = MZ;
    auto get = [&](int i, int j, int64_t k) { return RS[L::idx(i, j, (int)k)]; };
    for (int q = tid; q < C::CELLS; q += NTH) {
        const int I = q % MX, J = (q / MX) % MY, K = DIM == 3 ? q / (MX * MY) : 0;
        Fc[C::idx(I, J, K)] = fw_eval<T, DIM>(get, g, gc, wf, I, J, (int64_t)K);
    }
}

template <typename T, int DIM, int NX, int NY, int NZ, int LINEAR, int NTH = tc_threads<T, DIM>()>
__device__ __forceinline__ void tc_prolong(T* U, const T* V, T cl, int tid)
{
    using L = TcLev<DIM, NX, NY, NZ>;
    constexpr int MX = NX / 2, MY = NY / 2, MZ = DIM == 3 ? NZ / 2 : 1;
    using C = TcLev<DIM, MX, MY, MZ>;
    constexpr int CNT = L::CELLS;
#pragma unroll 1
    for (int q0 = 0; q0 < CNT; q0 += NTH) {
        const int q = q0 + tid;
        if (q < CNT) {
            const int i = q % NX, j = (q / NX) % NY, k = DIM == 3 ? q / (NX * NY) : 0;
            const int I = i >> 1, J = j >> 1, K = k >> 1;
            T v;
            if (!LINEAR) {
                v = V[C::idx(I, J, K)];
            } else {
                const T w0 = (T)0.75, w1 = (T)0.25;
                int In = (i & 1) ? I + 1 : I - 1, Jn = (j & 1) ? J + 1 : J - 1, Kn = (k & 1) ? K + 1 : K - 1;
                const bool ox = In < 0 || In >= MX, oy = Jn < 0 || Jn >= MY, oz = DIM == 3 && (Kn < 0 || Kn >= MZ);
                if (ox) In = I;
                if (oy) Jn = J;
                if (oz || DIM == 2) Kn = K;
                auto cv = [&](int a, int b, int d, bool fx, bool fy, bool fz) {  // cval()
                    T s = (T)1;
                    if (fx) s = -cl * s;
                    if (fy) s = -cl * s;
                    if (fz) s = -cl * s;
                    const T val = V[C::idx(a, b, d)];
                    return s == (T)1 ? val : s * val;
                };
                if (DIM == 2) {
                    const T a0 = w0 * cv(I, J, 0, false, false, false) + w1 * cv(In, J, 0, ox, false, false);
                    const T a1 = w0 * cv(I, Jn, 0, false, oy, false) + w1 * cv(In, Jn, 0, ox, oy, false);
                    v = w0 * a0 + w1 * a1;
                } else {
                    const T a00 = w0 * cv(I, J, K, false, false, false) + w1 * cv(In, J, K, ox, false, false);
                    const T a10 = w0 * cv(I, Jn, K, false, oy, false) + w1 * cv(In, Jn, K, ox, oy, false);
                    const T a01 = w0 * cv(I, J, Kn, false, false, oz) + w1 * cv(In, J, Kn, ox, false, oz);
                    const T a11 = w0 * cv(I, Jn, Kn, false, oy, oz) + w1 * cv(In, Jn, Kn, ox, oy, oz);
                    const T b0 = w0 * a00 + w1 * a10;
                    const T b1 = w0 * a01 + w1 * a11;
                    v = w0 * b0 + w1 * b1;
                }
            }
            const int x = L::idx(i, j, k);
            U[x] = U[x] + v;
        }
    }
}

// the packed global offset of LDS element q of a level (its (i, j, k), -1 in the halo)
template <int DIM, int NX, int NY, int NZ>
__device__ __forceinline__ int64_t tc_global(int q)
{
    using L = TcLev<DIM, NX, NY, NZ>;
    constexpr int HW = NX >= 2 ? NX / 2 : 1;
    constexpr int64_t H = (int64_t)HW * NY, P = 2 * H;
    const int i = q % L::W - 1, j = (q / L::W) % L::WY - 1, k = DIM == 3 ? q / (L::W * L::WY) - 1 : 0;
    const bool inside = q < L::P && i >= 0 && i < NX && j >= 0 && j < NY && k >= 0 && k < (DIM == 3 ? NZ : 1);
    return inside ? (int64_t)k * P + ((i + j + k) & 1) * H + (int64_t)j * HW + (i >> 1) : -1;
}

// level l of the tail: copy in (zero halo; a field the program writes before it reads it is not loaded: ld_u / ld_f
// false, zero) or out (f only where the program wrote it: st_f), packed global layout; a thread's loads are all issued
// before its LDS stores (compile-time trip count)
template <typename T, int DIM, int NX, int NY, int NZ>
__device__ __forceinline__ void tc_copy(T* U, T* F, T* gu, T* gf, bool in, bool ld_u, bool ld_f, bool st_f, int tid)
{
    using L = TcLev<DIM, NX, NY, NZ>;
    constexpr int IT = (L::P + tc_threads<T, DIM>() - 1) / tc_threads<T, DIM>();
    T uv[IT], fv[IT];
#pragma unroll
    for (int r = 0; r < IT; ++r) {
        const int q = tid + r * tc_threads<T, DIM>();
        const int64_t gi = tc_global<DIM, NX, NY, NZ>(q);
        if (in) {
            uv[r] = gi >= 0 && ld_u ? gu[gi] : (T)0;
            fv[r] = gi >= 0 && ld_f ? gf[gi] : (T)0;
        } else if (gi >= 0) {
            gu[gi] = U[q];
            if (st_f) gf[gi] = F[q];
        }
    }
    if (in) {
#pragma unroll
        for (int r = 0; r < IT; ++r) {
            const int q = tid + r * tc_threads<T, DIM>();
            if (q < L::P) {
                U[q] = uv[r];
                F[q] = fv[r];
            }
        }
    }
}

// Copy-in in two halves, so that every level's global loads are in flight together (round 4: tc_copy level by
// level waited for one level's loads before issuing the next level's: seven load latencies in a row in 2D)
template <typename T, int DIM, int NX, int NY, int NZ>
struct TcRegs {
    static constexpr int IT = (TcLev<DIM, NX, NY, NZ>::P + tc_threads<T, DIM>() - 1) / tc_threads<T, DIM>();
    T u[IT], f[IT];
};
template <typename T, int DIM, int NX, int NY, int NZ>
__device__ __forceinline__ void tc_load(TcRegs<T, DIM, NX, NY, NZ>& rg, const T* gu, const T* gf, bool ld_u, bool ld_f,
                                        int tid)
{
#pragma unroll
    for (int r = 0; r < TcRegs<T, DIM, NX, NY, NZ>::IT; ++r) {
        const int64_t gi = tc_global<DIM, NX, NY, NZ>(tid + r * tc_threads<T, DIM>());
        rg.u[r] = gi >= 0 && ld_u ? gu[gi] : (T)0;
        rg.f[r] = gi >= 0 && ld_f ? gf[gi] : (T)0;
    }
}
template <typename T, int DIM, int NX, int NY, int NZ>
__device__ __forceinline__ void tc_store(T* U, T* F, const TcRegs<T, DIM, NX, NY, NZ>& rg, int tid)
{
    using L = TcLev<DIM, NX, NY, NZ>;
#pragma unroll
    for (int r = 0; r < TcRegs<T, DIM, NX, NY, NZ>::IT; ++r) {
        const int q = tid + r * tc_threads<T, DIM>();
        if (q < L::P) {
            U[q] = rg.u[r];
            F[q] = rg.f[r];
        }
    }
}

template <typename T, int DIM, int LINEAR, int TX, int TY, int TZ>
__global__ __launch_bounds__((tc_threads<T, DIM>())) void k_tail_c(const TailArgs<T, DIM> a)
{
    constexpr int NL = tc_levels<DIM, TX, TY, TZ>();
    // the full weighting's residual scratch after the levels, where it fits (tc_lds_total)
    constexpr bool FWR = tc_fw_scratch<T, DIM, TX, TY, TZ>();
    constexpr int FWR_OFF = tc_off<DIM, TX, TY, TZ>(NL);
    extern __shared__ __align__(16) unsigned char tc_smem[];
    T* const lds = reinterpret_cast<T*>(tc_smem);
    // the level operators in LDS, read per op (held in registers for all levels they spill)
    __shared__ Op<T, DIM> sop[NL];
    if ((int)threadIdx.x < NL) sop[threadIdx.x] = a.op[threadIdx.x];
#define TC_NX(l) tc_dim_at<TX, (l)>()
#define TC_NY(l) tc_dim_at<TY, (l)>()
#define TC_NZ(l) (DIM == 3 ? tc_dim_at<TZ, (l)>() : 1)
#define TC_SH(l) TC_NX(l), TC_NY(l), TC_NZ(l)
#define TC_U(l) (lds + tc_off<DIM, TX, TY, TZ>(l))
#define TC_F(l) (lds + tc_off<DIM, TX, TY, TZ>(l) + TcLev<DIM, TC_SH(l)>::P)
#define TC_COPY(l, IN)                                                                                      \
    if constexpr ((l) < NL) tc_copy<T, DIM, TC_SH(l)>(TC_U(l), TC_F(l), a.u[l], a.f[l], IN, (a.in_u >> (l)) & 1,     \
                                                      (a.in_f >> (l)) & 1, (a.out_f >> (l)) & 1, threadIdx.x);
#define TC_LOAD(l)                                                                                          \
    TcRegs<T, DIM, TC_SH(l)> rg##l;                                                                         \
    if constexpr ((l) < NL) tc_load<T, DIM, TC_SH(l)>(rg##l, a.u[l], a.f[l], (a.in_u >> (l)) & 1, (a.in_f >> (l)) & 1, \
                                                      threadIdx.x);
#define TC_STORE(l) \
    if constexpr ((l) < NL) tc_store<T, DIM, TC_SH(l)>(TC_U(l), TC_F(l), rg##l, threadIdx.x);
    if constexpr (DIM == 2) {  // (3D: the held values push the kernel past 64 VGPRs into spills; level by level)
        TC_LOAD(0) TC_LOAD(1) TC_LOAD(2) TC_LOAD(3) TC_LOAD(4) TC_LOAD(5) TC_LOAD(6)
        TC_STORE(0) TC_STORE(1) TC_STORE(2) TC_STORE(3) TC_STORE(4) TC_STORE(5) TC_STORE(6)
    } else {
        TC_COPY(0, true) TC_COPY(1, true) TC_COPY(2, true) TC_COPY(3, true) TC_COPY(4, true) TC_COPY(5, true)
        TC_COPY(6, true)
    }
#undef TC_STORE
#undef TC_LOAD
    __syncthreads();
#ifdef TC_PROF  // timing experiment: wall-clock ticks (100 MHz) per op into f of the first level (tools/tail_prof.py)
    __shared__ long long tcp[130];
    if (threadIdx.x == 0) tcp[0] = wall_clock64();
#endif
    bool wave_prev = false;  // the last op ran on wave 0 alone (the same on every wave)
    for (int pc = 0; pc < a.nops; ++pc) {
        const uint32_t w = a.ops[pc];
        const int op = (int)(w & 15), l = (int)((w >> 4) & 15), arg = (int)(w >> 8);
        // an opaque copy of the thread index per op: the index arithmetic of every (level, op) would
        // otherwise be hoisted out of this loop and held in registers for the whole program
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
#define TC_CASE(L)                                                                                     \
    case L:                                                                                            \
        if constexpr ((L) < NL && (L) < TC_MAXL) {                                                     \
            using LV = TcLev<DIM, TC_SH(L)>;                                                           \
            /* a small level runs on wave 0 alone (the other waves skip to the next workgroup-wide op) */ \
            constexpr bool WV = tc_wave_level<DIM, TC_SH(L)>() && tc_threads<T, DIM>() > 64;          \
            constexpr int NTH = WV ? 64 : tc_threads<T, DIM>();                                        \
            if constexpr (WV) {                                                                        \
                wave_prev = true;                                                                      \
                if (tid >= 64) break;                                                                  \
            } else {                                                                                   \
                if (wave_prev) __syncthreads();                                                        \
                wave_prev = false;                                                                     \
            }                                                                                          \
            if (op == TAIL_SMOOTH) {                                                                   \
                for (int sw = 0; sw < arg; ++sw) {                                                     \
                    tc_half<T, DIM, TC_SH(L), NTH>(TC_U(L), TC_F(L), sop[L], 0, tid);                  \
                    tc_sync<WV>();                                                                     \
                    if (LV::CELLS >= 2) {                                                              \
                        tc_half<T, DIM, TC_SH(L), NTH>(TC_U(L), TC_F(L), sop[L], 1, tid);              \
                        tc_sync<WV>();                                                                 \
                    }                                                                                  \
                }                                                                                      \
            } else if (op == TAIL_ZERO) {                                                              \
                T* u = TC_U(L);                                                                        \
                constexpr int NXL = TC_NX(L), NYL = TC_NY(L);                                          \
                for (int q = tid; q < LV::CELLS; q += NTH)                                             \
                    u[LV::idx(q % NXL, (q / NXL) % NYL, DIM == 3 ? q / (NXL * NYL) : 0)] = (T)0;       \
                tc_sync<WV>();                                                                         \
            } else if constexpr ((L) + 1 < NL) {                                                       \
                if (op == TAIL_RR) {                                                                   \
                    if (a.fw) {                                                                        \
                        if constexpr (FWR)                                                             \
                            tc_rr_fw_s<T, DIM, TC_SH(L), NTH>(TC_U(L), TC_F(L), TC_F((L) + 1), sop[L],     \
                                                              (T)3 - sop[(L) + 1].cl, tid, lds + FWR_OFF); \
                        else                                                                           \
                            tc_rr_fw<T, DIM, TC_SH(L), NTH>(TC_U(L), TC_F(L), TC_F((L) + 1), sop[L],       \
                                                            (T)3 - sop[(L) + 1].cl, tid);                 \
                    } else                                                                             \
                        tc_rr<T, DIM, TC_SH(L), NTH>(TC_U(L), TC_F(L), TC_F((L) + 1), sop[L], tid);    \
                    /* a fresh guess of the next level (its ZERO op follows) in the same phase: RR writes */ \
                    /* that level's f, ZERO its u                                                        */ \
                    const uint32_t wn = pc + 1 < a.nops ? a.ops[pc + 1] : 0u;                          \
                    if ((int)(wn & 15) == TAIL_ZERO && (int)((wn >> 4) & 15) == (L) + 1) {              \
                        using CV = TcLev<DIM, TC_SH((L) + 1)>;                                         \
                        constexpr int MX = TC_NX((L) + 1), MY = TC_NY((L) + 1);                        \
                        T* uc = TC_U((L) + 1);                                                         \
                        for (int q = tid; q < CV::CELLS; q += NTH)                                     \
                            uc[CV::idx(q % MX, (q / MX) % MY, DIM == 3 ? q / (MX * MY) : 0)] = (T)0;   \
                        ++pc;                                                                          \
                    }                                                                                  \
                    tc_sync<WV>();                                                                     \
                } else if (op == TAIL_PROLONG) {                                                       \
                    tc_prolong<T, DIM, TC_SH(L), LINEAR, NTH>(TC_U(L), TC_U((L) + 1), sop[(L) + 1].cl, tid); \
                    tc_sync<WV>();                                                                     \
                }                                                                                      \
            }                                                                                          \
        }                                                                                              \
        break;
        switch (l) {
            TC_CASE(0)
            TC_CASE(1)
            TC_CASE(2)
            TC_CASE(3)
            TC_CASE(4)
            TC_CASE(5)
            TC_CASE(6)
            default: break;
        }
#undef TC_CASE
#ifdef TC_PROF
        __syncthreads();
        if (threadIdx.x == 0 && pc < 128) tcp[pc + 1] = wall_clock64();
#endif
    }
#ifdef TC_PROF
    if (threadIdx.x == 0) {
        // op q's ticks at cell (q % TX, q / TX, 0) of the first level's f, then 0; op code (op | level << 4) + 1
        // at the cell after the ticks' row block (rows 2 and 3)
        using L0 = TcLev<DIM, TC_SH(0)>;
        T* F0 = TC_F(0);
        const int n = a.nops < 2 * TX ? a.nops : 2 * TX;
        for (int q = 0; q < n; ++q) {
            F0[L0::idx(q % TX, q / TX, 0)] = (T)(tcp[q + 1] - tcp[q]);
            F0[L0::idx(q % TX, 2 + q / TX, 0)] = (T)((a.ops[q] & 255) + 1);
        }
        if (n < 2 * TX) {
            F0[L0::idx(n % TX, n / TX, 0)] = (T)0;
            F0[L0::idx(n % TX, 2 + n / TX, 0)] = (T)0;
        }
    }
    __syncthreads();
#endif
    if (wave_prev) __syncthreads();
    TC_COPY(0, false) TC_COPY(1, false) TC_COPY(2, false) TC_COPY(3, false) TC_COPY(4, false) TC_COPY(5, false)
    TC_COPY(6, false)
#undef TC_COPY
#undef TC_F
#undef TC_U
#undef TC_SH
#undef TC_NZ
#undef TC_NY
#undef TC_NX
}

template <int DIM, int TX, int TY, int TZ>
constexpr size_t tc_lds(int rb)
{
    return (size_t)tc_off<DIM, TX, TY, TZ>(tc_levels<DIM, TX, TY, TZ>()) * rb;
}
// the dynamic LDS of a launch: the levels, and the full weighting's scratch where it fits
template <typename T, int DIM, int TX, int TY, int TZ>
constexpr size_t tc_lds_total()
{
    return tc_lds<DIM, TX, TY, TZ>(sizeof(T)) +
           (tc_fw_scratch<T, DIM, TX, TY, TZ>() ? (size_t)TcLev<DIM, TX, TY, DIM == 3 ? TZ : 1>::P * sizeof(T) : 0);
}

// The compile-time tail shapes (first level nx x ny x nz; nz = 1 in 2D) and their kernels.  k_tail_c runs a
// tail whose first level is one of these (tail_shape); any other red/black tail runs the generic k_tail.
#define MGP_TC_SHAPES(X)   \
    X(3, 16, 16, 16)       \
    X(3, 32, 32, 4)        \
    X(3, 8, 8, 16)         \
    X(3, 8, 8, 32)         \
    X(3, 8, 8, 64)         \
    X(2, 64, 64, 1)

// ---- 3D-tiled smoothing phases of small levels (k_blk) ----------------------------------------
//
// Below ~128^3 a launch costs more than its work (≈5 us per kernel, most of it the kernel
// boundary), so a smoothing phase of nu RB-GS sweeps runs as ONE launch instead of 2 nu + 1:
//   PRE : nu sweeps of src, then residual + restriction   (smooth(l, nu1) + residual_restrict(l))
//   POST: src + P V, then nu sweeps                        (prolong_correct(l) + smooth(l, nu2))
// A workgroup owns a tx x ty x tz tile, loads it with a halo of E = 2 nu + 1 (PRE) / 2 nu (POST)
// cells (x halo rounded up to even so the LDS rows keep the global red/black packing) into LDS,
// and runs the half-sweeps there on a region that shrinks by one cell per half-sweep (the halo is
// recomputed redundantly by the neighbouring tiles with the same arithmetic), one barrier each.
// Only black cells of the input are read (Gauss-Seidel never reads the value it replaces: the red
// half-sweep overwrites the red ones); cells outside the box are 0 in LDS and never written.
// Every expression is half_item's / resrestrict_item's / prolong_value's, so the result is
// bit-identical to the launch-per-piece path and to the oracle.  src == nullptr: u = 0 (a fresh
// coarse guess, cpu.lua:138, without the memset).  src and dst are different buffers.

// 3D: 16 waves (the levels are small, so a workgroup is most of a CU); 2D tiles are 32 x 32
template <int DIM>
constexpr int blk_threads() { return DIM == 3 ? 1024 : 256; }

// Compile-time shape of a phase: owned B^DIM tile, halo E (y, z) and HX (x, even), NS sweeps.  FW (PRE):
// the full-weighting restriction reads the residuals of a one-cell ring around the tile, so the swept
// region ends one cell wider.
template <int DIM, bool PRE, int B, int NS, bool FW = false>
struct BlkShape {
    static constexpr int E = PRE ? 2 * NS + 1 + (FW ? 1 : 0) : 2 * NS;
    static constexpr int HX = (E + 1) & ~1;
    static constexpr int EX = B + 2 * HX, EY = B + 2 * E, EZ = DIM == 3 ? B + 2 * E : 1, EH = EX / 2;
    static constexpr int BZ = DIM == 3 ? B : 1;  // owned planes
    static constexpr int cells = EX * EY * EZ;
    static constexpr int owned = B * B * BZ;
    static constexpr int RB = FW ? B + 2 : B, RBZ = DIM == 3 ? RB : 1;  // residual region edge (PRE)
    static constexpr int rcells = RB * RB * RBZ;
    // POST: coarse cells x0/2 - 1 .. of the extended tile's parents and their neighbours
    static constexpr int CX = EX / 2 + 2, CY = EY / 2 + 3, CZ = DIM == 3 ? EZ / 2 + 3 : 1;
    static constexpr int ccells = CX * CY * CZ;
    static constexpr int lidx(int lz, int ly, int c, int mm) { return ((lz * EY + ly) * 2 + c) * EH + mm; }
};

// PRE: LINEAR selects the restriction (0: the 2^DIM average, 1: full weighting with face weight 3 - clc)
template <typename T, int DIM, bool PRE, int LINEAR, int B, int NS>
__global__ __launch_bounds__(blk_threads<DIM>()) void k_blk(const T* __restrict__ src, const T* __restrict__ f,
                                                            T* __restrict__ dst, T* __restrict__ R,
                                                            const T* __restrict__ V, Geo g, Geo gc, Op<T, DIM> op,
                                                            T clc)
{
    constexpr bool FW = PRE && LINEAR == 1;
    using S = BlkShape<DIM, PRE, B, NS, FW>;
    constexpr int E = S::E, HX = S::HX, EY = S::EY, EZ = S::EZ, EH = S::EH, BZ = S::BZ;
    constexpr int EZH = DIM == 3 ? E : 0;  // z halo
    constexpr int NT = blk_threads<DIM>();
    extern __shared__ __align__(16) unsigned char blk_smem[];
    T* const U = reinterpret_cast<T*>(blk_smem);
    T* const F = U + S::cells;
    T* const RS = F + S::cells;  // PRE: residuals of the owned cells (x fastest)
    T* const VC = F + S::cells;  // POST: the staged coarse region
    const int tid = threadIdx.x;
    __shared__ Op<T, DIM> sop;  // the operator in LDS: its diagonal table is indexed per cell
    if (tid == 0) sop = op;
    const int ntx = g.nx / B, nty = g.ny / B;
    const int b = blockIdx.x;
    const int X0 = (b % ntx) * B, Y0 = ((b / ntx) % nty) * B, Z0 = (b / (ntx * nty)) * BZ;
    const int xs = X0 - HX, ys = Y0 - E, zs = Z0 - EZH;  // global (local-plane) origin of the LDS box
    const int mxs = xs >> 1;                            // xs is even
    const int nzl = (int)g.nz, gnz = (int)g.gnz, gz0 = (int)g.z0;
    const int p0 = (ys + zs + gz0) & 1;                 // parity of LDS row (0, 0)
    auto faces = [&](int gi, int gj, int gk) {          // box faces of a cell (gk global)
        return (gi == 0) + (gi == g.nx - 1) + (gj == 0) + (gj == g.ny - 1) + (DIM == 3 ? (gk == 0) + (gk == gnz - 1) : 0);
    };

    // load: every LDS slot of both colours (u: black cells in the box, 0 elsewhere; f: cells in the
    // box), all of a thread's global loads in flight at once.  POST: the coarse region the tile's
    // prolongation reads is staged in LDS (VC, unpacked) with the same loads, and P V of the black
    // slots is evaluated from there (prolong_eval: prolong_value's arithmetic) after one barrier.
    {
        constexpr int n = EZ * EY * 2 * EH;
        constexpr int NB = (n + NT - 1) / NT;
        constexpr int CX = S::CX, CY = S::CY, NCB = (S::ccells + NT - 1) / NT;
        const int cx0 = (xs >> 1) - 1, cy0 = (ys >> 1) - 1, cz0 = DIM == 3 ? (zs >> 1) - 1 : 0;
        T uv[NB], fv[NB], cv[PRE ? 1 : NCB];
        if (!PRE) {
#pragma unroll
            for (int q = 0; q < NCB; ++q) {
                const int t = tid + q * NT;
                const int a = t % CX, bb = (t / CX) % CY, cc = t / (CX * CY);
                const int I = cx0 + a, J = cy0 + bb, K = cz0 + cc;
                const bool in = t < S::ccells && I >= 0 && I < gc.nx && J >= 0 && J < gc.ny && K >= 0 &&
                                (DIM == 2 || K < (int)gc.nz);
                cv[q] = in ? V[pidx(gc, I, J, (int64_t)K)] : (T)0;
            }
        }
#pragma unroll
        for (int q = 0; q < NB; ++q) {
            const int it = tid + q * NT;
            const int row = it / (2 * EH), rest = it % (2 * EH);
            const int lz = row / EY, ly = row % EY;
            const int c = rest >= EH, mm = rest - c * EH;
            const int gm = mxs + mm, gj = ys + ly, gk = zs + lz;
            const bool in = it < n && gm >= 0 && gm < g.hw && gj >= 0 && gj < g.ny && gk >= 0 && gk < nzl;
            const int64_t gi = (int64_t)gk * g.P + c * g.H + (int64_t)gj * g.hw + gm;
            fv[q] = in ? f[gi] : (T)0;
            uv[q] = in && c == 1 && src ? src[gi] : (T)0;
        }
        if (!PRE) {
#pragma unroll
            for (int q = 0; q < NCB; ++q) {
                const int t = tid + q * NT;
                if (t < S::ccells) VC[t] = cv[q];
            }
            __syncthreads();
            auto get = [&](int I, int J, int64_t K) { return VC[(((int)K - cz0) * CY + (J - cy0)) * CX + (I - cx0)]; };
#pragma unroll
            for (int q = 0; q < NB; ++q) {
                const int it = tid + q * NT;
                const int row = it / (2 * EH), rest = it % (2 * EH);
                const int lz = row / EY, ly = row % EY;
                const int c = rest >= EH, mm = rest - c * EH;
                const int gm = mxs + mm, gj = ys + ly, gk = zs + lz;
                const bool in = it < n && gm >= 0 && gm < g.hw && gj >= 0 && gj < g.ny && gk >= 0 && gk < nzl;
                if (in && c == 1) {
                    const int i = 2 * gm + (1 ^ ((ly + lz + p0) & 1));
                    uv[q] = uv[q] + prolong_eval<T, DIM, LINEAR>(get, gc, clc, i, gj, (int64_t)gk);
                }
            }
        }
#pragma unroll
        for (int q = 0; q < NB; ++q) {
            const int it = tid + q * NT;
            if (it < n) {
                U[it] = uv[q];
                F[it] = fv[q];
            }
        }
    }
    __syncthreads();

    // in-plane and z neighbour sum of LDS cell (lx, ly, lz) of colour c: half_item's order
    auto nbsum = [&](int lx, int ly, int lz, int c) {
        const int mm = lx >> 1, o = lx & 1;
        const int oth = S::lidx(lz, ly, c ^ 1, mm);
        T sum = U[oth - 1 + o] + U[oth + o];
        sum = sum + U[oth - 2 * EH];
        sum = sum + U[oth + 2 * EH];
        if (DIM == 3) {
            sum = sum + U[oth - 2 * EH * EY];
            sum = sum + U[oth + 2 * EH * EY];
        }
        return sum;
    };

    // half-sweeps: colour s & 1 (red first) on the tile extended by e = E - 1 - s cells (cells
    // outside the box are skipped: they stay 0)
#pragma unroll
    for (int s = 0; s < 2 * NS; ++s) {
        const int c = s & 1, e = E - 1 - s;
        const int xlo = HX - e, xhi = HX + B - 1 + e;
        const int mlo = xlo >> 1, nm = (xhi >> 1) - mlo + 1;
        const int ny = B + 2 * e, nz = DIM == 3 ? B + 2 * e : 1, n = nz * ny * nm;
        const int lz0 = DIM == 3 ? E - e : 0;
#pragma unroll
        for (int q = 0; q < (n + NT - 1) / NT; ++q) {
            const int it = tid + q * NT;
            const int row = it / nm, mm = mlo + it % nm;
            const int ly = E - e + row % ny, lz = lz0 + row / ny;
            const int o = c ^ ((ly + lz + p0) & 1);
            const int lx = 2 * mm + o;
            const int gi = xs + lx, gj = ys + ly, gkl = zs + lz;
            if (it < n && lx >= xlo && lx <= xhi && gi >= 0 && gi < g.nx && gj >= 0 && gj < g.ny && gkl >= 0 &&
                gkl < nzl) {
                const T sum = nbsum(lx, ly, lz, c);
                const int own = S::lidx(lz, ly, c, mm);
                U[own] = sop.relax_idx(sum, F[own], faces(gi, gj, gz0 + gkl));
            }
        }
        __syncthreads();
    }

    if (FW) {
        // residual of the owned cells and a one-cell ring (0 outside the box) into RS ...
        constexpr int RB = S::RB;
#pragma unroll
        for (int q = 0; q < (S::rcells + NT - 1) / NT; ++q) {
            const int it = tid + q * NT;
            if (it < S::rcells) {
                const int x = it % RB - 1, y = (it / RB) % RB - 1, z = DIM == 3 ? it / (RB * RB) - 1 : 0;
                const int gi = X0 + x, gj = Y0 + y, gk = Z0 + z;  // gk local
                T v = (T)0;
                if (gi >= 0 && gi < g.nx && gj >= 0 && gj < g.ny && (DIM == 2 || (gk >= 0 && gk < nzl))) {
                    const int lx = HX + x, ly = E + y, lz = EZH + z;
                    const int c = (lx & 1) ^ ((ly + lz + p0) & 1);
                    const int own = S::lidx(lz, ly, c, lx >> 1);
                    v = sop.residual_idx(nbsum(lx, ly, lz, c), F[own], U[own], faces(gi, gj, gz0 + gk));
                }
                RS[it] = v;
            }
        }
        __syncthreads();
        // ... then one coarse cell per thread by full weighting (fw_eval's order)
        constexpr int C = B / 2, CZ = DIM == 3 ? C : 1;
        const T wf = (T)3 - clc;
        for (int it = tid; it < C * C * CZ; it += NT) {
            const int I = it % C, J = (it / C) % C, K = it / (C * C);
            const int gI = (X0 >> 1) + I, gJ = (Y0 >> 1) + J, gK = (Z0 >> 1) + K;
            // RS holds fine local cell x at x + 1: coarse I reads RS columns 2I .. 2I + 3
            auto get = [&](int i, int j, int64_t k) {
                return RS[((DIM == 3 ? (int)k - Z0 + 1 : 0) * RB + (j - Y0 + 1)) * RB + (i - X0 + 1)];
            };
            R[pidx(gc, gI, gJ, (int64_t)gK)] = fw_eval<T, DIM>(get, g, gc, wf, gI, gJ, (int64_t)gK);
        }
    } else if (PRE) {
        // residual of every owned cell into RS (residual_at's expressions) ...
#pragma unroll
        for (int q = 0; q < (S::owned + NT - 1) / NT; ++q) {
            const int it = tid + q * NT;
            if (it < S::owned) {
                const int x = it % B, y = (it / B) % B, z = it / (B * B);
                const int lx = HX + x, ly = E + y, lz = EZH + z;
                const int c = (lx & 1) ^ ((ly + lz + p0) & 1);
                const int own = S::lidx(lz, ly, c, lx >> 1);
                const T sum = nbsum(lx, ly, lz, c);
                RS[it] = sop.residual_idx(sum, F[own], U[own], faces(X0 + x, Y0 + y, gz0 + Z0 + z));
            }
        }
        __syncthreads();
        // ... then one coarse cell per thread, children summed in resrestrict_item's order
        constexpr int C = B / 2, CZ = DIM == 3 ? C : 1;
        for (int it = tid; it < C * C * CZ; it += NT) {
            const int I = it % C, J = (it / C) % C, K = it / (C * C);
            const int r0 = (2 * K * B + 2 * J) * B + 2 * I;
            T sm = RS[r0] + RS[r0 + 1];
            sm = sm + RS[r0 + B];
            sm = sm + RS[r0 + B + 1];
            if (DIM == 3) {
                sm = sm + RS[r0 + B * B];
                sm = sm + RS[r0 + B * B + 1];
                sm = sm + RS[r0 + B * B + B];
                sm = sm + RS[r0 + B * B + B + 1];
            }
            R[pidx(gc, (X0 >> 1) + I, (Y0 >> 1) + J, (int64_t)((Z0 >> 1) + K))] = (DIM == 3 ? (T)0.125 : (T)0.25) * sm;
        }
    }
    // the owned cells to dst: both colours after POST; only the black ones after PRE (its output is read
    // only by POST, which loads black cells and whose first red half-sweep replaces the red ones)
    {
        constexpr int NC = PRE ? 1 : 2;  // colours stored
        constexpr int H2 = B / 2, n = BZ * B * NC * H2;
#pragma unroll
        for (int q = 0; q < (n + NT - 1) / NT; ++q) {
            const int it = tid + q * NT;
            if (it < n) {
                const int mm = it % H2, c = PRE ? 1 : (it / H2) & 1, ly = (it / (NC * H2)) % B, lz = it / (NC * H2 * B);
                dst[(int64_t)(Z0 + lz) * g.P + c * g.H + (int64_t)(Y0 + ly) * g.hw + (X0 >> 1) + mm] =
                    U[S::lidx(lz + EZH, ly + E, c, (HX >> 1) + mm)];
            }
        }
    }
}

// ---- copy-bandwidth probe ("a measured copy-kernel peak is also reported") --------

// Narrow-lane copies (W = 8 or 4 bytes per lane, one pass, 4 elements per thread a workgroup apart): the
// FETCH_SIZE calibration of loads narrower than 16 bytes (tools/fetch_calib.py; mgp_copy_bandwidth runs
// them only under MGP_COPY_CALIB=1).
template <int W>
__global__ __launch_bounds__(kBlock) void k_copy_w(const void* __restrict__ src, void* __restrict__ dst, int64_t n)
{
    typedef float f2v __attribute__((ext_vector_type(2)));
    using E = typename std::conditional<W == 8, f2v, float>::type;
    const E* s = reinterpret_cast<const E*>(src);
    E* d = reinterpret_cast<E*>(dst);
    const int64_t base = (int64_t)blockIdx.x * (4 * kBlock) + threadIdx.x;
    E v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t i = base + k * kBlock;
        if (i < n) v[k] = s[i];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t i = base + k * kBlock;
        if (i < n) d[i] = v[k];
    }
}

// dst = src in 16-byte lanes.  kind 0: grid-stride, 4 independent loads in flight per thread per
// iteration; kind 1: one pass, each thread 4 vectors a workgroup apart; kind 2: kind 1 with non-temporal
// loads and stores.  The probe reports the fastest.
template <int KIND>
__global__ __launch_bounds__(kBlock) void k_copy16(const float4* __restrict__ src, float4* __restrict__ dst, int64_t n)
{
    if (KIND == 0) {
        const int64_t stride = (int64_t)gridDim.x * kBlock;
        int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
        for (; i + 3 * stride < n; i += 4 * stride) {
            const float4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
            dst[i] = a;
            dst[i + stride] = b;
            dst[i + 2 * stride] = c;
            dst[i + 3 * stride] = d;
        }
        for (; i < n; i += stride) dst[i] = src[i];
        return;
    }
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v* s4 = reinterpret_cast<const f4v*>(src);
    f4v* d4 = reinterpret_cast<f4v*>(dst);
    const int64_t base = (int64_t)blockIdx.x * (4 * kBlock) + threadIdx.x;
    f4v v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t i = base + k * kBlock;
        if (i < n) v[k] = KIND == 2 ? __builtin_nontemporal_load(s4 + i) : s4[i];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t i = base + k * kBlock;
        if (i < n) {
            if (KIND == 2) __builtin_nontemporal_store(v[k], d4 + i);
            else d4[i] = v[k];
        }
    }
}

// ---- reductions -----------------------------------------------------------------------------

// ROUND: each square is first stored into the real-typed errorBuf (cpu-raw.lua:96-100, 249-253)
template <typename T, bool ROUND = false>
__global__ __launch_bounds__(kBlock) void k_sqdiff_partial(const T* __restrict__ a, const T* __restrict__ b,
                                                           int64_t n, double* __restrict__ partials)
{
    double acc = 0.0;
    for (int64_t c = (int64_t)blockIdx.x * kBlock + threadIdx.x; c < n; c += (int64_t)gridDim.x * kBlock) {
        const double d = (double)a[c] - (double)b[c];
        acc += ROUND ? (double)(T)(d * d) : d * d;
    }
    block_partial<T>(acc, partials);
}

// calcRelErr + count + calcFrobErr of gpu.lua:173-200 / test-gpu-obj.lua:96-123, 216-247 in one
// pass: per workgroup sum |1 - psi/psiOld| (in real, as errorBuf holds it), the number of nonzero
// errorBuf entries and sum (psi - psiOld)^2, each into its own block of kSumBlocks partials.
template <typename T>
__global__ __launch_bounds__(kBlock) void k_metrics_partial(const T* __restrict__ psi, const T* __restrict__ old,
                                                            int64_t n, double* __restrict__ partials)
{
    double rel = 0.0, cnt = 0.0, sq = 0.0;
    for (int64_t c = (int64_t)blockIdx.x * kBlock + threadIdx.x; c < n; c += (int64_t)gridDim.x * kBlock) {
        const T p = psi[c], o = old[c];
        const T e = (o != (T)0 && o != p) ? (T)fabs(1.0 - (double)(p / o)) : (T)0;
        if (e != (T)0) {
            rel += (double)e;
            cnt += 1.0;
        }
        const double d = (double)p - (double)o;
        sq += d * d;
    }
    __shared__ double red[3][kBlock];
    red[0][threadIdx.x] = rel;
    red[1][threadIdx.x] = cnt;
    red[2][threadIdx.x] = sq;
    __syncthreads();
    for (int w = kBlock / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w)
            for (int q = 0; q < 3; ++q) red[q][threadIdx.x] += red[q][threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0)
        for (int q = 0; q < 3; ++q) partials[q * gridDim.x + blockIdx.x] = red[q][0];
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

// ctr != nullptr: the result goes to out[*ctr] and *ctr advances (a replayed graph fills consecutive
// err slots without a per-cycle copy)
__global__ __launch_bounds__(1024) void k_sum_n(const double* __restrict__ partials, int n, double* __restrict__ out,
                                                int* __restrict__ ctr = nullptr)
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
    if (threadIdx.x == 0) {
        if (ctr) {
            const int k = *ctr;
            out[k] = sh[0];
            *ctr = k + 1;
        } else {
            *out = sh[0];
        }
    }
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
    MGP_REAL(rb, (k_init<T><<<nblk_gs(n), kBlock, 0, s>>>((T*)u, (T*)f, g, cx, cy, cz, dim == 3)));
    return hipGetLastError();
}

hipError_t launch_pack(int rb, const void* lex, void* packed, Geo g, hipStream_t s)
{
    const int64_t n = g.P * g.nz;
    MGP_REAL(rb, (k_pack<T><<<nblk_gs(n), kBlock, 0, s>>>((const T*)lex, (T*)packed, g)));
    return hipGetLastError();
}

hipError_t launch_unpack(int rb, const void* packed, void* lex, Geo g, hipStream_t s)
{
    const int64_t n = g.P * g.nz;
    MGP_REAL(rb, (k_unpack<T><<<nblk_gs(n), kBlock, 0, s>>>((const T*)packed, (T*)lex, g)));
    return hipGetLastError();
}

// k_resnorm_z: 3D levels whose rows hold whole vectors and whose planes split into kResZ-plane chunks
static bool resnorm_z_ok(int rb, const Geo& g)
{
    const int n = 16 / rb;
    return g.nz % kResZ == 0 && g.hw >= n && g.hw % n == 0 && g.nx >= 2;
}

int resnorm_blocks(int rb, Geo g)
{
    if (rb == kRealF32D) return (int)nblk(g.P * g.nz);
    const int n = 16 / rb;
    if (resnorm_z_ok(rb, g)) return (int)nblk((int64_t)(g.hw / n) * g.ny * (g.nz / kResZ));
    return (g.hw >= n && g.nx >= 2) ? (int)nblk(2 * (g.H / n) * g.nz) : (int)nblk(g.P * g.nz);
}

template <typename T, int D>
static void resnorm_t(const void* u, const void* f, Geo g, double h, double cl, double* partials, double* out,
                      hipStream_t s)
{
    const Op<T, D> op = make_op<T, D>(h, cl);
    constexpr int n = VN<T>::n;
    const unsigned nb = (unsigned)resnorm_blocks(sizeof(T), g);
    const int fofs = (int)nb + sum_scratch((int)nb);
    if (D == 3 && resnorm_z_ok(sizeof(T), g)) {
        k_resnorm_z<T><<<nb, kBlock, 0, s>>>((const T*)u, (const T*)f, g, make_op<T, 3>(h, cl), partials, fofs);
    } else if (g.hw >= n && g.nx >= 2) {
        const int64_t items = (g.H / n) * g.nz;
        k_resnorm<T, D><<<nb, kBlock, 0, s>>>((const T*)u, (const T*)f, g, op, items, partials, fofs);
    } else {
        k_resnorm_s<T, D><<<nb, kBlock, 0, s>>>((const T*)u, (const T*)f, g, op, partials, fofs);
    }
    // the two rows of partials (sum r^2, sum f^2), each to one value in fixed order
    (void)launch_sum_partials(partials, (int)nb, out, s);
    (void)launch_sum_partials(partials + fofs, (int)nb, out + 1, s);
}

hipError_t launch_residual_norm(int rb, int dim, const void* u, const void* f, Geo g, double h, double cl,
                                double* partials, double* out, hipStream_t s)
{
    if (rb == kRealF32D) {  // the scalar form, r evaluated in double (resnorm_blocks(kRealF32D) counts it)
        const unsigned nb = (unsigned)resnorm_blocks(rb, g);
        const int fofs = (int)nb + sum_scratch((int)nb);
        if (dim == 3)
            k_resnorm_s<float, 3, double><<<nb, kBlock, 0, s>>>((const float*)u, (const float*)f, g,
                                                                make_op<double, 3>(h, cl), partials, fofs);
        else
            k_resnorm_s<float, 2, double><<<nb, kBlock, 0, s>>>((const float*)u, (const float*)f, g,
                                                                make_op<double, 2>(h, cl), partials, fofs);
        (void)launch_sum_partials(partials, (int)nb, out, s);
        (void)launch_sum_partials(partials + fofs, (int)nb, out + 1, s);
        return hipGetLastError();
    }
    if (rb == 8) {
        if (dim == 3) resnorm_t<double, 3>(u, f, g, h, cl, partials, out, s);
        else resnorm_t<double, 2>(u, f, g, h, cl, partials, out, s);
    } else {
        if (dim == 3) resnorm_t<float, 3>(u, f, g, h, cl, partials, out, s);
        else resnorm_t<float, 2>(u, f, g, h, cl, partials, out, s);
    }
    return hipGetLastError();
}

hipError_t launch_residual_field(int rb, int dim, const void* u, const void* f, void* r, Geo g, double h, double cl,
                                 hipStream_t s)
{
    const unsigned nb = nblk_gs(g.P * g.nz);
    if (rb == kRealF32D) {
        if (dim == 3) k_residual_field<float, 3, double><<<nb, kBlock, 0, s>>>((const float*)u, (const float*)f, (float*)r, g, make_op<double, 3>(h, cl));
        else k_residual_field<float, 2, double><<<nb, kBlock, 0, s>>>((const float*)u, (const float*)f, (float*)r, g, make_op<double, 2>(h, cl));
        return hipGetLastError();
    }
    if (rb == 8) {
        if (dim == 3) k_residual_field<double, 3><<<nb, kBlock, 0, s>>>((const double*)u, (const double*)f, (double*)r, g, make_op<double, 3>(h, cl));
        else k_residual_field<double, 2><<<nb, kBlock, 0, s>>>((const double*)u, (const double*)f, (double*)r, g, make_op<double, 2>(h, cl));
    } else {
        if (dim == 3) k_residual_field<float, 3><<<nb, kBlock, 0, s>>>((const float*)u, (const float*)f, (float*)r, g, make_op<float, 3>(h, cl));
        else k_residual_field<float, 2><<<nb, kBlock, 0, s>>>((const float*)u, (const float*)f, (float*)r, g, make_op<float, 2>(h, cl));
    }
    return hipGetLastError();
}

hipError_t launch_sqdiff_field(int rb, const void* a, const void* b, void* out, int64_t n, hipStream_t s)
{
    if (rb == kRealF32D) {
        k_sqdiff_field<float, double><<<nblk_gs(n), kBlock, 0, s>>>((const float*)a, (const float*)b, (float*)out, n);
        return hipGetLastError();
    }
    MGP_REAL(rb, (k_sqdiff_field<T><<<nblk_gs(n), kBlock, 0, s>>>((const T*)a, (const T*)b, (T*)out, n)));
    return hipGetLastError();
}

hipError_t launch_field_stats(int rb, const void* packed, Geo g, uint64_t* hpart, double* dpart, uint64_t* out_h,
                              double* out_d, hipStream_t s)
{
    const int nb = kSumBlocks;
    MGP_REAL(rb, (k_field_stats<T><<<nb, kBlock, 0, s>>>((const T*)packed, g, hpart, dpart)));
    k_field_stats_final<<<1, kBlock, 0, s>>>(hpart, dpart, nb, out_h, out_d);
    return hipGetLastError();
}

static bool half_vector(int rb, const Geo& g) { return g.hw >= 16 / rb && g.nx >= 2; }

static int64_t half_items(int rb, const Geo& g)
{
    const int n = 16 / rb;
    return half_vector(rb, g) ? (g.H / n) * g.nz : g.H * g.nz;
}

static bool half_gs(int rb, const Geo& g, bool gs)
{
    return gs && half_vector(rb, g) && half_items(rb, g) >= (int64_t)kGsBlocks * kBlock * 2;
}

int half_blocks(int rb, Geo g, bool gs)
{
    if (rb == kRealF32D) return (int)nblk(g.H * g.nz);  // scalar k_half_s
    return half_gs(rb, g, gs) ? kGsBlocks : (int)nblk(half_items(rb, g));
}

template <typename T, int D>
static void half_t(bool fine, bool err, bool vec, bool gs, unsigned nb, int color, const void* other, const void* f, void* dst,
                   const void* old, double* partials, Geo g, double h, double cl, hipStream_t s)
{
    const Op<T, D> op = make_op<T, D>(h, cl);
    const T* o_ = (const T*)other;
    const T* f_ = (const T*)f;
    T* d_ = (T*)dst;
    const T* w_ = (const T*)old;
    if (vec && gs && half_gs(sizeof(T), g, gs)) {
        const int64_t items = half_items(sizeof(T), g);
        if (fine) {
            if (err) k_half_gs<T, D, 1, true><<<nb, kBlock, 0, s>>>(o_, f_, d_, w_, partials, g, color, op, items);
            else k_half_gs<T, D, 1, false><<<nb, kBlock, 0, s>>>(o_, f_, d_, w_, partials, g, color, op, items);
        } else {
            if (err) k_half_gs<T, D, 0, true><<<nb, kBlock, 0, s>>>(o_, f_, d_, w_, partials, g, color, op, items);
            else k_half_gs<T, D, 0, false><<<nb, kBlock, 0, s>>>(o_, f_, d_, w_, partials, g, color, op, items);
        }
    } else if (vec) {
        static const bool nt = [] {
            const char* v = std::getenv("MGP_NT");
            return v && std::atoi(v) != 0;
        }();
        if (fine && nt) {
            if (err) k_half<T, D, 2, true><<<nb, kBlock, 0, s>>>(o_, f_, d_, w_, partials, g, color, op);
            else k_half<T, D, 2, false><<<nb, kBlock, 0, s>>>(o_, f_, d_, w_, partials, g, color, op);
        } else if (fine) {
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

// cpu-raw.lua's float arithmetic: a thread per slot, evaluated in double, stored as float
template <int D>
static void half_f32d(bool err, unsigned nb, int color, const void* other, const void* f, void* dst, const void* old,
                      double* partials, Geo g, double h, double cl, hipStream_t s)
{
    const Op<double, D> op = make_op<double, D>(h, cl);
    const float *o_ = (const float*)other, *f_ = (const float*)f, *w_ = (const float*)old;
    if (err) k_half_s<float, D, true, double><<<nb, kBlock, 0, s>>>(o_, f_, (float*)dst, w_, partials, g, color, op);
    else k_half_s<float, D, false, double><<<nb, kBlock, 0, s>>>(o_, f_, (float*)dst, w_, partials, g, color, op);
}

hipError_t launch_half_sweep(int rb, int dim, bool fine, int color, const void* other, const void* f, void* dst,
                             const void* old, double* partials, Geo g, double h, double cl, bool gs, hipStream_t s)
{
    const unsigned nb = (unsigned)half_blocks(rb, g, gs);
    if (rb == kRealF32D) {
        if (dim == 3) half_f32d<3>(old != nullptr, nb, color, other, f, dst, old, partials, g, h, cl, s);
        else half_f32d<2>(old != nullptr, nb, color, other, f, dst, old, partials, g, h, cl, s);
        return hipGetLastError();
    }
    const bool err = old != nullptr, vec = half_vector(rb, g);
    if (rb == 8) {
        if (dim == 3) half_t<double, 3>(fine, err, vec, gs, nb, color, other, f, dst, old, partials, g, h, cl, s);
        else half_t<double, 2>(fine, err, vec, gs, nb, color, other, f, dst, old, partials, g, h, cl, s);
    } else {
        if (dim == 3) half_t<float, 3>(fine, err, vec, gs, nb, color, other, f, dst, old, partials, g, h, cl, s);
        else half_t<float, 2>(fine, err, vec, gs, nb, color, other, f, dst, old, partials, g, h, cl, s);
    }
    return hipGetLastError();
}

template <typename T, int D>
static hipError_t fresh_t(const void* f, void* u, Geo g, double h, double cl, bool red, hipStream_t s)
{
    const int64_t items = half_items(sizeof(T), g);
    if (red) k_fresh<T, D, true><<<nblk(items), kBlock, 0, s>>>((const T*)f, (T*)u, g, make_op<T, D>(h, cl));
    else k_fresh<T, D, false><<<nblk(items), kBlock, 0, s>>>((const T*)f, (T*)u, g, make_op<T, D>(h, cl));
    return hipGetLastError();
}

bool fresh_supported(int rb, const Geo& g) { return half_vector(rb, g); }

template <typename T, int D>
static hipError_t post1_t(int linear, void* u, const void* V, const void* f, Geo g, Geo gc, double h, double cl,
                          double clc, hipStream_t s)
{
    const int64_t items = half_items(sizeof(T), g);
    const Op<T, D> op = make_op<T, D>(h, cl);
    if (linear) k_post1<T, D, 1><<<nblk(items), kBlock, 0, s>>>((T*)u, (const T*)V, (const T*)f, g, gc, op, (T)clc);
    else k_post1<T, D, 0><<<nblk(items), kBlock, 0, s>>>((T*)u, (const T*)V, (const T*)f, g, gc, op, (T)clc);
    return hipGetLastError();
}

// the red cells of a row segment and their black neighbours' coarse rows come in whole vectors
bool post1_supported(int rb, const Geo& g, const Geo& gc)
{
    const int n = 16 / rb;
    return half_vector(rb, g) && gc.nx >= n && 2 * gc.nx == g.nx && g.z0 == 0 && g.gnz == g.nz;
}

hipError_t launch_post_first(int rb, int dim, int linear, void* u, const void* V, const void* f, Geo g, Geo gc,
                             double h, double cl, double clc, hipStream_t s)
{
    if (!post1_supported(rb, g, gc)) return hipErrorInvalidValue;
    if (rb == 8)
        return dim == 3 ? post1_t<double, 3>(linear, u, V, f, g, gc, h, cl, clc, s)
                        : post1_t<double, 2>(linear, u, V, f, g, gc, h, cl, clc, s);
    return dim == 3 ? post1_t<float, 3>(linear, u, V, f, g, gc, h, cl, clc, s)
                    : post1_t<float, 2>(linear, u, V, f, g, gc, h, cl, clc, s);
}

hipError_t launch_fresh_sweep(int rb, int dim, const void* f, void* u, Geo g, double h, double cl, hipStream_t s,
                              bool store_red)
{
    if (!fresh_supported(rb, g)) return hipErrorInvalidValue;
    if (rb == 8)
        return dim == 3 ? fresh_t<double, 3>(f, u, g, h, cl, store_red, s) : fresh_t<double, 2>(f, u, g, h, cl, store_red, s);
    return dim == 3 ? fresh_t<float, 3>(f, u, g, h, cl, store_red, s) : fresh_t<float, 2>(f, u, g, h, cl, store_red, s);
}

template <typename T, int D>
static void rr_t(const void* u, const void* f, void* R, Geo g, Geo gc, double h, double cl, hipStream_t s)
{
    const Op<T, D> op = make_op<T, D>(h, cl);
    constexpr int n = VN<T>::n;
    const int cx = g.nx / 2;
    const int64_t ncz = D == 3 ? g.nz / 2 : 1;
    // below 2^22 coarse cells one thread per coarse cell (more parallelism, shorter per-thread
    // chains) beats n cells along x: 256^3 -> 128^3 and below, 1.609 -> 1.570 ms per 512^3 cycle
    static const int64_t scalar_below = [] {
        const char* v = std::getenv("MGP_RR_SCALAR_CELLS");
        return v ? std::atoll(v) : (int64_t)1 << 22;
    }();
    // from MGP_RR_PAIR_CELLS coarse cells up to scalar_below: two coarse cells per thread (default: 2D from 2^18,
    // the 2048^2 level of configs[1]: cycle 0.2655 -> 0.2604 ms; 3D off, neutral at 512^3)
    static const int64_t pair_env = [] {
        const char* v = std::getenv("MGP_RR_PAIR_CELLS");
        return v ? std::atoll(v) : (int64_t)-1;
    }();
    const int64_t pair_from = pair_env >= 0 ? pair_env : (D == 2 ? (int64_t)1 << 18 : INT64_MAX);
    const int64_t ccells = (int64_t)cx * (g.ny / 2) * ncz;
    if (cx >= n && ccells >= scalar_below) {
        const int64_t items = (int64_t)(cx / n) * (g.ny / 2) * ncz;
        k_resrestrict<T, D><<<nblk(items), kBlock, 0, s>>>((const T*)u, (const T*)f, (T*)R, g, gc, op);
    } else if (n > 2 && cx >= 2 && ccells >= pair_from) {
        const int64_t items = (int64_t)(cx / 2) * (g.ny / 2) * ncz;
        k_resrestrict<T, D, 2><<<nblk(items), kBlock, 0, s>>>((const T*)u, (const T*)f, (T*)R, g, gc, op);
    } else {
        const int64_t items = (int64_t)cx * (g.ny / 2) * ncz;
        k_resrestrict_s<T, D><<<nblk(items), kBlock, 0, s>>>((const T*)u, (const T*)f, (T*)R, g, gc, op);
    }
}

hipError_t launch_residual_restrict(int rb, int dim, const void* u, const void* f, void* R, Geo g, Geo gc, double h,
                                    double cl, hipStream_t s)
{
    if (rb == kRealF32D) {
        const int64_t items = (int64_t)(g.nx / 2) * (g.ny / 2) * (dim == 3 ? g.nz / 2 : 1);
        if (dim == 3)
            k_resrestrict_s<float, 3, double><<<nblk(items), kBlock, 0, s>>>((const float*)u, (const float*)f, (float*)R, g,
                                                                            gc, make_op<double, 3>(h, cl));
        else
            k_resrestrict_s<float, 2, double><<<nblk(items), kBlock, 0, s>>>((const float*)u, (const float*)f, (float*)R, g,
                                                                            gc, make_op<double, 2>(h, cl));
        return hipGetLastError();
    }
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
static void resfield_t(const void* u, const void* f, void* r, Geo g, double h, double cl, hipStream_t s)
{
    const Op<T, D> op = make_op<T, D>(h, cl);
    if (half_vector(sizeof(T), g)) {
        const int64_t items = half_items(sizeof(T), g);
        k_resfield_v<T, D><<<nblk(2 * items), kBlock, 0, s>>>((const T*)u, (const T*)f, (T*)r, g, op, items);
    } else {
        k_residual_field<T, D><<<nblk_gs(g.P * g.nz), kBlock, 0, s>>>((const T*)u, (const T*)f, (T*)r, g, op);
    }
}

hipError_t launch_residual_field_v(int rb, int dim, const void* u, const void* f, void* r, Geo g, double h, double cl,
                                   hipStream_t s)
{
    if (rb == kRealF32D) return launch_residual_field(rb, dim, u, f, r, g, h, cl, s);
    if (rb == 8) {
        if (dim == 3) resfield_t<double, 3>(u, f, r, g, h, cl, s);
        else resfield_t<double, 2>(u, f, r, g, h, cl, s);
    } else {
        if (dim == 3) resfield_t<float, 3>(u, f, r, g, h, cl, s);
        else resfield_t<float, 2>(u, f, r, g, h, cl, s);
    }
    return hipGetLastError();
}

template <typename T, int D>
static void fw_t(const void* r, void* R, Geo g, Geo gc, double clc, hipStream_t s)
{
    constexpr int n = VN<T>::n;
    const int cx = g.nx / 2;
    const int64_t ncz = D == 3 ? g.nz / 2 : 1;
    const T wf = (T)3 - (T)clc;
    if (cx >= n) {
        const int64_t items = (int64_t)(cx / n) * (g.ny / 2) * ncz;
        k_fw_v<T, D><<<nblk(items), kBlock, 0, s>>>((const T*)r, (T*)R, g, gc, wf);
    } else {
        const int64_t items = (int64_t)cx * (g.ny / 2) * ncz;
        k_fw_s<T, D><<<nblk(items), kBlock, 0, s>>>((const T*)r, (T*)R, g, gc, wf);
    }
}

hipError_t launch_fw_restrict(int rb, int dim, const void* r, void* R, Geo g, Geo gc, double clc, hipStream_t s)
{
    if (rb == kRealF32D) {
        const int64_t items = (int64_t)(g.nx / 2) * (g.ny / 2) * (dim == 3 ? g.nz / 2 : 1);
        const double wf = 3.0 - clc;
        if (dim == 3) k_fw_s<float, 3, double><<<nblk(items), kBlock, 0, s>>>((const float*)r, (float*)R, g, gc, wf);
        else k_fw_s<float, 2, double><<<nblk(items), kBlock, 0, s>>>((const float*)r, (float*)R, g, gc, wf);
        return hipGetLastError();
    }
    if (rb == 8) {
        if (dim == 3) fw_t<double, 3>(r, R, g, gc, clc, s);
        else fw_t<double, 2>(r, R, g, gc, clc, s);
    } else {
        if (dim == 3) fw_t<float, 3>(r, R, g, gc, clc, s);
        else fw_t<float, 2>(r, R, g, gc, clc, s);
    }
    return hipGetLastError();
}

template <typename T, int D>
static hipError_t pr_t(int linear, void* u, const void* V, Geo g, Geo gc, double clc, bool black, hipStream_t s)
{
    constexpr int n = VN<T>::n;
    if (gc.nx >= n) {
        const int64_t items = (int64_t)(gc.nx / n) * g.ny * g.nz;
        const unsigned nb = nblk(items);
        if (black) {
            if (linear) k_prolong_v<T, D, 1, true><<<nb, kBlock, 0, s>>>((T*)u, (const T*)V, g, gc, (T)clc);
            else k_prolong_v<T, D, 0, true><<<nb, kBlock, 0, s>>>((T*)u, (const T*)V, g, gc, (T)clc);
        } else {
            if (linear) k_prolong_v<T, D, 1><<<nb, kBlock, 0, s>>>((T*)u, (const T*)V, g, gc, (T)clc);
            else k_prolong_v<T, D, 0><<<nb, kBlock, 0, s>>>((T*)u, (const T*)V, g, gc, (T)clc);
        }
        return hipGetLastError();
    }
    for (int color = black ? 1 : 0; color < 2; ++color) {
        const unsigned nb = nblk(g.H * g.nz);
        if (linear) k_prolong<T, D, 1><<<nb, kBlock, 0, s>>>((T*)u, (const T*)V, g, gc, clc, color);
        else k_prolong<T, D, 0><<<nb, kBlock, 0, s>>>((T*)u, (const T*)V, g, gc, clc, color);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

template <int D>
static hipError_t pr_f32d(int linear, void* u, const void* V, Geo g, Geo gc, double clc, bool black, hipStream_t s)
{
    for (int color = black ? 1 : 0; color < 2; ++color) {
        const unsigned nb = nblk(g.H * g.nz);
        if (linear) k_prolong<float, D, 1, double><<<nb, kBlock, 0, s>>>((float*)u, (const float*)V, g, gc, clc, color);
        else k_prolong<float, D, 0, double><<<nb, kBlock, 0, s>>>((float*)u, (const float*)V, g, gc, clc, color);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_prolong_correct(int rb, int dim, int linear, void* u, const void* V, Geo g, Geo gc, double clc,
                                  hipStream_t s, bool black_only)
{
    if (rb == kRealF32D)
        return dim == 3 ? pr_f32d<3>(linear, u, V, g, gc, clc, black_only, s) : pr_f32d<2>(linear, u, V, g, gc, clc, black_only, s);
    if (rb == 8)
        return dim == 3 ? pr_t<double, 3>(linear, u, V, g, gc, clc, black_only, s)
                        : pr_t<double, 2>(linear, u, V, g, gc, clc, black_only, s);
    return dim == 3 ? pr_t<float, 3>(linear, u, V, g, gc, clc, black_only, s)
                    : pr_t<float, 2>(linear, u, V, g, gc, clc, black_only, s);
}

// ---- fused smoothing phases ----

static int parse_patch(const char* v, int dflt)
{
    int px = 0, py = 0;
    if (!v) return dflt;
    if (std::sscanf(v, "%d,%d", &px, &py) != 2 || px < 1 || py < 1 || px > 255 || py > 255) return 0;
    return px | (py << 8);
}

FusedTuning fused_tuning_from_env()
{
    FusedTuning t;
    if (const char* v = std::getenv("MGP_ZS_WIDE")) t.wide = std::atoi(v) != 0;
    if (const char* v = std::getenv("MGP_YS_HALF")) t.ys_half = std::atoi(v);
    if (const char* v = std::getenv("MGP_YS_ROWS")) {
        const int r = std::atoi(v);
        t.ys_rows = r >= 8 && (r & 1) == 0 ? r : 32;
    }
    if (const char* v = std::getenv("MGP_ZS_WGS")) t.wgs = std::max<int64_t>(1, std::atoll(v));
    const char* vb = std::getenv("MGP_ZS_PATCH");
    const int both = parse_patch(vb, 0);
    t.patch_pre = parse_patch(std::getenv("MGP_ZS_PATCH_PRE"), both);
    // POST's default: 4 x 8 patches on planes of >= 4096 tiles (auto, -1; round 5: the configs[4] slab's POST
    // 32.7 -> 30.8 ms per F-cycle, while on the configs[3] slab's 2048 tiles per plane it lost 3.50 -> 3.80 ms)
    t.patch_post = parse_patch(std::getenv("MGP_ZS_PATCH_POST"), vb ? both : -1);
    if (const char* v = std::getenv("MGP_ZS_FWF")) t.fwf = std::atoi(v) != 0;
    if (const char* v = std::getenv("MGP_ZS_POST_ZC")) t.post_zc = std::max(0, std::atoi(v));
    if (const char* v = std::getenv("MGP_STAMP_R")) t.stamp_r = std::atoi(v) != 0;
    return t;
}

// Tile order of a launch with more tiles than run at once (FusedTuning::patch_pre / patch_post): consecutive
// tiles of an XCD's band as px x py patches instead of whole tile rows, so that the y neighbours whose halo
// rows a tile reads stream through z at the same time.  Returns px | py << 8, or 0 (tile rows).
static int zs_patch(int patch, int tiles_x, int tiles_y, unsigned nb)
{
    if (patch == -1) patch = tiles_x * tiles_y >= 4096 ? 4 | (8 << 8) : 0;  // POST's default (FusedTuning)
    const int px = patch & 255, py = patch >> 8;
    if (!patch || tiles_x % px || tiles_y % py || nb <= 512) return 0;
    return patch;
}

static const char* tf(bool v) { return v ? "true" : "false"; }

template <typename T, bool PRE, int LINEAR, bool ERR, bool CLZ, bool WIDE = false>
static hipError_t zs_launch(const FusedArgs& a, hipStream_t s)
{
    using S = ZsShape<T, PRE, CLZ, WIDE, PRE && LINEAR == 2>;
    const Op<T, 3> op = make_op<T, 3>(a.h, a.cl);
    const unsigned nb = (unsigned)((a.g.nx / S::TX) * (a.g.ny / S::TY) * (a.g.nz / a.zc));
    if (a.info) {  // rocprofv3's spelling of the instantiation
        std::snprintf(a.info->name, sizeof a.info->name, "k_zs<%s, %s, %d, %s, %s, %s>", sizeof(T) == 4 ? "float" : "double",
                      tf(PRE), LINEAR, tf(ERR), tf(CLZ), tf(WIDE));
        a.info->grid = (int64_t)nb * S::NTL;
    }
    k_zs<T, PRE, LINEAR, ERR, CLZ, WIDE><<<nb, S::NTL, S::lds_bytes, s>>>((const T*)a.src, (const T*)a.f, (T*)a.dst,
                                                                           (const T*)(a.old ? a.old : a.dst), (T*)a.R,
                                                                           (const T*)a.V, a.partials, a.g, a.gc,
                                                                           op, (T)a.clc, a.zc, a.ghost,
                                                                           zs_patch(PRE ? a.tu.patch_pre : a.tu.patch_post,
                                                                                    a.g.nx / S::TX, a.g.ny / S::TY, nb));
    return hipGetLastError();
}

// POST's wide tile (ZsTile::TXPOST_W): fp32, cl = 0 (or any level with ZS_WIDE_CL: on the 256^3 level of the
// 512^3 box measured +10-16 us per cycle, off), a box it divides, FusedTuning::wide
#ifndef ZS_WIDE_CL
#define ZS_WIDE_CL 0
#endif
static bool zs_wide(int rb, const Geo& g, bool clz, const FusedTuning& tu)
{
    if (rb != 4 || (!clz && !ZS_WIDE_CL) || !tu.wide) return false;
    return g.nx % ZsTile<float>::TXPOST_W == 0 && g.ny % ZsTile<float>::TYPOST_W == 0;
}

static int ys_tx(int rb, const Geo& g, const FusedTuning& tu);

template <typename T, bool PRE, int LINEAR, bool ERR, bool CLZ, int TXV>
static hipError_t ys_launch_tx(const FusedArgs& a, hipStream_t s)
{
    using S = YsShape<T, PRE, TXV>;
    const Op<T, 2> op = make_op<T, 2>(a.h, a.cl);
    const unsigned nb = (unsigned)((a.g.nx / S::TX) * (a.g.ny / a.zc));
    if (a.info) {
        std::snprintf(a.info->name, sizeof a.info->name, "k_ys<%s, %s, %d, %s, %s, %d>", sizeof(T) == 4 ? "float" : "double",
                      tf(PRE), LINEAR, tf(ERR), tf(CLZ), TXV);
        a.info->grid = (int64_t)nb * S::NTL;
    }
    k_ys<T, PRE, LINEAR, ERR, CLZ, TXV><<<nb, S::NTL, 0, s>>>((const T*)a.src, (const T*)a.f, (T*)a.dst,
                                                         (const T*)(a.old ? a.old : a.dst), (T*)a.R, (const T*)a.V,
                                                         a.partials, a.g, a.gc, op, (T)a.clc, a.zc);
    return hipGetLastError();
}

template <typename T, bool PRE, int LINEAR, bool ERR, bool CLZ>
static hipError_t ys_launch(const FusedArgs& a, hipStream_t s)
{
    constexpr int F = ys_tx_full<T>();
    return ys_tx(sizeof(T), a.g, a.tu) == F ? ys_launch_tx<T, PRE, LINEAR, ERR, CLZ, F>(a, s)
                                      : ys_launch_tx<T, PRE, LINEAR, ERR, CLZ, F / 2>(a, s);
}

template <typename T, bool CLZ>
static hipError_t fused_dispatch_2d(const FusedArgs& a, hipStream_t s)
{
    const bool err = a.partials != nullptr;
    if (a.pre) return a.linear ? ys_launch<T, true, 1, false, CLZ>(a, s) : ys_launch<T, true, 0, false, CLZ>(a, s);
    if (a.linear) return err ? ys_launch<T, false, 1, true, CLZ>(a, s) : ys_launch<T, false, 1, false, CLZ>(a, s);
    return err ? ys_launch<T, false, 0, true, CLZ>(a, s) : ys_launch<T, false, 0, false, CLZ>(a, s);
}

template <typename T, bool CLZ>
static hipError_t fused_dispatch(const FusedArgs& a, hipStream_t s)
{
    const bool err = a.partials != nullptr;
#ifdef ZS_CL_AS_CLZ  // timing experiment only (wrong at the box faces): cl != 0 PRE runs the cl = 0 code
    if (a.pre) return a.linear ? zs_launch<T, true, 1, false, true>(a, s) : zs_launch<T, true, 0, false, true>(a, s);
#endif
    if constexpr (std::is_same<T, float>::value && CLZ) {  // the full weighting fused into PRE (fused_fwf_supported)
        if (a.pre && a.linear == 2)
            return a.src ? zs_launch<T, true, 2, false, CLZ>(a, s) : zs_launch<T, true, 2, true, CLZ>(a, s);
    }
    if (a.pre && a.linear == 2) return hipErrorInvalidValue;
    if (a.pre && !a.src)  // a fresh zero guess (ERR marks it in PRE)
        return a.linear ? zs_launch<T, true, 1, true, CLZ>(a, s) : zs_launch<T, true, 0, true, CLZ>(a, s);
    if (a.pre) return a.linear ? zs_launch<T, true, 1, false, CLZ>(a, s) : zs_launch<T, true, 0, false, CLZ>(a, s);
    if constexpr (std::is_same<T, float>::value && CLZ) {
        if (zs_wide(4, a.g, true, a.tu)) {
            if (a.linear)
                return err ? zs_launch<T, false, 1, true, CLZ, true>(a, s) : zs_launch<T, false, 1, false, CLZ, true>(a, s);
            return err ? zs_launch<T, false, 0, true, CLZ, true>(a, s) : zs_launch<T, false, 0, false, CLZ, true>(a, s);
        }
    }
    if constexpr (std::is_same<T, float>::value && !CLZ && ZS_WIDE_CL) {
        if (!err && zs_wide(4, a.g, false, a.tu))
            return a.linear ? zs_launch<T, false, 1, false, CLZ, true>(a, s) : zs_launch<T, false, 0, false, CLZ, true>(a, s);
    }
    if (a.linear) return err ? zs_launch<T, false, 1, true, CLZ>(a, s) : zs_launch<T, false, 1, false, CLZ>(a, s);
    return err ? zs_launch<T, false, 0, true, CLZ>(a, s) : zs_launch<T, false, 0, false, CLZ>(a, s);
}

// tile of a phase (pre) or the largest of all (pre < 0); clz: the level operator has no boundary modification;
// wide: POST's wide tile (zs_wide)
static void zs_tile(int rb, int& tx, int& ty, int pre = -1, bool clz = true, bool wide = false)
{
    const int xa = rb == 4 ? ZsTile<float>::TXPRE : ZsTile<double>::TXPRE;
    const int xc = rb == 4 ? ZsTile<float>::TXPRE_CL : ZsTile<double>::TXPRE_CL;
    const int xb = rb == 4 ? ZsTile<float>::TXPOST : ZsTile<double>::TXPOST;
    const int a = rb == 4 ? ZsTile<float>::TYPRE : ZsTile<double>::TYPRE;
    const int ac = rb == 4 ? ZsTile<float>::TYPRE_CL : ZsTile<double>::TYPRE_CL;
    const int b = rb == 4 ? ZsTile<float>::TYPOST : ZsTile<double>::TYPOST;
    const int xp = clz ? xa : xc, yp = clz ? a : ac;
    auto mx = [](int u, int v, int w) { return u > v ? (u > w ? u : w) : (v > w ? v : w); };
    tx = pre < 0 ? mx(xa, xb, xc) : (pre ? xp : xb);
    ty = pre < 0 ? mx(a, b, ac) : (pre ? yp : b);
    if (pre == 0 && wide) {
        tx = ZsTile<float>::TXPOST_W;
        ty = ZsTile<float>::TYPOST_W;
    }
}

// 2D (k_ys): rows per z-chunk of a workgroup (FusedTuning::ys_rows, default 32; even)
static int ys_rows(const Geo& g, const FusedTuning& tu)
{
    int r = tu.ys_rows;
    while (r > 8 && g.ny % r != 0) r /= 2;
    return r;
}

// segment width of a 2D level: the full width, or half of it when the full width gives fewer than
// FusedTuning::wgs (default 256) workgroups (FusedTuning::ys_half: -1 that rule, 0 never, 1 always)
static int ys_tx(int rb, const Geo& g, const FusedTuning& tu)
{
    const int mode = tu.ys_half;
    const int64_t target = tu.wgs;
    const int full = rb == 4 ? ys_tx_full<float>() : ys_tx_full<double>();
    if (mode == 0 || g.nx % (full / 2) != 0) return full;
    if (mode == 1 || g.nx % full != 0) return full / 2;
    return (int64_t)(g.nx / full) * (g.ny / ys_rows(g, tu)) < target ? full / 2 : full;
}

bool fused_supported(int rb, int dim, int ns, const Geo& g, const FusedTuning& tu)
{
    if (dim == 2)
        return ns == 2 && g.nz == 1 && g.nx % ys_tx(rb, g, tu) == 0 && g.ny >= 16 && g.ny % ys_rows(g, tu) == 0;
    if (dim != 3 || ns != 2) return false;
    int TX, TY;
    zs_tile(rb, TX, TY);
    return g.nx % TX == 0 && g.ny % TY == 0 && g.nz >= 16 && (g.nz & 1) == 0;
}

// planes per workgroup: halve the z-chunk until there are >= FusedTuning::wgs (default 256, one per CU)
// workgroups or a chunk would drop below 16 planes
int fused_zc(int rb, const Geo& g, bool pre, bool clz, const FusedTuning& tu)
{
    if (g.gnz == 1 && g.nz == 1) return ys_rows(g, tu);  // 2D: rows per chunk
    int TX, TY;
    zs_tile(rb, TX, TY, pre ? 1 : 0, clz, !pre && zs_wide(rb, g, clz, tu));
    const int64_t target = tu.wgs;
    const int64_t tiles = (int64_t)(g.nx / TX) * (g.ny / TY);
    int64_t chunks = 1;
    while (tiles * chunks < target && g.nz / (chunks * 2) >= 16) chunks *= 2;
    // POST: streams of at most tu.post_zc planes (planes of many tiles run as one chunk otherwise: the 4096^2 x 512
    // slab's POST 30.5 -> 28.5 ms per F-cycle with 256-plane chunks; the workgroups drift apart over long streams and
    // the y-neighbours' halo rows miss in L2)
    while (!pre && tu.post_zc > 0 && g.nz / chunks > tu.post_zc && g.nz / (chunks * 2) >= 16) chunks *= 2;
    return (int)(g.nz / chunks);
}

int fused_blocks(int rb, const Geo& g, int zc, bool clz, const FusedTuning& tu)  // POST's workgroups (err partials)
{
    if (g.gnz == 1 && g.nz == 1) return (g.nx / ys_tx(rb, g, tu)) * (g.ny / zc);
    int TX, TY;
    zs_tile(rb, TX, TY, 0, clz, zs_wide(rb, g, clz, tu));
    return (int)((int64_t)(g.nx / TX) * (g.ny / TY) * (g.nz / zc));
}

int fused_halo(bool pre) { return pre ? 5 : 4; }

bool fused_fwf_supported(int rb, int dim, bool clz, bool dist, const FusedTuning& tu)
{
    // fp32 levels without a boundary-modified operator (level 0), one rank's whole level: the fused PRE's trapezoid
    // is 6 deep with the full weighting, deeper than a slab's kZsHaloPre ghost planes; fp64 tiles would exceed the LDS;
    // 3D only (k_ys has no such variant)
    return rb == 4 && dim == 3 && clz && !dist && tu.fwf;
}

template <typename T, bool CLZ>
static hipError_t fused_attr()
{
    const int pre = (int)ZsShape<T, true, CLZ>::lds_bytes, post = (int)ZsShape<T, false, CLZ>::lds_bytes;
    const auto A = hipFuncAttributeMaxDynamicSharedMemorySize;
    if constexpr (std::is_same<T, float>::value && CLZ) {
        const int w = (int)ZsShape<T, true, CLZ, false, true>::lds_bytes;
        hipError_t e = hipFuncSetAttribute((const void*)k_zs<T, true, 2, false, CLZ>, A, w);
        if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_zs<T, true, 2, true, CLZ>, A, w);
        if (e != hipSuccess) return e;
    }
    if constexpr (std::is_same<T, float>::value && CLZ) {
        const int w = (int)ZsShape<T, false, CLZ, true>::lds_bytes;
        hipError_t e = hipFuncSetAttribute((const void*)k_zs<T, false, 0, false, CLZ, true>, A, w);
        if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_zs<T, false, 0, true, CLZ, true>, A, w);
        if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_zs<T, false, 1, false, CLZ, true>, A, w);
        if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_zs<T, false, 1, true, CLZ, true>, A, w);
        if (e != hipSuccess) return e;
    }
    if constexpr (std::is_same<T, float>::value && !CLZ && ZS_WIDE_CL) {
        const int w = (int)ZsShape<T, false, CLZ, true>::lds_bytes;
        hipError_t e = hipFuncSetAttribute((const void*)k_zs<T, false, 0, false, CLZ, true>, A, w);
        if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_zs<T, false, 1, false, CLZ, true>, A, w);
        if (e != hipSuccess) return e;
    }
    hipError_t e = hipFuncSetAttribute((const void*)k_zs<T, true, 0, false, CLZ>, A, pre);
    if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_zs<T, true, 1, false, CLZ>, A, pre);
    if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_zs<T, true, 0, true, CLZ>, A, pre);
    if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_zs<T, true, 1, true, CLZ>, A, pre);
    if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_zs<T, false, 0, false, CLZ>, A, post);
    if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_zs<T, false, 0, true, CLZ>, A, post);
    if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_zs<T, false, 1, false, CLZ>, A, post);
    if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_zs<T, false, 1, true, CLZ>, A, post);
    return e;
}

#ifdef TAIL_PROF
constexpr int kTailStaticLds = 1024;
#else
constexpr int kTailStaticLds = 0;
#endif
template <typename T>
static hipError_t tail_c_attr();

template <typename T, int D>
static hipError_t tail_attr()
{
    hipError_t e = hipFuncSetAttribute((const void*)k_tail<T, D, 0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)kTailMaxLds - kTailStaticLds);
    if (e == hipSuccess)
        e = hipFuncSetAttribute((const void*)k_tail<T, D, 1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)kTailMaxLds - kTailStaticLds);
    return e;
}

template <typename T>
static hipError_t blk_attr();

hipError_t prepare_kernels(int rb)
{
    hipError_t e = hipSuccess;
#define MGP_CHAIN(x) \
    if (e == hipSuccess) e = (x)
    if (rb == 4) {
        MGP_CHAIN((fused_attr<float, true>()));
        MGP_CHAIN((fused_attr<float, false>()));
        MGP_CHAIN((tail_attr<float, 2>()));
        MGP_CHAIN((tail_attr<float, 3>()));
        MGP_CHAIN((tail_c_attr<float>()));
        MGP_CHAIN((blk_attr<float>()));
        MGP_CHAIN((blk2_attr(4)));
    } else {
        MGP_CHAIN((fused_attr<double, true>()));
        MGP_CHAIN((fused_attr<double, false>()));
        MGP_CHAIN((tail_attr<double, 2>()));
        MGP_CHAIN((tail_attr<double, 3>()));
        MGP_CHAIN((tail_c_attr<double>()));
        MGP_CHAIN((blk_attr<double>()));
        MGP_CHAIN((blk2_attr(8)));
    }
#undef MGP_CHAIN
    return e;
}

hipError_t launch_fused(int rb, const FusedArgs& a, hipStream_t s)
{
    const bool clz = a.cl == 0.0;
    if (a.g.gnz == 1 && a.g.nz == 1) {  // 2D level: k_ys
        if (rb == 4) return clz ? fused_dispatch_2d<float, true>(a, s) : fused_dispatch_2d<float, false>(a, s);
        return clz ? fused_dispatch_2d<double, true>(a, s) : fused_dispatch_2d<double, false>(a, s);
    }
    if (rb == 4) return clz ? fused_dispatch<float, true>(a, s) : fused_dispatch<float, false>(a, s);
    return clz ? fused_dispatch<double, true>(a, s) : fused_dispatch<double, false>(a, s);
}

size_t tail_lds_bytes(int rb, int dim, int jacobi, const Geo* g, int nlev)
{
    const int G = dim == 3 ? kGhost3D : 0;
    size_t n = 0;
    for (int l = 0; l < nlev; ++l) n += (size_t)((g[l].nz + 2 * G) * g[l].P) * (jacobi ? 3 : 2);
    return n * (size_t)rb;
}

// k_tail_c applies: red/black, the first level one of MGP_TC_SHAPES and the levels below it the tail's levels
// (one rank's replicated box); returns the shape's index, or -1 (MGP_TAIL_CUBIC=0: always the generic k_tail)
static int tail_shape(const TailSpec& t, int dim)
{
    const char* v = std::getenv("MGP_TAIL_CUBIC");
    if ((v && std::atoi(v) == 0) || t.jacobi) return -1;
    int idx = -1, found = -1;
    auto match = [&](int D, int TX, int TY, int TZ, int NL) {
        ++idx;
        if (found >= 0 || D != dim || t.nlev != NL) return;
        for (int l = 0; l < t.nlev; ++l) {
            const Geo& g = t.g[l];
            const int nx = TX >> l > 0 ? TX >> l : 1, ny = TY >> l > 0 ? TY >> l : 1, nz = TZ >> l > 0 ? TZ >> l : 1;
            if (g.nx != nx || g.ny != ny || g.z0 != 0 || (dim == 3 && (g.nz != nz || g.gnz != nz))) return;
        }
        found = idx;
    };
#define X(D, TX, TY, TZ) match(D, TX, TY, TZ, tc_levels<D, TX, TY, TZ>());
    MGP_TC_SHAPES(X)
#undef X
    return found;
}

// Which fields a tail program reads before writing them (in_u / in_f, bit l = level l: only those are loaded into
// LDS) and which f it writes (out_f: only those are stored back; u is always stored).  A V- or F-cycle tail reads
// level 0's f (and its u unless it is a fresh guess); every level below gets its f from the restriction and, with
// fresh coarse guesses, its u from the zeroing before anything reads them.
static void tail_io_masks(const TailSpec& t, uint32_t& in_u, uint32_t& in_f, uint32_t& out_f)
{
    uint32_t wu = t.zero_first ? 1u : 0u, wf = 0;
    in_u = in_f = 0;
    auto rd = [&](int l) {
        if (!((wu >> l) & 1)) in_u |= 1u << l;
        if (!((wf >> l) & 1)) in_f |= 1u << l;
    };
    for (int i = 0; i < t.nops; ++i) {
        const uint32_t w = t.ops[i];
        const int op = (int)(w & 15), l = (int)((w >> 4) & 15);
        if (op == TAIL_SMOOTH) {
            rd(l);
        } else if (op == TAIL_RR) {
            rd(l);
            wf |= 1u << (l + 1);
        } else if (op == TAIL_ZERO) {
            wu |= 1u << l;
        } else if (op == TAIL_PROLONG) {
            if (!((wu >> (l + 1)) & 1)) in_u |= 1u << (l + 1);
            if (!((wu >> l) & 1)) in_u |= 1u << l;
        }
    }
    out_f = wf;
}

template <typename T, int D>
static hipError_t tail_t(const TailSpec& t, hipStream_t s)
{
    TailArgs<T, D> a{};
    a.nlev = t.nlev;
    a.nops = t.nops;
    a.jacobi = t.jacobi;
    a.zero0 = t.zero_first;
    a.fw = t.fw;
    tail_io_masks(t, a.in_u, a.in_f, a.out_f);
    const int G = D == 3 ? kGhost3D : 0;
    int64_t off = 0;
    for (int l = 0; l < t.nlev; ++l) {
        a.g[l] = t.g[l];
        a.u[l] = (T*)t.u[l];
        a.f[l] = (T*)t.f[l];
        a.op[l] = make_op<T, D>(t.h[l], t.cl[l]);
        a.region[l] = (t.g[l].nz + 2 * G) * t.g[l].P;
        a.off[l] = off;
        off += a.region[l] * (t.jacobi ? 3 : 2);
    }
    for (int i = 0; i < t.nops; ++i) a.ops[i] = t.ops[i];
    const int sh = tail_shape(t, D);
    if (sh >= 0) {
        int idx = -1;
        bool done = false;
#define X(DD, TX, TY, TZ)                                                                                    \
        if constexpr (DD == D) {                                                                             \
            if (++idx == sh && !done) {                                                                      \
                auto kc = t.linear ? k_tail_c<T, D, 1, TX, TY, TZ> : k_tail_c<T, D, 0, TX, TY, TZ>;          \
                kc<<<1, tc_threads<T, D>(), tc_lds_total<T, D, TX, TY, TZ>(), s>>>(a);                               \
                done = true;                                                                                 \
            }                                                                                                \
        } else {                                                                                             \
            ++idx;                                                                                           \
        }
        MGP_TC_SHAPES(X)
#undef X
        return done ? hipGetLastError() : hipErrorInvalidValue;
    }
    const size_t bytes = (size_t)off * sizeof(T);
    auto kern = t.linear ? k_tail<T, D, 1> : k_tail<T, D, 0>;
    kern<<<1, tail_threads<T>(), bytes, s>>>(a);
    return hipGetLastError();
}

template <typename T>
static hipError_t tail_c_attr()
{
    const auto A = hipFuncAttributeMaxDynamicSharedMemorySize;
    hipError_t e = hipSuccess;
#define X(D, TX, TY, TZ)                                                                                 \
    if (e == hipSuccess)                                                                                 \
        e = hipFuncSetAttribute((const void*)k_tail_c<T, D, 0, TX, TY, TZ>, A, (int)tc_lds_total<T, D, TX, TY, TZ>()); \
    if (e == hipSuccess)                                                                                 \
        e = hipFuncSetAttribute((const void*)k_tail_c<T, D, 1, TX, TY, TZ>, A, (int)tc_lds_total<T, D, TX, TY, TZ>());
    MGP_TC_SHAPES(X)
#undef X
    return e;
}

hipError_t launch_tail(int rb, int dim, const TailSpec& t, hipStream_t s)
{
    if (t.nlev < 1 || t.nlev > kTailMaxLevels || t.nops > kTailMaxOps) return hipErrorInvalidValue;
    if (rb == 8) return dim == 3 ? tail_t<double, 3>(t, s) : tail_t<double, 2>(t, s);
    return dim == 3 ? tail_t<float, 3>(t, s) : tail_t<float, 2>(t, s);
}

// ---- 3D-tiled phases of small levels ----

template <int DIM>
constexpr int blk_tile() { return DIM == 3 ? kBlkTile : kBlkTile2D; }

template <typename T, int DIM, bool PRE, int NS, bool FW = false>
constexpr size_t blk_lds()
{
    using S = BlkShape<DIM, PRE, blk_tile<DIM>(), NS, FW>;
    return (2 * (size_t)S::cells + (PRE ? (size_t)S::rcells : (size_t)S::ccells)) * sizeof(T);
}

// the owned tile edge B divides every axis of the level (3D: B^3 tiles, 2D: B^2)
bool block_supported(int rb, int dim, int ns, const Geo& g)
{
    if ((dim != 2 && dim != 3) || ns < 1 || ns > kBlkMaxSweeps) return false;
    const int B = dim == 3 ? kBlkTile : kBlkTile2D;
    if (g.nx < B || g.ny < B || (dim == 3 && g.nz < B) || g.z0 != 0 || g.gnz != g.nz) return false;
    const size_t lds = rb == 8 ? (dim == 3 ? blk_lds<double, 3, true, kBlkMaxSweeps, true>() : blk_lds<double, 2, true, kBlkMaxSweeps, true>())
                               : (dim == 3 ? blk_lds<float, 3, true, kBlkMaxSweeps, true>() : blk_lds<float, 2, true, kBlkMaxSweeps, true>());
    return lds <= kTailMaxLds;
}

template <typename T, int D, int NS>
static hipError_t blk_attr_ns()
{
    constexpr int B = blk_tile<D>();
    const auto A = hipFuncAttributeMaxDynamicSharedMemorySize;
    const int pre = (int)blk_lds<T, D, true, NS>(), post = (int)blk_lds<T, D, false, NS>();
    const int pre_fw = (int)blk_lds<T, D, true, NS, true>();
    hipError_t e = hipFuncSetAttribute((const void*)k_blk<T, D, true, 0, B, NS>, A, pre);
    if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_blk<T, D, true, 1, B, NS>, A, pre_fw);
    if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_blk<T, D, false, 0, B, NS>, A, post);
    if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_blk<T, D, false, 1, B, NS>, A, post);
    return e;
}

template <typename T>
static hipError_t blk_attr()
{
    hipError_t e = blk_attr_ns<T, 3, 1>();
    if (e == hipSuccess) e = blk_attr_ns<T, 3, 2>();
    if (e == hipSuccess) e = blk_attr_ns<T, 2, 1>();
    if (e == hipSuccess) e = blk_attr_ns<T, 2, 2>();
    return e;
}

template <typename T, int D, int NS>
static hipError_t blk_t(const BlockArgs& a, hipStream_t s)
{
    constexpr int B = blk_tile<D>();
    constexpr int NT = blk_threads<D>();
    const Op<T, D> op = make_op<T, D>(a.h, a.cl);
    const unsigned nb = (unsigned)((a.g.nx / B) * (a.g.ny / B) * (D == 3 ? a.g.nz / B : 1));
    const T* src = (const T*)a.src;
    if (a.pre && a.linear)  // PRE: linear = full-weighting restriction
        k_blk<T, D, true, 1, B, NS><<<nb, NT, blk_lds<T, D, true, NS, true>(), s>>>(
            src, (const T*)a.f, (T*)a.dst, (T*)a.R, (const T*)a.V, a.g, a.gc, op, (T)a.clc);
    else if (a.pre)
        k_blk<T, D, true, 0, B, NS><<<nb, NT, blk_lds<T, D, true, NS>(), s>>>(
            src, (const T*)a.f, (T*)a.dst, (T*)a.R, (const T*)a.V, a.g, a.gc, op, (T)a.clc);
    else if (a.linear)
        k_blk<T, D, false, 1, B, NS><<<nb, NT, blk_lds<T, D, false, NS>(), s>>>(
            src, (const T*)a.f, (T*)a.dst, (T*)a.R, (const T*)a.V, a.g, a.gc, op, (T)a.clc);
    else
        k_blk<T, D, false, 0, B, NS><<<nb, NT, blk_lds<T, D, false, NS>(), s>>>(
            src, (const T*)a.f, (T*)a.dst, (T*)a.R, (const T*)a.V, a.g, a.gc, op, (T)a.clc);
    return hipGetLastError();
}

hipError_t launch_block(int rb, int dim, const BlockArgs& a, hipStream_t s)
{
    if (!block_supported(rb, dim, a.ns, a.g)) return hipErrorInvalidValue;
    if (rb == 8) {
        if (dim == 3) return a.ns == 1 ? blk_t<double, 3, 1>(a, s) : blk_t<double, 3, 2>(a, s);
        return a.ns == 1 ? blk_t<double, 2, 1>(a, s) : blk_t<double, 2, 2>(a, s);
    }
    if (dim == 3) return a.ns == 1 ? blk_t<float, 3, 1>(a, s) : blk_t<float, 3, 2>(a, s);
    return a.ns == 1 ? blk_t<float, 2, 1>(a, s) : blk_t<float, 2, 2>(a, s);
}

hipError_t launch_copy16(int kind, const void* src, void* dst, int64_t bytes, hipStream_t s)
{
    const int64_t n = bytes / 16;
    const unsigned one_pass = (unsigned)((n + 4 * kBlock - 1) / (4 * kBlock));
    if (kind == 0) k_copy16<0><<<2048, kBlock, 0, s>>>((const float4*)src, (float4*)dst, n);
    else if (kind == 1) k_copy16<1><<<one_pass, kBlock, 0, s>>>((const float4*)src, (float4*)dst, n);
    else if (kind == 2) k_copy16<2><<<one_pass, kBlock, 0, s>>>((const float4*)src, (float4*)dst, n);
    else if (kind == 3) k_copy_w<8><<<one_pass * 2, kBlock, 0, s>>>(src, dst, n * 2);
    else k_copy_w<4><<<one_pass * 4, kBlock, 0, s>>>(src, dst, n * 4);
    return hipGetLastError();
}

hipError_t launch_sqdiff_sum(int rb, const void* a, const void* b, int64_t n, double* partials, double* out,
                             hipStream_t s, int* ctr)
{
    if (rb == kRealF32D)  // cpu-raw.lua's float errorBuf: each square rounded to float before the sum
        k_sqdiff_partial<float, true><<<kSumBlocks, kBlock, 0, s>>>((const float*)a, (const float*)b, n, partials);
    else MGP_REAL(rb, (k_sqdiff_partial<T><<<kSumBlocks, kBlock, 0, s>>>((const T*)a, (const T*)b, n, partials)));
    k_sum_n<<<1, 1024, 0, s>>>(partials, kSumBlocks, out, ctr);
    return hipGetLastError();
}

hipError_t launch_metrics(int rb, const void* psi, const void* old, int64_t n, double* partials, double* out,
                          hipStream_t s)
{
    MGP_REAL(rb, (k_metrics_partial<T><<<kSumBlocks, kBlock, 0, s>>>((const T*)psi, (const T*)old, n, partials)));
    for (int q = 0; q < 3; ++q) k_sum_n<<<1, 1024, 0, s>>>(partials + q * kSumBlocks, kSumBlocks, out + q);
    return hipGetLastError();
}

// The reference's debugging check (cpu-raw.lua:135-139, gpu.lua:279-283: error "found a nan" when a dumped grid
// holds a non-finite cell): any cell of p[0, n) with an all-ones exponent lowers *first to `id`, the check's
// position in the cycle, so the host names the first phase that produced one.  16-byte loads, grid-stride.
// ---- lexicographic Gauss-Seidel (cpu.lua:24-37, the reference's inPlaceIterativeSolver = GaussSeidel) ----
//
// cpu.lua's sweep updates u in place in ascending lexicographic order, so a cell reads the NEW values of its lower
// neighbours (i-1, j-1, k-1) and the OLD values of its upper ones.  The cells of one hyperplane i + j + k = s
// therefore depend only on hyperplane s - 1 (already new) and s + 1 (still old), and updating the hyperplanes in
// order s = 0, 1, ... reproduces the sequential sweep bit for bit (same operands, same expression).  Every cell
// of a hyperplane has the colour of s's parity, so the packed red/black layout is read as it is.
//
// Tiled wavefront: tiles of TX x TY x TZ cells run in tile-hyperplanes I + J + K = S, one launch per S (face-
// adjacent tiles differ by one in S, so no tile of a launch reads a face halo another tile of the launch writes).
// A workgroup holds its tile with a one-cell face halo in LDS (lower faces: final values of earlier launches;
// upper faces: old values; outside the box: 0, the reference's ghost), walks the tile's TX + TY + TZ - 2 cell
// hyperplanes with one barrier each, and writes the tile back.
template <int DIM>
constexpr int gsl_edge() { return DIM == 3 ? 8 : 32; }
template <int DIM>
constexpr int gsl_threads() { return DIM == 3 ? 512 : 1024; }

// C: the type the update is evaluated in (C = double with T = float: cpu-raw.lua's GaussSeidel under real = 'float',
// cpu-raw.lua:22-32: LuaJIT doubles over the float image, rounded once at the store)
template <typename T, int DIM, typename C = T>
__global__ __launch_bounds__(gsl_threads<DIM>()) void k_gslex(T* __restrict__ u, const T* __restrict__ f, Geo g,
                                                             Op<C, DIM> op, int S, int TX, int TY, int TZ)
{
    constexpr int E = gsl_edge<DIM>() + 2;
    __shared__ T s[DIM == 3 ? E * E * E : E * E];
    const int ntx = g.nx / TX;
    int I, J, K;  // this workgroup's tile on tile-hyperplane S (workgroup-uniform exit before any barrier)
    if (DIM == 3) {
        I = (int)blockIdx.x % ntx;
        J = (int)blockIdx.x / ntx;
        K = S - I - J;
        if (K < 0 || K >= (int)g.nz / TZ) return;
    } else {
        I = (int)blockIdx.x;
        J = S - I;
        K = 0;
        if (J < 0 || J >= g.ny / TY) return;
    }
    const int x0 = I * TX, y0 = J * TY, z0 = K * TZ;
    const int EZ = DIM == 3 ? TZ + 2 : 1;
    const int ncells = (TX + 2) * (TY + 2) * EZ;
    // tile + face halo (edges and corners are never read by the 5 / 7-point stencil: skipped)
    for (int q = (int)threadIdx.x; q < ncells; q += (int)blockDim.x) {
        const int lx = q % (TX + 2) - 1, ly = (q / (TX + 2)) % (TY + 2) - 1;
        const int lz = DIM == 3 ? q / ((TX + 2) * (TY + 2)) - 1 : 0;
        const int outs = (lx < 0 || lx >= TX) + (ly < 0 || ly >= TY) + (lz < 0 || lz >= TZ);
        if (outs > 1) continue;
        const int gi = x0 + lx, gj = y0 + ly, gk = z0 + lz;
        const bool in = gi >= 0 && gi < g.nx && gj >= 0 && gj < g.ny && gk >= 0 && gk < (int)g.nz;
        s[(lx + 1) + E * ((ly + 1) + E * (DIM == 3 ? lz + 1 : 0))] = in ? u[pidx(g, gi, gj, gk)] : (T)0;
    }
    const int t = (int)threadIdx.x;
    const bool mine = t < TX * TY * TZ;
    const int lx = t % TX, ly = (t / TX) % TY, lz = DIM == 3 ? t / (TX * TY) : 0;
    const int gi = x0 + lx, gj = y0 + ly, gk = z0 + lz;
    const int c = (lx + 1) + E * ((ly + 1) + E * (DIM == 3 ? lz + 1 : 0));
    T fc = (T)0;
    int nb = 0;
    if (mine) {
        fc = f[pidx(g, gi, gj, gk)];
        nb = (gi == 0) + (gi == g.nx - 1) + (gj == 0) + (gj == g.ny - 1);
        if (DIM == 3) nb += (gk == 0) + (gk == (int)g.nz - 1);
    }
    __syncthreads();
    const int last = (TX - 1) + (TY - 1) + (DIM == 3 ? TZ - 1 : 0);
    const int mys = lx + ly + lz;
    for (int st = 0; st <= last; ++st) {
        if (mine && mys == st) {
            C sum = (C)s[c - 1] + (C)s[c + 1];  // ((((xl + xr) + yl) + yr) + zl) + zr, cpu.lua:28-33
            sum = sum + (C)s[c - E];
            sum = sum + (C)s[c + E];
            if (DIM == 3) {
                sum = sum + (C)s[c - E * E];
                sum = sum + (C)s[c + E * E];
            }
            s[c] = (T)op.relax(sum, (C)fc, nb);
        }
        __syncthreads();
    }
    if (mine) u[pidx(g, gi, gj, gk)] = s[c];
}

template <typename T, int D, typename C = T>
static hipError_t gslex_t(void* u, const void* f, Geo g, double h, double cl, hipStream_t st)
{
    constexpr int B = gsl_edge<D>();
    const int TX = std::min(B, g.nx), TY = std::min(B, g.ny), TZ = D == 3 ? (int)std::min<int64_t>(B, g.nz) : 1;
    const int ntx = g.nx / TX, nty = g.ny / TY, ntz = D == 3 ? (int)(g.nz / TZ) : 1;
    const Op<C, D> op = make_op<C, D>(h, cl);
    const unsigned nb = (unsigned)(D == 3 ? ntx * nty : ntx);
    for (int S = 0; S < ntx + nty + ntz - 2; ++S) {
        k_gslex<T, D, C><<<nb, gsl_threads<D>(), 0, st>>>((T*)u, (const T*)f, g, op, S, TX, TY, TZ);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_gslex_sweep(int rb, int dim, void* u, const void* f, Geo g, double h, double cl, hipStream_t s)
{
    if (rb == kRealF32D)  // float image, double arithmetic (cpu-raw.lua:22-32 under real = 'float')
        return dim == 3 ? gslex_t<float, 3, double>(u, f, g, h, cl, s) : gslex_t<float, 2, double>(u, f, g, h, cl, s);
    if (rb != 4 && rb != 8) return hipErrorInvalidValue;
    if (dim == 3) return rb == 8 ? gslex_t<double, 3>(u, f, g, h, cl, s) : gslex_t<float, 3>(u, f, g, h, cl, s);
    return rb == 8 ? gslex_t<double, 2>(u, f, g, h, cl, s) : gslex_t<float, 2>(u, f, g, h, cl, s);
}

// ---- test hook of the communication deadline (mgp_api.cpp stream_wait; MGP_TEST_STALL) ----

// One wave polls a host-pinned flag with system-scope vector loads (never the scalar cache) and leaves when it is
// set or after max_ticks of the 100 MHz wall clock: a stream held like an exchange whose peer never arrives.
__global__ __launch_bounds__(64) void k_stall(const int* flag, uint64_t max_ticks)
{
    const uint64_t t0 = wall_clock64();
    const int* p = flag + (threadIdx.x >> 6);  // a per-lane (VGPR) address
    while (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0 && wall_clock64() - t0 < max_ticks)
        __builtin_amdgcn_s_sleep(127);
}

hipError_t launch_stall(const int* flag, double max_s, hipStream_t s)
{
    int khz = 0;  // wall clock rate in kHz (100 MHz on CDNA)
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
        khz <= 0)
        khz = 100000;
    const uint64_t ticks = (uint64_t)(std::min(max_s, 120.0) * 1e3 * khz);
    k_stall<<<1, 64, 0, s>>>(flag, ticks);
    return hipGetLastError();
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_nonfinite(const T* __restrict__ p, int64_t n, int id, int* first, bool vec)
{
    using U = typename std::conditional<sizeof(T) == 8, uint64_t, uint32_t>::type;
    constexpr U kExp = sizeof(T) == 8 ? (U)0x7ff0000000000000ull : (U)0x7f800000u;
    constexpr int V = 16 / sizeof(T);
    const int64_t nv = vec ? n / V : 0;  // (vec: p is 16-byte aligned)
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    bool bad = false;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nv; i += stride) {
        const uint4 q = reinterpret_cast<const uint4*>(p)[i];
        const U* w = reinterpret_cast<const U*>(&q);
#pragma unroll
        for (int k = 0; k < V; ++k) bad = bad || (w[k] & kExp) == kExp;
    }
    for (int64_t i = nv * V + (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        U w;
        __builtin_memcpy(&w, p + i, sizeof(U));
        bad = bad || (w & kExp) == kExp;
    }
    if (bad) atomicMin(first, id);
}

hipError_t launch_nonfinite_check(int rb, const void* p, int64_t n, int id, int* first, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    const int64_t want = (n / (16 / (rb == 8 ? 8 : 4)) + kBlock - 1) / kBlock;
    const unsigned nb = (unsigned)std::max<int64_t>(1, std::min<int64_t>(want, 2048));
    MGP_REAL(rb, (k_nonfinite<T><<<nb, kBlock, 0, s>>>((const T*)p, n, id, first, ((uintptr_t)p & 15) == 0)));
    return hipGetLastError();
}

// one fixed-order kernel up to 65536 partials (64 per thread), two levels beyond
int sum_scratch(int n) { return n <= 65536 ? 0 : (n + 8191) / 8192; }

hipError_t launch_sum_partials(const double* partials, int n, double* out, hipStream_t s, int* ctr)
{
    const int nb = sum_scratch(n);
    if (nb == 0) {
        k_sum_n<<<1, 1024, 0, s>>>(partials, n, out, ctr);
    } else {
        // two fixed-order levels; the first level's sums go right after the partials
        double* mid = const_cast<double*>(partials) + n;
        k_sum_chunks<<<nb, 1024, 0, s>>>(partials, n, 8192, mid);
        k_sum_n<<<1, 1024, 0, s>>>(mid, nb, out, ctr);
    }
    return hipGetLastError();
}

}  // namespace mgp
