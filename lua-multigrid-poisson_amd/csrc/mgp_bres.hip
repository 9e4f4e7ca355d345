// mgp_bres.hip — fused passes of the per-piece red/black levels below the finest (round 6).
//
// A red/black sweep's red half reads only black cells and its black half only red ones.  Two fusions follow:
//
//  k_bres    the pre-smoothing's last black half-sweep + calcResidual + reduceResidual (cpu.lua:40-54 update,
//            cpu.lua:108-135).  Nothing reads u's black cells before the black half replaces them, so a thread that
//            owns one coarse cell relaxes the 4 black children of its 2^3 block (stored in place), recomputes the 12
//            black cells just outside the block that neighbour its red children (their owners compute the same
//            values with the same expression), and restricts the 8 residuals in the reference order.  One pass over
//            red u and f replaces k_half (black) + k_resrestrict.
//  k_rbsweep one whole sweep, out of place: the block's red cells from src's black cells, then its black cells from
//            those and from the red cells just outside the block (recomputed), into dst != src (no thread reads what
//            another writes).  Only the last sweep of a run needs its red cells (a red half-sweep replaces red cells
//            unread), so the others store black only: 2 (2.5) reals per cell instead of 3.
//
// Every cell of a block sits at a compile-time offset (DX, DY, DZ) from the block origin (2I, 2J, 2K), whose colour
// parity is even on a replicated level (z0 = 0), so colours, packed addresses (a base per colour + constants) and the
// neighbour sources are all static; only the box-face tests are runtime (one flag per side).  Expressions and their
// order are k_half's / residual_at's / k_resrestrict's, so the results are bit-identical to the separate pieces.
#include "mgp_device.h"

#include <cstdlib>

namespace mgp {
namespace {

constexpr int fdiv2(int d) { return d >= 0 ? d / 2 : -((1 - d) / 2); }  // floor(d / 2)
constexpr int par(int d) { return ((d % 2) + 2) % 2; }

template <typename T, int DIM>
struct Blk {
    const Geo& g;
    const Op<T, DIM>& op;
    int i0, j0;
    int64_t k0;
    int64_t base[2];  // packed index of (i0, j0, k0)'s row segment in the red / black half (m = I)
    bool xlo, xhi, ylo, yhi, zlo, zhi;  // the neighbouring block exists on that side

    __device__ __forceinline__ Blk(const Geo& g_, const Op<T, DIM>& op_, int I, int J, int64_t K) : g(g_), op(op_)
    {
        i0 = 2 * I;
        j0 = 2 * J;
        k0 = DIM == 3 ? 2 * K : 0;
        const int64_t row = k0 * g.P + (int64_t)j0 * g.hw + I;
        base[0] = row;
        base[1] = row + g.H;
        xlo = I > 0;
        xhi = I < (g.nx >> 1) - 1;
        ylo = J > 0;
        yhi = J < (g.ny >> 1) - 1;
        zlo = DIM == 3 && K > 0;
        zhi = DIM == 3 && K < (g.nz >> 1) - 1;
    }
    template <int DX, int DY, int DZ>
    static constexpr bool black() { return par(DX + DY + DZ) == 1; }
    template <int DX, int DY, int DZ>
    static constexpr bool in_block() { return DX >= 0 && DX < 2 && DY >= 0 && DY < 2 && DZ >= 0 && DZ < (DIM == 3 ? 2 : 1); }
    template <int DX, int DY, int DZ>
    __device__ __forceinline__ bool inside() const
    {
        bool r = true;
        if constexpr (DX < 0) r = r && xlo;
        if constexpr (DX > 1) r = r && xhi;
        if constexpr (DY < 0) r = r && ylo;
        if constexpr (DY > 1) r = r && yhi;
        if constexpr (DIM == 3 && DZ < 0) r = r && zlo;
        if constexpr (DIM == 3 && DZ > 1) r = r && zhi;
        return r;
    }
    template <int DX, int DY, int DZ>
    __device__ __forceinline__ int64_t at() const
    {
        return base[black<DX, DY, DZ>() ? 1 : 0] + (int64_t)DZ * g.P + (int64_t)DY * g.hw + fdiv2(DX);
    }
    template <int DX, int DY, int DZ>
    __device__ __forceinline__ T ld(const T* p) const
    {
        return inside<DX, DY, DZ>() ? p[at<DX, DY, DZ>()] : (T)0;
    }
    // faces of the cell on the box boundary (Op::diag / relax / residual's nb)
    template <int DX, int DY, int DZ>
    __device__ __forceinline__ int nb() const
    {
        const int i = i0 + DX, j = j0 + DY;
        int n = (i == 0) + (i == g.nx - 1) + (j == 0) + (j == g.ny - 1);
        if constexpr (DIM == 3) {
            const int64_t k = g.z0 + k0 + DZ;
            n += (k == 0) + (k == g.gnz - 1);
        }
        return n;
    }
    // relax the cell (DX, DY, DZ) (inside the box) from the other colour's values nbr<dx, dy, dz>() in k_half's order
    template <int DX, int DY, int DZ, typename Nbr>
    __device__ __forceinline__ T relax(const Nbr& nbr, const T* f) const
    {
        T s = nbr.template get<DX - 1, DY, DZ>() + nbr.template get<DX + 1, DY, DZ>();
        s = s + nbr.template get<DX, DY - 1, DZ>();
        s = s + nbr.template get<DX, DY + 1, DZ>();
        if constexpr (DIM == 3) {
            s = s + nbr.template get<DX, DY, DZ - 1>();
            s = s + nbr.template get<DX, DY, DZ + 1>();
        }
        return op.relax(s, f[at<DX, DY, DZ>()], nb<DX, DY, DZ>());
    }
    template <int DX, int DY, int DZ, typename Nbr>
    __device__ __forceinline__ T residual(const Nbr& nbr, const T* f, T uc) const
    {
        T s = nbr.template get<DX - 1, DY, DZ>() + nbr.template get<DX + 1, DY, DZ>();
        s = s + nbr.template get<DX, DY - 1, DZ>();
        s = s + nbr.template get<DX, DY + 1, DZ>();
        if constexpr (DIM == 3) {
            s = s + nbr.template get<DX, DY, DZ - 1>();
            s = s + nbr.template get<DX, DY, DZ + 1>();
        }
        return op.residual(s, f[at<DX, DY, DZ>()], uc, nb<DX, DY, DZ>());
    }
};

// index of an in-block cell among the block's 4 (2D: 2) cells of its colour
template <int DIM, int DX, int DY, int DZ>
constexpr int slot() { return DIM == 3 ? (DY * 2 + DZ) : DY; }  // (DX follows from the colour)

// ---- k_bres -------------------------------------------------------------------------------------------------------

template <typename T, int DIM>
struct BresRed {  // red cells: loaded from u (final after the red half-sweep)
    const Blk<T, DIM>& b;
    const T* u;
    template <int DX, int DY, int DZ>
    __device__ __forceinline__ T get() const { return b.template ld<DX, DY, DZ>(u); }
};

template <typename T, int DIM>
struct BresVal {  // any cell after the black half-sweep: red loaded, black from the block or recomputed
    const Blk<T, DIM>& b;
    const T* u;
    const T* f;
    const T* bv;
    template <int DX, int DY, int DZ>
    __device__ __forceinline__ T get() const
    {
        if constexpr (!Blk<T, DIM>::template black<DX, DY, DZ>()) {
            return b.template ld<DX, DY, DZ>(u);
        } else if constexpr (Blk<T, DIM>::template in_block<DX, DY, DZ>()) {
            return bv[slot<DIM, DX, DY, DZ>()];
        } else {
            return b.template inside<DX, DY, DZ>() ? b.template relax<DX, DY, DZ>(BresRed<T, DIM>{b, u}, f) : (T)0;
        }
    }
};

template <typename T, int DIM>
__global__ __launch_bounds__(kBlock) void k_bres(T* __restrict__ u, const T* __restrict__ f, T* __restrict__ R,
                                                 Geo g, Geo gc, Op<T, DIM> op)
{
    const int64_t it = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * kBlock + threadIdx.x;
    const int lcx = g.lx - 1, lcy = g.ly - 1;
    if (it >= ((int64_t)1 << (lcx + lcy)) * (DIM == 3 ? (g.nz >> 1) : 1)) return;
    const int I = (int)(it & ((1 << lcx) - 1));
    const int J = (int)((it >> lcx) & ((1 << lcy) - 1));
    const int64_t K = DIM == 3 ? it >> (lcx + lcy) : 0;
    const Blk<T, DIM> b(g, op, I, J, K);
    const BresRed<T, DIM> red{b, u};
    // the block's black cells: 3D (1,0,0) (0,1,0) (0,0,1) (1,1,1) in slots 0, 2, 1, 3; 2D (1,0) (0,1)
    T bv[DIM == 3 ? 4 : 2];
    if constexpr (DIM == 3) {
        bv[slot<3, 1, 0, 0>()] = b.template relax<1, 0, 0>(red, f);
        bv[slot<3, 0, 1, 0>()] = b.template relax<0, 1, 0>(red, f);
        bv[slot<3, 0, 0, 1>()] = b.template relax<0, 0, 1>(red, f);
        bv[slot<3, 1, 1, 1>()] = b.template relax<1, 1, 1>(red, f);
    } else {
        bv[slot<2, 1, 0, 0>()] = b.template relax<1, 0, 0>(red, f);
        bv[slot<2, 0, 1, 0>()] = b.template relax<0, 1, 0>(red, f);
    }
    const BresVal<T, DIM> val{b, u, f, bv};
    // R = 1/2^d (((r000 + r100) + r010) + r110 [+ r001 + r101 + r011 + r111]), k_resrestrict's order
    T acc = b.template residual<0, 0, 0>(val, f, b.template ld<0, 0, 0>(u)) +
            b.template residual<1, 0, 0>(val, f, bv[slot<DIM, 1, 0, 0>()]);
    acc = acc + b.template residual<0, 1, 0>(val, f, bv[slot<DIM, 0, 1, 0>()]);
    acc = acc + b.template residual<1, 1, 0>(val, f, b.template ld<1, 1, 0>(u));
    if constexpr (DIM == 3) {
        acc = acc + b.template residual<0, 0, 1>(val, f, bv[slot<3, 0, 0, 1>()]);
        acc = acc + b.template residual<1, 0, 1>(val, f, b.template ld<1, 0, 1>(u));
        acc = acc + b.template residual<0, 1, 1>(val, f, b.template ld<0, 1, 1>(u));
        acc = acc + b.template residual<1, 1, 1>(val, f, bv[slot<3, 1, 1, 1>()]);
    }
    R[pidx(gc, I, J, K)] = (DIM == 3 ? (T)0.125 : (T)0.25) * acc;
    u[b.template at<1, 0, 0>()] = bv[slot<DIM, 1, 0, 0>()];
    u[b.template at<0, 1, 0>()] = bv[slot<DIM, 0, 1, 0>()];
    if constexpr (DIM == 3) {
        u[b.template at<0, 0, 1>()] = bv[slot<3, 0, 0, 1>()];
        u[b.template at<1, 1, 1>()] = bv[slot<3, 1, 1, 1>()];
    }
}

// ---- k_rbsweep ----------------------------------------------------------------------------------------------------

template <typename T, int DIM>
struct SwBlack {  // black cells: the sweep's input, from src
    const Blk<T, DIM>& b;
    const T* src;
    template <int DX, int DY, int DZ>
    __device__ __forceinline__ T get() const { return b.template ld<DX, DY, DZ>(src); }
};

template <typename T, int DIM>
struct SwRed {  // red cells after the red half: the block's own, or recomputed outside it
    const Blk<T, DIM>& b;
    const T* src;
    const T* f;
    const T* rv;
    template <int DX, int DY, int DZ>
    __device__ __forceinline__ T get() const
    {
        if constexpr (Blk<T, DIM>::template in_block<DX, DY, DZ>()) {
            return rv[slot<DIM, DX, DY, DZ>()];
        } else {
            return b.template inside<DX, DY, DZ>() ? b.template relax<DX, DY, DZ>(SwBlack<T, DIM>{b, src}, f) : (T)0;
        }
    }
};

template <typename T, int DIM, bool STORE_RED>
__global__ __launch_bounds__(kBlock) void k_rbsweep(const T* __restrict__ src, const T* __restrict__ f,
                                                    T* __restrict__ dst, Geo g, Op<T, DIM> op)
{
    const int64_t it = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * kBlock + threadIdx.x;
    const int lcx = g.lx - 1, lcy = g.ly - 1;
    if (it >= ((int64_t)1 << (lcx + lcy)) * (DIM == 3 ? (g.nz >> 1) : 1)) return;
    const int I = (int)(it & ((1 << lcx) - 1));
    const int J = (int)((it >> lcx) & ((1 << lcy) - 1));
    const int64_t K = DIM == 3 ? it >> (lcx + lcy) : 0;
    const Blk<T, DIM> b(g, op, I, J, K);
    const SwBlack<T, DIM> blk{b, src};
    // the block's red cells: 3D (0,0,0) (0,1,1) (1,0,1) (1,1,0) in slots 0, 3, 1, 2; 2D (0,0) (1,1)
    T rv[DIM == 3 ? 4 : 2];
    rv[slot<DIM, 0, 0, 0>()] = b.template relax<0, 0, 0>(blk, f);
    rv[slot<DIM, 1, 1, 0>()] = b.template relax<1, 1, 0>(blk, f);
    if constexpr (DIM == 3) {
        rv[slot<3, 1, 0, 1>()] = b.template relax<1, 0, 1>(blk, f);
        rv[slot<3, 0, 1, 1>()] = b.template relax<0, 1, 1>(blk, f);
    }
    const SwRed<T, DIM> red{b, src, f, rv};
    const T b100 = b.template relax<1, 0, 0>(red, f);
    const T b010 = b.template relax<0, 1, 0>(red, f);
    dst[b.template at<1, 0, 0>()] = b100;
    dst[b.template at<0, 1, 0>()] = b010;
    if constexpr (DIM == 3) {
        const T b001 = b.template relax<0, 0, 1>(red, f);
        const T b111 = b.template relax<1, 1, 1>(red, f);
        dst[b.template at<0, 0, 1>()] = b001;
        dst[b.template at<1, 1, 1>()] = b111;
    }
    if constexpr (STORE_RED) {
        dst[b.template at<0, 0, 0>()] = rv[slot<DIM, 0, 0, 0>()];
        dst[b.template at<1, 1, 0>()] = rv[slot<DIM, 1, 1, 0>()];
        if constexpr (DIM == 3) {
            dst[b.template at<1, 0, 1>()] = rv[slot<3, 1, 0, 1>()];
            dst[b.template at<0, 1, 1>()] = rv[slot<3, 0, 1, 1>()];
        }
    }
}

// ---- vector forms: a thread owns N coarse cells along x (N packed cells of each fine row and colour) ----
//
// The fine rows of a thread's coarse cells I0 .. I0+N-1 (coarse row J, plane K) are rows j0 + dy, planes k0 + dz
// (j0 = 2J, k0 = 2K) at packed m0 .. m0+N-1 (m0 = I0) of either colour half: one 16-byte vector each.  The colour's
// x parity in a row is c ^ ((dy + dz) & 1) (block origins and z0 even), a compile-time constant once the loops over
// dy / dz are unrolled, so every vector, its neighbours and the one x-edge cell outside the segment are static.  Row
// vectors of rows / planes outside the box are zero (the reference's ghost 0).  Per 4 coarse cells k_bres_v loads
// 24 red row vectors and 16 f vectors where the scalar form issued ~150 loads per coarse cell.
template <typename T, int N, int DIM>
struct VB {
    const Geo& g;
    const Op<T, DIM>& op;
    int m0, j0;
    int64_t k0;
    __device__ __forceinline__ bool valid(int dz, int dy) const
    {
        const int j = j0 + dy;
        if (j < 0 || j >= g.ny) return false;
        if (DIM == 3) {
            const int64_t k = k0 + dz;
            return k >= 0 && k < g.nz;
        }
        return true;
    }
    __device__ __forceinline__ int64_t off(int dz, int dy, int c) const
    {
        return (k0 + dz) * g.P + c * g.H + (int64_t)(j0 + dy) * g.hw + m0;
    }
    __device__ __forceinline__ Vec<T, N> ld(const T* p, int dz, int dy, int c) const
    {
        return valid(dz, dy) ? vload<T, N>(p + off(dz, dy, c)) : vzero<T, N>();
    }
    // colour c's cell at packed m of row (dz, dy), 0 outside the box
    __device__ __forceinline__ T lds(const T* p, int dz, int dy, int c, int m) const
    {
        return valid(dz, dy) && m >= 0 && m < g.hw ? p[off(dz, dy, c) - m0 + m] : (T)0;
    }
    __device__ __forceinline__ int nbyz(int dz, int dy) const
    {
        const int j = j0 + dy;
        int n = (j == 0) + (j == g.ny - 1);
        if (DIM == 3) {
            const int64_t k = g.z0 + k0 + dz;
            n += (k == 0) + (k == g.gnz - 1);
        }
        return n;
    }
    // relax the N cells (x parity o) of a row from the other colour: the row's own vector cen with the x-edge value
    // outside it, rows y -+ 1 and planes z -+ 1 (k_half's half_store expression and order)
    __device__ __forceinline__ Vec<T, N> relax_row(int o, const Vec<T, N>& cen, T edge, const Vec<T, N>& yl,
                                                   const Vec<T, N>& yr, const Vec<T, N>& zl, const Vec<T, N>& zr,
                                                   const Vec<T, N>& fv, int nbyz_) const
    {
        T d0, y0, d1, y1;
        row_diag_fast(op, nbyz_, d0, y0, d1, y1);
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
            const bool xf = i == 0 || i == g.nx - 1;
            out.v[e] = div_rn(fv.v[e] - s * op.inv_hSq, xf ? d1 : d0, xf ? y1 : y0);
        }
        return out;
    }
    // the residuals f - (sum / h^2 + diag u) of the N cells (x parity o) of a row (k_resrestrict's expression)
    __device__ __forceinline__ void residual_row(int o, const Vec<T, N>& cen, T edge, const Vec<T, N>& yl,
                                                 const Vec<T, N>& yr, const Vec<T, N>& zl, const Vec<T, N>& zr,
                                                 const Vec<T, N>& fv, const Vec<T, N>& uc, int nbyz_, T (&r)[N]) const
    {
        T d0, y0, d1, y1;
        row_diag_fast(op, nbyz_, d0, y0, d1, y1);
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
            const bool xf = i == 0 || i == g.nx - 1;
            const T askew = s * op.inv_hSq;
            const T a_u = askew + (xf ? d1 : d0) * uc.v[e];
            r[e] = fv.v[e] - a_u;
        }
    }
    // the cell of colour x (x parity ox in row (dz, dy)) at packed me, relaxed from colour 1 - x read from p: the
    // x-edge value just outside a row vector (0 outside the box)
    __device__ __forceinline__ T edge_relax(const T* p, const T* f, int dz, int dy, int cx, int ox, int me) const
    {
        if (!valid(dz, dy) || me < 0 || me >= g.hw) return (T)0;
        const int cy = cx ^ 1;
        const int i = 2 * me + ox;
        T s = lds(p, dz, dy, cy, ox == 0 ? me - 1 : me) + lds(p, dz, dy, cy, ox == 0 ? me : me + 1);
        s = s + lds(p, dz, dy - 1, cy, me);
        s = s + lds(p, dz, dy + 1, cy, me);
        if (DIM == 3) {
            s = s + lds(p, dz - 1, dy, cy, me);
            s = s + lds(p, dz + 1, dy, cy, me);
        }
        return op.relax(s, f[off(dz, dy, cx) - m0 + me], nbyz(dz, dy) + (i == 0) + (i == g.nx - 1));
    }
};

// rows (dz, dy) a thread reads of the colour its rows are relaxed from, and the rows it relaxes: the block rows
// (dz, dy in 0..1) and the rows just outside the block in y and z whose cells neighbour the block's cells
template <int DIM>
__device__ constexpr bool vb_need_src(int dz, int dy)
{
    if (DIM == 2) return dz == 0 && dy >= -2 && dy <= 3;
    return ((dz == 0 || dz == 1) && dy >= -2 && dy <= 3) || ((dz == -1 || dz == 2) && dy >= -1 && dy <= 2) ||
           ((dz == -2 || dz == 3) && (dy == 0 || dy == 1));
}
template <int DIM>
__device__ constexpr bool vb_need_mid(int dz, int dy)
{
    if (DIM == 2) return dz == 0 && dy >= -1 && dy <= 2;
    return ((dz == 0 || dz == 1) && dy >= -1 && dy <= 2) || ((dz == -1 || dz == 2) && (dy == 0 || dy == 1));
}

template <typename T, int N, int DIM>
__device__ __forceinline__ bool vb_coords(const Geo& g, int& m0, int& J, int64_t& K)
{
    constexpr int LN = N == 4 ? 2 : (N == 2 ? 1 : 0);
    const int64_t it = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * kBlock + threadIdx.x;
    const int lgpr = (g.lx - 1) - LN;
    const int cy = g.ny >> 1;
    const int grp = (int)(it & ((1 << lgpr) - 1));
    J = (int)((it >> lgpr) & (cy - 1));
    K = DIM == 3 ? it >> (lgpr + g.ly - 1) : 0;
    m0 = grp * N;
    return DIM == 2 ? (it >> (lgpr + g.ly - 1)) == 0 : K < (g.nz >> 1);
}

#define VB_ZLO (DIM == 3 ? -2 : 0)
#define VB_ZHI (DIM == 3 ? 3 : 0)
#define VB_IDX(dz, dy) [(dz) - VB_ZLO][(dy) + 2]

template <typename T, int N, int DIM>
__global__ __launch_bounds__(kBlock) void k_bres_v(T* __restrict__ u, const T* __restrict__ f, T* __restrict__ R,
                                                   Geo g, Geo gc, Op<T, DIM> op)
{
    int m0, J;
    int64_t K;
    if (!vb_coords<T, N, DIM>(g, m0, J, K)) return;
    const VB<T, N, DIM> b{g, op, m0, 2 * J, DIM == 3 ? 2 * K : 0};
    constexpr int NZ = DIM == 3 ? 2 : 1;
    constexpr int ZS = VB_ZHI - VB_ZLO + 1;
    Vec<T, N> rv[ZS][6], bv[ZS][6], fb[ZS][6];
    T re[ZS][6];
    // the red rows (final after the red half-sweep) and, for the rows relaxed below, their x-edge red cell
#pragma unroll
    for (int dz = VB_ZLO; dz <= VB_ZHI; ++dz)
#pragma unroll
        for (int dy = -2; dy <= 3; ++dy) {
            if (!vb_need_src<DIM>(dz, dy)) continue;
            rv VB_IDX(dz, dy) = b.ld(u, dz, dy, 0);
            if (vb_need_mid<DIM>(dz, dy)) {
                const int ob = 1 ^ ((dy + dz) & 1);  // x parity of the black cells
                re VB_IDX(dz, dy) = b.lds(u, dz, dy, 0, ob == 0 ? m0 - 1 : m0 + N);
                fb VB_IDX(dz, dy) = b.ld(f, dz, dy, 1);
            }
        }
    // the black half-sweep on the block rows and the rows around the block
#pragma unroll
    for (int dz = VB_ZLO; dz <= VB_ZHI; ++dz)
#pragma unroll
        for (int dy = -2; dy <= 3; ++dy) {
            if (!vb_need_mid<DIM>(dz, dy)) continue;
            const int ob = 1 ^ ((dy + dz) & 1);
            const Vec<T, N> z0v = vzero<T, N>();
            bv VB_IDX(dz, dy) =
                b.valid(dz, dy)
                    ? b.relax_row(ob, rv VB_IDX(dz, dy), re VB_IDX(dz, dy), rv VB_IDX(dz, dy - 1), rv VB_IDX(dz, dy + 1),
                                  DIM == 3 ? rv VB_IDX(dz - (DIM == 3), dy) : z0v,
                                  DIM == 3 ? rv VB_IDX(dz + (DIM == 3), dy) : z0v, fb VB_IDX(dz, dy), b.nbyz(dz, dy))
                    : z0v;
        }
    // residuals of the block rows, both colours, restricted in k_resrestrict's order
    T acc[N];
#pragma unroll
    for (int dz = 0; dz < NZ; ++dz)
#pragma unroll
        for (int dy = 0; dy < 2; ++dy) {
            const int ob = 1 ^ ((dy + dz) & 1), orr = ob ^ 1;
            const int nb = b.nbyz(dz, dy);
            const Vec<T, N> z0v = vzero<T, N>();
            T rr[2][N], rb[N], rd[N];
            // black cells: red neighbours (loaded), own value the new black
            b.residual_row(ob, rv VB_IDX(dz, dy), re VB_IDX(dz, dy), rv VB_IDX(dz, dy - 1), rv VB_IDX(dz, dy + 1),
                           DIM == 3 ? rv VB_IDX(dz - (DIM == 3), dy) : z0v, DIM == 3 ? rv VB_IDX(dz + (DIM == 3), dy) : z0v,
                           fb VB_IDX(dz, dy), bv VB_IDX(dz, dy), nb, rb);
            // red cells: black neighbours (new; the x-edge one recomputed), own value loaded
            const T eb = b.edge_relax(u, f, dz, dy, 1, ob, orr == 0 ? m0 - 1 : m0 + N);
            b.residual_row(orr, bv VB_IDX(dz, dy), eb, bv VB_IDX(dz, dy - 1), bv VB_IDX(dz, dy + 1),
                           DIM == 3 ? bv VB_IDX(dz - (DIM == 3), dy) : z0v, DIM == 3 ? bv VB_IDX(dz + (DIM == 3), dy) : z0v,
                           b.ld(f, dz, dy, 0), rv VB_IDX(dz, dy), nb, rd);
#pragma unroll
            for (int e = 0; e < N; ++e) {
                rr[ob][e] = rb[e];
                rr[orr][e] = rd[e];
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
    const int64_t gK = gc.z0 + K;
    const int pc = (int)((J + gK) & 1);
    const int64_t rowc = K * gc.P + (int64_t)J * gc.hw;
#pragma unroll
    for (int e = 0; e < N; ++e) {
        const int I = m0 + e;
        R[rowc + ((I + pc) & 1) * gc.H + (I >> 1)] = (DIM == 3 ? (T)0.125 : (T)0.25) * acc[e];
    }
#pragma unroll
    for (int dz = 0; dz < NZ; ++dz)
#pragma unroll
        for (int dy = 0; dy < 2; ++dy) vstore<T, N>(u + b.off(dz, dy, 1), bv VB_IDX(dz, dy));
}

template <typename T, int N, int DIM, bool STORE_RED>
__global__ __launch_bounds__(kBlock) void k_rbsweep_v(const T* __restrict__ src, const T* __restrict__ f,
                                                      T* __restrict__ dst, Geo g, Op<T, DIM> op)
{
    int m0, J;
    int64_t K;
    if (!vb_coords<T, N, DIM>(g, m0, J, K)) return;
    const VB<T, N, DIM> b{g, op, m0, 2 * J, DIM == 3 ? 2 * K : 0};
    constexpr int NZ = DIM == 3 ? 2 : 1;
    constexpr int ZS = VB_ZHI - VB_ZLO + 1;
    Vec<T, N> bo[ZS][6], rn[ZS][6];
    T be[ZS][6];
    // the black rows (the sweep's input) and, for the rows whose red half is relaxed, their x-edge black cell
#pragma unroll
    for (int dz = VB_ZLO; dz <= VB_ZHI; ++dz)
#pragma unroll
        for (int dy = -2; dy <= 3; ++dy) {
            if (!vb_need_src<DIM>(dz, dy)) continue;
            bo VB_IDX(dz, dy) = b.ld(src, dz, dy, 1);
            if (vb_need_mid<DIM>(dz, dy)) {
                const int orr = (dy + dz) & 1;  // x parity of the red cells
                be VB_IDX(dz, dy) = b.lds(src, dz, dy, 1, orr == 0 ? m0 - 1 : m0 + N);
            }
        }
    // the red half-sweep on the block rows and the rows around the block
#pragma unroll
    for (int dz = VB_ZLO; dz <= VB_ZHI; ++dz)
#pragma unroll
        for (int dy = -2; dy <= 3; ++dy) {
            if (!vb_need_mid<DIM>(dz, dy)) continue;
            const int orr = (dy + dz) & 1;
            const Vec<T, N> z0v = vzero<T, N>();
            rn VB_IDX(dz, dy) =
                b.valid(dz, dy)
                    ? b.relax_row(orr, bo VB_IDX(dz, dy), be VB_IDX(dz, dy), bo VB_IDX(dz, dy - 1), bo VB_IDX(dz, dy + 1),
                                  DIM == 3 ? bo VB_IDX(dz - (DIM == 3), dy) : z0v,
                                  DIM == 3 ? bo VB_IDX(dz + (DIM == 3), dy) : z0v, b.ld(f, dz, dy, 0), b.nbyz(dz, dy))
                    : z0v;
        }
    // the black half-sweep on the block rows
#pragma unroll
    for (int dz = 0; dz < NZ; ++dz)
#pragma unroll
        for (int dy = 0; dy < 2; ++dy) {
            const int ob = 1 ^ ((dy + dz) & 1), orr = ob ^ 1;
            const Vec<T, N> z0v = vzero<T, N>();
            const T er = b.edge_relax(src, f, dz, dy, 0, orr, ob == 0 ? m0 - 1 : m0 + N);
            const Vec<T, N> nb_ = b.relax_row(ob, rn VB_IDX(dz, dy), er, rn VB_IDX(dz, dy - 1), rn VB_IDX(dz, dy + 1),
                                              DIM == 3 ? rn VB_IDX(dz - (DIM == 3), dy) : z0v,
                                              DIM == 3 ? rn VB_IDX(dz + (DIM == 3), dy) : z0v, b.ld(f, dz, dy, 1),
                                              b.nbyz(dz, dy));
            vstore<T, N>(dst + b.off(dz, dy, 1), nb_);
            if (STORE_RED) vstore<T, N>(dst + b.off(dz, dy, 0), rn VB_IDX(dz, dy));
        }
}

#undef VB_IDX
#undef VB_ZHI
#undef VB_ZLO

template <typename T, int D>
unsigned blocks_of(const Geo& g)
{
    return nblk((int64_t)(g.nx / 2) * (g.ny / 2) * (D == 3 ? g.nz / 2 : 1));
}

}  // namespace

bool bres_supported(int rb, const Geo& g)
{
    return (rb == 4 || rb == 8) && g.nx >= 2 && g.ny >= 2 && (g.z0 & 1) == 0;
}

// cells per thread of the vector forms (MGP_BRES_VN, read once: 0 = the scalar forms, 1 / 2 / 4; default one 16-byte
// vector) on levels whose half rows hold a whole number of them
static int bres_vn(int rb, const Geo& g)
{
    static const int env = [] {
        const char* v = std::getenv("MGP_BRES_VN");
        return v ? std::atoi(v) : -1;
    }();
    int n = env < 0 ? 16 / (rb == 8 ? 8 : 4) : env;
    if (n != 0 && n != 1 && n != 2 && n != 4) n = 16 / (rb == 8 ? 8 : 4);
    while (n > 1 && g.hw % n) n >>= 1;
    return n;
}

template <typename T, int D, int N>
static void bres_v_t(void* u, const void* f, void* R, const Geo& g, const Geo& gc, double h, double cl, hipStream_t s)
{
    const int64_t items = (int64_t)(g.nx / 2 / N) * (g.ny / 2) * (D == 3 ? g.nz / 2 : 1);
    k_bres_v<T, N, D><<<nblk(items), kBlock, 0, s>>>((T*)u, (const T*)f, (T*)R, g, gc, make_op<T, D>(h, cl));
}

template <typename T, int D>
static void bres_t(void* u, const void* f, void* R, const Geo& g, const Geo& gc, double h, double cl, hipStream_t s)
{
    const int n = bres_vn(sizeof(T), g);
    if (n == 4 && sizeof(T) == 4) bres_v_t<T, D, 4>(u, f, R, g, gc, h, cl, s);
    else if (n >= 2) bres_v_t<T, D, 2>(u, f, R, g, gc, h, cl, s);
    else if (n == 1) bres_v_t<T, D, 1>(u, f, R, g, gc, h, cl, s);
    else k_bres<T, D><<<blocks_of<T, D>(g), kBlock, 0, s>>>((T*)u, (const T*)f, (T*)R, g, gc, make_op<T, D>(h, cl));
}

hipError_t launch_black_residual_restrict(int rb, int dim, void* u, const void* f, void* R, Geo g, Geo gc, double h,
                                          double cl, hipStream_t s)
{
    if (!bres_supported(rb, g) || (dim == 3 && g.nz < 2)) return hipErrorInvalidValue;
    if (rb == 8) {
        if (dim == 3) bres_t<double, 3>(u, f, R, g, gc, h, cl, s);
        else bres_t<double, 2>(u, f, R, g, gc, h, cl, s);
    } else {
        if (dim == 3) bres_t<float, 3>(u, f, R, g, gc, h, cl, s);
        else bres_t<float, 2>(u, f, R, g, gc, h, cl, s);
    }
    return hipGetLastError();
}

template <typename T, int D, int N>
static void rbsweep_v_t(const void* src, const void* f, void* dst, const Geo& g, const Op<T, D>& op, bool store_red,
                        hipStream_t s)
{
    const int64_t items = (int64_t)(g.nx / 2 / N) * (g.ny / 2) * (D == 3 ? g.nz / 2 : 1);
    if (store_red) k_rbsweep_v<T, N, D, true><<<nblk(items), kBlock, 0, s>>>((const T*)src, (const T*)f, (T*)dst, g, op);
    else k_rbsweep_v<T, N, D, false><<<nblk(items), kBlock, 0, s>>>((const T*)src, (const T*)f, (T*)dst, g, op);
}

template <typename T, int D>
static void rbsweep_t(const void* src, const void* f, void* dst, Geo g, double h, double cl, bool store_red,
                      hipStream_t s)
{
    const Op<T, D> op = make_op<T, D>(h, cl);
    const int n = bres_vn(sizeof(T), g);
    if (n == 4 && sizeof(T) == 4) rbsweep_v_t<T, D, 4>(src, f, dst, g, op, store_red, s);
    else if (n >= 2) rbsweep_v_t<T, D, 2>(src, f, dst, g, op, store_red, s);
    else if (n == 1) rbsweep_v_t<T, D, 1>(src, f, dst, g, op, store_red, s);
    else if (store_red)
        k_rbsweep<T, D, true><<<blocks_of<T, D>(g), kBlock, 0, s>>>((const T*)src, (const T*)f, (T*)dst, g, op);
    else
        k_rbsweep<T, D, false><<<blocks_of<T, D>(g), kBlock, 0, s>>>((const T*)src, (const T*)f, (T*)dst, g, op);
}

hipError_t launch_rb_sweep(int rb, int dim, const void* src, const void* f, void* dst, Geo g, double h, double cl,
                           bool store_red, hipStream_t s)
{
    if (!bres_supported(rb, g) || (dim == 3 && g.nz < 2) || src == dst) return hipErrorInvalidValue;
    if (rb == 8) {
        if (dim == 3) rbsweep_t<double, 3>(src, f, dst, g, h, cl, store_red, s);
        else rbsweep_t<double, 2>(src, f, dst, g, h, cl, store_red, s);
    } else {
        if (dim == 3) rbsweep_t<float, 3>(src, f, dst, g, h, cl, store_red, s);
        else rbsweep_t<float, 2>(src, f, dst, g, h, cl, store_red, s);
    }
    return hipGetLastError();
}

}  // namespace mgp
