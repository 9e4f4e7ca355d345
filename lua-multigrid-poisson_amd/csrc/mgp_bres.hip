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

hipError_t launch_black_residual_restrict(int rb, int dim, void* u, const void* f, void* R, Geo g, Geo gc, double h,
                                          double cl, hipStream_t s)
{
    if (!bres_supported(rb, g) || (dim == 3 && g.nz < 2)) return hipErrorInvalidValue;
    if (rb == 8) {
        if (dim == 3)
            k_bres<double, 3><<<blocks_of<double, 3>(g), kBlock, 0, s>>>((double*)u, (const double*)f, (double*)R, g, gc,
                                                                          make_op<double, 3>(h, cl));
        else
            k_bres<double, 2><<<blocks_of<double, 2>(g), kBlock, 0, s>>>((double*)u, (const double*)f, (double*)R, g, gc,
                                                                          make_op<double, 2>(h, cl));
    } else {
        if (dim == 3)
            k_bres<float, 3><<<blocks_of<float, 3>(g), kBlock, 0, s>>>((float*)u, (const float*)f, (float*)R, g, gc,
                                                                        make_op<float, 3>(h, cl));
        else
            k_bres<float, 2><<<blocks_of<float, 2>(g), kBlock, 0, s>>>((float*)u, (const float*)f, (float*)R, g, gc,
                                                                        make_op<float, 2>(h, cl));
    }
    return hipGetLastError();
}

template <typename T, int D>
static void rbsweep_t(const void* src, const void* f, void* dst, Geo g, double h, double cl, bool store_red,
                      hipStream_t s)
{
    const Op<T, D> op = make_op<T, D>(h, cl);
    if (store_red)
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
