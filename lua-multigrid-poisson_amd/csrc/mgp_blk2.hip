// mgp_blk2.hip — the tiled smoothing phases of two consecutive small 2D levels in one launch (round 6).
//
// k_blk (mgp_kernels.hip) runs a small level's PRE (nu1 red/black sweeps, calcResidual, reduceResidual:
// cpu.lua:40-54, 108-135) as one launch per level; below 1024^2 a launch costs more than its work.  k_blk2_pre
// runs PRE of level l AND of level l + 1 in one launch (V-cycle, cpu.lua:138-139: the coarse level's PRE follows the
// fine level's restriction directly).  A workgroup owns a B x B tile of level l + 1 (2B x 2B of level l):
//   1. it loads level l's u (black cells) and f on its fine box: the children of its coarse box (the coarse tile
//      with k_blk's halo E = 2 nu + 1, x rounded to even) plus the same halo again at the fine level;
//   2. runs level l's 2 nu half-sweeps in LDS on shrinking regions (k_blk's scheme);
//   3. restricts the fine residuals onto the whole coarse box in LDS (the coarse tile's f and its halo: the
//      neighbouring workgroups compute the same numbers with the same expressions), stores its fine tile's black
//      cells and its coarse tile's f;
//   4. runs level l + 1's PRE on the coarse box exactly as k_blk does (u = 0 for a fresh guess, or the warm guess's
//      black cells), and stores the coarse tile's black cells and the restriction of its residuals (level l + 2's f).
// k_blk2_post runs POST of level l + 1 and then of level l (prolong_correct + nu2 sweeps each) in one launch: the
// workgroup corrects and smooths level l + 1 on its tile and the cells around it that level l's prolongation reads
// (k_blk's POST with a wider target region), stores its coarse tile, then corrects its fine box from those values in LDS
// and smooths its fine tile.
// Every expression and its order is half_item's / residual_at's / resrestrict_item's / prolong_value's, so the results
// are bit-identical to two k_blk launches and to the launch-per-piece path.
#include "mgp_device.h"

namespace mgp {
namespace {

constexpr int kB2Threads = 1024;
// owned tile edge of level l + 1: 32, or 16 where 32 would give fewer than B2_T16_BELOW workgroups (build knob)
#ifndef B2_T16_BELOW
#define B2_T16_BELOW 64
#endif

// An LDS box of a 2D level: EX x EY cells from a global origin (xs even, ys), k_blk's layout: the slots of row ly and
// colour c at (2 ly + c) EH, EH = EX / 2, so LDS cell (lx, ly) of colour c sits at slot lx >> 1 of that row.
template <int EX_, int EY_>
struct B2Box {
    static constexpr int EX = EX_, EY = EY_, EH = EX / 2, cells = EX * EY;
    static __device__ __forceinline__ int lidx(int ly, int c, int mm) { return (2 * ly + c) * EH + mm; }
};

template <int NS, int BT>
struct B2Shape {
    static constexpr int B = BT;
    static constexpr int EC = 2 * NS + 1, HXC = (EC + 1) & ~1;  // level l + 1: k_blk's PRE halo
    using C = B2Box<B + 2 * HXC, B + 2 * EC>;
    static constexpr int EF = 2 * NS + 1, HXF = (EF + 1) & ~1;  // level l: the same halo around the coarse box's children
    static constexpr int RX = 2 * C::EX, RY = 2 * C::EY;
    using F = B2Box<RX + 2 * HXF, RY + 2 * EF>;
    static constexpr size_t lds_reals = 2 * (size_t)F::cells + 2 * (size_t)C::cells;
};

// in-plane neighbour sum of LDS cell (lx, ly) of colour c: half_item's order (x-, x+, y-, y+)
template <typename T, class BX>
__device__ __forceinline__ T b2_nbsum(const T* U, int lx, int ly, int c)
{
    const int mm = lx >> 1, o = lx & 1;
    const int oth = BX::lidx(ly, c ^ 1, mm);
    T sum = U[oth - 1 + o] + U[oth + o];
    sum = sum + U[oth - 2 * BX::EH];
    sum = sum + U[oth + 2 * BX::EH];
    return sum;
}

__device__ __forceinline__ int b2_faces(int gi, int gj, int nx, int ny)
{
    return (gi == 0) + (gi == nx - 1) + (gj == 0) + (gj == ny - 1);
}

// 2 NS half-sweeps (red first) of box BX whose target region is [X0, X0 + WX) x [Y0, Y0 + WY) (LDS coordinates): half-
// sweep s runs on the region extended by E - 1 - s cells (cells outside the level skipped), one barrier each
template <typename T, class BX, int NS, int E, int X0, int WX, int Y0, int WY>
__device__ __forceinline__ void b2_sweeps(T* U, const T* F, const Op<T, 2>& op, int xs, int ys, int nx, int ny, int tid)
{
    const int p0 = ys & 1;
#pragma unroll
    for (int s = 0; s < 2 * NS; ++s) {
        const int c = s & 1, e = E - 1 - s;
        const int xlo = X0 - e, xhi = X0 + WX - 1 + e, ylo = Y0 - e;
        const int mlo = xlo >> 1, nm = (xhi >> 1) - mlo + 1, ny_ = WY + 2 * e, n = ny_ * nm;
#pragma unroll
        for (int q = 0; q < (n + kB2Threads - 1) / kB2Threads; ++q) {
            const int it = tid + q * kB2Threads;
            const int row = it / nm, mm = mlo + it % nm;
            const int ly = ylo + row;
            const int lx = 2 * mm + (c ^ ((ly + p0) & 1));
            const int gi = xs + lx, gj = ys + ly;
            if (it < n && lx >= xlo && lx <= xhi && gi >= 0 && gi < nx && gj >= 0 && gj < ny) {
                const T sum = b2_nbsum<T, BX>(U, lx, ly, c);
                const int own = BX::lidx(ly, c, mm);
                U[own] = op.relax_idx(sum, F[own], b2_faces(gi, gj, nx, ny));
            }
        }
        __syncthreads();
    }
}

// residual of LDS cell (lx, ly) of box BX (global origin xs, ys): residual_at's expression
template <typename T, class BX>
__device__ __forceinline__ T b2_res(const T* U, const T* F, const Op<T, 2>& op, int lx, int ly, int xs, int ys, int nx,
                                    int ny)
{
    const int c = (lx & 1) ^ ((ly + ys) & 1);
    const int own = BX::lidx(ly, c, lx >> 1);
    return op.residual_idx(b2_nbsum<T, BX>(U, lx, ly, c), F[own], U[own], b2_faces(xs + lx, ys + ly, nx, ny));
}

// the average restriction of the 4 children of coarse cell (I, J) whose child (2I, 2J) is LDS cell (lx, ly) of box
// BX: resrestrict_item's order
template <typename T, class BX>
__device__ __forceinline__ T b2_restrict(const T* U, const T* F, const Op<T, 2>& op, int lx, int ly, int xs, int ys,
                                         int nx, int ny)
{
    T sm = b2_res<T, BX>(U, F, op, lx, ly, xs, ys, nx, ny) + b2_res<T, BX>(U, F, op, lx + 1, ly, xs, ys, nx, ny);
    sm = sm + b2_res<T, BX>(U, F, op, lx, ly + 1, xs, ys, nx, ny);
    sm = sm + b2_res<T, BX>(U, F, op, lx + 1, ly + 1, xs, ys, nx, ny);
    return (T)0.25 * sm;
}

template <typename T, int NS, int BT>
__global__ __launch_bounds__(kB2Threads) void k_blk2_pre(const T* __restrict__ src, const T* __restrict__ f,
                                                         T* __restrict__ dst, T* __restrict__ f1,
                                                         const T* __restrict__ src1, T* __restrict__ dst1,
                                                         T* __restrict__ R, Geo g, Geo g1, Geo g2, Op<T, 2> op,
                                                         Op<T, 2> op1)
{
    using S = B2Shape<NS, BT>;
    using FB = typename S::F;
    using CB = typename S::C;
    constexpr int NT = kB2Threads, B = S::B, EC = S::EC, HXC = S::HXC, EF = S::EF, HXF = S::HXF;
    extern __shared__ __align__(16) unsigned char b2_smem[];
    T* const UF = reinterpret_cast<T*>(b2_smem);
    T* const FF = UF + FB::cells;
    T* const UC = FF + FB::cells;
    T* const FC = UC + CB::cells;
    __shared__ Op<T, 2> sop[2];  // the operators in LDS: their diagonal tables are indexed per cell
    const int tid = threadIdx.x;
    if (tid == 0) {
        sop[0] = op;
        sop[1] = op1;
    }
    const int ntx = g1.nx / B;
    const int XC0 = ((int)blockIdx.x % ntx) * B, YC0 = ((int)blockIdx.x / ntx) * B;  // the owned coarse tile
    const int xcs = XC0 - HXC, ycs = YC0 - EC;         // coarse box origin (even x)
    const int xfs = 2 * xcs - HXF, yfs = 2 * ycs - EF;  // fine box origin (even x)

    // 1. level l: u's black cells (0 for a fresh guess) and f of the fine box, 0 outside the level
    {
        constexpr int n = FB::cells, NB = (n + NT - 1) / NT;
        T uv[NB], fv[NB];
#pragma unroll
        for (int q = 0; q < NB; ++q) {
            const int it = tid + q * NT;
            const int row = it / (2 * FB::EH), rest = it % (2 * FB::EH);
            const int c = rest >= FB::EH, mm = rest - c * FB::EH;
            const int gm = (xfs >> 1) + mm, gj = yfs + row;
            const bool in = it < n && gm >= 0 && gm < g.hw && gj >= 0 && gj < g.ny;
            const int64_t gi = c * g.H + (int64_t)gj * g.hw + gm;
            fv[q] = in ? f[gi] : (T)0;
            uv[q] = in && c == 1 && src ? src[gi] : (T)0;
        }
#pragma unroll
        for (int q = 0; q < NB; ++q) {
            const int it = tid + q * NT;
            if (it < n) {
                UF[it] = uv[q];
                FF[it] = fv[q];
            }
        }
    }
    __syncthreads();

    // 2. level l's half-sweeps; the residual region is the coarse box's children
    b2_sweeps<T, FB, NS, EF, HXF, S::RX, EF, S::RY>(UF, FF, sop[0], xfs, yfs, (int)g.nx, (int)g.ny, tid);

    // 3. the coarse box: f = the restricted fine residuals (0 outside level l + 1), u = the warm guess's black cells
    //    or 0; then the owned fine tile's black cells to dst
    {
        constexpr int n = CB::cells;
#pragma unroll
        for (int q = 0; q < (n + NT - 1) / NT; ++q) {
            const int it = tid + q * NT;
            const int row = it / (2 * CB::EH), rest = it % (2 * CB::EH);
            const int c = rest >= CB::EH, mm = rest - c * CB::EH;
            const int lx = 2 * mm + (c ^ ((row + ycs) & 1));
            const int I = xcs + lx, J = ycs + row;
            T fc = (T)0, uc = (T)0;
            if (it < n && I >= 0 && I < g1.nx && J >= 0 && J < g1.ny) {
                fc = b2_restrict<T, FB>(UF, FF, sop[0], 2 * lx + HXF, 2 * row + EF, xfs, yfs, (int)g.nx, (int)g.ny);
                if (c == 1 && src1) uc = src1[g1.H + (int64_t)J * g1.hw + (I >> 1)];
            }
            if (it < n) {
                FC[it] = fc;
                UC[it] = uc;
            }
        }
        constexpr int H2 = B, nf = 2 * B * H2;  // 2B rows of B black slots
#pragma unroll
        for (int q = 0; q < (nf + NT - 1) / NT; ++q) {
            const int it = tid + q * NT;
            if (it < nf) {
                const int mm = it % H2, ly = it / H2;
                dst[g.H + (int64_t)(2 * YC0 + ly) * g.hw + XC0 + mm] =
                    UF[FB::lidx(2 * EC + EF + ly, 1, ((2 * HXC + HXF) >> 1) + mm)];
            }
        }
    }
    __syncthreads();
    // the owned coarse tile's f (both colours: level l + 1's POST reads it)
    {
        constexpr int H2 = B / 2, n = B * 2 * H2;
#pragma unroll
        for (int q = 0; q < (n + NT - 1) / NT; ++q) {
            const int it = tid + q * NT;
            if (it < n) {
                const int mm = it % H2, c = (it / H2) & 1, ly = it / (2 * H2);
                f1[c * g1.H + (int64_t)(YC0 + ly) * g1.hw + (XC0 >> 1) + mm] = FC[CB::lidx(EC + ly, c, (HXC >> 1) + mm)];
            }
        }
    }

    // 4. level l + 1's PRE on the coarse box (k_blk's), residual + restriction of the owned tile to level l + 2
    b2_sweeps<T, CB, NS, EC, HXC, B, EC, B>(UC, FC, sop[1], xcs, ycs, (int)g1.nx, (int)g1.ny, tid);
    {
        constexpr int C2 = B / 2;
        for (int it = tid; it < C2 * C2; it += NT) {
            const int I = it % C2, J = it / C2;
            const T v = b2_restrict<T, CB>(UC, FC, sop[1], HXC + 2 * I, EC + 2 * J, xcs, ycs, (int)g1.nx, (int)g1.ny);
            R[pidx(g2, (XC0 >> 1) + I, (YC0 >> 1) + J, 0)] = v;
        }
        constexpr int H2 = B / 2, n = B * H2;  // the owned coarse tile's black cells
#pragma unroll
        for (int q = 0; q < (n + NT - 1) / NT; ++q) {
            const int it = tid + q * NT;
            if (it < n) {
                const int mm = it % H2, ly = it / H2;
                dst1[g1.H + (int64_t)(YC0 + ly) * g1.hw + (XC0 >> 1) + mm] = UC[CB::lidx(EC + ly, 1, (HXC >> 1) + mm)];
            }
        }
    }
}

template <int NS, int BT>
struct B2PostShape {
    static constexpr int B = BT;                           // owned tile of level l + 1 (level l: 2B x 2B)
    static constexpr int EF = 2 * NS, HXF = (EF + 1) & ~1;  // level l: k_blk's POST halo
    using F = B2Box<2 * B + 2 * HXF, 2 * B + 2 * EF>;
    // level l + 1's final values that level l's prolongation reads: the tile and G cells around it (even)
    static constexpr int G = ((HXF / 2 + 2) + 1) & ~1;
    static constexpr int EC = 2 * NS, HXC = (EC + 1) & ~1;  // level l + 1's POST halo around that region
    using C = B2Box<B + 2 * (G + HXC), B + 2 * (G + EC)>;
    // level l + 2's values the coarse box's prolongation reads, unpacked (k_blk's POST staging region)
    static constexpr int CX2 = C::EX / 2 + 2, CY2 = C::EY / 2 + 3, c2cells = CX2 * CY2;
    static constexpr size_t lds_reals = 2 * (size_t)F::cells + 2 * (size_t)C::cells + (size_t)c2cells;
};

template <typename T, int NS, int LINEAR, int BT>
__global__ __launch_bounds__(kB2Threads) void k_blk2_post(const T* __restrict__ src, const T* __restrict__ f,
                                                          T* __restrict__ dst, const T* __restrict__ src1,
                                                          const T* __restrict__ f1, T* __restrict__ dst1,
                                                          const T* __restrict__ V2, Geo g, Geo g1, Geo g2, Op<T, 2> op,
                                                          Op<T, 2> op1, T cl1, T cl2)
{
    using S = B2PostShape<NS, BT>;
    using FB = typename S::F;
    using CB = typename S::C;
    constexpr int NT = kB2Threads, B = S::B, EC = S::EC, HXC = S::HXC, EF = S::EF, HXF = S::HXF, G = S::G;
    extern __shared__ __align__(16) unsigned char b2_smem[];
    T* const UF = reinterpret_cast<T*>(b2_smem);
    T* const FF = UF + FB::cells;
    T* const UC = FF + FB::cells;
    T* const FC = UC + CB::cells;
    T* const VC = FC + CB::cells;
    __shared__ Op<T, 2> sop[2];
    const int tid = threadIdx.x;
    if (tid == 0) {
        sop[0] = op;
        sop[1] = op1;
    }
    const int ntx = g1.nx / B;
    const int XC0 = ((int)blockIdx.x % ntx) * B, YC0 = ((int)blockIdx.x / ntx) * B;
    const int xcs = XC0 - G - HXC, ycs = YC0 - G - EC;  // coarse box origin (even x)
    const int xfs = 2 * XC0 - HXF, yfs = 2 * YC0 - EF;  // fine box origin (even x)
    const int cx0 = (xcs >> 1) - 1, cy0 = (ycs >> 1) - 1;

    // level l's u (black) and f, loaded now and stored to LDS after level l + 1 is done
    constexpr int nF = FB::cells, NBF = (nF + NT - 1) / NT;
    T ufv[NBF], ffv[NBF];
#pragma unroll
    for (int q = 0; q < NBF; ++q) {
        const int it = tid + q * NT;
        const int row = it / (2 * FB::EH), rest = it % (2 * FB::EH);
        const int c = rest >= FB::EH, mm = rest - c * FB::EH;
        const int gm = (xfs >> 1) + mm, gj = yfs + row;
        const bool in = it < nF && gm >= 0 && gm < g.hw && gj >= 0 && gj < g.ny;
        const int64_t gi = c * g.H + (int64_t)gj * g.hw + gm;
        ffv[q] = in ? f[gi] : (T)0;
        ufv[q] = in && c == 1 ? src[gi] : (T)0;
    }
    // 1. level l + 1: V2 staged, then u (black) + P V2 and f on the coarse box
    {
        constexpr int NB2 = (S::c2cells + NT - 1) / NT;
#pragma unroll
        for (int q = 0; q < NB2; ++q) {
            const int t = tid + q * NT;
            const int I = cx0 + t % S::CX2, J = cy0 + t / S::CX2;
            if (t < S::c2cells) VC[t] = I >= 0 && I < g2.nx && J >= 0 && J < g2.ny ? V2[pidx(g2, I, J, 0)] : (T)0;
        }
    }
    constexpr int nC = CB::cells, NBC = (nC + NT - 1) / NT;
    T ucv[NBC], fcv[NBC];
#pragma unroll
    for (int q = 0; q < NBC; ++q) {
        const int it = tid + q * NT;
        const int row = it / (2 * CB::EH), rest = it % (2 * CB::EH);
        const int c = rest >= CB::EH, mm = rest - c * CB::EH;
        const int gm = (xcs >> 1) + mm, gj = ycs + row;
        const bool in = it < nC && gm >= 0 && gm < g1.hw && gj >= 0 && gj < g1.ny;
        const int64_t gi = c * g1.H + (int64_t)gj * g1.hw + gm;
        fcv[q] = in ? f1[gi] : (T)0;
        ucv[q] = in && c == 1 ? src1[gi] : (T)0;
    }
    __syncthreads();
    {
        auto get = [&](int I, int J, int64_t) { return VC[(J - cy0) * S::CX2 + (I - cx0)]; };
#pragma unroll
        for (int q = 0; q < NBC; ++q) {
            const int it = tid + q * NT;
            const int row = it / (2 * CB::EH), rest = it % (2 * CB::EH);
            const int c = rest >= CB::EH, mm = rest - c * CB::EH;
            const int gm = (xcs >> 1) + mm, gj = ycs + row;
            if (it < nC && c == 1 && gm >= 0 && gm < g1.hw && gj >= 0 && gj < g1.ny) {
                const int i = 2 * gm + (1 ^ ((gj) & 1));
                ucv[q] = ucv[q] + prolong_eval<T, 2, LINEAR>(get, g2, cl2, i, gj, 0);
            }
            if (it < nC) {
                UC[it] = ucv[q];
                FC[it] = fcv[q];
            }
        }
    }
    __syncthreads();
    // 2. level l + 1's sweeps, down to the tile and G cells around it
    b2_sweeps<T, CB, NS, EC, HXC, B + 2 * G, EC, B + 2 * G>(UC, FC, sop[1], xcs, ycs, (int)g1.nx, (int)g1.ny, tid);
    // 3. the owned coarse tile to dst1; level l's u (black) + P V from the coarse box, and f, into LDS
    {
        constexpr int H2 = B / 2, n = B * 2 * H2;
#pragma unroll
        for (int q = 0; q < (n + NT - 1) / NT; ++q) {
            const int it = tid + q * NT;
            if (it < n) {
                const int mm = it % H2, c = (it / H2) & 1, ly = it / (2 * H2);
                dst1[c * g1.H + (int64_t)(YC0 + ly) * g1.hw + (XC0 >> 1) + mm] =
                    UC[CB::lidx(G + EC + ly, c, ((G + HXC) >> 1) + mm)];
            }
        }
        auto get = [&](int I, int J, int64_t) {
            const int lx = I - xcs, ly = J - ycs;
            return UC[CB::lidx(ly, (I + J) & 1, lx >> 1)];
        };
#pragma unroll
        for (int q = 0; q < NBF; ++q) {
            const int it = tid + q * NT;
            const int row = it / (2 * FB::EH), rest = it % (2 * FB::EH);
            const int c = rest >= FB::EH, mm = rest - c * FB::EH;
            const int gm = (xfs >> 1) + mm, gj = yfs + row;
            if (it < nF && c == 1 && gm >= 0 && gm < g.hw && gj >= 0 && gj < g.ny) {
                const int i = 2 * gm + (1 ^ (gj & 1));
                ufv[q] = ufv[q] + prolong_eval<T, 2, LINEAR>(get, g1, cl1, i, gj, 0);
            }
            if (it < nF) {
                UF[it] = ufv[q];
                FF[it] = ffv[q];
            }
        }
    }
    __syncthreads();
    // 4. level l's sweeps down to its tile; the tile (both colours) to dst
    b2_sweeps<T, FB, NS, EF, HXF, 2 * B, EF, 2 * B>(UF, FF, sop[0], xfs, yfs, (int)g.nx, (int)g.ny, tid);
    {
        constexpr int H2 = B, n = 2 * B * 2 * H2;
#pragma unroll
        for (int q = 0; q < (n + NT - 1) / NT; ++q) {
            const int it = tid + q * NT;
            if (it < n) {
                const int mm = it % H2, c = (it / H2) & 1, ly = it / (2 * H2);
                dst[c * g.H + (int64_t)(2 * YC0 + ly) * g.hw + XC0 + mm] = UF[FB::lidx(EF + ly, c, (HXF >> 1) + mm)];
            }
        }
    }
}

template <typename T, int NS, int BT>
constexpr size_t b2_pre_lds()
{
    return B2Shape<NS, BT>::lds_reals * sizeof(T);
}
template <typename T, int NS, int BT>
constexpr size_t b2_post_lds()
{
    return B2PostShape<NS, BT>::lds_reals * sizeof(T);
}

// the tile edge for level l + 1 (g1): 32 unless that leaves fewer than B2_T16_BELOW workgroups and 16 divides it;
// fp64 always 16 (its 32-tile PRE needs 180 KB of LDS)
int b2_tile(int rb, const Geo& g1)
{
    const bool t32 = g1.nx % 32 == 0 && g1.ny % 32 == 0, t16 = g1.nx % 16 == 0 && g1.ny % 16 == 0;
    if (rb == 8) return t16 ? 16 : 0;
    if (t32 && (g1.nx / 32) * (g1.ny / 32) >= B2_T16_BELOW) return 32;
    return t16 ? 16 : t32 ? 32 : 0;
}

template <typename T, typename F>
hipError_t b2_each(F&& f)  // every instantiation of real type T: f(kernel, lds bytes)
{
    hipError_t e = hipSuccess;
#define B2_EACH(BT)                                                                                         \
    if (e == hipSuccess) e = f((const void*)k_blk2_pre<T, 1, BT>, b2_pre_lds<T, 1, BT>());                  \
    if (e == hipSuccess) e = f((const void*)k_blk2_pre<T, 2, BT>, b2_pre_lds<T, 2, BT>());                  \
    if (e == hipSuccess) e = f((const void*)k_blk2_post<T, 1, 0, BT>, b2_post_lds<T, 1, BT>());             \
    if (e == hipSuccess) e = f((const void*)k_blk2_post<T, 1, 1, BT>, b2_post_lds<T, 1, BT>());             \
    if (e == hipSuccess) e = f((const void*)k_blk2_post<T, 2, 0, BT>, b2_post_lds<T, 2, BT>());             \
    if (e == hipSuccess) e = f((const void*)k_blk2_post<T, 2, 1, BT>, b2_post_lds<T, 2, BT>());
    B2_EACH(16)
    if constexpr (sizeof(T) == 4) {
        B2_EACH(32)
    }
#undef B2_EACH
    return e;
}

template <typename T, int BT>
hipError_t b2_launch(const Block2Args& a, hipStream_t s)
{
    const unsigned nb = (unsigned)((a.g1.nx / BT) * (a.g1.ny / BT));
    const Op<T, 2> op = make_op<T, 2>(a.h, a.cl), op1 = make_op<T, 2>(2 * a.h, a.cl1);
    if (!a.pre) {
        const T *src = (const T*)a.src, *f = (const T*)a.f, *src1 = (const T*)a.src1, *f1 = (const T*)a.f1,
                *V2 = (const T*)a.V2;
        T *dst = (T*)a.dst, *dst1 = (T*)a.dst1;
        const T cl1 = (T)a.cl1, cl2 = (T)a.cl2;
#define B2POST(NS, LIN)                                                                                             \
    k_blk2_post<T, NS, LIN, BT><<<nb, kB2Threads, b2_post_lds<T, NS, BT>(), s>>>(src, f, dst, src1, f1, dst1, V2, a.g, \
                                                                              a.g1, a.g2, op, op1, cl1, cl2)
        if (a.ns == 1) {
            if (a.linear) B2POST(1, 1); else B2POST(1, 0);
        } else {
            if (a.linear) B2POST(2, 1); else B2POST(2, 0);
        }
#undef B2POST
        return hipGetLastError();
    }
    if (a.ns == 1)
        k_blk2_pre<T, 1, BT><<<nb, kB2Threads, b2_pre_lds<T, 1, BT>(), s>>>(
            (const T*)a.src, (const T*)a.f, (T*)a.dst, (T*)a.f1, (const T*)a.src1, (T*)a.dst1, (T*)a.R, a.g, a.g1, a.g2,
            op, op1);
    else
        k_blk2_pre<T, 2, BT><<<nb, kB2Threads, b2_pre_lds<T, 2, BT>(), s>>>(
            (const T*)a.src, (const T*)a.f, (T*)a.dst, (T*)a.f1, (const T*)a.src1, (T*)a.dst1, (T*)a.R, a.g, a.g1, a.g2,
            op, op1);
    return hipGetLastError();
}

}  // namespace

static_assert(b2_pre_lds<float, 2, 32>() <= 160 * 1024 && b2_post_lds<float, 2, 32>() <= 160 * 1024 &&
                  b2_pre_lds<double, 2, 16>() <= 160 * 1024 && b2_post_lds<double, 2, 16>() <= 160 * 1024,
              "k_blk2 LDS");

// level l (g) and l + 1 (g1) of a 2D box (fp32 or fp64), level l + 2 (g2) below: a tile edge divides level l + 1
bool block2_supported(int rb, int dim, int ns, const Geo& g, const Geo& g1, const Geo& g2)
{
    if ((rb != 4 && rb != 8) || dim != 2 || (ns != 1 && ns != 2)) return false;
    if (g.z0 != 0 || g1.z0 != 0 || g.nz != 1 || g1.nz != 1 || g2.nz != 1) return false;
    if (b2_tile(rb, g1) == 0) return false;
    return g.nx == 2 * g1.nx && g.ny == 2 * g1.ny && g2.nx == g1.nx / 2 && g2.ny == g1.ny / 2;
}

hipError_t blk2_attr(int rb)
{
    auto set = [](const void* k, size_t lds) {
        return hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    };
    return rb == 8 ? b2_each<double>(set) : b2_each<float>(set);
}

hipError_t launch_block2(int rb, int dim, const Block2Args& a, hipStream_t s)
{
    if (!block2_supported(rb, dim, a.ns, a.g, a.g1, a.g2)) return hipErrorInvalidValue;
    if (rb == 8) return b2_launch<double, 16>(a, s);
    return b2_tile(rb, a.g1) == 16 ? b2_launch<float, 16>(a, s) : b2_launch<float, 32>(a, s);
}

}  // namespace mgp
