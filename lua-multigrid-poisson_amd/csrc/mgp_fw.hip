// mgp_fw.hip — calcResidual + the full-weighting restriction in one z-streamed pass (k_resfw).
//
// The full weighting (mgp_opts.restriction = MGP_RESTRICT_FULL_WEIGHTING, the north star's "full-weighting
// restriction") reads the residuals of the 4 x 4 (x 4) fine cells 2I-1 .. 2I+2 around each coarse cell, so the
// per-piece path materialised r once per level (k_resfield_v: read u, f, write r) and then restricted it
// (k_fw_v: read r, write R): 3 + 1 + 2^-d reals per fine cell, 0.55 ms of a 512^3 fp32 cycle (round-4 trace:
// 353 + 201 us).  Here a workgroup owns a TX x TY tile of fine cells (TX/2 x TY/2 coarse cells) and streams a
// chunk of coarse planes through z: per fine plane it stages u (both colours, unpacked, zero outside the box)
// in an LDS ring of three planes, evaluates r on the tile plus a one-cell ring into LDS, and reduces r along x
// and y to the coarse cells (fw_axis, then the y accumulation: fw_eval's `ay`); four consecutive `ay` planes give
// one coarse plane (fw_eval's `az`).  Per fine cell it reads u and f once (+ the tile halos, mostly from L2) and
// writes R / 2^d: 2 + 2^-d reals.  Every expression and its order is residual_at's / fw_eval's (mgp_kernels.hip),
// so R is bit-identical to the two-pass path and to the oracle (restrict_fw in oracle/mgp_oracle_impl.h).
#include "mgp_device.h"

namespace mgp {
namespace {

// fine tile of a workgroup (even, so that a tile's coarse cells are whole) and its threads: one coarse cell each
template <int DIM>
struct FwShape {
    static constexpr int TX = 64, TY = DIM == 3 ? 16 : 32;
    static constexpr int NT = (TX / 2) * (TY / 2);         // 256 (3D) / 512 (2D) threads
    static constexpr int UW = TX + 4, UH = TY + 4;         // u staged with 2 cells of halo per side
    static constexpr int RW = TX + 2, RH = TY + 2;         // r with one
    static constexpr int USLOT = UW * UH, RSLOT = RW * RH;
    static constexpr int NU = DIM == 3 ? 3 : 1;            // u planes in the ring (k - 1, k, k + 1)
    static constexpr int MW = TX / 2 + 2;                  // packed cells of one colour per staged row
};

// Stage u of local plane k (both colours, cells X0-2 .. X0+TX+1, Y0-2 .. Y0+TY+1, zero outside the box or the
// readable planes) into `dst`, unpacked: a thread reads runs of one colour's packed row (coalesced).
template <typename T, int DIM>
__device__ __forceinline__ void fw_stage(T* dst, const T* __restrict__ u, const Geo& g, int64_t k, int X0, int Y0,
                                         int gz, int tid)
{
    using S = FwShape<DIM>;
    const int64_t gk = g.z0 + k;
    const bool readable = DIM == 2 || (k >= -gz && k < g.nz + gz);
    const int m0 = X0 / 2 - 1;
    for (int q = tid; q < 2 * S::UH * S::MW; q += S::NT) {
        const int mm = q % S::MW, c = (q / S::MW) & 1, jl = q / (2 * S::MW);
        const int j = Y0 - 2 + jl, m = m0 + mm;
        const int par = (int)((c + j + gk) & 1);  // x parity of colour c's cells in row j
        const int i = 2 * m + par;
        T v = (T)0;
        if (readable && j >= 0 && j < g.ny && m >= 0 && m < g.hw && i < g.nx)
            v = u[k * g.P + c * g.H + (int64_t)j * g.hw + m];
        const int il = i - (X0 - 2);
        if (il >= 0 && il < S::UW) dst[jl * S::UW + il] = v;
    }
}

template <typename T, int DIM>
__global__ __launch_bounds__(FwShape<DIM>::NT) void k_resfw(const T* __restrict__ u, const T* __restrict__ f,
                                                            T* __restrict__ R, Geo g, Geo gc, Op<T, DIM> op, T wf,
                                                            int kc, int gz)
{
    using S = FwShape<DIM>;
    __shared__ T us[S::NU][S::USLOT];
    __shared__ T rs[S::RSLOT];
    const int tid = threadIdx.x;
    const int tiles_x = g.nx / S::TX, tiles_y = g.ny / S::TY;
    const int b = xcd_remap(blockIdx.x, gridDim.x);
    const int tx = b % tiles_x, ty = (b / tiles_x) % tiles_y;
    const int K0 = (b / (tiles_x * tiles_y)) * kc;  // first coarse plane (local) of this chunk
    const int X0 = tx * S::TX, Y0 = ty * S::TY;
    const int cx = g.nx >> 1, cy = g.ny >> 1;
    // my coarse cell and its weights (fw_eval's wb / wc per axis)
    const int Il = tid % (S::TX / 2), Jl = tid / (S::TX / 2);
    const int I = X0 / 2 + Il, J = Y0 / 2 + Jl;
    const T w3 = (T)3;
    const T wbx = I == 0 ? wf : w3, wcx = I == cx - 1 ? wf : w3;
    const T wby = J == 0 ? wf : w3, wcy = J == cy - 1 ? wf : w3;

    // r of local plane k on the tile and its one-cell ring into rs (0 outside the box), then my cell's `ay`
    auto plane_ay = [&](int64_t k, const T* um, const T* uc, const T* up) -> T {
        const int64_t gk = g.z0 + k;
        const bool kin = DIM == 2 || (gk >= 0 && gk < g.gnz);
        for (int q = tid; q < S::RSLOT; q += S::NT) {
            const int il = q % S::RW, jl = q / S::RW;
            const int i = X0 - 1 + il, j = Y0 - 1 + jl;
            T r = (T)0;
            if (kin && i >= 0 && i < g.nx && j >= 0 && j < g.ny) {
                const int x = (jl + 1) * S::UW + (il + 1);  // in the staged planes
                T s = uc[x - 1] + uc[x + 1];
                s = s + uc[x - S::UW];
                s = s + uc[x + S::UW];
                if (DIM == 3) {
                    s = s + um[x];
                    s = s + up[x];
                }
                const int nb = (i == 0) + (i == g.nx - 1) + (j == 0) + (j == g.ny - 1) +
                               (DIM == 3 ? (gk == 0) + (gk == g.gnz - 1) : 0);
                r = op.residual(s, f[pidx(g, i, j, k)], uc[x], nb);
            }
            rs[q] = r;
        }
        __syncthreads();
        T ay = (T)0;
#pragma unroll
        for (int dy = 0; dy < 4; ++dy) {
            const T* row = rs + (2 * Jl + dy) * S::RW + 2 * Il;  // fine rows 2J-1 .. 2J+2, cells 2I-1 .. 2I+2
            const T ax = fw_axis(row[0], row[1], row[2], row[3], wbx, wcx);
            if (dy == 0) ay = ax;
            else if (dy == 1) ay = ay + wby * ax;
            else if (dy == 2) ay = ay + wcy * ax;
            else ay = ay + ax;
        }
        return ay;
    };
    const T scale = DIM == 3 ? (T)(1.0 / 512.0) : (T)(1.0 / 64.0);
    if constexpr (DIM == 2) {
        fw_stage<T, 2>(us[0], u, g, 0, X0, Y0, gz, tid);
        __syncthreads();
        const T ay = plane_ay(0, us[0], us[0], us[0]);
        const int pc = J & 1;
        R[((I + pc) & 1) * gc.H + (int64_t)J * gc.hw + (I >> 1)] = scale * ay;
        return;
    } else {
        // ring slot of local plane k: (k + 3) mod 3 (k >= -2)
        auto slot = [&](int64_t k) { return us[(int)((k + 6) % 3)]; };
        const int64_t k0 = 2 * (int64_t)K0 - 1;  // the chunk's first fine plane
        fw_stage<T, 3>(slot(k0 - 1), u, g, k0 - 1, X0, Y0, gz, tid);
        fw_stage<T, 3>(slot(k0), u, g, k0, X0, Y0, gz, tid);
        T a0 = (T)0, a1 = (T)0, a2 = (T)0, a3 = (T)0;
        const int kend = K0 + kc < (int)(g.nz >> 1) ? K0 + kc : (int)(g.nz >> 1);
        for (int K = K0; K < kend; ++K) {
            // fine planes 2K-1 .. 2K+2 (the first coarse plane of the chunk computes all four, the others two)
            for (int64_t k = K == K0 ? 2 * (int64_t)K - 1 : 2 * (int64_t)K + 1; k <= 2 * (int64_t)K + 2; ++k) {
                fw_stage<T, 3>(slot(k + 1), u, g, k + 1, X0, Y0, gz, tid);
                __syncthreads();
                const T ay = plane_ay(k, slot(k - 1), slot(k), slot(k + 1));
                a0 = a1;
                a1 = a2;
                a2 = a3;
                a3 = ay;
                __syncthreads();  // rs and the ring slot about to be restaged are free again
            }
            const int64_t gK = gc.z0 + K;
            T az = a0;
            az = az + (gK == 0 ? wf : w3) * a1;
            az = az + (gK == gc.gnz - 1 ? wf : w3) * a2;
            az = az + a3;
            const int pc = (int)((J + gK) & 1);
            R[(int64_t)K * gc.P + ((I + pc) & 1) * gc.H + (int64_t)J * gc.hw + (I >> 1)] = scale * az;
        }
    }
}

template <typename T, int DIM>
hipError_t resfw_t(const void* u, const void* f, void* R, Geo g, Geo gc, double h, double cl, double clc, int gz,
                   hipStream_t s)
{
    using S = FwShape<DIM>;
    const Op<T, DIM> op = make_op<T, DIM>(h, cl);
    const T wf = (T)3 - (T)clc;
    const int64_t tiles = (int64_t)(g.nx / S::TX) * (g.ny / S::TY);
    int kc = 1, chunks = 1;
    if (DIM == 3) {
        const int cz = (int)(g.nz >> 1);
        // coarse planes per chunk: halve while there are fewer than 2048 workgroups (8 per CU) and a chunk keeps
        // >= 8 coarse planes (a chunk re-reads 2 of every 2 kc + 2 fine planes of its neighbours)
        kc = cz;
        while (tiles * (cz / kc) < 2048 && kc >= 16) kc /= 2;
        chunks = (cz + kc - 1) / kc;
    }
    const int64_t nb = tiles * chunks;
    k_resfw<T, DIM><<<(unsigned)nb, S::NT, 0, s>>>((const T*)u, (const T*)f, (T*)R, g, gc, op, wf, kc, gz);
    return hipGetLastError();
}

}  // namespace

bool resfw_supported(int rb, int dim, const Geo& g, int gz, bool dist)
{
    if (rb != 4 && rb != 8) return false;  // (the cpu-raw float arithmetic keeps the two scalar passes)
    const int tx = 64, ty = dim == 3 ? FwShape<3>::TY : FwShape<2>::TY;
    if (g.nx % tx || g.ny % ty) return false;
    if (dim == 3 && ((g.nz & 1) || g.nz < 2)) return false;
    // a slab level reads r at the neighbours' first planes: u two and f one ghost plane deep
    return !dist || gz >= 2;
}

hipError_t launch_resfw(int rb, int dim, const void* u, const void* f, void* R, Geo g, Geo gc, double h, double cl,
                        double clc, int gz, hipStream_t s)
{
    if (rb == 8)
        return dim == 3 ? resfw_t<double, 3>(u, f, R, g, gc, h, cl, clc, gz, s)
                        : resfw_t<double, 2>(u, f, R, g, gc, h, cl, clc, gz, s);
    return dim == 3 ? resfw_t<float, 3>(u, f, R, g, gc, h, cl, clc, gz, s)
                    : resfw_t<float, 2>(u, f, R, g, gc, h, cl, clc, gz, s);
}

}  // namespace mgp
