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

#include <type_traits>

namespace mgp {
namespace {

// fine tile of a workgroup (even, so that a tile's coarse cells are whole) and its threads: one coarse cell each
template <int DIM>
struct FwShape {
#ifndef FW_TX
#define FW_TX 64
#endif
#ifndef FW_TY3
#define FW_TY3 16
#endif
    static constexpr int TX = FW_TX, TY = DIM == 3 ? FW_TY3 : 32;
    static constexpr int NT = (TX / 2) * (TY / 2);         // 256 (3D) / 512 (2D) threads at 64 x 16 / 64 x 32
    static constexpr int UW = TX + 4, UH = TY + 4;         // u staged with 2 cells of halo per side
    static constexpr int RW = TX + 2, RH = TY + 2;         // r with one
    static constexpr int USLOT = UW * UH, RSLOT = RW * RH;
    static constexpr int NU = DIM == 3 ? 3 : 1;            // u planes in the ring (k - 1, k, k + 1)
    static constexpr int MW = TX / 2 + 2;                  // packed cells of one colour per staged row
};

// A thread's share of the staging of one u plane (both colours, cells X0-2 .. X0+TX+1, Y0-2 .. Y0+TY+1, zero outside
// the box; runs of one colour's packed row per wave, coalesced) and of the residual ring: fixed items, so the
// in-plane addressing is computed once and each plane's loads are issued a step ahead of their use.
template <int DIM>
struct FwItems {
    using S = FwShape<DIM>;
    static constexpr int NUI = 2 * S::UH * S::MW, IU = (NUI + S::NT - 1) / S::NT;  // u items per thread
    static constexpr int IR = (S::RSLOT + S::NT - 1) / S::NT;                      // r cells per thread
};

template <typename T, int DIM>
__global__ __launch_bounds__(FwShape<DIM>::NT) void k_resfw(const T* __restrict__ u, const T* __restrict__ f,
                                                            T* __restrict__ R, Geo g, Geo gc, Op<T, DIM> op, T wf,
                                                            int kc, int gz)
{
    using S = FwShape<DIM>;
    using I = FwItems<DIM>;
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
    const int Ic = X0 / 2 + Il, Jc = Y0 / 2 + Jl;
    const T w3 = (T)3;
    const T wbx = Ic == 0 ? wf : w3, wcx = Ic == cx - 1 ? wf : w3;
    const T wby = Jc == 0 ? wf : w3, wcy = Jc == cy - 1 ? wf : w3;

    // u items: in-plane packed offset (colour c's row j at m) and the LDS cell of each of the two plane parities
    // (the x parity of colour c's cells in row j flips with the plane); -1 = outside the box (stays 0)
    int uoff[I::IU], ul0[I::IU], ul1[I::IU];
#pragma unroll
    for (int e = 0; e < I::IU; ++e) {
        const int q = tid + e * S::NT;
        const int mm = q % S::MW, c = (q / S::MW) & 1, jl = q / (2 * S::MW);
        const int j = Y0 - 2 + jl, m = X0 / 2 - 1 + mm;
        const int par0 = (int)((c + j + g.z0) & 1);  // x parity of colour c's cells in row j at even local planes
        const bool ok = q < I::NUI && j >= 0 && j < g.ny && m >= 0 && m < g.hw;
        uoff[e] = ok ? (int)(c * g.H + (int64_t)j * g.hw + m) : -1;
        const int i0 = 2 * m + par0, i1 = 2 * m + (par0 ^ 1);
        ul0[e] = q < I::NUI && i0 - (X0 - 2) >= 0 && i0 - (X0 - 2) < S::UW ? jl * S::UW + i0 - (X0 - 2) : -1;
        ul1[e] = q < I::NUI && i1 - (X0 - 2) >= 0 && i1 - (X0 - 2) < S::UW ? jl * S::UW + i1 - (X0 - 2) : -1;
    }
    // r cells: in-plane packed offset of f (colour parity of even local planes), box face count, inside the box
    int foff[I::IR], fpar[I::IR], fnb[I::IR];
#pragma unroll
    for (int e = 0; e < I::IR; ++e) {
        const int q = tid + e * S::NT;
        const int il = q % S::RW, jl = q / S::RW;
        const int i = X0 - 1 + il, j = Y0 - 1 + jl;
        const bool in = q < S::RSLOT && i >= 0 && i < g.nx && j >= 0 && j < g.ny;
        foff[e] = in ? (int)((int64_t)j * g.hw + (i >> 1)) : -1;
        fpar[e] = (int)((i + j + g.z0) & 1);
        fnb[e] = (i == 0) + (i == g.nx - 1) + (j == 0) + (j == g.ny - 1);
    }
    auto uload = [&](T (&v)[I::IU], int64_t k) {
        const bool readable = DIM == 2 || (k >= -gz && k < g.nz + gz);
        const T* up = u + k * g.P;
#pragma unroll
        for (int e = 0; e < I::IU; ++e) v[e] = readable && uoff[e] >= 0 ? up[uoff[e]] : (T)0;
    };
    auto ustore = [&](T* dst, const T (&v)[I::IU], int64_t k) {
        const bool odd = ((k & 1) != 0);
#pragma unroll
        for (int e = 0; e < I::IU; ++e) {
            const int x = odd ? ul1[e] : ul0[e];
            if (x >= 0) dst[x] = v[e];
        }
    };
    auto fload = [&](T (&v)[I::IR], int64_t k) {
        const int64_t gk = g.z0 + k;
        const bool kin = DIM == 2 || (gk >= 0 && gk < g.gnz);
        const T* fp = f + k * g.P;
        const int kp = (int)(k & 1);
#pragma unroll
        for (int e = 0; e < I::IR; ++e) v[e] = kin && foff[e] >= 0 ? fp[((fpar[e] ^ kp) * g.H) + foff[e]] : (T)0;
    };
    // r of local plane k on the tile and its one-cell ring into rs (0 outside the box), then my cell's `ay`
    auto plane_ay = [&](int64_t k, const T* um, const T* uc, const T* up, const T (&fv)[I::IR]) -> T {
        const int64_t gk = g.z0 + k;
        const bool kin = DIM == 2 || (gk >= 0 && gk < g.gnz);
        const int nbz = DIM == 3 ? (gk == 0) + (gk == g.gnz - 1) : 0;
#pragma unroll
        for (int e = 0; e < I::IR; ++e) {
            const int q = tid + e * S::NT;
            if (q < S::RSLOT) {
                T r = (T)0;
                if (kin && foff[e] >= 0) {
                    const int il = q % S::RW, jl = q / S::RW;
                    const int x = (jl + 1) * S::UW + (il + 1);  // in the staged planes
                    T sm = uc[x - 1] + uc[x + 1];
                    sm = sm + uc[x - S::UW];
                    sm = sm + uc[x + S::UW];
                    if (DIM == 3) {
                        sm = sm + um[x];
                        sm = sm + up[x];
                    }
                    r = op.residual(sm, fv[e], uc[x], fnb[e] + nbz);
                }
                rs[q] = r;
            }
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
        T uv[I::IU], fv[I::IR];
        uload(uv, 0);
        fload(fv, 0);
        ustore(us[0], uv, 0);
        __syncthreads();
        const T ay = plane_ay(0, us[0], us[0], us[0], fv);
        R[((Ic + Jc) & 1) * gc.H + (int64_t)Jc * gc.hw + (Ic >> 1)] = scale * ay;
        return;
    } else {
        // ring slot of local plane k: (k + 6) mod 3 (k >= -3)
        auto slot = [&](int64_t k) { return us[(int)((k + 6) % 3)]; };
        const int64_t k0 = 2 * (int64_t)K0 - 1;  // the chunk's first fine plane
        const int kend = K0 + kc < (int)(g.nz >> 1) ? K0 + kc : (int)(g.nz >> 1);
        const int64_t klast = 2 * (int64_t)kend;  // the last fine plane (2 K + 2 of the last coarse plane)
        // plane k + 1's u (loaded during step k - 1) goes into its slot at the top of step k; f of plane k was loaded
        // during step k - 1 into the other of two buffers (a prefetch distance of 2 with double buffers measured slower:
        // 134 VGPRs, 3 workgroups per CU, 609 against 470 us at 512^3).  The step is unrolled by two so that the buffers
        // swap roles without a copy: copying the prefetched f at the end of a step made it wait for those loads there.
        T uv[I::IU], fa[I::IR], fb[I::IR];
        uload(uv, k0 - 1);
        ustore(slot(k0 - 1), uv, k0 - 1);
        uload(uv, k0);
        ustore(slot(k0), uv, k0);
        uload(uv, k0 + 1);  // in flight into the first step
        fload(fa, k0);
        T a0 = (T)0, a1 = (T)0, a2 = (T)0, a3 = (T)0;
        int K = K0;
        auto step = [&](int64_t k, const T (&fc)[I::IR], T (&fnx)[I::IR]) {
            ustore(slot(k + 1), uv, k + 1);
            if (k + 2 <= klast + 1) uload(uv, k + 2);
            if (k + 1 <= klast) fload(fnx, k + 1);
            __syncthreads();
            // (plane_ay's barrier also frees slot k - 1, restaged next step, and every read of rs precedes the next
            // step's first barrier: no barrier at the end of a step)
            const T ay = plane_ay(k, slot(k - 1), slot(k), slot(k + 1), fc);
            a0 = a1;
            a1 = a2;
            a2 = a3;
            a3 = ay;
            if (k == 2 * (int64_t)K + 2) {  // coarse plane K complete (fine planes 2K-1 .. 2K+2)
                const int64_t gK = gc.z0 + K;
                T az = a0;
                az = az + (gK == 0 ? wf : w3) * a1;
                az = az + (gK == gc.gnz - 1 ? wf : w3) * a2;
                az = az + a3;
                R[(int64_t)K * gc.P + ((Ic + Jc + gK) & 1) * gc.H + (int64_t)Jc * gc.hw + (Ic >> 1)] = scale * az;
                ++K;
            }
        };
        for (int64_t k = k0; k <= klast; k += 2) {
            step(k, fa, fb);
            if (k + 1 <= klast) step(k + 1, fb, fa);
        }
    }
}

#ifndef FW_KMIN  // (build knob: the smallest z-chunk in coarse planes; 128^3 -> 64^3: 39 -> 18.6 us at 2 against 8)
#define FW_KMIN 2
#endif
#ifndef FW_WGS  // (build knob: workgroups the z-chunking aims for; 512^3 FW cycle 1.600 ms at 1024, 1.620 at 2048, 1.639 at 4096)
#define FW_WGS 1024
#endif
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
        while (tiles * (cz / kc) < FW_WGS && kc >= 2 * FW_KMIN) kc /= 2;
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
    const int tx = FwShape<3>::TX, ty = dim == 3 ? FwShape<3>::TY : FwShape<2>::TY;
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
