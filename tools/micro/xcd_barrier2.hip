// Microbenchmark (not part of the library): barrier forms among the workgroups on XCD 0.
//  A: relaxed agent-scope atomic counter, relaxed polling (no release/acquire fences)
//  B: per-workgroup flag words; every workgroup polls all flags with one vector load (lane k: flag k)
// Bounded spins; timing by HIP events over `rounds` rounds.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ unsigned xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 15u; }

template <int MODE>
__global__ void k_bar(unsigned* ctr, unsigned* flags, unsigned* tickets, unsigned* flag, int rounds, int want)
{
    __shared__ unsigned my;
    __shared__ int go;
    if (threadIdx.x == 0) {
        go = 0;
        if (xcc_id() == 0) {
            my = atomicAdd(tickets, 1u);
            go = my < (unsigned)want;
        }
    }
    __syncthreads();
    if (!go) return;
    for (int r = 1; r <= rounds; ++r) {
        __syncthreads();
        if (MODE == 0) {
            if (threadIdx.x == 0) {
                __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                long spins = 0;
                while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)(r * want)) {
                    if (++spins > 20000000) { *flag = 1; break; }
                }
            }
        } else {
            if (threadIdx.x < 64) {
                if (threadIdx.x == 0) __hip_atomic_store(flags + my, (unsigned)r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                long spins = 0;
                while (true) {
                    const unsigned v = threadIdx.x < (unsigned)want
                                           ? __hip_atomic_load(flags + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                           : (unsigned)r;
                    if (__all(v >= (unsigned)r)) break;
                    if (++spins > 20000000) { *flag = 1; break; }
                }
            }
        }
        __syncthreads();
    }
}

int main(int argc, char** argv)
{
    const int rounds = argc > 1 ? atoi(argv[1]) : 1000;
    unsigned *ctr, *flags, *tickets, *flag;
    (void)hipMalloc(&ctr, 4); (void)hipMalloc(&flags, 256); (void)hipMalloc(&tickets, 4); (void)hipMalloc(&flag, 4);
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    for (int mode = 0; mode < 2; ++mode)
        for (int want : {1, 8, 16, 24, 32}) {
            (void)hipMemset(ctr, 0, 4); (void)hipMemset(flags, 0, 256); (void)hipMemset(tickets, 0, 4); (void)hipMemset(flag, 0, 4);
            (void)hipEventRecord(a);
            if (mode == 0) k_bar<0><<<256, 256>>>(ctr, flags, tickets, flag, rounds, want);
            else k_bar<1><<<256, 256>>>(ctr, flags, tickets, flag, rounds, want);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms = 0; (void)hipEventElapsedTime(&ms, a, b);
            unsigned f = 0, t = 0;
            (void)hipMemcpy(&f, flag, 4, hipMemcpyDeviceToHost); (void)hipMemcpy(&t, tickets, 4, hipMemcpyDeviceToHost);
            printf("%s participants %2d (XCD-0 WGs %u): %.3f us/round, timeout %u\n", mode ? "flags  " : "counter", want, t,
                   1e3 * ms / rounds, f);
        }
    return 0;
}
