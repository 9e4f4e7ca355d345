// Microbenchmark (not part of the library): cost of a workgroup barrier among the workgroups that run
// on ONE XCD, with the counter in that XCD's L2, versus the chip-wide kernel-launch floor.
// Every workgroup reads its XCC id; those on XCD 0 take a ticket and run `rounds` barrier rounds
// (one lane: atomic add, then poll with agent-scope loads until all participants arrived); spins are
// bounded, so a broken protocol ends with an error flag instead of a hang.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ unsigned xcc_id()
{
    // s_getreg_b32 HW_REG_XCC_ID (id 20 on gfx940+), bits [3:0]
    return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 15u;
}

__global__ void k_bar(unsigned* ctr, unsigned* tickets, unsigned* flag, long long* out, int rounds, int want)
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
    const long long t0 = (long long)__builtin_amdgcn_s_memtime();
    for (int r = 1; r <= rounds; ++r) {
        __syncthreads();
        if (threadIdx.x == 0) {
            __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned target = (unsigned)(r * want);
            long spins = 0;
            while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
                if (++spins > 20000000) { *flag = 1; break; }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __syncthreads();
    }
    const long long t1 = (long long)__builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) out[my] = t1 - t0;
}

__global__ void k_empty(float* p) { if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1.0f; }

int main(int argc, char** argv)
{
    const int rounds = argc > 1 ? atoi(argv[1]) : 1000;
    unsigned *ctr, *tickets, *flag;
    long long* out;
    float* p;
    hipMalloc(&ctr, 4); hipMalloc(&tickets, 4); hipMalloc(&flag, 4); hipMalloc(&out, 64 * 8); hipMalloc(&p, 4);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int want : {1, 4, 8, 16, 24}) {
        hipMemset(ctr, 0, 4); hipMemset(tickets, 0, 4); hipMemset(flag, 0, 4); hipMemset(out, 0, 64 * 8);
        hipEventRecord(a);
        k_bar<<<256, 256>>>(ctr, tickets, flag, out, rounds, want);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0; hipEventElapsedTime(&ms, a, b);
        unsigned f = 0, t = 0; long long o[64];
        hipMemcpy(&f, flag, 4, hipMemcpyDeviceToHost); hipMemcpy(&t, tickets, 4, hipMemcpyDeviceToHost);
        hipMemcpy(o, out, 64 * 8, hipMemcpyDeviceToHost);
        printf("participants %2d (XCD-0 workgroups %u): %d rounds in %.3f ms = %.3f us/round, memtime ticks/round %.1f, timeout %u\n",
               want, t, rounds, ms, 1e3 * ms / rounds, (double)o[0] / rounds, f);
    }
    // launch floor: back-to-back tiny kernels in one stream
    const int K = 2000;
    hipEventRecord(a);
    for (int i = 0; i < K; ++i) k_empty<<<16, 256>>>(p);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0; hipEventElapsedTime(&ms, a, b);
    printf("empty kernel back to back: %.3f us each\n", 1e3 * ms / K);
    return 0;
}
