// gather_ceiling.hip — what random 64-B Occ-bucket fetches can reach on this
// GPU: the access pattern of the seeding kernel (one 64-B bucket per rank,
// uniformly spread over a table far larger than L2 and the Infinity Cache)
// without its dependency chains or state machine.
//
//   hipcc --offload-arch=gfx950 -O3 -o gather_ceiling tools/gather_ceiling.hip
//   ./gather_ceiling [table_MB=1000] [waves_per_cu=12] [iters=2000] [mode]
//
// mode 0: cooperative LDS-DMA (4 lanes x 16 B per bucket, 16 buckets per
//         wave-instruction, 8 instructions = 128 buckets per wave round),
//         the seeding kernel's fetch;
// mode 1: per-lane, 4 x global_load_dwordx4 per bucket, 2 buckets per lane;
// mode 2: mode 0 with 32-B buckets (2 lanes x 16 B);
// mode 3: the cooperative layout through registers (global_load_dwordx4 + ds_write_b128);
// mode 4: per-lane buckets (2 per lane) by LDS-DMA, 4 chunk-planes per bucket;
// mode 5: mode 4 plus argv[8] lane-private cache-hit loads per round;
// mode 6: the Occ64 fetch, 2 random 32-B buckets per lane (2 x 16-B chunks each);
// mode 7: k-mer interval table probes, 2 random 16-B entries per lane (64-bit
//         indices: tables past 64 GB);
// mode 8: argv[6] random 32-B buckets per lane per round into registers, no LDS
//         (gather_regs, below: the occupancy asked for is the occupancy run).
// Every round waits for its data (vmcnt(0)) before the next, like the
// kernel; addresses are independent so only bandwidth/queueing limit it.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

template <int MODE>
__global__ __launch_bounds__(256) void gather(const uint4* __restrict__ tab, uint64_t n_buckets, int iters,
                                              uint32_t* __restrict__ sink, int active, int extra) {
    __shared__ uint4 img[4][256][4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t seed = (blockIdx.x * 4 + w) * 0x9E3779B9u + lane * 0x85EBCA6Bu;
    uint32_t acc = 0;
    for (int it = 0; it < iters; ++it) {
        if (MODE == 1) {
            uint4 a[8];
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                const uint32_t bk = mix(seed + it * 2 + b) % n_buckets;
#pragma unroll
                for (int q = 0; q < 4; ++q) a[b * 4 + q] = tab[(uint64_t)bk * 4 + q];
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) acc ^= a[q].x ^ a[q].w;
        } else if (MODE == 4) {
            // per-lane buckets by LDS-DMA: instruction (b, q) moves chunk q of every
            // lane's bucket b into plane [b*4+q][lane] of the image
            if (lane < active)
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                const uint32_t bk = mix(seed + it * 2 + b) % n_buckets;
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    __builtin_amdgcn_global_load_lds(tab + (uint64_t)bk * 4 + q,
                                                     (__attribute__((address_space(3))) void*)&img[w][(b * 4 + q) * 16][0],
                                                     16, 0, 0);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint4* pl = &img[w][0][0];
            const uint4 v = pl[lane], u = pl[7 * 64 + lane];
            acc ^= v.x ^ u.w;
        } else if (MODE == 6) {
            // the Occ64 fetch: 2 random 32-B buckets per lane, 2 x 16-B chunks each
            if (lane < active)
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                const uint32_t bk = mix(seed + it * 2 + b) % n_buckets;
#pragma unroll
                for (int q = 0; q < 2; ++q)
                    __builtin_amdgcn_global_load_lds(tab + (uint64_t)bk * 2 + q,
                                                     (__attribute__((address_space(3))) void*)&img[w][(b * 2 + q) * 16][0],
                                                     16, 0, 0);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint4* pl = &img[w][0][0];
            const uint4 v = pl[lane], u = pl[3 * 64 + lane];
            acc ^= v.x ^ u.w;
        } else if (MODE == 7) {
            // 2 random 16-B table entries per lane, 64-bit indices
            if (lane < active)
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                const uint32_t h = mix(seed + it * 2 + b);
                const uint64_t e = (((uint64_t)mix(h ^ 0x5bd1e995u) << 32) | h) % n_buckets;
                __builtin_amdgcn_global_load_lds(tab + e, (__attribute__((address_space(3))) void*)&img[w][b * 16][0],
                                                 16, 0, 0);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint4* pl = &img[w][0][0];
            const uint4 v = pl[lane], u = pl[64 + lane];
            acc ^= v.x ^ u.w;
        } else if (MODE == 5) {
            // mode 4 plus `extra` per-lane 16-B LDS-DMA loads from a lane-private
            // 4 KB arena (cache hits), like the list traffic of the seeding kernel
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                const uint32_t bk = mix(seed + it * 2 + b) % n_buckets;
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    __builtin_amdgcn_global_load_lds(tab + (uint64_t)bk * 4 + q,
                                                     (__attribute__((address_space(3))) void*)&img[w][(b * 4 + q) * 16][0],
                                                     16, 0, 0);
            }
            const uint4* arena = tab + ((uint64_t)(blockIdx.x * 256 + threadIdx.x) << 8);
            for (int e = 0; e < extra; ++e)
                __builtin_amdgcn_global_load_lds(arena + ((it * 7 + e) & 255),
                                                 (__attribute__((address_space(3))) void*)&img[w][(8 + (e & 7)) * 16][0], 16, 0, 0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint4* pl = &img[w][0][0];
            const uint4 v = pl[lane], u = pl[7 * 64 + lane];
            acc ^= v.x ^ u.w;
        } else if (MODE == 3) {
            // the cooperative layout through registers: 8 x global_load_dwordx4 + ds_write_b128
            uint4 a[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const uint32_t bk = mix(seed + it * 128 + r * 16 + lane / 4) % n_buckets;
                a[r] = tab[(uint64_t)bk * 4 + (lane % 4)];
            }
#pragma unroll
            for (int r = 0; r < 8; ++r) img[w][r * 16 + lane / 4][lane % 4] = a[r];
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
            const uint4 v = img[w][lane][0];
            acc ^= v.x ^ v.w;
        } else {
            // 128 buckets per wave round; lane l fetches 16 B of bucket (r*16 + l/4)
            const int per = MODE == 2 ? 2 : 4;  // lanes per bucket
            const int nb = 64 / per;            // buckets per instruction
#pragma unroll
            for (int r = 0; r < 128 / nb; ++r) {
                const uint32_t bk = mix(seed + it * 128 + r * nb + lane / per) % n_buckets;
                const uint4* src = MODE == 2 ? tab + (uint64_t)bk * 2 + (lane % per) : tab + (uint64_t)bk * 4 + (lane % per);
                __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)&img[w][r * nb][0], 16, 0, 0);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint4 v = img[w][lane][0];
            acc ^= v.x ^ v.w;
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// mode 8 (round 6): NB random 32-B buckets per lane per round (argv[6], 1..16) into
// registers (2 x global_load_dwordx4 each), no LDS: the other modes' 64-KB LDS image
// allowed at most 2 blocks (8 waves) per CU whatever waves_per_cu asked for, so
// their "12 waves/CU" ceiling ran at 8.  This one runs the asked occupancy and
// the asked memory-level parallelism (waves x lanes x NB outstanding buckets).
template <int NB>
__global__ __launch_bounds__(256) void gather_regs(const uint4* __restrict__ tab, uint64_t n_buckets, int iters,
                                                   uint32_t* __restrict__ sink) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t seed = (blockIdx.x * 4 + w) * 0x9E3779B9u + lane * 0x85EBCA6Bu;
    uint32_t acc = 0;
    for (int it = 0; it < iters; ++it) {
        uint4 a[2 * NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const uint32_t bk = mix(seed + it * NB + b) % n_buckets;
            a[2 * b] = tab[(uint64_t)bk * 2];
            a[2 * b + 1] = tab[(uint64_t)bk * 2 + 1];
        }
#pragma unroll
        for (int b = 0; b < 2 * NB; ++b) acc ^= a[b].x ^ a[b].w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char** argv) {
    const size_t mb = argc > 1 ? atol(argv[1]) : 1000;
    const int wpc = argc > 2 ? atoi(argv[2]) : 12;
    const int iters = argc > 3 ? atoi(argv[3]) : 2000;
    const int mode = argc > 4 ? atoi(argv[4]) : 0;
    const size_t bytes = mb << 20;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    uint4* tab;
    uint32_t* sink;
    // argv[7]: 1 = physically contiguous allocation (hipDeviceMallocContiguous: large TLB fragments)
    if (argc > 7 && atoi(argv[7]) == 1)
        CHECK(hipExtMallocWithFlags((void**)&tab, bytes, hipDeviceMallocContiguous));
    else
        CHECK(hipMalloc(&tab, bytes));
    CHECK(hipMalloc(&sink, 4));
    CHECK(hipMemset(tab, 1, bytes));
    const int bsz = mode == 7 ? 16 : (mode == 2 || mode == 6 || mode == 8) ? 32 : 64;
    // argv[5]: restrict the addresses to the first N buckets (e.g. 256 = L1-resident)
    uint64_t n_buckets = bytes / bsz;
    if (mode != 7 && n_buckets > 0xffffffffull) n_buckets = 0xffffffffull;
    if (argc > 5 && atol(argv[5]) > 0 && (uint64_t)atol(argv[5]) < n_buckets) n_buckets = (uint64_t)atol(argv[5]);
    const int grid = prop.multiProcessorCount * wpc / 4;
    int active = argc > 6 ? atoi(argv[6]) : (mode == 8 ? 2 : 64);  // mode 4: lanes that fetch; mode 8: buckets per lane
    if (active < 1 || active > 64) active = 64;
    const int extra = argc > 8 ? atoi(argv[8]) : 0;  // mode 5: extra lane-private loads per round
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int rep = 0; rep < 3; ++rep) {
        CHECK(hipEventRecord(e0));
        if (mode == 0) hipLaunchKernelGGL(gather<0>, dim3(grid), dim3(256), 0, 0, tab, n_buckets, iters, sink, active, extra);
        if (mode == 1) hipLaunchKernelGGL(gather<1>, dim3(grid), dim3(256), 0, 0, tab, n_buckets, iters, sink, active, extra);
        if (mode == 2) hipLaunchKernelGGL(gather<2>, dim3(grid), dim3(256), 0, 0, tab, n_buckets, iters, sink, active, extra);
        if (mode == 3) hipLaunchKernelGGL(gather<3>, dim3(grid), dim3(256), 0, 0, tab, n_buckets, iters, sink, active, extra);
        if (mode == 4) hipLaunchKernelGGL(gather<4>, dim3(grid), dim3(256), 0, 0, tab, n_buckets, iters, sink, active, extra);
        if (mode == 5) hipLaunchKernelGGL(gather<5>, dim3(grid), dim3(256), 0, 0, tab, n_buckets, iters, sink, active, extra);
        if (mode == 6) hipLaunchKernelGGL(gather<6>, dim3(grid), dim3(256), 0, 0, tab, n_buckets, iters, sink, active, extra);
        if (mode == 7) hipLaunchKernelGGL(gather<7>, dim3(grid), dim3(256), 0, 0, tab, n_buckets, iters, sink, active, extra);
        if (mode == 8) {
            switch (active) {
                case 1: hipLaunchKernelGGL(gather_regs<1>, dim3(grid), dim3(256), 0, 0, tab, n_buckets, iters, sink); break;
                case 2: hipLaunchKernelGGL(gather_regs<2>, dim3(grid), dim3(256), 0, 0, tab, n_buckets, iters, sink); break;
                case 4: hipLaunchKernelGGL(gather_regs<4>, dim3(grid), dim3(256), 0, 0, tab, n_buckets, iters, sink); break;
                case 8: hipLaunchKernelGGL(gather_regs<8>, dim3(grid), dim3(256), 0, 0, tab, n_buckets, iters, sink); break;
                default: hipLaunchKernelGGL(gather_regs<16>, dim3(grid), dim3(256), 0, 0, tab, n_buckets, iters, sink); break;
            }
        }
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double nbk = (double)grid * 4 * iters *
                           (mode == 8 ? 64.0 * (active == 1 || active == 2 || active == 4 || active == 8 ? active : 16)
                                      : (mode == 4 || mode == 6 || mode == 7) ? 2 * active : 128);  // buckets fetched
        printf("{\"table_MB\": %zu, \"waves_per_cu\": %d, \"mode\": %d, \"bucket_B\": %d, \"ms\": %.3f, "
               "\"Gbuckets_per_s\": %.2f, \"TB_per_s\": %.3f, \"active\": %d, \"us_per_round\": %.3f}\n",
               mb, wpc, mode, bsz, ms, nbk / ms * 1e-6, nbk * bsz / ms * 1e-9, active, ms * 1e3 / iters);
    }
    return 0;
}
