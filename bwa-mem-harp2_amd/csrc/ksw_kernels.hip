// SW extension on gfx950: ksw_extend2
// (software/ksw.c:379-476), the banded affine-gap extension mem_chain2aln
// runs left and right of every seed it keeps (software/bwamem.c:1136, 1164).
//
// One wave per extension problem; the wave walks the target rows in order
// (each row depends on the last) and its 64 lanes hold the query columns
// j = 64 c + lane, c < KC, in registers: per column the previous row's H one
// column to the left and this row's E -- the reference's column array -- plus
// the column's scores for the five target symbols.  Inside a row the serial
// loop carries F from column to column; here
//     F(j) = max(0, max_{beg <= k < j} D(k) - oe_ins - (j - 1 - k) e_ins),
//     D(k) = max(H(i-1, k-1) + s(k), E(i, k)),
// which is what the serial recurrence gives (an F-derived H never restarts a
// better F, since a restart pays o_ins again), so a prefix max of
// D(k) + k e_ins across the lanes replaces it.  The row maximum (its last
// column on ties), the to-end score, z-drop and the band refit follow the
// serial code step by step with wave reductions and ballots, so every output
// (score, qle, tle, gtle, gscore, max_off) is the reference's.
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>

#include "ksw_kernels.h"
#include "ksw_device.h"
#include "ksw_lane.h"

namespace smem {

__device__ __forceinline__ int imax(int a, int b) { return a > b ? a : b; }

// one problem per wave (kswd::extend_wave), columns per lane by its query
// length (64 KC - 1 columns)
__global__ __launch_bounds__(256) void ksw_extend_kernel(KswParams K) {
    const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int n_waves = (int)((gridDim.x * blockDim.x) >> 6);
    int top = 0;  // the largest matrix entry (from 0), software/ksw.c:398-400
    for (int k = 0; k < 25; ++k) top = imax(top, (int)K.mat[k]);
    for (int it = wave; it < K.n; it += n_waves) {
        const KswTask T = K.task[it];
        const uint8_t* q = K.q + T.q_off;
        const uint8_t* tg = K.t + T.t_off;
        const kswd::ExtIn E{T.qlen, T.tlen, T.w, T.end_bonus, T.zdrop, T.h0};
        auto qf = [&](int j) { return (int)q[j]; };
        auto tf = [&](int i) { return (int)tg[i]; };
        const int ql = __builtin_amdgcn_readfirstlane(T.qlen);
        KswResult r;
        if (ql < 64) r = kswd::extend_wave<1>(E, qf, tf, K.mat, K.o_del, K.e_del, K.o_ins, K.e_ins, top);
        else if (ql < 128) r = kswd::extend_wave<2>(E, qf, tf, K.mat, K.o_del, K.e_del, K.o_ins, K.e_ins, top);
        else r = kswd::extend_wave<KSW_COLS_PER_LANE>(E, qf, tf, K.mat, K.o_del, K.e_del, K.o_ins, K.e_ins, top);
        if ((threadIdx.x & 63) == 0) K.out[it] = r;
    }
}

// four problems per wave on 16-lane groups (kswd::extend_group16)
__global__ __launch_bounds__(256) void ksw_extend_g16_kernel(KswParams K) {
    const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int n_waves = (int)((gridDim.x * blockDim.x) >> 6);
    const int g = (threadIdx.x >> 4) & 3;
    int top = 0;
    for (int k = 0; k < 25; ++k) top = imax(top, (int)K.mat[k]);
    for (int base = wave * 4; base < K.n; base += n_waves * 4) {
        const int it = base + g;
        const bool active = it < K.n;
        const KswTask T = K.task[active ? it : base];
        const uint8_t* q = K.q + T.q_off;
        const uint8_t* tg = K.t + T.t_off;
        // columns per lane by the longest query of the wave's four problems
        int ql = active ? T.qlen : 0;
        ql = imax(ql, __shfl_xor(ql, 16));
        ql = imax(ql, __shfl_xor(ql, 32));
        ql = __builtin_amdgcn_readfirstlane(ql);
        const kswd::ExtIn E{T.qlen, T.tlen, T.w, T.end_bonus, T.zdrop, T.h0};
        auto qf = [&](int j) { return (int)q[j]; };
        auto tf = [&](int i) { return (int)tg[i]; };
        KswResult r;
        if (ql < 32) r = kswd::extend_group16<2>(E, active, qf, tf, K.mat, K.o_del, K.e_del, K.o_ins, K.e_ins, top);
        else if (ql < 64) r = kswd::extend_group16<4>(E, active, qf, tf, K.mat, K.o_del, K.e_del, K.o_ins, K.e_ins, top);
        else if (ql < 128) r = kswd::extend_group16<8>(E, active, qf, tf, K.mat, K.o_del, K.e_del, K.o_ins, K.e_ins, top);
        else r = kswd::extend_group16<16>(E, active, qf, tf, K.mat, K.o_del, K.e_del, K.o_ins, K.e_ins, top);
        if (active && (threadIdx.x & 15) == 0) K.out[it] = r;
    }
}

// One problem per lane (kswl::lane_engine) over a tier of the tasks sorted
// by query length (ksw_tier_*): the tier's problems are those with
// qlen <= KCOL (and past the tier below); the ones the lanes cannot take
// (scores past 16 bits) and queries past 128 columns run one per wave
// (ksw_extend_rest_kernel).
struct KswLanePol {
    const KswParams* K;
    const uint32_t* order;  // the tier's tasks
    uint8_t* rest;          // [n] 1: left to one wave per problem
    int top;
    int it = 0;
    const uint8_t* tg = nullptr;
    template <int KCOL>
    __device__ __forceinline__ bool start(uint32_t k, kswd::ExtIn& T, uint2* qs) {
        it = (int)order[k];
        const KswTask U = K->task[it];
        if (!kswl::extend_lane_ok(KCOL, U.qlen, U.h0, top)) {
            rest[it] = 1;
            return false;
        }
        T = kswd::ExtIn{U.qlen, U.tlen, U.w, U.end_bonus, U.zdrop, U.h0};
        kswl::load_query_fwd<KCOL>(qs, K->q + U.q_off, U.qlen);
        tg = K->t + U.t_off;
        return true;
    }
    __device__ __forceinline__ int tsym(int i) const { return (int)tg[i]; }
    __device__ __forceinline__ bool finish(const KswResult& r, kswd::ExtIn&) {
        K->out[it] = r;
        return false;
    }
};

// ctr: [0] tasks per bucket... (see smem_launch_ksw): the sorted order and the
// tier bounds
struct KswSort {
    uint32_t* hist;    // [KSW_BUCKETS] counts, then cursors
    uint32_t* bounds;  // [10]: queue q = [bounds[q], bounds[q + 1]) of order: query lengths 16q + 1 .. 16q + 16
                       // (q = 0 also 0), q = 0..7
    uint32_t* heads;   // [8] claim counters
    uint32_t* order;   // [n]
    uint8_t* rest;     // [n]
    unsigned long long* stats;  // diagnostics (SMEM_KSW_LANE_STATS): [3 tiers][8], or nullptr
};
constexpr int KSW_BUCKETS = 130;  // query lengths 0..128, longer

__device__ __forceinline__ int ksw_bucket(int qlen) { return qlen <= 128 ? qlen : 129; }

__global__ __launch_bounds__(256) void ksw_hist_kernel(KswParams K, KswSort S) {
    for (int it = blockIdx.x * blockDim.x + threadIdx.x; it < K.n; it += gridDim.x * blockDim.x) {
        atomicAdd(&S.hist[ksw_bucket(K.task[it].qlen)], 1u);
        S.rest[it] = 0;
    }
}

// exclusive scan of the buckets (one block) and the 16-column queues; the
// tiers take queues 0-1 (KCOL 32), 2-3 (64), 4-7 (128)
__global__ __launch_bounds__(256) void ksw_scan_kernel(KswSort S) {
    __shared__ uint32_t c[KSW_BUCKETS + 1];
    if (threadIdx.x == 0) {
        uint32_t a = 0;
        for (int b = 0; b < KSW_BUCKETS; ++b) {
            c[b] = a;
            a += S.hist[b];
        }
        c[KSW_BUCKETS] = a;
        S.bounds[0] = 0;
        for (int q = 1; q <= 8; ++q) S.bounds[q] = c[16 * q + 1];
        for (int q = 0; q < 8; ++q) S.heads[q] = 0;
    }
    __syncthreads();
    for (int b = threadIdx.x; b < KSW_BUCKETS; b += blockDim.x) S.hist[b] = c[b];
}

__global__ __launch_bounds__(256) void ksw_scatter_kernel(KswParams K, KswSort S) {
    for (int it = blockIdx.x * blockDim.x + threadIdx.x; it < K.n; it += gridDim.x * blockDim.x) {
        const int b = ksw_bucket(K.task[it].qlen);
        const uint32_t at = atomicAdd(&S.hist[b], 1u);
        S.order[at] = (uint32_t)it;
        if (b == 129) S.rest[it] = 1;
    }
}

template <int KCOL>
__global__ __launch_bounds__(256, KCOL > 64 ? 2 : 4) void ksw_lane_kernel(KswParams K, KswSort S) {
    __shared__ uint32_t stab[10];  // the five target symbols' row scores
    __shared__ uint2 qsl[4][KCOL / 8 * 64];  // each wave's query slab
    if (threadIdx.x < 5) kswl::row_scores(K.mat, threadIdx.x, stab[2 * threadIdx.x], stab[2 * threadIdx.x + 1]);
    __syncthreads();
    constexpr int t = KCOL == 32 ? 0 : KCOL == 64 ? 1 : 2;
    int top = 0;
    for (int k = 0; k < 25; ++k) top = imax(top, (int)K.mat[k]);
    KswLanePol pol{&K, S.order, S.rest, top};
    kswl::lane_engine<KCOL, 8>(pol, S.bounds, S.heads, KCOL == 32 ? 0 : KCOL / 32, KCOL / 16, stab, qsl[threadIdx.x >> 6], K.o_del, K.e_del, K.o_ins, K.e_ins, top,
                               S.stats ? S.stats + 8 * t : nullptr);
}

// the problems the lanes left: one per wave
__global__ __launch_bounds__(256) void ksw_extend_rest_kernel(KswParams K, KswSort S) {
    const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int n_waves = (int)((gridDim.x * blockDim.x) >> 6);
    int top = 0;
    for (int k = 0; k < 25; ++k) top = imax(top, (int)K.mat[k]);
    for (int it = wave; it < K.n; it += n_waves) {
        if (!__builtin_amdgcn_readfirstlane((int)S.rest[it])) continue;
        const KswTask U = K.task[it];
        const uint8_t* q = K.q + U.q_off;
        const uint8_t* tg = K.t + U.t_off;
        const kswd::ExtIn E{U.qlen, U.tlen, U.w, U.end_bonus, U.zdrop, U.h0};
        auto qf = [&](int j) { return (int)q[j]; };
        auto tf = [&](int i) { return (int)tg[i]; };
        const int ql = __builtin_amdgcn_readfirstlane(U.qlen);
        KswResult x;
        if (ql < 64) x = kswd::extend_wave<1>(E, qf, tf, K.mat, K.o_del, K.e_del, K.o_ins, K.e_ins, top);
        else if (ql < 128) x = kswd::extend_wave<2>(E, qf, tf, K.mat, K.o_del, K.e_del, K.o_ins, K.e_ins, top);
        else x = kswd::extend_wave<KSW_COLS_PER_LANE>(E, qf, tf, K.mat, K.o_del, K.e_del, K.o_ins, K.e_ins, top);
        if ((threadIdx.x & 63) == 0) K.out[it] = x;
    }
}

}  // namespace smem

// scratch of the lane path: KSW_BUCKETS + 10 + 8 words, then order (n words),
// rest (n bytes) and 24 u64 of diagnostics
extern "C" size_t smem_ksw_lane_scratch(int n) {
    return sizeof(uint32_t) * (smem::KSW_BUCKETS + 18 + (size_t)n) + (size_t)n + 256 + 24 * 8;
}

// SMEM_KSW_LANE=1: the lane engine (tasks sorted by query length on the
// device, three tiers, the rest one per wave); scratch: smem_ksw_lane_scratch(n) bytes
extern "C" hipError_t smem_launch_ksw_lane(const smem::KswParams* K, void* scratch, int n_cu, hipStream_t st) {
    if (K->n <= 0) return hipSuccess;
    smem::KswSort S;
    uint32_t* w = static_cast<uint32_t*>(scratch);
    S.hist = w, S.bounds = w + smem::KSW_BUCKETS, S.heads = w + smem::KSW_BUCKETS + 10,
    S.order = w + smem::KSW_BUCKETS + 18;
    S.rest = reinterpret_cast<uint8_t*>(S.order + K->n);
    S.stats = nullptr;
    hipError_t e = hipMemsetAsync(S.hist, 0, sizeof(uint32_t) * smem::KSW_BUCKETS, st);
    if (e != hipSuccess) return e;
    const char* se = getenv("SMEM_KSW_LANE_STATS");
    if (se && atoi(se)) {
        S.stats = reinterpret_cast<unsigned long long*>(
            (reinterpret_cast<uintptr_t>(S.rest + K->n) + 255) & ~static_cast<uintptr_t>(255));
        e = hipMemsetAsync(S.stats, 0, 24 * 8, st);
        if (e != hipSuccess) return e;
    }
    const int blocks = std::min(n_cu * 4, (K->n + 255) / 256);
    hipLaunchKernelGGL(smem::ksw_hist_kernel, dim3(blocks), dim3(256), 0, st, *K, S);
    hipLaunchKernelGGL(smem::ksw_scan_kernel, dim3(1), dim3(256), 0, st, S);
    hipLaunchKernelGGL(smem::ksw_scatter_kernel, dim3(blocks), dim3(256), 0, st, *K, S);
    // one block of 4 waves per SIMD slot the tier's registers leave (4, 4, 2)
    hipLaunchKernelGGL(smem::ksw_lane_kernel<32>, dim3(n_cu * 4), dim3(256), 0, st, *K, S);
    hipLaunchKernelGGL(smem::ksw_lane_kernel<64>, dim3(n_cu * 4), dim3(256), 0, st, *K, S);
    hipLaunchKernelGGL(smem::ksw_lane_kernel<128>, dim3(n_cu * 2), dim3(256), 0, st, *K, S);
    hipLaunchKernelGGL(smem::ksw_extend_rest_kernel, dim3(n_cu * 8), dim3(256), 0, st, *K, S);
    if (S.stats) {
        unsigned long long h[24];
        e = hipMemcpyAsync(h, S.stats, sizeof(h), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) return e;
        for (int t = 0; t < 3; ++t)
            fprintf(stderr, "ksw lane tier %d: wave rows %llu, lane rows %llu, chunks whole %llu / masked %llu, "
                            "refills %llu, problems %llu\n", 32 << t, h[8 * t], h[8 * t + 1], h[8 * t + 2],
                    h[8 * t + 3], h[8 * t + 4], h[8 * t + 5]);
    }
    return hipGetLastError();
}

extern "C" hipError_t smem_launch_ksw(const smem::KswParams* K, int n_cu, hipStream_t st) {
    if (K->n <= 0) return hipSuccess;
    const char* g16e = getenv("SMEM_KSW_G16");  // the 16-lane group kernel (A/B)
    const bool g16 = g16e && atoi(g16e);
    if (g16) {  // four problems per wave
        const int waves = (K->n + 3) / 4 < n_cu * 32 ? (K->n + 3) / 4 : n_cu * 32;
        hipLaunchKernelGGL(smem::ksw_extend_g16_kernel, dim3((waves + 3) / 4), dim3(256), 0, st, *K);
        return hipGetLastError();
    }
    const int waves = K->n < n_cu * 32 ? K->n : n_cu * 32;
    hipLaunchKernelGGL(smem::ksw_extend_kernel, dim3((waves + 3) / 4), dim3(256), 0, st, *K);
    return hipGetLastError();
}

// this file's code object loaded on the current device (see smem_preload_seed)
extern "C" hipError_t smem_preload_ksw(void) {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&smem::ksw_extend_kernel));
}
