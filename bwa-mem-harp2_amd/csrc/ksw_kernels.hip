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
#include <stdlib.h>

#include "ksw_kernels.h"
#include "ksw_device.h"

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

}  // namespace smem

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
