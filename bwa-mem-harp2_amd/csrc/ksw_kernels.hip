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
namespace {

constexpr int KC = KSW_COLS_PER_LANE;  // qlen <= 64 KC - 1
constexpr int NEG = -(1 << 28);

__device__ __forceinline__ int imax(int a, int b) { return a > b ? a : b; }

// Cross-lane steps by DPP (no LDS round trip): an inclusive prefix max over
// the 64 lanes (row_shr 1/2/4/8 inside each 16-lane row, then row_bcast 15
// and 31 across rows; lanes a step does not reach keep NEG), and the
// whole-wave shift by one lane (wave_shr 1, lane 0 takes `first`).
__device__ __forceinline__ int scan_max(int v) {
    v = imax(v, __builtin_amdgcn_update_dpp(NEG, v, 0x111, 0xf, 0xf, false));  // row_shr:1
    v = imax(v, __builtin_amdgcn_update_dpp(NEG, v, 0x112, 0xf, 0xf, false));  // row_shr:2
    v = imax(v, __builtin_amdgcn_update_dpp(NEG, v, 0x114, 0xf, 0xf, false));  // row_shr:4
    v = imax(v, __builtin_amdgcn_update_dpp(NEG, v, 0x118, 0xf, 0xf, false));  // row_shr:8
    v = imax(v, __builtin_amdgcn_update_dpp(NEG, v, 0x142, 0xa, 0xf, false));  // row_bcast:15
    v = imax(v, __builtin_amdgcn_update_dpp(NEG, v, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return v;
}

__device__ __forceinline__ int wave_shr1(int v, int first) {
    return __builtin_amdgcn_update_dpp(first, v, 0x138, 0xf, 0xf, false);  // wave_shr:1
}

__device__ __forceinline__ int rl(int v, int l) { return __builtin_amdgcn_readlane(v, l); }

}  // namespace

__global__ __launch_bounds__(256) void ksw_extend_kernel(KswParams K) {
    const int lane = threadIdx.x & 63;
    const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int n_waves = (int)((gridDim.x * blockDim.x) >> 6);
    const int oe_del = K.o_del + K.e_del, oe_ins = K.o_ins + K.e_ins;
    int top = 0;  // the largest matrix entry (from 0), software/ksw.c:398-400
    for (int k = 0; k < 25; ++k) top = imax(top, (int)K.mat[k]);
    for (int it = wave; it < K.n; it += n_waves) {
        const KswTask T = K.task[it];
        const int qlen = T.qlen, tlen = T.tlen;
        const uint8_t* q = K.q + T.q_off;
        const uint8_t* tg = K.t + T.t_off;
        const int h0 = T.h0 > 0 ? T.h0 : 0;
        const int eh1 = h0 > oe_ins ? h0 - oe_ins : 0;

        // columns: scores, first row (software/ksw.c:389-396)
        uint32_t sc[KC];
        int sc4[KC], hp[KC], ee[KC];
#pragma unroll
        for (int c = 0; c < KC; ++c) {
            const int j = 64 * c + lane;
            const int qc = j < qlen ? (int)q[j] : 0;
            sc[c] = (uint32_t)(uint8_t)K.mat[qc] | (uint32_t)(uint8_t)K.mat[5 + qc] << 8 |
                    (uint32_t)(uint8_t)K.mat[10 + qc] << 16 | (uint32_t)(uint8_t)K.mat[15 + qc] << 24;
            sc4[c] = K.mat[20 + qc];
            int h = 0;
            if (j == 0) h = h0;
            else if (j == 1) h = eh1;
            else if (j <= qlen && eh1 - (j - 2) * K.e_ins > K.e_ins) h = eh1 - (j - 1) * K.e_ins;
            hp[c] = h;
            ee[c] = 0;
        }
        // band limit (software/ksw.c:401-406)
        int w = T.w;
        {
            int lim = (int)((double)(qlen * top + T.end_bonus - K.o_ins) / K.e_ins + 1.);
            lim = imax(lim, 1);
            w = w < lim ? w : lim;
            lim = (int)((double)(qlen * top + T.end_bonus - K.o_del) / K.e_del + 1.);
            lim = imax(lim, 1);
            w = w < lim ? w : lim;
        }
        int mx = h0, max_i = -1, max_j = -1, max_ie = -1, gscore = -1, max_off = 0;
        int beg = 0, end = qlen;
        for (int i = 0; i < tlen; ++i) {
            const int tc = tg[i];
            int h1 = h0 - (K.o_del + K.e_del * (i + 1));
            if (h1 < 0) h1 = 0;
            if (beg < i - w) beg = i - w;
            if (end > i + w + 1) end = i + w + 1;
            if (end > qlen) end = qlen;
            // H of the row: D, then F by a prefix max across the columns
            int H[KC];
            int carry = NEG, key = NEG;
#pragma unroll
            for (int c = 0; c < KC; ++c) {
                const int j = 64 * c + lane;
                H[c] = 0;
                if (64 * c >= end || 64 * c + 63 < beg) continue;  // chunk outside the band (uniform)
                const bool valid = j >= beg && j < end;
                const int s = tc < 4 ? (int)(int8_t)(sc[c] >> (8 * tc)) : sc4[c];
                const int d = imax(hp[c] + s, ee[c]);
                const int incl = scan_max(valid ? d + j * K.e_ins : NEG);
                const int excl = imax(wave_shr1(incl, NEG), carry);
                carry = imax(carry, rl(incl, 63));
                const int f = imax(0, excl - oe_ins - (j - 1) * K.e_ins);
                const int h = imax(d, f);
                if (valid) {
                    H[c] = h;
                    key = imax(key, h << 8 | j);  // ascending j: ties keep the last column
                }
            }
            // row maximum m (0 when the band is empty) and its last column
            const bool nonempty = beg < end;
            int m = 0, mj = -1;
            if (nonempty) {
                const int kmax = rl(scan_max(key), 63);
                m = kmax >> 8;
                mj = kmax & 255;
            }
            // the column array for the next row: E updated, H shifted one
            // column right (column beg takes the row's first-column value)
            int prev_last = 0;  // H of the previous chunk's last column
#pragma unroll
            for (int c = 0; c < KC; ++c) {
                const int j = 64 * c + lane;
                if (64 * c >= end || 64 * c + 63 < beg) {  // outside the band (uniform)
                    prev_last = 0;
                    continue;
                }
                const int up = wave_shr1(H[c], prev_last);
                prev_last = rl(H[c], 63);
                if (j >= beg && j < end) {
                    ee[c] = imax(ee[c] - K.e_del, imax(H[c] - oe_del, 0));
                    hp[c] = j == beg ? h1 : up;
                }
            }
            int hlast = h1;
            if (nonempty) {
                const int ce = (end - 1) >> 6, le = (end - 1) & 63;
#pragma unroll
                for (int c = 0; c < KC; ++c)
                    if (c == ce) hlast = rl(H[c], le);
            }
#pragma unroll
            for (int c = 0; c < KC; ++c)
                if (64 * c + lane == end) {
                    hp[c] = hlast;
                    ee[c] = 0;
                }
            if ((nonempty ? end : beg) == qlen) {  // the scan reached the query end
                if (hlast >= gscore) max_ie = i;
                gscore = imax(gscore, hlast);
            }
            if (m == 0) break;
            if (m > mx) {
                mx = m, max_i = i, max_j = mj;
                const int o = mj > i ? mj - i : i - mj;
                max_off = imax(max_off, o);
            } else if (T.zdrop > 0) {
                const int di = i - max_i, dj = mj - max_j;
                const int drop = di > dj ? mx - m - (di - dj) * K.e_del : mx - m - (dj - di) * K.e_ins;
                if (drop > T.zdrop) break;
            }
            // refit the band around mj (software/ksw.c:463-466)
            int zlo = -1, zhi = 0x7fffffff;
#pragma unroll
            for (int c = 0; c < KC; ++c) {
                const int j = 64 * c + lane;
                const uint64_t lo = __ballot(hp[c] == 0 && j >= beg && j <= mj);
                const uint64_t hi = __ballot(hp[c] == 0 && j >= mj + 2 && j <= end);
                if (lo) zlo = 64 * c + 63 - __builtin_clzll(lo);
                if (hi && zhi == 0x7fffffff) zhi = 64 * c + __builtin_ctzll(hi);
            }
            beg = zlo >= 0 ? zlo + 1 : beg;
            end = zhi != 0x7fffffff ? zhi : end + 1;
        }
        if (lane == 0) K.out[it] = KswResult{mx, max_j + 1, max_i + 1, max_ie + 1, gscore, max_off};
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
