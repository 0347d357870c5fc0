// Wave-level SW building blocks shared by ksw_kernels.hip and aln_kernels.hip:
// DPP scans and shifts, ksw_extend2 (software/ksw.c:379-476) for one problem
// per wave, and the striped local SW behind ksw_align2 (software/ksw.c:110-364)
// for one problem per wave.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ksw_kernels.h"

namespace smem {
namespace kswd {

constexpr int NEG = -(1 << 28);

__device__ __forceinline__ int imax(int a, int b) { return a > b ? a : b; }
__device__ __forceinline__ int imin(int a, int b) { return a < b ? a : b; }

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

// The same scan for inputs that are >= 0 or NEG, whose scan is only read
// where it is >= 0 or where 0 and NEG give the same result: lanes with no
// source read 0 (bound_ctrl), so each row step is one v_max_i32_dpp.
__device__ __forceinline__ int scan_max_nn(int v) {
    v = imax(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true));  // row_shr:1
    v = imax(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true));  // row_shr:2
    v = imax(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true));  // row_shr:4
    v = imax(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true));  // row_shr:8
    v = imax(v, __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false));  // row_bcast:15
    v = imax(v, __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return v;
}

__device__ __forceinline__ int wave_shr1(int v, int first) {
    return __builtin_amdgcn_update_dpp(first, v, 0x138, 0xf, 0xf, false);  // wave_shr:1
}

__device__ __forceinline__ int rl(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ int wave_max(int v) { return rl(scan_max(v), 63); }

// the inputs of one ksw_extend2 call besides the sequences and the scoring
struct ExtIn {
    int qlen, tlen, w, end_bonus, zdrop, h0;
};

// ksw_extend2 by one wave.  Lanes hold query columns j = 64 c + lane, c < KC
// (so qlen <= 64 KC - 1), in registers: the column array's two values (the
// previous row's H one column to the left, this row's E) and the column's
// scores for the five target symbols.  Inside a row the serial loop carries
// F from column to column; here
//     F(j) = max(0, max_{beg <= k < j} D(k) - oe_ins - (j - 1 - k) e_ins),
//     D(k) = max(H(i-1, k-1) + s(k), E(i, k)),
// which is what the serial recurrence gives (an F-derived H never restarts a
// better F, since a restart pays o_ins again), so a prefix max of
// D(k) + k e_ins across the lanes replaces it.  The row maximum (its last
// column on ties), the to-end score, z-drop and the band refit follow the
// serial code step by step with wave reductions and ballots, so every output
// (score, qle, tle, gtle, gscore, max_off) is the reference's.  qsym(j) gives
// query column j (j < qlen), tsym(i) target row i (i < tlen); the target is
// fetched 64 rows at a time, one row per lane.  top: the largest matrix
// entry, at least 0 (software/ksw.c:398-400).
template <int KC, class QF, class TF>
__device__ __forceinline__ KswResult extend_wave(const ExtIn& T, QF qsym, TF tsym, const int8_t* mat, int o_del,
                                                 int e_del, int o_ins, int e_ins, int top, uint64_t* nrows = nullptr) {
    constexpr int JB = KC <= 4 ? 8 : 10;  // column bits of the (score, column) keys
    const int lane = threadIdx.x & 63;
    const int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
    const int qlen = T.qlen, tlen = T.tlen;
    const int h0 = T.h0 > 0 ? T.h0 : 0;
    const int eh1 = h0 > oe_ins ? h0 - oe_ins : 0;

    // columns: scores, first row (software/ksw.c:389-396)
    uint32_t sc[KC];
    int sc4[KC], hp[KC], ee[KC];
#pragma unroll
    for (int c = 0; c < KC; ++c) {
        const int j = 64 * c + lane;
        const int qc = j < qlen ? (int)qsym(j) : 0;
        sc[c] = (uint32_t)(uint8_t)mat[qc] | (uint32_t)(uint8_t)mat[5 + qc] << 8 |
                (uint32_t)(uint8_t)mat[10 + qc] << 16 | (uint32_t)(uint8_t)mat[15 + qc] << 24;
        sc4[c] = mat[20 + qc];
        int h = 0;
        if (j == 0) h = h0;
        else if (j == 1) h = eh1;
        else if (j <= qlen && eh1 - (j - 2) * e_ins > e_ins) h = eh1 - (j - 1) * e_ins;
        hp[c] = h;
        ee[c] = 0;
    }
    // band limit (software/ksw.c:401-406)
    int w = T.w;
    {
        int lim = (int)((double)(qlen * top + T.end_bonus - o_ins) / e_ins + 1.);
        lim = imax(lim, 1);
        w = w < lim ? w : lim;
        lim = (int)((double)(qlen * top + T.end_bonus - o_del) / e_del + 1.);
        lim = imax(lim, 1);
        w = w < lim ? w : lim;
    }
    int mx = h0, max_i = -1, max_j = -1, max_ie = -1, gscore = -1, max_off = 0;
    int beg = 0, end = qlen;
    int tcache = 0;
    for (int i = 0; i < tlen; ++i) {
        if (nrows) ++*nrows;  // diagnostics (rows the wave walked)
        if ((i & 63) == 0) tcache = i + lane < tlen ? (int)tsym(i + lane) : 0;
        const int tc = rl(tcache, i & 63);
        int h1 = h0 - (o_del + e_del * (i + 1));
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
            // d >= 0 (E >= 0), e_ins >= 1: a lane with no valid column before
            // it reads 0 instead of NEG, and f = max(0, 0 - oe_ins - ...) = 0
            // there as before
            const int incl = scan_max_nn(valid ? d + j * e_ins : NEG);
            const int excl = imax(wave_shr1(incl, NEG), carry);
            carry = imax(carry, rl(incl, 63));
            const int f = imax(0, excl - oe_ins - (j - 1) * e_ins);
            const int h = imax(d, f);
            if (valid) {
                H[c] = h;
                key = imax(key, h << JB | j);  // ascending j: ties keep the last column
            }
        }
        // row maximum m (0 when the band is empty) and its last column
        const bool nonempty = beg < end;
        int m = 0, mj = -1;
        if (nonempty) {
            const int kmax = rl(scan_max_nn(key), 63);  // some key >= 0
            m = kmax >> JB;
            mj = kmax & ((1 << JB) - 1);
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
                ee[c] = imax(ee[c] - e_del, imax(H[c] - oe_del, 0));
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
            const int drop = di > dj ? mx - m - (di - dj) * e_del : mx - m - (dj - di) * e_ins;
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
    return KswResult{mx, max_j + 1, max_i + 1, max_ie + 1, gscore, max_off};
}

// ---- ksw_extend2 on 16-lane groups: four problems per wave ----
// The same recurrences as extend_wave with the query columns of a problem on
// the 16 lanes of one DPP row (j = 16 c + lane16, c < KC): the in-row prefix
// max is four row_shr steps, the one-column shift a row_shr:1, and the row's
// lane 15 reaches its lanes by ds_swizzle (and 0x10, or 0x0f).  Every group
// walks its own problem's rows; a group whose problem ended (or that has
// none) idles until the wave's last group is done.
__device__ __forceinline__ int scan16_max(int v) {
    v = imax(v, __builtin_amdgcn_update_dpp(NEG, v, 0x111, 0xf, 0xf, false));  // row_shr:1
    v = imax(v, __builtin_amdgcn_update_dpp(NEG, v, 0x112, 0xf, 0xf, false));  // row_shr:2
    v = imax(v, __builtin_amdgcn_update_dpp(NEG, v, 0x114, 0xf, 0xf, false));  // row_shr:4
    v = imax(v, __builtin_amdgcn_update_dpp(NEG, v, 0x118, 0xf, 0xf, false));  // row_shr:8
    return v;
}
__device__ __forceinline__ int row_shr1(int v, int first) {
    return __builtin_amdgcn_update_dpp(first, v, 0x111, 0xf, 0xf, false);  // row_shr:1, lane16 0 takes first
}
__device__ __forceinline__ int bcast15(int v) { return __builtin_amdgcn_ds_swizzle(v, 0x1F0); }
__device__ __forceinline__ int from16(int v, int l16) {  // lane l16 of this lane's group
    return __builtin_amdgcn_ds_bpermute((((int)threadIdx.x & 0x30) | l16) << 2, v);
}

template <int KC, class QF, class TF>
__device__ __forceinline__ KswResult extend_group16(const ExtIn& T, bool active, QF qsym, TF tsym, const int8_t* mat,
                                                    int o_del, int e_del, int o_ins, int e_ins, int top) {
    static_assert(KC <= 16, "columns < 256");
    const int l16 = threadIdx.x & 15;
    const int g = (threadIdx.x >> 4) & 3;
    const int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
    const int qlen = active ? T.qlen : 0, tlen = active ? T.tlen : 0;
    const int h0 = T.h0 > 0 ? T.h0 : 0;
    const int eh1 = h0 > oe_ins ? h0 - oe_ins : 0;
    uint32_t sc[KC];
    int sc4[KC], hp[KC], ee[KC];
#pragma unroll
    for (int c = 0; c < KC; ++c) {
        const int j = 16 * c + l16;
        const int qc = j < qlen ? (int)qsym(j) : 0;
        sc[c] = (uint32_t)(uint8_t)mat[qc] | (uint32_t)(uint8_t)mat[5 + qc] << 8 |
                (uint32_t)(uint8_t)mat[10 + qc] << 16 | (uint32_t)(uint8_t)mat[15 + qc] << 24;
        sc4[c] = mat[20 + qc];
        int h = 0;
        if (j == 0) h = h0;
        else if (j == 1) h = eh1;
        else if (j <= qlen && eh1 - (j - 2) * e_ins > e_ins) h = eh1 - (j - 1) * e_ins;
        hp[c] = h;
        ee[c] = 0;
    }
    int w = T.w;
    if (active) {  // band limit (software/ksw.c:401-406)
        int lim = (int)((double)(qlen * top + T.end_bonus - o_ins) / e_ins + 1.);
        lim = imax(lim, 1);
        w = w < lim ? w : lim;
        lim = (int)((double)(qlen * top + T.end_bonus - o_del) / e_del + 1.);
        lim = imax(lim, 1);
        w = w < lim ? w : lim;
    }
    int mx = h0, max_i = -1, max_j = -1, max_ie = -1, gscore = -1, max_off = 0;
    int beg = 0, end = qlen;
    bool done = !active || tlen <= 0;
    int tcache = 0;
    for (int i = 0;; ++i) {
        if (__ballot(!done) == 0) break;
        if ((i & 15) == 0) tcache = !done && i + l16 < tlen ? (int)tsym(i + l16) : 0;
        const int tc = from16(tcache, i & 15);
        if (!done) {
            int h1 = h0 - (o_del + e_del * (i + 1));
            if (h1 < 0) h1 = 0;
            if (beg < i - w) beg = i - w;
            if (end > i + w + 1) end = i + w + 1;
            if (end > qlen) end = qlen;
            // D and the in-chunk prefix of every chunk first (independent),
            // then the carries across chunks from the chunk totals: the
            // swizzles of the totals pipeline instead of chaining
            int H[KC], D[KC], incl[KC], tot[KC];
#pragma unroll
            for (int c = 0; c < KC; ++c) {
                const int j = 16 * c + l16;
                const bool valid = j >= beg && j < end;
                const int sv = tc < 4 ? (int)(int8_t)(sc[c] >> (8 * tc)) : sc4[c];
                D[c] = imax(hp[c] + sv, ee[c]);
                incl[c] = NEG;
                tot[c] = NEG;
                if (16 * c >= end || 16 * c + 15 < beg) continue;  // chunk outside the band (group-uniform)
                incl[c] = scan16_max(valid ? D[c] + j * e_ins : NEG);
                tot[c] = bcast15(incl[c]);
            }
            int carry = NEG, key = NEG;
#pragma unroll
            for (int c = 0; c < KC; ++c) {
                const int j = 16 * c + l16;
                H[c] = 0;
                if (16 * c >= end || 16 * c + 15 < beg) continue;
                const bool valid = j >= beg && j < end;
                const int excl = imax(row_shr1(incl[c], NEG), carry);
                carry = imax(carry, tot[c]);
                const int f = imax(0, excl - oe_ins - (j - 1) * e_ins);
                const int h = imax(D[c], f);
                if (valid) {
                    H[c] = h;
                    key = imax(key, h << 8 | j);  // ascending j: ties keep the last column
                }
            }
            const bool nonempty = beg < end;
            int m = 0, mj = -1;
            if (nonempty) {
                const int kmax = bcast15(scan16_max(key));
                m = kmax >> 8;
                mj = kmax & 255;
            }
            int prev_last = 0;
#pragma unroll
            for (int c = 0; c < KC; ++c) {
                const int j = 16 * c + l16;
                if (16 * c >= end || 16 * c + 15 < beg) {
                    prev_last = 0;
                    continue;
                }
                const int up = row_shr1(H[c], prev_last);
                prev_last = bcast15(H[c]);
                if (j >= beg && j < end) {
                    ee[c] = imax(ee[c] - e_del, imax(H[c] - oe_del, 0));
                    hp[c] = j == beg ? h1 : up;
                }
            }
            int hlast = h1;
            if (nonempty) {
                const int ce = (end - 1) >> 4, le = (end - 1) & 15;
#pragma unroll
                for (int c = 0; c < KC; ++c)
                    if (c == ce) hlast = from16(H[c], le);
            }
#pragma unroll
            for (int c = 0; c < KC; ++c)
                if (16 * c + l16 == end) {
                    hp[c] = hlast;
                    ee[c] = 0;
                }
            if ((nonempty ? end : beg) == qlen) {
                if (hlast >= gscore) max_ie = i;
                gscore = imax(gscore, hlast);
            }
            bool stop = m == 0;
            if (!stop) {
                if (m > mx) {
                    mx = m, max_i = i, max_j = mj;
                    const int o = mj > i ? mj - i : i - mj;
                    max_off = imax(max_off, o);
                } else if (T.zdrop > 0) {
                    const int di = i - max_i, dj = mj - max_j;
                    const int drop = di > dj ? mx - m - (di - dj) * e_del : mx - m - (dj - di) * e_ins;
                    stop = drop > T.zdrop;
                }
            }
            if (!stop) {  // refit the band around mj (software/ksw.c:463-466)
                int zlo = -1, zhi = 0x7fffffff;
#pragma unroll
                for (int c = 0; c < KC; ++c) {
                    const int j = 16 * c + l16;
                    const uint32_t lo = (uint32_t)(__ballot(hp[c] == 0 && j >= beg && j <= mj) >> (16 * g)) & 0xFFFFu;
                    const uint32_t hi = (uint32_t)(__ballot(hp[c] == 0 && j >= mj + 2 && j <= end) >> (16 * g)) & 0xFFFFu;
                    if (lo) zlo = 16 * c + 31 - __builtin_clz(lo);
                    if (hi && zhi == 0x7fffffff) zhi = 16 * c + __builtin_ctz(hi);
                }
                beg = zlo >= 0 ? zlo + 1 : beg;
                end = zhi != 0x7fffffff ? zhi : end + 1;
            }
            done = stop || i + 1 >= tlen;
        }
    }
    return KswResult{mx, max_j + 1, max_i + 1, max_ie + 1, gscore, max_off};
}

// ---- ksw_align2's local SW (software/ksw.c:110-364), one wave per problem ----
constexpr int SW_XBYTE = 0x10000, SW_XSTOP = 0x20000, SW_XSUBO = 0x40000, SW_XSTART = 0x80000;

struct SwOut {
    int score, te, qe, score2, te2;
};

// One ksw_u8 (p = 16) or ksw_i16 (p = 8) pass.  The reference cuts the query
// into p blocks of slen = ceil(qlen / p) columns, one block per vector lane,
// pads it to qp = p slen columns that score 0, and per target row
//   pass 1:  H1 = max(D, Fb), Fb carried only inside a block, E from H1;
//   lazy F:  F carried across blocks until it can raise no H.
// In closed form, with D(q) = max(diag(q), E(q)):
//   Fb(q) = max(0, max_{k < q, same block} D(k) - oe_ins - (q-1-k) e_ins)
//   H(q)  = max(D(q), max(0, max_{k < q} D(k) - oe_ins - (q-1-k) e_ins))
// (F-derived H never starts a better F).  Both maxima are prefix maxima of
// D(k) + k e_ins over columns q = 64 c + lane (qp <= 256); the in-block one
// keys each value with its block number above bit 20, so a prefix max stays
// inside the block.  The row maximum of H1 (padding included) feeds the
// suboptimal list b (kept one entry per lane, slot = index / 64) and the
// best row; qe is the smallest column holding the best row's maximum.
template <class QF, class TF>
__device__ __forceinline__ SwOut sw_pass_wave(int p, int qlen, QF qsym, int tlen, TF tsym, const int8_t* mat,
                                              int o_del, int e_del, int o_ins, int e_ins, int minsc, int endsc,
                                              int shift, int top) {
    const int lane = threadIdx.x & 63;
    const bool u8 = p == 16;
    const int slen = (qlen + p - 1) / p, qp = slen * p;
    const int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
    uint32_t sc[4];
    int sc4[4], hp[4], ee[4], hm[4], sg[4], tv[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int q = 64 * c + lane;
        if (q < qlen) {
            const int qc = (int)qsym(q);
            sc[c] = (uint32_t)(uint8_t)mat[qc] | (uint32_t)(uint8_t)mat[5 + qc] << 8 |
                    (uint32_t)(uint8_t)mat[10 + qc] << 16 | (uint32_t)(uint8_t)mat[15 + qc] << 24;
            sc4[c] = mat[20 + qc];
        } else {
            sc[c] = 0;  // padding columns score 0 (software/ksw.c:95)
            sc4[c] = 0;
        }
        hp[c] = ee[c] = hm[c] = 0;
        sg[c] = q < qp ? q / slen : 0;
        tv[c] = q < tlen ? (int)tsym(q) : 0;  // target row 64 c + lane
    }
    int gmax = 0, te = -1;
    int bv[4] = {-1, -1, -1, -1}, br[4] = {0, 0, 0, 0};
    int n_b = 0, last_row = -2, last_val = 0;
    for (int i = 0; i < tlen; ++i) {
        const int ci = i >> 6;
        int t = tv[0];
        if (ci == 1) t = tv[1];
        if (ci == 2) t = tv[2];
        if (ci == 3) t = tv[3];
        t = rl(t, i & 63);
        int hn[4];
        int prev_last = 0, carry_b = NEG, carry_a = NEG, rmax = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int q = 64 * c + lane;
            hn[c] = 0;
            if (64 * c >= qp) continue;  // uniform
            const int up = wave_shr1(hp[c], prev_last);  // H(i-1, q-1), 0 at q = 0
            prev_last = rl(hp[c], 63);
            const bool valid = q < qp;
            const int s = t < 4 ? (int)(int8_t)(sc[c] >> (8 * t)) : sc4[c];
            int h = up + s;
            if (u8) h = imax(imin(h + shift, 255) - shift, 0);  // adds_epu8 then subs_epu8 of the bias
            const int d = imax(h, ee[c]);
            const int v = d + q * e_ins;
            const int ib = scan_max(valid ? (sg[c] << 20 | v) : NEG);
            const int ia = scan_max(valid ? v : NEG);
            const int xb = imax(wave_shr1(ib, NEG), carry_b);
            const int xa = imax(wave_shr1(ia, NEG), carry_a);
            carry_b = imax(carry_b, rl(ib, 63));
            carry_a = imax(carry_a, rl(ia, 63));
            const int fb = (xb >> 20) == sg[c] ? imax(0, (xb & 0xfffff) - oe_ins - (q - 1) * e_ins) : 0;
            const int fa = imax(0, xa - oe_ins - (q - 1) * e_ins);
            const int h1 = imax(d, fb);
            if (valid) {
                rmax = imax(rmax, h1);
                ee[c] = imax(imax(ee[c] - e_del, 0), imax(h1 - oe_del, 0));
                hn[c] = imax(d, fa);
            }
        }
#pragma unroll
        for (int c = 0; c < 4; ++c)
            if (64 * c < qp) hp[c] = hn[c];
        rmax = wave_max(rmax);
        if (rmax >= minsc) {  // the suboptimal list (software/ksw.c:191-199)
            int idx = -1;
            if (n_b == 0 || last_row + 1 != i) idx = n_b++;
            else if (last_val < rmax) idx = n_b - 1;
            if (idx >= 0) {
                last_row = i, last_val = rmax;
                if (lane == (idx & 63)) {
                    const int slot = idx >> 6;
#pragma unroll
                    for (int c = 0; c < 4; ++c)
                        if (c == slot) bv[c] = rmax, br[c] = i;
                }
            }
        }
        if (rmax > gmax) {
            gmax = rmax, te = i;
#pragma unroll
            for (int c = 0; c < 4; ++c) hm[c] = hp[c];
            if ((u8 && gmax + shift >= 255) || gmax >= endsc) break;
        }
    }
    SwOut r;
    r.score = u8 ? (gmax + shift < 255 ? gmax : 255) : gmax;
    r.te = te;
    r.qe = -1;
    r.score2 = -1;
    r.te2 = -1;
    if (!u8 || r.score != 255) {
        int m = NEG;
#pragma unroll
        for (int c = 0; c < 4; ++c)
            if (64 * c + lane < qp) m = imax(m, hm[c]);
        m = wave_max(m);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint64_t b = __ballot(64 * c + lane < qp && hm[c] == m);
            if (b && r.qe < 0) r.qe = 64 * c + __builtin_ctzll(b);
        }
        if (n_b) {
            const int d = (r.score + top - 1) / top, low = te - d, high = te + d;
            int cand = -1;
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (64 * c + lane < n_b && (br[c] < low || br[c] > high)) cand = imax(cand, bv[c]);
            r.score2 = imax(-1, wave_max(cand));
            // te2: the row of the first list entry holding score2 (the strict > scan)
            if (r.score2 >= 0) {
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const uint64_t hit = __ballot(64 * c + lane < n_b && (br[c] < low || br[c] > high) &&
                                                  bv[c] == r.score2);
                    if (hit && r.te2 < 0) r.te2 = rl(br[c], __builtin_ctzll(hit));
                }
            }
        }
    }
    return r;
}

struct SwAlign {
    int score, te, qe, score2, te2, tb, qb;  // kswr_t (software/ksw.h:13-15)
};

// ksw_align2 (software/ksw.c:342-364): the forward pass, then, for KSW_XSTART,
// the pass over the reversed query [0, qe] and target (first te + 1 rows
// reversed, the rest as is) that stops at the forward score; tb / qb = -1
// unless that pass reaches the same score
template <class QF, class TF>
__device__ __forceinline__ SwAlign sw_align_wave(int qlen, QF qsym, int tlen, TF tsym, const int8_t* mat, int o_del,
                                                 int e_del, int o_ins, int e_ins, int xtra, int shift, int top) {
    const int p = (xtra & SW_XBYTE) ? 16 : 8;
    const int minsc = (xtra & SW_XSUBO) ? xtra & 0xffff : 0x10000;
    const SwOut r = sw_pass_wave(p, qlen, qsym, tlen, tsym, mat, o_del, e_del, o_ins, e_ins, minsc, 0x10000, shift, top);
    SwAlign a{r.score, r.te, r.qe, r.score2, r.te2, -1, -1};
    if ((xtra & SW_XSTART) == 0 || ((xtra & SW_XSUBO) && r.score < (xtra & 0xffff)) || r.qe < 0) return a;
    const int qe = r.qe, te = r.te;
    const SwOut rr = sw_pass_wave(
        p, qe + 1, [&](int q) { return qsym(qe - q); }, tlen, [&](int i) { return i <= te ? tsym(te - i) : tsym(i); },
        mat, o_del, e_del, o_ins, e_ins, 0x10000, r.score, shift, top);
    if (r.score == rr.score) a.tb = te - rr.te, a.qb = qe - rr.qe;
    return a;
}

}  // namespace kswd
}  // namespace smem
