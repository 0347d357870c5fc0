// ksw_extend2 (software/ksw.c:379-476) with one problem per LANE: the
// reference's serial row loop, run by each of a wave's 64 lanes on its own
// problem in lockstep, so one wave instruction advances 64 problems by a
// cell.  The wave-per-problem form (ksw_device.h extend_wave) spends a row
// step of ~70 instructions -- two wave scans, shifts, ballots -- on at most 64
// columns, and the problems mem_chain2aln makes are 20-130 columns long; here
// a cell is ~14 instructions for 64 problems.
//
// The column array eh[0 .. qlen] lives in registers: one VGPR per column,
// H in the low and E in the high 16 bits, unrolled over KCOL columns, so a
// column index is a compile-time constant and every lane walks column j at
// the same time, each inside its own band [beg, end).  Per chunk of 8
// columns: skipped when no lane's band (or end column) reaches it, run as is
// when every live lane's band covers it, else with each column's results
// selected by the lane's band.  The query is held as its codes, four per word;
// one v_perm of a word against the target row's scores (mat[tc][0..3] as
// bytes, mat[tc][4] beside them) gives four columns' scores.
//
// The band refit (software/ksw.c:463-466) scans eh[].h for zeros around the
// row maximum; the row loop records which columns it wrote nonzero in a bit
// per column and the refit finds the zeros in those words.
//
// Applies when (extend_lane_ok) 1 <= qlen <= KCOL and h0 + qlen * top <= 65535
// (H and E fit 16 bits).  Outputs are the reference's, bit for bit
// (tests/test_gpu_parity.py ksw cases).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#include "ksw_device.h"

namespace smem {
namespace kswl {

using kswd::ExtIn;
using kswd::imax;
using kswd::imin;

// the row scores of target symbol tc: mat[tc][0..3] as the bytes of lo,
// mat[tc][4] as byte 0 of hi (v_perm selectors 0..3 and 4)
__device__ __forceinline__ void row_scores(const int8_t* mat, int tc, uint32_t& lo, uint32_t& hi) {
    lo = (uint32_t)(uint8_t)mat[tc * 5] | (uint32_t)(uint8_t)mat[tc * 5 + 1] << 8 |
         (uint32_t)(uint8_t)mat[tc * 5 + 2] << 16 | (uint32_t)(uint8_t)mat[tc * 5 + 3] << 24;
    hi = (uint32_t)(uint8_t)mat[tc * 5 + 4];
}

// can one lane run this problem at KCOL columns?
__device__ __forceinline__ bool extend_lane_ok(int kcol, int qlen, int h0, int top) {
    return qlen >= 1 && qlen <= kcol && (h0 > 0 ? h0 : 0) + qlen * top <= 65535;
}

// The query codes of a lane's problem, four columns per word, by unaligned
// dword loads of the code bytes (gfx950 global loads take any byte address),
// stored to the wave's query slab in LDS: qs[c * 64 + lane] holds columns
// 8c .. 8c + 7 of the lane's query (one ds_read_b64 per chunk of the row
// loop; in registers the query took 32 of the 128-column tier's VGPRs and
// pushed its column array into scratch).  Columns j < qlen are p[j]
// (load_query_fwd; the last word may read up to 3 bytes past the query: the
// code buffers carry tail padding) or p_end[-1 - j] (load_query_rev, the
// reversed query of a left extension, p_beg = p_end - qlen: never reads
// below p_beg -- a word that would is loaded from p_beg and shifted).  Every
// load is issued unconditionally (words past the query from a valid address,
// their columns never read), so a lane's loads are in flight together.
typedef uint32_t u32_unaligned __attribute__((aligned(1)));
template <int KCOL>
__device__ __forceinline__ void load_query_fwd(uint2* qs, const uint8_t* p, int qlen) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int c = 0; c < KCOL / 8; ++c) {
        const uint8_t* a0 = 8 * c < qlen ? p + 8 * c : p;
        const uint8_t* a1 = 8 * c + 4 < qlen ? p + 8 * c + 4 : p;
        qs[c * 64 + lane] = make_uint2(*reinterpret_cast<const u32_unaligned*>(a0),
                                       *reinterpret_cast<const u32_unaligned*>(a1));
    }
}
__device__ __forceinline__ uint32_t rev_word(const uint8_t* p_end, const uint8_t* p_beg, int o) {
    // bytes p_end - o - 4 .. p_end - o - 1, reversed (bytes below p_beg: 0)
    const uint8_t* a = p_end - o - 4;
    const int d = a < p_beg ? (int)(p_beg - a) : 0;
    const uint32_t v = *reinterpret_cast<const u32_unaligned*>(a + d) << (8 * d);
    return __builtin_amdgcn_perm(v, v, 0x00010203u);
}
template <int KCOL>
__device__ __forceinline__ void load_query_rev(uint2* qs, const uint8_t* p_end, int qlen) {
    const int lane = threadIdx.x & 63;
    const uint8_t* p_beg = p_end - qlen;
#pragma unroll
    for (int c = 0; c < KCOL / 8; ++c)
        qs[c * 64 + lane] = make_uint2(rev_word(p_end, p_beg, 8 * c < qlen ? 8 * c : 0),
                                       rev_word(p_end, p_beg, 8 * c + 4 < qlen ? 8 * c + 4 : 0));
}

// the first row of the column array (software/ksw.c:393-396): eh[0] = h0,
// eh[1] = eh1, eh[j] = max(eh1 - (j - 1) e_ins, 0) (columns past qlen are
// never read before the row loop writes them), E = 0; in place, 8 columns
// per block (the same arithmetic in C++ kept the old and the new array
// live side by side)
template <int KCOL>
__device__ __forceinline__ void init_row(uint32_t (&EH)[KCOL + 1], int h0, int eh1, int e_ins) {
    EH[0] = (uint32_t)h0;
    int v = eh1 + e_ins;  // eh[j] = max(v - j e_ins, 0) for j >= 1
#pragma unroll
    for (int j = 1; j <= KCOL; ++j)
        asm("v_subrev_u32 %[v], %[e], %[v]\n"
            "v_max_i32 %[h], 0, %[v]\n"
            : [v] "+v"(v), [h] "+v"(EH[j])
            : [e] "s"(e_ins));
}

// f(integral_constant<int, C>) for C = 0, 1, ...: a loop whose index is a
// compile-time constant in the body
template <class F, int... Cs>
__device__ __forceinline__ void for_chunks(F&& f, std::integer_sequence<int, Cs...>) {
    (f(std::integral_constant<int, Cs>{}), ...);
}

// bits lo..hi (inclusive) of bit word k (columns 32 k ..)
__device__ __forceinline__ uint32_t range_bits(int k, int a, int b) {
    const int lo = imax(a - 32 * k, 0), hi = imin(b - 32 * k, 31);
    if (lo > hi) return 0u;
    return (0xffffffffu >> (31 - hi)) & (0xffffffffu << lo);
}

// 1 when h > 0 (h >= 0), as one v_min_u32 (a compare and select otherwise)
__device__ __forceinline__ uint32_t nz1(int h) {
    uint32_t r;
    asm("v_min_u32 %0, 1, %1" : "=v"(r) : "v"(h));
    return r;
}

// KSWL_WHOLE_CHUNKS=1 adds the unmasked form of a chunk for when every live
// lane's band covers it (14 instructions a cell against 22).  Measured: on
// mem_chain2aln's extensions the bands are diagonal strips, so 1-2 % of the
// chunks qualified, and the doubled code (91 KB for the 128-column tier)
// overflowed the instruction cache two CUs share: off by default.
#ifndef KSWL_WHOLE_CHUNKS
#define KSWL_WHOLE_CHUNKS 0
#endif

// A chunk of 8 columns of the row loop (software/ksw.c:427-446) as one
// block of fixed code.  Written in C++, the compiler sank each column's cell
// into a branch of its own (exec-mask juggling per column) and, at the joins
// of the skip / full / masked paths, copied every eh[j] of the chunk twice;
// inside one asm statement the three paths share the registers.
//   mode 0: no lane's band reaches the chunk (nothing runs);
//   mode 1: every live lane's band covers it (14 instructions a cell);
//   mode 2: each column's results kept only inside the lane's band, and the
//           lane's end column takes eh[end] = {h1, 0} (22 a cell).
// Per cell: h = max(eh.h + s, eh.e, f) = H(i, j); eh <- {h1, max(e - e_del,
// h - oe_del, 0)}; f <- max(f - e_ins, h - oe_ins, 0); h1 <- h;
// nzw |= (h1 > 0) << (j mod 32); key = max(key, h << 10 | j).  h1 and f alternate with the temporaries hb / fb
// from cell to cell (8 cells: back in their own registers at the end).
// D = j0 - beg, je = end - j0, bw = end - beg (>= 0).
#define KSWL_STR(x) #x
// (the instructions of a cell ordered so that no result is read by the next
// instruction: with two waves a SIMD, back-to-back dependences left a third
// of the wave cycles waiting on the previous instruction)
#define KSWL_FAST(B, K, EH, SV, HI, HO, FI, FO)                                                                   \
    "v_add_u32_sdwa %[h], sext(%[" #SV "]), %[" #EH "] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_" #B      \
    " src1_sel:WORD_0\n"                                                                                          \
    "v_sub_u32_sdwa %[e], %[" #EH "], %[edel] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n" \
    "v_min_u32 %[t3], 1, %[" #HI "]\n"                                                                            \
    "v_subrev_u32 %[" #FO "], %[eins], %[" #FI "]\n"                                                              \
    "v_max_i32_sdwa %[h], %[h], %[" #EH "] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n"  \
    "v_lshl_or_b32 %[nzc], %[t3], " #K ", %[nzc]\n"                                                               \
    "v_max_i32 %[" #HO "], %[h], %[" #FI "]\n"                                                                    \
    "v_subrev_u32 %[t], %[oedel], %[" #HO "]\n"                                                                   \
    "v_subrev_u32 %[t4], %[oeins], %[" #HO "]\n"                                                                  \
    "v_lshl_or_b32 %[t5], %[" #HO "], 10, " #K "\n"                                                               \
    "v_max3_i32 %[e], %[e], %[t], 0\n"                                                                            \
    "v_max3_i32 %[" #FO "], %[" #FO "], %[t4], 0\n"                                                               \
    "v_max_i32 %[kc], %[kc], %[t5]\n"                                                                             \
    "v_lshl_or_b32 %[" #EH "], %[e], 16, %[" #HI "]\n"
#define KSWL_MASK(B, K, EH, SV, HI, HO, FI, FO)                                                                   \
    "v_add_u32_sdwa %[h], sext(%[" #SV "]), %[" #EH "] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_" #B      \
    " src1_sel:WORD_0\n"                                                                                          \
    "v_sub_u32_sdwa %[e], %[" #EH "], %[edel] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n" \
    "v_add_u32 %[t2], " #K ", %[D]\n"                                                                             \
    "v_cmp_eq_u32 %[se], " #K ", %[je]\n"                                                                         \
    "v_max_i32_sdwa %[h], %[h], %[" #EH "] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n"  \
    "v_cmp_gt_u32 vcc, %[bw], %[t2]\n"                                                                            \
    "v_min_u32 %[t3], 1, %[" #HI "]\n"                                                                            \
    "v_subrev_u32 %[" #FO "], %[eins], %[" #FI "]\n"                                                              \
    "v_max_i32 %[h], %[h], %[" #FI "]\n"                                                                          \
    "v_lshl_or_b32 %[nzc], %[t3], " #K ", %[nzc]\n"                                                               \
    "v_cndmask_b32 %[" #EH "], %[" #EH "], %[" #HI "], %[se]\n"                                                   \
    "v_subrev_u32 %[t], %[oedel], %[h]\n"                                                                         \
    "v_subrev_u32 %[t4], %[oeins], %[h]\n"                                                                        \
    "v_lshl_or_b32 %[t5], %[h], 10, " #K "\n"                                                                     \
    "v_max3_i32 %[e], %[e], %[t], 0\n"                                                                            \
    "v_max3_i32 %[" #FO "], %[" #FO "], %[t4], 0\n"                                                               \
    "v_cndmask_b32 %[t5], -1, %[t5], vcc\n"                                                                       \
    "v_cndmask_b32 %[" #HO "], %[" #HI "], %[h], vcc\n"                                                           \
    "v_lshl_or_b32 %[e], %[e], 16, %[" #HI "]\n"                                                                  \
    "v_cndmask_b32 %[" #FO "], %[" #FI "], %[" #FO "], vcc\n"                                                     \
    "v_max_i32 %[kc], %[kc], %[t5]\n"                                                                             \
    "v_cndmask_b32 %[" #EH "], %[" #EH "], %[e], vcc\n"
#define KSWL_CELLS(M)                                   \
    M(0, 0, e0, sv0, h1, hb, f, fb)                     \
    M(1, 1, e1, sv0, hb, h1, fb, f)                     \
    M(2, 2, e2, sv0, h1, hb, f, fb)                     \
    M(3, 3, e3, sv0, hb, h1, fb, f)                     \
    M(0, 4, e4, sv1, h1, hb, f, fb)                     \
    M(1, 5, e5, sv1, hb, h1, fb, f)                     \
    M(2, 6, e6, sv1, h1, hb, f, fb)                     \
    M(3, 7, e7, sv1, hb, h1, fb, f)

template <int J0>
__device__ __forceinline__ void chunk8(uint32_t* eh, int& h1, int& f, int& key, uint32_t& nzw, uint32_t qw0,
                                       uint32_t qw1, uint32_t plo, uint32_t phi, int e_del, int oe_del, int e_ins,
                                       int oe_ins, int mode, int b0, int e0, int bw) {
    // the chunk's scores, its offsets from the band and the accumulators are
    // made inside the block: made outside, they were hoisted to the top of
    // the row for every chunk at once (three registers a chunk)
    int hb, fb, h, e, t, t2, t3, t4, t5, D, je, kc;
    uint32_t sv0, sv1, nzc;
    uint64_t se;
    asm volatile(
        "s_cmp_eq_u32 %[mode], 0\n"
        "s_cbranch_scc1 3f\n"
        "v_perm_b32 %[sv0], %[phi], %[plo], %[qw0]\n"
        "v_perm_b32 %[sv1], %[phi], %[plo], %[qw1]\n"
        "v_mov_b32 %[kc], -1\n"
        "v_mov_b32 %[nzc], 0\n"
#if KSWL_WHOLE_CHUNKS
        "s_cmp_eq_u32 %[mode], 1\n"
        "s_cbranch_scc0 2f\n"
        KSWL_CELLS(KSWL_FAST)
        "s_branch 4f\n"
        "2:\n"
#endif
        "v_sub_u32 %[D], %[J0], %[b0]\n"
        "v_subrev_u32 %[je], %[J0], %[e0v]\n"
        KSWL_CELLS(KSWL_MASK)
        "4:\n"
        "v_or_b32 %[kc], %[J0], %[kc]\n"
        "v_max_i32 %[key], %[key], %[kc]\n"
        "v_lshl_or_b32 %[nzw], %[nzc], %[SH], %[nzw]\n"
        "3:\n"
        : [e0] "+v"(eh[0]), [e1] "+v"(eh[1]), [e2] "+v"(eh[2]), [e3] "+v"(eh[3]), [e4] "+v"(eh[4]), [e5] "+v"(eh[5]),
          [e6] "+v"(eh[6]), [e7] "+v"(eh[7]), [h1] "+v"(h1), [f] "+v"(f), [key] "+v"(key), [nzw] "+v"(nzw),
          [kc] "=&v"(kc), [nzc] "=&v"(nzc),
          [hb] "=&v"(hb), [fb] "=&v"(fb), [h] "=&v"(h), [e] "=&v"(e), [t] "=&v"(t), [t2] "=&v"(t2), [t3] "=&v"(t3),
          [t4] "=&v"(t4), [t5] "=&v"(t5), [D] "=&v"(D), [je] "=&v"(je),
          [sv0] "=&v"(sv0), [sv1] "=&v"(sv1), [se] "=&s"(se)
        : [qw0] "v"(qw0), [qw1] "v"(qw1), [plo] "v"(plo), [phi] "v"(phi), [edel] "s"(e_del), [oedel] "s"(oe_del),
          [eins] "s"(e_ins), [oeins] "s"(oe_ins), [mode] "s"(mode), [J0] "i"(J0), [SH] "i"(J0 & 24), [b0] "v"(b0),
          [e0v] "v"(e0), [bw] "v"(bw)
        : "vcc", "scc");
}

// The lane engine: a wave's lanes each run ksw_extend2 problems one after
// the other, pulling tasks from a queue, so no lane waits for the longest
// problem of its wave (rows per problem vary several-fold: a related target
// runs to its end, an unrelated one stops at the z-drop).  Lanes whose
// problem ended idle until REFILL of them (or all) are idle, then claim tasks
// together (one atomic per wave) and set their column arrays up in one pass.
//
// Pol, per lane (called with only the lanes concerned active):
//   bool start<KCOL>(k, T, qs): set up task k of the queues (T: qlen, tlen, w,
//     end_bonus, zdrop, h0; qs: the wave's query slab, load_query_*) --
//     false: nothing to extend (the task's outputs are written, or it is
//     left to another path);
//   int tsym(i): the target symbol of row i of the lane's problem (0..4);
//   bool finish(r, T): the problem ended with r -- true: run it again with T
//     (same query and target, e.g. a wider band), false: the task is done.
// Queues q0 .. q1 - 1, taken in turn: queue q holds tasks bounds[q] ..
// bounds[q + 1] - 1 (the tasks sorted by query length, 16 columns per queue,
// so the lanes of a wave hold similar lengths and the chunks past them are
// skipped or, inside them, run whole), claimed through heads[q].
// stab: row_scores(mat, tc) as stab[2 tc], stab[2 tc + 1], in LDS; qs: the
// wave's query slab, KCOL / 8 x 64 uint2 of LDS.  stats (diagnostics, or
// nullptr): [0] wave rows, [1] live lane rows, [2] chunks run whole,
// [3] chunks run masked, [4] refills, [5] problems finished, summed.
template <int KCOL, int REFILL, class Pol>
__device__ __forceinline__ void lane_engine(Pol& pol, const uint32_t* bounds, uint32_t* heads, int q0, int q1,
                                            const uint32_t* stab, uint2* qs,
                                            int o_del, int e_del, int o_ins, int e_ins, int top,
                                            unsigned long long* stats = nullptr) {
    uint32_t st_rows = 0, st_lrows = 0, st_full = 0, st_mask = 0, st_refill = 0, st_done = 0;
    constexpr int NW = KCOL / 32 + 1;  // bit words over columns 0..KCOL
    const int lane = threadIdx.x & 63;
    const int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
    uint32_t EH[KCOL + 1];
    ExtIn T{0, 0, 0, 0, 0, 0};
    int h0 = 0, w = 0, i = 0, beg = 0, end = 0, tc_next = 0;
    int mx = 0, max_i = -1, max_j = -1, max_ie = -1, gscore = -1, max_off = 0;
    int phase = 0;      // 0: no problem (claims a task), 1: running, 2: set up to (re)start
    int q = q0;         // wave-uniform: the queue claimed from (q1: none left)
    uint32_t qlo = bounds[q0], qn = bounds[q0 + 1] - qlo;
    for (;;) {
        const uint64_t running = __ballot(phase == 1);
        const uint64_t idle = __ballot(phase != 1);
        if (idle && (__popcll(idle) >= REFILL || running == 0)) {
            ++st_refill;
            const uint64_t want = q < q1 ? __ballot(phase == 0) : 0ull;
            if (want) {  // one claim for the wave's idle lanes
                const int nw = __popcll(want);
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(heads + q, (uint32_t)nw);
                base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
                const uint32_t ql = qlo, qc = qn;
                if (base + (uint32_t)nw >= qc) {  // this queue is drained: the next one
                    for (++q; q < q1 && bounds[q + 1] == bounds[q]; ++q) {
                    }
                    if (q < q1) qlo = bounds[q], qn = bounds[q + 1] - qlo;
                }
                if (phase == 0) {
                    const uint32_t k = base + (uint32_t)__builtin_amdgcn_mbcnt_hi(
                                                  (uint32_t)(want >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)want, 0u));
                    if (k < qc && pol.template start<KCOL>(ql + k, T, qs)) phase = 2;
                }
            }
            if (phase == 2) {  // the first row and the band (software/ksw.c:389-406)
                h0 = T.h0 > 0 ? T.h0 : 0;
                init_row<KCOL>(EH, h0, h0 > oe_ins ? h0 - oe_ins : 0, e_ins);
                w = T.w;
                int lim = (int)((double)(T.qlen * top + T.end_bonus - o_ins) / e_ins + 1.);
                lim = imax(lim, 1);
                w = w < lim ? w : lim;
                lim = (int)((double)(T.qlen * top + T.end_bonus - o_del) / e_del + 1.);
                lim = imax(lim, 1);
                w = w < lim ? w : lim;
                mx = h0, max_i = -1, max_j = -1, max_ie = -1, gscore = -1, max_off = 0;
                i = 0, beg = 0, end = T.qlen;
                tc_next = T.tlen > 0 ? pol.tsym(0) : 0;
                phase = 1;
            }
        }
        if (__ballot(phase == 1) == 0 && q >= q1 && __ballot(phase == 2) == 0) break;
        // one row of every running lane's problem (one path through the loop
        // body: with a `continue` for the iterations that only claim, the
        // compiler kept two copies of the column array and moved one into
        // the other every row)
        const bool live = phase == 1 && i < T.tlen;
        bool done = phase == 1 && !live;  // no rows left (an empty target)
        ++st_rows;
        st_lrows += (uint32_t)__popcll(__ballot(live));
        {
            const int tc = tc_next;
            if (live && i + 1 < T.tlen) tc_next = pol.tsym(i + 1);  // the next row's symbol, loaded under this row
            const uint32_t plo = stab[2 * tc], phi = stab[2 * tc + 1];
            int h1 = h0 - (o_del + e_del * (i + 1));
            if (h1 < 0) h1 = 0;
            if (beg < i - w) beg = i - w;
            if (end > i + w + 1) end = i + w + 1;
            if (end > T.qlen) end = T.qlen;
            const int b0 = live ? beg : KCOL + 1, e0 = live ? end : -1;  // other lanes: an empty band, no end column
            int f = 0, key = -1;
            uint32_t NZ[NW];
#pragma unroll
            for (int k = 0; k < NW; ++k) NZ[k] = 0;
            const int bw = imax(e0 - b0, 0);  // column j is in the band iff (unsigned)(j - b0) < bw
            auto chunk = [&](auto cc) {
                constexpr int c = decltype(cc)::value, j0 = 8 * c;
                const bool any = __ballot(j0 <= e0 && j0 + 8 > imin(b0, e0)) != 0;  // a band or end column here
                const bool full = __ballot(live && !(b0 <= j0 && e0 >= j0 + 8)) == 0;  // every live band covers it
                const int mode = !any ? 0 : full ? 1 : 2;
                st_full += mode == 1, st_mask += mode == 2;
                const uint2 q2 = qs[c * 64 + lane];
                chunk8<j0>(&EH[j0], h1, f, key, NZ[c >> 2], q2.x, q2.y, plo, phi, e_del, oe_del, e_ins, oe_ins, mode,
                           b0, e0, bw);
            };
            for_chunks(chunk, std::make_integer_sequence<int, KCOL / 8>{});
            if (live && e0 == KCOL) {  // end column past the unrolled chunks
                EH[KCOL] = (uint32_t)h1;
                NZ[KCOL >> 5] |= nz1(h1) << (KCOL & 31);
            }
            if (live) {
                // row maximum m (0 when the band is empty) and its last column
                int m = 0, mj = -1;
                if (key >= 0) m = key >> 10, mj = key & 1023;
                if ((beg < end ? end : beg) == T.qlen) {  // the row reached the query end
                    max_ie = gscore > h1 ? max_ie : i;
                    gscore = gscore > h1 ? gscore : h1;
                }
                if (m == 0) {
                    done = true;
                } else if (m > mx) {
                    mx = m, max_i = i, max_j = mj;
                    const int o = mj > i ? mj - i : i - mj;
                    max_off = imax(max_off, o);
                } else if (T.zdrop > 0) {
                    const int di = i - max_i, dj = mj - max_j;
                    const int drop = di > dj ? mx - m - (di - dj) * e_del : mx - m - (dj - di) * e_ins;
                    done = drop > T.zdrop;
                }
                if (!done) {
                    // refit the band around mj (software/ksw.c:463-466): the
                    // last zero H in [beg, mj] and the first in [mj + 2, end]
                    int zlo = -1, zhi = -1;
#pragma unroll
                    for (int k = NW - 1; k >= 0; --k) {
                        const uint32_t zl = ~NZ[k] & range_bits(k, beg, mj);
                        if (zlo < 0 && zl) zlo = 32 * k + 31 - __builtin_clz(zl);
                    }
#pragma unroll
                    for (int k = 0; k < NW; ++k) {
                        const uint32_t zh = ~NZ[k] & range_bits(k, mj + 2, end);
                        if (zhi < 0 && zh) zhi = 32 * k + __builtin_ctz(zh);
                    }
                    beg = zlo >= 0 ? zlo + 1 : beg;
                    end = zhi >= 0 ? zhi : end + 1;
                    ++i;
                    done = i >= T.tlen;
                }
            }
        }
        st_done += (uint32_t)__popcll(__ballot(done));
        if (done) phase = pol.finish(KswResult{mx, max_j + 1, max_i + 1, max_ie + 1, gscore, max_off}, T) ? 2 : 0;
    }
    if (stats && lane == 0) {
        atomicAdd(stats + 0, (unsigned long long)st_rows);
        atomicAdd(stats + 1, (unsigned long long)st_lrows);
        atomicAdd(stats + 2, (unsigned long long)st_full);
        atomicAdd(stats + 3, (unsigned long long)st_mask);
        atomicAdd(stats + 4, (unsigned long long)st_refill);
        atomicAdd(stats + 5, (unsigned long long)st_done);
    }
}

}  // namespace kswl
}  // namespace smem
