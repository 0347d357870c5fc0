// smem_kernels.hip — CDNA4 (gfx950) kernels of the SMEM seeding engine.
//
// seed_kernel runs, per read, the whole seeding loop BWA-MEM runs on the CPU
// (software/bwamem.c:453-460 -> smem_next2 :244-305 -> bwt_smem1
// software/bwt.c:776-835 -> bwt_extend :416-429 -> bwt_2occ4/bwt_occ4
// :207-215/:187-204), bit-exact, with no host round trip per iteration.
//
// Execution model:
//  * persistent grid, one read per lane; a lane that finishes pulls the next
//    read from a global work counter, so the grid drains when every read is
//    taken (every lane reaches the exit test each time it is idle);
//  * each lane is a state machine whose every transition path ends in exactly
//    one bwt_extend, so all live lanes of a wave issue their Occ-bucket loads
//    from the same instruction each iteration (one reconvergence point per
//    extend instead of four nested loops diverging);
//  * the FM index stays resident in HBM in the reference's interleaved layout
//    (64-B bucket = 4 x u64 checkpoint + 8 x u32 of 2-bit symbols per 128
//    BWT symbols, software/bwt.h:72-73); rank inside a bucket is computed
//    with bit-plane popcounts (v_bcnt) instead of the 1 KB byte LUT;
//  * Occ buckets are fetched cooperatively: every wave-instruction moves 16
//    whole 64-B buckets (4 lanes x 16 B) into the wave's LDS image by LDS-DMA;
//  * the forward / prev / curr lists live in a per-lane scratch arena as
//    16-B packed entries, prev[j+1] prefetched while prev[j] is extended;
//  * matches are appended to the read's output region as bwt_smem1 emits
//    them; reversing and merging (software/bwt.c:830, software/bwamem.c:280-301)
//    happen in finalize_kernel, off the latency-bound loop.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "smem_kernels.h"

namespace smem {

// one 64-B Occ bucket: 4 x u64 checkpoint, 8 x u32 of 16 MSB-first 2-bit symbols
struct Bucket {
    uint4 c01, c23, w03, w47;
};

__device__ __forceinline__ Bucket load_bucket(const uint32_t* __restrict__ bwt, uint64_t kk) {
    const uint4* p = reinterpret_cast<const uint4*>(bwt + ((kk >> 7) << 4));
    return Bucket{p[0], p[1], p[2], p[3]};
}

// Counts of C, G, T among the first pos+1 symbols of the bucket's 8 words
// (MSB-first 2-bit symbols). A = pos+1 - C - G - T, which is what
// bwt_occ4's "masked tail reads as A, subtract ~k&15" produces.
__device__ __forceinline__ void count_cgt(const Bucket& v, uint32_t pos, uint32_t& C, uint32_t& G, uint32_t& T) {
    const uint32_t w[8] = {v.w03.x, v.w03.y, v.w03.z, v.w03.w, v.w47.x, v.w47.y, v.w47.z, v.w47.w};
    const uint32_t nfull = pos >> 4;
    const uint32_t tail = ~((1u << ((15u - (pos & 15u)) << 1)) - 1u);
    uint32_t sT = 0, sLo = 0, sHi = 0;
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) {
        const uint32_t m = i < nfull ? 0xFFFFFFFFu : (i == nfull ? tail : 0u);
        const uint32_t x = w[i] & m;
        const uint32_t lo = x & 0x55555555u;
        const uint32_t hi = (x >> 1) & 0x55555555u;
        sT += __popc(lo & hi);
        sLo += __popc(lo);
        sHi += __popc(hi);
    }
    T = sT;
    C = sLo - sT;
    G = sHi - sT;
}

__device__ __forceinline__ uint64_t cnt64(const uint4& v, int hi) {
    return hi ? ((uint64_t)v.w << 32 | v.z) : ((uint64_t)v.y << 32 | v.x);
}

__device__ __forceinline__ uint64_t sel4(int c, uint64_t a, uint64_t b, uint64_t d, uint64_t e) {
    return c == 0 ? a : (c == 1 ? b : (c == 2 ? d : e));
}

// ---- packed list entries (forward / prev / curr lists): 16 B instead of 32 B.
// x0, x1, x2 < 2^34 (seq_len checked on the host), query end < 2^26.
struct PIntv {
    uint32_t x0, x1, x2, hi;  // hi = x0>>32 | x1>>32 << 2 | x2>>32 << 4 | end << 6
};

__device__ __forceinline__ uint4 pack_p(uint64_t x0, uint64_t x1, uint64_t x2, uint32_t end) {
    return make_uint4((uint32_t)x0, (uint32_t)x1, (uint32_t)x2,
                      (uint32_t)(x0 >> 32) | (uint32_t)(x1 >> 32) << 2 | (uint32_t)(x2 >> 32) << 4 | end << 6);
}

__device__ __forceinline__ uint4 load_p(const PIntv* p) { return *reinterpret_cast<const uint4*>(p); }
__device__ __forceinline__ uint64_t p_x0(const uint4& v) { return (uint64_t)(v.w & 3) << 32 | v.x; }
__device__ __forceinline__ uint64_t p_x1(const uint4& v) { return (uint64_t)((v.w >> 2) & 3) << 32 | v.y; }
__device__ __forceinline__ uint64_t p_x2(const uint4& v) { return (uint64_t)((v.w >> 4) & 3) << 32 | v.z; }
__device__ __forceinline__ uint32_t p_end(const uint4& v) { return v.w >> 6; }

// ---- query bases through a 16-byte register window (one load per 16 bases)
__device__ __forceinline__ int qget(const uint8_t* __restrict__ codes, uint64_t o0, int i, uint4& qv, uint64_t& qb) {
    const uint64_t a = o0 + (uint64_t)i;
    const uint64_t blk = a & ~15ull;
    if (blk != qb) {
        qv = *reinterpret_cast<const uint4*>(codes + blk);
        qb = blk;
    }
    const uint32_t sel = (uint32_t)(a >> 2) & 3;
    const uint32_t w = sel == 0 ? qv.x : (sel == 1 ? qv.y : (sel == 2 ? qv.z : qv.w));
    return (int)((w >> ((a & 3) * 8)) & 0xff);
}

enum Phase : int {
    P_BWD_RES = 0,  // consume a backward extend        (software/bwt.c:815-825)
    P_BWD_J,        // next prev[j] / end of a step      (software/bwt.c:812, 827-828)
    P_FWD_RES,      // consume a forward extend          (software/bwt.c:795-799)
    P_FWD,          // next forward position             (software/bwt.c:791-803)
    P_FWD_DONE,     // reverse + ret                     (software/bwt.c:805-808)
    P_BWD_STEP,     // start backward position i         (software/bwt.c:810-812)
    P_SMEM_END,     // end of one bwt_smem1              (software/bwamem.c:261-278)
    P_OVF,          // output capacity exceeded: hand the read to the overflow pass
    P_NEXT2,        // start of one smem_next2 call      (software/bwamem.c:247-258)
    P_SMEM_BEGIN,   // start of one bwt_smem1            (software/bwt.c:782-789)
    P_FETCH,        // next read from the work counter
    P_EXIT
};

constexpr uint32_t NO_BUCKET = 0xFFFFFFFFu;

// LDS image of the wave's Occ buckets: [wave][k|l][lane][4 x 16 B]
struct WaveLds {
    uint4 k[64][4];
    uint4 l[64][4];
};

// Fetch the 64-B Occ buckets of every live lane.  COOP: each wave-instruction
// moves 16 whole buckets (4 lanes x 16 B per bucket, one L1 access each)
// straight into the wave's LDS image with LDS-DMA; the owner lane then reads
// its bucket from LDS.  !COOP: each lane loads its own bucket (4 x 16 B).
template <bool COOP>
__device__ __forceinline__ void fetch_buckets(const uint32_t* __restrict__ bwt, WaveLds* W, int lane, bool want,
                                              uint64_t kk, uint64_t ll, Bucket& vk, Bucket& vl) {
    const bool needl = want && (kk >> 7) != (ll >> 7);
    if constexpr (COOP) {
        const uint32_t bk = want ? (uint32_t)(kk >> 7) : NO_BUCKET;
        const uint32_t bl = needl ? (uint32_t)(ll >> 7) : NO_BUCKET;
        const uint32_t chunk = (uint32_t)(lane & 3) * 4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t s = __shfl(bk, 16 * r + (lane >> 2));
            if (s != NO_BUCKET)
                __builtin_amdgcn_global_load_lds(bwt + (uint64_t)s * 16 + chunk,
                                                 (__attribute__((address_space(3))) void*)&W->k[16 * r][0], 16, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t s = __shfl(bl, 16 * r + (lane >> 2));
            if (s != NO_BUCKET)
                __builtin_amdgcn_global_load_lds(bwt + (uint64_t)s * 16 + chunk,
                                                 (__attribute__((address_space(3))) void*)&W->l[16 * r][0], 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        vk = Bucket{W->k[lane][0], W->k[lane][1], W->k[lane][2], W->k[lane][3]};
        const int ls = needl ? 1 : 0;  // read the l image only where it was fetched
        const uint4* src = ls ? &W->l[lane][0] : &W->k[lane][0];
        vl = Bucket{src[0], src[1], src[2], src[3]};
    } else if (want) {
        // per-lane: the l bucket is loaded again even when it equals k (an L1 hit)
        vk = load_bucket(bwt, kk);
        vl = load_bucket(bwt, needl ? ll : kk);
    }
}

// One bwt_extend in one direction, returning only the child for base c,
// from the two Occ buckets of k = a-1 and l = k+s.
//   a: coordinate searched through the BWT (x[1] forward, x[0] backward)
//   b: the other coordinate, s: interval size
//   -> na = L2[c] + 1 + Occ(c, a-1), ns = Occ(c, a-1+s) - Occ(c, a-1),
//      nb = b + [$ in interval] + sum_{c' > c} (Occ(c', a-1+s) - Occ(c', a-1))
// (software/bwt.c:416-429; the four-way cumulative in :425-428 restricted
// to the child actually taken).
__device__ __forceinline__ void extend_counts(const SeedParams& P, uint64_t a, uint64_t b, uint64_t s, int c,
                                              uint64_t kk, uint64_t ll, const Bucket& vk, const Bucket& vl,
                                              uint64_t& na, uint64_t& nb, uint64_t& ns) {
    uint32_t Ck, Gk, Tk, Cl, Gl, Tl;
    const uint32_t pk = (uint32_t)(kk & 127), pl = (uint32_t)(ll & 127);
    count_cgt(vk, pk, Ck, Gk, Tk);
    count_cgt(vl, pl, Cl, Gl, Tl);
    const uint32_t Ak = pk + 1 - Ck - Gk - Tk, Al = pl + 1 - Cl - Gl - Tl;
    const uint64_t tk0 = cnt64(vk.c01, 0) + Ak, tk1 = cnt64(vk.c01, 1) + Ck;
    const uint64_t tk2 = cnt64(vk.c23, 0) + Gk, tk3 = cnt64(vk.c23, 1) + Tk;
    const uint64_t tl0 = cnt64(vl.c01, 0) + Al, tl1 = cnt64(vl.c01, 1) + Cl;
    const uint64_t tl2 = cnt64(vl.c23, 0) + Gl, tl3 = cnt64(vl.c23, 1) + Tl;
    const uint64_t d0 = tl0 - tk0, d1 = tl1 - tk1, d2 = tl2 - tk2, d3 = tl3 - tk3;
    const uint64_t L2c = sel4(c, P.L2[0], P.L2[1], P.L2[2], P.L2[3]);
    na = L2c + 1 + sel4(c, tk0, tk1, tk2, tk3);
    ns = sel4(c, d0, d1, d2, d3);
    const uint64_t gt = (c < 1 ? d1 : 0) + (c < 2 ? d2 : 0) + (c < 3 ? d3 : 0);
    nb = b + (uint64_t)(a <= P.primary && a + s - 1 >= P.primary) + gt;
}

// Overwrite the query window with the 16-byte block holding position pos,
// ahead of its use, so the load is in flight with this iteration's buckets.
__device__ __forceinline__ void qprefetch(const uint8_t* __restrict__ codes, uint64_t o0, int pos, uint4& qv,
                                          uint64_t& qb) {
    const uint64_t blk = (o0 + (uint64_t)pos) & ~15ull;
    if (blk != qb) {
        qv = *reinterpret_cast<const uint4*>(codes + blk);
        qb = blk;
    }
}

template <bool COOP>
__global__ __launch_bounds__(256, 4) void seed_kernel(SeedParams P) {
    __shared__ WaveLds lds[COOP ? 4 : 1];  // COOP: 4 waves per 256-thread block, 8 KB each
    const int lane = threadIdx.x & 63;
    WaveLds* W = &lds[COOP ? (threadIdx.x >> 6) : 0];
    const uint64_t lane_g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t cap = P.cap_list;
    // per-lane scratch: two packed lists (B0 | B1) used as forward / prev / curr
    PIntv* __restrict__ bp = reinterpret_cast<PIntv*>(P.scratch + lane_g * 2ull * cap);

    int phase = P_FETCH;
    int item = -1, len = 0;
    uint64_t o0 = 0, qb = ~0ull;
    uint4 qv = {0, 0, 0, 0};
    uint32_t raw_n = 0, calls_n = 0;   // raw intervals / lists logged for the read
    int start = 0, ori_start = 0, split_len = 0;
    int x = 0, min_intv = 1, middle = 0, i = 0, j = 0, ret = 0, cur_c = 0;
    uint64_t ik0 = 0, ik1 = 0, ik2 = 0;
    uint32_t ikend = 0;
    uint32_t fwd_n = 0, prev_off = 0, prev_n = 0, curr_off = 0, curr_n = 0;
    uint32_t mem_n = 0, mem_last_start = 0, m_n = 0;
    uint64_t curr_last_x2 = 0;
    // longest match of the first bwt_smem1 (software/bwamem.c:266-270), tracked
    // as matches are emitted: pushes come in reverse final order, so ">="
    // keeps the first maximum in final order
    uint32_t max_len = 0;
    uint64_t max_x2 = 0, max_info = 0;
    uint4 pc = {0, 0, 0, 0}, pn = {0, 0, 0, 0}, head = {0, 0, 0, 0};
    uint64_t na = 0, nb = 0, ns = 0;

    for (;;) {
        // ---- advance the state machine until the lane needs an extend ----
        // one transition per pass (every block ends in continue/break: this
        // keeps the register allocation at 4 waves/SIMD); blocks are ordered
        // by frequency
        while (phase != P_EXIT) {
            if (phase == P_BWD_RES) {  // na = x[0], nb = x[1]
                if (ns < (uint64_t)min_intv) {
                    // only prev[0] can be kept, when nothing longer survived
                    if (curr_n == 0 && (mem_n == 0 || (uint32_t)(i + 1) < mem_last_start)) {
                        if (raw_n >= P.cap_intv) {
                            phase = P_OVF;
                        } else {
                            const uint64_t info = (uint64_t)p_end(pc) | ((uint64_t)(i + 1) << 32);
                            P.out_intv[(uint64_t)item * P.cap_intv + raw_n++] = Intv{p_x0(pc), p_x1(pc), p_x2(pc), info};
                            ++mem_n;
                            mem_last_start = (uint32_t)(i + 1);
                            if (!middle && p_end(pc) - (uint32_t)(i + 1) >= max_len) {
                                max_len = p_end(pc) - (uint32_t)(i + 1);
                                max_x2 = p_x2(pc);
                                max_info = info;
                            }
                        }
                    }
                } else if (curr_n == 0 || ns != curr_last_x2) {
                    const uint4 e = pack_p(na, nb, ns, p_end(pc));
                    *reinterpret_cast<uint4*>(bp + curr_off + curr_n) = e;
                    if (curr_n == 0) head = e;  // prev[0] of the next step
                    ++curr_n;
                    curr_last_x2 = ns;
                }
                ++j;
                if (phase != P_OVF) phase = P_BWD_J;
                continue;
            }
            if (phase == P_BWD_J) {
                if ((uint32_t)j < prev_n) {
                    pc = pn;
                    if ((uint32_t)j + 1 < prev_n) pn = load_p(bp + prev_off + j + 1);  // prefetch prev[j+1]
                    if (j == 0 && i > 0 && !(P.dbg & 1)) qprefetch(P.codes, o0, i - 1, qv, qb);       // next step's base
                    phase = P_BWD_RES;
                    break;  // -> extend (backward)
                }
                if (curr_n == 0) {
                    phase = P_SMEM_END;  // software/bwt.c:827
                } else {
                    prev_off = curr_off;
                    prev_n = curr_n;
                    pn = (P.dbg & 2) ? load_p(bp + curr_off) : head;  // curr[0], kept in registers
                    curr_off = curr_off == cap ? 0 : cap;
                    --i;
                    phase = P_BWD_STEP;
                }
                continue;
            }
            if (phase == P_FWD_RES) {  // na = x[1], nb = x[0]
                bool stop = false;
                if (ns != ik2) {
                    *reinterpret_cast<uint4*>(bp + cap - 1 - fwd_n) = pack_p(ik0, ik1, ik2, ikend);
                    ++fwd_n;
                    stop = ns < (uint64_t)min_intv;
                }
                if (stop) {
                    phase = P_FWD_DONE;
                } else {
                    ik0 = nb; ik1 = na; ik2 = ns;
                    ikend = (uint32_t)(i + 1);
                    ++i;
                    phase = P_FWD;
                }
                continue;
            }
            if (phase == P_FWD) {
                if (i < len) {
                    const int qi = qget(P.codes, o0, i, qv, qb);
                    if (qi < 4) {
                        cur_c = 3 - qi;
                        if (i + 1 < len && !(P.dbg & 1)) qprefetch(P.codes, o0, i + 1, qv, qb);
                        phase = P_FWD_RES;
                        break;  // -> extend (forward)
                    }
                }
                // ambiguous base, or end of query: push ik and stop
                *reinterpret_cast<uint4*>(bp + cap - 1 - fwd_n) = pack_p(ik0, ik1, ik2, ikend);
                ++fwd_n;
                phase = P_FWD_DONE;
                continue;
            }
            if (phase == P_FWD_DONE) {
                // the last push becomes prev[0] after the reversal; it is always the
                // current ik (the stop path pushes ik without advancing it)
                pn = (P.dbg & 2) ? load_p(bp + cap - fwd_n) : pack_p(ik0, ik1, ik2, ikend);
                ret = (int)p_end(pn);
                prev_off = cap - fwd_n;  // pushed downward: ascending = reversed
                prev_n = fwd_n;
                curr_off = cap;
                i = x - 1;
                phase = P_BWD_STEP;
                continue;
            }
            if (phase == P_BWD_STEP) {
                cur_c = i < 0 ? -1 : qget(P.codes, o0, i, qv, qb);
                if (cur_c > 3) cur_c = -1;
                curr_n = 0;
                if (cur_c < 0) {
                    // nothing extends: prev[0] (= pn) is the only candidate
                    if (mem_n == 0 || (uint32_t)(i + 1) < mem_last_start) {
                        if (raw_n >= P.cap_intv) {
                            phase = P_OVF;
                        } else {
                            const uint64_t info = (uint64_t)p_end(pn) | ((uint64_t)(i + 1) << 32);
                            P.out_intv[(uint64_t)item * P.cap_intv + raw_n++] = Intv{p_x0(pn), p_x1(pn), p_x2(pn), info};
                            ++mem_n;
                            mem_last_start = (uint32_t)(i + 1);
                            if (!middle && p_end(pn) - (uint32_t)(i + 1) >= max_len) {
                                max_len = p_end(pn) - (uint32_t)(i + 1);
                                max_x2 = p_x2(pn);
                                max_info = info;
                            }
                        }
                    }
                    if (phase != P_OVF) phase = P_SMEM_END;
                } else {
                    j = 0;
                    phase = P_BWD_J;
                    continue;
                }
                continue;
            }
            if (phase == P_SMEM_END) {
                if (!middle) {  // software/bwamem.c:261-272
                    start = ret;
                    m_n = mem_n;
                    if (m_n > 0 && split_len > 0 && (int)max_len >= split_len &&
                        max_x2 <= (uint64_t)(int64_t)P.split_width) {
                        // re-seed from the middle of the longest SMEM (software/bwamem.c:272-278)
                        x = (int)(((uint64_t)(uint32_t)max_info + (max_info >> 32)) >> 1);
                        min_intv = (int)(max_x2 + 1);
                        middle = 1;
                        phase = P_SMEM_BEGIN;
                        continue;
                    }
                }
                // log the list: matches (+ sub-matches) for the finalize pass
                if (calls_n >= P.cap_calls) {
                    phase = P_OVF;
                } else {
                    P.out_call[(uint64_t)item * P.cap_calls + calls_n++] =
                        CallRec{m_n, middle ? mem_n : 0u, (uint32_t)ori_start, max_len};
                    phase = P_NEXT2;
                }
                continue;
            }
            if (phase == P_OVF) {  // the read does not fit: hand it to the overflow pass
                P.n_intv[item] = SMEM_OVERFLOW;
                P.n_calls[item] = 0;
                const int slot = atomicAdd(P.ovf_count, 1);
                P.ovf_items[slot] = item;
                phase = P_FETCH;
                continue;
            }
            if (phase == P_NEXT2) {  // software/bwamem.c:247-261
                if (start < len && start >= 0)
                    while (start < len && qget(P.codes, o0, start, qv, qb) > 3) ++start;  // skip ambiguous bases
                if (start >= len || start < 0) {                                         // iterator exhausted
                    P.n_intv[item] = raw_n;
                    P.n_calls[item] = calls_n;
                    phase = P_FETCH;
                } else {
                    ori_start = start;
                    x = ori_start;
                    min_intv = P.start_width;
                    middle = 0;
                    max_len = 0;
                    phase = P_SMEM_BEGIN;
                }
                continue;
            }
            if (phase == P_SMEM_BEGIN) {  // software/bwt.c:782-789
                mem_n = 0;
                const int qx = qget(P.codes, o0, x, qv, qb);
                if (qx > 3) {
                    ret = x + 1;
                    phase = P_SMEM_END;
                    continue;
                }
                if (min_intv < 1) min_intv = 1;
                ik0 = P.L2[qx] + 1;
                ik2 = P.L2[qx + 1] - P.L2[qx];
                ik1 = P.L2[3 - qx] + 1;
                ikend = (uint32_t)(x + 1);
                fwd_n = 0;
                i = x + 1;
                phase = P_FWD;
                continue;
            }
            if (phase == P_FETCH) {
                item = atomicAdd(P.head, 1);
                if (item >= P.n_items) {
                    phase = P_EXIT;
                    break;
                }
                const int rid = P.read_ids ? P.read_ids[item] : item;
                o0 = P.offs[rid];
                len = (int)(P.offs[rid + 1] - o0);
                raw_n = 0;
                calls_n = 0;
                start = 0;
                if (len < P.min_seed_len) {  // mem_chain's guard (software/bwamem.c:600)
                    P.n_intv[item] = 0;
                    P.n_calls[item] = 0;
                    continue;
                }
                split_len = P.split_len_init < len ? P.split_len_init : len;  // software/bwamem.c:456-458
                phase = P_NEXT2;
            }
        }
        // ---- one bwt_extend per live lane; the loop exit is wave-uniform so
        // every lane takes part in the cooperative bucket fetch ----
        const bool want = phase != P_EXIT;
        if (!__any(want)) break;
        // the interval to extend: ik forward (a = x[1]), prev[j] backward (a = x[0])
        const bool fwd = phase == P_FWD_RES;
        const uint64_t ra = fwd ? ik1 : p_x0(pc), rb = fwd ? ik0 : p_x1(pc), rs = fwd ? ik2 : p_x2(pc);
        const uint64_t k = ra - 1, l = k + rs;
        const uint64_t kk = k - (k >= P.primary), ll = l - (l >= P.primary);
        Bucket vk, vl;
        fetch_buckets<COOP>(P.bwt, W, lane, want, kk, ll, vk, vl);
        if (want) extend_counts(P, ra, rb, rs, cur_c, kk, ll, vk, vl, na, nb, ns);
    }
}

// Raw logs -> the lists smem_next2 returns: reverse each bwt_smem1 output
// (software/bwt.c:830) and merge matches with sub-matches keyed by
// (start, len - end), keeping a sub-match only if it is at least half the
// longest match and ends after the call's start (software/bwamem.c:280-301).
// One thread per read; WRITE=false computes the sizes, WRITE=true writes them.
template <bool WRITE>
__global__ __launch_bounds__(256) void finalize_kernel(FinalizeParams F) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= F.n) return;
    const Intv* raw = F.main_intv + (uint64_t)r * F.cap_intv;
    const CallRec* rec = F.main_call + (uint64_t)r * F.cap_calls;
    uint32_t nc = F.n_calls[r];
    if (F.n_intv[r] == SMEM_OVERFLOW) {
        const int s = F.ovf_slot[r];
        raw = F.ovf_intv + (uint64_t)s * F.ovf_cap_intv;
        rec = F.ovf_call + (uint64_t)s * F.ovf_cap_calls;
        nc = F.ovf_n_calls[s];
    }
    const uint32_t len = (uint32_t)(F.offs[r + 1] - F.offs[r]);
    uint64_t out = WRITE ? F.intv_off[r] : 0, total = 0;
    const uint64_t cout = WRITE ? F.call_off[r] : 0;
    uint32_t pos = 0;
    for (uint32_t c = 0; c < nc; ++c) {
        const CallRec cr = rec[c];
        const Intv* M = raw + pos;           // M[m_n-1-a] is the a-th match in final order
        const Intv* S = raw + pos + cr.m_n;  // likewise for sub-matches
        const uint64_t half = (uint64_t)(cr.max_len >> 1);
        uint32_t a = 0, b = 0, n = 0;
        while (a < cr.m_n && b < cr.s_n) {
            const Intv ma = M[cr.m_n - 1 - a], sb = S[cr.s_n - 1 - b];
            const uint64_t xi = (ma.info >> 32 << 32) | (uint64_t)(uint32_t)(len - (uint32_t)ma.info);
            const uint64_t xj = (sb.info >> 32 << 32) | (uint64_t)(uint32_t)(len - (uint32_t)sb.info);
            if ((int64_t)xi < (int64_t)xj) {
                if (WRITE) F.flat_intv[out + n] = ma;
                ++n;
                ++a;
            } else {
                if ((uint64_t)(uint32_t)sb.info - (sb.info >> 32) >= half && (uint32_t)sb.info > cr.ori_start) {
                    if (WRITE) F.flat_intv[out + n] = sb;
                    ++n;
                }
                ++b;
            }
        }
        for (; a < cr.m_n; ++a) {
            if (WRITE) F.flat_intv[out + n] = M[cr.m_n - 1 - a];
            ++n;
        }
        for (; b < cr.s_n; ++b) {
            const Intv sb = S[cr.s_n - 1 - b];
            if ((uint64_t)(uint32_t)sb.info - (sb.info >> 32) >= half && (uint32_t)sb.info > cr.ori_start) {
                if (WRITE) F.flat_intv[out + n] = sb;
                ++n;
            }
        }
        if (WRITE) F.flat_calls[cout + c] = n;
        out += n;
        total += n;
        pos += cr.m_n + cr.s_n;
    }
    if (!WRITE) {
        F.s_intv[r] = total;
        F.s_calls[r] = nc;
    }
}

__global__ void fill_i32_kernel(int32_t* p, int32_t v, int n) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < n) p[r] = v;
}

__global__ void ovf_slot_kernel(const int32_t* __restrict__ items, int n_ovf, int32_t* __restrict__ ovf_slot) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < n_ovf) ovf_slot[items[s]] = s;
}

}  // namespace smem

// ------------------------------------------------------------ host launchers
extern "C" hipError_t smem_launch_seed(const smem::SeedParams* P, int grid, int block, int variant, hipStream_t st) {
    if (variant == 1)
        hipLaunchKernelGGL(smem::seed_kernel<false>, dim3(grid), dim3(block), 0, st, *P);
    else
        hipLaunchKernelGGL(smem::seed_kernel<true>, dim3(grid), dim3(block), 0, st, *P);
    return hipGetLastError();
}

extern "C" hipError_t smem_launch_finalize(const smem::FinalizeParams* F, int write, hipStream_t st) {
    if (F->n <= 0) return hipSuccess;
    const unsigned g = (unsigned)((F->n + 255) / 256);
    if (write)
        hipLaunchKernelGGL(smem::finalize_kernel<true>, dim3(g), dim3(256), 0, st, *F);
    else
        hipLaunchKernelGGL(smem::finalize_kernel<false>, dim3(g), dim3(256), 0, st, *F);
    return hipGetLastError();
}

extern "C" hipError_t smem_launch_fill_i32(int32_t* p, int32_t v, int n, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(smem::fill_i32_kernel, dim3((n + 255) / 256), dim3(256), 0, st, p, v, n);
    return hipGetLastError();
}

extern "C" hipError_t smem_launch_ovf_slot(const int32_t* items, int n_ovf, int32_t* ovf_slot, hipStream_t st) {
    if (n_ovf <= 0) return hipSuccess;
    hipLaunchKernelGGL(smem::ovf_slot_kernel, dim3((n_ovf + 255) / 256), dim3(256), 0, st, items, n_ovf, ovf_slot);
    return hipGetLastError();
}

// ---------------------------------------------------------------- scans
#include <hipcub/hipcub.hpp>

// out[0] = 0, out[1..n] = inclusive sums of in[0..n-1]; temp == nullptr
// queries the temporary size into *temp_bytes
extern "C" hipError_t smem_launch_offsets(const uint64_t* in, uint64_t* out, int n, void* temp, size_t* temp_bytes,
                                          hipStream_t st) {
    if (temp == nullptr) return hipcub::DeviceScan::InclusiveSum(nullptr, *temp_bytes, in, out + 1, n > 0 ? n : 1, st);
    hipError_t e = hipMemsetAsync(out, 0, sizeof(uint64_t), st);
    if (e != hipSuccess || n <= 0) return e;
    return hipcub::DeviceScan::InclusiveSum(temp, *temp_bytes, in, out + 1, n, st);
}
