// Chains -> alignment regions on gfx950: the loop of
// mem_align1_core over a read's chains (software/bwamem.c:1452-1460), each
// chain through mem_chain2aln_short (software/bwamem.c:805-852, ksw_align2)
// and, when that declines, mem_chain2aln (software/bwamem.c:1040-1188, two
// ksw_extend2 calls per extended seed), over the chains smem_batch_chain left
// in HBM and the .pac resident beside the index.
//
// One wave per read: a read's regions depend on each other (every seed is
// first tested for containment in the regions made before it, from this and
// earlier chains), so the wave walks its chains and seeds in the reference's
// order and spreads the work inside each step over its 64 lanes:
//   * the per-seed scans (reference span, containment in earlier regions,
//     overlap with longer seeds, seed coverage) run one region or seed per
//     lane and end in a ballot or a reduction;
//   * the seed order (ks_introsort_64 of len << 32 | index, distinct keys) is
//     each key's rank among the chain's keys, by lanes;
//   * every ksw_extend2 / ksw_align2 runs on the whole wave (ksw_device.h),
//     the reference fetched from the 2-bit .pac per row (bns_get_seq).
// Reads up to 256 bp go to aln_kernel<4> (query columns in 4 registers per
// lane), longer ones (up to 1024 bp) to aln_kernel<16>.
#include <algorithm>
#include <hipcub/hipcub.hpp>

#include "aln_kernels.h"
#include "ksw_device.h"
#include "ksw_lane.h"

namespace smem {
namespace {

__device__ __forceinline__ int pac_at(const uint8_t* pac, int64_t l) {
    return pac[l >> 2] >> ((~l & 3) << 1) & 3;  // _get_pac (software/bntseq.h)
}

// symbol p of the forward-reverse text (bns_get_seq, software/bntseq.c:355-376,
// over a span that does not bridge the strands)
__device__ __forceinline__ int ref_at(const AlnParams& P, int64_t p) {
    return p < P.l_pac ? pac_at(P.pac, p) : 3 - pac_at(P.pac, (P.l_pac << 1) - 1 - p);
}

// cal_max_gap (software/bwamem.c:854-861) in integers: (int)(x / e + 1.) with
// x = qlen a - o is trunc(x / e + 1) = (x + e) / e (C division truncates; the
// double quotient is exact when e divides x and otherwise at least 1/e from
// an integer, far past its rounding), without the double divisions (a
// containment test of the heavy-read walk makes two per region)
__device__ __forceinline__ int gap_div(int x, int e) { return e == 1 ? x + 1 : (x + e) / e; }
__device__ __forceinline__ int max_gap(const AlnParams& P, int qlen) {
    const int l_del = gap_div(qlen * P.a - P.o_del, P.e_del);
    const int l_ins = gap_div(qlen * P.a - P.o_ins, P.e_ins);
    int l = l_del > l_ins ? l_del : l_ins;
    l = l > 1 ? l : 1;
    return l < P.w << 1 ? l : P.w << 1;
}

__device__ __forceinline__ int64_t wmin64(int64_t v) {
    for (int o = 32; o; o >>= 1) {
        const int64_t t = __shfl_xor(v, o);
        v = t < v ? t : v;
    }
    return v;
}
__device__ __forceinline__ int64_t wmax64(int64_t v) {
    for (int o = 32; o; o >>= 1) {
        const int64_t t = __shfl_xor(v, o);
        v = t > v ? t : v;
    }
    return v;
}
__device__ __forceinline__ int wsum(int v) {
    for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l) |
           (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), l) << 32;
}
// A wave-uniform value in an SGPR.  Loop bounds of the wave-cooperative
// loops go through this: a bound the compiler keeps in a VGPR makes the loop
// exit a per-lane compare, and a loop with an exit of that shape hung gfx950
// waves (the seed-order loop of the heavy-read walk spun with no lane left
// to leave it).
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v) |
           (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32;
}

// Diagnostics (SMEM_ALN_SPLIT, aln_kernel<KC, true>): shader cycles of each
// phase of a read summed per wave, and counts.  t[k]:
//   0 read setup, 1 chain load + mem_chain2aln_short, 2 chain span + seed
//   order, 3 containment tests, 4 left extensions, 5 right extensions,
//   6 seed coverage + region store, 7 claims;
//   8 reads, 9 chains, 10 short regions, 11 seed regions, 12 left / 13 right
//   extension calls, 14 extension rows walked, 15 waves.
struct Split {
    uint64_t last;
    uint64_t t[ALN_SPLITS];
};
__device__ __forceinline__ void stamp(Split* sp, int k) {
    if (sp) {
        const uint64_t t = __builtin_amdgcn_s_memtime();
        sp->t[k] += t - sp->last;
        sp->last = t;
    }
}
__device__ __forceinline__ void count(Split* sp, int k) {
    if (sp) ++sp->t[k];
}

// mem_chain2aln_short (software/bwamem.c:805-852): 0 when it wrote region
// *out, 1 when it declines (then mem_chain2aln runs).  One exit: the
// declines are flags, not early returns (an early return out of this wave-
// cooperative body, inlined into a persistent loop, hung gfx950 waves).
__device__ __forceinline__ int chain_short(const AlnParams& P, const uint8_t* query, int L, const SeedRec* S, int n,
                                           AlnReg* out, int lane, uint32_t* sw_ctr = nullptr) {
    int64_t qb = L, qe = 0, rb = P.l_pac << 1, re = 0;
    int cov = 0;
    for (int i = lane; i < n; i += 64) {
        const SeedRec s = S[i];
        qb = s.qbeg < qb ? s.qbeg : qb;
        qe = s.qbeg + s.len > qe ? s.qbeg + s.len : qe;
        rb = s.rbeg < rb ? s.rbeg : rb;
        re = s.rbeg + s.len > re ? s.rbeg + s.len : re;
        cov += s.len;
    }
    cov = wsum(cov);
    qb = wmin64(qb) - 50, qe = wmax64(qe) + 50;  // MEM_SHORT_EXT
    rb = wmin64(rb) - 50, re = wmax64(re) + 50;
    bool decline = qb <= 10 || qe >= L - 10;
    rb = rb > 0 ? rb : 0;
    re = re < P.l_pac << 1 ? re : P.l_pac << 1;
    if (rb < P.l_pac && P.l_pac < re) {
        if (S[0].rbeg < P.l_pac) re = P.l_pac;
        else rb = P.l_pac;
    }
    decline = decline || (re - rb) - (qe - qb) > 50 || (qe - qb) - (re - rb) > 50;
    decline = decline || qe - qb >= P.w * 4 || re - rb >= P.w * 4;
    decline = decline || qe - qb >= 200 || re - rb >= 200;  // MEM_SHORT_LEN
    if (!decline) {
        if (sw_ctr && lane == 0) atomicAdd(sw_ctr, 1u);  // SMEM_ALN_STATS: chains that run the SW
        const int ql = (int)(qe - qb), tl = (int)(re - rb);
        const int xtra =
            kswd::SW_XSUBO | kswd::SW_XSTART | (ql * P.a < 250 ? kswd::SW_XBYTE : 0) | (P.min_seed_len * P.a);
        const uint8_t* qw = query + qb;
        const int64_t r0 = rb;
        const kswd::SwAlign x = kswd::sw_align_wave(
            ql, [&](int q) { return (int)qw[q]; }, tl, [&](int i) { return ref_at(P, r0 + i); }, P.mat, P.o_del,
            P.e_del, P.o_ins, P.e_ins, xtra, P.sw_shift, P.top);
        decline = x.tb < 25 || x.te > tl - 25;
        if (!decline && lane == 0) {
            AlnReg a;
            a.rb = rb + x.tb, a.re = rb + x.te + 1;
            a.qb = (int)qb + x.qb, a.qe = (int)qb + x.qe + 1;
            a.score = x.score, a.truesc = 0, a.sub = 0, a.csub = x.score2, a.sub_n = 0, a.w = 0, a.seedcov = cov;
            a.secondary = 0, a.hash = 0;
            *out = a;
        }
    }
    return decline ? 1 : 0;
}

// the span of reference any extension of the chain may reach (software/bwamem.c:1050-1065)
__device__ __forceinline__ void chain_span(const AlnParams& P, int L, const SeedRec* S, int n, int lane, int64_t& r0, int64_t& r1) {
    r0 = P.l_pac << 1, r1 = 0;
    for (int i = lane; i < n; i += 64) {
        const SeedRec t = S[i];
        const int64_t b = t.rbeg - (t.qbeg + max_gap(P, t.qbeg));
        const int64_t e = t.rbeg + t.len + ((L - t.qbeg - t.len) + max_gap(P, L - t.qbeg - t.len));
        r0 = b < r0 ? b : r0;
        r1 = e > r1 ? e : r1;
    }
    r0 = wmin64(r0), r1 = wmax64(r1);
    r0 = r0 > 0 ? r0 : 0;
    r1 = r1 < P.l_pac << 1 ? r1 : P.l_pac << 1;
    if (r0 < P.l_pac && P.l_pac < r1) {
        if (S[0].rbeg < P.l_pac) r1 = P.l_pac;
        else r0 = P.l_pac;
    }
}

// the chain's seeds ascending by (len, index) (software/bwamem.c:1070-1073):
// each key lands at its rank in srt
__device__ __forceinline__ void chain_order(const SeedRec* S, int n, uint64_t* srt, int lane) {
    n = uni(n);
    for (int ib = 0; ib < n; ib += 64) {
        const int i = ib + lane;
        const uint64_t ki = i < n ? ((uint64_t)(uint32_t)S[i].len << 32 | (uint32_t)i) : ~0ull;
        int rank = 0;
        for (int jb = 0; jb < n; jb += 64) {
            const int j = jb + lane;
            const uint64_t kj = j < n ? ((uint64_t)(uint32_t)S[j].len << 32 | (uint32_t)j) : ~0ull;
            const int m = n - jb < 64 ? n - jb : 64;
            for (int t = 0; t < m; ++t) rank += rl64(kj, t) < ki;
        }
        if (i < n) srt[rank] = ki;
    }
    __threadfence_block();
}

// does seed s (srt position k) get extended?  Not when it is (almost)
// contained in a region made before (software/bwamem.c:1079-1094), unless a
// long overlapping seed later in the order disagrees with it (:1098-1109).
// A skipped seed's srt entry is zeroed (the reference's srt[k] = 0).
__device__ __forceinline__ bool seed_wanted(const AlnParams& P, const SeedRec* S, int n, uint64_t* srt, int k, const SeedRec& s,
                            const AlnReg* regs, int nreg, int lane) {
    n = uni(n), k = uni(k), nreg = uni(nreg);
    bool hit = false;
    // newest regions first: a seed is mostly contained in its own chain's
    // region, made just before (any hit gives the same answer)
    for (int ib = 0; ib < nreg && !hit; ib += 64) {
        const int i = nreg - 1 - ib - lane;
        bool ok = false;
        if (i >= 0) {
            const AlnReg p = regs[i];
            if (!(s.rbeg < p.rb || s.rbeg + s.len > p.re || s.qbeg < p.qb || s.qbeg + s.len > p.qe)) {
                int qd = s.qbeg - p.qb;
                int64_t rd = s.rbeg - p.rb;
                int g = max_gap(P, (int)(qd < rd ? qd : rd));
                int w = g < P.w ? g : P.w;
                if (qd - rd < w && rd - qd < w) ok = true;
                qd = p.qe - (s.qbeg + s.len);
                rd = p.re - (s.rbeg + s.len);
                g = max_gap(P, (int)(qd < rd ? qd : rd));
                w = g < P.w ? g : P.w;
                if (qd - rd < w && rd - qd < w) ok = true;
            }
        }
        hit = __ballot(ok) != 0;
    }
    bool brk = false;
    for (int ib = k + 1; hit && ib < n && !brk; ib += 64) {
        const int i = ib + lane;
        bool ok = false;
        if (i < n) {
            const uint64_t v = srt[i];
            if (v != 0) {
                const SeedRec t = S[(uint32_t)v];
                if (!(t.len < s.len * .95)) {
                    if (s.qbeg <= t.qbeg && s.qbeg + s.len - t.qbeg >= s.len >> 2 &&
                        (int64_t)(t.qbeg - s.qbeg) != t.rbeg - s.rbeg)
                        ok = true;
                    if (t.qbeg <= s.qbeg && t.qbeg + t.len - s.qbeg >= s.len >> 2 &&
                        (int64_t)(s.qbeg - t.qbeg) != s.rbeg - t.rbeg)
                        ok = true;
                }
            }
        }
        brk = __ballot(ok) != 0;
    }
    if (hit && !brk) {
        if (lane == 0) srt[k] = 0;  // not extended
        __threadfence_block();
    }
    return !hit || brk;
}

// the region mem_chain2aln makes of seed s (software/bwamem.c:1110-1186):
// left and right ksw_extend2 with MAX_BAND_TRY, and the chain's seeds it
// covers.  Depends on the chain, the read and the reference only -- not on
// the regions made before -- so heavy reads compute it ahead, in parallel.
template <int KC>
__device__ __forceinline__ AlnReg seed_region(const AlnParams& P, const uint8_t* query, int L, const SeedRec* S, int n, const SeedRec& s,
                              int64_t r0, int64_t r1, int lane, Split* sp = nullptr) {
    int aw0 = P.w, aw1 = P.w, score = -1, truesc = -1, aqb, aqe;
    int64_t arb, are;
    if (s.qbeg) {  // left: the reversed query against the reversed reference
        const int64_t tmp = s.rbeg - r0;
        KswResult x{};
        for (int t = 0; t < 2; ++t) {  // MAX_BAND_TRY
            const int prev = score;
            aw0 = P.w << t;
            count(sp, 12);
            x = kswd::extend_wave<KC>(
                kswd::ExtIn{s.qbeg, (int)tmp, aw0, P.pen_clip5, P.zdrop, s.len * P.a},
                [&](int j) { return (int)query[s.qbeg - 1 - j]; }, [&](int i) { return ref_at(P, s.rbeg - 1 - i); },
                P.mat, P.o_del, P.e_del, P.o_ins, P.e_ins, P.top, sp ? &sp->t[14] : nullptr);
            score = x.score;
            if (score == prev || x.max_off < (aw0 >> 1) + (aw0 >> 2)) break;
        }
        if (x.gscore <= 0 || x.gscore <= score - P.pen_clip5) {  // local extension
            aqb = s.qbeg - x.qle, arb = s.rbeg - x.tle;
            truesc = score;
        } else {  // to the query start
            aqb = 0, arb = s.rbeg - x.gtle;
            truesc = x.gscore;
        }
    } else {
        score = truesc = s.len * P.a;
        aqb = 0, arb = s.rbeg;
    }
    stamp(sp, 4);
    if (s.qbeg + s.len != L) {  // right
        const int qe = s.qbeg + s.len, sc0 = score;
        const int64_t rs = s.rbeg + s.len;
        KswResult x{};
        for (int t = 0; t < 2; ++t) {
            const int prev = score;
            aw1 = P.w << t;
            count(sp, 13);
            x = kswd::extend_wave<KC>(kswd::ExtIn{L - qe, (int)(r1 - rs), aw1, P.pen_clip3, P.zdrop, sc0},
                                      [&](int j) { return (int)query[qe + j]; },
                                      [&](int i) { return ref_at(P, rs + i); }, P.mat, P.o_del, P.e_del, P.o_ins,
                                      P.e_ins, P.top, sp ? &sp->t[14] : nullptr);
            score = x.score;
            if (score == prev || x.max_off < (aw1 >> 1) + (aw1 >> 2)) break;
        }
        if (x.gscore <= 0 || x.gscore <= score - P.pen_clip3) {
            aqe = qe + x.qle, are = rs + x.tle;
            truesc += score - sc0;
        } else {
            aqe = L, are = rs + x.gtle;
            truesc += x.gscore - sc0;
        }
    } else {
        aqe = L, are = s.rbeg + s.len;
    }
    stamp(sp, 5);
    int cov = 0;  // seeds inside the region (software/bwamem.c:1180-1184)
    for (int i = lane; i < n; i += 64) {
        const SeedRec t = S[i];
        if (t.qbeg >= aqb && t.qbeg + t.len <= aqe && t.rbeg >= arb && t.rbeg + t.len <= are) cov += t.len;
    }
    cov = wsum(cov);
    AlnReg a;
    a.rb = arb, a.re = are, a.qb = aqb, a.qe = aqe;
    a.score = score, a.truesc = truesc, a.sub = 0, a.csub = 0, a.sub_n = 0;
    a.w = aw0 > aw1 ? aw0 : aw1, a.seedcov = cov, a.secondary = 0, a.hash = 0;
    return a;
}

// the region of seed si of a chain, behind a call (see aln_heavy_task_kernel)
template <int KC>
__device__ __attribute__((noinline)) void seed_region_call(const AlnParams& P, const uint8_t* query, int L,
                                                           const SeedRec* S, int n, int si, int64_t r0, int64_t r1,
                                                           AlnReg* out) {
    const AlnReg a = seed_region<KC>(P, query, L, S, n, S[si], r0, r1, threadIdx.x & 63);
    if ((threadIdx.x & 63) == 0) *out = a;
}

enum ChainMode { CM_PLAIN = 0, CM_RECORD = 1, CM_REPLAY = 2, CM_REPLAY_INL = 3 };

// mem_chain2aln (software/bwamem.c:1040-1188); regs[0 .. nreg) are the read's
// regions so far, srt the chain's n-word scratch.
//  CM_RECORD: also leave each extended seed's region at pre[i] (pre_ok[i] = 1);
//  CM_REPLAY: take a seed's region from pre[i] when pre_ok[i], else compute it
//    (the heavy-read walk over the chain walks recorded ahead, r0 / r1 given);
//  CM_REPLAY_INL: the same with the computation inlined (the light reads'
//    walk: a call would cost it half its waves, the callee's registers).
template <int KC, int MODE = CM_PLAIN>
__device__ __forceinline__ void chain_full(const AlnParams& P, const uint8_t* query, int L, const SeedRec* S, int n,
                                           uint64_t* srt, AlnReg* regs, int& nreg, int lane, AlnReg* pre = nullptr,
                                           uint8_t* pre_ok = nullptr, int64_t r0 = 0, int64_t r1 = 0,
                                           Split* sp = nullptr) {
    n = uni(n);
    if constexpr (MODE != CM_REPLAY && MODE != CM_REPLAY_INL) chain_span(P, L, S, n, lane, r0, r1);
    chain_order(S, n, srt, lane);
    stamp(sp, 2);
    for (int k = n - 1; k >= 0; --k) {
        const uint32_t si = (uint32_t)srt[k];
        const SeedRec s = S[si];
        const bool want = seed_wanted(P, S, n, srt, k, s, regs, nreg, lane);
        stamp(sp, 3);
        if (want) {
            if constexpr (MODE == CM_REPLAY || MODE == CM_REPLAY_INL) {
                if (uni((int)pre_ok[si])) {
                    if (lane == 0) regs[nreg] = pre[si];
                } else if constexpr (MODE == CM_REPLAY_INL) {
                    count(sp, 11);
                    const AlnReg a = seed_region<KC>(P, query, L, S, n, s, r0, r1, lane, sp);
                    if (lane == 0) regs[nreg] = a;
                } else {
                    seed_region_call<KC>(P, query, L, S, n, (int)si, r0, r1, regs + nreg);
                }
            } else {
                count(sp, 11);
                const AlnReg a = seed_region<KC>(P, query, L, S, n, s, r0, r1, lane, sp);
                if (lane == 0) {
                    regs[nreg] = a;
                    if constexpr (MODE == CM_RECORD) {
                        pre[si] = a;
                        pre_ok[si] = 1;
                    }
                }
            }
            ++nreg;
            __threadfence_block();
            stamp(sp, 6);
        }
    }
}

// KC = 4 at 4 waves per SIMD (128 VGPRs, 2 spilled): 3 waves at its free
// allocation (136).  SPLIT: the diagnostic instantiation (Split).  LANE: the
// walk over regions computed ahead (lane_on): the extensions left to it are
// behind a call (seed_region_call), so the walk keeps 4 waves a SIMD.
template <int KC, bool SPLIT = false, bool LANE = false>
__global__ __launch_bounds__(256, KC > 4 ? 1 : 4) void aln_kernel(AlnParams P) {
    const int lane = threadIdx.x & 63;
    Split spl{};
    Split* sp = SPLIT ? &spl : nullptr;
    if constexpr (SPLIT) spl.last = __builtin_amdgcn_s_memtime();
    count(sp, 15);
    constexpr uint32_t CLAIM = 4;  // reads per work-queue claim
    // light_claims > 0: the wave leaves after that many claims (the grid then
    // covers every read), so blocks retire while kernels of another stream wait
    // for CU slots
    for (uint32_t k = 0; P.light_claims == 0 || k < P.light_claims; ++k) {
        uint32_t r0 = 0;
        if (lane == 0) r0 = atomicAdd(&P.ctr[KC > 4 ? 1 : 0], CLAIM);
        r0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)r0);
        stamp(sp, 7);
        if (r0 >= (uint32_t)P.n_reads) break;
        const uint32_t r1 = r0 + CLAIM < (uint32_t)P.n_reads ? r0 + CLAIM : (uint32_t)P.n_reads;
        for (uint32_t r = r0; r < r1; ++r) {
            const uint64_t q0 = P.offs[r];
            const int L = (int)(P.offs[r + 1] - q0);
            if ((L > 256) != (KC > 4)) continue;  // the other instantiation's read
            const uint8_t* query = P.codes + q0;
            const uint64_t t_read = P.cyc ? __builtin_amdgcn_s_memtime() : 0;
            const uint64_t c0 = uni64(P.chain_off[r]), c1 = uni64(P.chain_off[r + 1]);
            if (P.heavy_min && (c1 - c0 >= P.heavy_min || P.seed_off[r + 1] - P.seed_off[r] >= P.heavy_seeds))
                continue;  // aln_heavy_kernel's read
            AlnReg* regs = P.raw + P.seed_off[r];
            int nreg = 0;
            count(sp, 8);
            stamp(sp, 0);
            for (uint64_t c = c0; c < c1; ++c) {
                OutChain ch = P.chains[c];
                ch.n = uni(ch.n);
                if (ch.n <= 0) continue;  // mem_chain2aln_short returns -1, nothing is made
                count(sp, 9);
                const SeedRec* S = P.seeds + ch.seed_off;
                // lane_on: the chains aln_chain_prep_kernel saw declined skip the
                // SW, and their seeds' regions come from pre where computed
                const int declined = LANE && uni((int)P.sdec[c]) ? 1 : chain_short(P, query, L, S, ch.n, regs + nreg, lane);
                stamp(sp, 1);
                if (declined == 0) {
                    count(sp, 10);
                    ++nreg;
                    __threadfence_block();
                } else if constexpr (LANE) {
                    chain_full<KC, CM_REPLAY_INL>(P, query, L, S, ch.n, P.srt + ch.seed_off, regs, nreg, lane,
                                              P.pre + ch.seed_off, P.pre_ok + ch.seed_off, P.span[2 * c],
                                              P.span[2 * c + 1], sp);
                } else {
                    chain_full<KC>(P, query, L, S, ch.n, P.srt + ch.seed_off, regs, nreg, lane, nullptr, nullptr, 0,
                                   0, sp);
                }
            }
            if (lane == 0) P.n_regs[r] = (uint64_t)nreg;
            stamp(sp, 0);
            if (P.cyc && lane == 0) P.cyc[r] = __builtin_amdgcn_s_memtime() - t_read;
        }
    }
    if constexpr (SPLIT) {
        if (lane == 0)
            for (int k = 0; k < ALN_SPLITS; ++k)
                atomicAdd(reinterpret_cast<unsigned long long*>(P.split + k), (unsigned long long)spl.t[k]);
    }
}

// heavy reads (at least heavy_min chains or heavy_seeds seeds), listed in
// any order with their chain and seed counts
__global__ __launch_bounds__(256) void aln_classify_kernel(AlnParams P) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= P.n_reads) return;
    const uint64_t nc = P.chain_off[r + 1] - P.chain_off[r], ns = P.seed_off[r + 1] - P.seed_off[r];
    if (nc >= P.heavy_min || ns >= P.heavy_seeds) {
        const uint32_t h = atomicAdd(&P.ctr[2], 1u);
        P.heavy[h] = r;
        P.hcnt[h] = nc;
        P.hscnt[h] = ns;
    }
}

// the heavy read of task t: h with off[h] <= t < off[h + 1]
__device__ __forceinline__ uint32_t heavy_of(const uint64_t* off, uint32_t nh, uint64_t t) {
    uint32_t lo = 0, hi = nh;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (off[mid] <= t) lo = mid;
        else hi = mid;
    }
    return (uint32_t)uni((int)lo);
}

// The heavy-path kernels are persistent loops that claim a task and run its
// body.  Every loop bound and branch of the wave-cooperative bodies is made
// an SGPR value (uni); the read walk is a call (see heavy_chain_walk).  A
// call around the extensions cost 20 % (register save / restore).

// chain task t of the heavy reads: mem_chain2aln_short's region (or its
// decline) and, when it declines, the region of every seed of the chain
// (pre, pre_ok = 1).  Measured against recording only the seeds the chain's
// own walk extends (CM_RECORD): on the human-like profile that left more
// extensions to the serial read walk and was 20 % slower.
template <int KC>
__device__ __forceinline__ void heavy_chain_task(const AlnParams& P, uint32_t nh, uint64_t t) {
    const int lane = threadIdx.x & 63;
    const uint32_t h = heavy_of(P.hoff, nh, t);
    const int r = uni(P.heavy[h]);
    const uint64_t q0 = P.offs[r];
    const int L = uni((int)(P.offs[r + 1] - q0));
    const uint64_t c = uni64(P.chain_off[r] + (t - P.hoff[h]));
    OutChain ch = P.chains[c];
    ch.n = uni(ch.n);
    if ((L > 256) == (KC > 4) && ch.n > 0) {  // this instantiation's read, a chain with seeds
        const uint8_t* query = P.codes + q0;
        const SeedRec* S = P.seeds + ch.seed_off;
        if (lane == 0) atomicAdd(&P.ctr[11], 1u);  // SMEM_ALN_STATS: heavy chains
        const int ok = chain_short(P, query, L, S, ch.n, P.pre_short + c, lane, P.ctr + 12) == 0;
        int64_t r0, r1;
        chain_span(P, L, S, ch.n, lane, r0, r1);
        if (lane == 0) {
            P.short_ok[c] = (uint8_t)ok;
            P.span[2 * c] = r0;
            P.span[2 * c + 1] = r1;
        }
        const bool local = P.spec_local != 0;
        for (int i = lane; i < ch.n; i += 64) P.pre_ok[ch.seed_off + i] = (uint8_t)(!ok && !local && !P.lane_on);
        __threadfence_block();
        if (!ok && local) {  // the seeds the chain's own walk extends (the read's walk computes any other)
            int nl = 0;
            chain_full<KC, CM_RECORD>(P, query, L, S, ch.n, P.srt + ch.seed_off, P.loc + ch.seed_off, nl, lane,
                                      P.pre + ch.seed_off, P.pre_ok + ch.seed_off);
        } else if (!ok && P.lane_on) {  // every seed's region, by the lane engine (aln_region_lane_kernel)
            uint32_t base = 0;
            if (lane == 0) {
                atomicAdd(&P.ctr[8], (uint32_t)ch.n);  // regions computed ahead (SMEM_ALN_STATS)
                base = atomicAdd(&P.lq[LQ_NTASK], (uint32_t)ch.n);
            }
            base = (uint32_t)uni((int)base);
            for (int i = lane; i < ch.n; i += 64) P.tasks[base + i] = RegTask{c, (uint32_t)r, (uint32_t)i};
        } else if (!ok) {  // every seed's region: the read's walk decides which of them are made
            if (lane == 0) atomicAdd(&P.ctr[8], (uint32_t)ch.n);  // regions computed ahead (SMEM_ALN_STATS)
            for (int i = 0; i < ch.n; ++i) {
                const AlnReg a = seed_region<KC>(P, query, L, S, ch.n, S[i], r0, r1, lane);
                if (lane == 0) P.pre[ch.seed_off + i] = a;
            }
        }
    }
}

// one wave per chain of the heavy reads at a time
template <int KC>
__global__ __launch_bounds__(256, KC > 4 ? 1 : 4) void aln_heavy_task_kernel(AlnParams P) {
    const uint32_t nh = P.ctr[2];
    const uint64_t total = P.hoff[nh];
    unsigned long long* head = reinterpret_cast<unsigned long long*>(P.ctr + (KC > 4 ? 6 : 4));
    for (;;) {
        uint64_t t = 0;
        if ((threadIdx.x & 63) == 0) t = atomicAdd(head, 1ull);
        t = uni64(t);
        if (t >= total) break;
        heavy_chain_task<KC>(P, nh, t);
    }
}

// is seed (s_rb, s_qb, s_len) (almost) contained in region p?
// (software/bwamem.c:1079-1094, the test seed_wanted makes per region)
__device__ __forceinline__ bool reg_contains(const AlnParams& P, int64_t s_rb, int s_qb, int s_len, int64_t p_rb,
                                             int64_t p_re, int p_qb, int p_qe) {
    if (s_rb < p_rb || s_rb + s_len > p_re || s_qb < p_qb || s_qb + s_len > p_qe) return false;
    int qd = s_qb - p_qb;
    int64_t rd = s_rb - p_rb;
    int g = max_gap(P, (int)(qd < rd ? qd : rd));
    int w = g < P.w ? g : P.w;
    if (qd - rd < w && rd - qd < w) return true;
    qd = p_qe - (s_qb + s_len);
    rd = p_re - (s_rb + s_len);
    g = max_gap(P, (int)(qd < rd ? qd : rd));
    w = g < P.w ? g : P.w;
    return qd - rd < w && rd - qd < w;
}

// A heavy read's regions hashed by 512-bp reference bin of their start, in
// a per-wave table of ALN_HT slots in global memory: slot = the bin's region
// count << 44 | bin << 20 | (index of the bin's newest region + 1), 0 =
// empty; older regions of a bin chain through rnext.  A region contains a
// seed only if it starts within the read's longest region before the seed,
// so a containment test visits one or two bins instead of every region made
// so far -- unless those bins hold more regions than a scan of all of them
// 64 at a time takes rounds (a tandem-repeat read piles its regions into a
// few bins: one round trip per hop made a 2,000-region read's walk 19 ms of
// dependent loads), and then it scans.
constexpr int HT_BIN = 9;
// Fibonacci hashing onto all ALN_HT slots (the top log2(ALN_HT) bits of the product)
constexpr uint32_t ALN_HT_BITS = __builtin_ctz((unsigned)ALN_HT);
static_assert((1u << ALN_HT_BITS) == (uint32_t)ALN_HT, "ALN_HT is a power of 2");
__device__ __forceinline__ uint32_t ht_home(uint64_t bin) { return ((uint32_t)bin * 2654435761u) >> (32 - ALN_HT_BITS); }

// the slot of bin (found, or the empty slot where it goes): one 64-slot
// window per round trip, the lanes probing in parallel
__device__ __forceinline__ int ht_find(const uint64_t* ht, uint64_t bin, int lane, uint64_t& entry) {
    uint32_t h = ht_home(bin);
    for (int w = 0; w < ALN_HT / 64; ++w) {
        const uint32_t sl = (h + (uint32_t)lane) & (ALN_HT - 1);
        const uint64_t e = ht[sl];
        const uint64_t m = __ballot(e == 0 || ((e >> 20) & 0xFFFFFFu) == bin);
        if (m) {
            const int f = __builtin_ctzll(m);
            entry = rl64(e, f);
            return (int)((h + (uint32_t)f) & (ALN_HT - 1));
        }
        h += 64;
    }
    entry = 0;
    return -1;  // full (not reached: the walk stops hashing a read before that)
}

__device__ __forceinline__ void ht_insert(uint64_t* ht, int32_t* rnext, int64_t rb, int idx, int lane) {
    uint64_t e;
    const uint64_t bin = (uint64_t)rb >> HT_BIN;
    const int sl = uni(ht_find(ht, bin, lane, e));
    if (lane == 0) {
        rnext[idx] = e ? (int32_t)(e & 0xFFFFF) - 1 : -1;
        if (sl >= 0) ht[sl] = ((e >> 44) + 1) << 44 | bin << 20 | (uint64_t)(idx + 1);
    }
    __threadfence_block();  // the next probe of this wave must see the slot
}

__device__ __forceinline__ int64_t shr64(int64_t v, int64_t first) {  // wave_shr:1, lane 0 takes first
    return (int64_t)((uint64_t)(uint32_t)kswd::wave_shr1((int)(uint32_t)v, (int)(uint32_t)first) |
                     (uint64_t)(uint32_t)kswd::wave_shr1((int)(v >> 32), (int)(first >> 32)) << 32);
}

// The walk of heavy read r: aln_kernel's chain loop over the regions computed
// ahead.  A heavy read walks thousands of chains one after the other, so the
// walk keeps what it touches in registers instead of round trips to memory:
//  * the newest 64 regions in a register ring (lane i: the i-th newest), so
//    the containment test of a seed is one ballot unless it must look further
//    back (then the older regions are scanned in memory, newest first);
//  * a chain of <= 64 seeds in registers, lane k holding the seed of rank k in
//    the reference's order (ks_introsort of len << 32 | index) and its region
//    computed ahead, so the "long overlapping seed disagrees" test
//    (software/bwamem.c:1098-1109) is one ballot over the lanes above k and a
//    made region is one store from lane k.
// Longer chains take chain_full (and empty the ring).
// GUARD (the inlined diagnostic instantiation, SMEM_ALN_WALK_INLINE=1): every
// loop iteration of the walk counts against P.walk_guard; past it the wave
// sets ctr[15] and leaves the read, so a walk that would spin ends instead of
// hanging the GPU (the round-2 hang).
#define WALK_GUARD_L()                                                        \
    if constexpr (GUARD) {                                                    \
        if (++guard > P.walk_guard) {                                         \
            if (lane == 0) atomicAdd(&P.ctr[15], 1u);                         \
            tripped = true;                                                   \
            return true;                                                      \
        }                                                                     \
    }
#define WALK_GUARD()                                                          \
    if constexpr (GUARD) {                                                    \
        if (++guard > P.walk_guard) {                                         \
            if (lane == 0) atomicAdd(&P.ctr[15], 1u);                         \
            return;                                                           \
        }                                                                     \
    }
template <int KC, bool GUARD>
__device__ __forceinline__ void heavy_read_walk_body(const AlnParams& P, int r) {
    const int lane = threadIdx.x & 63;
    uint32_t guard = 0;
    const uint64_t t_read = P.cyc ? __builtin_amdgcn_s_memtime() : 0;  // SMEM_ALN_CYCLES
    const int L = uni((int)(P.offs[r + 1] - P.offs[r]));
    const uint8_t* query = P.codes + P.offs[r];
    const uint64_t c0 = uni64(P.chain_off[r]), c1 = uni64(P.chain_off[r + 1]);
    AlnReg* regs = P.raw + P.seed_off[r];
    int nreg = 0;
    int64_t g_rb = 0, g_re = 0;  // the ring
    int g_qb = 0, g_qe = 0, rc = 0;
    // the bin hash, for reads with many regions (not with more than the
    // table holds, or than 20-bit indices do)
    const uint64_t cap = uni64(P.seed_off[r + 1] - P.seed_off[r]);
    // the candidate index (built for every heavy read when P.cand_made is set)
    // until the walk makes a region the index does not hold (dirty: a region
    // computed here, or chain_full's); then, as without the index, the bin
    // hash or a scan of every older region
    const bool indexed = P.cand_made != nullptr;
    bool dirty = false;
    const bool hashed = !indexed && c1 - c0 >= P.hash_min && cap < (1u << 20) - 1 && cap + (c1 - c0) < ALN_HT / 2 &&
                        ((uint64_t)(2 * P.l_pac) >> HT_BIN) < (1ull << 24);  // bins fit the slot's 24 bits
    uint64_t* ht = P.ht + (size_t)((blockIdx.x * blockDim.x + threadIdx.x) >> 6) * ALN_HT;
    int32_t* rnext = P.rnext + P.seed_off[r];
    int64_t maxlen = 0;  // the longest region so far
    uint32_t n_used = 0, n_serial = 0;  // regions taken from the chain tasks / computed here (SMEM_ALN_STATS)
    uint64_t w_full = 0, w_hash = 0, w_big = 0, w_hops = 0;  // SMEM_ALN_CYCLES: the walk's split
    if (hashed) {
        for (int i = lane; i < ALN_HT; i += 64) ht[i] = 0;
        __threadfence_block();
    }
    // a seed contained in a region made before it (software/bwamem.c:1079-1094):
    // the ring of the newest 64 in registers, then the candidate index (x, y:
    // the seed's candidates), the bin hash or a scan of every older region
    bool tripped = false;  // GUARD: a lambda's loop ran past the guard
    auto contained = [&](int64_t k_rb, int k_qb, int k_len, uint32_t x, uint32_t y) -> bool {
        bool hit = __ballot(lane < rc && reg_contains(P, k_rb, k_qb, k_len, g_rb, g_re, g_qb, g_qe)) != 0;
        const int older = nreg - rc;  // regions only in memory: regs[0 .. older)
        bool scan = !hit && older > 0 && !hashed && (!indexed || dirty);
        if (!hit && older > 0 && indexed && !dirty) {  // the candidates that contain it, made so far
            if (x < y) __threadfence_block();
            for (uint32_t q0 = x; q0 < y && !hit; q0 += 64) {
                WALK_GUARD_L();
                const uint32_t q = q0 + (uint32_t)lane;
                bool ok = false;
                if (q < y) {
                    const uint8_t made = P.cand_made[q];
                    const int64_t prb = P.cand_rb[q], pre_ = P.cand_re[q];
                    const uint32_t pq = P.cand_q[q];
                    ok = made && reg_contains(P, k_rb, k_qb, k_len, prb, pre_, (int)(pq & 0xFFFFu), (int)(pq >> 16));
                }
                hit = __ballot(ok) != 0;
                ++w_hops;
            }
        } else if (!hit && older > 0 && hashed) {  // the bins a containing region can start in
            const uint64_t th = P.cyc ? __builtin_amdgcn_s_memtime() : 0;
            __threadfence_block();
            const uint64_t b1 = (uint64_t)k_rb >> HT_BIN;
            const uint64_t b0 = (uint64_t)(k_rb - maxlen > 0 ? k_rb - maxlen : 0) >> HT_BIN;
            // their heads and counts first: one round per bin (usually 1-2 bins)
            const bool wide = b1 - b0 >= 64;  // (not with reads of <= 1024 bp)
            uint64_t heads = 0, in_bins = 0;  // lane (b - b0) holds bin b's entry
            for (uint64_t b = b0; b <= b1 && !wide; ++b) {
                WALK_GUARD_L();
                uint64_t e;
                (void)ht_find(ht, b, lane, e);
                if ((uint64_t)lane == b - b0) heads = e;
                in_bins += e >> 44;
            }
            if (wide || in_bins > (uint64_t)(older >> 6) + 2) {
                scan = true;  // fewer rounds 64 regions at a time than one per hop
            } else {
                for (uint64_t b = b0; b <= b1 && !hit; ++b) {
                    WALK_GUARD_L();
                    const uint64_t e = rl64(heads, (int)(b - b0));
                    int i = e ? uni((int)(e & 0xFFFFF) - 1) : -1;
                    while (i >= 0 && !hit) {
                        WALK_GUARD_L();
                        const AlnReg* p = regs + i;
                        hit = reg_contains(P, k_rb, k_qb, k_len, (int64_t)uni64((uint64_t)p->rb),
                                           (int64_t)uni64((uint64_t)p->re), uni(p->qb), uni(p->qe));
                        i = uni(rnext[i]);
                        ++w_hops;
                    }
                }
            }
            if (P.cyc) w_hash += __builtin_amdgcn_s_memtime() - th;
        }
        if (scan) {  // every older region, newest first, 64 a round
            __threadfence_block();
            for (int ib = 0; ib < older && !hit; ib += 64) {
                WALK_GUARD_L();
                const int i = older - 1 - ib - lane;
                bool ok = false;
                if (i >= 0) {
                    const AlnReg p = regs[i];
                    ok = reg_contains(P, k_rb, k_qb, k_len, p.rb, p.re, p.qb, p.qe);
                }
                hit = __ballot(ok) != 0;
            }
        }
        return hit;
    };
    // a made region: into regs (done by the caller), the ring, the hash
    auto push = [&](int64_t a_rb, int64_t a_re, int a_qb, int a_qe) {
        g_rb = shr64(g_rb, a_rb), g_re = shr64(g_re, a_re);
        g_qb = kswd::wave_shr1(g_qb, a_qb), g_qe = kswd::wave_shr1(g_qe, a_qe);
        rc = rc < 64 ? rc + 1 : 64;
        if (hashed) {
            maxlen = a_re - a_rb > maxlen ? a_re - a_rb : maxlen;
            ht_insert(ht, rnext, a_rb, nreg, lane);
        }
        ++nreg;
    };
    // The chains 64 at a time: lane t loads chain cb + t's header, and for a
    // short chain (mem_chain2aln_short made its region) or a single-seed chain
    // everything its walk step reads, so such a chain costs no round trip of
    // its own (on the human-like profile's heavy reads ~90 % of the chains
    // have one seed, and the walk waited on 3 round trips per chain).
    for (uint64_t cb = c0; cb < c1; cb += 64) {
        WALK_GUARD();
        const uint64_t cl = cb + (uint64_t)lane;
        int h_n = 0, h_sh = 0, h_ok = 0;
        uint64_t h_so = 0;
        uint32_t h_pc = 0, h_ps = 0;
        uint2 h_rng = {0, 0};
        SeedRec h_s{0, 0, 0};
        AlnReg h_reg{};
        if (cl < c1) {
            const OutChain hc = P.chains[cl];
            h_n = hc.n, h_so = hc.seed_off;
            h_sh = P.short_ok[cl];
            if (indexed) h_pc = P.cand_pos_c[cl];
            if (h_n > 0 && h_sh) {
                h_reg = P.pre_short[cl];
            } else if (h_n == 1) {
                h_s = P.seeds[h_so];
                h_reg = P.pre[h_so];
                h_ok = P.pre_ok[h_so];
                if (indexed) {
                    h_rng = P.cand_rng[h_so];
                    h_ps = P.cand_pos_s[h_so];
                }
            }
        }
        const uint64_t ce = cb + 64 < c1 ? cb + 64 : c1;
        for (uint64_t c = cb; c < ce; ++c) {
        WALK_GUARD();
        const int t = (int)(c - cb);
        const int n = kswd::rl(h_n, t);
        if (n <= 0) continue;
        if (kswd::rl(h_sh, t)) {  // mem_chain2aln_short's region
            if (lane == t) {
                regs[nreg] = h_reg;
                if (indexed) P.cand_made[h_pc] = 1;
            }
            push((int64_t)rl64((uint64_t)h_reg.rb, t), (int64_t)rl64((uint64_t)h_reg.re, t), kswd::rl(h_reg.qb, t),
                 kswd::rl(h_reg.qe, t));
            continue;
        }
        OutChain ch;
        ch.seed_off = rl64(h_so, t);
        ch.n = n;
        if (n == 1) {  // one seed: extended unless contained (no seed above it can disagree)
            const int64_t k_rb = (int64_t)rl64((uint64_t)h_s.rbeg, t);
            const int k_qb = kswd::rl(h_s.qbeg, t), k_len = kswd::rl(h_s.len, t);
            const bool hit1 = contained(k_rb, k_qb, k_len, (uint32_t)kswd::rl((int)h_rng.x, t),
                                        (uint32_t)kswd::rl((int)h_rng.y, t));
            if constexpr (GUARD) {
                if (tripped) return;
            }
            if (hit1) continue;
            int64_t a_rb, a_re;
            int a_qb, a_qe;
            if (kswd::rl(h_ok, t)) {
                ++n_used;
                if (lane == t) {
                    regs[nreg] = h_reg;
                    if (indexed) P.cand_made[h_ps] = 1;
                }
                a_rb = (int64_t)rl64((uint64_t)h_reg.rb, t), a_re = (int64_t)rl64((uint64_t)h_reg.re, t);
                a_qb = kswd::rl(h_reg.qb, t), a_qe = kswd::rl(h_reg.qe, t);
            } else {
                ++n_serial;
                dirty = true;  // a region the index does not hold
                const SeedRec* S = P.seeds + ch.seed_off;
                __threadfence_block();
                if constexpr (GUARD) {
                    const AlnReg a = seed_region<KC>(P, query, L, S, 1, S[0], P.span[2 * c], P.span[2 * c + 1], lane);
                    if (lane == 0) regs[nreg] = a;
                } else {
                    seed_region_call<KC>(P, query, L, S, 1, 0, P.span[2 * c], P.span[2 * c + 1], regs + nreg);
                }
                __threadfence_block();
                a_rb = (int64_t)uni64((uint64_t)regs[nreg].rb), a_re = (int64_t)uni64((uint64_t)regs[nreg].re);
                a_qb = uni(regs[nreg].qb), a_qe = uni(regs[nreg].qe);
            }
            push(a_rb, a_re, a_qb, a_qe);
            continue;
        }
        const SeedRec* S = P.seeds + ch.seed_off;
        if (n > 128) {
            __threadfence_block();
            const int before = nreg;
            const uint64_t tf = P.cyc ? __builtin_amdgcn_s_memtime() : 0;
            chain_full<KC, CM_REPLAY>(P, query, L, S, n, P.srt + ch.seed_off, regs, nreg, lane, P.pre + ch.seed_off,
                                      P.pre_ok + ch.seed_off, P.span[2 * c], P.span[2 * c + 1]);
            rc = 0;
            dirty = true;  // its regions are not marked in the index
            if (P.cyc) {
                w_full += __builtin_amdgcn_s_memtime() - tf;
                w_big += 1 + ((uint64_t)n << 32);
            }
            if (hashed) {
                __threadfence_block();
                for (int i = before; i < nreg; ++i) {
                    WALK_GUARD();
                    const int64_t rb = (int64_t)uni64((uint64_t)regs[i].rb), re = (int64_t)uni64((uint64_t)regs[i].re);
                    maxlen = re - rb > maxlen ? re - rb : maxlen;
                    ht_insert(ht, rnext, rb, i, lane);
                }
            }
            continue;
        }
        // the chain's seeds in the reference's order (len << 32 | index ascending,
        // software/bwamem.c:1070-1073), rank k at lane k & 63 of slot k >> 6:
        // up to 64 seeds in slot 0 (ranked and permuted across the lanes), up
        // to 128 with slot 1 (two: ranked through the chain's srt rows; the
        // regions computed ahead then come from memory when a seed is made)
        const bool two = n > 64;
        int64_t s_rb, s_rb1 = 0;
        int s_qb, s_len, s_idx, s_qb1 = 0, s_len1 = 0, s_idx1 = 0;
        AlnReg mine{};
        int mine_ok = 0, mine_ok1 = 0;
        uint2 rng = {0, 0}, rng1 = {0, 0};  // indexed: the candidates of rank lane / 64 + lane
        uint32_t pos = 0, pos1 = 0;         // and the index position of its own region
        if (!two) {
            SeedRec my{0, 0, 0};
            if (lane < n) my = S[lane];
            const uint64_t key = lane < n ? ((uint64_t)(uint32_t)my.len << 32 | (uint32_t)lane) : ~0ull;
            int rank = 0;
            for (int t = 0; t < n; ++t) {
                WALK_GUARD();
                rank += rl64(key, t) < key;
            }
            const int dst = (lane < n ? rank : lane) << 2;  // a permutation of the 64 lanes
            s_rb = (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_ds_permute(dst, (int)(uint32_t)my.rbeg) |
                             (uint64_t)(uint32_t)__builtin_amdgcn_ds_permute(dst, (int)(my.rbeg >> 32)) << 32);
            s_qb = __builtin_amdgcn_ds_permute(dst, my.qbeg);
            s_len = __builtin_amdgcn_ds_permute(dst, my.len);
            s_idx = __builtin_amdgcn_ds_permute(dst, lane);
            if (lane < n) {
                mine = P.pre[ch.seed_off + s_idx];
                mine_ok = P.pre_ok[ch.seed_off + s_idx];
                if (indexed) {
                    rng = P.cand_rng[ch.seed_off + s_idx];
                    pos = P.cand_pos_s[ch.seed_off + s_idx];
                }
            }
        } else {
            uint64_t* srt = P.srt + ch.seed_off;
            const bool v1 = 64 + lane < n;
            const SeedRec m0 = S[lane];
            const SeedRec m1 = v1 ? S[64 + lane] : SeedRec{0, 0, 0};
            const uint64_t k0 = (uint64_t)(uint32_t)m0.len << 32 | (uint32_t)lane;
            const uint64_t k1 = v1 ? ((uint64_t)(uint32_t)m1.len << 32 | (uint32_t)(64 + lane)) : ~0ull;
            int r0 = 0, r1 = 0;
            for (int t = 0; t < 64; ++t) {
                const uint64_t v = rl64(k0, t);
                r0 += v < k0, r1 += v < k1;
            }
            for (int t = 0; t < n - 64; ++t) {
                WALK_GUARD();
                const uint64_t v = rl64(k1, t);
                r0 += v < k0, r1 += v < k1;
            }
            srt[r0] = k0;
            if (v1) srt[r1] = k1;
            __threadfence_block();
            s_idx = (int)(uint32_t)srt[lane];
            s_idx1 = v1 ? (int)(uint32_t)srt[64 + lane] : 0;
            const SeedRec q0 = S[s_idx], q1 = S[s_idx1];
            s_rb = q0.rbeg, s_qb = q0.qbeg, s_len = q0.len;
            s_rb1 = q1.rbeg, s_qb1 = q1.qbeg, s_len1 = q1.len;
            mine_ok = P.pre_ok[ch.seed_off + s_idx];
            mine_ok1 = v1 ? P.pre_ok[ch.seed_off + s_idx1] : 0;
            if (indexed) {
                rng = P.cand_rng[ch.seed_off + s_idx];
                pos = P.cand_pos_s[ch.seed_off + s_idx];
                if (v1) {
                    rng1 = P.cand_rng[ch.seed_off + s_idx1];
                    pos1 = P.cand_pos_s[ch.seed_off + s_idx1];
                }
            }
        }
        bool skipped = false, skipped1 = false;
        for (int k = n - 1; k >= 0; --k) {
            WALK_GUARD();
            const bool hi = k >= 64;  // wave-uniform: which slot holds rank k
            const int kl = k & 63;
            const int64_t k_rb = (int64_t)rl64((uint64_t)(hi ? s_rb1 : s_rb), kl);
            const int k_qb = kswd::rl(hi ? s_qb1 : s_qb, kl), k_len = kswd::rl(hi ? s_len1 : s_len, kl);
            bool hit = contained(k_rb, k_qb, k_len, (uint32_t)kswd::rl((int)(hi ? rng1.x : rng.x), kl),
                                 (uint32_t)kswd::rl((int)(hi ? rng1.y : rng.y), kl));
            if constexpr (GUARD) {
                if (tripped) return;
            }
            bool wanted = !hit;
            if (hit) {  // extended anyway if a longer overlapping seed above k disagrees with it
                // (software/bwamem.c:1098-1109; a skipped seed no longer counts)
                auto disagrees = [&](int i, bool skp, int64_t t_rb, int t_qb, int t_len) {
                    if (i <= k || i >= n || skp || t_len < k_len * .95) return false;
                    if (k_qb <= t_qb && k_qb + k_len - t_qb >= k_len >> 2 && (int64_t)(t_qb - k_qb) != t_rb - k_rb)
                        return true;
                    return t_qb <= k_qb && t_qb + t_len - k_qb >= k_len >> 2 && (int64_t)(k_qb - t_qb) != k_rb - t_rb;
                };
                bool ok = disagrees(lane, skipped, s_rb, s_qb, s_len);
                if (two) ok = ok || disagrees(64 + lane, skipped1, s_rb1, s_qb1, s_len1);
                wanted = __ballot(ok) != 0;
                if (!wanted && lane == kl) {
                    if (hi) skipped1 = true;
                    else skipped = true;
                }
            }
            if (!wanted) continue;
            int64_t a_rb, a_re;
            int a_qb, a_qe;
            if (kswd::rl(hi ? mine_ok1 : mine_ok, kl)) {
                ++n_used;
                if (indexed && lane == kl) P.cand_made[hi ? pos1 : pos] = 1;
                if (!two) {
                    if (lane == k) regs[nreg] = mine;
                    a_rb = (int64_t)rl64((uint64_t)mine.rb, k), a_re = (int64_t)rl64((uint64_t)mine.re, k);
                    a_qb = kswd::rl(mine.qb, k), a_qe = kswd::rl(mine.qe, k);
                } else {
                    const AlnReg* pr = P.pre + ch.seed_off + kswd::rl(hi ? s_idx1 : s_idx, kl);
                    const AlnReg a = *pr;
                    if (lane == 0) regs[nreg] = a;
                    a_rb = (int64_t)uni64((uint64_t)a.rb), a_re = (int64_t)uni64((uint64_t)a.re);
                    a_qb = uni(a.qb), a_qe = uni(a.qe);
                }
            } else {
                ++n_serial;
                dirty = true;  // a region the index does not hold
                const int si = kswd::rl(hi ? s_idx1 : s_idx, kl);
                __threadfence_block();
                if constexpr (GUARD) {  // inlined too
                    const AlnReg a = seed_region<KC>(P, query, L, S, n, S[si], P.span[2 * c], P.span[2 * c + 1], lane);
                    if (lane == 0) regs[nreg] = a;
                } else {
                    seed_region_call<KC>(P, query, L, S, n, si, P.span[2 * c], P.span[2 * c + 1], regs + nreg);
                }
                __threadfence_block();
                a_rb = (int64_t)uni64((uint64_t)regs[nreg].rb), a_re = (int64_t)uni64((uint64_t)regs[nreg].re);
                a_qb = uni(regs[nreg].qb), a_qe = uni(regs[nreg].qe);
            }
            push(a_rb, a_re, a_qb, a_qe);
        }
        }
    }
    if (lane == 0) {
        P.n_regs[r] = (uint64_t)nreg;
        if (n_used) atomicAdd(&P.ctr[9], n_used);
        if (n_serial) atomicAdd(&P.ctr[10], n_serial);
        if (P.cyc) {
            P.cyc[r] = __builtin_amdgcn_s_memtime() - t_read;
            uint64_t* w = P.cyc + P.n_reads + 4ull * r;
            w[0] = w_full, w[1] = w_hash, w[2] = w_big, w[3] = w_hops;
        }
    }
}
#undef WALK_GUARD
#undef WALK_GUARD_L

// The product instantiation: the walk behind a call.  Round 2 saw gfx950
// waves hang with the walk inlined into aln_heavy_kernel's persistent loop;
// SMEM_ALN_WALK_INLINE=1 runs the inlined, guarded instantiation to test that
// (DESIGN.md §5).
template <int KC>
__device__ __attribute__((noinline)) void heavy_read_walk(const AlnParams& P, int r) {
    heavy_read_walk_body<KC, false>(P, r);
}

// one wave per heavy read at a time
template <int KC, bool INL = false>
__global__ __launch_bounds__(256) void aln_heavy_kernel(AlnParams P) {
    const uint32_t nh = P.ctr[2];
    for (;;) {
        uint32_t h = 0;
        if ((threadIdx.x & 63) == 0) h = atomicAdd(&P.ctr[KC > 4 ? 13 : 3], 1u);
        h = (uint32_t)uni((int)h);
        if (h >= nh) break;
        const int r = uni(P.heavy[h]);
        if ((uni((int)(P.offs[r + 1] - P.offs[r])) > 256) == (KC > 4)) {
            if constexpr (INL) heavy_read_walk_body<KC, true>(P, r);
            else heavy_read_walk<KC>(P, r);
        }
    }
}


// The giant split: the heavy list copied in the same bucket order (seeds +
// chains, most first), its first n_giant reads marked giant.  (One block; the
// reads of a bucket in any order.)
__global__ __launch_bounds__(1024) void aln_heavy_split_kernel(AlnParams P, uint32_t nh, uint32_t ng, int32_t* heavy2,
                                                               uint64_t* hcnt2, uint64_t* hscnt2, uint8_t* rgiant,
                                                               uint32_t* ctr_g, uint32_t* ctr_r) {
    __shared__ uint32_t cnt[64];
    const uint32_t t = threadIdx.x;
    if (t < 64) cnt[t] = 0;
    for (int r = (int)t; r < P.n_reads; r += (int)blockDim.x) rgiant[r] = 0;
    __syncthreads();
    auto bucket = [&](uint32_t h) -> uint32_t {
        const uint64_t w = P.hcnt[h] + P.hscnt[h];
        return 63u - (uint32_t)__builtin_clzll(w | 1ull);
    };
    for (uint32_t h = t; h < nh; h += blockDim.x) atomicAdd(&cnt[bucket(h)], 1u);
    __syncthreads();
    if (t == 0) {
        uint32_t o = 0;
        for (int b = 63; b >= 0; --b) {
            const uint32_t c = cnt[b];
            cnt[b] = o;
            o += c;
        }
        ctr_g[2] = ng;
        ctr_r[2] = nh - ng;
    }
    __syncthreads();
    for (uint32_t h = t; h < nh; h += blockDim.x) {
        const uint32_t pos = atomicAdd(&cnt[bucket(h)], 1u);
        const int32_t r = P.heavy[h];
        heavy2[pos] = r;
        hcnt2[pos] = P.hcnt[h];
        hscnt2[pos] = P.hscnt[h];
        if (pos < ng) rgiant[r] = 1;
    }
}

// ---- the heavy walk's candidate index (AlnParams::cand_*) ----
// Every region a heavy read's walk can make is known before the walk: its
// short chains' pre_short and its other chains' seeds' pre.  Sorted by
// reference start per read, the regions that can contain a seed are those
// starting within the read's longest candidate before it, and the walk tests
// them 64 a round, counting only those it made so far (cand_made) -- instead
// of one dependent round trip per region of a bin (the bin hash) on reads
// whose regions pile into few bins.
constexpr uint64_t CAND_RB_NONE = (1ull << 34) - 1;

__global__ __launch_bounds__(256) void aln_cand_count_kernel(AlnParams P, uint32_t nh, uint64_t* cnt, uint32_t* hord) {
    const uint32_t h = blockIdx.x * blockDim.x + threadIdx.x;
    if (h < nh) {
        cnt[h] = P.hcnt[h] + P.hscnt[h];
        hord[P.heavy[h]] = h;
    }
}

// one thread per chain of a heavy read (chain_read bit 31): its slot and its
// seeds' slots keyed, the read's longest candidate by atomicMax (hmax zeroed).
// A read's seeds are exactly its chains' seeds, so every slot is written.
__global__ __launch_bounds__(256) void aln_cand_fill_kernel(AlnParams P, CandParams C, uint64_t n_chains) {
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < n_chains;
         c += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t cr = P.chain_read[c];
        if (!(cr & 0x80000000u)) continue;
        const int r = (int)(cr & 0x3FFFFFFFu);
        const uint32_t h = C.hord[r];
        if (h == 0xFFFFFFFFu) continue;  // a heavy read of the other instance (giant split)
        const uint64_t base = C.off[h], s0 = P.seed_off[r], ns = P.seed_off[r + 1] - s0;
        const uint64_t c0 = P.chain_off[r];
        const uint64_t hk = 0;  // the segments are the reads' slots: keys are rb alone
        const OutChain ch = P.chains[c];
        const bool sh = ch.n > 0 && P.short_ok[c];
        int64_t mx = 0;
        uint64_t kc = hk | CAND_RB_NONE;
        if (sh) {
            const int64_t rb = P.pre_short[c].rb, re = P.pre_short[c].re;
            kc = hk | (uint64_t)rb;
            mx = re - rb;
        }
        C.key[base + ns + (c - c0)] = kc;
        C.val[base + ns + (c - c0)] = 0x80000000u | (uint32_t)c;
        for (int i = 0; i < ch.n; ++i) {
            const uint64_t j = ch.seed_off + (uint64_t)i;
            uint64_t k = hk | CAND_RB_NONE;
            if (!sh && P.pre_ok[j]) {
                const int64_t rb = P.pre[j].rb, re = P.pre[j].re;
                k = hk | (uint64_t)rb;
                mx = re - rb > mx ? re - rb : mx;
            }
            C.key[base + (j - s0)] = k;
            C.val[base + (j - s0)] = (uint32_t)j;
        }
        if (mx > 0) atomicMax(reinterpret_cast<unsigned long long*>(C.hmax + h), (unsigned long long)mx);
    }
}

// one thread per sorted slot: the candidate's fields in index order, its position
__global__ __launch_bounds__(256) void aln_cand_place_kernel(AlnParams P, CandParams C) {
    for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < C.m; q += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t key = C.key2[q];
        const uint32_t v = C.val2[q];
        P.cand_made[q] = 0;
        if ((key & CAND_RB_NONE) == CAND_RB_NONE) {
            P.cand_rb[q] = INT64_MAX;
            P.cand_re[q] = 0;
            P.cand_q[q] = 0;
            continue;
        }
        const bool sc = (v & 0x80000000u) != 0;
        const AlnReg& a = sc ? P.pre_short[v & 0x7FFFFFFFu] : P.pre[v];
        P.cand_rb[q] = a.rb;
        P.cand_re[q] = a.re;
        P.cand_q[q] = (uint32_t)a.qb | (uint32_t)a.qe << 16;
        if (sc) P.cand_pos_c[v & 0x7FFFFFFFu] = (uint32_t)q;
        else P.cand_pos_s[v] = (uint32_t)q;
    }
}

// the first position in [lo, hi) whose key is >= k (> k: upper)
__device__ __forceinline__ uint64_t cand_bound(const uint64_t* key, uint64_t lo, uint64_t hi, uint64_t k, bool upper) {
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        const uint64_t v = key[mid];
        if (upper ? v <= k : v < k) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// one thread per seed slot of the index (the unsorted slots: a heavy read's
// seeds first, in seed order; its read from the slot offsets): the
// candidates starting in [rbeg - the read's longest candidate, rbeg] (a
// region that contains the seed starts there), narrowed to the first .. last
// of them that contain it (a static test: whether the walk made them is its
// own business) other than the seed's own region (made, if at all, after the
// seed is tested).  A seed no other candidate contains gets an empty range and
// costs the walk no round trip.  (A thread per chain left the tandem-repeat
// reads' long ranges to a few threads: 2.7 / 4.9 ms on the walk's path.)
__global__ __launch_bounds__(256) void aln_cand_range_kernel(AlnParams P, CandParams C) {
    for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < C.m; u += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t lo_h = 0, hi_h = C.n_heavy;  // the read h with off[h] <= u < off[h + 1]
        while (hi_h - lo_h > 1) {
            const uint32_t mid = (lo_h + hi_h) >> 1;
            if (C.off[mid] <= u) lo_h = mid;
            else hi_h = mid;
        }
        const uint32_t h = lo_h;
        const int r = P.heavy[h];
        const uint64_t s0 = P.seed_off[r];
        if (u - C.off[h] >= P.seed_off[r + 1] - s0) continue;  // a chain slot
        const uint64_t j = s0 + (u - C.off[h]);
        const uint64_t lo = C.off[h], hi = C.off[h + 1];
        const int64_t mx = C.hmax[h];
        const SeedRec sd = P.seeds[j];
        const uint64_t x = cand_bound(C.key2, lo, hi, (uint64_t)(sd.rbeg - mx > 0 ? sd.rbeg - mx : 0), false);
        const uint64_t y = cand_bound(C.key2, x, hi, (uint64_t)sd.rbeg, true);
        const uint32_t own = P.pre_ok[j] ? P.cand_pos_s[j] : 0xFFFFFFFFu;
        uint32_t f = 0xFFFFFFFFu, l = 0;
        for (uint64_t q = x; q < y; ++q) {
            const uint32_t pq = P.cand_q[q];
            if ((uint32_t)q != own &&
                reg_contains(P, sd.rbeg, sd.qbeg, sd.len, P.cand_rb[q], P.cand_re[q], (int)(pq & 0xFFFFu), (int)(pq >> 16))) {
                f = f < (uint32_t)q ? f : (uint32_t)q;
                l = (uint32_t)q + 1;
            }
        }
        P.cand_rng[j] = f == 0xFFFFFFFFu ? make_uint2(0, 0) : make_uint2(f, l);
    }
}

// ---- regions computed ahead, one seed per lane (lane_on) ----
// The light reads' walk (aln_kernel) extends a seed of a chain only where no
// region made before contains it; the chain's first seed in the order (its
// longest) is extended unless an earlier chain's region covers it, and on
// mem_chain2aln's inputs that is 94 % of the extensions (oracle seed_uses,
// profiles/r03).  So those seeds' regions -- and every seed of the heavy
// reads' chains, as before -- are tasks: the left extensions of all tasks run
// as one pass of the lane engine (kswl::lane_engine, one problem per lane,
// tasks sorted by query length), then the right ones (each needs its left
// score), then a pass adds the seed coverage.  The walks take the regions
// from pre / pre_ok and extend what is left one wave per problem, as before.

// the read of every chain (bit 31: a heavy read), one thread per read
__global__ __launch_bounds__(256) void aln_chain_read_kernel(AlnParams P) {
    for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < P.n_reads; r += gridDim.x * blockDim.x) {
        const uint64_t c0 = P.chain_off[r], c1 = P.chain_off[r + 1];
        const bool heavy =
            P.heavy_min && (c1 - c0 >= P.heavy_min || P.seed_off[r + 1] - P.seed_off[r] >= P.heavy_seeds);
        const uint32_t v = (uint32_t)r | (heavy ? 0x80000000u : 0u) | (heavy && P.rgiant && P.rgiant[r] ? 0x40000000u : 0u);
        for (uint64_t c = c0; c < c1; ++c) P.chain_read[c] = v;
    }
}

// Every chain, one lane each: its reference span (chain_span), whether
// mem_chain2aln_short declines it without its SW (chain_short's tests on the
// seeds alone, software/bwamem.c:815-828), and its tasks:
//   a light read's chain: when declined, its first seed in the order (the
//     walk, aln_kernel, runs the SW of the others itself);
//   a heavy read's chain: when declined, every seed (short_ok = 0); else it is
//     listed for its SW (aln_heavy_sw_kernel).
// pre_ok cleared for the chain's seeds.  (One wave per heavy chain, with a
// binary search for its read and wave reductions, took 75 ms on the human-like
// profile's 3.2 M heavy chains: latency-bound.)
__global__ __launch_bounds__(256) void aln_chain_prep_kernel(AlnParams P, uint32_t n_chains) {
    const int64_t l2 = P.l_pac << 1;
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < n_chains; c += gridDim.x * blockDim.x) {
        const uint32_t rv = P.chain_read[c];
        const uint32_t r = rv & 0x3fffffffu;
        const bool giant = (rv >> 30 & 1u) != 0;
        const bool heavy = (rv >> 31) != 0;
        const OutChain ch = P.chains[c];
        P.sdec[c] = 0;
        if (heavy) P.short_ok[c] = 0;
        if (ch.n <= 0) continue;
        const int L = (int)(P.offs[r + 1] - P.offs[r]);
        const SeedRec* S = P.seeds + ch.seed_off;
        int64_t qb = L, qe = 0, rb = l2, re = 0, r0 = l2, r1 = 0;
        uint64_t best = 0;
        int top = 0;
        for (int i = 0; i < ch.n; ++i) {
            const SeedRec s = S[i];
            qb = s.qbeg < qb ? s.qbeg : qb;
            qe = s.qbeg + s.len > qe ? s.qbeg + s.len : qe;
            rb = s.rbeg < rb ? s.rbeg : rb;
            re = s.rbeg + s.len > re ? s.rbeg + s.len : re;
            const int64_t b = s.rbeg - (s.qbeg + max_gap(P, s.qbeg));
            const int64_t e = s.rbeg + s.len + ((L - s.qbeg - s.len) + max_gap(P, L - s.qbeg - s.len));
            r0 = b < r0 ? b : r0;
            r1 = e > r1 ? e : r1;
            const uint64_t key = (uint64_t)(uint32_t)s.len << 32 | (uint32_t)i;  // distinct: the largest is srt[n - 1]
            if (key > best) best = key, top = i;
            P.pre_ok[ch.seed_off + i] = 0;
        }
        qb -= 50, qe += 50, rb -= 50, re += 50;  // MEM_SHORT_EXT
        bool decline = qb <= 10 || qe >= L - 10;
        rb = rb > 0 ? rb : 0;
        re = re < l2 ? re : l2;
        if (rb < P.l_pac && P.l_pac < re) {
            if (S[0].rbeg < P.l_pac) re = P.l_pac;
            else rb = P.l_pac;
        }
        decline = decline || (re - rb) - (qe - qb) > 50 || (qe - qb) - (re - rb) > 50;
        decline = decline || qe - qb >= P.w * 4 || re - rb >= P.w * 4;
        decline = decline || qe - qb >= 200 || re - rb >= 200;  // MEM_SHORT_LEN
        r0 = r0 > 0 ? r0 : 0;
        r1 = r1 < l2 ? r1 : l2;
        if (r0 < P.l_pac && P.l_pac < r1) {
            if (S[0].rbeg < P.l_pac) r1 = P.l_pac;
            else r0 = P.l_pac;
        }
        P.span[2 * (uint64_t)c] = r0;
        P.span[2 * (uint64_t)c + 1] = r1;
        P.sdec[c] = (uint8_t)decline;
        if (!heavy) {
            if (decline) P.tasks[atomicAdd(&P.lq[LQ_NTASK], 1u)] = RegTask{c, r, (uint32_t)top};
        } else if (decline) {
            // one atomic per list at a uniform address (the compiler's atomic optimizer
            // folds a wave's into one; at a per-lane selected address it cannot:
            // 37 ms instead of 0.9 for the human-like profile's 3.2 M heavy chains)
            RegTask* const tl = giant ? P.gtasks : P.htasks;
            const uint32_t n = (uint32_t)ch.n;
            uint32_t base = atomicAdd(&P.hlq[LQ_NTASK], giant ? 0u : n);
            if (P.glq) {
                const uint32_t bg = atomicAdd(&P.glq[LQ_NTASK], giant ? n : 0u);
                base = giant ? bg : base;
            }
            for (int i = 0; i < ch.n; ++i) tl[base + i] = RegTask{c, r, (uint32_t)i};
        } else {
            P.swlist[atomicAdd(&P.hlq[LQ_NSW], 1u)] = c;
        }
    }
}

// the listed heavy chains, one wave each: mem_chain2aln_short's SW (its
// region to pre_short, short_ok = 1), or, when it declines, every seed as a task
__global__ __launch_bounds__(256) void aln_heavy_sw_kernel(AlnParams P) {
    const int lane = threadIdx.x & 63;
    const uint32_t n = P.hlq[LQ_NSW];
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, n_waves = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t k = wave; k < n; k += n_waves) {
        const uint32_t c = (uint32_t)uni((int)P.swlist[k]);
        const uint32_t rv = (uint32_t)uni((int)P.chain_read[c]);
        const uint32_t r = rv & 0x3fffffffu;
        const bool giant = (rv >> 30 & 1u) != 0;
        const uint64_t q0 = P.offs[r];
        const int L = uni((int)(P.offs[r + 1] - q0));
        OutChain ch = P.chains[c];
        ch.n = uni(ch.n);
        const SeedRec* S = P.seeds + ch.seed_off;
        const int ok = chain_short(P, P.codes + q0, L, S, ch.n, P.pre_short + c, lane, P.ctr + 12) == 0;
        if (lane == 0) P.short_ok[c] = (uint8_t)ok;
        if (!ok) {
            RegTask* const tl = giant ? P.gtasks : P.htasks;
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(&(giant ? P.glq : P.hlq)[LQ_NTASK], (uint32_t)ch.n);
            base = (uint32_t)uni((int)base);
            for (int i = lane; i < ch.n; i += 64) tl[base + i] = RegTask{c, r, (uint32_t)i};
        }
    }
}

// the query length of task t's extension in pass `side` (0 left, 1 right);
// LQ_BUCKETS - 1: not run by the lanes (longer than LQ_MAXQ, or failed before)
__device__ __forceinline__ int task_key(const AlnParams& P, uint32_t t, int side) {
    const RegTask T = P.tasks[t];
    const SeedRec s = P.seeds[P.chains[T.c].seed_off + T.si];
    int q;
    if (side == 0) {
        q = s.qbeg;
    } else {
        if (P.tfail[t]) return LQ_BUCKETS - 1;
        q = (int)(P.offs[T.r + 1] - P.offs[T.r]) - s.qbeg - s.len;
    }
    const bool gap = P.max_len > 0 && P.max_len <= LQ_GAP_HI + 1;  // no 256 tier in this batch
    return q <= LQ_MAXQ && !(gap && q >= LQ_GAP_LO && q <= LQ_GAP_HI) ? q : LQ_BUCKETS - 1;
}

// counting sort of the tasks by the pass's query length: block histograms in
// LDS, one global add per length per block
__global__ __launch_bounds__(256) void aln_task_hist_kernel(AlnParams P, int side) {
    __shared__ uint32_t h[LQ_BUCKETS];
    for (int k = threadIdx.x; k < LQ_BUCKETS; k += blockDim.x) h[k] = 0;
    __syncthreads();
    const uint32_t n = P.lq[LQ_NTASK];
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
        if (side == 0) P.tfail[t] = 0;
        atomicAdd(&h[task_key(P, t, side)], 1u);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < LQ_BUCKETS; k += blockDim.x)
        if (h[k]) atomicAdd(&P.lq[LQ_HIST + k], h[k]);
}

// cursors (exclusive scan) and the 16-column queues; heads cleared
__global__ __launch_bounds__(64) void aln_task_scan_kernel(AlnParams P) {
    if (threadIdx.x != 0) return;
    uint32_t a = 0;
    for (int k = 0; k < LQ_BUCKETS; ++k) {  // in place (a private array of LQ_BUCKETS went to scratch)
        const uint32_t v = P.lq[LQ_HIST + k];
        P.lq[LQ_HIST + k] = a;
        a += v;
    }
    P.lq[LQ_BOUNDS] = 0;
    for (int q = 1; q <= LQ_QUEUES; ++q) P.lq[LQ_BOUNDS + q] = P.lq[LQ_HIST + 16 * q + 1];
    for (int q = 0; q < LQ_QUEUES; ++q) P.lq[LQ_HEADS + q] = 0;
}

// the tasks in pass order (a block reserves its share of each length with one
// global add); tasks past LQ_MAXQ columns are marked failed (left to the walk)
__global__ __launch_bounds__(256) void aln_task_scatter_kernel(AlnParams P, int side) {
    __shared__ uint32_t h[LQ_BUCKETS], base[LQ_BUCKETS];
    const uint32_t n = P.lq[LQ_NTASK];
    const uint32_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint32_t t0 = blockIdx.x * per, t1 = t0 + per < n ? t0 + per : n;
    for (int k = threadIdx.x; k < LQ_BUCKETS; k += blockDim.x) h[k] = 0;
    __syncthreads();
    for (uint32_t t = t0 + threadIdx.x; t < t1; t += blockDim.x) atomicAdd(&h[task_key(P, t, side)], 1u);
    __syncthreads();
    for (int k = threadIdx.x; k < LQ_BUCKETS; k += blockDim.x) {
        base[k] = h[k] ? atomicAdd(&P.lq[LQ_HIST + k], h[k]) : 0u;
        h[k] = 0;
    }
    __syncthreads();
    for (uint32_t t = t0 + threadIdx.x; t < t1; t += blockDim.x) {
        const int k = task_key(P, t, side);
        P.torder[base[k] + atomicAdd(&h[k], 1u)] = t;
        if (k == LQ_BUCKETS - 1) P.tfail[t] = 1;
    }
}

// A task's pass through the lane engine: the left extension (reversed query
// and reference, software/bwamem.c:1118-1137) or the right one (:1144-1166)
// with MAX_BAND_TRY, the pass's share of the region written to pre (the left
// pass: qb, rb, score, truesc, w; the right pass: the rest, then
// aln_region_cov_kernel the seed coverage and pre_ok).
struct RegionPol {
    const AlnParams* P;
    int side, top;
    uint32_t t = 0;
    AlnReg* out = nullptr;
    int64_t tpos = 0;  // the reference position of row 0; left rows run downwards
    int64_t rbeg = 0;
    int qbeg = 0, len = 0, L = 0, tr = 0, prev = 0, sc0 = 0;

    template <int KCOL>
    __device__ __forceinline__ bool start(uint32_t k, kswd::ExtIn& T, uint2* qs) {
        t = P->torder[k];
        const RegTask R = P->tasks[t];
        const OutChain ch = P->chains[R.c];
        const SeedRec s = P->seeds[ch.seed_off + R.si];
        const uint64_t q0 = P->offs[R.r];
        const uint8_t* query = P->codes + q0;
        L = (int)(P->offs[R.r + 1] - q0);
        out = P->pre + ch.seed_off + R.si;
        rbeg = s.rbeg, qbeg = s.qbeg, len = s.len, tr = 0;
        if (side == 0) {
            if (qbeg == 0) {  // no left extension
                out->qb = 0, out->rb = rbeg, out->score = out->truesc = len * P->a, out->w = P->w;
                return false;
            }
            T = kswd::ExtIn{qbeg, (int)(rbeg - P->span[2 * R.c]), P->w, P->pen_clip5, P->zdrop, len * P->a};
            if (!kswl::extend_lane_ok(KCOL, T.qlen, T.h0, top)) {
                P->tfail[t] = 1;
                return false;
            }
            kswl::load_query_rev<KCOL>(qs, query + qbeg, qbeg);
            tpos = rbeg - 1, prev = -1;
        } else {
            const int qe = qbeg + len;
            sc0 = prev = out->score;
            if (qe == L) {  // no right extension
                out->qe = L, out->re = rbeg + len, out->w = P->w > out->w ? P->w : out->w;
                return false;
            }
            const int64_t rs = rbeg + len;
            T = kswd::ExtIn{L - qe, (int)(P->span[2 * R.c + 1] - rs), P->w, P->pen_clip3, P->zdrop, sc0};
            if (!kswl::extend_lane_ok(KCOL, T.qlen, T.h0, top)) {
                P->tfail[t] = 1;
                return false;
            }
            kswl::load_query_fwd<KCOL>(qs, query + qe, L - qe);
            tpos = rs;
        }
        return true;
    }
    __device__ __forceinline__ int tsym(int i) const { return ref_at(*P, side == 0 ? tpos - i : tpos + i); }
    __device__ __forceinline__ bool finish(const KswResult& x, kswd::ExtIn& T) {
        const int aw = P->w << tr;
        if (tr == 0 && !(x.score == prev || x.max_off < (aw >> 1) + (aw >> 2))) {  // MAX_BAND_TRY
            prev = x.score, tr = 1, T.w = P->w << 1;
            return true;
        }
        if (side == 0) {
            out->score = x.score, out->w = aw;
            if (x.gscore <= 0 || x.gscore <= x.score - P->pen_clip5) {
                out->qb = qbeg - x.qle, out->rb = rbeg - x.tle, out->truesc = x.score;
            } else {
                out->qb = 0, out->rb = rbeg - x.gtle, out->truesc = x.gscore;
            }
        } else {
            const int qe = qbeg + len;
            const int64_t rs = rbeg + len;
            out->score = x.score, out->w = aw > out->w ? aw : out->w;
            if (x.gscore <= 0 || x.gscore <= x.score - P->pen_clip3) {
                out->qe = qe + x.qle, out->re = rs + x.tle, out->truesc += x.score - sc0;
            } else {
                out->qe = L, out->re = rs + x.gtle, out->truesc += x.gscore - sc0;
            }
        }
        return false;
    }
};

// KCOL-column lane engine over the pass's queues of query lengths up to KCOL
// (32: queues 0-1, 64: 2-3, 144: 4-8, 256: 9-15).  The 144 tier, not 128: a
// 150-bp read's seeds near its ends make extensions of 129-131 columns (2.8 %
// of the human-like profile's tasks), which one wave each took 6.2 ms of the
// heavy reads' critical path (profiles/r06/aln/s6d_human_kernel_stats.csv).
// The 256 tier takes the 250-bp reads' longer extensions (c4), one wave each
// before: its 257-entry column array needs one wave a SIMD (VGPRs + AGPRs).
template <int KCOL>
__global__ __launch_bounds__(256, KCOL > 144 ? 1 : KCOL > 64 ? 2 : 4) void aln_region_lane_kernel(AlnParams P,
                                                                                                 int side) {
    __shared__ uint32_t stab[10];
    __shared__ uint2 qsl[4][KCOL / 8 * 64];
    if (threadIdx.x < 5) kswl::row_scores(P.mat, threadIdx.x, stab[2 * threadIdx.x], stab[2 * threadIdx.x + 1]);
    __syncthreads();
    RegionPol pol{&P, side, P.top};
    kswl::lane_engine<KCOL, 8>(pol, P.lq + LQ_BOUNDS, P.lq + LQ_HEADS, LQ_TIER_Q0(KCOL), LQ_TIER_Q1(KCOL), stab,
                               qsl[threadIdx.x >> 6], P.o_del, P.e_del, P.o_ins, P.e_ins, P.top);
}

// the tasks the lanes left (a query past LQ_MAXQ columns, scores past 16 bits):
// the whole region one wave per task, as the heavy chain tasks did (left to
// the walks, they made the human-like profile's heavy walk 4x slower)
template <int KC>
__global__ __launch_bounds__(256, KC > 4 ? 1 : 4) void aln_region_rest_kernel(AlnParams P) {
    const int lane = threadIdx.x & 63;
    const uint32_t n = P.lq[LQ_NTASK];
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, n_waves = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t t = wave; t < n; t += n_waves) {
        if (!uni((int)P.tfail[t])) continue;
        if (lane == 0) atomicAdd(&P.ctr[14], 1u);  // SMEM_ALN_STATS: tasks left by the lanes
        const RegTask R = P.tasks[t];
        const uint64_t q0 = P.offs[R.r];
        const int L = uni((int)(P.offs[R.r + 1] - q0));
        if ((L > 256) != (KC > 4)) continue;  // the other instantiation's read
        const OutChain ch = P.chains[R.c];
        const SeedRec* S = P.seeds + ch.seed_off;
        const AlnReg a = seed_region<KC>(P, P.codes + q0, L, S, uni(ch.n), S[R.si], P.span[2 * R.c],
                                         P.span[2 * R.c + 1], lane);
        if (lane == 0) {
            P.pre[ch.seed_off + R.si] = a;
            P.pre_ok[ch.seed_off + R.si] = 1;
        }
    }
}

// the regions' seed coverage (software/bwamem.c:1180-1184) and pre_ok, one
// task per thread
__global__ __launch_bounds__(256) void aln_region_cov_kernel(AlnParams P) {
    const uint32_t n = P.lq[LQ_NTASK];
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
        if (P.tfail[t]) continue;
        const RegTask R = P.tasks[t];
        const OutChain ch = P.chains[R.c];
        const SeedRec* S = P.seeds + ch.seed_off;
        AlnReg* a = P.pre + ch.seed_off + R.si;
        const int64_t rb = a->rb, re = a->re;
        const int qb = a->qb, qe = a->qe;
        int cov = 0;
        for (int i = 0; i < ch.n; ++i) {
            const SeedRec u = S[i];
            if (u.qbeg >= qb && u.qbeg + u.len <= qe && u.rbeg >= rb && u.rbeg + u.len <= re) cov += u.len;
        }
        a->sub = 0, a->csub = 0, a->sub_n = 0, a->seedcov = cov, a->secondary = 0, a->hash = 0;
        P.pre_ok[ch.seed_off + R.si] = 1;
    }
}

// regions compacted per read: one wave per read at a time, its regions as 16-B
// words over the lanes (coalesced).  One thread per read copying its regions
// one after the other took 3.1 ms per 1M reads on the human-like profile: a
// tandem-repeat read's thousands of regions on a single lane were the tail.
static_assert(sizeof(AlnReg) % 16 == 0, "regions copy as 16-B words");
__global__ __launch_bounds__(256) void aln_write_kernel(AlnParams P) {
    const int lane = threadIdx.x & 63;
    const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int n_waves = (int)((gridDim.x * blockDim.x) >> 6);
    constexpr uint32_t W = sizeof(AlnReg) / 16;
    for (int r = wave; r < P.n_reads; r += n_waves) {
        const uint64_t nw = uni64(P.n_regs[r]) * W;
        const uint4* src = reinterpret_cast<const uint4*>(P.raw + uni64(P.seed_off[r]));
        uint4* dst = reinterpret_cast<uint4*>(P.out + uni64(P.reg_off[r]));
        for (uint64_t k0 = 0; k0 < nw; k0 += 64) {  // (a wave-uniform loop)
            const uint64_t k = k0 + (uint64_t)lane;
            if (k < nw) dst[k] = src[k];
        }
    }
}

// ksw_align2 of a batch of independent problems, one wave each (qlen <= 256)
__global__ __launch_bounds__(256) void ksw_align2_kernel(KswAParams K) {
    const int lane = threadIdx.x & 63;
    const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int n_waves = (int)((gridDim.x * blockDim.x) >> 6);
    for (int it = wave; it < K.n; it += n_waves) {
        const KswATask T = K.task[it];
        const uint8_t* q = K.q + T.q_off;
        const uint8_t* tg = K.t + T.t_off;
        const kswd::SwAlign a = kswd::sw_align_wave(
            T.qlen, [&](int j) { return (int)q[j]; }, T.tlen, [&](int i) { return (int)tg[i]; }, K.mat, K.o_del,
            K.e_del, K.o_ins, K.e_ins, T.xtra, K.shift, K.top);
        if (lane == 0) K.out[it] = KswAResult{a.score, a.te, a.qe, a.score2, a.te2, a.tb, a.qb};
    }
}

}  // namespace
}  // namespace smem

extern "C" hipError_t smem_launch_ksw_align2(const smem::KswAParams* K, int n_cu, hipStream_t st) {
    if (K->n <= 0) return hipSuccess;
    const int waves = K->n < n_cu * 32 ? K->n : n_cu * 32;
    hipLaunchKernelGGL(smem::ksw_align2_kernel, dim3((waves + 3) / 4), dim3(256), 0, st, *K);
    return hipGetLastError();
}

extern "C" hipError_t smem_launch_aln(const smem::AlnParams* P, int n_cu, int long_reads, hipStream_t st) {
    if (P->n_reads <= 0) return hipSuccess;
    // up to 8 blocks of 4 waves per CU, every wave claiming reads from the
    // queue; with light_claims, enough blocks for every read
    const int waves = (P->n_reads + 3) / 4;
    int blocks = std::max(1, std::min(n_cu * 8, (waves + 3) / 4)), blocks16 = std::max(1, std::min(n_cu * 2, blocks));
    if (P->light_claims) {
        const uint64_t per_block = 4ull * 4 * P->light_claims;  // 4 waves x 4 reads per claim
        blocks = blocks16 = (int)std::max<uint64_t>(1, (P->n_reads + per_block - 1) / per_block);
    }
    if (P->lane_on) {
        if (P->split) hipLaunchKernelGGL((smem::aln_kernel<4, true, true>), dim3(blocks), dim3(256), 0, st, *P);
        else hipLaunchKernelGGL((smem::aln_kernel<4, false, true>), dim3(blocks), dim3(256), 0, st, *P);
    } else {
        if (P->split) hipLaunchKernelGGL((smem::aln_kernel<4, true>), dim3(blocks), dim3(256), 0, st, *P);
        else hipLaunchKernelGGL(smem::aln_kernel<4>, dim3(blocks), dim3(256), 0, st, *P);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !long_reads) return e;
    if (P->lane_on) {
        if (P->split) hipLaunchKernelGGL((smem::aln_kernel<16, true, true>), dim3(blocks16), dim3(256), 0, st, *P);
        else hipLaunchKernelGGL((smem::aln_kernel<16, false, true>), dim3(blocks16), dim3(256), 0, st, *P);
    } else {
        if (P->split) hipLaunchKernelGGL((smem::aln_kernel<16, true>), dim3(blocks16), dim3(256), 0, st, *P);
        else hipLaunchKernelGGL(smem::aln_kernel<16>, dim3(blocks16), dim3(256), 0, st, *P);
    }
    return hipGetLastError();
}

extern "C" hipError_t smem_launch_aln_classify(const smem::AlnParams* P, hipStream_t st) {
    if (P->n_reads <= 0 || !P->heavy_min) return hipSuccess;
    hipLaunchKernelGGL(smem::aln_classify_kernel, dim3((P->n_reads + 255) / 256), dim3(256), 0, st, *P);
    return hipGetLastError();
}

extern "C" hipError_t smem_launch_aln_heavy(const smem::AlnParams* P, int n_cu, int long_reads, int parts,
                                            hipStream_t st) {
    if (parts & 1) {
        hipLaunchKernelGGL(smem::aln_heavy_task_kernel<4>, dim3(n_cu * 8), dim3(256), 0, st, *P);
        if (long_reads) hipLaunchKernelGGL(smem::aln_heavy_task_kernel<16>, dim3(n_cu * 2), dim3(256), 0, st, *P);
    }
    if (!(parts & 2)) return hipGetLastError();
    // the walk kernels use the per-wave hash tables in turn (same stream);
    // walk_guard != 0: the inlined, guarded walk (diagnostic)
    const int wb = P->walk_waves ? (int)(P->walk_waves + 3) / 4  // blocks of 4 waves
                                 : n_cu * (int)(P->walk_wpc ? P->walk_wpc : smem::ALN_WALK_WAVES) / 4;
    if (P->walk_guard) {
        hipLaunchKernelGGL((smem::aln_heavy_kernel<4, true>), dim3(wb), dim3(256), 0, st, *P);
        if (long_reads) hipLaunchKernelGGL((smem::aln_heavy_kernel<16, true>), dim3(wb), dim3(256), 0, st, *P);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(smem::aln_heavy_kernel<4>, dim3(wb), dim3(256), 0, st, *P);
    if (long_reads) hipLaunchKernelGGL(smem::aln_heavy_kernel<16>, dim3(wb), dim3(256), 0, st, *P);
    return hipGetLastError();
}

extern "C" hipError_t smem_launch_aln_heavy_split(const smem::AlnParams* P, uint32_t n_heavy, uint32_t n_giant,
                                                  int32_t* heavy2, uint64_t* hcnt2, uint64_t* hscnt2, uint8_t* rgiant,
                                                  uint32_t* ctr_g, uint32_t* ctr_r, hipStream_t st) {
    hipLaunchKernelGGL(smem::aln_heavy_split_kernel, dim3(1), dim3(1024), 0, st, *P, n_heavy, n_giant, heavy2, hcnt2,
                       hscnt2, rgiant, ctr_g, ctr_r);
    return hipGetLastError();
}

extern "C" hipError_t smem_launch_aln_cand_count(const smem::AlnParams* P, uint32_t n_heavy, uint64_t* cnt,
                                                 uint32_t* hord, hipStream_t st) {
    if (!n_heavy) return hipSuccess;
    hipLaunchKernelGGL(smem::aln_cand_count_kernel, dim3((n_heavy + 255) / 256), dim3(256), 0, st, *P, n_heavy, cnt,
                       hord);
    return hipGetLastError();
}

extern "C" hipError_t smem_launch_aln_cand(const smem::AlnParams* P, const smem::CandParams* C, void* tmp,
                                           size_t* tmp_bytes, int n_cu, hipStream_t st) {
    // each read's slots sorted by rb (its segment [off[h], off[h + 1]))
    if (!tmp) {
        return hipcub::DeviceSegmentedRadixSort::SortPairs(nullptr, *tmp_bytes, C->key, C->key2, C->val, C->val2,
                                                           (int)std::max<uint64_t>(C->m, 1), (int)C->n_heavy, C->off,
                                                           C->off + 1, 0, 34, st);
    }
    if (!C->n_heavy || !C->m) return hipSuccess;
    hipError_t e0 = hipMemsetAsync(C->hmax, 0, sizeof(int64_t) * C->n_heavy, st);
    if (e0 != hipSuccess) return e0;
    hipLaunchKernelGGL(smem::aln_cand_fill_kernel, dim3(n_cu * 16), dim3(256), 0, st, *P, *C, C->n_chains);
    hipError_t e = hipcub::DeviceSegmentedRadixSort::SortPairs(tmp, *tmp_bytes, C->key, C->key2, C->val, C->val2,
                                                               (int)C->m, (int)C->n_heavy, C->off, C->off + 1, 0, 34, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(smem::aln_cand_place_kernel, dim3(n_cu * 16), dim3(256), 0, st, *P, *C);
    hipLaunchKernelGGL(smem::aln_cand_range_kernel, dim3(n_cu * 16), dim3(256), 0, st, *P, *C);
    return hipGetLastError();
}

// the lane path before the walks: every chain's prep and tasks, the heavy
// chains' SWs (smem_launch_aln_prep); then, per task list, per pass (left,
// right) the sort and the three tiers of the lane engine, the coverage pass
// and the tasks the lanes left (smem_launch_aln_passes; long_reads: the batch
// holds reads past 256 bp)
extern "C" hipError_t smem_launch_aln_prep(const smem::AlnParams* P, uint64_t n_chains, int n_cu, int parts,
                                           hipStream_t st) {
    if (P->n_reads <= 0) return hipSuccess;
    if (parts & 1) {
        const int rb = std::max(1, std::min(n_cu * 4, (P->n_reads + 255) / 256));
        const int cb = std::max<int>(1, (int)std::min<uint64_t>((uint64_t)n_cu * 8, (n_chains + 255) / 256));
        hipLaunchKernelGGL(smem::aln_chain_read_kernel, dim3(rb), dim3(256), 0, st, *P);
        hipLaunchKernelGGL(smem::aln_chain_prep_kernel, dim3(cb), dim3(256), 0, st, *P, (uint32_t)n_chains);
    }
    if (parts & 2) hipLaunchKernelGGL(smem::aln_heavy_sw_kernel, dim3(n_cu * 4), dim3(256), 0, st, *P);
    return hipGetLastError();
}

extern "C" hipError_t smem_launch_aln_passes(const smem::AlnParams* P, int n_cu, int long_reads, hipStream_t st) {
    if (P->n_reads <= 0) return hipSuccess;
    for (int side = 0; side < 2; ++side) {
        hipError_t e = hipMemsetAsync(P->lq + smem::LQ_HIST, 0, sizeof(uint32_t) * smem::LQ_BUCKETS, st);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(smem::aln_task_hist_kernel, dim3(n_cu * 2), dim3(256), 0, st, *P, side);
        hipLaunchKernelGGL(smem::aln_task_scan_kernel, dim3(1), dim3(64), 0, st, *P);
        hipLaunchKernelGGL(smem::aln_task_scatter_kernel, dim3(n_cu * 2), dim3(256), 0, st, *P, side);
        hipLaunchKernelGGL(smem::aln_region_lane_kernel<32>, dim3(n_cu * 4), dim3(256), 0, st, *P, side);
        hipLaunchKernelGGL(smem::aln_region_lane_kernel<64>, dim3(n_cu * 4), dim3(256), 0, st, *P, side);
        hipLaunchKernelGGL(smem::aln_region_lane_kernel<144>, dim3(n_cu * 2), dim3(256), 0, st, *P, side);
        if (P->max_len <= 0 || P->max_len > smem::LQ_GAP_HI + 1)
            hipLaunchKernelGGL(smem::aln_region_lane_kernel<256>, dim3(n_cu), dim3(256), 0, st, *P, side);
    }
    hipLaunchKernelGGL(smem::aln_region_cov_kernel, dim3(n_cu * 4), dim3(256), 0, st, *P);
    hipLaunchKernelGGL(smem::aln_region_rest_kernel<4>, dim3(n_cu * 8), dim3(256), 0, st, *P);
    if (long_reads) hipLaunchKernelGGL(smem::aln_region_rest_kernel<16>, dim3(n_cu * 2), dim3(256), 0, st, *P);
    return hipGetLastError();
}

extern "C" hipError_t smem_launch_aln_write(const smem::AlnParams* P, hipStream_t st) {
    if (P->n_reads <= 0) return hipSuccess;
    // one wave per read at a time: 4 waves a block, at most 16 blocks per CU of a 256-CU device
    hipLaunchKernelGGL(smem::aln_write_kernel, dim3(std::min(4096, (P->n_reads + 3) / 4)), dim3(256), 0, st, *P);
    return hipGetLastError();
}

// this file's code object loaded on the current device (see smem_preload_seed)
extern "C" hipError_t smem_preload_aln(void) {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&smem::aln_classify_kernel));
}
