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
//  * Occ buckets are fetched cooperatively by LDS-DMA: every wave-instruction
//    moves 16 whole 64-B buckets (4 lanes x 16 B) into the wave's LDS image;
//  * the forward / prev / curr lists live in a per-lane scratch arena as
//    16-B packed entries, prev[j+1] prefetched while prev[j] is extended;
//  * matches are appended to the read's output region as bwt_smem1 emits
//    them; reversing and merging (software/bwt.c:830, software/bwamem.c:280-301)
//    happen in finalize_kernel, off the latency-bound loop.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include "smem_kernels.h"

namespace smem {

// one 64-B Occ bucket: 4 x u64 checkpoint, 8 x u32 of 16 MSB-first 2-bit symbols
struct Bucket {
    uint4 c01, c23, w03, w47;
};

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

__host__ __device__ __forceinline__ uint4 pack_p(uint64_t x0, uint64_t x1, uint64_t x2, uint32_t end) {
    return make_uint4((uint32_t)x0, (uint32_t)x1, (uint32_t)x2,
                      (uint32_t)(x0 >> 32) | (uint32_t)(x1 >> 32) << 2 | (uint32_t)(x2 >> 32) << 4 | end << 6);
}

__device__ __forceinline__ uint4 load_p(const PIntv* p) { return *reinterpret_cast<const uint4*>(p); }
__device__ __forceinline__ uint64_t p_x0(const uint4& v) { return (uint64_t)(v.w & 3) << 32 | v.x; }
__device__ __forceinline__ uint64_t p_x1(const uint4& v) { return (uint64_t)((v.w >> 2) & 3) << 32 | v.y; }
__device__ __forceinline__ uint64_t p_x2(const uint4& v) { return (uint64_t)((v.w >> 4) & 3) << 32 | v.z; }
__device__ __forceinline__ uint32_t p_end(const uint4& v) { return v.w >> 6; }

// ---- query bases through a 16-byte window held in registers; the window
// is loaded in the uniform section (the state machine yields until it is)
__device__ __forceinline__ int qsel(uint32_t o0, int i, const uint4& qv) {
    const uint32_t a = o0 + (uint32_t)i;  // batches hold < 2^32 bases
    const uint32_t sel = (a >> 2) & 3;
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
    P_BWD_WAIT,     // seed_wp_kernel: the wave is extending the step's entries
    P_BWD_DONE,     // seed_wp_kernel: every entry of the step extended
    P_EXIT
};

constexpr uint32_t NO_BUCKET = 0xFFFFFFFFu;
// backward-list entries per lane kept in LDS.  On the bench workload 86 % of
// curr pushes and 80 % of prev reads fall below 7 (99 % below 12); 7 entries
// keep the wave at 13 KB of LDS, so 3 blocks of 4 waves fit a CU, which
// measured faster than 12 entries at 2 blocks (39.5 vs 42.1 ms per 1M reads).
// The forward list itself stays in global memory.
[[maybe_unused]] constexpr int LIST_LDS = 7;

// Wave-private LDS.  img: the Occ bucket image (FETCH_OCC64: 4 planes
// [slot*2 + chunk][lane]; FETCH_LANE: 8 planes [k0..k3, l0..l3][lane];
// FETCH_COOP: [k|l][lane][4 chunks]).  pn / q: one 16-B landing slot per lane
// for prev[j+1] and for the query window, filled by LDS-DMA.  The first
// NLIST entries of the lane's backward interval list (curr, which becomes
// prev) live in WaveListT, entry-major so that a wave's accesses are
// bank-conflict free whatever entry each lane is at.
template <int NIMG>
struct WaveLdsT {
    uint4 img[NIMG][64];
    uint4 pn[64];
    uint4 q[64];
};
template <>
struct WaveLdsT<0> {  // VSLOT: the bucket slots live in registers
    uint4 pn[64];
    uint4 q[64];
};

// the backward-list entries kept in LDS, per wave [entry][lane].  A separate
// __shared__ object from the LDS-DMA targets above, so the compiler can see
// that reading a list entry does not wait for bucket DMAs in flight.
template <int NLIST>
struct WaveListT {
    uint4 e[NLIST > 0 ? NLIST : 1][64];
};

// The lane id, recomputed where it is used: the register allocator would
// otherwise keep it (and addresses derived from it) live across the whole
// state machine, or spill them.
__device__ __forceinline__ int vlane() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

// bucket b's 16-B chunk as scalar base + 32-bit byte offset (the host keeps
// the index below 4 GiB), so the DMA takes the saddr form
__device__ __forceinline__ const uint32_t* boff(const uint32_t* __restrict__ bwt, uint32_t b, uint32_t chunk) {
    return reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(bwt) + (b * 64u + chunk * 4u));
}

#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

enum FetchMode { FETCH_LANE = 0, FETCH_COOP = 1, FETCH_OCC64 = 2 };

// Fetch the 64-B Occ buckets of k and l (l only when it is another bucket,
// bwt_2occ4's same-bucket case) for every lane that has an extend request,
// by LDS-DMA, and return them in registers.
//  FETCH_COOP (default): each instruction moves 16 whole buckets (4 lanes x
//    16 B, bucket indices exchanged by ds_bpermute).
//  FETCH_LANE: every lane DMAs its own bucket, one 16-B chunk per
//    instruction (8 instructions: 4 chunks x k, l), into chunk planes.
//  On uniformly random buckets of a 1 GB table (tools/gather_ceiling.hip)
//  FETCH_LANE reads 3.1x faster (43.6 vs 13.9 G buckets/s), but in the
//  seeding kernel, whose accesses share upper FM-index levels, FETCH_COOP
//  is 14 % faster (51.8 vs 60.5 ms per 1M reads, 1 Gbp): kept both for A/B.
template <int FETCH, class WL>
__device__ __forceinline__ void fetch_buckets(const uint32_t* __restrict__ bwt, WL* W, bool want,
                                              uint64_t kk, uint64_t ll, Bucket& vk, Bucket& vl) {
    const bool needl = want && (kk >> 7) != (ll >> 7);
    if constexpr (FETCH == FETCH_LANE) {
        const uint32_t bk = (uint32_t)(kk >> 7), bl = (uint32_t)(ll >> 7);
        if (want) {
#pragma unroll
            for (int q = 0; q < 4; ++q)
                __builtin_amdgcn_global_load_lds(boff(bwt, bk, 4 * q), LDS_PTR(&W->img[q][0]), 16, 0, 0);
        }
        if (needl) {
#pragma unroll
            for (int q = 0; q < 4; ++q)
                __builtin_amdgcn_global_load_lds(boff(bwt, bl, 4 * q), LDS_PTR(&W->img[4 + q][0]), 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int lane = vlane();
        vk = Bucket{W->img[0][lane], W->img[1][lane], W->img[2][lane], W->img[3][lane]};
        const int o = needl ? 4 : 0;  // read the l planes only where they were fetched
        vl = Bucket{W->img[o][lane], W->img[o + 1][lane], W->img[o + 2][lane], W->img[o + 3][lane]};
    } else {
        uint4(*img)[4] = reinterpret_cast<uint4(*)[4]>(&W->img[0][0]);  // [k 64 | l 64][4 chunks]
        const uint32_t bk = want ? (uint32_t)(kk >> 7) : NO_BUCKET;
        const uint32_t bl = needl ? (uint32_t)(ll >> 7) : NO_BUCKET;
        const int lane = vlane();
        const uint32_t chunk = (uint32_t)(lane & 3) * 4;
        // all 8 source lookups first (one LDS wait), then the 8 DMAs
        uint32_t sk[4], sl[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int src = (16 * r + (lane >> 2)) << 2;  // ds_bpermute byte address
            sk[r] = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)bk);
            sl[r] = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)bl);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (sk[r] != NO_BUCKET) __builtin_amdgcn_global_load_lds(boff(bwt, sk[r], chunk), LDS_PTR(&img[16 * r][0]), 16, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (sl[r] != NO_BUCKET)
                __builtin_amdgcn_global_load_lds(boff(bwt, sl[r], chunk), LDS_PTR(&img[64 + 16 * r][0]), 16, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        vk = Bucket{img[lane][0], img[lane][1], img[lane][2], img[lane][3]};
        const uint4* src = needl ? &img[64 + lane][0] : &img[lane][0];
        vl = Bucket{src[0], src[1], src[2], src[3]};
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

// ---- Occ64: the index re-laid for the GPU as one 32-B bucket per 64 BWT
// symbols (same 0.5 B/symbol as the reference's 64 B per 128).  Words 0-2:
// Occ(C), Occ(G), Occ(T) before the bucket, low 32 bits; word 3: their bits
// 32-33 (C | G << 2 | T << 4); words 4-7: the 64 symbols, 16 per word,
// MSB-first as in the reference (software/bwt.h:71-78).  Occ(A) is implied:
// the $ row is not in the BWT, so A + C + G + T = position.  A rank then reads
// one 32-B bucket and popcounts at most 4 words.
struct Bucket32 {
    uint4 cnt, sym;
};

__device__ __forceinline__ uint64_t occ_cgt(const uint4& c, int i) {
    const uint32_t lo = i == 0 ? c.x : (i == 1 ? c.y : c.z);
    return (uint64_t)((c.w >> (2 * i)) & 3) << 32 | lo;
}

// C, G, T among the first pos+1 (pos < 64) symbols of the bucket: the 64
// MSB-first 2-bit symbols as two 64-bit halves, each masked to its share of
// the prefix by one shift (8 fewer VALU per rank than four masked words)
__device__ __forceinline__ void count_cgt4(const uint4& v, uint32_t pos, uint32_t& C, uint32_t& G, uint32_t& T) {
    const uint64_t a = (uint64_t)v.x << 32 | v.y, b = (uint64_t)v.z << 32 | v.w;
    const uint32_t n = pos + 1;  // symbols counted, 1..64
    const uint64_t ma = n >= 32 ? ~0ull : ~0ull << (64 - 2 * n);
    const uint64_t mb = n <= 32 ? 0ull : ~0ull << (128 - 2 * n);
    const uint64_t xa = a & ma, xb = b & mb;
    constexpr uint64_t K = 0x5555555555555555ull;
    const uint64_t loa = xa & K, hia = (xa >> 1) & K, lob = xb & K, hib = (xb >> 1) & K;
    T = __popcll(loa & hia) + __popcll(lob & hib);
    C = __popcll(loa) + __popcll(lob) - T;
    G = __popcll(hia) + __popcll(hib) - T;
}

// ---- Occ192: 64-B lines of 192 BWT symbols (a third fewer index bytes than
// Occ64, and more k / l pairs in one line).  Chunk 0: Occ(C), Occ(G), Occ(T)
// before the line's second 64-symbol block (34 bits: low 32 in words 0-2,
// bits 32-33 in word 3 bits 0-5) and the C / G / T counts of that block
// (7 bits each, word 3 bits 6-26).  Chunks 1-3: the line's three blocks of
// 64 symbols, as Occ64's symbol words.  A rank in block r of a line reads
// chunk 0 and chunk 1 + r (still two 16-B loads): r = 0 subtracts the
// block's symbols after the position, r = 1 adds those up to it, r = 2 adds
// the middle block's counts as well.  Slot tags stay the 64-symbol block.
__device__ __forceinline__ void rank192(const Bucket32& v, uint64_t kk, uint64_t& tC, uint64_t& tG, uint64_t& tT) {
    const uint32_t b = (uint32_t)(kk >> 6), r = b - 3u * (b / 3u), p = (uint32_t)(kk & 63);
    uint32_t C, G, T;
    count_cgt4(v.sym, p, C, G, T);
    const uint64_t c0 = occ_cgt(v.cnt, 0), g0 = occ_cgt(v.cnt, 1), t0 = occ_cgt(v.cnt, 2);
    if (r == 0) {
        uint32_t C6, G6, T6;
        count_cgt4(v.sym, 63, C6, G6, T6);
        tC = c0 - (C6 - C);
        tG = g0 - (G6 - G);
        tT = t0 - (T6 - T);
    } else {
        const uint32_t w = r == 2 ? v.cnt.w : 0u;
        tC = c0 + ((w >> 6) & 127u) + C;
        tG = g0 + ((w >> 13) & 127u) + G;
        tT = t0 + ((w >> 20) & 127u) + T;
    }
}

// bwt_extend for the child c only (as extend_counts) on Occ64 buckets (or
// Occ192 lines)
template <bool L192 = false>
__device__ __forceinline__ void extend_counts64(const SeedParams& P, uint64_t a, uint64_t b, uint64_t s, int c,
                                                uint64_t kk, uint64_t ll, const Bucket32& vk, const Bucket32& vl,
                                                uint64_t& na, uint64_t& nb, uint64_t& ns) {
    uint64_t tk1, tk2, tk3, tl1, tl2, tl3;
    if constexpr (L192) {
        rank192(vk, kk, tk1, tk2, tk3);
        rank192(vl, ll, tl1, tl2, tl3);
    } else {
        uint32_t Ck, Gk, Tk, Cl, Gl, Tl;
        count_cgt4(vk.sym, (uint32_t)(kk & 63), Ck, Gk, Tk);
        count_cgt4(vl.sym, (uint32_t)(ll & 63), Cl, Gl, Tl);
        tk1 = occ_cgt(vk.cnt, 0) + Ck, tk2 = occ_cgt(vk.cnt, 1) + Gk, tk3 = occ_cgt(vk.cnt, 2) + Tk;
        tl1 = occ_cgt(vl.cnt, 0) + Cl, tl2 = occ_cgt(vl.cnt, 1) + Gl, tl3 = occ_cgt(vl.cnt, 2) + Tl;
    }
    const uint64_t tk0 = kk + 1 - tk1 - tk2 - tk3, tl0 = ll + 1 - tl1 - tl2 - tl3;
    const uint64_t d0 = tl0 - tk0, d1 = tl1 - tk1, d2 = tl2 - tk2, d3 = tl3 - tk3;
    const uint64_t L2c = sel4(c, P.L2[0], P.L2[1], P.L2[2], P.L2[3]);
    na = L2c + 1 + sel4(c, tk0, tk1, tk2, tk3);
    ns = sel4(c, d0, d1, d2, d3);
    const uint64_t gt = (c < 1 ? d1 : 0) + (c < 2 ? d2 : 0) + (c < 3 ? d3 : 0);
    nb = b + (uint64_t)(a <= P.primary && a + s - 1 >= P.primary) + gt;
}

// Fetch the Occ64 buckets of k and l (issue: DMAs, tags; read: after the
// wave's vmcnt wait).  Each lane keeps the two buckets it
// fetched last in two LDS slots (planes [2*slot + chunk][lane]) with their
// indices in t0 / t1: consecutive extends of one lane often need the same
// bucket again (nested intervals of one backward step: 30 % of the buckets
// on the bench workload), and those are not fetched again.  Every lane DMAs
// its own buckets, one 16-B chunk per instruction (at most 4 instructions).
// the two 16-B chunks of 64-symbol block b: Occ64 bucket b, or Occ192 line b / 3
template <bool L192>
__device__ __forceinline__ void block_chunks(const uint32_t* __restrict__ occ, uint32_t b, const uint32_t*& c0,
                                             const uint32_t*& c1) {
    if constexpr (L192) {
        const uint32_t line = b / 3u;
        c0 = boff(occ, line, 0);
        c1 = boff(occ, line, 4u * (1u + b - 3u * line));
    } else {
        c0 = boff(occ, b >> 1, (b & 1) * 8);
        c1 = boff(occ, b >> 1, (b & 1) * 8 + 4);
    }
}

template <class WL, bool L192 = false>
__device__ __forceinline__ void fetch_occ64_issue(const uint32_t* __restrict__ occ, WL* W, uint64_t kk, uint64_t ll,
                                                  uint32_t& t0, uint32_t& t1, int& ks, int& ls) {
    const uint32_t bk = (uint32_t)(kk >> 6), bl = (uint32_t)(ll >> 6);
    const bool needl = bk != bl;
    ks = bk == t0 ? 0 : (bk == t1 ? 1 : -1);
    ls = !needl ? ks : (bl == t0 ? 0 : (bl == t1 ? 1 : -1));
    const bool kmiss = ks < 0, lmiss = needl && ls < 0;
    if (kmiss) ks = (needl && ls == 0) ? 1 : 0;  // keep the slot l hits
    if (!needl) ls = ks;
    else if (lmiss) ls = ks ^ 1;
    const bool f0 = (kmiss && ks == 0) || (lmiss && ls == 0);
    const bool f1 = (kmiss && ks == 1) || (lmiss && ls == 1);
    const uint32_t b0 = (kmiss && ks == 0) ? bk : bl, b1 = (kmiss && ks == 1) ? bk : bl;
    if (f0) {
        const uint32_t *a0, *a1;
        block_chunks<L192>(occ, b0, a0, a1);
        __builtin_amdgcn_global_load_lds(a0, LDS_PTR(&W->img[0][0]), 16, 0, 0);
        __builtin_amdgcn_global_load_lds(a1, LDS_PTR(&W->img[1][0]), 16, 0, 0);
        t0 = b0;
    }
    if (f1) {
        const uint32_t *a0, *a1;
        block_chunks<L192>(occ, b1, a0, a1);
        __builtin_amdgcn_global_load_lds(a0, LDS_PTR(&W->img[2][0]), 16, 0, 0);
        __builtin_amdgcn_global_load_lds(a1, LDS_PTR(&W->img[3][0]), 16, 0, 0);
        t1 = b1;
    }
}

// The same slot policy with the two slots in registers (VSLOT): the missing
// buckets are loaded straight into s0 / s1 (the lanes that hit keep theirs)
// NT: the bucket loads non-temporal (streamed through L2 without displacing
// the lanes' list-arena and output lines)
typedef uint32_t nt_v4u __attribute__((ext_vector_type(4)));
template <bool L192 = false, bool NT = false>
__device__ __forceinline__ uint4 ld_bucket16(const uint32_t* a) {
    if constexpr (NT) {
        const nt_v4u v = __builtin_nontemporal_load(reinterpret_cast<const nt_v4u*>(a));
        return make_uint4(v.x, v.y, v.z, v.w);
    }
    return *reinterpret_cast<const uint4*>(a);
}
template <bool L192 = false, bool NT = false>
__device__ __forceinline__ void fetch_occ64_issue_regs(const uint32_t* __restrict__ occ, uint64_t kk, uint64_t ll,
                                                       uint32_t& t0, uint32_t& t1, int& ks, int& ls, uint4& s0a,
                                                       uint4& s0b, uint4& s1a, uint4& s1b) {
    const uint32_t bk = (uint32_t)(kk >> 6), bl = (uint32_t)(ll >> 6);
    const bool needl = bk != bl;
    ks = bk == t0 ? 0 : (bk == t1 ? 1 : -1);
    ls = !needl ? ks : (bl == t0 ? 0 : (bl == t1 ? 1 : -1));
    const bool kmiss = ks < 0, lmiss = needl && ls < 0;
    if (kmiss) ks = (needl && ls == 0) ? 1 : 0;  // keep the slot l hits
    if (!needl) ls = ks;
    else if (lmiss) ls = ks ^ 1;
    const bool f0 = (kmiss && ks == 0) || (lmiss && ls == 0);
    const bool f1 = (kmiss && ks == 1) || (lmiss && ls == 1);
    const uint32_t b0 = (kmiss && ks == 0) ? bk : bl, b1 = (kmiss && ks == 1) ? bk : bl;
    if (f0) {
        const uint32_t *a0, *a1;
        block_chunks<L192>(occ, b0, a0, a1);
        s0a = ld_bucket16<L192, NT>(a0);
        s0b = ld_bucket16<L192, NT>(a1);
        t0 = b0;
    }
    if (f1) {
        const uint32_t *a0, *a1;
        block_chunks<L192>(occ, b1, a0, a1);
        s1a = ld_bucket16<L192, NT>(a0);
        s1b = ld_bucket16<L192, NT>(a1);
        t1 = b1;
    }
}

// after the wait: the lane's k and l buckets from its slots
template <class WL>
__device__ __forceinline__ void fetch_occ64_read(WL* W, int ks, int ls, Bucket32& vk, Bucket32& vl) {
    const int lane = vlane();
    ks = ks < 0 ? 0 : ks;  // lanes without a request read a slot and ignore it
    ls = ls < 0 ? 0 : ls;
    vk = Bucket32{W->img[2 * ks][lane], W->img[2 * ks + 1][lane]};
    vl = Bucket32{W->img[2 * ls][lane], W->img[2 * ls + 1][lane]};
}

// offsets of work item `it` (read_ids maps overflow-pass items to reads)
__device__ __forceinline__ void next_offsets(const SeedParams& P, int it, uint32_t& o0, int& len, int& rid) {
    if (it >= P.n_items) {
        len = 0;
        return;
    }
    rid = P.read_ids ? P.read_ids[it] : it;
    const uint64_t a = P.offs[rid], b = P.offs[rid + 1];
    o0 = (uint32_t)a;
    len = (int)(b - a);
}

// a raw output record (Intv 32 B / CallRec 16 B), non-temporal when NT
template <bool NT, class T>
__device__ __forceinline__ void put_rec(T* p, const T& v) {
    static_assert(sizeof(T) % 16 == 0, "16-B records");
    if constexpr (NT) {
        const uint4* s = reinterpret_cast<const uint4*>(&v);
        nt_v4u* d = reinterpret_cast<nt_v4u*>(p);
#pragma unroll
        for (int k = 0; k < (int)(sizeof(T) / 16); ++k) {
            nt_v4u w;
            w.x = s[k].x, w.y = s[k].y, w.z = s[k].z, w.w = s[k].w;
            __builtin_nontemporal_store(w, d + k);
        }
    } else {
        *p = v;
    }
}

// chip-wide 100 MHz clock: wave start / end times comparable across XCDs
__device__ __forceinline__ uint64_t rtstamp() {
    uint64_t t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

__device__ __forceinline__ uint64_t stamp() {
    uint64_t t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

// STAMP: diagnostic build only (variant 9) — per-wave cycle split written to P.dbg_buf
// FRING: the forward list goes to the LDS list slots too, as a ring of the
// last NLIST pushes (an older entry is written to the arena when the ring
// wraps), so that the first backward step reads prev[0 .. NLIST) from LDS and
// only longer forward lists touch HBM.  List index k < NLIST of every list of
// one bwt_smem1 call then lives in slot (R - k) mod NLIST, R = the slot of the
// last forward push (prev[0]): curr[k] still overwrites prev[k] only after it
// was read.
// DUAL: a lane in a backward step with two or more entries left extends
// prev[j] and prev[j+1] in the same iteration (the entries of one step are
// independent, software/bwt.c:812-826) and consumes both results in order
// next iteration: half the iterations -- state-machine passes and memory
// round trips -- for the multi-entry steps.  The second extend's buckets
// come from the lane's LDS slots when the first fetched them, else straight
// into registers.
// VSLOT: the two bucket slots per lane in registers instead of LDS (4 KB of
// LDS per wave back for list entries); with DUAL the second extend is issued
// only when both its buckets are in the slots after the first one's fetch.
// KT: an extend whose result is a string of at most P.kt_k bases reads that
// string's bi-interval from the k-mer table (one 16-B probe, no rank) instead
// of two Occ buckets: a bi-interval is a function of the string alone, so the
// result is the one bwt_extend computes.  The lane keeps the 2-bit codes of
// its forward string (first kt_k bases) and, in the backward phase, of the
// kt_k bases from the current position (rolled one base per step).
// PRIO (A/B): wave priority by phase -- 1: raised from the top of an
// iteration (the advance) until its loads are issued, 2: raised for the
// extend arithmetic after the wait (s_setprio; the SQ's arbitration between
// the three waves of a SIMD)
// NTM (A/B, bits): 1 the Occ bucket loads non-temporal; 2 the raw outputs
// (intervals, list records) stored non-temporal -- finalize_kernel reads them
// once, later, so they need not occupy L2 beside the list arena
template <int FETCH, bool STAMP, int WPE, int NLIST, bool SINGLE = true, bool EARLY = false, bool L192 = false,
          bool FRING = false, bool DUAL = false, bool VSLOT = false, bool KTAB = false, bool PFCH = false, int PRIO = 0,
          int NTM = 0>
__global__ __launch_bounds__(256, WPE) void seed_kernel(SeedParams P) {
    // backward lists: the first NLIST entries live in LDS
    constexpr int NL = NLIST;
    constexpr bool VS = VSLOT && FETCH == FETCH_OCC64 && !EARLY;
    constexpr bool KT = KTAB && VS && !DUAL;
    using WaveLds = WaveLdsT<VS ? 0 : (FETCH == FETCH_OCC64 ? 4 : 8)>;
    __shared__ WaveLds lds[4];  // one per wave of the 256-thread block
    __shared__ WaveListT<NL> lists[4];
    __shared__ uint32_t scnt[STAMP ? 4 : 1][16];  // STAMP: per-wave block-execution counts
    if constexpr (STAMP) {
        if ((threadIdx.x & 63) < 16) scnt[threadIdx.x >> 6][threadIdx.x & 63] = 0;
    }
    const int lane = threadIdx.x & 63;
    WaveLds* W = &lds[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)];
    WaveListT<NL>* WLs = &lists[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)];
    const uint64_t lane_g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t cap = P.cap_list;
    // per-lane scratch: two packed lists (B0 | B1) used as forward / prev / curr
    PIntv* __restrict__ bp = reinterpret_cast<PIntv*>(P.scratch + lane_g * 2ull * cap);

    // All loads the state machine needs are issued in the uniform section
    // below, next to the bucket DMAs, and consumed in the following
    // iteration: a load consumed inside the divergent advance would stall
    // the whole wave for one memory round trip.  A lane whose next step needs
    // data that is not in flight yet "yields" one iteration instead.
    int phase = P_FETCH;
    int item = -1, len = 0;
    int nitem = 0, nlen = -2;  // next read: -2 nothing claimed, -1 claimed, >= 0 offsets loaded
    int rid = 0, nrid = 0;     // read index of the item (overflow pass: through read_ids)
    // PFCH: the next read's claim and loads are issued in the uniform section
    // beside the bucket loads and consumed at the top of the next iteration,
    // so no wave ever waits on them (the blocking claim at the top stalled
    // the whole wave for two memory round trips in ~12 % of iterations,
    // profiles/r03/stamps): nst walks NST_CLAIM -> NST_CLAIMING -> (overflow
    // pass: NST_RID -> NST_RIDING) -> NST_OFF -> NST_OFFING -> NST_READY, and
    // a lane takes its next read the iteration after it finished one.
    enum { NST_CLAIM = 0, NST_CLAIMING, NST_RID, NST_RIDING, NST_OFF, NST_OFFING, NST_READY };
    int nst = NST_CLAIM;
    int natom = 0, nrank = 0;      // the wave's claim (leader lane's atomic return), this lane's rank in it
    int nridv = 0;                 // overflow pass: read_ids[nitem] in flight
    uint32_t clead = 0;            // the claim's leader lane (wave-uniform)
    uint4 noffv = {0, 0, 0, 0};    // offs[rid], offs[rid + 1] in flight
    uint32_t keep_n = 0;       // intervals of the read that smem_next2 returns (matches + kept sub-matches)
    uint32_t o0 = 0, no0 = 0;
    uint32_t qb = ~0u, qwant = ~0u;      // 16-B query window held / wanted (offsets into codes)
    uint4 qv = {0, 0, 0, 0};
    uint32_t raw_n = 0, calls_n = 0;     // raw intervals / lists logged for the read
    int start = 0, ori_start = 0;
    int x = 0, min_intv = 1, middle = 0, i = 0, j = 0, ret = 0, cur_c = 0;
    uint64_t ik0 = 0, ik1 = 0, ik2 = 0;
    uint32_t ikend = 0;
    // per-lane arena: [0, cap) the forward list (pushed downward, so ascending
    // order is the reversed list bwt_smem1 iterates), [cap, 2 cap) the backward
    // list beyond its first NL entries (which live in LDS).  curr is written in
    // place over prev: curr[k] is pushed after prev[j >= k] has been read.
    uint32_t fwd_n = 0, prev_off = 0, prev_n = 0, curr_n = 0;
    // FRING: the ring position (forward phase), then the slot of list index 0
    uint32_t lr = 0;
    constexpr bool RING = FRING && NL > 0;
    constexpr bool DU = DUAL && RING && NL > 1 && FETCH == FETCH_OCC64 && !EARLY && !L192;
    bool dq = false;                    // DU: the lane's request covers prev[j] and prev[j + 1]
    uint4 pn2 = {0, 0, 0, 0};           // DU: prev[j + 1] for the next request
    uint4 ent2 = {0, 0, 0, 0};          // DU: the second entry of the current request
    uint64_t na2 = 0, nb2 = 0, ns2 = 0; // DU: its result
    uint4 s0a = {0, 0, 0, 0}, s0b = {0, 0, 0, 0}, s1a = {0, 0, 0, 0}, s1b = {0, 0, 0, 0};  // VS: the slots
    // KT: codes of the forward string (its first K bases), of the requested
    // forward string, and of the K bases from backward position i
    uint32_t kc = 0, kreq = 0, kb = 0;
    const int K = KT ? P.kt_k : 0;
    bool prev_lds = false;  // prev is the backward list (LDS + region 2), not the forward list
    uint32_t mem_n = 0, mem_last_start = 0, m_n = 0;
    uint64_t curr_last_x2 = 0;
    // longest match of the first bwt_smem1 (software/bwamem.c:266-270), tracked
    // as matches are emitted: pushes come in reverse final order, so ">="
    // keeps the first maximum in final order
    uint32_t max_len = 0, max_x2 = 0, max_mid = 0;  // x2 saturated to 32 bits
    uint4 pn = {0, 0, 0, 0}, head = {0, 0, 0, 0};  // prev[j+1] in flight, curr[0]
    uint64_t na = 0, nb = 0, ns = 0;
    uint32_t tag0 = ~0u, tag1 = ~0u;  // FETCH_OCC64: buckets held in the lane's two LDS slots
    // wave-cooperative backward step (tail of the batch): idle lanes extend
    // entries of owner lanes' prev lists
    int bat_m = 0;        // this lane's helped entries for its next BWD_RES (owner only)
    uint64_t bat_h = 0;   // the lanes that computed them, in entry order
    uint64_t st_adv = 0, st_fetch = 0, st_comp = 0, st_iter = 0, st_active = 0, st_t0 = 0, st_t1 = 0;
    if constexpr (STAMP) st_t0 = rtstamp();
    // the launch's span on the chip clock: first wave start, last wave end
    if (P.tspan && lane == 0) atomicMax(reinterpret_cast<unsigned long long*>(P.tspan), ~(unsigned long long)rtstamp());

#define QBLK(pos) ((o0 + (uint32_t)(pos)) & ~15u)
// one forward-list push: the arena (pushed downward: ascending order is the
// reversed list) or, RING, the LDS ring, spilling the entry it displaces
#define FWD_PUSH(e_)                                                                        \
    {                                                                                       \
        const uint4 fe_ = (e_);                                                             \
        if constexpr (RING) {                                                               \
            if (fwd_n >= (uint32_t)NL)                                                      \
                *reinterpret_cast<uint4*>(bp + cap - 1 - (fwd_n - NL)) = WLs->e[lr][vlane()]; \
            WLs->e[lr][vlane()] = fe_;                                                      \
            lr = lr + 1 == (uint32_t)NL ? 0u : lr + 1;                                      \
        } else {                                                                            \
            *reinterpret_cast<uint4*>(bp + cap - 1 - fwd_n) = fe_;                          \
        }                                                                                   \
        ++fwd_n;                                                                            \
    }
// the LDS slot of list index k (< NL) of the current bwt_smem1 call
#define LSLOT(r_, k_) (RING ? ((r_) >= (k_) ? (r_) - (k_) : (r_) + (uint32_t)NL - (k_)) : (k_))
#define YIELD_FOR(pos)            \
    {                             \
        qwant = QBLK(pos);        \
        break;                    \
    }

    for (;;) {
        uint64_t ta = 0;
        if constexpr (STAMP) ta = stamp();
        if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(2);
        // claiming the next read and loading its offsets: here, at the top of the
        // iteration, where no bucket DMA is in flight yet for their waits to cover
        if constexpr (PFCH) {
            // what the last iteration's uniform section issued has landed
            // (its vmcnt(0) wait): consume it, issue nothing here
            if (nst == NST_CLAIMING) {
                nitem = __builtin_amdgcn_readlane(natom, clead) + nrank;
                nst = nitem >= P.n_items ? NST_READY : (P.read_ids ? NST_RID : NST_OFF);
                nrid = nitem;
            } else if (nst == NST_RIDING) {
                nrid = nridv;
                nst = NST_OFF;
            } else if (nst == NST_OFFING) {
                no0 = noffv.x;
                nlen = (int)(noffv.z - noffv.x);
                nst = NST_READY;
            }
        } else if (phase == P_FETCH) {
            if (nlen == -2) {  // claim the next read
                nitem = atomicAdd(P.head, 1);
                nlen = -1;
            } else if (nlen == -1) {  // its offsets (the claim returned last iteration)
                next_offsets(P, nitem, no0, nlen, nrid);
            }
        }
        // ---- advance the state machine until the lane needs an extend ----
        // Blocks are laid out in the order the common transitions take, and a
        // block hands over to a LATER block by setting `phase` and falling
        // through: result -> next forward base, forward stop -> list reversal
        // -> first backward step, end of a backward step -> next step all
        // complete in one pass of the wave.  Going back to an earlier block
        // (end of a bwt_smem1 call, next read) takes another pass.  A lane sets
        // `out` when it has an extend request (or yields); the pass has a
        // single exit at the bottom, which keeps the exec-mask bookkeeping of
        // the structurized loop (and so the register count) small.
        // ONE pass per iteration (SINGLE): a lane that still needs an earlier
        // block after this pass (end of a bwt_smem1 call: ~1 % of lane-
        // iterations) continues next iteration without an extend, instead of
        // the whole wave running a second pass.
        bool out = false;
        bool early = false;  // FETCH_OCC64: this lane's bucket fetch was issued in BWD_RES
        int fks = -1, fls = -1;  // its bucket slots
        for (int pass = 0; phase != P_EXIT && (pass == 0 || !SINGLE); ++pass) {
            if constexpr (STAMP) {  // which blocks this pass of the wave starts in (any lane)
                const uint64_t act = __ballot(1);
                uint32_t any = 0;
                for (int ph = 0; ph < P_EXIT; ++ph) any |= (__ballot(phase == ph) ? 1u : 0u) << ph;
                if (lane == __ffsll((unsigned long long)act) - 1) {
                    scnt[threadIdx.x >> 6][15] += 1;
                    for (int ph = 0; ph < P_EXIT; ++ph) scnt[threadIdx.x >> 6][ph] += (any >> ph) & 1;
                }
            }
            out = false;
            if (phase == P_SMEM_END) {
                if (!middle) {  // software/bwamem.c:261-272
                    start = ret;
                    m_n = mem_n;
                    // split_len = min(k * split_factor + .499, len) (software/bwamem.c:456-458)
                    const int split_len = P.split_len_init < len ? P.split_len_init : len;
                    if (m_n > 0 && split_len > 0 && (int)max_len >= split_len &&
                        (uint64_t)max_x2 <= (uint64_t)(int64_t)P.split_width) {
                        // re-seed from the middle of the longest SMEM (software/bwamem.c:272-278)
                        x = (int)max_mid;
                        min_intv = (int)(max_x2 + 1);
                        middle = 1;
                        phase = P_SMEM_BEGIN;
                    }
                }
                if (phase == P_SMEM_END) {
                    // log the list: matches (+ sub-matches) for the finalize pass
                    if (calls_n >= P.cap_calls) {
                        phase = P_OVF;
                    } else {
                        put_rec<(NTM & 2) != 0>(P.out_call + (uint64_t)item * P.cap_calls + calls_n++,
                                                CallRec{m_n, middle ? mem_n : 0u, (uint32_t)ori_start, max_len});
                        phase = P_NEXT2;
                    }
                }
            }
            if (phase == P_OVF) {  // the read does not fit: hand it to the overflow pass
                P.n_intv[item] = SMEM_OVERFLOW;
                P.n_calls[item] = 0;
                const int slot = atomicAdd(P.ovf_count, 1);
                P.ovf_items[slot] = item;
                phase = P_FETCH;
            }
            if (phase == P_FETCH) {
                // claiming the next read and loading its offsets happen in the
                // uniform section; yield until both are done
                if (PFCH ? nst != NST_READY : nlen < 0) {
                    out = true;
                } else if (nitem >= P.n_items) {
                    phase = P_EXIT;
                    out = true;
                } else {
                    item = nitem;
                    rid = nrid;
                    keep_n = 0;
                    o0 = no0;
                    len = nlen;
                    nlen = -2;
                    nst = NST_CLAIM;  // PFCH: the next claim goes out in this iteration's uniform section
                    raw_n = 0;
                    calls_n = 0;
                    start = 0;
                    if (len < P.min_seed_len) {  // mem_chain's guard (software/bwamem.c:600)
                        P.n_intv[item] = 0;
                        P.n_calls[item] = 0;
                        P.s_intv[rid] = 0;
                        P.s_calls[rid] = 0;
                        out = true;  // stays in P_FETCH: the next claim is issued below
                    } else {
                        phase = P_NEXT2;
                    }
                }
            }
            if (phase == P_NEXT2) {  // software/bwamem.c:247-261
                bool wait_q = false;
                if (start < len && start >= 0) {
                    for (;;) {  // skip ambiguous bases
                        if (start >= len) break;
                        if (QBLK(start) != qb) { wait_q = true; break; }
                        if (qsel(o0, start, qv) <= 3) break;
                        ++start;
                    }
                }
                if (wait_q) {
                    qwant = QBLK(start);
                    out = true;
                } else if (start >= len || start < 0) {  // iterator exhausted
                    P.n_intv[item] = raw_n;
                    P.n_calls[item] = calls_n;
                    P.s_intv[rid] = keep_n;  // sizes for the compaction scan (no count pass)
                    P.s_calls[rid] = calls_n;
                    phase = P_FETCH;
                } else {
                    ori_start = start;
                    x = ori_start;
                    min_intv = P.start_width;
                    middle = 0;
                    max_len = 0;
                    phase = P_SMEM_BEGIN;
                }
            }
            if (phase == P_SMEM_BEGIN) {  // software/bwt.c:782-789
                if (QBLK(x) != qb) {
                    qwant = QBLK(x);
                    out = true;
                } else {
                    mem_n = 0;
                    const int qx = qsel(o0, x, qv);
                    if (qx > 3) {
                        ret = x + 1;
                        phase = P_SMEM_END;
                    } else {
                        if (min_intv < 1) min_intv = 1;
                        const uint64_t lq = sel4(qx, P.L2[0], P.L2[1], P.L2[2], P.L2[3]);
                        const uint64_t lq1 = sel4(qx, P.L2[1], P.L2[2], P.L2[3], P.L2[4]);
                        ik0 = lq + 1;
                        ik2 = lq1 - lq;
                        ik1 = sel4(qx, P.L2[3], P.L2[2], P.L2[1], P.L2[0]) + 1;
                        ikend = (uint32_t)(x + 1);
                        if constexpr (KT) kc = (uint32_t)qx;
                        fwd_n = 0;
                        lr = 0;
                        i = x + 1;
                        phase = P_FWD;
                    }
                }
            }
            if (phase == P_BWD_RES) {  // software/bwt.c:815-825; na = x[0], nb = x[1]
                // the lane's own result for prev[j], then (helped owner only) the
                // results idle lanes computed for prev[j+1 .. j+bat_m], in order
                const int own = DU && dq ? 2 : 1;
                const int nres = own + bat_m;
                uint64_t hm = bat_h;
                for (int r = 0; r < nres; ++r) {
                    if (DU && r == 1 && own == 2) {  // the lane's own second result, prev[j + 1]
                        ik0 = p_x0(ent2); ik1 = p_x1(ent2); ik2 = p_x2(ent2); ikend = p_end(ent2);
                        na = na2; nb = nb2; ns = ns2;
                    } else if (r > 0) {
                        const int h = __builtin_ctzll(hm);
                        hm &= hm - 1;
                        const uint4 ent = W->pn[h], res = W->q[h];
                        ik0 = p_x0(ent); ik1 = p_x1(ent); ik2 = p_x2(ent); ikend = p_end(ent);
                        na = p_x0(res); nb = p_x1(res); ns = p_x2(res);
                    }
                    if (ns < (uint64_t)min_intv) {
                        // only prev[0] can be kept, when nothing longer survived
                        if (curr_n == 0 && (mem_n == 0 || (uint32_t)(i + 1) < mem_last_start)) {
                            if (raw_n >= P.cap_intv) {
                                phase = P_OVF;
                                break;
                            }
                            const uint64_t info = (uint64_t)ikend | ((uint64_t)(i + 1) << 32);
                            put_rec<(NTM & 2) != 0>(P.out_intv + (uint64_t)item * P.cap_intv + raw_n++, Intv{ik0, ik1, ik2, info});
                            // the merge keeps a sub-match if it is at least half the longest
                            // match and ends after the call's start (software/bwamem.c:284-292)
                            keep_n += !middle || (ikend - (uint32_t)(i + 1) >= (max_len >> 1) && ikend > (uint32_t)ori_start);
                            ++mem_n;
                            mem_last_start = (uint32_t)(i + 1);
                            if (!middle && ikend - (uint32_t)(i + 1) >= max_len) {
                                max_len = ikend - (uint32_t)(i + 1);
                                max_x2 = ik2 > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)ik2;
                                max_mid = (ikend + (uint32_t)(i + 1)) >> 1;
                            }
                        }
                    } else if (curr_n == 0 || ns != curr_last_x2) {
                        const uint4 e = pack_p(na, nb, ns, ikend);
                        if (NL > 0 && curr_n < (uint32_t)NL)
                            WLs->e[LSLOT(lr, curr_n)][vlane()] = e;
                        else
                            *reinterpret_cast<uint4*>(bp + cap + curr_n) = e;
                        if (curr_n == 0) head = e;  // prev[0] of the next step
                        ++curr_n;
                        curr_last_x2 = ns;
                    }
                    ++j;
                }
                if (phase == P_BWD_RES) {
                    if ((uint32_t)j < prev_n) {  // extend prev[j] (read into pn last iteration) right away
                        ik0 = p_x0(pn); ik1 = p_x1(pn); ik2 = p_x2(pn); ikend = p_end(pn);
                        out = true;
                        if constexpr (DU) {  // and prev[j + 1] (in pn2) with it
                            dq = (uint32_t)j + 1 < prev_n;
                            ent2 = pn2;
                        }
                        if constexpr (FETCH == FETCH_OCC64 && EARLY) {
                            // issue its bucket fetch now: it overlaps the rest of the pass
                            const uint64_t k = ik0 - 1, l = k + ik2;
                            fetch_occ64_issue<WaveLds, L192>(L192 ? P.occ192 : P.occ64, W, k - (k >= P.primary), l - (l >= P.primary), tag0, tag1,
                                              fks, fls);
                            early = true;
                        }
                    } else if (curr_n == 0) {  // software/bwt.c:827
                        phase = P_SMEM_END;
                    } else {
                        prev_off = cap;  // software/bwt.c:828: swap, next position
                        prev_n = curr_n;
                        prev_lds = true;
                        pn = head;
                        --i;
                        phase = P_BWD_STEP;
                    }
                }
            }
            if (phase == P_FWD_RES) {  // software/bwt.c:795-799; na = x[1], nb = x[0]
                bool stop = false;
                if (ns != ik2) {
                    FWD_PUSH(pack_p(ik0, ik1, ik2, ikend));
                    stop = ns < (uint64_t)min_intv;
                }
                if (stop) {
                    phase = P_FWD_DONE;
                } else {
                    ik0 = nb; ik1 = na; ik2 = ns;
                    ikend = (uint32_t)(i + 1);
                    if constexpr (KT) {
                        if (i + 1 - x <= K) kc = kreq;  // saturates at the first K bases
                    }
                    ++i;
                    phase = P_FWD;
                }
            }
            if (phase == P_FWD) {  // software/bwt.c:791-803
                bool push = true;
                if (i < len) {
                    if (QBLK(i) != qb) {
                        qwant = QBLK(i);
                        out = true;
                        push = false;
                    } else {
                        const int qi = qsel(o0, i, qv);
                        if (qi < 4) {
                            cur_c = 3 - qi;
                            if constexpr (KT) kreq = kc << 2 | (uint32_t)qi;
                            if (i + 1 < len) qwant = QBLK(i + 1);
                            phase = P_FWD_RES;  // -> extend (forward)
                            out = true;
                            push = false;
                        }
                    }
                }
                if (push) {  // ambiguous base, or end of query: push ik and stop
                    FWD_PUSH(pack_p(ik0, ik1, ik2, ikend));
                    phase = P_FWD_DONE;
                }
            }
            if (phase == P_FWD_DONE) {  // software/bwt.c:805-808
                // the last push becomes prev[0] after the reversal; it is always the
                // current ik (the stop path pushes ik without advancing it)
                pn = pack_p(ik0, ik1, ik2, ikend);
                ret = (int)ikend;
                prev_off = cap - fwd_n;  // pushed downward: ascending = reversed
                prev_n = fwd_n;
                prev_lds = RING;         // RING: prev[0 .. NL) in the LDS ring
                if constexpr (RING) lr = lr == 0 ? (uint32_t)NL - 1 : lr - 1;  // slot of the last push
                if constexpr (KT) {  // the K bases from x (those past the forward string are never read)
                    const uint32_t lf = ikend - (uint32_t)x;
                    kb = lf >= (uint32_t)K ? kc : kc << (2 * ((uint32_t)K - lf));
                }
                i = x - 1;
                phase = P_BWD_STEP;
            }
            if (phase == P_BWD_STEP) {  // software/bwt.c:810-812; prev[0] is in pn
                if (i >= 0 && QBLK(i) != qb) {
                    qwant = QBLK(i);
                    out = true;
                } else {
                    cur_c = i < 0 ? -1 : qsel(o0, i, qv);
                    if (cur_c > 3) cur_c = -1;
                    curr_n = 0;
                    if (cur_c >= 0) {
                        j = 0;
                        ik0 = p_x0(pn); ik1 = p_x1(pn); ik2 = p_x2(pn); ikend = p_end(pn);
                        if constexpr (KT) kb = (uint32_t)cur_c << (2 * (K - 1)) | kb >> 2;
                        if (i > 0) qwant = QBLK(i - 1);  // the next step's base
                        phase = P_BWD_RES;  // -> extend prev[0]; prev[1] is fetched meanwhile
                        out = true;
                        if constexpr (DU) {  // prev[1] is in its LDS slot (ring or last step's curr)
                            dq = prev_n > 1;
                            if (dq) ent2 = WLs->e[LSLOT(lr, 1u)][vlane()];
                        }
                    } else {
                        // nothing extends: prev[0] is the only candidate
                        phase = P_SMEM_END;
                        if (mem_n == 0 || (uint32_t)(i + 1) < mem_last_start) {
                            if (raw_n >= P.cap_intv) {
                                phase = P_OVF;
                            } else {
                                const uint64_t info = (uint64_t)p_end(pn) | ((uint64_t)(i + 1) << 32);
                                put_rec<(NTM & 2) != 0>(P.out_intv + (uint64_t)item * P.cap_intv + raw_n++,
                                                        Intv{p_x0(pn), p_x1(pn), p_x2(pn), info});
                                keep_n += !middle || (p_end(pn) - (uint32_t)(i + 1) >= (max_len >> 1) &&
                                                      p_end(pn) > (uint32_t)ori_start);
                                ++mem_n;
                                mem_last_start = (uint32_t)(i + 1);
                                if (!middle && p_end(pn) - (uint32_t)(i + 1) >= max_len) {
                                    max_len = p_end(pn) - (uint32_t)(i + 1);
                                    max_x2 = p_x2(pn) > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)p_x2(pn);
                                    max_mid = (p_end(pn) + (uint32_t)(i + 1)) >> 1;
                                }
                            }
                        }
                    }
                }
            }
            if (out) break;
        }
#undef YIELD_FOR
#undef QBLK
        // ---- uniform section: every lane takes part in the cooperative
        // bucket fetch; the loads for the next iteration are issued here ----
        const bool live = phase != P_EXIT;
        bool want = out && (phase == P_BWD_RES || phase == P_FWD_RES);  // an extend request
        uint64_t tb = 0;
        if constexpr (STAMP) {
            tb = stamp();
            st_adv += tb - ta;
            st_iter += 1;
            st_active += __popcll(__ballot(want));
        }
        if (!__any(live)) break;
        // DU with VS: the second extend is kept only when both its buckets are
        // the first extend's (no extra loads); otherwise prev[j + 1] waits for
        // the next iteration.  Decided before the helpers and the prefetch
        // index, which depend on it.
        if constexpr (DU && VS) {
            if (dq && phase == P_BWD_RES && out) {
                const uint64_t k1 = ik0 - 1, l1 = k1 + ik2;
                const uint32_t b1k = (uint32_t)((k1 - (k1 >= P.primary)) >> 6), b1l = (uint32_t)((l1 - (l1 >= P.primary)) >> 6);
                const uint64_t k2 = p_x0(ent2) - 1, l2 = k2 + p_x2(ent2);
                const uint32_t b2k = (uint32_t)((k2 - (k2 >= P.primary)) >> 6), b2l = (uint32_t)((l2 - (l2 >= P.primary)) >> 6);
                dq = (b2k == b1k || b2k == b1l) && (b2l == b1k || b2l == b1l);
            }
        }
        // Lanes that found the work queue empty help: when the wave has idle
        // lanes and a lane in a backward step with more entries left, each idle
        // lane extends one of those entries (same base, independent of each
        // other, software/bwt.c:812-826) and leaves entry + result in its pn / q
        // slots; the owner consumes them in order next iteration.  This cuts the
        // dependent chain of the few repeat-rich reads left at the end.
        bat_m = 0;
        bat_h = 0;
        bool helper = false;
        uint4 hent = {0, 0, 0, 0};
        int hc = 0;
        if constexpr (FETCH == FETCH_OCC64) {
            const uint64_t idle = __ballot(phase == P_EXIT);
            if (idle) {
                // owners in lane order take the idle lanes in rank order, each as
                // many as it has entries left in its step
                uint64_t elig = __ballot(phase == P_BWD_RES && (uint32_t)j + 1 + (DU && dq ? 1u : 0u) < prev_n);
                const uint32_t nidle = (uint32_t)__popcll(idle);
                const int me = vlane();
                const uint32_t r = (uint32_t)__popcll(idle & ((1ull << me) - 1));
                uint32_t base = 0, he = 0, hpoff = 0, hlr = 0;
                int ho = -1, hplds = 0;
                while (elig && base < nidle) {
                    // o is wave-uniform: its state is read with v_readlane (valid
                    // whatever the exec mask, unlike a shuffle from an inactive lane)
                    const int o = __builtin_ctzll(elig);
                    elig &= elig - 1;
                    const uint32_t jo = __builtin_amdgcn_readlane((int)j, o);
                    const uint32_t pno = __builtin_amdgcn_readlane((int)prev_n, o);
                    const uint32_t poff_o = __builtin_amdgcn_readlane((int)prev_off, o);
                    const int plds_o = __builtin_amdgcn_readlane((int)prev_lds, o);
                    const int c_o = __builtin_amdgcn_readlane(cur_c, o);
                    const uint32_t lr_o = RING ? __builtin_amdgcn_readlane((int)lr, o) : 0u;
                    const uint32_t dq_o = DU ? (uint32_t)__builtin_amdgcn_readlane((int)dq, o) : 0u;
                    const uint32_t m = min(nidle - base, pno - jo - 1 - dq_o);
                    const bool mine = phase == P_EXIT && r >= base && r < base + m;
                    if (mine) {
                        ho = o;
                        he = jo + 1 + dq_o + (r - base);
                        hc = c_o;
                        hpoff = poff_o;
                        hplds = plds_o;
                        hlr = lr_o;
                    }
                    const uint64_t hmask = __ballot(mine);
                    if (me == o) {
                        bat_m = (int)m;
                        bat_h = hmask;
                    }
                    base += m;
                }
                helper = ho >= 0;
                if (helper) {
                    // the owner's list: its first NL entries in LDS (after the first
                    // step), the rest in its arena; prev_off / prev_lds are per owner
                    if (NL > 0 && hplds && he < (uint32_t)NL) {
                        hent = WLs->e[LSLOT(hlr, he)][ho];
                    } else {
                        const PIntv* obp = reinterpret_cast<const PIntv*>(
                            P.scratch + ((uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u) + ho) * 2ull * cap);
                        // the entry into this (idle) lane's pn slot by LDS-DMA: no
                        // VGPR-destination load on the main path
                        __builtin_amdgcn_global_load_lds(obp + hpoff + he, LDS_PTR(&W->pn[0]), 16, 0, 0);
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        hent = W->pn[me];
                    }
                }
            }
        }
        if constexpr (PFCH) {
            // the next read's claim / loads, waited for by this iteration's
            // vmcnt(0) below and consumed at the top of the next one
            if (nst == NST_RID) {
                nridv = P.read_ids[nitem];
                nst = NST_RIDING;
            } else if (nst == NST_OFF) {
                const uint2* op = reinterpret_cast<const uint2*>(P.offs + nrid);
                const uint2 a = op[0], b = op[1];   // batches hold < 2^32 bases: the low words
                noffv = make_uint4(a.x, a.y, b.x, b.y);
                nst = NST_OFFING;
            }
            const uint64_t want_claim = __ballot(nst == NST_CLAIM && phase != P_EXIT);
            if (want_claim) {
                const int me = vlane();
                clead = (uint32_t)(__builtin_ffsll((long long)want_claim) - 1);
                if (nst == NST_CLAIM && phase != P_EXIT) {
                    nrank = (int)__popcll(want_claim & ((1ull << me) - 1));
                    if ((uint32_t)me == clead) {
                        // the returning atomic by hand: the compiler's form
                        // (the atomic optimizer's readfirstlane of the result)
                        // waits for it right here.  The value is read at the top
                        // of the next iteration, after this iteration's
                        // s_waitcnt vmcnt(0) below has drained it.
                        const int cnt = (int)__popcll(want_claim);
                        asm volatile("global_atomic_add %0, %1, %2, off sc0"
                                     : "=v"(natom)
                                     : "v"(P.head), "v"(cnt)
                                     : "memory");
                    }
                    nst = NST_CLAIMING;
                }
            }
        }
        // prev[j+1] (the owner of a helped batch: prev[j+1+bat_m]) and the query
        // window land in LDS slots (no VGPR-destination load the compiler would
        // wait on right away); read back after the wait
        const uint32_t pidx = (uint32_t)j + 1 + (DU && dq ? 1u : 0u) + (uint32_t)bat_m;
        const bool ld_pn = phase == P_BWD_RES && pidx < prev_n && !(NL > 0 && prev_lds && pidx < (uint32_t)NL);
        const bool ld_q = qwant != qb && qwant != ~0u;
        if (ld_pn)
            __builtin_amdgcn_global_load_lds(bp + prev_off + pidx, LDS_PTR(&W->pn[0]),
                                             16, 0, 0);
        if (ld_q)
            __builtin_amdgcn_global_load_lds(P.codes + qwant, LDS_PTR(&W->q[0]), 16, 0, 0);
        // the interval to extend: ik forward (a = x[1]), prev[j] backward (a = x[0]),
        // a helper's entry backward
        want = want || helper;
        const bool fwd = phase == P_FWD_RES;
        const uint64_t hx0 = p_x0(hent), hx1 = p_x1(hent), hx2 = p_x2(hent);
        const uint64_t ra = helper ? hx0 : (fwd ? ik1 : ik0), rb = helper ? hx1 : (fwd ? ik0 : ik1),
                       rs = helper ? hx2 : ik2;
        const int rc = helper ? hc : cur_c;
        const uint64_t k = ra - 1, l = k + rs;
        const uint64_t kk = k - (k >= P.primary), ll = l - (l >= P.primary);
        Bucket vk, vl;
        Bucket32 wk, wl;
        // DU: the second extend (prev[j + 1], same base) and the next pn2
        const bool want2 = DU && want && !helper && phase == P_BWD_RES && dq;
        uint64_t ra2 = 0, rb2 = 0, rs2 = 0, kk2 = 0, ll2 = 0;
        int s_k2 = -1, s_l2 = -1;
        uint4 v2k0 = {0, 0, 0, 0}, v2k1 = {0, 0, 0, 0}, v2l0 = {0, 0, 0, 0}, v2l1 = {0, 0, 0, 0};
        const bool ld_pn2 = DU && phase == P_BWD_RES && pidx + 1 < prev_n;
        const bool pn2_lds = NL > 0 && prev_lds && pidx + 1 < (uint32_t)NL;
        uint4 pn2_g = {0, 0, 0, 0};
        if constexpr (DU) {
            if (ld_pn2 && !pn2_lds) pn2_g = *reinterpret_cast<const uint4*>(bp + prev_off + pidx + 1);
        }
        // KT: the result string's length and codes; a short one is one table probe
        bool ktp = false;
        uint4 ktv = {0, 0, 0, 0};
        if constexpr (KT) {
            const int lq = fwd ? i + 1 - x : (int)ikend - i;
            ktp = want && !helper && lq <= K;
            if (ktp) {
                const uint32_t code = fwd ? kreq : kb >> (2 * (K - lq));
                const uint64_t base = ((1ull << (2 * lq)) - 4) / 3;
                ktv = P.kt[base + code];
            }
        }
        if constexpr (VS) {
            if (want && !ktp)
                fetch_occ64_issue_regs<L192, (NTM & 1) != 0>(L192 ? P.occ192 : P.occ64, kk, ll, tag0, tag1, fks, fls, s0a,
                                                             s0b, s1a, s1b);
            if constexpr (DU) {
                if (want2) {
                    ra2 = p_x0(ent2), rb2 = p_x1(ent2), rs2 = p_x2(ent2);
                    const uint64_t k2 = ra2 - 1, l2 = k2 + rs2;
                    kk2 = k2 - (k2 >= P.primary), ll2 = l2 - (l2 >= P.primary);
                    const uint32_t bk2 = (uint32_t)(kk2 >> 6), bl2 = (uint32_t)(ll2 >> 6);
                    s_k2 = bk2 == tag0 ? 0 : 1;  // both are in the slots (checked above)
                    s_l2 = bl2 == tag0 ? 0 : 1;
                }
            }
            if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(2);
            const int ks = fks < 0 ? 0 : fks, ls = fls < 0 ? 0 : fls;
            wk = ks == 0 ? Bucket32{s0a, s0b} : Bucket32{s1a, s1b};
            wl = ls == 0 ? Bucket32{s0a, s0b} : Bucket32{s1a, s1b};
        } else if constexpr (FETCH == FETCH_OCC64) {
            // lanes whose fetch was not issued early in BWD_RES issue it now
            if (want && !early)
                fetch_occ64_issue<WaveLds, L192>(L192 ? P.occ192 : P.occ64, W, kk, ll, tag0, tag1, fks, fls);
            if constexpr (DU) {
                if (want2) {
                    ra2 = p_x0(ent2), rb2 = p_x1(ent2), rs2 = p_x2(ent2);
                    const uint64_t k2 = ra2 - 1, l2 = k2 + rs2;
                    kk2 = k2 - (k2 >= P.primary), ll2 = l2 - (l2 >= P.primary);
                    const uint32_t bk2 = (uint32_t)(kk2 >> 6), bl2 = (uint32_t)(ll2 >> 6);
                    s_k2 = bk2 == tag0 ? 0 : (bk2 == tag1 ? 1 : -1);
                    s_l2 = bl2 == tag0 ? 0 : (bl2 == tag1 ? 1 : (bl2 == bk2 ? 2 : -1));
                    if (s_k2 < 0) {
                        const uint32_t *c0, *c1;
                        block_chunks<false>(P.occ64, bk2, c0, c1);
                        v2k0 = *reinterpret_cast<const uint4*>(c0);
                        v2k1 = *reinterpret_cast<const uint4*>(c1);
                    }
                    if (s_l2 < 0) {
                        const uint32_t *c0, *c1;
                        block_chunks<false>(P.occ64, bl2, c0, c1);
                        v2l0 = *reinterpret_cast<const uint4*>(c0);
                        v2l1 = *reinterpret_cast<const uint4*>(c1);
                    }
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            fetch_occ64_read(W, fks, fls, wk, wl);
        } else {
            fetch_buckets<FETCH>(P.bwt, W, want, kk, ll, vk, vl);  // ends with vmcnt(0)
        }
        if (ld_pn) pn = W->pn[vlane()];
        if constexpr (NL > 0) {  // prev[pidx] from the LDS list: read here, off the advance's critical path
            if (phase == P_BWD_RES && prev_lds && pidx < prev_n && pidx < (uint32_t)NL)
                pn = WLs->e[LSLOT(lr, pidx)][vlane()];
        }
        if constexpr (DU) {
            if (ld_pn2) pn2 = pn2_lds ? WLs->e[LSLOT(lr, pidx + 1)][vlane()] : pn2_g;
        }
        if (ld_q) {
            qv = W->q[vlane()];
            qb = qwant;
        }
        uint64_t tc = 0;
        if constexpr (STAMP) {
            tc = stamp();
            st_fetch += tc - tb;
        }
        if constexpr (DU && VS) {
            if (want2) {
                const Bucket32 wk2 = s_k2 == 0 ? Bucket32{s0a, s0b} : Bucket32{s1a, s1b};
                const Bucket32 wl2 = s_l2 == 0 ? Bucket32{s0a, s0b} : Bucket32{s1a, s1b};
                extend_counts64<false>(P, ra2, rb2, rs2, cur_c, kk2, ll2, wk2, wl2, na2, nb2, ns2);
            }
        } else if constexpr (DU) {
            if (want2) {
                const int lane2 = vlane();
                const Bucket32 wk2 = s_k2 >= 0 ? Bucket32{W->img[2 * s_k2][lane2], W->img[2 * s_k2 + 1][lane2]}
                                               : Bucket32{v2k0, v2k1};
                const Bucket32 wl2 = s_l2 == 2 ? wk2
                                     : s_l2 >= 0 ? Bucket32{W->img[2 * s_l2][lane2], W->img[2 * s_l2 + 1][lane2]}
                                                 : Bucket32{v2l0, v2l1};
                extend_counts64<false>(P, ra2, rb2, rs2, cur_c, kk2, ll2, wk2, wl2, na2, nb2, ns2);
            }
        }
        if (ktp) {  // forward: na is the x[1] side (ik1), backward: the x[0] side
            na = fwd ? p_x1(ktv) : p_x0(ktv);
            nb = fwd ? p_x0(ktv) : p_x1(ktv);
            ns = p_x2(ktv);
        } else if (want) {
            if constexpr (FETCH == FETCH_OCC64)
                extend_counts64<L192>(P, ra, rb, rs, rc, kk, ll, wk, wl, na, nb, ns);
            else
                extend_counts(P, ra, rb, rs, rc, kk, ll, vk, vl, na, nb, ns);
        }
        if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(0);
        if (helper) {  // entry + result for the owner's next BWD_RES
            W->pn[vlane()] = hent;
            W->q[vlane()] = pack_p(na, nb, ns, 0);
        }
        if constexpr (STAMP) {
            asm volatile("" ::"v"(na), "v"(nb), "v"(ns));
            st_comp += stamp() - tc;
        }
    }
#undef FWD_PUSH
#undef LSLOT
    if (P.tspan && lane == 0) atomicMax(reinterpret_cast<unsigned long long*>(P.tspan) + 1, (unsigned long long)rtstamp());
    if constexpr (STAMP) {
        st_t1 = rtstamp();
        if (lane == 0 && P.dbg_buf) {
            uint64_t* o = P.dbg_buf + (lane_g >> 6) * 32;
            o[0] = st_adv; o[1] = st_fetch; o[2] = st_comp; o[3] = st_iter; o[4] = st_active; o[5] = st_t0; o[6] = st_t1;
            for (int k = 0; k < 16; ++k) o[8 + k] = scnt[threadIdx.x >> 6][k];
        }
    }
}

// ======================================================================
// seed_wp_kernel: the same loop with the backward phase wave-parallel over
// list entries (variants 40-43).
//
// A backward step at position i extends every interval of `prev` with the
// same base q[i], and the extends are independent (software/bwt.c:812-826).
// prev is nested (prev[0] is the longest match, each entry's SA interval
// contains the one before it), so the extended sizes are non-decreasing in
// the entry index: the entries that fail (size < min_intv) are a prefix,
// only entry 0 can become a SMEM (the fail branch needs curr->n == 0 and, for
// a second failure, mem's last start is already i + 1), and the survivors
// keep the first of each run of equal sizes (:823).  So a step is one ballot
// of "survives", one of "kept", and a prefix rank of the kept entries -- no
// entry depends on another's result.
//
// Lanes 0 .. OWN-1 of a wave own reads (the smem_next2 / bwt_smem1 state
// machine, as seed_kernel's lanes); every lane of the wave executes one
// bwt_extend per iteration:
//  * an owner in a forward extension (software/bwt.c:791-805: a serial chain)
//    extends its own interval;
//  * every other lane (owners waiting on a backward step, lanes >= OWN, idle
//    owners) takes the next entry of some owner's backward step: the owners'
//    remaining entry counts are prefix-summed across the wave (DPP), owner o
//    gets the free lanes of ranks [excl_o, excl_o + take_o), and each worker
//    finds its owner from the start marks (one LDS scatter + one ballot);
//  * the worker extends the entry, and the kept results are written straight
//    into the owner's curr list (in place over prev: curr[k] is written after
//    prev[>= k] was read, software/bwt.c:828) at the rank the kept ballot gives.
// An owner's step therefore takes one iteration when enough lanes are free,
// instead of one per entry, and the per-entry advance (seed_kernel's
// BWD_RES block) is gone; the lists live in LDS (NL entries per owner, OWN
// owners per wave: twice seed_kernel's entries per list in the same LDS),
// entries beyond NL in the owner's arena.
// ======================================================================
template <int OWN, int NL, bool PAIR, bool DPOS = false>
struct WpWave {
    uint4 e[NL][OWN];     // owners' lists: index k < NL at slot (lr - k) mod NL
    // step descriptors, by owner lane (DPOS: by the task position where the owner's entries start):
    // j, curr_n, prev_off, c | lr << 2 | last_x2 bits 32-33 << 8 | i << 10; min_intv, last_x2 low word,
    // prev_n (DPOS: the owner lane), kb
    uint4 d0[DPOS ? 64 : OWN];
    uint4 d1[DPOS ? 64 : OWN];
    uint4 q[OWN];         // query windows (LDS-DMA landing slots)
    uint4 noff[OWN];      // the next read's offs[rid], offs[rid + 1] (LDS-DMA landing slots)
    uint64_t res[DPOS ? 1 : 64];  // extend result sizes by lane (PAIR: of the lane's last entry; DPOS: in d1,
                                  // which the workers have read before the results are written)
    uint64_t res1[PAIR ? 64 : 1];  // PAIR: of the lane's first entry
    uint8_t tabS[64];     // owner whose segment starts at task position p (0xFF: none)
    uint8_t tabP[64];     // free-lane rank -> lane
};

// the OR of v over the 64 lanes (the same pattern; lane 63 holds it)
__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// inclusive prefix sum over the 64 lanes (the row_shr / row_bcast pattern of
// ksw_device.h's scan_max)
__device__ __forceinline__ uint32_t wave_scan_add(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

// set bits of m below this lane
__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ int hibit64(uint64_t m) { return 63 - __builtin_clzll(m); }

// LDS accesses of one wave execute in order; this keeps the compiler from
// moving them across the point where another lane's write must be seen
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

// PAIR: a worker lane takes two consecutive entries of a step (two extends
// in flight per lane: twice the requests per wave-iteration)
// KT: an extend whose result is a string of at most P.kt_k bases reads that
// string's bi-interval from the k-mer table (one 16-B probe; the table of
// k = 11 is 90 MB and stays in the 256 MB MALL) instead of two Occ buckets
// and the rank: a bi-interval is a function of the string alone, so the
// result is bwt_extend's.  Owners keep the codes of their forward string's
// first k bases and of the k bases from the backward position (variant 23's
// bookkeeping); the step descriptor carries the latter and the position.
// DPOS: the segment starts' mask by a DPP OR over the owners and each owner's
// descriptor stored at its start position, so a worker reads its owner's
// descriptor one LDS round after the scan (three rounds before the loads:
// start marks, owner, descriptor, entry -> descriptor, entry)
// OPT (A/B of the memory-issue order; default all): 1 claim the next read when the current one ends
// (else as soon as it starts), 2 arena entries in a wave-uniform branch with their own wait (else
// inline: the join's wait then runs every iteration and covers the owners' result-store acks), 4 the
// query-window / offsets DMA and the claim issued after the entry has landed (else before it: the
// compiler's wait for the entry covers them), 8 the claim as one hand-issued atomic per wave waited
// for by the iteration's vmcnt(0) (else the compiler's atomicAdd at the top, which waits for it)
template <int OWN, int NL, int PRIO, int WPE = 3, bool PAIR = false, bool KT = false, bool DPOS = false, int OPT = 15>
__global__ __launch_bounds__(256, WPE) void seed_wp_kernel(SeedParams P) {
    static_assert(!(DPOS && PAIR), "DPOS keeps the owner lane where PAIR keeps prev_n");
    constexpr uint32_t PR = PAIR ? 2u : 1u;  // entries per worker lane
    const int K = KT && P.kt ? P.kt_k : 0;
    static_assert(OWN >= 1 && OWN <= 64 && NL >= 2 && NL < 32, "owners per wave / list entries");
    __shared__ WpWave<OWN, NL, PAIR, DPOS> wlds[4];
    WpWave<OWN, NL, PAIR, DPOS>* L = &wlds[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)];
    uint64_t* const RES = DPOS ? reinterpret_cast<uint64_t*>(&L->d1[0]) : &L->res[0];
    const int me = (int)(threadIdx.x & 63);
    const uint64_t wave_g = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u);  // lane 0's global index
    const uint32_t cap = P.cap_list;
    // an owner's arena: [0, cap) the forward list beyond the ring, [cap, 2 cap) curr / prev beyond NL;
    // one per owner (OWN a wave, numbered from wown), not per lane: the batch's scratch is 64 / OWN
    // times smaller (smem_gpu.cpp seed_arenas)
#ifdef SMEM_WP_ARENA_PER_LANE  // (A/B: round 5's one arena per lane)
    const uint64_t wown = wave_g;
    PIntv* __restrict__ bp = reinterpret_cast<PIntv*>(P.scratch + (wown + (uint64_t)me) * 2ull * cap);
#else
    const uint64_t wown = (wave_g >> 6) * (uint64_t)OWN;
    PIntv* __restrict__ bp = reinterpret_cast<PIntv*>(P.scratch + (wown + (uint64_t)(me < OWN ? me : 0)) * 2ull * cap);
#endif

    int phase = me < OWN ? P_FETCH : P_EXIT;  // lanes >= OWN only execute extends
    int item = -1, len = 0;
    // next read: -2 nothing claimed, -5 claim in flight, -1 claimed, -3 its offsets to be fetched, -4 in
    // flight, >= 0 loaded.  Claimed when the current read ends (OPT 1; claimed when it starts, a read
    // held in reserve behind a busy owner lengthened the launch's tail).  The claim's atomic (OPT 8)
    // and the offsets' LDS-DMA are waited for by the iteration's vmcnt(0), never on their own: a wave
    // stalled a memory round trip per read for each before (the compiler's atomicAdd waits for the
    // result to broadcast it)
    int nitem = 0, nlen = -2;
    uint32_t clead = 0;  // the last claim's leader lane (wave-uniform); its atomic's return lands in no0
    int rid = 0, nrid = 0;
    uint32_t keep_n = 0;
    uint32_t o0 = 0, no0 = 0;
    uint32_t qb = ~0u, qwant = ~0u;
    uint4 qv = {0, 0, 0, 0};
    uint32_t raw_n = 0, calls_n = 0;
    int start = 0, ori_start = 0;
    int x = 0, min_intv = 1, middle = 0, i = 0, ret = 0, cur_c = 0;
    uint32_t j = 0;
    uint32_t kc = 0, kb = 0;  // KT: the forward string's codes, the K bases from backward position i
    uint64_t ik0 = 0, ik1 = 0, ik2 = 0;
    uint32_t ikend = 0;
    uint32_t fwd_n = 0, prev_off = 0, prev_n = 0, curr_n = 0;
    uint32_t lr = 0;           // forward: the ring position; backward: the slot of list index 0
    uint32_t fail0 = 0;        // entry 0 of the current step failed (its SMEM candidate)
    uint64_t last_x2 = 0;      // size of the last entry kept in curr (dedup across chunks of a step)
    uint32_t mem_n = 0, mem_last_start = 0, m_n = 0;
    uint32_t max_len = 0, max_x2 = 0, max_mid = 0;
    uint4 head = {0, 0, 0, 0};  // prev[0] of the current step
    uint64_t na = 0, nb = 0, ns = 0;
    if (P.tspan && me == 0) atomicMax(reinterpret_cast<unsigned long long*>(P.tspan), ~(unsigned long long)rtstamp());

#define QBLK(pos) ((o0 + (uint32_t)(pos)) & ~15u)
#define WSLOT(r_, k_) ((r_) >= (k_) ? (r_) - (k_) : (r_) + (uint32_t)NL - (k_))
// a SMEM of the current call: the raw log entry, the merge's keep count and
// the longest match (software/bwt.c:817-819, software/bwamem.c:266-270, 284-292)
#define WP_EMIT(e_)                                                                                          \
    {                                                                                                        \
        const uint4 me_ = (e_);                                                                              \
        if (raw_n >= P.cap_intv) {                                                                           \
            phase = P_OVF;                                                                                   \
        } else {                                                                                             \
            const uint32_t b_ = (uint32_t)(i + 1), en_ = p_end(me_);                                         \
            put_rec<false>(P.out_intv + (uint64_t)item * P.cap_intv + raw_n++,                               \
                           Intv{p_x0(me_), p_x1(me_), p_x2(me_), (uint64_t)en_ | ((uint64_t)b_ << 32)});    \
            keep_n += !middle || (en_ - b_ >= (max_len >> 1) && en_ > (uint32_t)ori_start);                 \
            ++mem_n;                                                                                         \
            mem_last_start = b_;                                                                             \
            if (!middle && en_ - b_ >= max_len) {                                                            \
                max_len = en_ - b_;                                                                          \
                max_x2 = p_x2(me_) > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)p_x2(me_);                      \
                max_mid = (en_ + b_) >> 1;                                                                   \
            }                                                                                                \
        }                                                                                                    \
    }

// the query window for owners that want one, the next read's offsets, and (OPT 8) one returning atomic
// per wave for every owner that wants its next read, issued by hand: not waited for here, read at the
// top of the next iteration after the iteration's vmcnt(0); early clobber, so that the return
// register does not overlap the address.  OPT 4 issues this after the entry has landed and before the
// buckets (all land in one round trip); else before the entry, whose wait then covers them.
#define WP_ISSUE()                                                                                                            \
    {                                                                                                                         \
        if (ld_q) __builtin_amdgcn_global_load_lds(P.codes + qwant, LDS_PTR(&L->q[0]), 16, 0, 0);                             \
        if (nlen == -3) {                                                                                                     \
            __builtin_amdgcn_global_load_lds(P.offs + nrid, LDS_PTR(&L->noff[0]), 16, 0, 0);                                  \
            nlen = -4;                                                                                                        \
        }                                                                                                                     \
        const bool wc_ = nlen == -2 && ((OPT & 1) ? phase == P_FETCH : phase != P_EXIT);                                      \
        const uint64_t want_claim = (OPT & 8) ? __ballot(wc_) : 0ull;                                                         \
        if (want_claim) {                                                                                                     \
            clead = (uint32_t)(__builtin_ffsll((long long)want_claim) - 1);                                                   \
            if (wc_) {                                                                                                        \
                nitem = (int)__popcll(want_claim & ((1ull << me) - 1));                                                       \
                if ((uint32_t)me == clead) {                                                                                  \
                    const int cnt = (int)__popcll(want_claim);                                                                \
                    asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=&v"(no0) : "v"(P.head), "v"(cnt) : "memory");    \
                }                                                                                                             \
                nlen = -5;                                                                                                    \
            }                                                                                                                 \
        }                                                                                                                     \
    }

    for (;;) {
        if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(2);
        if (phase != P_EXIT) {
            if (!(OPT & 8) && nlen == -2 && phase == P_FETCH) {
                nitem = atomicAdd(P.head, 1);  // (the compiler waits for the result here)
                nlen = -1;
            } else {
                if ((OPT & 8) && nlen == -5) {  // the claim returned: the leader's base + this lane's rank
                    nitem += (int)__builtin_amdgcn_readlane(no0, clead);
                    nlen = -1;
                }
                if (nlen == -1) {
                    if (nitem >= P.n_items) {
                        nlen = 0;  // nothing left: the FETCH block exits
                    } else if (P.read_ids) {  // overflow pass: through read_ids (a small launch)
                        next_offsets(P, nitem, no0, nlen, nrid);
                    } else {
                        nrid = nitem;
                        nlen = -3;  // offsets fetched in the uniform section
                    }
                } else if (nlen == -4) {  // landed last iteration
                    const uint4 v = L->noff[me];
                    no0 = v.x;  // batches hold < 2^32 bases: the low words
                    nlen = (int)(v.z - v.x);
                }
            }
        }
        // ---- owners: advance the state machine one pass (seed_kernel's
        // blocks, without the per-entry backward block) ----
        bool out = false;
        if (phase != P_EXIT) {
            if (phase == P_SMEM_END) {
                if (!middle) {  // software/bwamem.c:261-272
                    start = ret;
                    m_n = mem_n;
                    const int split_len = P.split_len_init < len ? P.split_len_init : len;
                    if (m_n > 0 && split_len > 0 && (int)max_len >= split_len &&
                        (uint64_t)max_x2 <= (uint64_t)(int64_t)P.split_width) {
                        x = (int)max_mid;  // re-seed from the middle (software/bwamem.c:272-278)
                        min_intv = (int)(max_x2 + 1);
                        middle = 1;
                        phase = P_SMEM_BEGIN;
                    }
                }
                if (phase == P_SMEM_END) {
                    if (calls_n >= P.cap_calls) {
                        phase = P_OVF;
                    } else {
                        put_rec<false>(P.out_call + (uint64_t)item * P.cap_calls + calls_n++,
                                       CallRec{m_n, middle ? mem_n : 0u, (uint32_t)ori_start, max_len});
                        phase = P_NEXT2;
                    }
                }
            }
            if (phase == P_OVF) {
                P.n_intv[item] = SMEM_OVERFLOW;
                P.n_calls[item] = 0;
                const int slot = atomicAdd(P.ovf_count, 1);
                P.ovf_items[slot] = item;
                phase = P_FETCH;
            }
            if (phase == P_FETCH) {
                if (nlen < 0) {
                    out = true;
                } else if (nitem >= P.n_items) {
                    phase = P_EXIT;
                } else {
                    item = nitem;
                    rid = nrid;
                    keep_n = 0;
                    o0 = no0;
                    len = nlen;
                    nlen = -2;
                    raw_n = 0;
                    calls_n = 0;
                    start = 0;
                    if (len < P.min_seed_len) {  // mem_chain's guard (software/bwamem.c:600)
                        P.n_intv[item] = 0;
                        P.n_calls[item] = 0;
                        P.s_intv[rid] = 0;
                        P.s_calls[rid] = 0;
                        out = true;
                    } else {
                        phase = P_NEXT2;
                    }
                }
            }
            if (phase == P_NEXT2) {  // software/bwamem.c:247-261
                bool wait_q = false;
                if (start < len && start >= 0) {
                    for (;;) {
                        if (start >= len) break;
                        if (QBLK(start) != qb) { wait_q = true; break; }
                        if (qsel(o0, start, qv) <= 3) break;
                        ++start;
                    }
                }
                if (wait_q) {
                    qwant = QBLK(start);
                    out = true;
                } else if (start >= len || start < 0) {
                    P.n_intv[item] = raw_n;
                    P.n_calls[item] = calls_n;
                    P.s_intv[rid] = keep_n;
                    P.s_calls[rid] = calls_n;
                    phase = P_FETCH;
                } else {
                    ori_start = start;
                    x = ori_start;
                    min_intv = P.start_width;
                    middle = 0;
                    max_len = 0;
                    phase = P_SMEM_BEGIN;
                }
            }
            if (phase == P_SMEM_BEGIN) {  // software/bwt.c:782-789
                if (QBLK(x) != qb) {
                    qwant = QBLK(x);
                    out = true;
                } else {
                    mem_n = 0;
                    const int qx = qsel(o0, x, qv);
                    if (qx > 3) {
                        ret = x + 1;
                        phase = P_SMEM_END;
                    } else {
                        if (min_intv < 1) min_intv = 1;
                        const uint64_t lq = sel4(qx, P.L2[0], P.L2[1], P.L2[2], P.L2[3]);
                        const uint64_t lq1 = sel4(qx, P.L2[1], P.L2[2], P.L2[3], P.L2[4]);
                        ik0 = lq + 1;
                        ik2 = lq1 - lq;
                        ik1 = sel4(qx, P.L2[3], P.L2[2], P.L2[1], P.L2[0]) + 1;
                        ikend = (uint32_t)(x + 1);
                        if constexpr (KT) kc = (uint32_t)qx;
                        fwd_n = 0;
                        lr = 0;
                        i = x + 1;
                        phase = P_FWD;
                    }
                }
            }
            if (phase == P_BWD_DONE) {  // every entry of step i extended (software/bwt.c:815-828)
                if (fail0 && (mem_n == 0 || (uint32_t)(i + 1) < mem_last_start)) WP_EMIT(head);
                if (phase == P_BWD_DONE) {
                    if (curr_n == 0) {  // software/bwt.c:827
                        phase = P_SMEM_END;
                    } else {            // :828 swap, next position
                        prev_n = curr_n;
                        prev_off = cap;
                        head = L->e[lr][me];  // curr[0]: index 0 sits in slot lr
                        --i;
                        phase = P_BWD_STEP;
                    }
                }
            }
            if (phase == P_FWD_RES) {  // software/bwt.c:795-799; na = x[1], nb = x[0]
                bool stop = false;
                if (ns != ik2) {
                    const uint4 fe = pack_p(ik0, ik1, ik2, ikend);
                    if (fwd_n >= (uint32_t)NL) *reinterpret_cast<uint4*>(bp + cap - 1 - (fwd_n - NL)) = L->e[lr][me];
                    L->e[lr][me] = fe;
                    lr = lr + 1 == (uint32_t)NL ? 0u : lr + 1;
                    ++fwd_n;
                    stop = ns < (uint64_t)min_intv;
                }
                if (stop) {
                    phase = P_FWD_DONE;
                } else {
                    ik0 = nb; ik1 = na; ik2 = ns;
                    ikend = (uint32_t)(i + 1);
                    if constexpr (KT) {
                        if (i + 1 - x <= K) kc = kc << 2 | (uint32_t)(3 - cur_c);  // saturates at the first K bases
                    }
                    ++i;
                    phase = P_FWD;
                }
            }
            if (phase == P_FWD) {  // software/bwt.c:791-803
                bool push = true;
                if (i < len) {
                    if (QBLK(i) != qb) {
                        qwant = QBLK(i);
                        out = true;
                        push = false;
                    } else {
                        const int qi = qsel(o0, i, qv);
                        if (qi < 4) {
                            cur_c = 3 - qi;
                            if (i + 1 < len) qwant = QBLK(i + 1);
                            phase = P_FWD_RES;  // -> extend (forward), on this lane
                            out = true;
                            push = false;
                        }
                    }
                }
                if (push) {  // ambiguous base, or end of query: push ik and stop
                    const uint4 fe = pack_p(ik0, ik1, ik2, ikend);
                    if (fwd_n >= (uint32_t)NL) *reinterpret_cast<uint4*>(bp + cap - 1 - (fwd_n - NL)) = L->e[lr][me];
                    L->e[lr][me] = fe;
                    lr = lr + 1 == (uint32_t)NL ? 0u : lr + 1;
                    ++fwd_n;
                    phase = P_FWD_DONE;
                }
            }
            if (phase == P_FWD_DONE) {  // software/bwt.c:805-808 (the ring read backwards is the reversal)
                head = pack_p(ik0, ik1, ik2, ikend);  // the last push: prev[0]
                ret = (int)ikend;
                if constexpr (KT) {  // the K bases from x (those past the forward string are never read)
                    const uint32_t lf = ikend - (uint32_t)x;
                    kb = lf >= (uint32_t)K ? kc : kc << (2 * ((uint32_t)K - lf));
                }
                prev_off = cap - fwd_n;
                prev_n = fwd_n;
                lr = lr == 0 ? (uint32_t)NL - 1 : lr - 1;  // slot of the last push
                i = x - 1;
                phase = P_BWD_STEP;
            }
            if (phase == P_BWD_STEP) {  // software/bwt.c:810-812
                if (i >= 0 && QBLK(i) != qb) {
                    qwant = QBLK(i);
                    out = true;
                } else {
                    cur_c = i < 0 ? -1 : qsel(o0, i, qv);
                    if (cur_c > 3) cur_c = -1;
                    if (cur_c >= 0) {
                        j = 0;
                        curr_n = 0;
                        fail0 = 0;
                        if constexpr (KT) kb = (uint32_t)cur_c << (2 * (K - 1)) | kb >> 2;
                        if (i > 0) qwant = QBLK(i - 1);  // the next step's base
                        phase = P_BWD_WAIT;               // -> the wave extends the step's entries
                    } else {
                        // nothing extends: prev[0] is the only candidate (software/bwt.c:816-819)
                        phase = P_SMEM_END;
                        if (mem_n == 0 || (uint32_t)(i + 1) < mem_last_start) WP_EMIT(head);
                    }
                }
            }
        }
        // ---- uniform section ----
        if (!__any(phase != P_EXIT)) break;
        const bool fwdreq = out && phase == P_FWD_RES;
        const uint32_t rem = phase == P_BWD_WAIT ? prev_n - j : 0u;
        const uint32_t slots = (rem + PR - 1) / PR;  // worker lanes the step still needs
        if (!DPOS && rem) {  // what a worker needs of this owner's step
            L->d0[me] = make_uint4(j, curr_n, prev_off,
                                   (uint32_t)cur_c | lr << 2 | (uint32_t)(last_x2 >> 32) << 8 | (uint32_t)i << 10);
            L->d1[me] = make_uint4((uint32_t)min_intv, (uint32_t)last_x2, prev_n, kb);
        }
        // the owners' remaining entries laid out in lane order over the free lanes
        const uint32_t incl = wave_scan_add(slots);
        const uint32_t excl = incl - slots;
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        const uint64_t fmask = ~(uint64_t)__ballot(fwdreq);
        const uint32_t nfree = (uint32_t)__popcll(fmask);
        const uint32_t ntask = total < nfree ? total : nfree;
        const uint32_t take = (slots && excl < nfree) ? min(slots, nfree - excl) : 0u;
        const bool freel = (fmask >> me) & 1;
        const uint32_t rank = mbcnt64(fmask);
        uint64_t marks;
        if constexpr (DPOS) {
            if (take) {  // the descriptor where the owner's entries start
                L->d0[excl] = make_uint4(j, curr_n, prev_off,
                                         (uint32_t)cur_c | lr << 2 | (uint32_t)(last_x2 >> 32) << 8 | (uint32_t)i << 10);
                L->d1[excl] = make_uint4((uint32_t)min_intv, (uint32_t)last_x2, (uint32_t)me, kb);
            }
            if (freel) L->tabP[rank] = (uint8_t)me;
            const uint32_t mlo = wave_or(take && excl < 32 ? 1u << excl : 0u);
            const uint32_t mhi = wave_or(take && excl >= 32 ? 1u << (excl - 32) : 0u);
            marks = (uint64_t)mhi << 32 | mlo;
            wave_lds_fence();
        } else {
            L->tabS[me] = 0xFFu;
            wave_lds_fence();
            if (take) L->tabS[excl] = (uint8_t)me;
            if (freel) L->tabP[rank] = (uint8_t)me;
            wave_lds_fence();
            marks = __ballot(L->tabS[me] != 0xFFu);
        }
        const bool worker = freel && rank < ntask;
        uint32_t s = 0, o = 0, jj = 0, lro = 0;
        bool has2 = false;
        uint4 w0 = {0, 0, 0, 0}, w1 = {0, 0, 0, 0}, ent = {0, 0, 0, 0}, ent2 = {0, 0, 0, 0};
        bool far = false, far2 = false;  // the entry (PAIR: the second) is in the owner's arena
        if (worker) {
            s = (uint32_t)hibit64(marks & ((2ull << rank) - 1ull));  // the segment holding task `rank`
            if constexpr (DPOS) {
                w0 = L->d0[s];
                w1 = L->d1[s];
                o = w1.z;
            } else {
                o = L->tabS[s];
                w0 = L->d0[o];
                w1 = L->d1[o];
            }
            jj = w0.x + PR * (rank - s);
            lro = (w0.w >> 2) & 31u;
            if (jj < (uint32_t)NL) {
                ent = L->e[WSLOT(lro, jj)][o];
            } else if constexpr (OPT & 2) {
                far = true;
            } else {
                const PIntv* obp = reinterpret_cast<const PIntv*>(P.scratch + (wown + o) * 2ull * cap);
                const uint32_t at = w0.z + jj;
                ent = *reinterpret_cast<const uint4*>(obp + (at < 2 * cap ? at : 0u));
            }
            if constexpr (PAIR) {
                has2 = jj + 1 < w1.z;
                if (has2) {
                    if (jj + 1 < (uint32_t)NL) {
                        ent2 = L->e[WSLOT(lro, jj + 1)][o];
                    } else if constexpr (OPT & 2) {
                        far2 = true;
                    } else {
                        const PIntv* obp = reinterpret_cast<const PIntv*>(P.scratch + (wown + o) * 2ull * cap);
                        const uint32_t at = w0.z + jj + 1;
                        ent2 = *reinterpret_cast<const uint4*>(obp + (at < 2 * cap ? at : 0u));
                    }
                }
            }
        }
        const bool ld_q = qwant != qb && qwant != ~0u;
        if constexpr (!(OPT & 4)) WP_ISSUE();
        // entries beyond the LDS list: the owner's arena (the bound only guards a broken list), in a
        // wave-uniform branch that waits for them itself -- a wait at the join would run every
        // iteration, and one vmcnt counts the owners' result stores too (their acks, every iteration)
        if (OPT & 2 && __builtin_expect(__any(far || far2), 0)) {
            const PIntv* obp = reinterpret_cast<const PIntv*>(P.scratch + (wown + o) * 2ull * cap);
            if (far) {
                const uint32_t at = w0.z + jj;
                ent = *reinterpret_cast<const uint4*>(obp + (at < 2 * cap ? at : 0u));
            }
            if (PAIR && far2) {
                const uint32_t at = w0.z + jj + 1;
                ent2 = *reinterpret_cast<const uint4*>(obp + (at < 2 * cap ? at : 0u));
            }
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        }
        // the extend: forward owners their own ik (a = x[1]), workers an entry backward (a = x[0])
        const bool task = worker || fwdreq;
        const uint64_t ra = fwdreq ? ik1 : p_x0(ent), rb = fwdreq ? ik0 : p_x1(ent), rs = fwdreq ? ik2 : p_x2(ent);
        const int rc = fwdreq ? cur_c : (int)(w0.w & 3u);
        const uint64_t k = ra - 1, l = k + rs;
        uint64_t kk = k - (k >= P.primary), ll = l - (l >= P.primary);
        // rows past the BWT only come from a broken entry: keep the loads inside the index
        // (the results then differ from the oracle instead of faulting the device)
        if (kk >= P.L2[4]) kk = 0;
        if (ll >= P.L2[4]) ll = 0;
        const uint32_t bk = (uint32_t)(kk >> 6), bl = (uint32_t)(ll >> 6);
        if constexpr (OPT & 4) {
            // the bucket indices exist here (the entry has landed) before anything below is issued
            asm volatile("" ::"v"(bk), "v"(bl) : "memory");
            WP_ISSUE();
        }
        uint4 k0 = {0, 0, 0, 0}, k1 = {0, 0, 0, 0}, l0 = {0, 0, 0, 0}, l1 = {0, 0, 0, 0};
        // KT: a result of at most K bases from the table (forward: q[x, i]; backward: q[i, end))
        bool ktp = false;
        if constexpr (KT) {
            if (task && K > 0) {
                const int lq = fwdreq ? i + 1 - x : (int)p_end(ent) - (int)(w0.w >> 10);
                if (lq <= K) {
                    const uint32_t code = fwdreq ? kc << 2 | (uint32_t)(3 - cur_c) : w1.w >> (2 * (K - lq));
                    const uint64_t base = ((1ull << (2 * lq)) - 4) / 3;
                    k0 = P.kt[base + code];
                    ktp = true;
                }
            }
        }
        if (task && !ktp) {
            const uint32_t *a0, *a1;
            block_chunks<false>(P.occ64, bk, a0, a1);
            k0 = *reinterpret_cast<const uint4*>(a0);
            k1 = *reinterpret_cast<const uint4*>(a1);
            if (bl != bk) {
                block_chunks<false>(P.occ64, bl, a0, a1);
                l0 = *reinterpret_cast<const uint4*>(a0);
                l1 = *reinterpret_cast<const uint4*>(a1);
            }
        }
        // PAIR: the lane's second entry (same base), its buckets in flight beside the first's
        uint64_t ra2 = 0, rb2 = 0, rs2 = 0, kk2 = 0, ll2 = 0;
        uint32_t bk2 = 0, bl2 = 0;
        uint4 m0 = {0, 0, 0, 0}, m1 = {0, 0, 0, 0}, n0 = {0, 0, 0, 0}, n1 = {0, 0, 0, 0};
        if constexpr (PAIR) {
            if (has2) {
                ra2 = p_x0(ent2), rb2 = p_x1(ent2), rs2 = p_x2(ent2);
                const uint64_t k2 = ra2 - 1, l2 = k2 + rs2;
                kk2 = k2 - (k2 >= P.primary), ll2 = l2 - (l2 >= P.primary);
                if (kk2 >= P.L2[4]) kk2 = 0;
                if (ll2 >= P.L2[4]) ll2 = 0;
                bk2 = (uint32_t)(kk2 >> 6), bl2 = (uint32_t)(ll2 >> 6);
                const uint32_t *a0, *a1;
                block_chunks<false>(P.occ64, bk2, a0, a1);
                m0 = *reinterpret_cast<const uint4*>(a0);
                m1 = *reinterpret_cast<const uint4*>(a1);
                if (bl2 != bk2) {
                    block_chunks<false>(P.occ64, bl2, a0, a1);
                    n0 = *reinterpret_cast<const uint4*>(a0);
                    n1 = *reinterpret_cast<const uint4*>(a1);
                }
            }
        }
        if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(0);
        // vmcnt(0) as the builtin, not inline asm: the compiler's wait insertion sees it and knows the
        // LDS-DMA above has landed (after an opaque asm wait it re-waited vmcnt(0) before the next
        // iteration's LDS reads, i.e. for the acks of the result stores)
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
        if (ld_q) {
            qv = L->q[me];
            qb = qwant;
        }
        if (ktp) {  // forward: na is the x[1] side, backward: the x[0] side
            na = fwdreq ? p_x1(k0) : p_x0(k0);
            nb = fwdreq ? p_x0(k0) : p_x1(k0);
            ns = p_x2(k0);
        } else if (task) {
            const Bucket32 wk{k0, k1};
            const Bucket32 wl = bl != bk ? Bucket32{l0, l1} : wk;
            extend_counts64<false>(P, ra, rb, rs, rc, kk, ll, wk, wl, na, nb, ns);
        }
        uint64_t na2 = 0, nb2 = 0, ns2 = 0;
        if constexpr (PAIR) {
            if (has2) {
                const Bucket32 wk{m0, m1};
                const Bucket32 wl = bl2 != bk2 ? Bucket32{n0, n1} : wk;
                extend_counts64<false>(P, ra2, rb2, rs2, rc, kk2, ll2, wk, wl, na2, nb2, ns2);
            }
        }
        // ---- the backward results: survive, dedup, rank, write into curr ----
        // entries of a segment in order: lane by lane, (PAIR) first then second entry
        const bool surv = worker && ns >= (uint64_t)w1.x;
        const bool surv2 = PAIR && has2 && ns2 >= (uint64_t)w1.x;
        const uint64_t smask = __ballot(surv);
        const uint64_t smask2 = PAIR ? (uint64_t)__ballot(surv2) : 0ull;
        RES[me] = PAIR && has2 ? ns2 : ns;  // the lane's last entry
        if constexpr (PAIR) L->res1[me] = ns;
        wave_lds_fence();
        bool keep = false;
        if (surv) {
            if (rank == s) {  // first entry of this chunk: against the last entry kept before it
                const uint64_t lx = (uint64_t)((w0.w >> 8) & 3u) << 32 | w1.y;
                keep = w0.y == 0 || ns != lx;
            } else {          // against the previous entry: the previous free lane's last one
                const int pp = hibit64(fmask & ((1ull << me) - 1ull));
                keep = !(((PAIR ? smask2 : smask) >> pp) & 1) || ns != RES[pp];
            }
        }
        const bool keep2 = surv2 && (!surv || ns2 != ns);
        const uint64_t kmask = __ballot(keep);
        const uint64_t kmask2 = PAIR ? (uint64_t)__ballot(keep2) : 0ull;
        if (keep || keep2) {
            const uint32_t pf = L->tabP[s];
            const uint64_t before = (1ull << me) - 1ull & ~((1ull << pf) - 1ull);
            const uint32_t kr = (uint32_t)(__popcll(kmask & before) + __popcll(kmask2 & before));
            PIntv* obp = reinterpret_cast<PIntv*>(P.scratch + (wown + o) * 2ull * cap);
            if (keep) {
                const uint32_t idx = w0.y + kr;
                const uint4 e = pack_p(na, nb, ns, p_end(ent));
                if (idx < (uint32_t)NL) L->e[WSLOT(lro, idx)][o] = e;
                else if (idx < cap) *reinterpret_cast<uint4*>(obp + cap + idx) = e;
            }
            if (PAIR && keep2) {
                const uint32_t idx = w0.y + kr + (keep ? 1u : 0u);
                const uint4 e = pack_p(na2, nb2, ns2, p_end(ent2));
                if (idx < (uint32_t)NL) L->e[WSLOT(lro, idx)][o] = e;
                else if (idx < cap) *reinterpret_cast<uint4*>(obp + cap + idx) = e;
            }
        }
        // ---- owners whose entries ran: the chunk's outcome ----
        if (take) {
            const uint32_t pf = L->tabP[excl], pl = L->tabP[excl + take - 1];
            const uint64_t seg = ((2ull << pl) - 1ull) & ~((1ull << pf) - 1ull);
            const uint64_t km = kmask & seg, km2 = kmask2 & seg;
            if (j == 0) fail0 = !((smask >> pf) & 1);
            if (km | km2) {  // the last entry kept: the highest lane's second entry if it kept one
                const int hb = hibit64(km | km2);
                last_x2 = ((km2 >> hb) & 1) ? RES[hb] : (PAIR ? L->res1[hb] : RES[hb]);
            }
            curr_n += (uint32_t)(__popcll(km) + __popcll(km2));
            j += min(rem, PR * take);
            if (j == prev_n) phase = P_BWD_DONE;
        }
        wave_lds_fence();  // this iteration's LDS reads before the next one's writes
    }
#undef WP_EMIT
#undef WSLOT
#undef QBLK
    if (P.tspan && me == 0) atomicMax(reinterpret_cast<unsigned long long*>(P.tspan) + 1, (unsigned long long)rtstamp());
}

// Raw logs -> the lists smem_next2 returns: reverse each bwt_smem1 output
// (software/bwt.c:830) and merge matches with sub-matches keyed by
// (start, len - end), keeping a sub-match only if it is at least half the
// longest match and ends after the call's start (software/bwamem.c:280-301).
// Four threads per read, one per 8-B word of bwtintv_t: all four walk the
// same merge (on the info words) and each moves its own word, so a wave's
// loads and stores touch 16 intervals' lines instead of 64.  The per-read
// sizes come from the seeding kernel.
__global__ __launch_bounds__(256) void finalize_kernel(FinalizeParams F) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int r = (int)(t >> 2), w = (int)(t & 3);
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
    const uint64_t* rw = reinterpret_cast<const uint64_t*>(raw);
    uint64_t* ow = reinterpret_cast<uint64_t*>(F.flat_intv + F.intv_off[r]);
    const uint64_t cout = F.call_off[r];
    uint32_t pos = 0, out = 0;
    for (uint32_t c = 0; c < nc; ++c) {
        const CallRec cr = rec[c];
        // M[m_n-1-a] is the a-th match in final order; likewise S for sub-matches
        const uint64_t* M = rw + (uint64_t)pos * 4;
        const uint64_t* S = rw + (uint64_t)(pos + cr.m_n) * 4;
        const uint64_t half = (uint64_t)(cr.max_len >> 1);
        uint32_t a = 0, b = 0, n = 0;
        while (a < cr.m_n || b < cr.s_n) {
            bool take_m;
            uint64_t si = 0;
            if (b >= cr.s_n) {
                take_m = true;
            } else {
                si = S[(uint64_t)(cr.s_n - 1 - b) * 4 + 3];
                if (a >= cr.m_n) {
                    take_m = false;
                } else {
                    const uint64_t mi = M[(uint64_t)(cr.m_n - 1 - a) * 4 + 3];
                    const uint64_t xi = (mi >> 32 << 32) | (uint64_t)(uint32_t)(len - (uint32_t)mi);
                    const uint64_t xj = (si >> 32 << 32) | (uint64_t)(uint32_t)(len - (uint32_t)si);
                    take_m = (int64_t)xi < (int64_t)xj;
                }
            }
            if (take_m) {
                ow[(uint64_t)(out + n) * 4 + w] = M[(uint64_t)(cr.m_n - 1 - a) * 4 + w];
                ++n;
                ++a;
            } else {
                if ((uint64_t)(uint32_t)si - (si >> 32) >= half && (uint32_t)si > cr.ori_start) {
                    ow[(uint64_t)(out + n) * 4 + w] = S[(uint64_t)(cr.s_n - 1 - b) * 4 + w];
                    ++n;
                }
                ++b;
            }
        }
        if (w == 0) F.flat_calls[cout + c] = n;
        out += n;
        pos += cr.m_n + cr.s_n;
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
// The product build instantiates the default kernel (seed_wp_kernel variant 49;
// 0 names it too) and its k-mer table twin (54).  Every other seeding kernel
// measured in rounds 1-5 (seed_kernel variants 2-31; the seed_wp_kernel shapes
// and OPT-bit twins 40-62 other than 49 / 54) is compiled only
// with SMEM_AB_VARIANTS (make AB=1): the library ships no kernel whose numbers
// are already recorded.
extern "C" int smem_seed_variant_built(int variant) {
#ifdef SMEM_AB_VARIANTS
    return variant == 0 || (variant >= 2 && variant <= 31) || (variant >= 40 && variant <= 62);
#else
    return variant == 0 || variant == 49 || variant == 54;
#endif
}

extern "C" hipError_t smem_launch_seed(const smem::SeedParams* P, int grid, int block, int variant, hipStream_t st) {
    switch (variant) {
#ifdef SMEM_AB_VARIANTS
        // 2 (20 and 26 name it too): round 4's default seed_kernel -- Occ64, the two bucket slots per
        // lane in registers, 11 list entries per lane in LDS (the forward list as a ring of its last 11
        // pushes), wave priority raised from the top of an iteration until its loads are issued (PRIO 1)
        case 2: case 20: case 26: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_OCC64, false, 3, 11, true, false, false, true, false, true, false, false, 1>), dim3(grid), dim3(block), 0, st, *P); break;
        // 9: variant 2 (wave priority included) with cycle stamps
        case 9: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_OCC64, true, 3, 11, true, false, false, true, false, true, false, false, 1>), dim3(grid), dim3(block), 0, st, *P); break;
        // 23: the default with the k-mer table (P->kt)
        case 23: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_OCC64, false, 3, 11, true, false, false, true, false, true, true>), dim3(grid), dim3(block), 0, st, *P); break;
        // 24: the default with the next read claimed and loaded in the uniform section (PFCH); 25: its stamped twin
        case 24: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_OCC64, false, 3, 11, true, false, false, true, false, true, false, true>), dim3(grid), dim3(block), 0, st, *P); break;
        case 25: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_OCC64, true, 3, 11, true, false, false, true, false, true, false, true>), dim3(grid), dim3(block), 0, st, *P); break;
        // 27: wave priority raised in the extend arithmetic instead (PRIO 2: no change measured);
        // 28: the default without wave priority (round-2 default; 2 % slower, profiles/r03/ab/prio)
        case 28: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_OCC64, false, 3, 11, true, false, false, true, false, true>), dim3(grid), dim3(block), 0, st, *P); break;
        case 27: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_OCC64, false, 3, 11, true, false, false, true, false, true, false, false, 2>), dim3(grid), dim3(block), 0, st, *P); break;
        // 29-31: the default with non-temporal bucket loads (29), raw output stores (30), both (31)
        case 29: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_OCC64, false, 3, 11, true, false, false, true, false, true, false, false, 1, 1>), dim3(grid), dim3(block), 0, st, *P); break;
        case 30: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_OCC64, false, 3, 11, true, false, false, true, false, true, false, false, 1, 2>), dim3(grid), dim3(block), 0, st, *P); break;
        case 31: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_OCC64, false, 3, 11, true, false, false, true, false, true, false, false, 1, 3>), dim3(grid), dim3(block), 0, st, *P); break;
        // 40-43: the backward phase wave-parallel over list entries (seed_wp_kernel<owners per wave,
        // LDS list entries per owner, wave priority>)
        case 40: hipLaunchKernelGGL((smem::seed_wp_kernel<32, 20, 1>), dim3(grid), dim3(block), 0, st, *P); break;
        case 41: hipLaunchKernelGGL((smem::seed_wp_kernel<32, 16, 1>), dim3(grid), dim3(block), 0, st, *P); break;
        case 42: hipLaunchKernelGGL((smem::seed_wp_kernel<24, 24, 1>), dim3(grid), dim3(block), 0, st, *P); break;
        case 43: hipLaunchKernelGGL((smem::seed_wp_kernel<32, 20, 0>), dim3(grid), dim3(block), 0, st, *P); break;
        // 44-46: 4 blocks (16 waves) per CU with shorter lists: <24 owners, 16 entries>, <32, 12>, <28, 14>
        case 44: hipLaunchKernelGGL((smem::seed_wp_kernel<24, 16, 1, 4>), dim3(grid), dim3(block), 0, st, *P); break;
        case 45: hipLaunchKernelGGL((smem::seed_wp_kernel<32, 12, 1, 4>), dim3(grid), dim3(block), 0, st, *P); break;
        case 46: hipLaunchKernelGGL((smem::seed_wp_kernel<28, 14, 1, 4>), dim3(grid), dim3(block), 0, st, *P); break;
        // 47-48: two entries per worker lane (PAIR): <32, 20>, <24, 24> (3 blocks per CU)
        case 47: hipLaunchKernelGGL((smem::seed_wp_kernel<32, 20, 1, 3, true>), dim3(grid), dim3(block), 0, st, *P); break;
        case 48: hipLaunchKernelGGL((smem::seed_wp_kernel<24, 24, 1, 3, true>), dim3(grid), dim3(block), 0, st, *P); break;
        // 49-51: 4 blocks per CU: <24, 18>, <20, 22>, 44 without wave priority
        case 50: hipLaunchKernelGGL((smem::seed_wp_kernel<20, 22, 1, 4>), dim3(grid), dim3(block), 0, st, *P); break;
        case 51: hipLaunchKernelGGL((smem::seed_wp_kernel<24, 16, 0, 4>), dim3(grid), dim3(block), 0, st, *P); break;
        // 52-53: 4 blocks per CU: <24, 20>, <28, 16>
        case 52: hipLaunchKernelGGL((smem::seed_wp_kernel<24, 20, 1, 4>), dim3(grid), dim3(block), 0, st, *P); break;
        case 53: hipLaunchKernelGGL((smem::seed_wp_kernel<28, 16, 1, 4>), dim3(grid), dim3(block), 0, st, *P); break;
        // 55: with the k-mer table (KT; smem_gpu_set_kmer_table, no table: plain), 40's shape
        case 55: hipLaunchKernelGGL((smem::seed_wp_kernel<32, 20, 1, 3, false, true>), dim3(grid), dim3(block), 0, st, *P); break;
        // 56-57: descriptors by start position (DPOS): 49's shape, and with the k-mer table
        case 56: hipLaunchKernelGGL((smem::seed_wp_kernel<24, 18, 1, 4, false, false, true>), dim3(grid), dim3(block), 0, st, *P); break;
        case 57: hipLaunchKernelGGL((smem::seed_wp_kernel<24, 18, 1, 4, false, true, true>), dim3(grid), dim3(block), 0, st, *P); break;
        // 58-62: 49 with the memory-issue order taken apart (OPT bits, seed_wp_kernel): 58 none, 59 no
        // uniform arena branch, 60 the DMA / claim before the entry, 61 the claim when a read starts,
        // 62 the compiler's atomicAdd
        case 58: hipLaunchKernelGGL((smem::seed_wp_kernel<24, 18, 1, 4, false, false, false, 0>), dim3(grid), dim3(block), 0, st, *P); break;
        case 59: hipLaunchKernelGGL((smem::seed_wp_kernel<24, 18, 1, 4, false, false, false, 13>), dim3(grid), dim3(block), 0, st, *P); break;
        case 60: hipLaunchKernelGGL((smem::seed_wp_kernel<24, 18, 1, 4, false, false, false, 11>), dim3(grid), dim3(block), 0, st, *P); break;
        case 61: hipLaunchKernelGGL((smem::seed_wp_kernel<24, 18, 1, 4, false, false, false, 14>), dim3(grid), dim3(block), 0, st, *P); break;
        case 62: hipLaunchKernelGGL((smem::seed_wp_kernel<24, 18, 1, 4, false, false, false, 7>), dim3(grid), dim3(block), 0, st, *P); break;
        // 3: reference-layout buckets, cooperative fetch, lists in global memory;
        // 4: reference layout, per-lane fetch; 5: Occ64 with 12 list entries in
        // LDS at 2 blocks per CU; 6: Occ64, lists in global memory; 7: the
        // default with the bucket fetch of BWD_RES lanes issued inside the
        // advance (no gain measured: the fetch is throughput-bound); 8: 4 blocks per CU
        // with 4 list entries in LDS
        case 3: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_COOP, false, 3, 0>), dim3(grid), dim3(block), 0, st, *P); break;
        case 4: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_LANE, false, 3, 0>), dim3(grid), dim3(block), 0, st, *P); break;
        case 5: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_OCC64, false, 2, 12>), dim3(grid), dim3(block), 0, st, *P); break;
        case 6: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_OCC64, false, 3, 0>), dim3(grid), dim3(block), 0, st, *P); break;
        case 7: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_OCC64, false, 3, smem::LIST_LDS, true, true>), dim3(grid), dim3(block), 0, st, *P); break;
        case 8: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_OCC64, false, 4, 4>), dim3(grid), dim3(block), 0, st, *P); break;
        case 10: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_OCC64, false, 3, smem::LIST_LDS, true, false, true>), dim3(grid), dim3(block), 0, st, *P); break;
        // 11: the first round-2 layout (LDS bucket slots, 7 list entries, forward ring)
        case 11: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_OCC64, false, 3, smem::LIST_LDS, true, false, false, true>), dim3(grid), dim3(block), 0, st, *P); break;
        case 12: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_OCC64, false, 2, 12, true, false, false, true>), dim3(grid), dim3(block), 0, st, *P); break;
        case 13: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_OCC64, false, 3, smem::LIST_LDS>), dim3(grid), dim3(block), 0, st, *P); break;
        case 14: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_OCC64, false, 4, 4, true, false, false, true>), dim3(grid), dim3(block), 0, st, *P); break;
        case 15: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_OCC64, false, 4, 3, true, false, false, true>), dim3(grid), dim3(block), 0, st, *P); break;
        case 16: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_OCC64, false, 3, smem::LIST_LDS, true, false, false, true, true>), dim3(grid), dim3(block), 0, st, *P); break;
        case 17: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_OCC64, false, 2, 12, true, false, false, true, true>), dim3(grid), dim3(block), 0, st, *P); break;
        case 18: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_OCC64, false, 2, 13, true, false, false, true, true>), dim3(grid), dim3(block), 0, st, *P); break;
        case 19: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_OCC64, false, 3, 11, true, false, false, true, true, true>), dim3(grid), dim3(block), 0, st, *P); break;
        case 21: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_OCC64, false, 4, 7, true, false, false, true, false, true>), dim3(grid), dim3(block), 0, st, *P); break;
        case 22: hipLaunchKernelGGL((smem::seed_kernel<smem::FETCH_OCC64, false, 3, 11, true, false, true, true, false, true>), dim3(grid), dim3(block), 0, st, *P); break;
#endif
        // 54: the default's shape with the k-mer table (KT; smem_gpu_set_kmer_table, no table: plain)
        case 54: hipLaunchKernelGGL((smem::seed_wp_kernel<24, 18, 1, 4, false, true>), dim3(grid), dim3(block), 0, st, *P); break;
        // default (49; 0 names it): seed_wp_kernel<24 owners per wave, 18 LDS list entries per owner,
        // wave priority, 4 blocks per CU> with every OPT bit
        default: hipLaunchKernelGGL((smem::seed_wp_kernel<24, 18, 1, 4>), dim3(grid), dim3(block), 0, st, *P); break;
    }
    return hipGetLastError();
}

extern "C" hipError_t smem_launch_finalize(const smem::FinalizeParams* F, int write, hipStream_t st) {
    if (F->n <= 0 || !write) return hipSuccess;  // sizes come from the seeding kernel: no count pass
    const unsigned g = (unsigned)((4ull * F->n + 255) / 256);
    hipLaunchKernelGGL(smem::finalize_kernel, dim3(g), dim3(256), 0, st, *F);
    return hipGetLastError();
}

namespace smem {
// flat bwtintv_t (32 B) -> the 16-B wire entry smem_pintv_t (include/smem_gpu.h):
// x0, x1, x2 low words, then x0/x1/x2 bits 32-33 and the query begin / end
// (13 bits each: reads < 8192 bp, checked on the host)
__global__ __launch_bounds__(256) void pack_intv_kernel(const Intv* __restrict__ in, uint64_t n, uint4* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const Intv v = in[i];
    const uint32_t beg = (uint32_t)(v.info >> 32), end = (uint32_t)v.info;
    out[i] = make_uint4((uint32_t)v.x0, (uint32_t)v.x1, (uint32_t)v.x2,
                        (uint32_t)(v.x0 >> 32) | (uint32_t)(v.x1 >> 32) << 2 | (uint32_t)(v.x2 >> 32) << 4 | beg << 6 |
                            end << 19);
}
}  // namespace smem

extern "C" hipError_t smem_launch_pack_intv(const smem::Intv* in, uint64_t n, uint4* out, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(smem::pack_intv_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, in, n, out);
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
// Size -> offset scans with (almost) no LDS: three small launches (tile sums,
// one-block scan of the tile sums, tile rescans with carry-in), wave scans by
// shuffles and 32 B of LDS per block.  The persistent seeding kernel of
// another worker's chunk holds all but 4 KB of every CU's LDS; a library scan
// (16 KB+ of LDS per block) then waits for that whole kernel, and with it the
// chunk's copies and the next chunk (profiles/r02/stream/).
namespace smem {
constexpr int SCAN_T = 256, SCAN_I = 8, SCAN_TILE = SCAN_T * SCAN_I;

__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

// exclusive prefix of this thread's SCAN_I elements within the block, and the block total
__device__ __forceinline__ uint64_t block_excl(uint64_t tsum, uint64_t& total) {
    __shared__ uint64_t ws[SCAN_T / 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t inc = wave_incl_scan(tsum, lane);
    if (lane == 63) ws[w] = inc;
    __syncthreads();
    uint64_t before = 0;
    total = 0;
#pragma unroll
    for (int k = 0; k < SCAN_T / 64; ++k) {
        before += k < w ? ws[k] : 0;
        total += ws[k];
    }
    __syncthreads();  // ws is reused by the next call
    return before + inc - tsum;
}

__global__ __launch_bounds__(SCAN_T) void scan_tile_sums(const uint64_t* __restrict__ in, int n, uint64_t* __restrict__ bsum) {
    const int64_t b0 = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_I;
    uint64_t t = 0;
#pragma unroll
    for (int k = 0; k < SCAN_I; ++k) t += b0 + k < n ? in[b0 + k] : 0;
    uint64_t total;
    (void)block_excl(t, total);
    if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

// one block: bsum[0..nb) -> exclusive offsets in place
__global__ __launch_bounds__(SCAN_T) void scan_tile_offsets(uint64_t* __restrict__ bsum, int nb) {
    uint64_t carry = 0;
    for (int base = 0; base < nb; base += SCAN_TILE) {
        const int b0 = base + (int)threadIdx.x * SCAN_I;
        uint64_t v[SCAN_I], t = 0;
#pragma unroll
        for (int k = 0; k < SCAN_I; ++k) {
            v[k] = b0 + k < nb ? bsum[b0 + k] : 0;
            t += v[k];
        }
        uint64_t total;
        uint64_t run = carry + block_excl(t, total);
#pragma unroll
        for (int k = 0; k < SCAN_I; ++k) {
            if (b0 + k < nb) bsum[b0 + k] = run;
            run += v[k];
        }
        carry += total;
    }
}

__global__ __launch_bounds__(SCAN_T) void scan_tiles(const uint64_t* __restrict__ in, int n,
                                                     const uint64_t* __restrict__ boff, uint64_t* __restrict__ out) {
    const int64_t b0 = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_I;
    uint64_t v[SCAN_I], t = 0;
#pragma unroll
    for (int k = 0; k < SCAN_I; ++k) {
        v[k] = b0 + k < n ? in[b0 + k] : 0;
        t += v[k];
    }
    uint64_t total;
    uint64_t run = boff[blockIdx.x] + block_excl(t, total);
    if (blockIdx.x == 0 && threadIdx.x == 0) out[0] = 0;
#pragma unroll
    for (int k = 0; k < SCAN_I; ++k) {
        run += v[k];
        if (b0 + k < n) out[b0 + k + 1] = run;
    }
}
}  // namespace smem

// out[0] = 0, out[1..n] = inclusive sums of in[0..n-1]; temp == nullptr
// queries the temporary size into *temp_bytes
extern "C" hipError_t smem_launch_offsets(const uint64_t* in, uint64_t* out, int n, void* temp, size_t* temp_bytes,
                                          hipStream_t st) {
    const int nb = n > 0 ? (n + smem::SCAN_TILE - 1) / smem::SCAN_TILE : 1;
    if (temp == nullptr) {
        *temp_bytes = sizeof(uint64_t) * (size_t)(nb + 1);
        return hipSuccess;
    }
    if (*temp_bytes < sizeof(uint64_t) * (size_t)nb) return hipErrorInvalidValue;
    if (n <= 0) return hipMemsetAsync(out, 0, sizeof(uint64_t), st);
    uint64_t* bsum = static_cast<uint64_t*>(temp);
    hipLaunchKernelGGL(smem::scan_tile_sums, dim3(nb), dim3(smem::SCAN_T), 0, st, in, n, bsum);
    hipLaunchKernelGGL(smem::scan_tile_offsets, dim3(1), dim3(smem::SCAN_T), 0, st, bsum, nb);
    hipLaunchKernelGGL(smem::scan_tiles, dim3(nb), dim3(smem::SCAN_T), 0, st, in, n, bsum, out);
    return hipGetLastError();
}

namespace smem {
// reference interleaved buckets (software/bwtindex.c:128-150: 4 x u64 Occ +
// 8 x u32 symbols per 128) -> Occ64 (see Bucket32); one thread per 64 symbols
__global__ __launch_bounds__(256) void occ64_kernel(const uint32_t* __restrict__ bwt, uint64_t n_ref,
                                                     uint32_t* __restrict__ out) {
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= 2 * n_ref) return;
    const uint32_t* r = bwt + (b >> 1) * 16;
    uint64_t c1 = (uint64_t)r[3] << 32 | r[2], c2 = (uint64_t)r[5] << 32 | r[4], c3 = (uint64_t)r[7] << 32 | r[6];
    const uint32_t* sw = r + 8 + (b & 1) * 4;
    if (b & 1) {  // add the first 64 symbols of the 128-block
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t lo = r[8 + i] & 0x55555555u, hi = (r[8 + i] >> 1) & 0x55555555u;
            const uint32_t t = __popc(lo & hi);
            c1 += __popc(lo) - t;
            c2 += __popc(hi) - t;
            c3 += t;
        }
    }
    uint4* o = reinterpret_cast<uint4*>(out + b * 8);
    o[0] = make_uint4((uint32_t)c1, (uint32_t)c2, (uint32_t)c3,
                      (uint32_t)(c1 >> 32) | (uint32_t)(c2 >> 32) << 2 | (uint32_t)(c3 >> 32) << 4);
    o[1] = make_uint4(sw[0], sw[1], sw[2], sw[3]);
}
}  // namespace smem

namespace smem {
// k-mer table level L from level L - 1: one thread per (L-1)-mer W extends
// its bi-interval backward by each base c (bwt_extend, software/bwt.c:416-429)
// and writes cW's entry at index c << 2(L-1) | code(W)
__global__ __launch_bounds__(256) void kmer_table_kernel(SeedParams P, uint4* __restrict__ kt, int L) {
    const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t n_par = 1ull << (2 * (L - 1));
    if (w >= n_par) return;
    const uint4* par = kt + ((1ull << (2 * (L - 1))) - 4) / 3;
    uint4* lev = kt + ((1ull << (2 * L)) - 4) / 3;
    const uint4 e = par[w];
    const uint64_t a = p_x0(e), b = p_x1(e), s = p_x2(e);
    if (s == 0) {  // absent string: so are its extensions
        for (int c = 0; c < 4; ++c) lev[(uint64_t)c << (2 * (L - 1)) | w] = make_uint4(0, 0, 0, 0);
        return;
    }
    const uint64_t k = a - 1, l = k + s;
    const uint64_t kk = k - (k >= P.primary), ll = l - (l >= P.primary);
    const uint4* o = reinterpret_cast<const uint4*>(P.occ64);  // block b: o[2b] counts, o[2b + 1] symbols
    const Bucket32 vk{o[2 * (kk >> 6)], o[2 * (kk >> 6) + 1]}, vl{o[2 * (ll >> 6)], o[2 * (ll >> 6) + 1]};
    for (int c = 0; c < 4; ++c) {
        uint64_t na, nb, ns;
        extend_counts64<false>(P, a, b, s, c, kk, ll, vk, vl, na, nb, ns);
        lev[(uint64_t)c << (2 * (L - 1)) | w] = ns ? pack_p(na, nb, ns, 0) : make_uint4(0, 0, 0, 0);
    }
}

// Occ64 -> Occ192 (see rank192); one thread per 64-B line of 192 symbols
__global__ __launch_bounds__(256) void occ192_kernel(const uint32_t* __restrict__ occ64, uint64_t n_blocks,
                                                      uint64_t n_lines, uint32_t* __restrict__ out) {
    const uint64_t L = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (L >= n_lines) return;
    const uint4* o = reinterpret_cast<const uint4*>(occ64);  // block b: o[2b] counts, o[2b + 1] symbols
    const uint64_t b0 = 3 * L;
    uint4 sym[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) sym[i] = b0 + i < n_blocks ? o[2 * (b0 + i) + 1] : make_uint4(0, 0, 0, 0);
    uint64_t c, g, t;
    if (b0 + 1 < n_blocks) {
        const uint4 cnt = o[2 * (b0 + 1)];
        c = occ_cgt(cnt, 0), g = occ_cgt(cnt, 1), t = occ_cgt(cnt, 2);
    } else {  // the line's first block is the last one: counts through its end
        const uint4 cnt = o[2 * b0];
        uint32_t C, G, T;
        count_cgt4(sym[0], 63, C, G, T);
        c = occ_cgt(cnt, 0) + C, g = occ_cgt(cnt, 1) + G, t = occ_cgt(cnt, 2) + T;
    }
    uint32_t dC, dG, dT;
    count_cgt4(sym[1], 63, dC, dG, dT);
    uint4* w = reinterpret_cast<uint4*>(out) + 4 * L;
    w[0] = make_uint4((uint32_t)c, (uint32_t)g, (uint32_t)t,
                      (uint32_t)(c >> 32) | (uint32_t)(g >> 32) << 2 | (uint32_t)(t >> 32) << 4 | dC << 6 | dG << 13 |
                          dT << 20);
    w[1] = sym[0];
    w[2] = sym[1];
    w[3] = sym[2];
}
}  // namespace smem

extern "C" hipError_t smem_launch_kmer_table(const uint32_t* occ64, uint64_t primary, const uint64_t* L2, int k,
                                              uint4* kt, hipStream_t st) {
    if (k < 1 || k > 15) return hipErrorInvalidValue;
    smem::SeedParams P;
    memset(&P, 0, sizeof(P));
    P.occ64 = occ64;
    P.primary = primary;
    for (int c = 0; c < 5; ++c) P.L2[c] = L2[c];
    uint4 lev1[4];  // bwt_set_intv (software/bwt.h:80)
    for (int c = 0; c < 4; ++c)
        lev1[c] = smem::pack_p(L2[c] + 1, L2[3 - c] + 1, L2[c + 1] - L2[c], 0);
    hipError_t e = hipMemcpyAsync(kt, lev1, sizeof(lev1), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);  // lev1 is on this stack
    for (int L = 2; L <= k && e == hipSuccess; ++L) {
        const uint64_t n = 1ull << (2 * (L - 1));
        hipLaunchKernelGGL(smem::kmer_table_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, P, kt, L);
        e = hipGetLastError();
    }
    return e;
}

extern "C" hipError_t smem_launch_occ192(const uint32_t* occ64, uint64_t n_blocks, uint32_t* out, hipStream_t st) {
    const uint64_t n_lines = (n_blocks + 2) / 3;
    if (n_lines == 0) return hipSuccess;
    hipLaunchKernelGGL(smem::occ192_kernel, dim3((unsigned)((n_lines + 255) / 256)), dim3(256), 0, st, occ64, n_blocks,
                       n_lines, out);
    return hipGetLastError();
}

extern "C" hipError_t smem_launch_occ64(const uint32_t* bwt, uint64_t n_ref_buckets, uint32_t* out, hipStream_t st) {
    const uint64_t n = 2 * n_ref_buckets;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(smem::occ64_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, bwt, n_ref_buckets, out);
    return hipGetLastError();
}

// ------------------------------------------------------------------ bwt_sa
// The SA lookup mem_insert_seed() does for every seed occurrence
// (software/bwamem.c:462-474): for each interval of the smem_next2 lists
// with seed length >= k and x2 <= max_occ, bwt_sa(bwt, x0 + j), j < x2
// (software/bwt.c:104-114): LF steps (bwt_invPsi, software/bwt.c:71-77)
// until the row is a multiple of sa_intv, then the sampled SA.  Each LF step
// is one rank in one Occ64 bucket: the symbol at the row and its count are in
// the same 32 B.
namespace smem {


// occurrences of each interval (software/bwamem.c:467)
__global__ __launch_bounds__(256) void sa_count_kernel(SaParams S) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= S.n_intv) return;
    const Intv v = S.intv[t];
    const int slen = (int)((uint32_t)v.info - (uint32_t)(v.info >> 32));
    S.n_occ_intv[t] = (slen < S.min_seed_len || v.x2 > S.max_occ) ? 0 : v.x2;
}

// rows x0 .. x0 + n - 1 of every interval at its occurrence offset
__global__ __launch_bounds__(256) void sa_fill_kernel(SaParams S) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= S.n_intv) return;
    const uint64_t o = S.occ_off[t], n = S.occ_off[t + 1] - o;
    const uint64_t x0 = S.intv[t].x0;
    for (uint64_t j = 0; j < n; ++j) S.kstart[o + j] = x0 + j;
}

// One lane per occurrence, occurrences dealt lane-strided.  Lanes of a wave
// walk different numbers of LF steps (0 .. sa_intv-1); a lane that finishes
// takes its next occurrence in the same loop.  Every iteration makes exactly
// two 16-B loads per lane from per-lane addresses — the Occ64 bucket (counts,
// symbols) for a lane that steps, or the 16 B around its SA sample and
// around its next occurrence's row for a lane that finishes — so the wave
// waits for one memory round trip per iteration whatever its lanes do.
__global__ __launch_bounds__(256) void sa_walk_kernel(SaParams S) {
    const uint64_t lanes = (uint64_t)gridDim.x * blockDim.x;
    uint64_t o = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t mask = (1ull << S.sa_shift) - 1;
    const uint4* occ = reinterpret_cast<const uint4*>(S.occ64);
    const uint4* sa16 = reinterpret_cast<const uint4*>(S.sa);
    const uint4* ks16 = reinterpret_cast<const uint4*>(S.kstart);
    bool live = o < S.n_occ;
    uint64_t k = live ? S.kstart[o] : 0, steps = 0;
    while (__any(live)) {
        const bool step = live && (k & mask) != 0;
        const uint64_t on = o + lanes;  // next occurrence of this lane
        const uint64_t kk = k - (k > S.primary);
        const uint4* pa = step ? occ + (kk >> 6) * 2 : sa16 + ((k >> S.sa_shift) >> 1);
        const uint4* pb = step ? pa + 1 : ks16 + ((on < S.n_occ ? on : 0) >> 1);
        uint4 va = {0, 0, 0, 0}, vb = {0, 0, 0, 0};
        if (live) {
            va = *pa;
            vb = *pb;
        }
        if (step) {  // bwt_invPsi (software/bwt.c:71-77) on the Occ64 bucket
            if (k == S.primary) {
                k = 0;
            } else {
                const uint32_t pos = (uint32_t)(kk & 63), sel = pos >> 4;
                const uint32_t w = sel == 0 ? vb.x : (sel == 1 ? vb.y : (sel == 2 ? vb.z : vb.w));
                const int c = (int)((w >> ((~pos & 15u) << 1)) & 3u);
                uint32_t C, G, T;
                count_cgt4(vb, pos, C, G, T);
                const uint64_t oc = occ_cgt(va, 0) + C, og = occ_cgt(va, 1) + G, ot = occ_cgt(va, 2) + T;
                const uint64_t n = c == 0 ? kk + 1 - oc - og - ot : (c == 1 ? oc : (c == 2 ? og : ot));
                k = sel4(c, S.L2[0], S.L2[1], S.L2[2], S.L2[3]) + n;
            }
            ++steps;
        } else if (live) {
            // sa[0] = -1: unsigned wrap as in software/bwt.c:110-113
            const uint64_t si = k >> S.sa_shift;
            S.pos[o] = steps + ((si & 1) ? ((uint64_t)va.w << 32 | va.z) : ((uint64_t)va.y << 32 | va.x));
            o = on;
            live = o < S.n_occ;
            k = (o & 1) ? ((uint64_t)vb.w << 32 | vb.z) : ((uint64_t)vb.y << 32 | vb.x);
            steps = 0;
        }
    }
}

// A denser device copy of the sampled SA: dense[i] = bwt_sa(i * D) for
// D = 2^dshift dividing sa_intv, each computed by the same LF walk to the
// next stored sample.  bwt_sa(k) walked to the first multiple of D and
// finished from dense[] equals the reference's walk to the first multiple of
// sa_intv (same steps, same unsigned arithmetic, sa[0] = -1 included), so
// lookups take (D-1)/2 steps on average instead of (sa_intv-1)/2.
__global__ __launch_bounds__(256) void sa_densify_kernel(SaParams S, uint32_t dshift, uint64_t n_dense,
                                                          uint64_t* __restrict__ dense) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_dense) return;
    const uint64_t mask = (1ull << S.sa_shift) - 1;
    const uint4* occ = reinterpret_cast<const uint4*>(S.occ64);
    uint64_t k = i << dshift, steps = 0;
    while (k & mask) {
        if (k == S.primary) {
            k = 0;
        } else {
            const uint64_t kk = k - (k > S.primary);
            const uint4 va = occ[(kk >> 6) * 2], vb = occ[(kk >> 6) * 2 + 1];
            const uint32_t pos = (uint32_t)(kk & 63), sel = pos >> 4;
            const uint32_t w = sel == 0 ? vb.x : (sel == 1 ? vb.y : (sel == 2 ? vb.z : vb.w));
            const int c = (int)((w >> ((~pos & 15u) << 1)) & 3u);
            uint32_t C, G, T;
            count_cgt4(vb, pos, C, G, T);
            const uint64_t oc = occ_cgt(va, 0) + C, og = occ_cgt(va, 1) + G, ot = occ_cgt(va, 2) + T;
            const uint64_t n = c == 0 ? kk + 1 - oc - og - ot : (c == 1 ? oc : (c == 2 ? og : ot));
            k = sel4(c, S.L2[0], S.L2[1], S.L2[2], S.L2[3]) + n;
        }
        ++steps;
    }
    dense[i] = steps + S.sa[k >> S.sa_shift];
}

// The same dense[] in two passes that share the walks.  The walk from row
// i * D passes through other multiples of D on its way to a stored sample,
// and every dense row's walk from there on is that row's own walk, so:
//   hop pass:   every dense row that is not a stored sample walks only to the
//               next multiple of D: link[i] = (that row / D) | steps << 32.
//               The walks end at the first dense row, so together they step
//               over each BWT row once: seq_len LF steps instead of
//               n_dense * (sa_intv / D) * ~(D - 1).
//   chase pass: dense[i] = the steps summed along the links up to a stored
//               sample + that sample (unsigned, sa[0] = -1 wrapping as in
//               software/bwt.c:110-113), one 8-B load per link; a finished
//               row's link is replaced by its total (path compression), so
//               chains that reach it later stop there.
// Walks and chains differ in length across the lanes of a wave, so both
// passes deal their rows lane-strided and a lane that finishes takes its
// next row in the same loop (the sa_walk_kernel scheme).  Link targets need
// 32 bits: the host uses these passes while n_dense < 2^32.
__global__ __launch_bounds__(256) void sa_densify_hop_kernel(SaParams S, uint32_t dshift, uint64_t n_dense,
                                                              uint64_t* __restrict__ link) {
    const uint64_t lanes = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t smask = (1ull << (S.sa_shift - dshift)) - 1;  // dense rows that are stored samples
    const uint64_t dmask = (1ull << dshift) - 1;
    const uint4* occ = reinterpret_cast<const uint4*>(S.occ64);
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool live = i < n_dense;
    uint64_t k = i << dshift, steps = 0;
    while (__any(live)) {
        if (live && ((i & smask) == 0 || (steps && (k & dmask) == 0))) {
            if (i & smask) link[i] = (k >> dshift) | steps << 32;
            i += lanes;
            live = i < n_dense;
            k = i << dshift;
            steps = 0;
        } else if (live) {  // bwt_invPsi (software/bwt.c:71-77) on the Occ64 bucket
            if (k == S.primary) {
                k = 0;
            } else {
                const uint64_t kk = k - (k > S.primary);
                const uint4 va = occ[(kk >> 6) * 2], vb = occ[(kk >> 6) * 2 + 1];
                const uint32_t pos = (uint32_t)(kk & 63), sel = pos >> 4;
                const uint32_t w = sel == 0 ? vb.x : (sel == 1 ? vb.y : (sel == 2 ? vb.z : vb.w));
                const int c = (int)((w >> ((~pos & 15u) << 1)) & 3u);
                uint32_t C, G, T;
                count_cgt4(vb, pos, C, G, T);
                const uint64_t oc = occ_cgt(va, 0) + C, og = occ_cgt(va, 1) + G, ot = occ_cgt(va, 2) + T;
                const uint64_t n = c == 0 ? kk + 1 - oc - og - ot : (c == 1 ? oc : (c == 2 ? og : ot));
                k = sel4(c, S.L2[0], S.L2[1], S.L2[2], S.L2[3]) + n;
            }
            ++steps;
        }
    }
}

__global__ __launch_bounds__(256) void sa_densify_chase_kernel(SaParams S, uint32_t dshift, uint64_t n_dense,
                                                                uint64_t* link, uint64_t* __restrict__ dense) {
    const uint64_t lanes = (uint64_t)gridDim.x * blockDim.x;
    const uint32_t rshift = S.sa_shift - dshift;
    const uint64_t smask = (1ull << rshift) - 1;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool live = i < n_dense;
    uint64_t j = i, acc = 0;
    while (__any(live)) {
        if (live && (j & smask) == 0) {
            dense[i] = acc + S.sa[j >> rshift];
            // path compression: a later chain through row i jumps straight to
            // the sample (its link still says "acc steps to row j", the same
            // walk).  Other lanes may read link[i] before or after this store
            // (an aligned 8-B store, never torn), and either value is right.
            if (acc) link[i] = j | acc << 32;
            i += lanes;
            live = i < n_dense;
            j = i;
            acc = 0;
        } else if (live) {
            const uint64_t l = link[j];
            acc += l >> 32;
            j = (uint32_t)l;
        }
    }
}

}  // namespace smem

// lane-strided passes: enough waves to fill the chip several times over
static unsigned densify_grid(uint64_t n) {
    const uint64_t want = (n + 255) / 256;
    return (unsigned)(want < 256 * 64 ? (want ? want : 1) : 256 * 64);
}

extern "C" hipError_t smem_launch_sa_densify2(const smem::SaParams* S, uint32_t dshift, uint64_t n_dense,
                                              uint64_t* link, uint64_t* dense, unsigned max_blocks, hipStream_t st) {
    if (n_dense == 0) return hipSuccess;
    if (n_dense >= (1ull << 32) || dshift >= S->sa_shift) return hipErrorInvalidValue;
    unsigned grid = densify_grid(n_dense);
    if (max_blocks && grid > max_blocks) grid = max_blocks;
    hipLaunchKernelGGL(smem::sa_densify_hop_kernel, dim3(grid), dim3(256), 0, st, *S, dshift, n_dense, link);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(smem::sa_densify_chase_kernel, dim3(grid), dim3(256), 0, st, *S, dshift, n_dense, link,
                       dense);
    return hipGetLastError();
}

extern "C" hipError_t smem_launch_sa_densify(const smem::SaParams* S, uint32_t dshift, uint64_t n_dense,
                                             uint64_t* dense, hipStream_t st) {
    if (n_dense == 0) return hipSuccess;
    hipLaunchKernelGGL(smem::sa_densify_kernel, dim3((unsigned)((n_dense + 255) / 256)), dim3(256), 0, st, *S, dshift,
                       n_dense, dense);
    return hipGetLastError();
}

extern "C" hipError_t smem_launch_sa_count(const smem::SaParams* S, hipStream_t st) {
    if (S->n_intv == 0) return hipSuccess;
    hipLaunchKernelGGL(smem::sa_count_kernel, dim3((unsigned)((S->n_intv + 255) / 256)), dim3(256), 0, st, *S);
    return hipGetLastError();
}

extern "C" hipError_t smem_launch_sa_walk(const smem::SaParams* S, int grid, hipStream_t st) {
    if (S->n_occ == 0) return hipSuccess;
    hipLaunchKernelGGL(smem::sa_fill_kernel, dim3((unsigned)((S->n_intv + 255) / 256)), dim3(256), 0, st, *S);
    hipLaunchKernelGGL(smem::sa_walk_kernel, dim3(grid), dim3(256), 0, st, *S);
    return hipGetLastError();
}

// this file's code object loaded on the current device without running
// anything (smem_gpu_reserve_slots: the first batch does not pay the load)
extern "C" hipError_t smem_preload_seed(void) {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&smem::sa_count_kernel));
}
