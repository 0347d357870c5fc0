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
//  * the per-read interval lists (forward list, prev/curr, matches, sub)
//    live in a per-lane scratch arena in HBM (L1/L2-resident in practice).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "smem_kernels.h"

namespace smem {

__device__ __forceinline__ void load_bucket(const uint32_t* __restrict__ bwt, uint64_t kk, uint4 (&v)[4]) {
    const uint4* p = reinterpret_cast<const uint4*>(bwt + ((kk >> 7) << 4));
    v[0] = p[0];
    v[1] = p[1];
    v[2] = p[2];
    v[3] = p[3];
}

// Counts of C, G, T among the first pos+1 symbols of the bucket's 8 words
// (MSB-first 2-bit symbols). A = pos+1 - C - G - T, which is what
// bwt_occ4's "masked tail reads as A, subtract ~k&15" produces.
__device__ __forceinline__ void count_cgt(const uint4 (&v)[4], uint32_t pos, uint32_t& C, uint32_t& G, uint32_t& T) {
    const uint32_t w[8] = {v[2].x, v[2].y, v[2].z, v[2].w, v[3].x, v[3].y, v[3].z, v[3].w};
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

// One bwt_extend in one direction, returning only the child for base c.
//   a: coordinate searched through the BWT (x[1] forward, x[0] backward)
//   b: the other coordinate, s: interval size
//   -> na = L2[c] + 1 + Occ(c, a-1), ns = Occ(c, a-1+s) - Occ(c, a-1),
//      nb = b + [$ in interval] + sum_{c' > c} (Occ(c', a-1+s) - Occ(c', a-1))
// (software/bwt.c:416-429; the four-way cumulative in :425-428 restricted
// to the child actually taken).
__device__ __forceinline__ void extend1(const SeedParams& P, uint64_t a, uint64_t b, uint64_t s, int c,
                                        uint64_t& na, uint64_t& nb, uint64_t& ns) {
    const uint64_t k = a - 1, l = k + s;
    const uint64_t kk = k - (k >= P.primary), ll = l - (l >= P.primary);
    uint4 vk[4], vl[4];
    load_bucket(P.bwt, kk, vk);
    if ((kk >> 7) != (ll >> 7)) {
        load_bucket(P.bwt, ll, vl);
    } else {
        vl[0] = vk[0]; vl[1] = vk[1]; vl[2] = vk[2]; vl[3] = vk[3];
    }
    uint32_t Ck, Gk, Tk, Cl, Gl, Tl;
    const uint32_t pk = (uint32_t)(kk & 127), pl = (uint32_t)(ll & 127);
    count_cgt(vk, pk, Ck, Gk, Tk);
    count_cgt(vl, pl, Cl, Gl, Tl);
    const uint32_t Ak = pk + 1 - Ck - Gk - Tk, Al = pl + 1 - Cl - Gl - Tl;
    const uint64_t tk0 = cnt64(vk[0], 0) + Ak, tk1 = cnt64(vk[0], 1) + Ck;
    const uint64_t tk2 = cnt64(vk[1], 0) + Gk, tk3 = cnt64(vk[1], 1) + Tk;
    const uint64_t tl0 = cnt64(vl[0], 0) + Al, tl1 = cnt64(vl[0], 1) + Cl;
    const uint64_t tl2 = cnt64(vl[1], 0) + Gl, tl3 = cnt64(vl[1], 1) + Tl;
    const uint64_t d0 = tl0 - tk0, d1 = tl1 - tk1, d2 = tl2 - tk2, d3 = tl3 - tk3;
    const uint64_t L2c = sel4(c, P.L2[0], P.L2[1], P.L2[2], P.L2[3]);
    na = L2c + 1 + sel4(c, tk0, tk1, tk2, tk3);
    ns = sel4(c, d0, d1, d2, d3);
    const uint64_t gt = (c < 1 ? d1 : 0) + (c < 2 ? d2 : 0) + (c < 3 ? d3 : 0);
    nb = b + (uint64_t)(a <= P.primary && a + s - 1 >= P.primary) + gt;
}

enum Phase : int {
    P_FETCH = 0,
    P_NEXT2,
    P_SMEM_BEGIN,
    P_FWD,
    P_FWD_RES,
    P_FWD_DONE,
    P_BWD_STEP,
    P_BWD_J,
    P_BWD_RES,
    P_SMEM_END,
    P_EXIT
};

__global__ __launch_bounds__(256) void seed_kernel(SeedParams P) {
    const uint64_t lane_g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t cap = P.cap_list;
    Intv* __restrict__ base = P.scratch + lane_g * 4ull * cap;
    const uint32_t MOFF = 2 * cap, SOFF = 3 * cap;

    int phase = P_FETCH;
    int item = -1, len = 0;
    const uint8_t* q = nullptr;
    Intv* out = nullptr;
    uint32_t* callv = nullptr;
    uint32_t out_n = 0, calls_n = 0;
    int start = 0, ori_start = 0, split_len = 0;
    int x = 0, min_intv = 1, middle = 0, i = 0, j = 0, ret = 0, cur_c = 0;
    uint64_t ik0 = 0, ik1 = 0, ik2 = 0, ikinfo = 0, last_fwd_info = 0;
    uint32_t fwd_n = 0, prev_off = 0, prev_n = 0, curr_off = 0, curr_n = 0;
    uint32_t mem_off = 0, mem_n = 0, mem_last_start = 0, m_n = 0;
    uint64_t curr_last_x2 = 0;
    int max_len = 0;
    Intv pc = {0, 0, 0, 0};
    uint64_t ra = 0, rb = 0, rs = 0, na = 0, nb = 0, ns = 0;

    for (;;) {
        // ---- advance the lane's state machine until it needs an extend ----
        for (;;) {
            if (phase == P_FETCH) {
                item = atomicAdd(P.head, 1);
                if (item >= P.n_items) { phase = P_EXIT; break; }
                const int rid = P.read_ids ? P.read_ids[item] : item;
                const uint64_t o0 = P.offs[rid], o1 = P.offs[rid + 1];
                q = P.codes + o0;
                len = (int)(o1 - o0);
                out = P.out_intv + (uint64_t)item * P.cap_intv;
                callv = P.out_call_n + (uint64_t)item * P.cap_calls;
                out_n = 0;
                calls_n = 0;
                start = 0;
                if (len < P.min_seed_len) {  // mem_chain's guard (software/bwamem.c:600)
                    P.n_intv[item] = 0;
                    P.n_calls[item] = 0;
                    continue;
                }
                split_len = P.split_len_init < len ? P.split_len_init : len;  // software/bwamem.c:456-458
                phase = P_NEXT2;
                continue;
            }
            if (phase == P_NEXT2) {  // software/bwamem.c:247-261
                if (start < len && start >= 0)
                    while (start < len && q[start] > 3) ++start;  // skip ambiguous bases
                if (start >= len || start < 0) {                   // iterator exhausted
                    P.n_intv[item] = out_n;
                    P.n_calls[item] = calls_n;
                    phase = P_FETCH;
                    continue;
                }
                ori_start = start;
                x = ori_start;
                min_intv = P.start_width;
                middle = 0;
                mem_off = MOFF;
                phase = P_SMEM_BEGIN;
                continue;
            }
            if (phase == P_SMEM_BEGIN) {  // software/bwt.c:782-789
                mem_n = 0;
                const int qx = q[x];
                if (qx > 3) { ret = x + 1; phase = P_SMEM_END; continue; }
                if (min_intv < 1) min_intv = 1;
                ik0 = P.L2[qx] + 1;
                ik2 = P.L2[qx + 1] - P.L2[qx];
                ik1 = P.L2[3 - qx] + 1;
                ikinfo = (uint64_t)(x + 1);
                fwd_n = 0;
                i = x + 1;
                phase = P_FWD;
                continue;
            }
            if (phase == P_FWD) {  // software/bwt.c:791-805
                if (i < len) {
                    const int qi = q[i];
                    if (qi < 4) {
                        cur_c = 3 - qi;
                        ra = ik1; rb = ik0; rs = ik2;
                        phase = P_FWD_RES;
                        break;  // -> extend (forward)
                    }
                }
                // ambiguous base, or end of query: push ik and stop
                base[cap - 1 - fwd_n] = Intv{ik0, ik1, ik2, ikinfo};
                ++fwd_n;
                last_fwd_info = ikinfo;
                phase = P_FWD_DONE;
                continue;
            }
            if (phase == P_FWD_RES) {  // na = x[1], nb = x[0]
                if (ns != ik2) {
                    base[cap - 1 - fwd_n] = Intv{ik0, ik1, ik2, ikinfo};
                    ++fwd_n;
                    last_fwd_info = ikinfo;
                    if (ns < (uint64_t)min_intv) { phase = P_FWD_DONE; continue; }
                }
                ik0 = nb; ik1 = na; ik2 = ns;
                ikinfo = (uint64_t)(i + 1);
                ++i;
                phase = P_FWD;
                continue;
            }
            if (phase == P_FWD_DONE) {  // reverse + ret (software/bwt.c:806-808)
                ret = (int)last_fwd_info;
                prev_off = cap - fwd_n;  // pushed downward: ascending = reversed
                prev_n = fwd_n;
                curr_off = cap;
                i = x - 1;
                phase = P_BWD_STEP;
                continue;
            }
            if (phase == P_BWD_STEP) {  // software/bwt.c:810-812
                cur_c = i < 0 ? -1 : (q[i] < 4 ? (int)q[i] : -1);
                curr_n = 0;
                if (cur_c < 0) {
                    // Nothing can extend: only prev[0] (the longest) can be kept,
                    // exactly what the j-loop of software/bwt.c:812-826 does here.
                    if (mem_n == 0 || (uint32_t)(i + 1) < mem_last_start) {
                        const Intv p0 = base[prev_off];
                        base[mem_off + cap - 1 - mem_n] = Intv{p0.x0, p0.x1, p0.x2, p0.info | ((uint64_t)(i + 1) << 32)};
                        ++mem_n;
                        mem_last_start = (uint32_t)(i + 1);
                    }
                    phase = P_SMEM_END;
                    continue;
                }
                j = 0;
                phase = P_BWD_J;
                continue;
            }
            if (phase == P_BWD_J) {
                if ((uint32_t)j < prev_n) {
                    pc = base[prev_off + j];
                    ra = pc.x0; rb = pc.x1; rs = pc.x2;
                    phase = P_BWD_RES;
                    break;  // -> extend (backward)
                }
                if (curr_n == 0) { phase = P_SMEM_END; continue; }  // software/bwt.c:827
                prev_off = curr_off;
                prev_n = curr_n;
                curr_off = curr_off == cap ? 0 : cap;
                --i;
                phase = P_BWD_STEP;
                continue;
            }
            if (phase == P_BWD_RES) {  // na = x[0], nb = x[1]; software/bwt.c:815-825
                if (ns < (uint64_t)min_intv) {
                    if (curr_n == 0 && (mem_n == 0 || (uint32_t)(i + 1) < mem_last_start)) {
                        base[mem_off + cap - 1 - mem_n] = Intv{pc.x0, pc.x1, pc.x2, pc.info | ((uint64_t)(i + 1) << 32)};
                        ++mem_n;
                        mem_last_start = (uint32_t)(i + 1);
                    }
                } else if (curr_n == 0 || ns != curr_last_x2) {
                    base[curr_off + curr_n] = Intv{na, nb, ns, pc.info};
                    ++curr_n;
                    curr_last_x2 = ns;
                }
                ++j;
                phase = P_BWD_J;
                continue;
            }
            if (phase == P_SMEM_END) {
                bool ovf = false;
                if (!middle) {  // first bwt_smem1 of smem_next2 (software/bwamem.c:261-272)
                    start = ret;
                    m_n = mem_n;
                    const Intv* M = base + MOFF + cap - m_n;  // final (start-sorted) order
                    uint32_t max_i = 0;
                    max_len = 0;
                    for (uint32_t f = 0; f < m_n; ++f) {
                        const uint64_t inf = M[f].info;
                        const int l = (int)((uint32_t)inf - (uint32_t)(inf >> 32));
                        if (max_len < l) { max_len = l; max_i = f; }
                    }
                    if (m_n > 0 && split_len > 0 && max_len >= split_len &&
                        M[max_i].x2 <= (uint64_t)(int64_t)P.split_width) {
                        // re-seed from the middle of the longest SMEM (software/bwamem.c:272-278)
                        const uint64_t inf = M[max_i].info;
                        x = (int)(((uint64_t)(uint32_t)inf + (inf >> 32)) >> 1);
                        min_intv = (int)(M[max_i].x2 + 1);
                        middle = 1;
                        mem_off = SOFF;
                        phase = P_SMEM_BEGIN;
                        continue;
                    }
                    // emit matches as one smem_next2 list
                    if (out_n + m_n > P.cap_intv || calls_n >= P.cap_calls) {
                        ovf = true;
                    } else {
                        for (uint32_t f = 0; f < m_n; ++f) out[out_n + f] = M[f];
                        out_n += m_n;
                        callv[calls_n++] = m_n;
                    }
                } else {  // ordered merge of matches and sub (software/bwamem.c:280-301)
                    const Intv* M = base + MOFF + cap - m_n;
                    const Intv* S = base + SOFF + cap - mem_n;
                    uint32_t a = 0, b = 0, n = 0;
                    const uint64_t half = (uint64_t)(int64_t)(max_len >> 1);
                    const uint32_t cap_left = P.cap_intv - out_n;
                    if (calls_n >= P.cap_calls) ovf = true;
                    while (!ovf && a < m_n && b < mem_n) {
                        const Intv ma = M[a], sb = S[b];
                        const uint64_t xi = (ma.info >> 32 << 32) | (uint64_t)(uint32_t)(len - (uint32_t)ma.info);
                        const uint64_t xj = (sb.info >> 32 << 32) | (uint64_t)(uint32_t)(len - (uint32_t)sb.info);
                        if ((int64_t)xi < (int64_t)xj) {
                            if (n >= cap_left) { ovf = true; break; }
                            out[out_n + n++] = ma;
                            ++a;
                        } else {
                            if ((uint64_t)(uint32_t)sb.info - (sb.info >> 32) >= half && (uint32_t)sb.info > (uint32_t)ori_start) {
                                if (n >= cap_left) { ovf = true; break; }
                                out[out_n + n++] = sb;
                            }
                            ++b;
                        }
                    }
                    for (; !ovf && a < m_n; ++a) {
                        if (n >= cap_left) { ovf = true; break; }
                        out[out_n + n++] = M[a];
                    }
                    for (; !ovf && b < mem_n; ++b) {
                        const Intv sb = S[b];
                        if ((uint64_t)(uint32_t)sb.info - (sb.info >> 32) >= half && (uint32_t)sb.info > (uint32_t)ori_start) {
                            if (n >= cap_left) { ovf = true; break; }
                            out[out_n + n++] = sb;
                        }
                    }
                    if (!ovf) {
                        out_n += n;
                        callv[calls_n++] = n;
                    }
                }
                if (ovf) {  // result does not fit: hand the read to the overflow pass
                    P.n_intv[item] = SMEM_OVERFLOW;
                    P.n_calls[item] = 0;
                    const int slot = atomicAdd(P.ovf_count, 1);
                    P.ovf_items[slot] = item;
                    phase = P_FETCH;
                    continue;
                }
                phase = P_NEXT2;
                continue;
            }
            // P_EXIT (unreachable here)
            break;
        }
        if (phase == P_EXIT) break;
        // ---- the one bwt_extend of this iteration (all live lanes together) ----
        extend1(P, ra, rb, rs, cur_c, na, nb, ns);
    }
}

// counts (u32, overflow marker) -> u64 sizes for the scans
__global__ void sizes_kernel(const uint32_t* __restrict__ n_intv, const uint32_t* __restrict__ n_calls,
                             const int32_t* __restrict__ ovf_slot, const uint32_t* __restrict__ ovf_n_intv,
                             const uint32_t* __restrict__ ovf_n_calls, uint64_t* __restrict__ s_intv,
                             uint64_t* __restrict__ s_calls, int n) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    uint32_t ni = n_intv[r], nc = n_calls[r];
    if (ni == SMEM_OVERFLOW) {
        const int s = ovf_slot[r];
        ni = s >= 0 ? ovf_n_intv[s] : 0;
        nc = s >= 0 ? ovf_n_calls[s] : 0;
    }
    s_intv[r] = ni;
    s_calls[r] = nc;
}

// one wave per read: copy its intervals and list sizes to the flat output
__global__ __launch_bounds__(256) void gather_kernel(GatherParams G) {
    const int lane = threadIdx.x & 63;
    const int r = (int)((blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6);
    if (r >= G.n) return;
    const Intv* src = G.main_intv + (uint64_t)r * G.cap_intv;
    const uint32_t* srcc = G.main_calls + (uint64_t)r * G.cap_calls;
    if (G.n_intv[r] == SMEM_OVERFLOW) {
        const int s = G.ovf_slot[r];
        if (s < 0) return;
        src = G.ovf_intv + (uint64_t)s * G.ovf_cap_intv;
        srcc = G.ovf_calls + (uint64_t)s * G.ovf_cap_calls;
    }
    const uint64_t o = G.intv_off[r], ni = G.intv_off[r + 1] - o;
    const uint64_t co = G.call_off[r], nc = G.call_off[r + 1] - co;
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    uint4* d4 = reinterpret_cast<uint4*>(G.flat_intv + o);
    for (uint64_t k = lane; k < 2 * ni; k += 64) d4[k] = s4[k];
    for (uint64_t k = lane; k < nc; k += 64) G.flat_calls[co + k] = srcc[k];
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
extern "C" hipError_t smem_launch_seed(const smem::SeedParams* P, int grid, int block, hipStream_t st) {
    hipLaunchKernelGGL(smem::seed_kernel, dim3(grid), dim3(block), 0, st, *P);
    return hipGetLastError();
}

extern "C" hipError_t smem_launch_sizes(const uint32_t* n_intv, const uint32_t* n_calls, const int32_t* ovf_slot,
                                        const uint32_t* ovf_n_intv, const uint32_t* ovf_n_calls, uint64_t* s_intv,
                                        uint64_t* s_calls, int n, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(smem::sizes_kernel, dim3((n + 255) / 256), dim3(256), 0, st, n_intv, n_calls, ovf_slot,
                       ovf_n_intv, ovf_n_calls, s_intv, s_calls, n);
    return hipGetLastError();
}

extern "C" hipError_t smem_launch_gather(const smem::GatherParams* G, hipStream_t st) {
    if (G->n <= 0) return hipSuccess;
    const uint64_t threads = (uint64_t)G->n * 64;
    hipLaunchKernelGGL(smem::gather_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, *G);
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
