// Seed chaining + chain filter on gfx950.
//
// chain_build_kernel: one lane per read runs mem_chain's loop over the
// read's seed sequence (software/bwamem.c:462-499) with the chain tree kept
// in HBM exactly as kbtree(chn) shapes it (same node order, split rule,
// equal-key handling: software/kbtree.h:97-110, 150-224), so the chain that
// test_and_merge sees for every seed and the in-order chain list
// (software/kbtree.h:336-358) are the reference's; then, when asked,
// mem_chain_flt (software/bwamem.c:629-690) with ks_introsort's exact
// comparison sequence (software/ksort.h:146-224).
// chain_write_kernel: chains and their seeds, compacted per read.
#include "chain_kernels.h"

namespace smem {
namespace {

// Every wave-cooperative routine below runs in a one-wave workgroup
// (chain_heavy_kernel), where lanes hand data to each other through LDS or
// HBM: a wavefront-scope fence orders those accesses for the compiler and
// costs no wait (a wave's memory operations are performed in order), where a
// workgroup-scope fence waited for every outstanding store -- the chain
// records' HBM stores -- at each tree insertion.
__device__ __forceinline__ void wave_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

// The chain tree in two node formats with one code path: BNode (u32 ids and
// children, HBM pools) and LNode (u16, the LDS pool of the heavy path).

// leftmost key == k (eq) or else the last key < k (-1 if none): kbtree's
// __kb_getp_aux (software/kbtree.h:97-110).  Keys are sorted, so that is the
// count of keys below k; all 15 are loaded unconditionally (the slots past n
// are ignored) so the loads issue together.
template <class N>
__device__ __forceinline__ int node_find(const N* x, int64_t k, bool& eq) {
    const int n = x->n;
    int64_t kv[BT_MAX];
#pragma unroll
    for (int i = 0; i < BT_MAX; ++i) kv[i] = x->key[i];
    int below = 0;
#pragma unroll
    for (int i = 0; i < BT_MAX; ++i) below += (i < n) & (kv[i] < k);
    int64_t at = kv[0];
#pragma unroll
    for (int i = 1; i < BT_MAX; ++i) at = below == i ? kv[i] : at;
    eq = below < n && at == k;
    return eq ? below : below - 1;
}

// kb_intervalp's `lower` (software/kbtree.h:150-166)
template <class N>
__device__ __forceinline__ int tree_lower(const N* pool, uint32_t root, int64_t k) {
    uint32_t x = root;
    int lower = -1;
    for (;;) {
        const N* nd = pool + x;
        bool eq;
        const int i = node_find(nd, k, eq);
        if (i >= 0 && eq) return (int)nd->id[i];
        if (i >= 0) lower = (int)nd->id[i];
        if (nd->leaf) return lower;
        x = nd->child[i + 1];
    }
}

template <class N>
__device__ __forceinline__ void node_init(N* x, int leaf) {
    x->n = 0;
    x->leaf = leaf;
}

// __kb_split (software/kbtree.h:172-186): full child y = x.child[i] keeps its
// lower 7 keys, a new right sibling takes the upper 7, the middle moves up
template <class N>
__device__ __forceinline__ void node_split(N* pool, uint32_t xi, int i, uint32_t yi, uint32_t& n_nodes) {
    N* x = pool + xi;
    N* y = pool + yi;
    const uint32_t zi = n_nodes++;
    N* z = pool + zi;
    node_init(z, y->leaf);
    z->n = BT_T - 1;
    for (int j = 0; j < BT_T - 1; ++j) {
        z->key[j] = y->key[BT_T + j];
        z->id[j] = y->id[BT_T + j];
    }
    if (!y->leaf)
        for (int j = 0; j < BT_T; ++j) z->child[j] = y->child[BT_T + j];
    y->n = BT_T - 1;
    const int n = x->n;
    for (int j = n; j >= i + 1; --j) x->child[j + 1] = x->child[j];
    x->child[i + 1] = zi;
    for (int j = n - 1; j >= i; --j) {
        x->key[j + 1] = x->key[j];
        x->id[j + 1] = x->id[j];
    }
    x->key[i] = y->key[BT_T - 1];
    x->id[i] = y->id[BT_T - 1];
    x->n = n + 1;
}

// kb_putp (software/kbtree.h:188-224)
template <class N>
__device__ __forceinline__ void tree_insert(N* pool, uint32_t& root, uint32_t& n_nodes, uint32_t id, int64_t k) {
    uint32_t x = root;
    bool eq;
    if (pool[x].n == BT_MAX) {
        const uint32_t s = n_nodes++;
        node_init(pool + s, 0);
        pool[s].child[0] = x;
        node_split(pool, s, 0, x, n_nodes);
        root = x = s;
    }
    while (!pool[x].leaf) {
        int i = node_find(pool + x, k, eq) + 1;
        const uint32_t c = pool[x].child[i];
        if (pool[c].n == BT_MAX) {
            node_split(pool, x, i, c, n_nodes);
            if (k > pool[x].key[i]) ++i;
        }
        x = pool[x].child[i];
    }
    N* nd = pool + x;
    const int i = node_find(nd, k, eq);
    for (int j = nd->n - 1; j >= i + 1; --j) {
        nd->key[j + 1] = nd->key[j];
        nd->id[j + 1] = nd->id[j];
    }
    nd->key[i + 1] = k;
    nd->id[i + 1] = id;
    nd->n += 1;
}

// __kb_traverse (software/kbtree.h:336-358): in-order chain ids into out
template <class N>
__device__ __forceinline__ int tree_inorder(const N* pool, uint32_t root, uint32_t* out) {
    uint32_t sx[24];
    int si[24];
    int top = 0, n_out = 0;
    sx[0] = root;
    si[0] = 0;
    for (;;) {
        while (sx[top] != BT_NONE && si[top] <= pool[sx[top]].n) {
            const N* nd = pool + sx[top];
            sx[top + 1] = nd->leaf ? BT_NONE : (uint32_t)nd->child[si[top]];
            si[top + 1] = 0;
            ++top;
        }
        --top;
        if (top < 0) break;
        if (sx[top] != BT_NONE && si[top] < pool[sx[top]].n) out[n_out++] = pool[sx[top]].id[si[top]];
        ++si[top];
    }
    return n_out;
}

// the same traversal for a tree of at most two levels (fewer than 127 keys:
// a third level needs 2 t^2 - 1 = 127), without the stack the general walk
// keeps in scratch
template <class N>
__device__ __forceinline__ int tree_inorder2(const N* pool, uint32_t root, uint32_t* out) {
    const N* r = pool + root;
    int n_out = 0;
    if (r->leaf) {
        for (int j = 0; j < r->n; ++j) out[n_out++] = r->id[j];
        return n_out;
    }
    for (int i = 0; i <= r->n; ++i) {
        const N* c = pool + r->child[i];
        for (int j = 0; j < c->n; ++j) out[n_out++] = c->id[j];
        if (i < r->n) out[n_out++] = r->id[i];
    }
    return n_out;
}

// mem_chain_weight (software/bwamem.c:501-521), the second loop's `end`
// advanced by query coordinates as the reference writes it
__device__ __forceinline__ int chain_weight(const ChainRec& c, const SeedRec* seed, const uint32_t* next) {
    int64_t end = 0;
    int w = 0;
    uint32_t o = c.first;
    for (int j = 0; j < c.n; ++j, o = next[o]) {
        const SeedRec s = seed[o];
        if (s.qbeg >= end) w += s.len;
        else if (s.qbeg + s.len > end) w = (int)(w + (s.qbeg + s.len - end));
        end = end > s.qbeg + s.len ? end : s.qbeg + s.len;
    }
    const int tmp = w;
    end = 0;
    o = c.first;
    for (int j = 0; j < c.n; ++j, o = next[o]) {
        const SeedRec s = seed[o];
        if (s.rbeg >= end) w += s.len;
        else if (s.rbeg + s.len > end) w = (int)(w + (s.rbeg + s.len - end));
        end = end > s.qbeg + s.len ? end : s.qbeg + s.len;
    }
    return w < tmp ? w : tmp;
}

__device__ __forceinline__ bool flt_lt(const FltRec& a, const FltRec& b) { return a.w > b.w; }
__device__ __forceinline__ void flt_swap(FltRec* a, size_t i, size_t j) {
    const FltRec t = a[i];
    a[i] = a[j];
    a[j] = t;
}

__device__ __forceinline__ void flt_insertsort(FltRec* a, size_t n) {
    for (size_t i = 1; i < n; ++i)
        for (size_t j = i; j > 0 && flt_lt(a[j], a[j - 1]); --j) flt_swap(a, j, j - 1);
}

__device__ __forceinline__ void flt_combsort(FltRec* a, size_t n) {
    const double shrink = 1.2473309501039786540366528676643;
    size_t gap = n;
    bool swapped;
    do {
        if (gap > 2) {
            gap = (size_t)((double)gap / shrink);
            if (gap == 9 || gap == 10) gap = 11;
        }
        swapped = false;
        for (size_t i = 0; i + gap < n; ++i)
            if (flt_lt(a[i + gap], a[i])) {
                flt_swap(a, i, i + gap);
                swapped = true;
            }
    } while (swapped || gap > 2);
    if (gap != 1) flt_insertsort(a, n);
}

// ks_introsort(mem_flt) (software/ksort.h:176-224), comparison for comparison.
// The pending segments go to stk (3 words each: s, t, depth budget) in the
// caller's LDS or HBM, not to a private array: a 1.3 KB per-lane stack made
// every queue that ran the chain kernels allocate scratch for 64 lanes x
// every wave slot, and with 16 hardware queues the runtime ran out of scratch
// and aborted queues (failure contract).  The loop pushes only
// segments of more than 16 records and always the larger half, so at most
// log2(n / 16) + 1 <= 29 are pending for n < 2^32: 64 entries.
__device__ __forceinline__ void flt_sort(FltRec* a, uint32_t n, uint32_t* stk) {
    int top = 0, d;
    if (n < 1) return;
    if (n == 2) {
        if (flt_lt(a[1], a[0])) flt_swap(a, 0, 1);
        return;
    }
    for (d = 2; (1ull << d) < n; ++d) {
    }
    d <<= 1;
    uint32_t s = 0, t = n - 1;
    for (;;) {
        if (s < t) {
            if (--d == 0) {
                flt_combsort(a + s, t - s + 1);
                t = s;
                continue;
            }
            uint32_t i = s, j = t, k = i + ((j - i) >> 1) + 1;
            if (flt_lt(a[k], a[i])) {
                if (flt_lt(a[k], a[j])) k = j;
            } else {
                k = flt_lt(a[j], a[i]) ? i : j;
            }
            const FltRec rp = a[k];
            if (k != t) flt_swap(a, k, t);
            for (;;) {
                do ++i;
                while (flt_lt(a[i], rp));
                do --j;
                while (i <= j && flt_lt(rp, a[j]));
                if (j <= i) break;
                flt_swap(a, i, j);
            }
            flt_swap(a, i, t);
            if (i - s > t - i) {
                if (i - s > 16) {
                    stk[3 * top] = s;
                    stk[3 * top + 1] = i - 1;
                    stk[3 * top + 2] = (uint32_t)d;
                    ++top;
                }
                s = t - i > 16 ? i + 1 : t;
            } else {
                if (t - i > 16) {
                    stk[3 * top] = i + 1;
                    stk[3 * top + 1] = t;
                    stk[3 * top + 2] = (uint32_t)d;
                    ++top;
                }
                t = i - s > 16 ? i - 1 : s;
            }
        } else {
            if (top == 0) {
                flt_insertsort(a, n);
                return;
            }
            --top;
            s = stk[3 * top];
            t = stk[3 * top + 1];
            d = (int)stk[3 * top + 2];
        }
    }
}

// Where mem_insert_seed's loop over a read stands (software/bwamem.c:462-499).
struct InsState {
    uint64_t iv, o;               // next interval / occurrence
    uint32_t n_ch, root, n_nodes;
};

__device__ __forceinline__ void ins_start(InsState& st, const ChainParams& P, uint64_t i0) {
    st.iv = i0;
    st.o = P.occ_off[i0];
    st.n_ch = 0;
    st.root = 0;
    st.n_nodes = 1;
}

// Run the loop over read [i0, i1) (occurrences from S) with the chain tree in
// `pool` (cap nodes).  false: a new chain would need more nodes than cap;
// `st` then names the seed to resume at (nothing of it has been applied).
template <class N>
__device__ __forceinline__ bool insert_read(const ChainParams& P, uint64_t i1, uint64_t S, N* pool, uint32_t cap,
                                            InsState& st) {
    ChainRec* chn = P.chn + S;
    if (st.n_nodes == 1 && st.n_ch == 0) node_init(pool, 1);
    for (; st.iv < i1; ++st.iv) {
        const uint64_t b = P.occ_off[st.iv + 1];
        if (st.o >= b) continue;
        const uint64_t info = P.intv[st.iv * 4 + 3];
        const int32_t qbeg = (int32_t)(info >> 32);
        const int32_t len = (int32_t)((uint32_t)info - (uint32_t)(info >> 32));
        for (; st.o < b; ++st.o) {
            const uint64_t o = st.o;
            const int64_t rb = (int64_t)P.pos[o];
            if (rb < P.l_pac && P.l_pac < rb + len) continue;  // bridges the strands
            P.seed[o] = SeedRec{rb, qbeg, len};
            if (st.n_ch) {
                const int lw = tree_lower(pool, st.root, rb);
                if (lw >= 0) {
                    // test_and_merge (software/bwamem.c:334-354)
                    ChainRec c = chn[lw];
                    if (qbeg >= c.first_qbeg && qbeg + len <= c.last_qbeg + c.last_len && rb >= c.pos &&
                        rb + len <= c.last_rbeg + c.last_len)
                        continue;  // contained
                    const bool strand_ok = !((c.last_rbeg < P.l_pac || c.pos < P.l_pac) && rb >= P.l_pac);
                    const int64_t x = (int64_t)qbeg - c.last_qbeg, y = rb - c.last_rbeg;
                    if (strand_ok && y >= 0 && x - y <= P.w && y - x <= P.w && x - c.last_len < P.max_chain_gap &&
                        y - c.last_len < P.max_chain_gap) {
                        P.next[S + c.last] = (uint32_t)(o - S);
                        c.last = (uint32_t)(o - S);
                        c.last_rbeg = rb;
                        c.last_qbeg = qbeg;
                        c.last_len = len;
                        c.n += 1;
                        chn[lw] = c;
                        continue;
                    }
                }
            }
            // one insertion allocates at most one node per level plus a root
            if (st.n_nodes + 24 > cap || st.n_ch >= N::MAX_ID) return false;
            ChainRec c;
            c.pos = rb;
            c.last_rbeg = rb;
            c.first_qbeg = qbeg;
            c.last_qbeg = qbeg;
            c.last_len = len;
            c.n = 1;
            c.first = c.last = (uint32_t)(o - S);
            chn[st.n_ch] = c;
            tree_insert(pool, st.root, st.n_nodes, st.n_ch, rb);
            ++st.n_ch;
        }
    }
    return true;
}

// mem_chain_flt's drop loop (software/bwamem.c:652-664) by one lane
__device__ __forceinline__ int flt_drop_serial(FltRec* a, int n, float mask_level, float drop_ratio, int msl) {
    int m = 1;
    for (int i = 1; i < n; ++i) {
        int j;
        for (j = 0; j < m; ++j) {
            const int b_max = a[j].beg > a[i].beg ? a[j].beg : a[i].beg;
            const int e_min = a[j].end < a[i].end ? a[j].end : a[i].end;
            if (e_min > b_max) {
                const int li = a[i].end - a[i].beg, lj = a[j].end - a[j].beg;
                const int min_l = li < lj ? li : lj;
                if ((float)(e_min - b_max) >= (float)min_l * mask_level) {
                    if (a[j].p2 < 0) a[j].p2 = a[i].p;
                    if ((float)a[i].w < (float)a[j].w * drop_ratio && a[j].w - a[i].w >= msl << 1) break;
                }
            }
        }
        if (j == m) a[m++] = a[i];
    }
    return m;
}

// the same loop with the 64 lanes of a wave scanning the kept list j in
// order, 64 entries at a time: the first j that drops chain i ends the scan
// (p2 is set on the significant overlaps up to and including it)
__device__ __forceinline__ int flt_drop_wave(FltRec* a, int n, float mask_level, float drop_ratio, int msl, int lane) {
    int m = 1;
    for (int i = 1; i < n; ++i) {
        const FltRec ai = a[i];
        bool dropped = false;
        for (int base = 0; base < m; base += 64) {
            const int j = base + lane;
            bool sig = false, drop = false;
            if (j < m) {
                const FltRec aj = a[j];
                const int b_max = aj.beg > ai.beg ? aj.beg : ai.beg;
                const int e_min = aj.end < ai.end ? aj.end : ai.end;
                if (e_min > b_max) {
                    const int li = ai.end - ai.beg, lj = aj.end - aj.beg;
                    const int min_l = li < lj ? li : lj;
                    if ((float)(e_min - b_max) >= (float)min_l * mask_level) {
                        sig = true;
                        drop = (float)ai.w < (float)aj.w * drop_ratio && aj.w - ai.w >= msl << 1;
                    }
                }
            }
            const uint64_t bd = __ballot(sig && drop);
            const int limit = bd ? base + (int)__builtin_ctzll(bd) : 0x7fffffff;
            if (sig && j <= limit && a[j].p2 < 0) a[j].p2 = ai.p;
            if (bd) {
                dropped = true;
                break;
            }
        }
        if (!dropped) {
            if (lane == 0) a[m] = ai;
            ++m;
        }
        __builtin_amdgcn_wave_barrier();
    }
    return m;
}

// The same loop again, pruned, for drop_ratio > 0.  The kept list is in
// weight order (descending), and drop(i, j) -- w_i < w_j * drop_ratio and
// w_j - w_i >= 2 min_seed_len -- is monotone in w_j, so the j that can drop
// i form a prefix [0, J_i) of it: the first dropping j is searched there
// only.  p2 is set on the significant overlaps j <= that j (all j if none);
// once set it never changes, so only the kept chains with p2 still unset are
// visited for it: they are listed in U (any order; a marked j leaves U).
// Same kept list and p2 values as flt_drop_serial.
__device__ __forceinline__ bool flt_sig(const FltRec& ai, const FltRec& aj, float mask_level) {
    const int b_max = aj.beg > ai.beg ? aj.beg : ai.beg;
    const int e_min = aj.end < ai.end ? aj.end : ai.end;
    if (e_min <= b_max) return false;
    const int li = ai.end - ai.beg, lj = aj.end - aj.beg;
    const int min_l = li < lj ? li : lj;
    return (float)(e_min - b_max) >= (float)min_l * mask_level;
}

__device__ __forceinline__ int flt_drop_pruned(FltRec* a, uint32_t* U, int n, float mask_level, float drop_ratio,
                                               int msl, int lane) {
    int m = 1, nu = 1;
    if (lane == 0) U[0] = 0;
    wave_fence();
    __builtin_amdgcn_wave_barrier();
    for (int i = 1; i < n; ++i) {
        const FltRec ai = a[i];
        // first j of the droppers' prefix with a significant overlap
        int jstar = -1;
        for (int base = 0; base < m; base += 64) {
            const int j = base + lane;
            bool can = false, hit = false;
            if (j < m) {
                const FltRec aj = a[j];
                can = (float)ai.w < (float)aj.w * drop_ratio && aj.w - ai.w >= msl << 1;
                hit = can && flt_sig(ai, aj, mask_level);
            }
            const uint64_t bh = __ballot(hit);
            if (bh) {
                jstar = base + (int)__builtin_ctzll(bh);
                break;
            }
            if (__ballot(can) != __ballot(j < m)) break;  // the prefix ends in this chunk
        }
        const int limit = jstar >= 0 ? jstar : m - 1;
        // p2 on the significant overlaps j <= limit among those still unset
        int out = 0;
        for (int base = 0; base < nu; base += 64) {
            const int u = base + lane;
            uint32_t j = 0;
            bool keep = false;
            if (u < nu) {
                j = U[u];
                keep = true;
                if ((int)j <= limit && flt_sig(ai, a[j], mask_level)) {
                    a[j].p2 = ai.p;
                    keep = false;
                }
            }
            const uint64_t bk = __ballot(keep);
            wave_fence();
            __builtin_amdgcn_wave_barrier();
            if (keep) U[out + __builtin_popcountll(bk & ((1ull << lane) - 1))] = j;
            out += __builtin_popcountll(bk);
        }
        nu = out;
        if (jstar < 0) {
            if (lane == 0) {
                a[m] = ai;
                U[nu] = (uint32_t)m;
            }
            ++m;
            ++nu;
        }
        wave_fence();
        __builtin_amdgcn_wave_barrier();
    }
    return m;
}

// The same loop once more, in two passes (drop_ratio > 0).  Which chains are
// kept does not depend on p2: chain i is dropped by the first kept j (in
// kept order) that overlaps it significantly and may drop it, and only the
// prefix of the kept list heavy enough to drop i is searched (as in
// flt_drop_pruned).  Every i that the heaviest chain a[0] cannot drop is kept
// outright (no lighter j can drop it either): that prefix [0, I0) is settled
// in parallel, and only i >= I0 walk the kept list, one at a time, leaving
// jst[i] (the dropping kept index, -1 if kept) and the kept list's original
// positions in kidx.  Then p2: kept chain j gets the first later i whose
// scan reached it (i kept, or kpos(j) <= jst[i]) with a significant overlap
// -- the reference's first write.  Those are found 64 i at a time against
// the list U of kept chains still without one: each lane holds a kept chain
// and tests the block's 64 chains, broadcast by readlane, so the loop's
// round trips are per block, not per chain.  Last, a[0 .. m) is compacted
// from kidx (a[k] <- a[kidx[k]], kidx[k] >= k, chunk by chunk).  Same kept
// list and p2 as flt_drop_serial.
__device__ __forceinline__ bool flt_can_drop(const FltRec& ai, const FltRec& aj, float drop_ratio, int msl) {
    return (float)ai.w < (float)aj.w * drop_ratio && aj.w - ai.w >= msl << 1;
}

__device__ int flt_drop_blocked(FltRec* a, uint32_t* kidx, int32_t* jst, uint4* U, int n, float mask_level,
                                float drop_ratio, int msl, int lane, uint64_t* dbg = nullptr) {
    n = __builtin_amdgcn_readfirstlane(n);  // arguments come in VGPRs: loop bounds uniform
    // I0: the first i >= 1 that a[0] can drop
    const FltRec a0 = a[0];
    int I0 = n;
    for (int base = 1; base < n; base += 64) {
        const int i = base + lane;
        const uint64_t bc = __ballot(i < n && flt_can_drop(a[i], a0, drop_ratio, msl));
        if (bc) {
            I0 = base + (int)__builtin_ctzll(bc);
            break;
        }
    }
    I0 = __builtin_amdgcn_readfirstlane(I0);
    for (int k = lane; k < I0; k += 64) kidx[k] = (uint32_t)k;
    wave_fence();
    __builtin_amdgcn_wave_barrier();
    // the kept list's first 64 records live in registers (lane j: kept j);
    // the chains i go 64 at a time, one per lane (round 5; before, one chain
    // at a time against the kept list across the lanes: ~900 cycles a chain
    // on the giants, whose drop loops walk 8,000-10,000 chains).  A block:
    // (1) every lane walks the kept list as it stands, in order, while the
    //     kept chain can drop its chain (a prefix: the list is in weight
    //     order), to the first significant overlap -- one broadcast record a
    //     step for all lanes;
    // (2) the lanes left undecided, in order: the first is kept (it was tested
    //     against every kept chain before it), and the later undecided lanes
    //     are tested against it.
    // Same jst / kept list as the chain-at-a-time loop.
    int m = I0;
    FltRec kr{0, 0, 0, 0, -1};
    if (lane < I0) kr = a[lane];
    for (int blk = I0; blk < n; blk += 64) {
        const int i = blk + lane;
        const bool valid = i < n;
        FltRec ai{0, 0, 0, 0, -1};
        if (valid) ai = a[i];
        int jstar = -1;
        const int m0 = m;
        uint64_t srch = __ballot(valid);
        // the kept list 64 records at a time: the first 64 from the registers,
        // later tiles gathered one record a lane (one round trip a tile)
        for (int j0 = 0; srch && j0 < m0; j0 += 64) {
            FltRec tile = kr;
            if (j0) {
                const int jj = j0 + lane;
                if (jj < m0) tile = a[kidx[jj]];
            }
            const int jn = m0 - j0 < 64 ? m0 - j0 : 64;
            // flt_can_drop and flt_sig as straight-line selects (short-circuit
            // tests compiled to nested branches on exec)
            const int32_t li = ai.end - ai.beg;
            for (int jl = 0; srch && jl < jn; ++jl) {
                const int32_t bj = __builtin_amdgcn_readlane(tile.beg, jl), ej = __builtin_amdgcn_readlane(tile.end, jl);
                const int32_t wj = __builtin_amdgcn_readlane(tile.w, jl), lj = ej - bj;
                const bool on = (srch >> lane) & 1;
                const bool can = on & ((float)ai.w < (float)wj * drop_ratio) & (wj - ai.w >= msl << 1);
                const int32_t b_max = bj > ai.beg ? bj : ai.beg, e_min = ej < ai.end ? ej : ai.end;
                const int32_t min_l = li < lj ? li : lj;
                const bool hit = can & (e_min > b_max) & ((float)(e_min - b_max) >= (float)min_l * mask_level);
                jstar = hit ? j0 + jl : jstar;
                srch &= ~__ballot(on & (hit | !can));
            }
        }
        uint64_t und = __ballot(valid && jstar < 0);
        while (und) {
            const int t = (int)__builtin_ctzll(und);
            und &= und - 1;
            const FltRec at{__builtin_amdgcn_readlane(ai.beg, t), __builtin_amdgcn_readlane(ai.end, t),
                            __builtin_amdgcn_readlane(ai.w, t), blk + t, -1};
            const int km = m++;
            if (lane == 0) kidx[km] = (uint32_t)(blk + t);
            if (lane == km) kr = at;
            const bool later = (und >> lane) & 1;
            const bool hit = later && flt_can_drop(ai, at, drop_ratio, msl) && flt_sig(ai, at, mask_level);
            if (hit) jstar = km;
            und &= ~__ballot(hit);
        }
        if (valid) jst[i] = jstar;
        wave_fence();
        __builtin_amdgcn_wave_barrier();
    }
    wave_fence();
    __builtin_amdgcn_wave_barrier();
    if (dbg && lane == 0) dbg[13] = __builtin_readcyclecounter();  // SMEM_CHAIN_DBG: the kept list's end
    // p2, 64 chains i at a time
    int nu = 0, m_run = 0;
    uint32_t n_steps = 0, n_memb = 0;  // SMEM_CHAIN_DBG: p2's broadcast steps and U entries visited
    for (int b = 0; b < n; b += 64) {
        const int i = b + lane;
        int32_t bi = 0, ei = 0, ji = 0;
        bool kept = false;
        if (i < n) {
            const FltRec r = a[i];
            bi = r.beg;
            ei = r.end;
            ji = i < I0 ? -1 : jst[i];
            kept = ji < 0;
        }
        // the block's kept chains join U (they can be marked by later i of the
        // block); a U entry carries what the test needs (kept index, position,
        // query span): one load a member, not three dependent ones
        const uint64_t bk = __ballot(kept);
        const uint32_t below = (uint32_t)__builtin_popcountll(bk & ((1ull << lane) - 1));
        if (kept) U[nu + below] = make_uint4(m_run + below, (uint32_t)i, (uint32_t)bi, (uint32_t)ei);
        nu += __builtin_popcountll(bk);
        m_run += __builtin_popcountll(bk);
        wave_fence();
        __builtin_amdgcn_wave_barrier();
        const int nb = n - b < 64 ? n - b : 64;
        int out = 0;
        n_memb += (uint32_t)nu;
        for (int c = 0; c < nu; c += 64) {
            const int u = c + lane;
            const bool act = u < nu;
            uint4 ue = make_uint4(0, 0, 0, 0);
            if (act) ue = U[u];
            const uint32_t kp = ue.x, oj = ue.y;
            const FltRec rj{(int32_t)ue.z, (int32_t)ue.w, 0, 0, -1};
            int hit = -1;
            // from the first chain after the earliest searching member; done
            // when every member found its chain
            int t0 = nb;
            {
                const int st = act ? ((int)oj + 1 - b > 0 ? (int)oj + 1 - b : 0) : nb;
                t0 = st;
                for (int off = 32; off > 0; off >>= 1) {
                    const int o2 = __shfl_xor(t0, off);
                    t0 = o2 < t0 ? o2 : t0;
                }
            }
            // t0 uniform (readfirstlane): a loop on a VGPR counter compiled
            // to a divergent loop, every condition a branch on exec (~420
            // cycles a step on the giants' one wave per CU); now four steps
            // of straight-line selects at a time (independent tests, one
            // first-hit pick) -- the same test as flt_sig
            t0 = __builtin_amdgcn_readfirstlane(t0);
            const int32_t lj = rj.end - rj.beg;
            for (int t = t0; t < nb; t += 4) {
                if (!__ballot(act && hit < 0)) break;
                n_steps += (uint32_t)(nb - t < 4 ? nb - t : 4);
                int first = -1;
#pragma unroll
                for (int k = 3; k >= 0; --k) {
                    const int tk = t + k < nb ? t + k : t;  // past the block: a repeat of step t
                    const int32_t bt = __builtin_amdgcn_readlane(bi, tk), et = __builtin_amdgcn_readlane(ei, tk);
                    const int32_t jt = __builtin_amdgcn_readlane(ji, tk);
                    const int32_t jlim = jt < 0 ? INT32_MAX : jt, li = et - bt;
                    const int32_t b_max = bt > rj.beg ? bt : rj.beg, e_min = et < rj.end ? et : rj.end;
                    const int32_t min_l = li < lj ? li : lj;
                    const bool sig = (e_min > b_max) & ((float)(e_min - b_max) >= (float)min_l * mask_level);
                    const bool h = ((uint32_t)(b + tk) > oj) & ((int32_t)kp <= jlim) & sig;
                    first = h ? b + tk : first;  // k descending: the lowest hitting step wins
                }
                hit = (act & (hit < 0)) ? first : hit;
            }
            if (hit >= 0) a[oj].p2 = hit;
            const bool keep = act && hit < 0;
            const uint64_t bq = __ballot(keep);
            wave_fence();
            __builtin_amdgcn_wave_barrier();
            if (keep) U[out + __builtin_popcountll(bq & ((1ull << lane) - 1))] = ue;
            out += __builtin_popcountll(bq);
        }
        nu = out;
        wave_fence();
        __builtin_amdgcn_wave_barrier();
    }
    if (dbg && lane == 0) dbg[30] = n_steps, dbg[31] = n_memb;
    // compact the kept records (with their p2) to a[0 .. m): kidx[k] >= k, so
    // a chunk's loads never read a slot an earlier chunk stored, and its own
    // stores wait for its loads (their data); a kept prefix stays in place
    // (the heaviest chain drops nothing of it: a whole all-kept read moves nothing)
    for (int base = I0 & ~63; base < m; base += 64) {
        const int k = base + lane;
        const uint32_t src = k < m ? kidx[k] : (uint32_t)k;
        if (__ballot(src != (uint32_t)k) == 0) continue;
        FltRec r{};
        if (src != (uint32_t)k) r = a[src];
        if (src != (uint32_t)k) a[k] = r;
    }
    wave_fence();
    __builtin_amdgcn_wave_barrier();
    return m;
}

// weights + sort + reorder of mem_chain_flt (software/bwamem.c:636-651) by
// one lane; ord holds the tree order, ord2 receives the sorted order; stk:
// the sort's 64-entry stack (192 words)
__device__ __forceinline__ void flt_prepare_serial(const ChainParams& P, uint64_t S, FltRec* a, const uint32_t* ord,
                                                   uint32_t* ord2, int n, uint32_t* stk) {
    const ChainRec* chn = P.chn + S;
    for (int i = 0; i < n; ++i) {
        const ChainRec c = chn[ord[i]];
        a[i] = FltRec{c.first_qbeg, c.last_qbeg + c.last_len, chain_weight(c, P.seed + S, P.next + S), i, -1};
    }
    flt_sort(a, (uint32_t)n, stk);
    for (int i = 0; i < n; ++i) {
        ord2[i] = ord[a[i].p];
        a[i].p = i;
    }
}

// chains kept by mark + squeeze (software/bwamem.c:665-688): flags in ord
// (free by now), kept order compacted in ord2; returns the count
__device__ __forceinline__ int flt_squeeze_serial(const FltRec* a, int m, uint32_t* ord, uint32_t* ord2, int n) {
    for (int i = 0; i < n; ++i) ord[i] = 0;
    for (int i = 0; i < m; ++i) {
        ord[a[i].p] = 1;
        if (a[i].p2 >= 0) ord[a[i].p2] = 1;
    }
    int k = 0;
    for (int i = 0; i < n; ++i)
        if (ord[i]) ord2[k++] = ord2[i];
    return k;
}

__device__ __forceinline__ uint64_t seeds_in(const ChainParams& P, uint64_t S, const uint32_t* ord2, int n_keep) {
    uint64_t ns = 0;
    for (int i = 0; i < n_keep; ++i) ns += (uint64_t)P.chn[S + ord2[i]].n;
    return ns;
}

constexpr int ACT_NONE = 0, ACT_APPEND = 1, ACT_NEW = 2;

__device__ __forceinline__ int rl32(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint32_t rlu(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
__device__ __forceinline__ int64_t rl64(int64_t v, int l) {
    const uint32_t lo = rlu((uint32_t)(uint64_t)v, l), hi = rlu((uint32_t)((uint64_t)v >> 32), l);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
// kb_putp by a whole wave (same result as tree_insert): lane i handles key
// slot i of a node -- one LDS round per node search, parallel shifts and
// split copies
template <class N>
__device__ __forceinline__ int node_find_wave(const N* x, int64_t k, int lane, bool& eq) {
    const int n = x->n;
    const int64_t kv = lane < BT_MAX ? x->key[lane] : INT64_MAX;
    const int below = __builtin_popcountll(__ballot(lane < n && kv < k));
    eq = __ballot(lane == below && lane < n && kv == k) != 0;
    return eq ? below : below - 1;
}

template <class N>
__device__ __forceinline__ void node_split_wave(N* pool, uint32_t xi, int i, uint32_t yi, uint32_t& n_nodes,
                                                int lane) {
    N* x = pool + xi;
    N* y = pool + yi;
    const uint32_t zi = n_nodes++;
    N* z = pool + zi;
    const int leaf = y->leaf;
    const int n = x->n;
    // reads first (all lanes), then writes
    int64_t zk = 0, xk = 0;
    uint32_t zid = 0, zc = 0, xid = 0, xc = 0;
    if (lane < BT_T - 1) {
        zk = y->key[BT_T + lane];
        zid = y->id[BT_T + lane];
    }
    if (!leaf && lane < BT_T) zc = y->child[BT_T + lane];
    if (lane >= i + 1 && lane <= n) xc = x->child[lane];
    if (lane >= i && lane < n) {
        xk = x->key[lane];
        xid = x->id[lane];
    }
    const int64_t mk = y->key[BT_T - 1];
    const uint32_t mid = y->id[BT_T - 1];
    __builtin_amdgcn_wave_barrier();
    if (lane < BT_T - 1) {
        z->key[lane] = zk;
        z->id[lane] = zid;
    }
    if (!leaf && lane < BT_T) z->child[lane] = zc;
    if (lane >= i + 1 && lane <= n) x->child[lane + 1] = xc;
    if (lane >= i && lane < n) {
        x->key[lane + 1] = xk;
        x->id[lane + 1] = xid;
    }
    if (lane == 0) {
        z->n = BT_T - 1;
        z->leaf = leaf;
        y->n = BT_T - 1;
        x->child[i + 1] = zi;
        x->key[i] = mk;
        x->id[i] = mid;
        x->n = n + 1;
    }
    wave_fence();  // other lanes read these next (HBM pool too)
    __builtin_amdgcn_wave_barrier();
}

// one node into the wave, one LDS round: lane l holds key / id slot l and
// child slot l; n and leaf wave-uniform
template <class N>
__device__ __forceinline__ void node_load_wave(const N* nd, int lane, int& n, int& leaf, int64_t& kv, uint32_t& idv,
                                               uint32_t& chv) {
    const int n0 = nd->n, l0 = nd->leaf;
    kv = lane < BT_MAX ? nd->key[lane] : INT64_MAX;
    idv = lane < BT_MAX ? (uint32_t)nd->id[lane] : 0u;
    chv = lane <= BT_MAX ? (uint32_t)nd->child[lane] : 0u;
    n = __builtin_amdgcn_readfirstlane(n0);
    leaf = __builtin_amdgcn_readfirstlane(l0);
}

// __kb_getp_aux on a loaded node: the slot index (eq: the leftmost equal key)
__device__ __forceinline__ int node_find_regs(int n, int64_t kv, int64_t k, int lane, bool& eq) {
    const int below = __builtin_popcountll(__ballot(lane < n && kv < k));
    eq = __ballot(lane == below && lane < n && kv == k) != 0;
    return eq ? below : below - 1;
}

// kb_putp by the wave: a node per LDS round on the way down (plus its
// child's fill, for the pre-emptive split), the leaf's shift from registers
template <class N>
__device__ __forceinline__ void tree_insert_wave(N* pool, uint32_t& root, uint32_t& n_nodes, uint32_t id, int64_t k,
                                                 int lane) {
    uint32_t x = root;
    bool eq;
    if (pool[x].n == BT_MAX) {
        const uint32_t s = n_nodes++;
        if (lane == 0) {
            node_init(pool + s, 0);
            pool[s].child[0] = x;
        }
        wave_fence();
        __builtin_amdgcn_wave_barrier();
        node_split_wave(pool, s, 0, x, n_nodes, lane);
        root = x = s;
    }
    for (;;) {
        int n, leaf;
        int64_t kv;
        uint32_t idv, chv;
        node_load_wave(pool + x, lane, n, leaf, kv, idv, chv);
        if (leaf) {
            N* nd = pool + x;
            const int i = node_find_regs(n, kv, k, lane, eq);
            if (lane >= i + 1 && lane < n) {
                nd->key[lane + 1] = kv;
                nd->id[lane + 1] = idv;
            }
            if (lane == 0) {
                nd->key[i + 1] = k;
                nd->id[i + 1] = id;
                nd->n = n + 1;
            }
            wave_fence();
            __builtin_amdgcn_wave_barrier();
            return;
        }
        int i = node_find_regs(n, kv, k, lane, eq) + 1;
        uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)chv, i);
        if (__builtin_amdgcn_readfirstlane((int)pool[c].n) == BT_MAX) {
            node_split_wave(pool, x, i, c, n_nodes, lane);
            if (k > pool[x].key[i]) ++i;
            c = (uint32_t)__builtin_amdgcn_readfirstlane((int)pool[x].child[i]);
        }
        x = c;
    }
}

// Wave form of the same loop for one read, exact by construction: a window
// of 64 seeds, one per lane, whose tree lookups and chain-record loads run
// in parallel against the chains as they stood before the window, then a
// scan over the window's seeds in order in which the whole wave decides each
// seed from registers: its lower chain is the snapshot's unless a chain
// created earlier in the window has a pos in between, and a chain's state
// is the snapshot's unless an earlier seed of the window changed it (both
// found from lane masks).  Where the real tree could answer differently --
// equal keys: a window chain tying the lower chain or another window chain,
// or a lower chain whose pos is duplicated in the tree once the window has
// created chains -- the scan stops and the next window starts at that seed,
// whose snapshot lookup is then exact.  Chain records and links are
// committed per window, the window's new chains inserted in seed order.
// Returns false when the node pool cannot take a window's new chains; `o`
// then names the first seed not yet applied.
template <class N>
__device__ __forceinline__ bool insert_read_wave(const ChainParams& P, uint64_t S, uint64_t E, N* pool, uint32_t cap,
                                                 uint64_t& o, uint32_t& n_ch, uint32_t& root, uint32_t& n_nodes,
                                                 int lane, int64_t* dups, int& n_dup, uint64_t* dbg) {
    ChainRec* chn = P.chn + S;
    uint64_t t_look = 0, t_scan = 0, t_commit = 0, n_win = 0, t0, t1;
    while (o < E) {
        t0 = __builtin_readcyclecounter();
        ++n_win;
        const uint64_t so = o + (uint64_t)lane;
        const int n_live = E - o < 64 ? (int)(E - o) : 64;
        const bool live = lane < n_live;
        SeedRec sd{0, 0, 0};
        if (live) sd = P.seed[so];
        const int64_t rb = sd.rbeg;
        const bool skip = !live || (rb < P.l_pac && P.l_pac < rb + sd.len);
        const uint64_t skm = __ballot(skip);
        int lw0 = -1;
        if (!skip && n_ch) lw0 = tree_lower(pool, root, rb);
        ChainRec c0{};
        if (lw0 >= 0) c0 = chn[lw0];
        // pot: earlier seeds of the window whose pos would sit between my
        // snapshot lower chain and me, were they to start chains
        uint64_t pot = 0;
        for (int t = 0; t < n_live; ++t) {
            if ((skm >> t) & 1) continue;
            const int64_t rt = rl64(rb, t);
            if (t < lane && rt <= rb && (lw0 < 0 || rt >= c0.pos)) pot |= 1ull << t;
        }
        t1 = __builtin_readcyclecounter();
        t_look += t1 - t0;
        t0 = t1;
        // window slots, filled by the scan
        int m_id = -1;
        ChainRec ms{};
        uint32_t m_prev = 0;
        uint64_t new_mask = 0, app_mask = 0;
        int n_done = n_live;
        for (int s = 0; s < n_live; ++s) {
            if ((skm >> s) & 1) continue;
            const int64_t rbs = rl64(rb, s);
            const int32_t qs = rl32(sd.qbeg, s), ls = rl32(sd.len, s);
            const int lw0s = rl32(lw0, s);
            const int64_t v0 = rl64(c0.pos, s);
            const uint64_t pm = (uint64_t)rl64((int64_t)pot, s) & new_mask;
            int low = lw0s;
            bool from_window = false;
            if (pm) {
                int64_t best = INT64_MIN;
                int bt = -1, ties = 0;
                for (uint64_t m = pm; m; m &= m - 1) {
                    const int t = __builtin_ctzll(m);
                    const int64_t r = rl64(rb, t);
                    if (r > best) {
                        best = r;
                        bt = t;
                        ties = 1;
                    } else if (r == best) {
                        ++ties;
                    }
                }
                if ((lw0s >= 0 && best == v0) || ties > 1) {
                    n_done = s;
                    break;
                }
                low = rl32(m_id, bt);
                from_window = true;
            } else if (lw0s >= 0 && new_mask && n_dup != 0) {
                // the snapshot's answer among duplicate keys may move once
                // window chains are in the tree
                bool dup = n_dup < 0;
                for (int j = lane; !dup && j < n_dup; j += 64) dup = dups[j] == v0;
                if (__ballot(dup)) {
                    n_done = s;
                    break;
                }
            }
            int act = ACT_NEW;
            ChainRec c{};
            if (low >= 0) {
                // the lower chain's state: its last change in the window, else the snapshot's
                const uint64_t chm = __ballot(m_id == low) & ((1ull << s) - 1) & (new_mask | app_mask);
                if (chm) {
                    const int t = 63 - __builtin_clzll(chm);
                    c.pos = rl64(ms.pos, t);
                    c.last_rbeg = rl64(ms.last_rbeg, t);
                    c.first_qbeg = rl32(ms.first_qbeg, t);
                    c.last_qbeg = rl32(ms.last_qbeg, t);
                    c.last_len = rl32(ms.last_len, t);
                    c.n = rl32(ms.n, t);
                    c.first = rlu(ms.first, t);
                    c.last = rlu(ms.last, t);
                } else {
                    c.pos = v0;
                    c.last_rbeg = rl64(c0.last_rbeg, s);
                    c.first_qbeg = rl32(c0.first_qbeg, s);
                    c.last_qbeg = rl32(c0.last_qbeg, s);
                    c.last_len = rl32(c0.last_len, s);
                    c.n = rl32(c0.n, s);
                    c.first = rlu(c0.first, s);
                    c.last = rlu(c0.last, s);
                }
                (void)from_window;
                // test_and_merge (software/bwamem.c:334-354)
                if (qs >= c.first_qbeg && qs + ls <= c.last_qbeg + c.last_len && rbs >= c.pos &&
                    rbs + ls <= c.last_rbeg + c.last_len) {
                    act = ACT_NONE;
                } else {
                    const bool strand_ok = !((c.last_rbeg < P.l_pac || c.pos < P.l_pac) && rbs >= P.l_pac);
                    const int64_t x = (int64_t)qs - c.last_qbeg, y = rbs - c.last_rbeg;
                    if (strand_ok && y >= 0 && x - y <= P.w && y - x <= P.w && x - c.last_len < P.max_chain_gap &&
                        y - c.last_len < P.max_chain_gap)
                        act = ACT_APPEND;
                }
            }
            const uint32_t me = (uint32_t)(o + (uint64_t)s - S);
            if (act == ACT_APPEND) {
                if (lane == s) {
                    m_id = low;
                    ms = c;
                    m_prev = c.last;
                    ms.last = me;
                    ms.last_rbeg = rbs;
                    ms.last_qbeg = qs;
                    ms.last_len = ls;
                    ms.n = c.n + 1;
                }
                app_mask |= 1ull << s;
            } else if (act == ACT_NEW) {
                if (lane == s) {
                    m_id = (int)(n_ch + (uint32_t)__builtin_popcountll(new_mask));
                    ms.pos = rbs;
                    ms.last_rbeg = rbs;
                    ms.first_qbeg = qs;
                    ms.last_qbeg = qs;
                    ms.last_len = ls;
                    ms.n = 1;
                    ms.first = ms.last = me;
                }
                // a key equal to the lower chain's: the tree holds it twice from now on
                if (low >= 0 && c.pos == rbs) {
                    if (lane == 0 && n_dup >= 0 && n_dup < 256) dups[n_dup] = rbs;
                    n_dup = (n_dup >= 0 && n_dup < 256) ? n_dup + 1 : -1;
                }
                new_mask |= 1ull << s;
            }
        }
        t1 = __builtin_readcyclecounter();
        t_scan += t1 - t0;
        t0 = t1;
        // commit seeds [0, n_done) of the window
        const uint64_t done_mask = n_done >= 64 ? ~0ull : ((1ull << n_done) - 1);
        const uint64_t nm = new_mask & done_mask, am = app_mask & done_mask;
        const int k_new = __builtin_popcountll(nm);
        if (k_new && (n_nodes + 24u * (uint32_t)k_new > cap || n_ch + (uint32_t)k_new >= N::MAX_ID)) return false;
        // chain records: each modified chain's last state in the window
        const uint64_t mod = nm | am;
        bool final_state = ((mod >> lane) & 1) != 0;
        for (uint64_t m = mod; m; m &= m - 1) {
            const int u = __builtin_ctzll(m);
            const int idu = rl32(m_id, u);
            if (lane < u && m_id == idu) final_state = false;
        }
        if (final_state) chn[m_id] = ms;
        if ((am >> lane) & 1) P.next[S + m_prev] = (uint32_t)(so - S);
        uint32_t id = n_ch;
        for (uint64_t m = nm; m; m &= m - 1) {
            const int t = __builtin_ctzll(m);
            tree_insert_wave(pool, root, n_nodes, id++, rl64(rb, t), lane);
        }
        n_ch += (uint32_t)k_new;
        o += (uint64_t)n_done;
        __syncthreads();  // this window's stores before the next window's loads
        t_commit += __builtin_readcyclecounter() - t0;
    }
    if (dbg && lane == 0) {
        dbg[10] += n_win;
        dbg[11] += t_look;
        dbg[12] += t_scan;
        dbg[13] += t_commit;
    }
    return true;
}

// ---------------------------------------------------------------------------
// Heavy reads by position clusters.  Sort the read's seeds by rbeg; cut the
// sorted list where two neighbours are G = max(max_chain_gap, 1) + the
// longest seed apart or more.  A chain's consecutive seeds are less than G
// apart (test_and_merge appends only when y - last_len < max_chain_gap,
// contains only when rb + len <= last_rbeg + last_len), so every chain lies
// in one cluster, and a seed whose lower chain (kb_intervalp) lies in an
// earlier cluster is at least G past that chain's last seed: test_and_merge
// fails and the seed starts a chain -- what it does with no lower chain.  So
// each cluster runs mem_insert_seed's loop on its own seeds, in their order,
// against its own chains: the lower chain is the cluster's chain with the
// largest pos <= rb.  That is the tree's answer while no two chains share a
// pos; a cluster that creates an equal pos (kbtree's answer then depends on
// the node layout) sends the read back to the tree path.  With distinct keys
// the in-order traversal is pos order: clusters in order, pos order inside.
// One lane runs one cluster (64 per round).  Its chains are marks on the
// ranks of their first seeds in rbeg order (a bitmap + summary in LDS after
// the keys): the lower chain of a seed is the highest mark below the seed's
// own rank -- among equal rbeg, ranks follow seed order, so that is the
// chain with the largest pos <= rb, the latest one on a tie -- found in one
// or two LDS reads, and a new chain is one mark, where a sorted chain list
// took a binary search and a shift per seed (quadratic in giant clusters).
// ---------------------------------------------------------------------------
constexpr int CL_OBITS = 20;  // seed index bits in the sort keys
constexpr uint64_t CL_OMASK = (1ull << CL_OBITS) - 1;

// One bitonic stage (k, j) over npad keys: a lane's pairs of a stage are
// independent, so their loads go out BB at a time under one LDS wait (one
// pair per round trip left the giants' cluster pass waiting on LDS: 105
// stages x 128 round trips per 16k-key sort).
template <int BB, class T>
__device__ __forceinline__ void bitonic_stage(T* key, uint32_t npad, uint32_t k, uint32_t j, int lane) {
    const uint32_t np = npad >> 1;
    for (uint32_t t0 = 0; t0 < np; t0 += 64 * BB) {
        T a[BB], b[BB];
        uint32_t ii[BB];
#pragma unroll
        for (int q = 0; q < BB; ++q) {
            const uint32_t t = t0 + (uint32_t)(q * 64 + lane);
            ii[q] = 2 * t - (t & (j - 1));
            if (t < np) {
                a[q] = key[ii[q]];
                b[q] = key[ii[q] + j];
            }
        }
#pragma unroll
        for (int q = 0; q < BB; ++q) {
            const uint32_t t = t0 + (uint32_t)(q * 64 + lane);
            const bool up = (ii[q] & k) == 0;
            if (t < np && (a[q] > b[q]) == up) {
                key[ii[q]] = b[q];
                key[ii[q] + j] = a[q];
            }
        }
    }
}

__device__ __forceinline__ void wave_bitonic(uint64_t* key, uint32_t npad, int lane) {
    for (uint32_t k = 2; k <= npad; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            if (npad >= 64 * 2 * 8) bitonic_stage<8>(key, npad, k, j, lane);
            else bitonic_stage<1>(key, npad, k, j, lane);
            wave_fence();
            __builtin_amdgcn_wave_barrier();
        }
    }
}

__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, int lane, uint32_t& total) {
    uint32_t incl = v;
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t t = __shfl_up(incl, off, 64);
        if (lane >= off) incl += t;
    }
    total = __shfl(incl, 63, 64);
    return incl - v;
}

constexpr uint32_t CODE_SKIP = 0, CODE_NEW = 1, CODE_REPLAY = 2;
constexpr int MERGE_NEW = 0, MERGE_CONTAINED = 1, MERGE_APPEND = 2;

// test_and_merge (software/bwamem.c:334-354) of seed (rb, qb, ln) against chain c
__device__ __forceinline__ int merge_test(const ChainParams& P, const ChainRec& c, int64_t rb, int32_t qb,
                                          int32_t ln) {
    if (qb >= c.first_qbeg && qb + ln <= c.last_qbeg + c.last_len && rb >= c.pos &&
        rb + ln <= c.last_rbeg + c.last_len)
        return MERGE_CONTAINED;
    const bool strand_ok = !((c.last_rbeg < P.l_pac || c.pos < P.l_pac) && rb >= P.l_pac);
    const int64_t x = (int64_t)qb - c.last_qbeg, y = rb - c.last_rbeg;
    if (strand_ok && y >= 0 && x - y <= P.w && y - x <= P.w && x - c.last_len < P.max_chain_gap &&
        y - c.last_len < P.max_chain_gap)
        return MERGE_APPEND;
    return MERGE_NEW;
}

__device__ __forceinline__ void chain_append(ChainRec& c, uint32_t o, int64_t rb, int32_t qb, int32_t ln) {
    c.last = o;
    c.last_rbeg = rb;
    c.last_qbeg = qb;
    c.last_len = ln;
    c.n += 1;
}

// The chains of a cluster as marks on the ranks of their first seeds (the
// read's seeds sorted by rbeg): bm holds one bit per rank, sm one bit per
// non-empty bm word.  Lanes mark disjoint rank ranges whose end words may be
// shared, hence the LDS atomics.
__device__ __forceinline__ uint32_t cluster_bm_words(uint32_t npad) { return (npad + 31) / 32; }
__device__ __host__ __forceinline__ uint64_t cluster_lds_need(uint64_t npad) {
    const uint64_t nbw = (npad + 31) / 32;
    return npad * 8 + 4 * (nbw + (nbw + 31) / 32);
}

__device__ __forceinline__ void mark_set(uint32_t* bm, uint32_t* sm, uint32_t q) {
    atomicOr(bm + (q >> 5), 1u << (q & 31));
    atomicOr(sm + (q >> 10), 1u << ((q >> 5) & 31));
}

// the highest marked rank in [cs, r), -1 if none
__device__ __forceinline__ int mark_pred(const uint32_t* bm, const uint32_t* sm, uint32_t cs, uint32_t r) {
    if (r <= cs) return -1;
    const uint32_t wlo = cs >> 5;
    uint32_t w = (r - 1) >> 5;
    uint32_t bits = bm[w] & (0xffffffffu >> (31 - ((r - 1) & 31)));
    for (;;) {
        if (w == wlo) bits &= ~0u << (cs & 31);
        if (bits) return (int)(w * 32 + 31 - __builtin_clz(bits));
        if (w == wlo) return -1;
        --w;  // the next lower non-empty word, from the summary
        uint32_t sw = w >> 5;
        uint32_t sb = sm[sw] & (0xffffffffu >> (31 - (w & 31)));
        while (!sb) {
            if ((sw << 5) <= wlo) return -1;
            --sw;
            sb = sm[sw];
        }
        w = sw * 32 + 31 - __builtin_clz(sb);
        if (w < wlo) return -1;
        bits = bm[w];
    }
}

// A big cluster's pass by the whole wave (round 5): the lane-per-cluster loop
// left one lane walking a cluster of thousands of seeds (the human-like
// profile's satellite reads: 8,500 seeds, 8,500 chains, 7-13 M cycles on one
// lane).  Optimistic batches of 64 seeds in seed order: assume every seed of
// the batch starts a chain; then a seed's lower chain (kb_intervalp) is the
// higher of the last committed mark below its rank (mark_pred) and the
// highest rank below it among the batch's earlier seeds, every lane tests its
// merge at once (test_and_merge, software/bwamem.c:334-354), and the seeds
// before the first one that does not start a clean chain (it merges, is
// contained, or makes an equal chain key) are exactly what the serial loop
// would have done: they are committed together.  That first seed is applied
// as the serial loop applies it, and the next batch starts after it.  A
// tandem-repeat cluster (several seeds per chain) advances a few seeds per
// batch, a satellite cluster (a chain per seed) 64.  Returns true when the
// cluster made an equal chain key (its later seeds are CODE_REPLAY).
__device__ __forceinline__ bool cluster_wave(const ChainParams& P, uint64_t S, uint64_t* key, uint32_t* bm, uint32_t* sm, uint32_t cs,
                             uint32_t ce, ChainRec* chn, const SeedRec* seed, uint32_t* code, int lane,
                             uint32_t& n_mine) {
    uint32_t pb = cs;
    bool cdup = false;
    // batch size: halved while batches end early (a cluster whose seeds merge
    // often: its lower-chain records are a round trip per batch), doubled
    // back while they commit at least half
    uint32_t nbmax = 64;
    while (pb < ce && !cdup) {
        const uint32_t p = pb + (uint32_t)lane;
        const bool valid = p < ce && (uint32_t)lane < nbmax;
        uint64_t e = 0;
        SeedRec sd{0, 0, 0};
        uint32_t o = 0, rk = 0;
        int A = -1;
        if (valid) {
            e = key[p];
            o = (uint32_t)(e >> CL_OBITS) & (uint32_t)CL_OMASK;
            rk = (uint32_t)e & (uint32_t)CL_OMASK;
            sd = seed[o];
            A = mark_pred(bm, sm, cs, rk);  // committed marks only
        }
        const uint32_t nb = (uint32_t)__popcll(__ballot(valid));
        // the highest rank below mine among the batch's earlier seeds
        int B = -1, Bl = -1;
        for (uint32_t t = 0; t + 1 < nb; ++t) {
            const int rt = __builtin_amdgcn_readlane((int)rk, (int)t);
            if ((uint32_t)lane > t && rt < (int)rk && rt > B) {
                B = rt;
                Bl = (int)t;
            }
        }
        // the batch chain's record is its first seed's, from that lane
        const int bl4 = (Bl < 0 ? 0 : Bl) << 2;
        const int64_t brb = (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(bl4, (int)(uint32_t)sd.rbeg) |
                                      (uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(bl4, (int)((uint64_t)sd.rbeg >> 32))
                                          << 32);
        const int32_t bqb = __builtin_amdgcn_ds_bpermute(bl4, sd.qbeg), bln = __builtin_amdgcn_ds_bpermute(bl4, sd.len);
        const uint32_t bo = (uint32_t)__builtin_amdgcn_ds_bpermute(bl4, (int)o);
        ChainRec c{};
        uint32_t id = 0;
        int mg = MERGE_NEW;
        const bool has_lower = valid && (A >= 0 || B >= 0);
        if (valid && B > A) {
            c = ChainRec{brb, brb, bqb, bqb, bln, 1, bo, bo};
            id = bo;
        } else if (valid && A >= 0) {
            id = (uint32_t)(key[A] >> (2 * CL_OBITS));
            c = chn[id];
        }
        if (has_lower) mg = merge_test(P, c, sd.rbeg, sd.qbeg, sd.len);
        const bool clean = mg == MERGE_NEW && !(has_lower && c.pos == sd.rbeg);
        const uint64_t bad = __ballot(valid && !clean);
        const uint32_t first = bad ? (uint32_t)__builtin_ctzll(bad) : nb;
        if (valid && (uint32_t)lane < first) {  // starts a chain, as the serial loop would have it
            chn[o] = ChainRec{sd.rbeg, sd.rbeg, sd.qbeg, sd.qbeg, sd.len, 1, o, o};
            code[o] = CODE_NEW;
            mark_set(bm, sm, rk);
        }
        n_mine += (uint32_t)lane < first && valid ? 1u : 0u;
        wave_fence();
        __builtin_amdgcn_wave_barrier();
        if (first < nb) {  // the serial loop's step for that seed
            if ((uint32_t)lane == first) {
                if (mg == MERGE_APPEND) {
                    P.next[S + c.last] = o;
                    chain_append(c, o, sd.rbeg, sd.qbeg, sd.len);
                    chn[id] = c;
                    code[o] = CODE_SKIP;
                } else if (mg == MERGE_CONTAINED) {
                    code[o] = CODE_SKIP;
                } else {  // an equal chain key: it starts a chain, unmarked; the replay decides the rest
                    chn[o] = ChainRec{sd.rbeg, sd.rbeg, sd.qbeg, sd.qbeg, sd.len, 1, o, o};
                    code[o] = CODE_NEW;
                    ++n_mine;
                }
            }
            cdup = __builtin_amdgcn_readlane(mg == MERGE_NEW ? 1 : 0, (int)first) != 0;  // lane `first`'s
            wave_fence();
            __builtin_amdgcn_wave_barrier();
        }
        pb += first < nb ? first + 1 : nb;  // the committed seeds, and the one handled after them
        nbmax = first >= nbmax / 2 ? (nbmax < 64 ? 2 * nbmax : 64u) : (nbmax > 8 ? nbmax / 2 : 8u);
    }
    if (cdup) {  // past the equal chain key: the tree replay decides
        for (uint32_t p = pb + (uint32_t)lane; p < ce; p += 64) {
            code[(uint32_t)(key[p] >> CL_OBITS) & (uint32_t)CL_OMASK] = CODE_REPLAY;
            ++n_mine;
        }
    }
    return cdup;
}

// true: chains built, tree order in ord[0, n_out); false: a cluster made an
// equal chain key and the tree replay must finish the read.  Chain ids are
// the index of the chain's first seed.  code[o] records, per seed, what the
// replay does with it: CODE_NEW (this seed starts a chain: kb_putp it),
// CODE_REPLAY (a seed of a cluster past its first equal key), or CODE_SKIP;
// n_cand counts the first two.
__device__ __forceinline__ bool insert_read_clusters(const ChainParams& P, uint64_t S, uint64_t E, uint64_t* key, int lane,
                                     int& n_out, uint32_t& n_cand) {
    const uint32_t N = (uint32_t)(E - S);
    uint32_t npad = 2;
    while (npad < N) npad <<= 1;
    ChainRec* chn = P.chn + S;
    const SeedRec* seed = P.seed + S;
    uint32_t* ord = P.ord + S;
    uint32_t* cstart = P.ord2 + S;  // free until the filter's reorder
    uint32_t* code = reinterpret_cast<uint32_t*>(P.flt + S);  // free until the filter
    // keys (rb, o); seeds bridging the strands sort last and are not used
    int32_t lmax = 0;
    for (uint32_t o = lane; o < npad; o += 64) {
        uint64_t k = ~0ull;
        if (o < N) {
            const SeedRec sd = seed[o];
            if (!(sd.rbeg < P.l_pac && P.l_pac < sd.rbeg + sd.len)) {
                k = ((uint64_t)sd.rbeg << CL_OBITS) | o;
                lmax = sd.len > lmax ? sd.len : lmax;
            } else {
                code[o] = CODE_SKIP;
            }
        }
        key[o] = k;
    }
    for (int off = 32; off > 0; off >>= 1) {
        const int32_t t = __shfl_xor(lmax, off);
        lmax = t > lmax ? t : lmax;
    }
    wave_fence();
    __builtin_amdgcn_wave_barrier();
    wave_bitonic(key, npad, lane);
    const int64_t G = (int64_t)(P.max_chain_gap > 1 ? P.max_chain_gap : 1) + lmax;
    // clusters: heads where the gap to the previous seed is >= G; second
    // keys (cluster, o) in place; cluster starts to cstart
    uint32_t n_valid = 0, n_cl = 0;
    uint64_t carry = 0;  // the previous chunk's last key, before it was rewritten
    for (uint32_t base = 0; base < N; base += 64) {
        const uint32_t p = base + lane;
        uint64_t k = 0;
        bool valid = false;
        if (p < N) {
            k = key[p];
            valid = k != ~0ull;
        }
        uint64_t kp = __shfl_up(k, 1, 64);
        if (lane == 0) kp = carry;
        carry = __shfl(k, 63, 64);
        const bool head = valid && (p == 0 || (int64_t)(k >> CL_OBITS) - (int64_t)(kp >> CL_OBITS) >= G);
        const uint64_t hm = __ballot(head);
        const uint32_t cid = n_cl + (uint32_t)__builtin_popcountll(hm & ((2ull << lane) - 1)) - 1;
        wave_fence();
        __builtin_amdgcn_wave_barrier();
        if (valid) key[p] = ((uint64_t)cid << (2 * CL_OBITS)) | ((k & CL_OMASK) << CL_OBITS) | p;
        if (head) cstart[cid] = p;
        n_cl += (uint32_t)__builtin_popcountll(hm);
        n_valid += (uint32_t)__builtin_popcountll(__ballot(valid));
    }
    wave_fence();
    __builtin_amdgcn_wave_barrier();
    wave_bitonic(key, npad, lane);  // cluster order kept, seed order inside
    // key[p] = o << 20 | rank (seed order inside each cluster), and bits 40+
    // of key[rank] = the seed at that rank; the marks cleared
    const uint32_t nbw = cluster_bm_words(npad), nsw = (nbw + 31) / 32;
    uint32_t* bm = reinterpret_cast<uint32_t*>(key + npad);
    uint32_t* sm = bm + nbw;
    for (uint32_t p = lane; p < n_valid; p += 64) key[p] &= (1ull << (2 * CL_OBITS)) - 1;
    for (uint32_t w = lane; w < nbw + nsw; w += 64) bm[w] = 0;
    wave_fence();
    __builtin_amdgcn_wave_barrier();
    for (uint32_t p = lane; p < n_valid; p += 64) {
        const uint64_t e = key[p];
        atomicOr(reinterpret_cast<unsigned long long*>(key + (e & CL_OMASK)),
                 (unsigned long long)((e >> CL_OBITS) & CL_OMASK) << (2 * CL_OBITS));
    }
    wave_fence();
    __builtin_amdgcn_wave_barrier();
    bool dup = false;
    uint32_t n_mine = 0;
    for (uint32_t r0 = 0; r0 < n_cl; r0 += 64) {
        const uint32_t kc = r0 + lane;
        uint32_t cs = 0, ce = 0;
        if (kc < n_cl) {
            cs = cstart[kc];
            ce = kc + 1 < n_cl ? cstart[kc + 1] : n_valid;
        }
        if (ce - cs > P.wave_min) ce = cs;  // a big cluster: the whole wave takes it below
        bool cdup = false;
        // seed p + 1's record and its lower chain's record are loaded while
        // seed p is decided (against the marks before p); p's own mark or
        // append then corrects them from registers
        uint64_t e_n = 0;
        SeedRec sd_n{0, 0, 0};
        int L_n = -1;
        ChainRec c_n{};
        if (cs < ce) {
            e_n = key[cs];
            sd_n = seed[(uint32_t)(e_n >> CL_OBITS) & (uint32_t)CL_OMASK];
        }
        for (uint32_t p = cs; p < ce; ++p) {
            const uint64_t e = e_n;
            const uint32_t o = (uint32_t)(e >> CL_OBITS) & (uint32_t)CL_OMASK, rk = (uint32_t)e & (uint32_t)CL_OMASK;
            const SeedRec sd = sd_n;
            const int Lp = L_n;
            ChainRec cp = c_n;
            uint32_t rk_n = 0;
            if (!cdup && p + 1 < ce) {
                e_n = key[p + 1];
                const uint32_t o_n = (uint32_t)(e_n >> CL_OBITS) & (uint32_t)CL_OMASK;
                rk_n = (uint32_t)e_n & (uint32_t)CL_OMASK;
                sd_n = seed[o_n];
                L_n = mark_pred(bm, sm, cs, rk_n);
                if (L_n >= 0) c_n = chn[(uint32_t)(key[L_n] >> (2 * CL_OBITS))];
            } else if (p + 1 < ce) {
                e_n = key[p + 1];
            }
            if (cdup) {  // past an equal chain key: the tree replay decides
                code[o] = CODE_REPLAY;
                ++n_mine;
                continue;
            }
            const int64_t rb = sd.rbeg;
            // lower chain: the highest mark below the seed's rank (the first
            // seed of the cluster has none)
            const int L = p == cs ? -1 : Lp;
            bool make = true;
            uint32_t id = 0;
            ChainRec c = cp;
            if (L >= 0) {
                id = (uint32_t)(key[L] >> (2 * CL_OBITS));
                const int mg = merge_test(P, c, rb, sd.qbeg, sd.len);
                if (mg == MERGE_APPEND) {
                    P.next[S + c.last] = o;
                    chain_append(c, o, rb, sd.qbeg, sd.len);
                    chn[id] = c;
                    if (L_n == L) c_n = c;  // the prefetched record is this chain's
                }
                make = mg == MERGE_NEW;
                if (make && c.pos == rb) cdup = true;
            }
            code[o] = make ? CODE_NEW : CODE_SKIP;
            if (make) {
                const ChainRec nc{rb, rb, sd.qbeg, sd.qbeg, sd.len, 1, o, o};
                chn[o] = nc;
                ++n_mine;
                if (!cdup) {
                    mark_set(bm, sm, rk);
                    // the new mark is seed p + 1's lower chain when it lies between
                    if (p + 1 < ce && rk < rk_n && (L_n < 0 || (uint32_t)L_n < rk)) {
                        L_n = (int)rk;
                        c_n = nc;
                    }
                }
            }
        }
        dup = dup || cdup;
    }
    wave_fence();
    __builtin_amdgcn_wave_barrier();
    // the big clusters, one at a time by the whole wave
    for (uint32_t r0 = 0; r0 < n_cl; r0 += 64) {
        const uint32_t kc = r0 + lane;
        uint32_t sz = 0;
        if (kc < n_cl) sz = (kc + 1 < n_cl ? cstart[kc + 1] : n_valid) - cstart[kc];
        uint64_t big = __ballot(sz > P.wave_min);
        while (big) {
            const uint32_t k = r0 + (uint32_t)__builtin_ctzll(big);
            big &= big - 1;
            const uint32_t cs = cstart[k], ce = k + 1 < n_cl ? cstart[k + 1] : n_valid;
            if (cluster_wave(P, S, key, bm, sm, cs, ce, chn, seed, code, lane, n_mine)) dup = true;
        }
    }
    wave_fence();
    __builtin_amdgcn_wave_barrier();
    // every cluster's chains in pos order: the marks in rank order (ranks are
    // the read's seeds in rbeg order, and clusters are rank ranges in order)
    uint32_t n_tot = 0;
    for (uint32_t w0 = 0; w0 < nbw; w0 += 64) {
        const uint32_t w = w0 + lane;
        uint32_t bits = w < nbw ? bm[w] : 0u;
        if (w * 32 >= n_valid) bits = 0;
        uint32_t tot;
        uint32_t q = n_tot + wave_excl_scan((uint32_t)__builtin_popcount(bits), lane, tot);
        while (bits) {
            const uint32_t b = (uint32_t)__builtin_ctz(bits);
            bits &= bits - 1;
            ord[q++] = (uint32_t)(key[w * 32 + b] >> (2 * CL_OBITS));
        }
        n_tot += tot;
    }
    n_out = (int)n_tot;
    for (int off = 32; off > 0; off >>= 1) n_mine += __shfl_xor(n_mine, off);
    n_cand = n_mine;
    return __ballot(dup) == 0;
}

// kb_intervalp's `lower` by a whole wave (as tree_lower): one LDS round per
// node; every value the descent branches on is wave-uniform
// What a search leaves for a kb_putp of the same key: the leaf it reached
// and that leaf's slots, valid (ok) when no node on the path was full (so
// kb_putp would split nothing and descend the same way) and the search did
// not stop at an equal key above the leaf.
struct LeafHand {
    bool ok;
    uint32_t x;
    int n;
    int64_t kv;
    uint32_t idv;
};

template <class N>
__device__ __forceinline__ int tree_lower_wave(const N* pool, uint32_t root, int64_t k, int lane,
                                               LeafHand* hand = nullptr, int64_t* lkey = nullptr) {
    uint32_t x = root;
    int lower = -1;
    bool full = false;
    if (hand) hand->ok = false;
    for (;;) {
        int n, leaf;
        int64_t kv;
        uint32_t idv, chv;
        node_load_wave(pool + x, lane, n, leaf, kv, idv, chv);
        full = full || n == BT_MAX;
        bool eq;
        const int i = node_find_regs(n, kv, k, lane, eq);
        if (i >= 0) {
            lower = __builtin_amdgcn_readlane((int)idv, i);
            if (lkey) *lkey = rl64(kv, i);  // the lower chain's key: its pos
        }
        if (i >= 0 && eq && !leaf) return lower;
        if (leaf) {
            if (hand) *hand = LeafHand{!full, x, n, kv, idv};
            return lower;
        }
        x = (uint32_t)__builtin_amdgcn_readlane((int)chv, i + 1);
    }
}

// kb_putp of key k into the leaf a search handed over (LeafHand::ok): the
// leaf's shift and the new slot from registers, no descent
template <class N>
__device__ __forceinline__ void leaf_insert_hand(N* pool, const LeafHand& h, uint32_t id, int64_t k, int lane) {
    N* nd = pool + h.x;
    bool eq;
    const int i = node_find_regs(h.n, h.kv, k, lane, eq);
    if (lane >= i + 1 && lane < h.n) {
        nd->key[lane + 1] = h.kv;
        nd->id[lane + 1] = h.idv;
    }
    if (lane == 0) {
        nd->key[i + 1] = k;
        nd->id[i + 1] = id;
        nd->n = h.n + 1;
    }
    wave_fence();
    __builtin_amdgcn_wave_barrier();
}

// __kb_traverse (as tree_inorder) by the wave, for the heavy path: the
// stack of (node, next child) lives in the lanes (lane d: depth d, read by
// readlane, written by a lane select), a node is one LDS round, and a leaf's
// ids go out in one store.  tree_inorder keeps its stack in scratch: a
// lane-serial walk of a several-thousand-chain tree waited on a scratch
// round trip per step, most of the kbtree replay's time.
template <class N>
__device__ __forceinline__ int tree_inorder_wave(const N* pool, uint32_t root, uint32_t* out, int lane) {
    int sxv = lane == 0 ? (int)root : 0, siv = 0;
    int top = 0, n_out = 0;
    while (top >= 0) {
        const uint32_t x = (uint32_t)__builtin_amdgcn_readlane(sxv, top);
        const int i = __builtin_amdgcn_readlane(siv, top);
        int n, leaf;
        int64_t kv;
        uint32_t idv, chv;
        node_load_wave(pool + x, lane, n, leaf, kv, idv, chv);
        (void)kv;
        if (leaf) {
            if (lane < n) out[n_out + lane] = idv;
            n_out += n;
            --top;
            continue;
        }
        // back from child i - 1: its key; then child i, or up
        if (i > 0 && i - 1 < n) {
            if (lane == 0) out[n_out] = (uint32_t)__builtin_amdgcn_readlane((int)idv, i - 1);
            ++n_out;
        }
        if (i <= n) {
            if (lane == top) siv = i + 1;
            ++top;
            const int c = __builtin_amdgcn_readlane((int)chv, i);
            if (lane == top) {
                sxv = c;
                siv = 0;
            }
        } else {
            --top;
        }
    }
    return n_out;
}

// The kbtree pass of a read whose clusters made an equal chain key: which of
// two equal keys kb_intervalp returns, and where kb_putp puts a new one,
// depend on the node layout (software/kbtree.h:150-166, 193-207), so the
// tree is rebuilt in seed order, kb_putp for every chain as it is created.
// Chains of clean clusters, and the seeds of a dup cluster up to its first
// equal key, are as the cluster pass decided them (exact: no equal keys
// there yet); the later seeds of a dup cluster (CODE_REPLAY) are decided
// here against the tree, as mem_insert_seed does.  The seeds go one at a
// time in seed order, each tree search and kb_putp by the whole wave (one
// LDS round per node, shifts and splits in parallel: 35 -> 20 M cycles on
// the bench's worst read against lane 0 walking the tree alone); lane 0
// reads and writes the chain records.  The wave loads codes and seeds 64 at
// a time.  A search whose path holds no full node hands its leaf to the
// insert (no second descent).
// Record cache (round 5): lane 0's read of the lower chain's record was a
// dependent HBM round trip per seed, about half of a candidate's ~3,300
// cycles.  The records of the chains the replay touches are kept in a
// direct-mapped, write-through LDS cache keyed by chain id (32-B entries;
// pos is the tree key the search returns): a chain made here is installed as
// it is made, a cluster-pass chain as it is inserted (its record loaded with
// its window's seeds), an append updates the entry and the HBM record.  The
// cache takes the LDS the tree does not use, from the top down, and halves
// when the growing tree needs its space (halving keeps every entry below the
// new size where lookups find it; the HBM records are always current).  On the
// heaviest uniform reads a 256-entry cache would serve 84 % of the lookups,
// 1024 entries 99 % (tools/chain_cache_sim.py).
struct CRec {
    int64_t last_rbeg;
    int32_t first_qbeg, last_qbeg, last_len, n;
    uint32_t last, tag;
};
static_assert(sizeof(CRec) == 32, "CRec is 32 B");

template <class N>
__device__ __forceinline__ int replay_tree(const ChainParams& P, uint64_t S, uint32_t ns, N* pool, int lane, unsigned char* lds,
                           uint32_t lds_bytes, bool pool_in_lds, uint64_t* dbg = nullptr) {
    uint64_t t_search = 0, t_merge = 0, t_insert = 0, n_search = 0, n_insert = 0;  // SMEM_CHAIN_DBG
    const uint32_t* code = reinterpret_cast<const uint32_t*>(P.flt + S);
    const SeedRec* seed = P.seed + S;
    ChainRec* chn = P.chn + S;
    uint32_t root = 0, n_nodes = 1, n_ch = 0;
    // cache slot q at crec[-1 - q]: the top of the LDS region, growing down
    CRec* crec = reinterpret_cast<CRec*>(lds + (lds_bytes & ~31u));
    const uint32_t lo = pool_in_lds ? 8u * (uint32_t)sizeof(N) : 0u;  // the tree's first nodes
    uint32_t C = 0;
    {
        const uint32_t room = lds_bytes > lo ? (lds_bytes - lo) / 32u : 0u;
        C = !P.replay_cache ? 0u : (room >= 2048 ? 2048u : 0u);
        if (!C && P.replay_cache) {
            C = 1;
            while (2 * C <= room) C *= 2;
            if (C < 16) C = 0;
        }
    }
    for (uint32_t q = (uint32_t)lane; q < C; q += 64) crec[-1 - (int)q].tag = 0xffffffffu;
    if (lane == 0) node_init(pool, 1);
    wave_fence();
    __builtin_amdgcn_wave_barrier();
    for (uint32_t base = 0; base < ns; base += 64) {
        const uint32_t o = base + (uint32_t)lane;
        const uint32_t cd = o < ns ? code[o] : CODE_SKIP;
        SeedRec sd{0, 0, 0};
        if (cd != CODE_SKIP) sd = seed[o];
        ChainRec cn{};  // a cluster-pass chain's record, installed when it is inserted
        if (cd == CODE_NEW && C) cn = chn[o];
        uint64_t m = __ballot(cd != CODE_SKIP);
        while (m) {
            const int t = __builtin_ctzll(m);
            m &= m - 1;
            const uint32_t ct = rlu(cd, t);
            const int64_t rb = rl64(sd.rbeg, t);
            const int32_t qb = rl32(sd.qbeg, t), ln = rl32(sd.len, t);
            const uint32_t ot = base + (uint32_t)t;
            int lw = -1;
            int64_t lpos = 0;
            LeafHand hand{false, 0, 0, 0, 0};
            uint64_t c0 = dbg ? __builtin_readcyclecounter() : 0;
            if (ct == CODE_REPLAY && n_ch) {
                lw = tree_lower_wave(pool, root, rb, lane, &hand, &lpos);
                if (dbg) {
                    const uint64_t c1 = __builtin_readcyclecounter();
                    t_search += c1 - c0, ++n_search, c0 = c1;
                }
            }
            int make = 1;
            if (lw >= 0) {
                if (lane == 0) {
                    const uint32_t q = (uint32_t)lw & (C - 1);
                    CRec* e = C ? crec - 1 - (int)q : nullptr;
                    ChainRec c;
                    const bool hit = e && e->tag == (uint32_t)lw;
                    if (hit) {
                        const CRec r = *e;
                        c = ChainRec{lpos, r.last_rbeg, r.first_qbeg, r.last_qbeg, r.last_len, r.n, (uint32_t)lw, r.last};
                    } else {
                        c = chn[lw];
                    }
                    const int mg = merge_test(P, c, rb, qb, ln);
                    if (mg == MERGE_APPEND) {
                        P.next[S + c.last] = ot;
                        chain_append(c, ot, rb, qb, ln);
                        chn[lw] = c;
                    }
                    if (e && (mg == MERGE_APPEND || !hit))
                        *e = CRec{c.last_rbeg, c.first_qbeg, c.last_qbeg, c.last_len, c.n, c.last, (uint32_t)lw};
                    make = mg == MERGE_NEW;
                }
                make = __builtin_amdgcn_readfirstlane(make);
                if (dbg) {
                    const uint64_t c1 = __builtin_readcyclecounter();
                    t_merge += c1 - c0, c0 = c1;
                }
            }
            if (make) {
                if (ct == CODE_REPLAY) {
                    if (lane == 0) {
                        chn[ot] = ChainRec{rb, rb, qb, qb, ln, 1, ot, ot};
                        if (C) crec[-1 - (int)(ot & (C - 1))] = CRec{rb, qb, qb, ln, 1, ot, ot};
                    }
                } else if (lane == t && C) {
                    crec[-1 - (int)(ot & (C - 1))] =
                        CRec{cn.last_rbeg, cn.first_qbeg, cn.last_qbeg, cn.last_len, cn.n, cn.last, ot};
                }
                if (pool_in_lds) {  // an insert splits at most one node per level: keep the cache above them
                    while (C && (n_nodes + 8) * (uint32_t)sizeof(N) > lds_bytes - C * 32u) C = C > 16 ? C / 2 : 0;
                }
                wave_fence();
                __builtin_amdgcn_wave_barrier();
                if (hand.ok) {  // no split on the search's path: insert into its leaf
                    leaf_insert_hand(pool, hand, ot, rb, lane);
                } else {
                    tree_insert_wave(pool, root, n_nodes, ot, rb, lane);
                    root = (uint32_t)__builtin_amdgcn_readfirstlane((int)root);
                    n_nodes = (uint32_t)__builtin_amdgcn_readfirstlane((int)n_nodes);
                }
                ++n_ch;
                if (dbg) t_insert += __builtin_readcyclecounter() - c0, ++n_insert;
            }
        }
    }
    if (dbg && lane == 0) dbg[25] = t_search, dbg[26] = t_merge, dbg[27] = t_insert, dbg[28] = n_search, dbg[29] = n_insert;
    return n_ch ? tree_inorder_wave(pool, root, P.ord + S, lane) : 0;
}

// ---------------------------------------------------------------------------
// ks_introsort(mem_flt) by a wave (software/ksort.h:176-224), the result of
// flt_sort.  Segments are disjoint and each one's depth budget is fixed by
// its depth in the recursion, so the order they are cut in does not matter:
// segments longer than sort_lane_max are cut by the whole wave, one Hoare
// partition at a time; shorter ones get a lane each and the serial loop.  In
// a partition the serial scans swap the k-th left stopper (w <= pivot, from
// the left) with the k-th right stopper (w >= pivot, from the right) while
// the first lies left of the second -- neither scan revisits a position --
// and the pivot goes to the first unpaired left stopper or the last paired
// right stopper, whichever comes first.  The closing insertion sort over the
// whole array is stable and leaves it sorted, so its result is the stable
// sort by weight (descending) of what the partitions left: a bitonic sort of
// (weight, position) keys and a permute.
// ---------------------------------------------------------------------------

// The sort runs on 32-bit keys w << 16 | p (p: the record's position before
// the sort, w < 2^16), not on the 20-byte records: a swap moves one word, the
// keys sit in LDS even when the records are in HBM (the giants), and the
// records move once, in the closing sort's permute.  Only weights are
// compared -- x.w > y.w iff Kx > (Ky | 0xFFFF) -- so every key goes where
// ks_introsort moves its record.
typedef __attribute__((address_space(3))) uint32_t LdsU32;

template <typename KP>
__device__ __forceinline__ void key_swap(KP k, uint32_t i, uint32_t j) {
    const uint32_t x = k[i];
    k[i] = k[j];
    k[j] = x;
}

// flt_combsort on keys (ks_combsort, software/ksort.h:153-174)
template <typename KP>
__device__ __forceinline__ void key_combsort(KP k, uint32_t n) {
    const double shrink = 1.2473309501039786540366528676643;
    uint32_t gap = n;
    bool swapped;
    do {
        if (gap > 2) {
            gap = (uint32_t)((double)gap / shrink);
            if (gap == 9 || gap == 10) gap = 11;
        }
        swapped = false;
        for (uint32_t i = 0; i + gap < n; ++i)
            if (k[i + gap] > (k[i] | 0xFFFFu)) {
                key_swap(k, i, i + gap);
                swapped = true;
            }
    } while (swapped || gap > 2);
    if (gap != 1)
        for (uint32_t i = 1; i < n; ++i)
            for (uint32_t j = i; j > 0 && k[j] > (k[j - 1] | 0xFFFFu); --j) key_swap(k, j, j - 1);
}

// the serial loop from segment [s, t] (t < 2^16: flt_sort_wave takes n <
// 2^16) with depth budget d, without the closing insertion sort; at most
// log2(2^16 / 16) + 1 = 13 segments are pending (see flt_sort), kept as
// s | t << 16 and d in 16-entry arrays small enough for registers.  KP is
// uint32_t* or, for keys in LDS, an LDS-qualified pointer: the scans' loads
// and the swaps are then ds_ operations, not flat ones that wait on both
// counters.
template <typename KP>
__device__ void key_sort_seg_serial(KP k, uint32_t s, uint32_t t, int d) {
    uint32_t sst[16];
    uint8_t sdd[16];
    int top = 0;
    for (;;) {
        if (s < t) {
            if (--d == 0) {
                key_combsort(k + s, t - s + 1);
                t = s;
                continue;
            }
            uint32_t i = s, j = t, m = i + ((j - i) >> 1) + 1;
            {
                const uint32_t wi = k[i] >> 16, wj = k[j] >> 16, wm = k[m] >> 16;
                if (wm > wi) {
                    if (wm > wj) m = j;
                } else {
                    m = wj > wi ? i : j;
                }
            }
            const uint32_t rp = k[m], hi = rp | 0xFFFFu, lo = rp & 0xFFFF0000u;
            if (m != t) key_swap(k, m, t);
            for (;;) {
                do ++i;
                while (k[i] > hi);  // a[i].w > pivot
                do --j;
                while (i <= j && k[j] < lo);  // pivot > a[j].w
                if (j <= i) break;
                key_swap(k, i, j);
            }
            key_swap(k, i, t);
            if (i - s > t - i) {
                if (i - s > 16) {
                    sst[top] = s | (i - 1) << 16;
                    sdd[top] = (uint8_t)d;
                    ++top;
                }
                s = t - i > 16 ? i + 1 : t;
            } else {
                if (t - i > 16) {
                    sst[top] = (i + 1) | t << 16;
                    sdd[top] = (uint8_t)d;
                    ++top;
                }
                t = i - s > 16 ? i - 1 : s;
            }
        } else {
            if (top == 0) return;
            --top;
            s = sst[top] & 0xffffu;
            t = sst[top] >> 16;
            d = sdd[top];
        }
    }
}

__device__ __forceinline__ void wave_sync_mem() {
    wave_fence();
    __builtin_amdgcn_wave_barrier();
}

// one partition of keys ky[s..t] (s < t) as ks_introsort makes it; returns the
// pivot's final position.  tl / tr: the stopper positions by rank
__device__ uint32_t key_partition_wave(uint32_t* ky, uint32_t s, uint32_t t, uint32_t* tl, uint32_t* tr, int lane) {
    s = __builtin_amdgcn_readfirstlane(s);  // arguments come in VGPRs: loop bounds uniform
    t = __builtin_amdgcn_readfirstlane(t);
    uint32_t k = s + ((t - s) >> 1) + 1;
    {
        const uint32_t wi = ky[s] >> 16, wj = ky[t] >> 16, wk = ky[k] >> 16;  // flt_lt(x, y) = x.w > y.w
        if (wk > wi) {
            if (wk > wj) k = t;
        } else {
            k = wj > wi ? s : t;
        }
    }
    const uint32_t pw = ky[k] >> 16;
    if (k != t) {
        if (lane == 0) key_swap(ky, k, t);
        wave_sync_mem();
    }
    uint32_t tot_r = 0;
    for (uint32_t b = s; b < t; b += 64) {
        const uint32_t p = b + (uint32_t)lane;
        tot_r += (uint32_t)__builtin_popcountll(__ballot(p < t && ky[p] >> 16 >= pw));
    }
    const uint64_t below = (1ull << lane) - 1;
    uint32_t run_l = 0, run_r = 0, K = 0;
    for (uint32_t b = s; b <= t; b += 64) {
        const uint32_t p = b + (uint32_t)lane;
        const uint32_t w = p <= t ? ky[p] >> 16 : 0u;
        const bool is_l = p > s && p <= t && w <= pw;
        const bool is_r = p < t && w >= pw;
        const uint64_t ml = __ballot(is_l), mr = __ballot(is_r);
        const uint32_t rl = run_l + (uint32_t)__builtin_popcountll(ml & below);
        // right stoppers after p (p's rank from the right when it is one)
        const uint32_t after = tot_r - run_r - (uint32_t)__builtin_popcountll(mr & (below | (1ull << lane)));
        if (is_l) tl[rl] = p;
        if (is_r) tr[after] = p;
        K += (uint32_t)__builtin_popcountll(__ballot(is_l && after > rl));
        run_l += (uint32_t)__builtin_popcountll(ml);
        run_r += (uint32_t)__builtin_popcountll(mr);
    }
    wave_sync_mem();
    // the K swapped pairs touch 2K distinct positions
    for (uint32_t q0 = 0; q0 < K; q0 += 64) {
        const uint32_t q = q0 + (uint32_t)lane;
        if (q < K) {
            const uint32_t pl = tl[q], pr = tr[q];
            const uint32_t x = ky[pl], y = ky[pr];
            ky[pl] = y;
            ky[pr] = x;
        }
    }
    wave_sync_mem();
    uint32_t i = tl[K];  // t is a left stopper that is never swapped
    if (K > 0) {
        const uint32_t r = tr[K - 1];
        i = r < i ? r : i;
    }
    if (lane == 0) key_swap(ky, i, t);
    wave_sync_mem();
    return i;
}

__device__ void wave_bitonic32(uint32_t* key, uint32_t npad, int lane) {
    npad = __builtin_amdgcn_readfirstlane(npad);
    for (uint32_t k = 2; k <= npad; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            if (npad >= 64 * 2 * 8) bitonic_stage<8>(key, npad, k, j, lane);
            else bitonic_stage<1>(key, npad, k, j, lane);
            wave_sync_mem();
        }
    }
}

// the whole ks_introsort(mem_flt) for n < 2^16 chains of weights in
// [0, 2^16); K: 3 n words (the keys, then two n-word stopper lists, whose
// room the bitonic sort's npad < 2 n keys reuse), k_lds: K is in LDS;
// small: 3 words per lane-cut segment, stk: 3 words per wave-cut segment (at
// most 64 pending); tmp: n records; cnt / cnt_cap: LDS words free once the
// partitions are done, apart from the keys (the closing sort's weight
// counts); wmax: the largest weight
__device__ void flt_sort_wave(FltRec* a, uint32_t n, uint32_t lane_max, uint32_t* K, bool k_lds, FltRec* tmp,
                              uint32_t* small, uint32_t* stk, int lane, int wmin, int wmax, uint32_t* cnt,
                              uint32_t cnt_cap, uint64_t* dbg = nullptr) {
    n = __builtin_amdgcn_readfirstlane(n);  // arguments come in VGPRs: loop bounds uniform
    lane_max = __builtin_amdgcn_readfirstlane(lane_max);
    wmin = __builtin_amdgcn_readfirstlane(wmin);
    wmax = __builtin_amdgcn_readfirstlane(wmax);
    cnt_cap = __builtin_amdgcn_readfirstlane(cnt_cap);
    if (n < 2) return;
    if (n == 2) {
        if (lane == 0 && flt_lt(a[1], a[0])) flt_swap(a, 0, 1);
        wave_sync_mem();
        return;
    }
    uint32_t* tl = K + n;
    uint32_t* tr = K + 2 * n;
    for (uint32_t p = lane; p < n; p += 64) K[p] = (uint32_t)a[p].w << 16 | p;
    int d = 2;
    while ((1ull << d) < n) ++d;
    d <<= 1;
    uint32_t top = 0, n_small = 0;
    auto add = [&](uint32_t s, uint32_t t, int dd) {
        uint32_t* dst;
        if (t - s + 1 > lane_max && top < 64) dst = stk + 3 * top++;
        else dst = small + 3 * n_small++;
        if (lane == 0) {
            dst[0] = s;
            dst[1] = t;
            dst[2] = (uint32_t)dd;
        }
    };
    add(0, n - 1, d);
    wave_sync_mem();
    while (top > 0) {
        --top;
        const uint32_t s = stk[3 * top], t = stk[3 * top + 1];
        int dd = (int)stk[3 * top + 2];
        wave_sync_mem();
        if (--dd == 0) {
            if (lane == 0) key_combsort(K + s, t - s + 1);
            if (dbg && lane == 0) dbg[16] += 1, dbg[17] += t - s + 1;
        } else {
            const uint32_t i = key_partition_wave(K, s, t, tl, tr, lane);
            if (dbg && lane == 0) dbg[18] += 1, dbg[19] += t - s + 1;
            if (i - s > 16) add(s, i - 1, dd);
            if (t - i > 16) add(i + 1, t, dd);
        }
        wave_sync_mem();
    }
    if (dbg && lane == 0) dbg[20] = __builtin_readcyclecounter(), dbg[21] = n_small;
    if (k_lds) {
        LdsU32* kl = (LdsU32*)K;
        for (uint32_t q = lane; q < n_small; q += 64)
            key_sort_seg_serial(kl, small[3 * q], small[3 * q + 1], (int)small[3 * q + 2]);
    } else {
        for (uint32_t q = lane; q < n_small; q += 64)
            key_sort_seg_serial(K, small[3 * q], small[3 * q + 1], (int)small[3 * q + 2]);
    }
    wave_sync_mem();
    if (dbg && lane == 0) dbg[22] = __builtin_readcyclecounter();
    // the closing insertion sort: a stable sort by weight, descending
    const uint32_t R = (uint32_t)(wmax - wmin) + 1u;
    if (cnt && R <= cnt_cap) {
        // by counting (weights span R <= cnt_cap values): counts by wmax - w
        // in LDS, their exclusive scan, then the records scattered 64 at a
        // time in array order, each lane behind the earlier lanes of its
        // weight -- stable, as the insertion sort (round 5: the bitonic sort of
        // (weight, position) keys over the node pool took ~2.8 M cycles of a
        // 5,000-chain read)
        for (uint32_t q = lane; q < R; q += 64) cnt[q] = 0;
        wave_sync_mem();
        for (uint32_t p = lane; p < n; p += 64) atomicAdd(&cnt[(uint32_t)wmax - (K[p] >> 16)], 1u);
        wave_sync_mem();
        uint32_t run = 0;
        for (uint32_t q0 = 0; q0 < R; q0 += 64) {
            const uint32_t q = q0 + lane;
            const uint32_t v = q < R ? cnt[q] : 0u;
            uint32_t tot;
            const uint32_t ex = wave_excl_scan(v, lane, tot);
            if (q < R) cnt[q] = run + ex;
            run += tot;
        }
        wave_sync_mem();
        for (uint32_t c = 0; c < n; c += 64) {
            const uint32_t p = c + (uint32_t)lane;
            const bool valid = p < n;
            FltRec r{};
            uint32_t d = 0xFFFFFFFFu;
            if (valid) {
                const uint32_t kp = K[p];
                r = a[kp & 0xFFFFu];
                d = (uint32_t)wmax - (kp >> 16);
            }
            uint64_t rem = __ballot(valid);
            uint32_t pos = 0;
            while (rem) {
                const int ld = (int)__builtin_ctzll(rem);
                const uint32_t dl = (uint32_t)__builtin_amdgcn_readlane((int)d, ld);
                const uint64_t m = __ballot(d == dl);
                const uint32_t b = cnt[dl];
                if (d == dl) pos = b + (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1));
                wave_sync_mem();
                if (lane == ld) cnt[dl] = b + (uint32_t)__builtin_popcountll(m);
                wave_sync_mem();
                rem &= ~m;
            }
            if (valid) tmp[pos] = r;
        }
        wave_sync_mem();
    } else {
        uint32_t npad = 2;
        while (npad < n) npad <<= 1;
        uint32_t* keys = tl;
        for (uint32_t p = lane; p < npad; p += 64)
            keys[p] = p < n ? ((0xFFFFu - (K[p] >> 16)) << 16) | p : 0xFFFFFFFFu;
        wave_sync_mem();
        wave_bitonic32(keys, npad, lane);
        for (uint32_t r = lane; r < n; r += 64) tmp[r] = a[K[keys[r] & 0xFFFFu] & 0xFFFFu];
        wave_sync_mem();
    }
    if (dbg && lane == 0) dbg[24] = __builtin_readcyclecounter();
    for (uint32_t r = lane; r < n; r += 64) a[r] = tmp[r];
    wave_sync_mem();
}

}  // namespace

// one lane per read with at most P.heavy_min seed occurrences; heavier
// reads are listed for chain_heavy_kernel (giants, > P.giant_min, first)
__global__ __launch_bounds__(256) void chain_build_kernel(ChainParams P) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= P.n_reads) return;
    const uint64_t i0 = P.intv_off[r], i1 = P.intv_off[r + 1];
    const uint64_t S = P.occ_off[i0], E = P.occ_off[i1];
    if (S == E) {
        P.n_out[r] = 0;
        P.ns_out[r] = 0;
        return;
    }
    if (E - S > (uint64_t)P.heavy_min) {
        const int gi = E - S > (uint64_t)P.giant_min ? 0 : 1;
        const uint32_t slot = atomicAdd(P.heavy_ctr + gi, 1u);
        P.heavy[gi * (uint64_t)P.n_reads + slot] = (uint32_t)r;
        return;
    }
    BNode* pool = P.node + (S / 7 + 3ull * (uint64_t)r);
    InsState st;
    ins_start(st, P, i0);
    insert_read(P, i1, S, pool, 0xffffffffu, st);
    uint32_t* ord = P.ord + S;
    uint32_t* ord2 = P.ord2 + S;
    const int n = !st.n_ch ? 0 : (st.n_ch < 127 ? tree_inorder2(pool, st.root, ord) : tree_inorder(pool, st.root, ord));
    int n_keep = n;
    if (!P.filter || n <= 1) {
        for (int i = 0; i < n; ++i) ord2[i] = ord[i];
    } else {
        FltRec* a = P.flt + S;
        // the sort's stack in the read's kbtree node pool (>= 3 nodes of 256 B),
        // free once the chains are listed
        flt_prepare_serial(P, S, a, ord, ord2, n, reinterpret_cast<uint32_t*>(pool));
        const int m = flt_drop_serial(a, n, P.mask_level, P.drop_ratio, P.min_seed_len);
        n_keep = flt_squeeze_serial(a, m, ord, ord2, n);
    }
    P.n_out[r] = (uint64_t)n_keep;
    P.ns_out[r] = seeds_in(P, S, ord2, n_keep);
}

// one wave per heavy read, persistent over the two lists (giants first):
// the chain tree and the filter's records live in LDS (dynamic, P.lds_bytes)
// while they fit and in the read's HBM pool otherwise; insertion, traversal
// and the introsort run on lane 0 (their order is the reference's), the
// weights and the drop loop on all 64 lanes
__global__ __launch_bounds__(64) void chain_heavy_kernel(ChainParams P) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    __shared__ uint32_t s_item;
    __shared__ int64_t s_dups[256];
    __shared__ uint32_t s_stk[3 * 64];
    const int lane = threadIdx.x;
    const uint32_t n_giant = P.heavy_ctr[0], n_all = n_giant + P.heavy_ctr[1];
    const uint32_t it_lo = P.tier == 1 ? n_giant : 0, it_hi = P.tier == 0 ? n_giant : n_all;
    for (;;) {
        if (lane == 0) s_item = it_lo + atomicAdd(P.heavy_ctr + 2 + (P.tier == 1 ? 1 : 0), 1u);
        __syncthreads();
        const uint32_t item = s_item;
        __syncthreads();
        if (item >= it_hi) break;
        const uint32_t r = item < n_giant ? P.heavy[item] : P.heavy[(uint64_t)P.n_reads + (item - n_giant)];
        const uint64_t i0 = P.intv_off[r], i1 = P.intv_off[r + 1];
        const uint64_t S = P.occ_off[i0];
        uint32_t* ord = P.ord + S;
        uint32_t* ord2 = P.ord2 + S;
        __shared__ int s_n;
        uint64_t* dbg = (P.dbg && item - P.dbg_lo < 256u) ? P.dbg + (item - P.dbg_lo) * 32 : nullptr;  // 32 words a read
        if (dbg && lane == 0) {
            dbg[0] = r;
            dbg[1] = P.occ_off[i1] - S;
            dbg[2] = __builtin_readcyclecounter();
            dbg[14] = __builtin_amdgcn_s_memrealtime();
        }
        // seed records of the read, all lanes (mem_seed_t of every occurrence)
        for (uint64_t iv = i0; iv < i1; ++iv) {
            const uint64_t a = P.occ_off[iv], b = P.occ_off[iv + 1];
            if (a == b) continue;
            const uint64_t info = P.intv[iv * 4 + 3];
            const int32_t qbeg = (int32_t)(info >> 32);
            const int32_t len = (int32_t)((uint32_t)info - (uint32_t)(info >> 32));
            for (uint64_t o = a + (uint64_t)lane; o < b; o += 64) P.seed[o] = SeedRec{(int64_t)P.pos[o], qbeg, len};
        }
        __syncthreads();
        bool done = false;
        if (P.cluster) {
            const uint64_t E = P.occ_off[i1];
            uint32_t npad = 2;
            while (npad < E - S) npad <<= 1;
            if (E - S < (1ull << CL_OBITS) && cluster_lds_need(npad) <= P.lds_bytes) {
                int n = 0;
                uint32_t n_cand = 0;
                const bool clean =
                    insert_read_clusters(P, S, E, reinterpret_cast<uint64_t*>(lds_raw), lane, n, n_cand);
                if (dbg && lane == 0) {
                    dbg[11] = __builtin_readcyclecounter();
                    dbg[12] = n_cand;
                }
                if (!clean) {
                    // an equal chain key: rebuild the tree in seed order
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                    __syncthreads();
                    if (n_cand / (BT_T - 1) + 8 <= P.lds_bytes / sizeof(LNode))
                        n = replay_tree(P, S, (uint32_t)(E - S), reinterpret_cast<LNode*>(lds_raw), lane, lds_raw,
                                        P.lds_bytes, true, dbg);
                    else
                        n = replay_tree(P, S, (uint32_t)(E - S), P.node + (S / 7 + 3ull * (uint64_t)r), lane,
                                        lds_raw, P.lds_bytes, false, dbg);
                }
                if (lane == 0) {
                    s_n = n;
                    if (dbg) {
                        dbg[3] = __builtin_readcyclecounter();
                        dbg[4] = n;
                        dbg[10] = clean ? 0 : 1;
                    }
                }
                done = true;
                __syncthreads();
            }
        }
        if (!done) {
            const uint64_t E = P.occ_off[i1];
            LNode* lpool = reinterpret_cast<LNode*>(lds_raw);
            uint64_t o = S;
            uint32_t n_ch = 0, root = 0, n_nodes = 1;
            if (lane == 0) node_init(lpool, 1);
            __syncthreads();
            int n_dup = 0;
            const bool in_lds = insert_read_wave(P, S, E, lpool, P.lds_bytes / sizeof(LNode), o, n_ch, root, n_nodes,
                                                 lane, s_dups, n_dup, dbg);
            BNode* gpool = P.node + (S / 7 + 3ull * (uint64_t)r);
            if (!in_lds) {
                // out of LDS: move the tree to the read's HBM pool, go on there
                for (uint32_t j = lane; j < n_nodes; j += 64) {
                    const LNode& l = lpool[j];
                    BNode& g = gpool[j];
                    g.n = l.n;
                    g.leaf = l.leaf;
                    for (int q = 0; q < BT_MAX; ++q) {
                        g.key[q] = l.key[q];
                        g.id[q] = l.id[q];
                    }
                    for (int q = 0; q <= BT_MAX; ++q) g.child[q] = l.child[q];
                }
                __syncthreads();
                insert_read_wave(P, S, E, gpool, 0xffffffffu, o, n_ch, root, n_nodes, lane, s_dups, n_dup, dbg);
            }
            int n_io = 0;
            if (n_ch) n_io = in_lds ? tree_inorder_wave(lpool, root, ord, lane) : tree_inorder_wave(gpool, root, ord, lane);
            if (lane == 0) {
                const int n = n_io;
                s_n = n;
                if (dbg) {
                    dbg[3] = __builtin_readcyclecounter();
                    dbg[4] = n;
                }
            }
        }
        __syncthreads();
        const int n = s_n;
        int n_keep = n;
        if (!P.filter || n <= 1) {
            for (int i = lane; i < n; i += 64) ord2[i] = ord[i];
        } else {
            const bool in_lds = (uint64_t)n * sizeof(FltRec) <= (uint64_t)P.lds_bytes;
            if (dbg && lane == 0) dbg[23] = in_lds;
            FltRec* la = reinterpret_cast<FltRec*>(lds_raw);
            FltRec* ga = P.flt + S;
            // weights, four chains per lane at a time: their seed walks are
            // independent, so each step's loads overlap (one walk per lane was
            // a dependent round trip per seed, ~2 M cycles on a 5,000-chain
            // read).  Only the query-coordinate loop of mem_chain_weight: its
            // second loop starts from the first's total and only adds (this
            // version never resets w), so min(w, tmp) is tmp (chain_weight)
            for (int i0 = lane; i0 < n; i0 += 256) {
                ChainRec c[4];
                uint32_t o[4];
                int rem[4], w[4];
                int64_t end[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int i = i0 + 64 * k;
                    rem[k] = 0;
                    if (i < n) {
                        c[k] = P.chn[S + ord[i]];
                        rem[k] = c[k].n;
                        o[k] = c[k].first;
                    }
                    w[k] = 0;
                    end[k] = 0;
                }
                while (rem[0] > 0 || rem[1] > 0 || rem[2] > 0 || rem[3] > 0) {
                    SeedRec sd[4];
                    uint32_t nx[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        if (rem[k] > 0) {
                            sd[k] = P.seed[S + o[k]];
                            nx[k] = P.next[S + o[k]];
                        }
                    }
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        if (rem[k] > 0) {
                            const SeedRec& q = sd[k];
                            if (q.qbeg >= end[k]) w[k] += q.len;
                            else if (q.qbeg + q.len > end[k]) w[k] = (int)(w[k] + (q.qbeg + q.len - end[k]));
                            end[k] = end[k] > q.qbeg + q.len ? end[k] : q.qbeg + q.len;
                            o[k] = nx[k];
                            --rem[k];
                        }
                    }
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int i = i0 + 64 * k;
                    if (i < n) {
                        const FltRec f{c[k].first_qbeg, c[k].last_qbeg + c[k].last_len, w[k], i, -1};
                        if (in_lds) la[i] = f;
                        else ga[i] = f;
                    }
                }
            }
            __syncthreads();
            if (dbg && lane == 0) dbg[5] = __builtin_readcyclecounter();
            int wmin = INT32_MAX, wmax = INT32_MIN;
            for (int i = lane; i < n; i += 64) {
                const int w = in_lds ? la[i].w : ga[i].w;
                wmin = w < wmin ? w : wmin;
                wmax = w > wmax ? w : wmax;
            }
            for (int off = 32; off > 0; off >>= 1) {
                const int a0 = __shfl_xor(wmin, off), a1 = __shfl_xor(wmax, off);
                wmin = a0 < wmin ? a0 : wmin;
                wmax = a1 > wmax ? a1 : wmax;
            }
            if (P.wave_sort && n < 0x10000 && wmin >= 0 && wmax < 0x10000) {
                // scratch: the keys and stopper lists (3 n words) in LDS,
                // after the records when they are there, while they fit, else
                // (and the permute's copy always) in the read's kbtree node
                // pool, free once the chains are listed (>= 36 n bytes, see
                // below: the copy takes 20 n, the keys 12 n)
                const uint64_t need = (uint64_t)n * 12;
                uint8_t* gs = reinterpret_cast<uint8_t*>(P.node + (S / 7 + 3ull * (uint64_t)r));
                const uint64_t k_off = in_lds ? (uint64_t)n * sizeof(FltRec) : 0;
                const bool k_lds = k_off + need <= P.lds_bytes;
                uint32_t* K = k_lds ? reinterpret_cast<uint32_t*>(lds_raw + k_off)
                                    : reinterpret_cast<uint32_t*>(gs + (uint64_t)n * sizeof(FltRec));
                // the closing sort's counts: the LDS after the records and
                // the keys (the stopper lists there are dead by then)
                const uint64_t c_off = k_off + (k_lds ? (uint64_t)n * 4 : 0);
                uint32_t* cnt = reinterpret_cast<uint32_t*>(lds_raw + c_off);
                const uint64_t cnt_room = ((uint64_t)P.lds_bytes - c_off) / 4;
                const uint32_t cnt_cap = P.sort_count ? (uint32_t)(cnt_room < 65536 ? cnt_room : 65536) : 0u;
                flt_sort_wave(in_lds ? la : ga, (uint32_t)n, P.sort_lane_max, K, k_lds, reinterpret_cast<FltRec*>(gs),
                              ord2, s_stk, lane, wmin, wmax, cnt, cnt_cap, dbg);
            } else if (lane == 0) {
                if (in_lds) flt_sort(la, (uint32_t)n, s_stk);
                else flt_sort(ga, (uint32_t)n, s_stk);
            }
            __syncthreads();
            if (dbg && lane == 0) dbg[6] = __builtin_readcyclecounter();
            for (int i = lane; i < n; i += 64) {
                if (in_lds) {
                    ord2[i] = ord[la[i].p];
                    la[i].p = i;
                } else {
                    ord2[i] = ord[ga[i].p];
                    ga[i].p = i;
                }
            }
            __syncthreads();
            int m;
            if (P.drop_ratio > 0.f && P.drop_blocked) {
                // kidx / jst / U: LDS after the records while all fit, else
                // kidx in the read's ord rows (free until the marks below),
                // jst and U in its kbtree node pool (free after the sort; the
                // pool holds >= (E - S) / 7 + 2 nodes of 256 B, > 36 n bytes
                // as n <= E - S: jst takes 4 n, U 16 n)
                const bool x_lds = in_lds && (uint64_t)n * (sizeof(FltRec) + 24) + 16 <= (uint64_t)P.lds_bytes;
                uint32_t* kidx;
                int32_t* jst;
                uint4* U;
                if (x_lds) {
                    kidx = reinterpret_cast<uint32_t*>(la + n);
                } else {
                    kidx = ord;
                }
                uint32_t* xs = x_lds ? kidx + n : reinterpret_cast<uint32_t*>(P.node + (S / 7 + 3ull * (uint64_t)r));
                jst = reinterpret_cast<int32_t*>(xs);
                // 16-B entries (kept index, position, span), 16-B aligned
                U = reinterpret_cast<uint4*>((reinterpret_cast<uintptr_t>(xs + n) + 15) & ~(uintptr_t)15);
                m = in_lds ? flt_drop_blocked(la, kidx, jst, U, n, P.mask_level, P.drop_ratio, P.min_seed_len, lane, dbg)
                           : flt_drop_blocked(ga, kidx, jst, U, n, P.mask_level, P.drop_ratio, P.min_seed_len, lane, dbg);
            } else if (P.drop_ratio > 0.f) {
                // U: LDS after the records while both fit, else the read's ord
                // rows (free until the marks below)
                const bool u_lds = in_lds && (uint64_t)n * (sizeof(FltRec) + 4) <= (uint64_t)P.lds_bytes;
                uint32_t* U = u_lds ? reinterpret_cast<uint32_t*>(la + n) : ord;
                m = in_lds ? flt_drop_pruned(la, U, n, P.mask_level, P.drop_ratio, P.min_seed_len, lane)
                           : flt_drop_pruned(ga, U, n, P.mask_level, P.drop_ratio, P.min_seed_len, lane);
            } else {
                m = in_lds ? flt_drop_wave(la, n, P.mask_level, P.drop_ratio, P.min_seed_len, lane)
                           : flt_drop_wave(ga, n, P.mask_level, P.drop_ratio, P.min_seed_len, lane);
            }
            __syncthreads();
            if (dbg && lane == 0) {
                dbg[7] = __builtin_readcyclecounter();
                dbg[8] = m;
            }
            for (int i = lane; i < n; i += 64) ord[i] = 0;
            __syncthreads();
            for (int i = lane; i < m; i += 64) {
                const FltRec f = in_lds ? la[i] : ga[i];
                ord[f.p] = 1;
                if (f.p2 >= 0) ord[f.p2] = 1;
            }
            __syncthreads();
            // squeeze in order, 64 at a time
            n_keep = 0;
            for (int base = 0; base < n; base += 64) {
                const int i = base + lane;
                const bool keep = i < n && ord[i] != 0;
                const uint64_t bk = __ballot(keep);
                const uint32_t v = keep ? ord2[i] : 0;
                __syncthreads();
                if (keep) ord2[n_keep + __builtin_popcountll(bk & ((1ull << lane) - 1))] = v;
                n_keep += __builtin_popcountll(bk);
                __syncthreads();
            }
        }
        uint64_t ns = 0;
        for (int i = lane; i < n_keep; i += 64) ns += (uint64_t)P.chn[S + ord2[i]].n;
        for (int off = 32; off > 0; off >>= 1) ns += __shfl_xor(ns, off);
        if (lane == 0) {
            P.n_out[r] = (uint64_t)n_keep;
            P.ns_out[r] = ns;
            if (dbg) {
                dbg[9] = __builtin_readcyclecounter();
                dbg[15] = __builtin_amdgcn_s_memrealtime();
            }
        }
        __syncthreads();
    }
}

__device__ __forceinline__ void write_chains(const ChainParams& P, uint32_t r, int lane, int width) {
    const uint64_t c0 = P.chain_off[r], nc = P.chain_off[r + 1] - c0;
    if (nc == 0) return;
    const uint64_t S = P.occ_off[P.intv_off[r]];
    const uint32_t* ord2 = P.ord2 + S;
    const ChainRec* chn = P.chn + S;
    const SeedRec* seed = P.seed + S;
    const uint32_t* next = P.next + S;
    uint64_t so = P.seed_off[r];
    // chains in order, `width` lanes at a time; seed offsets by a prefix sum
    for (uint64_t base = 0; base < nc; base += (uint64_t)width) {
        const uint64_t i = base + (uint64_t)lane;
        const bool live = i < nc;
        const ChainRec c = live ? chn[ord2[i]] : ChainRec{};
        uint64_t incl = live ? (uint64_t)c.n : 0;
        for (int off = 1; off < width; off <<= 1) {
            const uint64_t t = __shfl_up(incl, off, width);
            if (lane >= off) incl += t;
        }
        const uint64_t total = __shfl(incl, width - 1, width);
        if (live) {
            uint64_t w = so + incl - (uint64_t)c.n;
            P.out_chain[c0 + i] = OutChain{c.pos, w, c.n, 0};
            uint32_t o = c.first;
            for (int j = 0; j < c.n; ++j, o = next[o]) P.out_seed[w++] = seed[o];
        }
        so += total;
    }
}

__global__ __launch_bounds__(256) void chain_write_kernel(ChainParams P) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= P.n_reads) return;
    const uint64_t S = P.occ_off[P.intv_off[r]], E = P.occ_off[P.intv_off[r + 1]];
    if (E - S > (uint64_t)P.heavy_min) return;  // chain_write_heavy_kernel
    write_chains(P, (uint32_t)r, 0, 1);
}

__global__ __launch_bounds__(64) void chain_write_heavy_kernel(ChainParams P) {
    const uint32_t n_giant = P.heavy_ctr[0], n_all = n_giant + P.heavy_ctr[1];
    for (uint32_t item = blockIdx.x; item < n_all; item += gridDim.x) {
        const uint32_t r = item < n_giant ? P.heavy[item] : P.heavy[(uint64_t)P.n_reads + (item - n_giant)];
        write_chains(P, r, threadIdx.x, 64);
    }
}

}  // namespace smem

// The heavy reads in two tiers: the giants (> giant_min seeds) with the big
// LDS allotment, one wave per CU, and the rest with lds_rest (several waves
// per CU; their trees, clusters and filter records fit it) on st2 beside
// them, picking up the CUs as giant waves retire.  One launch of both with
// the big allotment left 3 of 4 SIMDs idle while the bulk of the heavy reads
// went through it.
namespace smem {

// The giants reordered by occurrences (the cost's proxy), longest first
// (P.giant_order 1) or shortest first (2): the heavy queue hands items out in
// list order.  Measured and off by default (r6y/r6z, human-like 1M reads):
// either order takes the giant tier from 18.8 to 25.5 ms while the rest tier
// ends sooner (17.1 -> 12.0 ms) -- the listing order's mix of long and short
// giants shares the CUs with the 28 KB tier better.  One workgroup, a bitonic
// sort of (occurrences, read) keys in LDS; a longer list than
// GIANT_ORDER_MAX keeps its listing order.  No result depends on the order:
// each read's chains are its own.
constexpr uint32_t GIANT_ORDER_MAX = 4096;

__global__ __launch_bounds__(1024) void chain_giant_order_kernel(ChainParams P) {
    __shared__ uint64_t key[GIANT_ORDER_MAX];
    const uint32_t n = P.heavy_ctr[0];
    const bool desc = P.giant_order == 1;  // 2: shortest first
    if (n < 2 || n > GIANT_ORDER_MAX) return;
    uint32_t npad = 2;
    while (npad < n) npad <<= 1;
    for (uint32_t i = threadIdx.x; i < npad; i += blockDim.x) {
        uint64_t v = desc ? 0 : ~0ull;  // padding sorts last
        if (i < n) {
            const uint32_t r = P.heavy[i];
            v = (P.occ_off[P.intv_off[r + 1]] - P.occ_off[P.intv_off[r]]) << 32 | r;
        }
        key[i] = v;
    }
    __syncthreads();
    for (uint32_t k = 2; k <= npad; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = threadIdx.x; i < npad; i += blockDim.x) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const uint64_t a = key[i], b = key[l];
                    if (((i & k) == 0) == desc ? a < b : a > b) {
                        key[i] = b;
                        key[l] = a;
                    }
                }
            }
            __syncthreads();
        }
    }
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) P.heavy[i] = (uint32_t)key[i];
}

}  // namespace smem

extern "C" hipError_t smem_launch_chain_build(const smem::ChainParams* P, int n_cu, hipStream_t st, hipStream_t st2,
                                              hipEvent_t ev_fork, hipEvent_t ev_join) {
    if (P->n_reads <= 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(P->heavy_ctr, 0, 4 * sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(smem::chain_build_kernel, dim3((P->n_reads + 255) / 256), dim3(256), 0, st, *P);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    // more than the default 64 KB of dynamic LDS per workgroup (gfx950 has 160 KB per CU)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(smem::chain_heavy_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)P->lds_bytes);
    if (!st2) {
        if (P->giant_order) {
            hipLaunchKernelGGL(smem::chain_giant_order_kernel, dim3(1), dim3(1024), 0, st, *P);
            if ((e = hipGetLastError()) != hipSuccess) return e;
        }
        smem::ChainParams Q = *P;
        Q.tier = -1;
        hipLaunchKernelGGL(smem::chain_heavy_kernel, dim3(n_cu), dim3(64), Q.lds_bytes, st, Q);
        return hipGetLastError();
    }
    if ((e = hipEventRecord(ev_fork, st)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(st2, ev_fork, 0)) != hipSuccess) return e;
    smem::ChainParams G = *P, R = *P;
    G.tier = 0;
    R.tier = 1;
    R.lds_bytes = P->lds_rest < P->lds_bytes ? P->lds_rest : P->lds_bytes;
    if (P->giant_order) {  // the rest tier does not wait for it (its items are the list's second half)
        hipLaunchKernelGGL(smem::chain_giant_order_kernel, dim3(1), dim3(1024), 0, st, *P);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(smem::chain_heavy_kernel, dim3(P->giant_waves ? P->giant_waves : (uint32_t)n_cu), dim3(64),
                       G.lds_bytes, st, G);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const uint32_t per_cu = 160u * 1024u / (R.lds_bytes + 4096u);
    hipLaunchKernelGGL(smem::chain_heavy_kernel, dim3(n_cu * (per_cu < 1 ? 1 : (per_cu > 8 ? 8 : per_cu))), dim3(64),
                       R.lds_bytes, st2, R);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = hipEventRecord(ev_join, st2)) != hipSuccess) return e;
    return hipStreamWaitEvent(st, ev_join, 0);
}

extern "C" hipError_t smem_launch_chain_write(const smem::ChainParams* P, int n_cu, hipStream_t st) {
    if (P->n_reads <= 0) return hipSuccess;
    hipLaunchKernelGGL(smem::chain_write_kernel, dim3((P->n_reads + 255) / 256), dim3(256), 0, st, *P);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(smem::chain_write_heavy_kernel, dim3(n_cu * 4), dim3(64), 0, st, *P);
    return hipGetLastError();
}

// this file's code object loaded on the current device (see smem_preload_seed)
extern "C" hipError_t smem_preload_chain(void) {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&smem::chain_write_kernel));
}
