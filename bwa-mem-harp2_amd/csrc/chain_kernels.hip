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

// leftmost key == k (eq) or else the last key < k (-1 if none): kbtree's
// __kb_getp_aux (software/kbtree.h:97-110); keys are sorted, so that is the
// count of keys below k, all 15 loaded independently
__device__ __forceinline__ int node_find(const BNode* x, int64_t k, bool& eq) {
    const int n = x->n;
    int below = 0;
#pragma unroll
    for (int i = 0; i < BT_MAX; ++i) below += (i < n && x->key[i] < k) ? 1 : 0;
    eq = below < n && x->key[below] == k;
    return eq ? below : below - 1;
}

// kb_intervalp's `lower` (software/kbtree.h:150-166)
__device__ int tree_lower(const BNode* pool, uint32_t root, int64_t k) {
    uint32_t x = root;
    int lower = -1;
    for (;;) {
        const BNode* nd = pool + x;
        bool eq;
        const int i = node_find(nd, k, eq);
        if (i >= 0 && eq) return (int)nd->id[i];
        if (i >= 0) lower = (int)nd->id[i];
        if (nd->leaf) return lower;
        x = nd->child[i + 1];
    }
}

__device__ __forceinline__ void node_init(BNode* x, int leaf) {
    x->n = 0;
    x->leaf = leaf;
}

// __kb_split (software/kbtree.h:172-186): full child y = x.child[i] keeps its
// lower 7 keys, a new right sibling takes the upper 7, the middle moves up
__device__ void node_split(BNode* pool, uint32_t xi, int i, uint32_t yi, uint32_t& n_nodes) {
    BNode* x = pool + xi;
    BNode* y = pool + yi;
    const uint32_t zi = n_nodes++;
    BNode* z = pool + zi;
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
__device__ void tree_insert(BNode* pool, uint32_t& root, uint32_t& n_nodes, uint32_t id, int64_t k) {
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
    BNode* nd = pool + x;
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
__device__ int tree_inorder(const BNode* pool, uint32_t root, uint32_t* out) {
    uint32_t sx[24];
    int si[24];
    int top = 0, n_out = 0;
    sx[0] = root;
    si[0] = 0;
    for (;;) {
        while (sx[top] != BT_NONE && si[top] <= pool[sx[top]].n) {
            const BNode* nd = pool + sx[top];
            sx[top + 1] = nd->leaf ? BT_NONE : nd->child[si[top]];
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

// mem_chain_weight (software/bwamem.c:501-521), the second loop's `end`
// advanced by query coordinates as the reference writes it
__device__ int chain_weight(const ChainRec& c, const SeedRec* seed, const uint32_t* next) {
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

__device__ void flt_insertsort(FltRec* a, size_t n) {
    for (size_t i = 1; i < n; ++i)
        for (size_t j = i; j > 0 && flt_lt(a[j], a[j - 1]); --j) flt_swap(a, j, j - 1);
}

__device__ void flt_combsort(FltRec* a, size_t n) {
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

// ks_introsort(mem_flt) (software/ksort.h:176-224), comparison for comparison
__device__ void flt_sort(FltRec* a, size_t n) {
    size_t sl[64], sr[64];
    int sd[64];
    int top = 0, d;
    if (n < 1) return;
    if (n == 2) {
        if (flt_lt(a[1], a[0])) flt_swap(a, 0, 1);
        return;
    }
    for (d = 2; (1ull << d) < n; ++d) {
    }
    d <<= 1;
    size_t s = 0, t = n - 1;
    for (;;) {
        if (s < t) {
            if (--d == 0) {
                flt_combsort(a + s, t - s + 1);
                t = s;
                continue;
            }
            size_t i = s, j = t, k = i + ((j - i) >> 1) + 1;
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
                    sl[top] = s;
                    sr[top] = i - 1;
                    sd[top] = d;
                    ++top;
                }
                s = t - i > 16 ? i + 1 : t;
            } else {
                if (t - i > 16) {
                    sl[top] = i + 1;
                    sr[top] = t;
                    sd[top] = d;
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
            s = sl[top];
            t = sr[top];
            d = sd[top];
        }
    }
}

}  // namespace

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
    BNode* pool = P.node + (S / 7 + 3ull * (uint64_t)r);
    ChainRec* chn = P.chn + S;
    uint32_t root = 0, n_nodes = 1, n_ch = 0;
    node_init(pool, 1);
    // the seed loop of mem_insert_seed (software/bwamem.c:462-499)
    for (uint64_t iv = i0; iv < i1; ++iv) {
        const uint64_t a = P.occ_off[iv], b = P.occ_off[iv + 1];
        if (a == b) continue;
        const uint64_t info = P.intv[iv * 4 + 3];
        const int32_t qbeg = (int32_t)(info >> 32);
        const int32_t len = (int32_t)((uint32_t)info - (uint32_t)(info >> 32));
        for (uint64_t o = a; o < b; ++o) {
            const int64_t rb = (int64_t)P.pos[o];
            if (rb < P.l_pac && P.l_pac < rb + len) continue;  // bridges the strands
            P.seed[o] = SeedRec{rb, qbeg, len};
            if (n_ch) {
                const int lw = tree_lower(pool, root, rb);
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
            ChainRec c;
            c.pos = rb;
            c.last_rbeg = rb;
            c.first_qbeg = qbeg;
            c.last_qbeg = qbeg;
            c.last_len = len;
            c.n = 1;
            c.first = c.last = (uint32_t)(o - S);
            chn[n_ch] = c;
            tree_insert(pool, root, n_nodes, n_ch, rb);
            ++n_ch;
        }
    }
    uint32_t* ord = P.ord + S;
    uint32_t* ord2 = P.ord2 + S;
    const SeedRec* seed = P.seed + S;
    const uint32_t* next = P.next + S;
    const int n = n_ch ? tree_inorder(pool, root, ord) : 0;
    int n_keep = n;
    if (!P.filter || n <= 1) {
        for (int i = 0; i < n; ++i) ord2[i] = ord[i];
    } else {
        // mem_chain_flt (software/bwamem.c:629-690)
        FltRec* a = P.flt + S;
        for (int i = 0; i < n; ++i) {
            const ChainRec c = chn[ord[i]];
            a[i] = FltRec{c.first_qbeg, c.last_qbeg + c.last_len, chain_weight(c, seed, next), i, -1};
        }
        flt_sort(a, (size_t)n);
        for (int i = 0; i < n; ++i) {
            ord2[i] = ord[a[i].p];
            a[i].p = i;
        }
        int m = 1;
        for (int i = 1; i < n; ++i) {
            int j;
            for (j = 0; j < m; ++j) {
                const int b_max = a[j].beg > a[i].beg ? a[j].beg : a[i].beg;
                const int e_min = a[j].end < a[i].end ? a[j].end : a[i].end;
                if (e_min > b_max) {
                    const int li = a[i].end - a[i].beg, lj = a[j].end - a[j].beg;
                    const int min_l = li < lj ? li : lj;
                    if ((float)(e_min - b_max) >= (float)min_l * P.mask_level) {
                        if (a[j].p2 < 0) a[j].p2 = a[i].p;
                        if ((float)a[i].w < (float)a[j].w * P.drop_ratio && a[j].w - a[i].w >= P.min_seed_len << 1)
                            break;
                    }
                }
            }
            if (j == m) a[m++] = a[i];
        }
        // keep flags by sorted position (ord is free now), then squeeze
        for (int i = 0; i < n; ++i) ord[i] = 0;
        for (int i = 0; i < m; ++i) {
            ord[a[i].p] = 1;
            if (a[i].p2 >= 0) ord[a[i].p2] = 1;
        }
        n_keep = 0;
        for (int i = 0; i < n; ++i)
            if (ord[i]) ord2[n_keep++] = ord2[i];
    }
    uint64_t ns = 0;
    for (int i = 0; i < n_keep; ++i) ns += (uint64_t)chn[ord2[i]].n;
    P.n_out[r] = (uint64_t)n_keep;
    P.ns_out[r] = ns;
}

__global__ __launch_bounds__(256) void chain_write_kernel(ChainParams P) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= P.n_reads) return;
    const uint64_t c0 = P.chain_off[r], nc = P.chain_off[r + 1] - c0;
    if (nc == 0) return;
    const uint64_t S = P.occ_off[P.intv_off[r]];
    const uint32_t* ord2 = P.ord2 + S;
    const ChainRec* chn = P.chn + S;
    const SeedRec* seed = P.seed + S;
    const uint32_t* next = P.next + S;
    uint64_t so = P.seed_off[r];
    for (uint64_t i = 0; i < nc; ++i) {
        const ChainRec c = chn[ord2[i]];
        P.out_chain[c0 + i] = OutChain{c.pos, so, c.n, 0};
        uint32_t o = c.first;
        for (int j = 0; j < c.n; ++j, o = next[o]) P.out_seed[so++] = seed[o];
    }
}

}  // namespace smem

extern "C" hipError_t smem_launch_chain_build(const smem::ChainParams* P, hipStream_t st) {
    if (P->n_reads <= 0) return hipSuccess;
    hipLaunchKernelGGL(smem::chain_build_kernel, dim3((P->n_reads + 255) / 256), dim3(256), 0, st, *P);
    return hipGetLastError();
}

extern "C" hipError_t smem_launch_chain_write(const smem::ChainParams* P, hipStream_t st) {
    if (P->n_reads <= 0) return hipSuccess;
    hipLaunchKernelGGL(smem::chain_write_kernel, dim3((P->n_reads + 255) / 256), dim3(256), 0, st, *P);
    return hipGetLastError();
}
