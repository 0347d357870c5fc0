// bwt_build_gpu.hip — FM-index construction on the GPU (SURVEY.md §8(f) item 2:
// index provisioning on the box).  Produces exactly the .bwt that
// `bwa index -a is` writes (software/bwtindex.c:187; same bytes as the CPU
// SA-IS builder in bwt_build.c), so a multi-Gbp synthetic reference can be
// indexed in seconds inside a benchmark run instead of an hour of CPU.
//
// Algorithm: prefix doubling (Manber–Myers) with LSD radix sorts.
//   text   T = forward + reverse complement (software/bntseq.c:303-309), n symbols
//   pass 0 key(i) = T[i..i+20], 3 bits per symbol (symbol+1, 0 past the end,
//          so a suffix that ends sorts first — the $ convention)
//   pass h key(i) = rank(i) << 32 | rank(i+h)   (rank 0 past the end)
//   ranks  = 1 + index of the first suffix of the equal-key group
//   stop when every group is a singleton.
// Then BWT row 0 is the $ suffix (char T[n-1]), row r>0 the r-th suffix;
// primary = the row of suffix 0, which is dropped from the stored string
// (software/is.c:215-220), and the Occ checkpoints are interleaved every 128
// symbols (software/bwtindex.c:128-150).
//
// Limits: n = 2 x genome < 2^32 - 1 (32-bit suffix positions and ranks).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include <stdlib.h>
#include "smem_gpu.h"

namespace {

constexpr int K0 = 21;  // symbols in the first key (21 x 3 bits = 63 bits)

__global__ void make_text(const uint8_t* __restrict__ fwd, uint64_t nf, uint8_t* __restrict__ T) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= nf) return;
    const uint8_t c = fwd[i];
    T[i] = c;
    T[2 * nf - 1 - i] = (uint8_t)(3 - c);
}

__global__ void init_keys(const uint8_t* __restrict__ T, uint64_t n, uint64_t* __restrict__ key, uint32_t* __restrict__ val) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t k = 0;
#pragma unroll
    for (int d = 0; d < K0; ++d) {
        const uint64_t p = i + d;
        k = (k << 3) | (p < n ? (uint64_t)(T[p] + 1) : 0ull);
    }
    key[i] = k;
    val[i] = (uint32_t)i;
}

// head[i] = i if key differs from its predecessor (group start), else 0
__global__ void mark_heads(const uint64_t* __restrict__ key, uint64_t n, uint32_t* __restrict__ head,
                           unsigned long long* __restrict__ n_groups) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    bool h = false;
    if (i < n) {
        h = (i == 0) || key[i] != key[i - 1];
        head[i] = h ? (uint32_t)i : 0u;
    }
    const unsigned long long m = __ballot(h);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(n_groups, (unsigned long long)__popcll(m));
}

// rank[sa[i]] = group start + 1
__global__ void scatter_rank(const uint32_t* __restrict__ gs, const uint32_t* __restrict__ sa, uint64_t n,
                             uint32_t* __restrict__ rank) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i < n) rank[sa[i]] = gs[i] + 1;
}

__global__ void next_keys(const uint32_t* __restrict__ sa, const uint32_t* __restrict__ rank, uint64_t n, uint64_t h,
                          uint64_t* __restrict__ key) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t s = sa[i];
    const uint64_t r2 = s + h < n ? rank[s + h] : 0u;
    key[i] = ((uint64_t)rank[s] << 32) | r2;
}

// one thread per 32-bit word of the $-free BWT string; also per-word base counts
template <typename SA>
__global__ void pack_bwt(const uint8_t* __restrict__ T, const SA* __restrict__ sa, uint64_t n,
                         uint64_t primary, uint32_t* __restrict__ words, uint32_t* __restrict__ wcnt) {
    const uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t nw = (n + 15) >> 4;
    if (w >= nw) return;
    uint32_t x = 0, c4 = 0;
    for (int d = 0; d < 16; ++d) {
        const uint64_t j = w * 16 + d;  // position in the stored string
        uint32_t b = 0;
        if (j < n) {
            const uint64_t row = j < primary ? j : j + 1;  // skip the $ row
            b = row == 0 ? T[n - 1] : T[sa[row - 1] - 1];  // row 0: the $ suffix
            c4 += 1u << (8 * b);
        }
        x |= b << ((15 - d) << 1);
    }
    words[w] = x;
    wcnt[w] = c4;  // 4 x 8-bit counts (<= 16 each)
}

// per-bucket (128 symbols) counts, split per base for the scans
__global__ void bucket_counts(const uint32_t* __restrict__ wcnt, uint64_t nw, uint64_t nb, uint64_t* __restrict__ bc) {
    const uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (b >= nb) return;
    uint32_t c[4] = {0, 0, 0, 0};
    for (uint64_t w = b * 8; w < b * 8 + 8 && w < nw; ++w) {
        const uint32_t x = wcnt[w];
        c[0] += x & 0xff; c[1] += (x >> 8) & 0xff; c[2] += (x >> 16) & 0xff; c[3] += x >> 24;
    }
    for (int k = 0; k < 4; ++k) bc[k * nb + b] = c[k];
}

// interleave: bucket b at 16*b = 4 x u64 cumulative counts + up to 8 words
__global__ void interleave(const uint32_t* __restrict__ words, uint64_t nw, const uint64_t* __restrict__ cum, uint64_t nb,
                           uint32_t* __restrict__ out, uint64_t out_words) {
    const uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (b > nb) return;
    uint64_t* o64;
    if (b == nb) {  // trailing count block
        o64 = reinterpret_cast<uint64_t*>(out + (out_words - 8));
    } else {
        o64 = reinterpret_cast<uint64_t*>(out + 16 * b);
        for (uint64_t w = b * 8; w < b * 8 + 8 && w < nw; ++w) out[16 * b + 8 + (w - b * 8)] = words[w];
    }
    for (int k = 0; k < 4; ++k) o64[k] = cum[k * (nb + 1) + b];
}

struct Buf {
    void* p = nullptr;
    ~Buf() { if (p) (void)hipFree(p); }
};

}  // namespace

#define GB_TRY(x)                                                                          \
    do {                                                                                   \
        hipError_t _e = (x);                                                               \
        if (_e != hipSuccess) {                                                            \
            fprintf(stderr, "[smem_bwt_build_gpu] %s: %s\n", #x, hipGetErrorString(_e));   \
            return _e == hipErrorOutOfMemory ? SMEM_E_NOMEM : SMEM_E_DEVICE;               \
        }                                                                                  \
    } while (0)

static inline unsigned blocks(uint64_t n, unsigned t = 256) { return (unsigned)((n + t - 1) / t); }

// sampled SA (software/bwt.c:80-102): row r holds SA = (r == 0 ? n : sa[r-1]);
// samples at rows i * intv, i >= 1 (sa[0] = -1 is set on the host)
template <typename SA>
__global__ void sample_sa(const SA* __restrict__ sa, uint64_t n_sa, uint64_t intv, uint64_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x + 1;
    if (i < n_sa) out[i] = sa[i * intv - 1];
}

// Shared tail of both builders: BWT string from the suffix array, Occ
// checkpoints interleaved every 128 symbols (software/bwtindex.c:128-150), the
// sampled SA (software/bwt.c:80-102), copies to the host.  sa[p] is the text
// position of the p-th smallest non-empty suffix (row p + 1; row 0 is $).
template <typename SA>
static int finish_build(hipStream_t st, const uint8_t* T, const SA* sa, uint64_t n, uint64_t primary, int sa_intv,
                        smem_index_t* idx, smem_sa_t* sa_out) {
    if (sa_out) {
        const uint64_t intv = (uint64_t)sa_intv, n_sa = (n + intv) / intv;
        Buf bS;
        GB_TRY(hipMalloc(&bS.p, 8 * (n_sa + 1)));
        GB_TRY(hipMemsetAsync(bS.p, 0, 8 * (n_sa + 1), st));
        if (n_sa > 1) sample_sa<<<blocks(n_sa - 1), 256, 0, st>>>(sa, n_sa, intv, (uint64_t*)bS.p);
        memset(sa_out, 0, sizeof(*sa_out));
        sa_out->sa = (uint64_t*)malloc(8 * (n_sa + 1));
        if (!sa_out->sa) return SMEM_E_NOMEM;
        sa_out->owns = 1;
        GB_TRY(hipMemcpyAsync(sa_out->sa, bS.p, 8 * (n_sa + 1), hipMemcpyDeviceToHost, st));
        GB_TRY(hipStreamSynchronize(st));
        sa_out->sa[0] = (uint64_t)-1;
        sa_out->sa_intv = intv;
        sa_out->n_sa = n_sa;
        sa_out->seq_len = n;
    }
    const uint64_t nw = (n + 15) >> 4, nb = (n + 127) >> 7;
    Buf bW, bBc, bCum, bIn, bTmp;
    GB_TRY(hipMalloc(&bW.p, nw * 8 + 64));
    uint32_t* words = (uint32_t*)bW.p;
    uint32_t* wcnt = words + nw;
    pack_bwt<<<blocks(nw), 256, 0, st>>>(T, sa, n, primary, words, wcnt);
    GB_TRY(hipMalloc(&bBc.p, 4 * nb * 8 + 64));
    uint64_t* bc = (uint64_t*)bBc.p;
    bucket_counts<<<blocks(nb), 256, 0, st>>>(wcnt, nw, nb, bc);
    // exclusive sums over nb+1 entries (a zero tail makes entry nb the total)
    GB_TRY(hipMalloc(&bCum.p, 4 * (nb + 1) * 8));
    GB_TRY(hipMalloc(&bIn.p, 4 * (nb + 1) * 8));
    uint64_t* cum = (uint64_t*)bCum.p;
    uint64_t* in1 = (uint64_t*)bIn.p;
    size_t tmp_bytes = 0;
    GB_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, in1, cum, nb + 1, st));
    GB_TRY(hipMalloc(&bTmp.p, tmp_bytes + 256));
    for (int k = 0; k < 4; ++k) {
        GB_TRY(hipMemcpyAsync(in1 + k * (nb + 1), bc + k * nb, nb * 8, hipMemcpyDeviceToDevice, st));
        GB_TRY(hipMemsetAsync(in1 + k * (nb + 1) + nb, 0, 8, st));
        size_t tb = tmp_bytes + 256;
        GB_TRY(hipcub::DeviceScan::ExclusiveSum(bTmp.p, tb, in1 + k * (nb + 1), cum + k * (nb + 1), nb + 1, st));
    }
    const uint64_t n_occ = nb + 1;
    const uint64_t out_words = nw + n_occ * 8;
    Buf bOut;
    GB_TRY(hipMalloc(&bOut.p, (out_words + 16) * 4));
    GB_TRY(hipMemsetAsync(bOut.p, 0, (out_words + 16) * 4, st));
    interleave<<<blocks(nb + 1), 256, 0, st>>>(words, nw, cum, nb, (uint32_t*)bOut.p, out_words);
    uint64_t tot[4];
    for (int k = 0; k < 4; ++k) GB_TRY(hipMemcpyAsync(&tot[k], cum + k * (nb + 1) + nb, 8, hipMemcpyDeviceToHost, st));
    uint32_t* host = (uint32_t*)calloc(out_words + 16, 4);
    if (!host) return SMEM_E_NOMEM;
    const hipError_t e = hipMemcpyAsync(host, bOut.p, out_words * 4, hipMemcpyDeviceToHost, st);
    if (e != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
        free(host);
        return SMEM_E_DEVICE;
    }
    idx->bwt = host;
    idx->bwt_size = out_words;
    idx->primary = primary;
    idx->L2[0] = 0;
    for (int k = 0; k < 4; ++k) idx->L2[k + 1] = idx->L2[k] + tot[k];
    idx->seq_len = n;
    idx->owns = 1;
    if (idx->L2[4] != n) {
        fprintf(stderr, "[smem_bwt_build_gpu] count mismatch: %llu != %llu\n", (unsigned long long)idx->L2[4],
                (unsigned long long)n);
        free(host);
        memset(idx, 0, sizeof(*idx));
        return SMEM_E_INTERNAL;
    }
    if (sa_out) {
        sa_out->primary = primary;
        memcpy(sa_out->L2, idx->L2, sizeof(idx->L2));
    }
    return SMEM_OK;
}

static int upload_text(int device, const uint8_t* fwd, uint64_t n_fwd, hipStream_t* st, Buf& bT) {
    for (uint64_t i = 0; i < n_fwd; ++i)
        if (fwd[i] > 3) return SMEM_E_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return SMEM_E_DEVICE;
    GB_TRY(hipSetDevice(device));
    GB_TRY(hipStreamCreateWithFlags(st, hipStreamNonBlocking));
    const uint64_t n = 2 * n_fwd;
    GB_TRY(hipMalloc(&bT.p, n + 64));
    GB_TRY(hipMemsetAsync(bT.p, 0, n + 64, *st));
    Buf bF;
    GB_TRY(hipMalloc(&bF.p, n_fwd));
    GB_TRY(hipMemcpyAsync(bF.p, fwd, n_fwd, hipMemcpyHostToDevice, *st));
    make_text<<<blocks(n_fwd), 256, 0, *st>>>((const uint8_t*)bF.p, n_fwd, (uint8_t*)bT.p);
    GB_TRY(hipStreamSynchronize(*st));
    return SMEM_OK;
}

struct StreamGuard {
    hipStream_t s = nullptr;
    ~StreamGuard() { if (s) (void)hipStreamDestroy(s); }
};

// Prefix doubling over the whole text with 32-bit positions and ranks
// (n < 2^32 - 1).
static int build_gpu(int device, const uint8_t* fwd, uint64_t n_fwd, int sa_intv, smem_index_t* idx, smem_sa_t* sa_out) {
    if (!fwd || !idx || n_fwd == 0) return SMEM_E_ARG;
    const uint64_t n = 2 * n_fwd;
    if (n + 1 >= 0xFFFFFFFEull) return SMEM_E_ARG;
    memset(idx, 0, sizeof(*idx));
    StreamGuard sg;
    Buf bT;
    int rc = upload_text(device, fwd, n_fwd, &sg.s, bT);
    if (rc != SMEM_OK) return rc;
    hipStream_t st = sg.s;
    const uint8_t* T = (const uint8_t*)bT.p;
    uint64_t primary = 0;
    Buf bSA;
    {
        Buf bK0, bK1, bV0, bV1, bRank, bHead, bTmp, bCnt;
        GB_TRY(hipMalloc(&bK0.p, n * 8));
        GB_TRY(hipMalloc(&bK1.p, n * 8));
        GB_TRY(hipMalloc(&bV0.p, n * 4));
        GB_TRY(hipMalloc(&bV1.p, n * 4));
        GB_TRY(hipMalloc(&bRank.p, n * 4));
        GB_TRY(hipMalloc(&bHead.p, n * 4));
        GB_TRY(hipMalloc(&bCnt.p, 64));
        hipcub::DoubleBuffer<uint64_t> keys((uint64_t*)bK0.p, (uint64_t*)bK1.p);
        hipcub::DoubleBuffer<uint32_t> vals((uint32_t*)bV0.p, (uint32_t*)bV1.p);
        size_t sort_tmp = 0, scan_tmp = 0;
        GB_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_tmp, keys, vals, n, 0, 64, st));
        GB_TRY(hipcub::DeviceScan::InclusiveScan(nullptr, scan_tmp, (uint32_t*)bHead.p, (uint32_t*)bK1.p,
                                                 hipcub::Max(), n, st));
        const size_t tmp_bytes = std::max(sort_tmp, scan_tmp) + 256;
        GB_TRY(hipMalloc(&bTmp.p, tmp_bytes));
        unsigned long long* d_groups = (unsigned long long*)bCnt.p;
        uint32_t* rank = (uint32_t*)bRank.p;
        uint32_t* head = (uint32_t*)bHead.p;

        init_keys<<<blocks(n), 256, 0, st>>>(T, n, keys.Current(), vals.Current());
        int key_bits = 63;
        for (uint64_t h = K0;; h *= 2) {
            size_t tb = tmp_bytes;
            GB_TRY(hipcub::DeviceRadixSort::SortPairs(bTmp.p, tb, keys, vals, n, 0, key_bits, st));
            GB_TRY(hipMemsetAsync(d_groups, 0, 8, st));
            mark_heads<<<blocks(n), 256, 0, st>>>(keys.Current(), n, head, d_groups);
            tb = tmp_bytes;
            uint32_t* gs = reinterpret_cast<uint32_t*>(keys.Alternate());  // free until the next sort
            GB_TRY(hipcub::DeviceScan::InclusiveScan(bTmp.p, tb, head, gs, hipcub::Max(), n, st));
            scatter_rank<<<blocks(n), 256, 0, st>>>(gs, vals.Current(), n, rank);
            unsigned long long groups = 0;
            GB_TRY(hipMemcpyAsync(&groups, d_groups, 8, hipMemcpyDeviceToHost, st));
            GB_TRY(hipStreamSynchronize(st));
            if (groups == n) break;
            if (h > n) {
                fprintf(stderr, "[smem_bwt_build_gpu] no convergence: %llu groups of %llu suffixes at h=%llu\n",
                        groups, (unsigned long long)n, (unsigned long long)h);
                return SMEM_E_INTERNAL;
            }
            next_keys<<<blocks(n), 256, 0, st>>>(vals.Current(), rank, n, h, keys.Current());
            key_bits = 64;
        }
        // primary = 1 + position of suffix 0 = rank[0] (rank = position + 1)
        uint32_t r0 = 0;
        GB_TRY(hipMemcpyAsync(&r0, rank, 4, hipMemcpyDeviceToHost, st));
        GB_TRY(hipStreamSynchronize(st));
        primary = r0;  // rows: 0 = $, then suffix at sorted position p -> row p+1
        // keep the sorted positions, free the rest
        if (vals.Current() == (uint32_t*)bV0.p) std::swap(bSA.p, bV0.p);
        else std::swap(bSA.p, bV1.p);
    }
    return finish_build(st, T, (const uint32_t*)bSA.p, n, primary, sa_intv, idx, sa_out);
}

// ---------------------------------------------------------------------------
// Bucketed builder with 64-bit positions and ranks, for texts of 2^32
// symbols and more (both strands of a human-size genome: 6.2 G).  Whole-text
// prefix doubling would need ~40 B per suffix of sort buffers (250 GB at
// human size) and more than 2^31 items per radix sort.  Instead:
//   A. suffixes are binned by their first PB symbols; runs of consecutive
//      bins of at most SB_MAX suffixes (super-buckets) are gathered one at a
//      time, radix-sorted by their first K0 symbols and written to their
//      final SA range; ranks (1 + first position of the equal-key group) are
//      scattered and the positions of non-singleton groups are appended, in
//      SA order, to the unresolved list U;
//   B. Larsson–Sadakane doubling on U only: key = (group index, rank[s + h]),
//      a sort, new ranks, singletons dropped, h doubles — until U is empty.
//      Every rank is at depth >= h throughout, so (rank_h[s], rank_h[s + h])
//      orders at depth 2h.
// Same order as build_gpu (symbol + 1, 0 past the end: a suffix that ends
// sorts first), hence the same bytes.  Memory: 17 B per suffix + buffers.
// ---------------------------------------------------------------------------
constexpr int PB = 6;                        // bin prefix symbols (4^6 full bins)
constexpr uint64_t SB_MAX = 1ull << 28;      // suffixes per super-bucket
constexpr int BIN_BITS = 3 * PB;             // bins are 3-bit keys (past-end = 0)

__device__ __forceinline__ uint64_t sym3(const uint8_t* T, uint64_t n, uint64_t p) {
    return p < n ? (uint64_t)T[p] + 1 : 0ull;
}

// histogram of the 3-bit PB-symbol prefixes: full-length prefixes in LDS
// (4^PB counters) per block, the PB-1 short ones straight to global
__global__ void __launch_bounds__(256) bin_hist(const uint8_t* __restrict__ T, uint64_t n,
                                                unsigned long long* __restrict__ hist) {
    __shared__ uint32_t h[1 << (2 * PB)];
    for (int i = threadIdx.x; i < (1 << (2 * PB)); i += blockDim.x) h[i] = 0;
    __syncthreads();
    constexpr int PER = 64;  // positions per thread
    const uint64_t p0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * PER;
    if (p0 < n) {
        uint32_t code = 0;
        for (int d = 0; d < PB - 1; ++d) code = (code << 2) | (p0 + d < n ? T[p0 + d] : 0);
        for (int k = 0; k < PER && p0 + k < n; ++k) {
            const uint64_t p = p0 + k;
            code = ((code << 2) | (p + PB - 1 < n ? T[p + PB - 1] : 0)) & ((1u << (2 * PB)) - 1);
            if (p + PB <= n) {
                atomicAdd(&h[code], 1u);
            } else {
                uint64_t b = 0;
                for (int d = 0; d < PB; ++d) b = (b << 3) | sym3(T, n, p + d);
                atomicAdd(&hist[b], 1ull);
            }
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < (1 << (2 * PB)); c += blockDim.x) {
        const uint32_t v = h[c];
        if (!v) continue;
        uint64_t b = 0;
        for (int d = PB - 1; d >= 0; --d) b = (b << 3) | (((c >> (2 * d)) & 3) + 1);
        atomicAdd(&hist[b], (unsigned long long)v);
    }
}

// Counting sort of all suffixes by bin into the SA array (one pass; the
// order inside a bin is arbitrary, the super-bucket sort fixes it).  Block b
// takes positions [b SC, (b + 1) SC): an LDS histogram of its full-length
// prefixes, one global reservation per (block, bin), then the positions.
constexpr int SC = 1 << 18;  // positions per block
__global__ void __launch_bounds__(256) bin_scatter(const uint8_t* __restrict__ T, uint64_t n,
                                                   unsigned long long* __restrict__ cursor, uint64_t* __restrict__ sa) {
    constexpr int NC = 1 << (2 * PB);
    __shared__ uint32_t cnt[NC];
    __shared__ uint64_t base[NC];
    for (int i = threadIdx.x; i < NC; i += blockDim.x) cnt[i] = 0;
    __syncthreads();
    constexpr int PER = SC / 256;
    const uint64_t p0 = (uint64_t)blockIdx.x * SC + (uint64_t)threadIdx.x * PER;
    const uint64_t last = n >= PB ? n - PB : 0;  // positions <= last have all PB symbols
    auto walk = [&](auto&& f) {
        if (n < PB || p0 > last) return;
        uint32_t code = 0;
        for (int d = 0; d < PB - 1; ++d) code = (code << 2) | T[p0 + d];
        for (int k = 0; k < PER && p0 + k <= last; ++k) {
            code = ((code << 2) | T[p0 + k + PB - 1]) & (NC - 1);
            f(code, p0 + k);
        }
    };
    walk([&](uint32_t c, uint64_t) { atomicAdd(&cnt[c], 1u); });
    __syncthreads();
    for (int c = threadIdx.x; c < NC; c += blockDim.x) {
        const uint32_t v = cnt[c];
        if (v) {
            uint64_t b = 0;
            for (int d = PB - 1; d >= 0; --d) b = (b << 3) | (((c >> (2 * d)) & 3) + 1);
            base[c] = atomicAdd(&cursor[b], (unsigned long long)v);
        }
        cnt[c] = 0;
    }
    __syncthreads();
    walk([&](uint32_t c, uint64_t p) { sa[base[c] + atomicAdd(&cnt[c], 1u)] = p; });
}

// the PB - 1 suffixes too short for a full prefix
__global__ void bin_scatter_tail(const uint8_t* __restrict__ T, uint64_t n, unsigned long long* __restrict__ cursor,
                                 uint64_t* __restrict__ sa) {
    const uint64_t p = (n >= PB ? n - PB + 1 : 0) + threadIdx.x;
    if (p >= n) return;
    uint64_t b = 0;
    for (int d = 0; d < PB; ++d) b = (b << 3) | sym3(T, n, p + d);
    sa[atomicAdd(&cursor[b], 1ull)] = p;
}

// a super-bucket's positions (SA rows [base, base + m)) with their K0-symbol keys
__global__ void sb_load(const uint8_t* __restrict__ T, uint64_t n, const uint64_t* __restrict__ sa, uint64_t base,
                        uint64_t m, uint64_t* __restrict__ key, uint64_t* __restrict__ pos) {
    const uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (j >= m) return;
    const uint64_t p = sa[base + j];
    uint64_t k = 0;
    for (int d = 0; d < K0; ++d) k = (k << 3) | sym3(T, n, p + d);
    key[j] = k;
    pos[j] = p;
}

// after the super-bucket sort: SA range, group heads (key changes)
__global__ void sb_place(const uint64_t* __restrict__ key, const uint64_t* __restrict__ pos, uint64_t m, uint64_t base,
                         uint64_t* __restrict__ sa, uint64_t* __restrict__ gstart) {
    const uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (j >= m) return;
    sa[base + j] = pos[j];
    gstart[j] = (j == 0 || key[j] != key[j - 1]) ? base + j + 1 : 0;  // 1 + group start (max-scanned)
}

// rank[s] = 1 + group start; flag non-singleton groups for U
__global__ void sb_rank(const uint64_t* __restrict__ key, const uint64_t* __restrict__ pos,
                        const uint64_t* __restrict__ gs, uint64_t m, uint64_t* __restrict__ rank,
                        uint8_t* __restrict__ flag) {
    const uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (j >= m) return;
    rank[pos[j]] = gs[j];
    const bool single = (j == 0 || key[j] != key[j - 1]) && (j + 1 == m || key[j + 1] != key[j]);
    flag[j] = single ? 0 : 1;
}

// round of B, step 1: head flags of U's groups (rank[s] - 1 == position)
__global__ void u_heads(const uint64_t* __restrict__ U, uint64_t m, const uint64_t* __restrict__ sa,
                        const uint64_t* __restrict__ rank, uint32_t* __restrict__ hf) {
    const uint64_t u = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (u >= m) return;
    const uint64_t p = U[u];
    hf[u] = rank[sa[p]] - 1 == p ? 1u : 0u;
}

// step 2: key = (group index, rank[s + h]) — group index < 2^30, ranks < 2^34
__global__ void u_keys(const uint64_t* __restrict__ U, uint64_t m, const uint32_t* __restrict__ g,
                       const uint64_t* __restrict__ sa, const uint64_t* __restrict__ rank, uint64_t n, uint64_t h,
                       uint64_t* __restrict__ key, uint64_t* __restrict__ val) {
    const uint64_t u = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (u >= m) return;
    const uint64_t s = sa[U[u]];
    const uint64_t r2 = s + h < n ? rank[s + h] : 0;
    key[u] = ((uint64_t)(g[u] - 1) << 34) | r2;
    val[u] = s;
}

// step 3: write back in sorted order, mark new group heads
__global__ void u_place(const uint64_t* __restrict__ U, uint64_t m, const uint64_t* __restrict__ key,
                        const uint64_t* __restrict__ val, uint64_t* __restrict__ sa, uint64_t* __restrict__ gstart) {
    const uint64_t u = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (u >= m) return;
    sa[U[u]] = val[u];
    gstart[u] = (u == 0 || key[u] != key[u - 1]) ? U[u] + 1 : 0;
}

// step 4: new ranks, keep the members of non-singleton groups
__global__ void u_rank(uint64_t m, const uint64_t* __restrict__ key, const uint64_t* __restrict__ val,
                       const uint64_t* __restrict__ gs, uint64_t* __restrict__ rank, uint8_t* __restrict__ flag) {
    const uint64_t u = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (u >= m) return;
    rank[val[u]] = gs[u];
    const bool single = (u == 0 || key[u] != key[u - 1]) && (u + 1 == m || key[u + 1] != key[u]);
    flag[u] = single ? 0 : 1;
}

static int build_gpu_large(int device, const uint8_t* fwd, uint64_t n_fwd, int sa_intv, smem_index_t* idx,
                           smem_sa_t* sa_out) {
    if (!fwd || !idx || n_fwd == 0) return SMEM_E_ARG;
    const uint64_t n = 2 * n_fwd;
    if (n >= (1ull << 34) - 2) return SMEM_E_ARG;
    memset(idx, 0, sizeof(*idx));
    StreamGuard sg;
    Buf bT;
    int rc = upload_text(device, fwd, n_fwd, &sg.s, bT);
    if (rc != SMEM_OK) return rc;
    hipStream_t st = sg.s;
    const uint8_t* T = (const uint8_t*)bT.p;
    Buf bSA;
    uint64_t primary = 0;
    {
        Buf bRank, bHist, bCnt;
        GB_TRY(hipMalloc(&bSA.p, n * 8));
        GB_TRY(hipMalloc(&bRank.p, n * 8));
        uint64_t* sa = (uint64_t*)bSA.p;
        uint64_t* rank = (uint64_t*)bRank.p;
        const uint64_t n_bins = 1ull << BIN_BITS;
        GB_TRY(hipMalloc(&bHist.p, n_bins * 8));
        GB_TRY(hipMalloc(&bCnt.p, 64));
        unsigned long long* d_cnt = (unsigned long long*)bCnt.p;
        GB_TRY(hipMemsetAsync(bHist.p, 0, n_bins * 8, st));
        bin_hist<<<blocks((n + 63) / 64), 256, 0, st>>>(T, n, (unsigned long long*)bHist.p);
        uint64_t* hist = (uint64_t*)malloc(n_bins * 8);
        if (!hist) return SMEM_E_NOMEM;
        struct HostFree { void* p; ~HostFree() { free(p); } } hf_{hist};
        GB_TRY(hipMemcpyAsync(hist, bHist.p, n_bins * 8, hipMemcpyDeviceToHost, st));
        GB_TRY(hipStreamSynchronize(st));
        uint64_t big = 0, tot = 0;
        for (uint64_t b = 0; b < n_bins; ++b) big = std::max(big, hist[b]), tot += hist[b];
        if (tot != n) {
            fprintf(stderr, "[smem_bwt_build_gpu] bin histogram sums to %llu of %llu\n", (unsigned long long)tot,
                    (unsigned long long)n);
            return SMEM_E_INTERNAL;
        }
        // (test hook: SMEM_BUILD_SB_MAX shrinks the super-buckets)
        uint64_t sb_max = SB_MAX;
        if (const char* v = getenv("SMEM_BUILD_SB_MAX")) sb_max = std::max<uint64_t>(1, strtoull(v, nullptr, 10));
        uint64_t cap = std::max(std::min(sb_max, n), big);
        if (cap >= (1ull << 31)) return SMEM_E_CAPACITY;

        Buf bK0, bK1, bV0, bV1, bG, bFlag, bTmp, bU0, bU1;
        GB_TRY(hipMalloc(&bK0.p, cap * 8));
        GB_TRY(hipMalloc(&bK1.p, cap * 8));
        GB_TRY(hipMalloc(&bV0.p, cap * 8));
        GB_TRY(hipMalloc(&bV1.p, cap * 8));
        GB_TRY(hipMalloc(&bG.p, cap * 8));
        GB_TRY(hipMalloc(&bFlag.p, cap + 64));
        size_t t_sort = 0, t_scan = 0, t_sum = 0, t_sel = 0;
        {
            hipcub::DoubleBuffer<uint64_t> k((uint64_t*)bK0.p, (uint64_t*)bK1.p), v((uint64_t*)bV0.p, (uint64_t*)bV1.p);
            GB_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, t_sort, k, v, (int)cap, 0, 64, st));
            GB_TRY(hipcub::DeviceScan::InclusiveScan(nullptr, t_scan, (uint64_t*)bG.p, (uint64_t*)bG.p, hipcub::Max(),
                                                     (int)cap, st));
            GB_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, t_sum, (uint32_t*)bG.p, (uint32_t*)bG.p, (int)cap, st));
            GB_TRY(hipcub::DeviceSelect::Flagged(nullptr, t_sel, (uint64_t*)bV0.p, (uint8_t*)bFlag.p,
                                                 (uint64_t*)bV1.p, d_cnt, (int)cap, st));
            size_t t_sel2 = 0;
            GB_TRY(hipcub::DeviceSelect::Flagged(nullptr, t_sel2, hipcub::CountingInputIterator<uint64_t>(0),
                                                 (uint8_t*)bFlag.p, (uint64_t*)bV1.p, d_cnt, (int)cap, st));
            t_sel = std::max(t_sel, t_sel2);
        }
        size_t tmp_bytes = std::max(std::max(t_sort, t_scan), std::max(t_sum, t_sel)) + 256;
        GB_TRY(hipMalloc(&bTmp.p, tmp_bytes));
        uint64_t u_cap = std::max<uint64_t>(cap, 1 << 20), n_u = 0;
        GB_TRY(hipMalloc(&bU0.p, u_cap * 8));

        // A. every suffix to its bin's SA range (counting sort), then the
        // super-buckets, in bin (= SA) order
        {
            uint64_t* start = (uint64_t*)malloc(n_bins * 8);
            if (!start) return SMEM_E_NOMEM;
            uint64_t acc = 0;
            for (uint64_t b = 0; b < n_bins; ++b) start[b] = acc, acc += hist[b];
            const hipError_t e = hipMemcpyAsync(bHist.p, start, n_bins * 8, hipMemcpyHostToDevice, st);
            const hipError_t e2 = hipStreamSynchronize(st);
            free(start);
            GB_TRY(e);
            GB_TRY(e2);
            bin_scatter<<<(unsigned)((n + SC - 1) / SC), 256, 0, st>>>(T, n, (unsigned long long*)bHist.p, sa);
            bin_scatter_tail<<<1, 64, 0, st>>>(T, n, (unsigned long long*)bHist.p, sa);
            GB_TRY(hipGetLastError());
        }
        uint64_t base = 0;
        for (uint64_t blo = 0; blo < n_bins;) {
            uint64_t bhi = blo, m = 0;
            while (bhi < n_bins && (m + hist[bhi] <= cap)) m += hist[bhi++];
            if (m == 0) { blo = bhi; continue; }
            sb_load<<<blocks(m), 256, 0, st>>>(T, n, sa, base, m, (uint64_t*)bK0.p, (uint64_t*)bV0.p);
            hipcub::DoubleBuffer<uint64_t> k((uint64_t*)bK0.p, (uint64_t*)bK1.p), v((uint64_t*)bV0.p, (uint64_t*)bV1.p);
            size_t tb = tmp_bytes;
            GB_TRY(hipcub::DeviceRadixSort::SortPairs(bTmp.p, tb, k, v, (int)m, 0, 3 * K0, st));
            uint64_t* gs = (uint64_t*)bG.p;
            uint64_t* scr = k.Alternate();
            sb_place<<<blocks(m), 256, 0, st>>>(k.Current(), v.Current(), m, base, sa, scr);
            tb = tmp_bytes;
            GB_TRY(hipcub::DeviceScan::InclusiveScan(bTmp.p, tb, scr, gs, hipcub::Max(), (int)m, st));
            sb_rank<<<blocks(m), 256, 0, st>>>(k.Current(), v.Current(), gs, m, rank, (uint8_t*)bFlag.p);
            // append the non-singleton positions (base + j) to U, in order
            if (n_u + m > u_cap) {
                const uint64_t nc = std::max(u_cap * 2, n_u + m);
                Buf bN;
                GB_TRY(hipMalloc(&bN.p, nc * 8));
                GB_TRY(hipMemcpyAsync(bN.p, bU0.p, n_u * 8, hipMemcpyDeviceToDevice, st));
                std::swap(bN.p, bU0.p);
                GB_TRY(hipStreamSynchronize(st));
                u_cap = nc;
            }
            tb = tmp_bytes;
            GB_TRY(hipcub::DeviceSelect::Flagged(bTmp.p, tb, hipcub::CountingInputIterator<uint64_t>(base),
                                                 (uint8_t*)bFlag.p, (uint64_t*)bU0.p + n_u, d_cnt, (int)m, st));
            unsigned long long sel = 0;
            GB_TRY(hipMemcpyAsync(&sel, d_cnt, 8, hipMemcpyDeviceToHost, st));
            GB_TRY(hipStreamSynchronize(st));
            n_u += sel;
            base += m;
            blo = bhi;
        }
        if (base != n) return SMEM_E_INTERNAL;

        // B. doubling on the unresolved groups, all of U in one sort
        if (n_u >= (1ull << 31)) return SMEM_E_CAPACITY;
        if (n_u > cap) {
            cap = n_u;
            for (Buf* b : {&bK0, &bK1, &bV0, &bV1, &bG}) {
                GB_TRY(hipFree(b->p));
                b->p = nullptr;
                GB_TRY(hipMalloc(&b->p, cap * 8));
            }
            GB_TRY(hipFree(bFlag.p));
            bFlag.p = nullptr;
            GB_TRY(hipMalloc(&bFlag.p, cap + 64));
            size_t a = 0, b2 = 0, c = 0, d = 0;
            hipcub::DoubleBuffer<uint64_t> k((uint64_t*)bK0.p, (uint64_t*)bK1.p), v((uint64_t*)bV0.p, (uint64_t*)bV1.p);
            GB_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, a, k, v, (int)cap, 0, 64, st));
            GB_TRY(hipcub::DeviceScan::InclusiveScan(nullptr, b2, (uint64_t*)bG.p, (uint64_t*)bG.p, hipcub::Max(),
                                                     (int)cap, st));
            GB_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, c, (uint32_t*)bG.p, (uint32_t*)bG.p, (int)cap, st));
            GB_TRY(hipcub::DeviceSelect::Flagged(nullptr, d, (uint64_t*)bV0.p, (uint8_t*)bFlag.p, (uint64_t*)bV1.p,
                                                 d_cnt, (int)cap, st));
            const size_t need = std::max(std::max(a, b2), std::max(c, d)) + 256;
            if (need > tmp_bytes) {
                GB_TRY(hipFree(bTmp.p));
                bTmp.p = nullptr;
                GB_TRY(hipMalloc(&bTmp.p, need));
                tmp_bytes = need;
            }
        }
        GB_TRY(hipMalloc(&bU1.p, std::max<uint64_t>(n_u, 1) * 8));
        uint64_t* U = (uint64_t*)bU0.p;
        uint64_t* U2 = (uint64_t*)bU1.p;
        for (uint64_t h = K0; n_u > 0; h *= 2) {
            if (h > n) {
                fprintf(stderr, "[smem_bwt_build_gpu] no convergence: %llu unresolved at h=%llu\n",
                        (unsigned long long)n_u, (unsigned long long)h);
                return SMEM_E_INTERNAL;
            }
            const uint64_t m = n_u;
            uint32_t* hf = (uint32_t*)bG.p;
            uint32_t* g = (uint32_t*)bK1.p;  // consumed by u_keys before the sort reuses it
            u_heads<<<blocks(m), 256, 0, st>>>(U, m, sa, rank, hf);
            size_t tb = tmp_bytes;
            GB_TRY(hipcub::DeviceScan::InclusiveSum(bTmp.p, tb, hf, g, (int)m, st));
            u_keys<<<blocks(m), 256, 0, st>>>(U, m, g, sa, rank, n, h, (uint64_t*)bK0.p, (uint64_t*)bV0.p);
            hipcub::DoubleBuffer<uint64_t> k((uint64_t*)bK0.p, (uint64_t*)bK1.p), v((uint64_t*)bV0.p, (uint64_t*)bV1.p);
            tb = tmp_bytes;
            GB_TRY(hipcub::DeviceRadixSort::SortPairs(bTmp.p, tb, k, v, (int)m, 0, 64, st));
            uint64_t* scr = (uint64_t*)bG.p;
            u_place<<<blocks(m), 256, 0, st>>>(U, m, k.Current(), v.Current(), sa, scr);
            uint64_t* gs = k.Alternate();
            tb = tmp_bytes;
            GB_TRY(hipcub::DeviceScan::InclusiveScan(bTmp.p, tb, scr, gs, hipcub::Max(), (int)m, st));
            u_rank<<<blocks(m), 256, 0, st>>>(m, k.Current(), v.Current(), gs, rank, (uint8_t*)bFlag.p);
            tb = tmp_bytes;
            GB_TRY(hipcub::DeviceSelect::Flagged(bTmp.p, tb, U, (uint8_t*)bFlag.p, U2, d_cnt, (int)m, st));
            unsigned long long sel = 0;
            GB_TRY(hipMemcpyAsync(&sel, d_cnt, 8, hipMemcpyDeviceToHost, st));
            GB_TRY(hipStreamSynchronize(st));
            std::swap(U, U2);
            n_u = sel;
        }
        uint64_t r0 = 0;
        GB_TRY(hipMemcpyAsync(&r0, rank, 8, hipMemcpyDeviceToHost, st));
        GB_TRY(hipStreamSynchronize(st));
        primary = r0;
    }
    return finish_build(st, T, (const uint64_t*)bSA.p, n, primary, sa_intv, idx, sa_out);
}

// the 32-bit builder while positions fit, the bucketed one beyond
static int build_any(int device, const uint8_t* fwd, uint64_t n_fwd, int sa_intv, smem_index_t* idx, smem_sa_t* sa,
                     int large) {
    if (large || 2 * n_fwd + 1 >= 0xFFFFFFFEull) return build_gpu_large(device, fwd, n_fwd, sa_intv, idx, sa);
    return build_gpu(device, fwd, n_fwd, sa_intv, idx, sa);
}

extern "C" int smem_bwt_build_gpu(int device, const uint8_t* fwd, uint64_t n_fwd, smem_index_t* idx) {
    return build_any(device, fwd, n_fwd, 0, idx, nullptr, 0);
}

static int build_sa_checked(int device, const uint8_t* fwd, uint64_t n_fwd, int sa_intv, smem_index_t* idx,
                            smem_sa_t* sa, int large) {
    if (!sa || sa_intv <= 0 || (sa_intv & (sa_intv - 1))) return SMEM_E_ARG;
    const int rc = build_any(device, fwd, n_fwd, sa_intv, idx, sa, large);
    if (rc != SMEM_OK) {
        smem_sa_free(sa);
        smem_index_free(idx);
    }
    return rc;
}

extern "C" int smem_bwt_build_gpu_sa(int device, const uint8_t* fwd, uint64_t n_fwd, int sa_intv, smem_index_t* idx,
                                     smem_sa_t* sa) {
    return build_sa_checked(device, fwd, n_fwd, sa_intv, idx, sa, 0);
}

extern "C" int smem_bwt_build_gpu_large(int device, const uint8_t* fwd, uint64_t n_fwd, int sa_intv,
                                        smem_index_t* idx, smem_sa_t* sa) {
    if (sa) return build_sa_checked(device, fwd, n_fwd, sa_intv, idx, sa, 1);
    const int rc = build_any(device, fwd, n_fwd, 0, idx, nullptr, 1);
    if (rc != SMEM_OK) smem_index_free(idx);
    return rc;
}
