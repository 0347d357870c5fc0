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
__global__ void pack_bwt(const uint8_t* __restrict__ T, const uint32_t* __restrict__ sa, uint64_t n,
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
__global__ void sample_sa(const uint32_t* __restrict__ sa, uint64_t n_sa, uint64_t intv, uint64_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x + 1;
    if (i < n_sa) out[i] = sa[i * intv - 1];
}

static int build_gpu(int device, const uint8_t* fwd, uint64_t n_fwd, int sa_intv, smem_index_t* idx, smem_sa_t* sa_out) {
    if (!fwd || !idx || n_fwd == 0) return SMEM_E_ARG;
    const uint64_t n = 2 * n_fwd;
    if (n + 1 >= 0xFFFFFFFEull) return SMEM_E_ARG;
    for (uint64_t i = 0; i < n_fwd; ++i)
        if (fwd[i] > 3) return SMEM_E_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return SMEM_E_DEVICE;
    GB_TRY(hipSetDevice(device));
    memset(idx, 0, sizeof(*idx));
    hipStream_t st;
    GB_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    struct StreamGuard { hipStream_t s; ~StreamGuard() { (void)hipStreamDestroy(s); } } sg{st};

    Buf bT, bK0, bK1, bV0, bV1, bRank, bHead, bTmp, bCnt;
    GB_TRY(hipMalloc(&bT.p, n + 16));
    {
        Buf bF;
        GB_TRY(hipMalloc(&bF.p, n_fwd));
        GB_TRY(hipMemcpyAsync(bF.p, fwd, n_fwd, hipMemcpyHostToDevice, st));
        make_text<<<blocks(n_fwd), 256, 0, st>>>((const uint8_t*)bF.p, n_fwd, (uint8_t*)bT.p);
        GB_TRY(hipStreamSynchronize(st));
    }
    uint8_t* T = (uint8_t*)bT.p;
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
    const uint64_t nb_all = (n + 127) >> 7;
    size_t sum_tmp = 0;
    GB_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, sum_tmp, (uint64_t*)bK0.p, (uint64_t*)bK1.p, nb_all + 1, st));
    const size_t tmp_bytes = std::max(std::max(sort_tmp, scan_tmp), sum_tmp) + 256;
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
    const uint32_t* sa = vals.Current();
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
    // primary = 1 + position of suffix 0 = rank[0] (rank = position + 1)
    uint32_t r0 = 0;
    GB_TRY(hipMemcpyAsync(&r0, rank, 4, hipMemcpyDeviceToHost, st));
    GB_TRY(hipStreamSynchronize(st));
    const uint64_t primary = r0;  // rows: 0 = $, then suffix at sorted position p -> row p+1
    // free the sort buffers we no longer need, keep T, sa
    const uint64_t nw = (n + 15) >> 4, nb = (n + 127) >> 7;
    uint32_t* words = (uint32_t*)keys.Alternate();            // reuse: nw*4 <= n*8
    uint32_t* wcnt = words + nw;                               // nw*4 more, still within n*8
    pack_bwt<<<blocks(nw), 256, 0, st>>>(T, sa, n, primary, words, wcnt);
    uint64_t* bc = keys.Current();                             // 4*nb u64 <= n*8
    bucket_counts<<<blocks(nb), 256, 0, st>>>(wcnt, nw, nb, bc);
    // exclusive sums over nb+1 entries (a zero tail makes entry nb the total)
    Buf bCum, bIn;
    GB_TRY(hipMalloc(&bCum.p, 4 * (nb + 1) * 8));
    GB_TRY(hipMalloc(&bIn.p, 4 * (nb + 1) * 8));
    uint64_t* cum = (uint64_t*)bCum.p;
    uint64_t* in1 = (uint64_t*)bIn.p;
    for (int k = 0; k < 4; ++k) {
        GB_TRY(hipMemcpyAsync(in1 + k * (nb + 1), bc + k * nb, nb * 8, hipMemcpyDeviceToDevice, st));
        GB_TRY(hipMemsetAsync(in1 + k * (nb + 1) + nb, 0, 8, st));
        size_t tb = tmp_bytes;
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
    GB_TRY(hipMemcpyAsync(host, bOut.p, out_words * 4, hipMemcpyDeviceToHost, st));
    GB_TRY(hipStreamSynchronize(st));
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

extern "C" int smem_bwt_build_gpu(int device, const uint8_t* fwd, uint64_t n_fwd, smem_index_t* idx) {
    return build_gpu(device, fwd, n_fwd, 0, idx, nullptr);
}

extern "C" int smem_bwt_build_gpu_sa(int device, const uint8_t* fwd, uint64_t n_fwd, int sa_intv, smem_index_t* idx,
                                     smem_sa_t* sa) {
    if (!sa || sa_intv <= 0 || (sa_intv & (sa_intv - 1))) return SMEM_E_ARG;
    const int rc = build_gpu(device, fwd, n_fwd, sa_intv, idx, sa);
    if (rc != SMEM_OK) {
        smem_sa_free(sa);
        smem_index_free(idx);
    }
    return rc;
}
