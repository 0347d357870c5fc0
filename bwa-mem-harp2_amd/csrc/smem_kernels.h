// smem_kernels.h — device-side parameter blocks shared by smem_kernels.hip
// (kernels) and smem_gpu.cpp (runtime).  Not part of the public C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SMEM_OVERFLOW 0xFFFFFFFFu

namespace smem {

// bwtintv_t (software/bwt.h:60-62)
struct Intv {
    uint64_t x0, x1, x2, info;
};

// One smem_next2 call as the seeding kernel logs it: the call's raw region
// holds m_n matches then s_n sub-matches, each in the order bwt_smem1 pushed
// them (the reverse of their final order); max_len is the longest match.
struct CallRec {
    uint32_t m_n, s_n, ori_start, max_len;
};

struct SeedParams {
    const uint32_t* bwt;       // interleaved BWT + Occ, resident in HBM (reference layout)
    const uint32_t* occ64;     // the same index as 32-B buckets per 64 symbols (smem_launch_occ64)
    const uint32_t* occ192;    // the same index as 64-B lines of 192 symbols (smem_launch_occ192; variant 10)
    uint64_t primary;
    uint64_t L2[5];
    const uint8_t* codes;      // reads, concatenated nt4 codes (+32 B pad)
    const uint64_t* offs;      // n_reads + 1
    const int32_t* read_ids;   // work item -> read (nullptr: identity)
    int n_items;
    int min_seed_len, split_len_init, split_width, start_width;
    Intv* out_intv;            // raw lists [item][cap_intv]
    uint32_t cap_intv;
    CallRec* out_call;         // [item][cap_calls]
    uint32_t cap_calls;
    uint32_t* n_intv;          // [item] raw intervals, or SMEM_OVERFLOW
    uint32_t* n_calls;         // [item]
    uint64_t* s_intv;          // [read] intervals smem_next2 returns for the read (compaction sizes)
    uint64_t* s_calls;         // [read] smem_next2 lists of the read
    int32_t* ovf_count;
    int32_t* ovf_items;
    int32_t* head;             // work counter, zeroed before each launch
    uint4* scratch;            // per lane: 2 * cap_list packed 16-B list entries
    uint32_t cap_list;
    int dbg;                   // debug switches (0 in production)
    uint64_t* dbg_buf;         // stamped diagnostic variant: 8 x u64 per wave
    uint64_t* tspan;           // [0] max of ~(wave start), [1] max of wave end (s_memrealtime), nullptr: none
    const uint4* kt;           // k-mer bi-interval table (smem_launch_kmer_table; variant 23), nullptr: none
    int kt_k;                  // its longest k-mer
};

// bwt_sa over the seeding output (software/bwamem.c:462-474, software/bwt.c:104-114)
struct SaParams {
    const uint32_t* occ64;
    uint64_t primary;
    uint64_t L2[5];
    const uint64_t* sa;        // sampled SA, sa[0] = -1
    uint32_t sa_shift;         // log2(sa_intv)
    const Intv* intv;          // flat smem_next2 intervals
    uint64_t n_intv;
    const uint64_t* occ_off;   // [n_intv + 1] exclusive prefix of occurrences per interval
    uint64_t n_occ;
    int min_seed_len;
    uint64_t max_occ;
    uint64_t* n_occ_intv;      // [n_intv] occurrences per interval (count kernel output)
    uint64_t* kstart;          // [n_occ + 2] the row of each occurrence (fill kernel)
    uint64_t* pos;             // [n_occ] bwt_sa results
};

// raw logs -> final smem_next2 lists (reverse + ordered merge, software/bwamem.c:280-301)
struct FinalizeParams {
    int n;
    const uint64_t* offs;          // read lengths for the merge key
    const uint32_t* n_intv;
    const uint32_t* n_calls;
    const Intv* main_intv;
    const CallRec* main_call;
    uint32_t cap_intv, cap_calls;
    const int32_t* ovf_slot;
    const Intv* ovf_intv;
    const CallRec* ovf_call;
    const uint32_t* ovf_n_calls;
    uint32_t ovf_cap_intv, ovf_cap_calls;
    // count pass writes sizes; write pass reads offsets and writes flat outputs
    uint64_t* s_intv;
    uint64_t* s_calls;
    const uint64_t* intv_off;
    const uint64_t* call_off;
    Intv* flat_intv;
    uint32_t* flat_calls;
};

}  // namespace smem

extern "C" {
hipError_t smem_launch_seed(const smem::SeedParams* P, int grid, int block, int variant, hipStream_t st);
// 1 when this build instantiates seeding-kernel variant `variant` (A/B variants need SMEM_AB_VARIANTS)
int smem_seed_variant_built(int variant);
// reference interleaved words (n_ref_buckets x 64 B) -> 2 * n_ref_buckets 32-B buckets
hipError_t smem_launch_occ64(const uint32_t* bwt, uint64_t n_ref_buckets, uint32_t* out, hipStream_t st);
hipError_t smem_launch_occ192(const uint32_t* occ64, uint64_t n_blocks, uint32_t* out, hipStream_t st);
// the bi-intervals of every string of 1..k bases (k <= 15): table L at entry
// (4^L - 4) / 3, index = the string's 2-bit codes, first base highest; 16-B
// packed entries (x0, x1, x2 low words, bits 32-33 in word 3), x2 = 0 when absent
hipError_t smem_launch_kmer_table(const uint32_t* occ64, uint64_t primary, const uint64_t* L2, int k, uint4* kt,
                                  hipStream_t st);
hipError_t smem_launch_finalize(const smem::FinalizeParams* F, int write, hipStream_t st);
hipError_t smem_launch_fill_i32(int32_t* p, int32_t v, int n, hipStream_t st);
hipError_t smem_launch_pack_intv(const smem::Intv* in, uint64_t n, uint4* out, hipStream_t st);
hipError_t smem_launch_ovf_slot(const int32_t* items, int n_ovf, int32_t* ovf_slot, hipStream_t st);
hipError_t smem_launch_sa_count(const smem::SaParams* S, hipStream_t st);
hipError_t smem_launch_sa_densify(const smem::SaParams* S, uint32_t dshift, uint64_t n_dense, uint64_t* dense,
                                  hipStream_t st);
// the same dense[] by hop + chase passes (link: n_dense words of scratch; n_dense < 2^32;
// max_blocks != 0 caps the lane-strided grids, leaving CUs to other work)
hipError_t smem_launch_sa_densify2(const smem::SaParams* S, uint32_t dshift, uint64_t n_dense, uint64_t* link,
                                   uint64_t* dense, unsigned max_blocks, hipStream_t st);
hipError_t smem_launch_sa_walk(const smem::SaParams* S, int grid, hipStream_t st);
hipError_t smem_launch_offsets(const uint64_t* in, uint64_t* out, int n, void* temp, size_t* temp_bytes,
                               hipStream_t st);
}
