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

struct SeedParams {
    const uint32_t* bwt;       // interleaved BWT + Occ, resident in HBM
    uint64_t primary;
    uint64_t L2[5];
    const uint8_t* codes;      // reads, concatenated nt4 codes
    const uint64_t* offs;      // n_reads + 1
    const int32_t* read_ids;   // work item -> read (nullptr: identity)
    int n_items;
    int min_seed_len, split_len_init, split_width, start_width;
    Intv* out_intv;            // [item][cap_intv]
    uint32_t cap_intv;
    uint32_t* out_call_n;      // [item][cap_calls]
    uint32_t cap_calls;
    uint32_t* n_intv;          // [item] count, or SMEM_OVERFLOW
    uint32_t* n_calls;         // [item]
    int32_t* ovf_count;
    int32_t* ovf_items;
    int32_t* head;             // work counter, zeroed before each launch
    Intv* scratch;             // [lane][4][cap_list]
    uint32_t cap_list;
};

struct GatherParams {
    int n;
    const uint32_t* n_intv;
    const Intv* main_intv;
    const uint32_t* main_calls;
    uint32_t cap_intv, cap_calls;
    const int32_t* ovf_slot;
    const Intv* ovf_intv;
    const uint32_t* ovf_calls;
    uint32_t ovf_cap_intv, ovf_cap_calls;
    const uint64_t* intv_off;   // n + 1
    const uint64_t* call_off;   // n + 1
    Intv* flat_intv;
    uint32_t* flat_calls;
};

}  // namespace smem

extern "C" {
hipError_t smem_launch_seed(const smem::SeedParams* P, int grid, int block, hipStream_t st);
hipError_t smem_launch_sizes(const uint32_t* n_intv, const uint32_t* n_calls, const int32_t* ovf_slot,
                             const uint32_t* ovf_n_intv, const uint32_t* ovf_n_calls, uint64_t* s_intv,
                             uint64_t* s_calls, int n, hipStream_t st);
hipError_t smem_launch_gather(const smem::GatherParams* G, hipStream_t st);
hipError_t smem_launch_fill_i32(int32_t* p, int32_t v, int n, hipStream_t st);
hipError_t smem_launch_ovf_slot(const int32_t* items, int n_ovf, int32_t* ovf_slot, hipStream_t st);
}
extern "C" hipError_t smem_launch_offsets(const uint64_t* in, uint64_t* out, int n, void* temp, size_t* temp_bytes,
                                          hipStream_t st);
