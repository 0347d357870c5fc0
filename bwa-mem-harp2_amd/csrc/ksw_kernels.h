// SW extension on the device: ksw_extend2
// (software/ksw.c:379-476), one wave per extension problem.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace smem {

constexpr int KSW_COLS_PER_LANE = 4;  // query columns 0..qlen held per wave: qlen <= 255

// smem_ksw_task_t / smem_ksw_result_t (include/smem_gpu.h)
struct KswTask {
    uint64_t q_off, t_off;
    int32_t qlen, tlen, w, end_bonus, zdrop, h0;
};
struct KswResult {
    int32_t score, qle, tle, gtle, gscore, max_off;
};

struct KswParams {
    const KswTask* task;
    int n;
    const uint8_t* q;   // query code pool (0..4)
    const uint8_t* t;   // target code pool
    int8_t mat[28];     // m = 5 scoring matrix (25 used)
    int o_del, e_del, o_ins, e_ins;
    KswResult* out;
};

}  // namespace smem

extern "C" hipError_t smem_launch_ksw(const smem::KswParams* K, int n_cu, hipStream_t st);
// one problem per lane (kswl::lane_engine), scratch of smem_ksw_lane_scratch(n) bytes
extern "C" size_t smem_ksw_lane_scratch(int n);
extern "C" hipError_t smem_launch_ksw_lane(const smem::KswParams* K, void* scratch, int n_cu, hipStream_t st);
