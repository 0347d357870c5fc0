// Seed chaining on the device: mem_chain's tree
// insertion loop and mem_chain_flt, one lane per read, over the SA positions
// smem_batch_sa left in HBM.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace smem {

// mem_seed_t (software/bwamem.c:317-320)
struct SeedRec {
    int64_t rbeg;
    int32_t qbeg, len;
};

// a chain while it grows: its first seed (pos = first rbeg, first_qbeg) and
// last seed (what test_and_merge reads, software/bwamem.c:334-354); seeds
// are linked through ChainParams::next by occurrence index
struct ChainRec {
    int64_t pos, last_rbeg;
    int32_t first_qbeg, last_qbeg, last_len, n;
    uint32_t first, last;
};

// kbtree(chn) node at KB_DEFAULT_SIZE: t = 8, at most 15 keys / 16 children
// (software/kbtree.h:52-60, 369); children are node indices in the read's pool
constexpr int BT_T = 8;
constexpr int BT_MAX = 2 * BT_T - 1;
constexpr uint32_t BT_NONE = 0xffffffffu;
struct BNode {
    static constexpr uint32_t MAX_ID = 0xfffffff0u;
    int64_t key[BT_MAX];
    int32_t n, leaf;
    uint32_t id[BT_MAX];
    uint32_t child[BT_MAX + 1];
    uint32_t pad[1];
};
static_assert(sizeof(BNode) == 256, "BNode is one 256-B record");
// the same node with 16-bit chain ids and children (the heavy path's LDS
// pool: 184 B, 835 nodes in 150 KB)
struct LNode {
    static constexpr uint32_t MAX_ID = 0xffffu;
    int64_t key[BT_MAX];
    uint16_t id[BT_MAX];
    uint16_t child[BT_MAX + 1];
    uint8_t n, leaf;
    uint8_t pad[6];
};
static_assert(sizeof(LNode) == 192, "LNode size");

// flt_aux_t of mem_chain_flt (software/bwamem.c:619-624); p, p2 are chain
// positions, p2 = -1 for none
struct FltRec {
    int32_t beg, end, w, p, p2;
};

// one chain of the output: its seeds are seeds[seed_off .. seed_off + n)
struct OutChain {
    int64_t pos;
    uint64_t seed_off;
    int32_t n, pad;
};

struct ChainParams {
    // inputs: the batch's flat intervals (x0, x1, x2, info) and bwt_sa results
    const uint64_t* intv;      // 4 words per interval
    const uint64_t* intv_off;  // [n_reads + 1]
    const uint64_t* occ_off;   // [n_intv + 1], occurrences of kept intervals
    const uint64_t* pos;       // [n_occ]
    int n_reads;
    int64_t l_pac;
    int w, max_chain_gap, min_seed_len, filter;
    float mask_level, drop_ratio;
    // scratch, indexed by occurrence (a read owns [occ_off[intv_off[r]], ...))
    SeedRec* seed;
    uint32_t* next;
    ChainRec* chn;
    BNode* node;               // read r's pool starts at occ_begin / 7 + 3 r
    uint32_t* ord;             // tree order
    uint32_t* ord2;            // filtered order
    FltRec* flt;
    uint64_t* n_out;           // [n_reads] chains kept
    uint64_t* ns_out;          // [n_reads] seeds in them
    // reads with more than heavy_min occurrences go to chain_heavy_kernel:
    // heavy[0 .. ) giants (> giant_min), heavy[n_reads .. ) the rest;
    // heavy_ctr = {giants, rest, claimed}
    uint32_t heavy_min, giant_min;
    uint32_t* heavy;           // [2 n_reads]
    uint32_t* heavy_ctr;       // [4]
    uint32_t lds_bytes;        // dynamic LDS of chain_heavy_kernel
    int cluster;               // heavy path: position-cluster decomposition (0: tree path only)
    int wave_sort;             // heavy path: mem_chain_flt's introsort by the wave (0: lane 0 alone)
    uint32_t sort_lane_max;    // wave sort: segments up to this size are cut by one lane
    int tier;                  // chain_heavy_kernel's items: 0 giants, 1 the rest, -1 both (one launch)
    uint32_t lds_rest;         // dynamic LDS of the tier-1 launch
    int drop_blocked;          // heavy path: drop loop's kept list first, then p2 in blocks (0: flt_drop_pruned)
    int replay_cache;          // heavy path: the kbtree replay's LDS chain-record cache (0: records from HBM only)
    int sort_count;            // mem_chain_flt's closing stable sort by weight counts (else a bitonic sort of keys)
    int giant_order;           // giants in listing order (0), longest first (1) or shortest first (2)
    uint32_t giant_waves;      // the giant tier's waves (0: one per CU)
    uint32_t dbg_lo;           // SMEM_CHAIN_DBG: the first heavy item recorded (SMEM_CHAIN_DBG_LO)
    uint32_t wave_min;         // heavy path: clusters of more seeds are passed by the whole wave (cluster_wave)
    uint64_t* dbg;             // optional phase clocks of the heavy path (32 words per item)
    // output (write kernel)
    const uint64_t* chain_off; // [n_reads + 1]
    const uint64_t* seed_off;  // [n_reads + 1]
    OutChain* out_chain;
    SeedRec* out_seed;
};

}  // namespace smem

extern "C" {
// st2 (may be null: one launch on st): the heavy reads' second tier runs
// there beside the giants, between ev_fork and ev_join
hipError_t smem_launch_chain_build(const smem::ChainParams* P, int n_cu, hipStream_t st, hipStream_t st2,
                                   hipEvent_t ev_fork, hipEvent_t ev_join);
hipError_t smem_launch_chain_write(const smem::ChainParams* P, int n_cu, hipStream_t st);
}
