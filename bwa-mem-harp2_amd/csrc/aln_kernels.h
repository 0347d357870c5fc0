// Chains -> alignment regions on the device:
// mem_chain2aln_short / mem_chain2aln of every chain of every read
// (software/bwamem.c:805-852, 1040-1188), one wave per read.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "chain_kernels.h"

namespace smem {

// mem_alnreg_t (software/bwamem.h:62-74)
struct AlnReg {
    int64_t rb, re;
    int32_t qb, qe, score, truesc, sub, csub, sub_n, w, seedcov, secondary;
    uint64_t hash;
};
static_assert(sizeof(AlnReg) == 64, "mem_alnreg_t layout");

constexpr int ALN_CTRS = 16;
constexpr int ALN_SPLITS = 16;     // SMEM_ALN_SPLIT accumulators (aln_kernel's phases and counts)
constexpr int ALN_HT = 65536;       // hash slots per walk wave
constexpr int ALN_WALK_WAVES = 4;   // walk waves per CU (aln_heavy_kernel blocks of 256)

// a seed whose region is computed ahead by the lane engine (ksw_lane.h):
// chain c (absolute), read r, seed si of the chain
struct RegTask {
    uint64_t c;
    uint32_t r, si;
};

// the lane path's queue words (AlnParams::lq)
constexpr int LQ_NTASK = 0;     // tasks listed
constexpr int LQ_NSW = 1;       // heavy chains listed for mem_chain2aln_short's SW
constexpr int LQ_QUEUES = 16;   // 16-column queues: pass lengths 1 .. 256 (LQ_MAXQ)
constexpr int LQ_MAXQ = 16 * LQ_QUEUES;
constexpr int LQ_BOUNDS = 8;    // [LQ_QUEUES + 1] queue q = order[bounds[q] .. bounds[q + 1]): lengths 16q + 1 .. 16q + 16
constexpr int LQ_HEADS = 25;    // [LQ_QUEUES] claim counters
constexpr int LQ_HIST = 41;     // [LQ_BUCKETS] tasks per pass length (0..LQ_MAXQ, longer), then cursors
constexpr int LQ_BUCKETS = LQ_MAXQ + 2;
constexpr int LQ_WORDS = 320;
// the lane engine's tiers: columns, and the queues each takes (32: 0-1, 64: 2-3, 144: 4-8,
// 256: 9-15 -- the 250-bp reads' extensions; its column array is past the 256 VGPRs a lane
// has at two waves a SIMD, so that tier runs one wave a SIMD with the rest in AGPRs)
constexpr int LQ_TIER_Q0(int kcol) { return kcol == 32 ? 0 : kcol == 64 ? 2 : kcol == 144 ? 4 : 9; }
// in a batch of reads of at most LQ_GAP_HI + 1 bp the 256 tier is not launched, and the pass
// lengths LQ_GAP_LO .. LQ_GAP_HI (queue 9: a 150-bp read's seeds in its last 5 bases) go to one
// wave each (aln_region_rest_kernel) -- the tier's launch, one block a CU with 64 KB of LDS,
// waited for CUs behind the other streams' lane passes even with nothing to do: 59.4 -> 61.0 ms
// human-like; with longer reads queue 9 is the 256 tier's (c4: 242 -> 212 ms)
constexpr int LQ_GAP_LO = 145, LQ_GAP_HI = 160;
constexpr int LQ_TIER_Q1(int kcol) { return kcol == 32 ? 2 : kcol == 64 ? 4 : kcol == 144 ? 9 : LQ_QUEUES; }
static_assert(LQ_BOUNDS + LQ_QUEUES + 1 <= LQ_HEADS && LQ_HEADS + LQ_QUEUES <= LQ_HIST &&
              LQ_HIST + LQ_BUCKETS <= LQ_WORDS, "lane queue words");

struct AlnParams {
    // reads (nt4 codes, 4 = N) and the chains smem_batch_chain wrote
    const uint8_t* codes;
    const uint64_t* offs;       // [n_reads + 1]
    const OutChain* chains;
    const uint64_t* chain_off;  // [n_reads + 1]
    const SeedRec* seeds;       // chain seeds (OutChain::seed_off is absolute)
    const uint64_t* seed_off;   // [n_reads + 1]: read r owns seeds[seed_off[r] ..)
    // the 2-bit .pac of the forward strand (software/bntseq.c:303-309)
    const uint8_t* pac;
    int64_t l_pac;
    int n_reads;
    int max_len;   // the batch's longest read (<= 0: unknown): the 256-column lane tier is launched past LQ_GAP_HI + 1
    // mem_opt_t scoring and extension options (software/bwamem.h:33-45)
    int8_t mat[28];
    int o_del, e_del, o_ins, e_ins, a, w, zdrop, pen_clip5, pen_clip3, min_seed_len;
    int top;       // largest matrix entry (>= 0): ksw_extend2's max, ksw_qinit's q->max
    int sw_shift;  // ksw_qinit's byte bias
    // scratch and output, indexed like seeds: a read's regions never
    // outnumber its seeds (one per extended seed, or one per chain)
    uint64_t* srt;     // per chain: the seed order (software/bwamem.c:1070-1073)
    AlnReg* raw;       // read r's regions at raw[seed_off[r] ..)
    uint64_t* n_regs;  // [n_reads]
    uint32_t* ctr;     // [ALN_CTRS]: work-queue heads (reads <= 256 bp, longer), heavy-read count, heavy-path heads
    uint64_t* cyc;     // diagnostics (SMEM_ALN_CYCLES): [n_reads] shader cycles per read, then [4 n_reads]
                       // the heavy walk's split (smem_gpu.cpp), nullptr: off
    uint64_t* split;   // diagnostics (SMEM_ALN_SPLIT): [ALN_SPLITS] aln_kernel's cycles by phase and counts, nullptr: off
    // heavy reads (at least heavy_min chains or heavy_seeds seeds; 0 = none):
    // every chain walked ahead on its own, one wave per chain, then the read's
    // walk replays them (aln_heavy_kernel)
    uint32_t heavy_min, heavy_seeds;
    uint32_t hash_min;        // heavy reads with at least this many chains hash their regions by bin
    uint32_t spec_local;      // 1: a heavy chain precomputes only the seeds its own walk extends (0: all)
    uint32_t light_claims;    // aln_kernel: work-queue claims per wave before it exits (0: until the queue is empty)
    uint32_t walk_guard;      // != 0: the inlined walk, at most this many loop iterations per read (ctr[15] counts trips)
    int32_t* heavy;           // [n_reads] heavy read ids (ctr[2] of them, any order)
    uint32_t walk_wpc;        // the walk's waves per CU (aln_heavy_kernel grid; 0: ALN_WALK_WAVES)
    uint32_t walk_waves;      // != 0: the walk's grid in waves (the giant reads' walk: one wave each)
    // The giant split (smem_launch_aln_heavy_split): the heaviest heavy reads (rgiant[r] = 1;
    // chain_read bit 30) get their own task list and candidate index, and their passes and walk
    // run on a stream of their own from the start -- a tandem-repeat read's walk, ~20 ms on one
    // wave, then overlaps the other heavy and light reads' passes instead of ending the stage.
    const uint8_t* rgiant;    // [n_reads] 1: a giant read (nullptr: no split)
    RegTask* gtasks;          // [n_seeds] the giant reads' chain tasks (glq[LQ_NTASK] of them)
    uint32_t* glq;            // [LQ_WORDS] their lane queues (as lq)
    uint64_t* hcnt;           // [n_reads] their chain counts, then
    uint64_t* hoff;           // [n_heavy + 1] prefix: chain task t of the heavy reads
    uint64_t* hscnt;          // [n_reads] their seed counts
    int64_t* span;            // [2 n_chains] the chain's reference span (chain_span)
    uint64_t* ht;             // [walk waves x ALN_HT] per-wave hash of a heavy read's regions by 512-bp bin
    int32_t* rnext;           // [n_seeds] the next region of the same bin (index in the read), -1: none
    AlnReg* pre;              // [n_seeds] the region of each seed its chain's own walk extended, heavy reads only
    uint8_t* pre_ok;          // [n_seeds] 1: pre holds it
    AlnReg* loc;              // [n_seeds] the regions of each chain's own walk (scratch at the chain's seeds)
    AlnReg* pre_short;        // [n_chains] mem_chain2aln_short's region, heavy reads only
    uint8_t* short_ok;        // [n_chains] 1: that region was made (0: mem_chain2aln runs)
    // regions computed ahead one seed per lane (lane_on; SMEM_ALN_LANE=0 turns
    // it off): the light reads' chains' first seeds, the heavy reads' chains'
    // every seed; the walks take them from pre / pre_ok
    uint32_t lane_on;
    RegTask* tasks;           // [n_seeds + n_chains]
    uint32_t* torder;         // [n_seeds + n_chains] the tasks in pass order (by the pass's query length)
    uint8_t* tfail;           // [n_seeds + n_chains] 1: left to the walk (query past LQ_MAXQ columns, or scores past 16 bits)
    uint8_t* sdec;            // [n_chains] light chains: 1 when mem_chain2aln_short declines before its SW
    uint32_t* lq;             // [LQ_WORDS] the lane path's counters, queue bounds and histogram
    uint32_t* chain_read;     // [n_chains] the read of each chain, bit 31: a heavy read
    // the heavy reads' task list (the prep kernels write it beside tasks / lq,
    // the light reads' list; the two lists run their passes on two streams)
    RegTask* htasks;
    uint32_t* hlq;
    uint32_t* swlist;         // [n_chains] heavy chains whose mem_chain2aln_short runs its SW (lq[LQ_NSW] of them)
    // the heavy walk's candidate index (lane_on, SMEM_ALN_CAND != 0; nullptr: off): every region a
    // heavy read's walk can make -- its short chains' pre_short, its other chains' seeds' pre -- sorted
    // by (heavy read, rb).  A seed the ring misses is tested against the candidates that start within
    // the read's longest candidate before it, 64 a round, counting only those the walk made so far
    int64_t* cand_rb;         // [m] sorted candidates: reference start (INT64_MAX: no region)
    int64_t* cand_re;
    uint32_t* cand_q;         // qb | qe << 16
    uint8_t* cand_made;       // [m] 1: the walk made this region
    uint32_t* cand_pos_s;     // [n_seeds] a heavy read's seed's region: its index position
    uint32_t* cand_pos_c;     // [n_chains] a heavy read's short chain's region: its position
    uint2* cand_rng;          // [n_seeds] the positions [x, y) a heavy read's seed is tested against
    // compaction
    const uint64_t* reg_off;  // [n_reads + 1]
    AlnReg* out;
};

// building the candidate index: per heavy read h (ordinal in AlnParams::heavy)
// slots [off[h], off[h + 1]) -- its seeds, then its chains -- keyed by rb
// (no region: all 34 bits ones), each read's segment sorted by key
struct CandParams {
    uint64_t* key;   // [m] unsorted, then
    uint64_t* key2;  // [m] sorted
    uint32_t* val;   // [m] seed index, or 0x80000000 | chain index
    uint32_t* val2;
    uint64_t* off;   // [n_heavy + 1]
    int64_t* hmax;   // [n_heavy] the longest candidate region of the read
    uint32_t* hord;  // [n_reads] a heavy read's ordinal
    uint32_t n_heavy;
    uint64_t m;
    uint64_t n_chains;
};

// one ksw_align2 call (software/ksw.c:342) as mem_chain2aln_short makes it
struct KswATask {
    uint64_t q_off, t_off;
    int32_t qlen, tlen, xtra, pad;
};
struct KswAResult {
    int32_t score, te, qe, score2, te2, tb, qb;
};
struct KswAParams {
    const KswATask* task;
    int n;
    const uint8_t* q;
    const uint8_t* t;
    int8_t mat[28];
    int o_del, e_del, o_ins, e_ins;
    int shift, top;
    KswAResult* out;
};

}  // namespace smem

extern "C" {
hipError_t smem_launch_ksw_align2(const smem::KswAParams* K, int n_cu, hipStream_t st);
// long_reads != 0: the batch holds reads of 257..1024 bp (second instantiation)
hipError_t smem_launch_aln(const smem::AlnParams* P, int n_cu, int long_reads, hipStream_t st);
hipError_t smem_launch_aln_write(const smem::AlnParams* P, hipStream_t st);
// heavy reads: list them (ctr[2]), then, after the host scanned hcnt into
// hoff, compute their chains' regions ahead and walk them
hipError_t smem_launch_aln_classify(const smem::AlnParams* P, hipStream_t st);
// parts: 1 the chain tasks, 2 the walk, 3 both
hipError_t smem_launch_aln_heavy(const smem::AlnParams* P, int n_cu, int long_reads, int parts, hipStream_t st);
// the giant split: P->heavy / hcnt / hscnt (n_heavy of them) copied into heavy2 / hcnt2 / hscnt2
// in the same bucket order (seeds + chains, most first); the first n_giant of them marked in
// rgiant (cleared for every read first); ctr_g[2] = n_giant, ctr_r[2] = n_heavy - n_giant
hipError_t smem_launch_aln_heavy_split(const smem::AlnParams* P, uint32_t n_heavy, uint32_t n_giant, int32_t* heavy2,
                                       uint64_t* hcnt2, uint64_t* hscnt2, uint8_t* rgiant, uint32_t* ctr_g,
                                       uint32_t* ctr_r, hipStream_t st);
// the candidate index: slot counts per heavy read (hcnt + hscnt) into cnt[n_heavy];
// then (C.off scanned, C.m slots) fill, sort, place and every heavy seed's range;
// tmp / tmp_bytes: the sort's scratch (tmp nullptr: *tmp_bytes is set, nothing runs)
hipError_t smem_launch_aln_cand_count(const smem::AlnParams* P, uint32_t n_heavy, uint64_t* cnt, uint32_t* hord,
                                      hipStream_t st);
hipError_t smem_launch_aln_cand(const smem::AlnParams* P, const smem::CandParams* C, void* tmp, size_t* tmp_bytes,
                                int n_cu, hipStream_t st);
// lane_on: the regions computed ahead one seed per lane, before the walks
// (lq / hlq zeroed; heavy_min / heavy_seeds set): every chain's prep and
// tasks (light reads' to tasks / lq, heavy reads' to htasks / hlq), then, per
// list (P with tasks / lq, torder, tfail of that list), the passes
// parts: 1 every chain's prep and the light / heavy task lists, 2 the heavy chains' short SW
// (aln_heavy_sw_kernel: their tasks when it declines), 3 both -- the light reads' passes need
// only part 1 (c4's 250-bp reads: part 2 is 36 ms of one-wave-a-chain SW)
hipError_t smem_launch_aln_prep(const smem::AlnParams* P, uint64_t n_chains, int n_cu, int parts, hipStream_t st);
hipError_t smem_launch_aln_passes(const smem::AlnParams* P, int n_cu, int long_reads, hipStream_t st);
}
