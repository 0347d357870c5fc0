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
    uint32_t* ctr;     // [2] work-queue heads (reads <= 256 bp, longer)
    // compaction
    const uint64_t* reg_off;  // [n_reads + 1]
    AlnReg* out;
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
}
