/*
 * smem_oracle.h — TEST INFRASTRUCTURE ONLY (parity checker + CPU "port"
 * baseline).  A plain-C restatement of the reference SMEM seeding path:
 *
 *   mem_insert_seed loop   software/bwamem.c:453-460
 *   smem_next2             software/bwamem.c:244-305
 *   bwt_smem1              software/bwt.c:776-835
 *   bwt_extend             software/bwt.c:416-429
 *   bwt_2occ4 / bwt_occ4   software/bwt.c:207-215 / 187-204
 *   .bwt reader            software/bwt.c:899-918
 *
 * Pinned against golden vectors produced by the compiled reference
 * (oracle/_ref/ref_harness, see tests/golden/make_golden.py).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it; the
 * product (bwa-mem-harp2_amd/) never links it.
 */
#ifndef SMEM_ORACLE_H
#define SMEM_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
	uint64_t primary;
	uint64_t L2[5];
	uint64_t seq_len;
	uint64_t bwt_size;     /* in uint32 words, Occ checkpoints included */
	uint32_t *bwt;
	uint32_t cnt_table[256];
	int owns;
} orc_bwt_t;

typedef struct { uint64_t x[3], info; } orc_intv_t;

typedef struct {
	int min_seed_len;      /* -k, software/bwamem.c:58 */
	float split_factor;    /* -r, software/bwamem.c:65 */
	int split_width;       /* -s, software/bwamem.c:59 */
	int start_width;       /* 1, or 2 with MEM_F_NO_EXACT (software/bwamem.c:457) */
} orc_opt_t;

typedef struct {
	uint64_t n_calls;       /* non-NULL smem_next2 returns */
	uint64_t n_intv;        /* intervals returned */
	uint64_t n_smem1;       /* bwt_smem1 invocations */
	uint64_t n_ext;         /* bwt_extend calls whose result is used */
	uint64_t n_ext_ref;     /* bwt_extend calls the reference makes (incl. c<0 ones) */
	uint64_t n_bkt;         /* distinct 64-B Occ buckets over n_ext (1 or 2 each) */
	uint64_t n_bkt_ref;     /* same over n_ext_ref */
	uint64_t n_bases;       /* query bases of reads that entered the loop */
	uint64_t n_bkt64;       /* distinct 32-B Occ64 buckets (64 symbols) over n_ext: the GPU layout */
	uint64_t n_ext_fwd;     /* n_ext in forward loops (software/bwt.c:791-805) */
	uint64_t n_ext_u1_fwd;  /* forward extends of a size-1 interval (x2 == 1) */
	uint64_t n_ext_u1_bwd;  /* backward extends (c >= 0) of a size-1 interval */
	uint64_t n_run_u1;      /* maximal runs of size-1 extends of one interval (fwd or bwd) */
	uint64_t n_ext_fwd_k12; /* forward extends at depth i - x < 12 with no N before them */
	uint64_t n_ext_len[33]; /* used extends by the length of the string they produce (32 = 32 or more) */
	uint64_t n_fwd_push;    /* forward-list pushes (software/bwt.c:798, 801, 804) */
	uint64_t n_bwd_push_hi; /* backward-list (curr) pushes at index >= NL (ORC_LIST_LDS, default 11) */
	uint64_t n_bwd_read_hi; /* backward-list (prev, steps >= 2) reads at index >= NL */
	uint64_t n_fwd_spill;   /* forward-list entries beyond NL (the kernel's LDS ring spills them) */
	uint64_t n_bwd_step;    /* backward steps with a base to extend by (c >= 0, software/bwt.c:812) */
	uint64_t n_step_hist[17]; /* those steps by prev->n: 1..15, 16 = 16 or more */
	uint64_t n_bwd_task_hi; /* backward extends (c >= 0, any step) of prev[j], j >= NL */
	/* the unique-interval text mode, modelled (tools/text_mode_model.py): an
	 * extend whose input has x2 == 1 decided by comparing the read with the reference text
	 * instead of by Occ64 buckets; a full SA and ISA resident give the text position and the
	 * exact x0 / x1 of a text-mode interval when it is pushed or emitted */
	uint64_t n_tm_saved;    /* Occ64 bucket loads (n_bkt64's count) of those extends */
	uint64_t n_tm_sa;       /* SA loads: a size-1 interval's text position, once per run */
	uint64_t n_tm_isa;      /* ISA loads: exact x1 (forward push) / x0 (backward emit) of a text-mode result */
	uint64_t n_tm_runs;     /* runs of text compares (each starts a 16-B .pac block load) */
	uint64_t n_tm_bases;    /* bases compared against the text */
} orc_stats_t;

orc_bwt_t *orc_bwt_load(const char *fn);
/* wrap caller memory (not copied, not freed) */
orc_bwt_t *orc_bwt_wrap(const uint32_t *bwt, uint64_t bwt_size, uint64_t primary, const uint64_t L2[5]);
void orc_bwt_free(orc_bwt_t *b);

void orc_occ4(const orc_bwt_t *b, uint64_t k, uint64_t cnt[4]);
void orc_extend(const orc_bwt_t *b, const orc_intv_t *ik, orc_intv_t ok[4], int is_back);

/*
 * Seed n_reads reads (codes concatenated, offs[n_reads+1]).  For each read
 * writes the SMGO record into *out (malloc'ed, caller frees with
 * orc_free) when out != NULL, and accumulates stats.  Also fills
 * per-read arrays when non-NULL: n_intv_per_read, n_calls_per_read,
 * bytes_per_read (algorithmic bytes).
 * n_threads > 1 splits reads into contiguous chunks (pthreads).
 * Returns 0 on success.
 */
int orc_seed(const orc_bwt_t *b, int64_t n_reads, const uint8_t *codes, const int64_t *offs,
		const orc_opt_t *opt, int n_threads,
		uint8_t **out, uint64_t *out_len,
		uint32_t *n_intv_per_read, uint32_t *n_calls_per_read, uint64_t *bytes_per_read,
		orc_stats_t *stats);

/* timed variant for the CPU baseline: seeds reads, returns wall seconds */
/* every Occ64 bucket load of the GPU kernel in extend order (bit 31: the
 * extend's second bucket), read r's at out[read_off[r] .. read_off[r+1]);
 * one thread; returns the total (> cap: truncated) */
int64_t orc_seed_trace(const orc_bwt_t *b, int64_t n_reads, const uint8_t *codes, const int64_t *offs,
		const orc_opt_t *opt, uint32_t *out, uint64_t cap, uint64_t *read_off);
double orc_seed_timed(const orc_bwt_t *b, int64_t n_reads, const uint8_t *codes, const int64_t *offs,
		const orc_opt_t *opt, int n_threads, orc_stats_t *stats);

void orc_free(void *p);

/* ------------------------------------------------------- SA lookup (bwt_sa) */
/* sampled suffix array as bwa keeps it (software/bwt.c:80-102, .sa file
 * software/bwt.c:852-897): sa[i] = SA[i * sa_intv], sa[0] = (uint64_t)-1 */
typedef struct {
	uint64_t sa_intv, n_sa, seq_len;
	uint64_t *sa;
	int owns;
} orc_sa_t;

orc_sa_t *orc_sa_load(const char *fn);
orc_sa_t *orc_sa_wrap(const uint64_t *sa, uint64_t n_sa, uint64_t sa_intv, uint64_t seq_len);
void orc_sa_free(orc_sa_t *s);
/* bwt_sa(bwt, k) (software/bwt.c:104-114) */
uint64_t orc_sa_lookup(const orc_bwt_t *b, const orc_sa_t *s, uint64_t k);
/* out[i] = bwt_sa(bwt, k[i]) for n positions, n_threads pthreads */
void orc_sa_batch(const orc_bwt_t *b, const orc_sa_t *s, const uint64_t *k, uint64_t n, uint64_t *out, int n_threads);

/* ------------------------------------------------ chaining (chain_oracle.c) */
typedef struct { int64_t rbeg; int32_t qbeg, len; } orc_seed_t;   /* mem_seed_t */
typedef struct {
	int w;                 /* band width, software/bwamem.c:53 */
	int max_chain_gap;     /* software/bwamem.c:61 */
	int min_seed_len;      /* the filter's drop margin (min_seed_len << 1) */
	float mask_level;      /* software/bwamem.c:63 */
	float drop_ratio;      /* chain_drop_ratio, software/bwamem.c:64 */
	int filter;            /* 1: mem_chain_flt after mem_chain */
} orc_chain_opt_t;
/* mem_chain (+ mem_chain_flt) of every read; read i's seed sequence is
 * seeds[seed_off[i] .. seed_off[i+1]).  *out = SMCH stream (orc_free). */
int orc_chain(int64_t n_reads, const orc_seed_t *seeds, const uint64_t *seed_off, int64_t l_pac,
		const orc_chain_opt_t *o, int n_threads, uint8_t **out, uint64_t *out_len);

#ifdef __cplusplus
}
#endif
/* ---- SW extension (ksw_oracle.c): ksw_extend2, software/ksw.c:379-476 ---- */
typedef struct {
	uint64_t q_off, t_off;          /* into the query / target code pools (0..4) */
	int32_t qlen, tlen, w, end_bonus, zdrop, h0;
} orc_ksw_task_t;                   /* the layout of smem_ksw_task_t */
typedef struct { int32_t score, qle, tle, gtle, gscore, max_off; } orc_ksw_result_t;
typedef struct {
	int8_t mat[25], pad[3];          /* m = 5 */
	int32_t o_del, e_del, o_ins, e_ins;
} orc_ksw_opt_t;
int orc_ksw_extend(const orc_ksw_task_t *t, const uint8_t *query, const uint8_t *target, const orc_ksw_opt_t *o,
		orc_ksw_result_t *res);
/* DP cells this thread computed since the last reset: out[0] in-band cells of
 * ksw_extend2 (the columns [lo, hi) of every row), out[1] query x target cells
 * of every ksw_align2 pass */
void orc_cells(uint64_t out[2], int reset);
/* chain2aln's extensions by qlen bucket (<= 16, 32, 64, 128, 256, longer):
 * out[2 b] calls, out[2 b + 1] in-band cells */
void orc_ext_shapes(uint64_t out[12], int reset);
void orc_seed_uses(uint64_t out[4], int reset);
int orc_ksw_batch(int64_t n, const orc_ksw_task_t *tasks, const uint8_t *q, const uint8_t *t, const orc_ksw_opt_t *o,
		orc_ksw_result_t *out);

/* ---- chains -> alignment regions (aln_oracle.c): mem_chain2aln_short /
 * mem_chain2aln, software/bwamem.c:805-852, 1040-1188 ---- */
typedef struct {
	int8_t mat[25], pad[3];
	int32_t o_del, e_del, o_ins, e_ins;
	int32_t a, w, zdrop, pen_clip5, pen_clip3, min_seed_len;
} orc_aln_opt_t;                     /* the layout of smem_aln_opt_t */
typedef struct {
	int64_t rb, re;
	int32_t qb, qe, score, truesc, sub, csub, sub_n, w, seedcov, secondary;
	uint64_t hash;
} orc_alnreg_t;                      /* mem_alnreg_t, the layout of smem_alnreg_t */
typedef struct { int64_t pos; uint64_t seed_off; int32_t n, pad; } orc_aln_chain_t;   /* smem_chain_t */
void orc_sw_shift_top(const int8_t *mat, int *shift, int *top);
void orc_ksw_align2(int qlen, const uint8_t *query, int tlen, const uint8_t *target, const int8_t *mat, int o_del,
		int e_del, int o_ins, int e_ins, int xtra, int32_t out[7]);
int orc_aln_read(const orc_aln_opt_t *o, int64_t l_pac, const uint8_t *pac, int l_query, const uint8_t *query,
		int n_chains, const orc_aln_chain_t *chains, const orc_seed_t *seeds, orc_alnreg_t **out);
int orc_aln_batch(const orc_aln_opt_t *o, int64_t l_pac, const uint8_t *pac, int64_t n_reads, const uint8_t *codes,
		const uint64_t *offs, const orc_aln_chain_t *chains, const uint64_t *chain_off, const orc_seed_t *seeds,
		orc_alnreg_t **regs, uint64_t *reg_off);

#endif
