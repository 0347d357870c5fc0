/*
 * ref_harness.c — TEST INFRASTRUCTURE ONLY.  Drives the *unmodified* reference
 * C sources (compiled in place from /root/reference/software by
 * oracle/Makefile into oracle/_ref/) so that golden vectors and the
 * "reference" CPU baseline come from the reference itself.  Nothing in the
 * product links this file.
 *
 * Commands
 *   index <in.fa> <prefix>
 *       bwa_index(-a is) — software/bwtindex.c:187 (BWT by software/is.c:208,
 *       Occ interleave by software/bwtindex.c:128-150, .bwt dump software/bwt.c:841)
 *   smem  <in.bwt> <reads.smrd> <out.smgo> <k> <split_factor> <split_width> <start_width>
 *       For every read, the mem_chain() guard (software/bwamem.c:600) and the
 *       mem_insert_seed() loop (software/bwamem.c:453-460) calling the
 *       reference smem_next2() (software/bwamem.c:244); every returned list
 *       is written in SMGO format (include/smem_formats.h).
 *   bench <in.bwt> <reads.smrd> <n_threads> <max_reads> <k> <split_factor> <split_width> <start_width>
 *       Same loop, timed, pthreads over contiguous read chunks; prints one
 *       line: "reads=<n> seconds=<t> threads=<T> reads_per_s=<r>".
 *   sa    <in.bwt> <in.sa> <in.smgo> <out.smsa> <k> <max_occ>
 *       For every interval of the SMGO stream that mem_insert_seed() turns
 *       into seeds (software/bwamem.c:467), the reference bwt_sa()
 *       (software/bwt.c:104-114) of each occurrence x0 + j, j < x2
 *       (software/bwamem.c:469-474), written as SMSA (include/smem_formats.h).
 *   chain <in.bwt> <in.sa> <reads.smrd> <out.smch> <k> <r> <s> <start_width> <max_occ> <w>
 *         <max_chain_gap> <mask_level> <drop_ratio> <filter>
 *       For every read, the reference mem_chain() (software/bwamem.c:593) and,
 *       when filter != 0, mem_chain_flt() (software/bwamem.c:629) as
 *       mem_align1_core calls them (software/bwamem.c:1448-1449); chains
 *       written as SMCH (include/smem_formats.h).
 *   aln   <in.bwt> <in.sa> <in.pac> <reads.smrd> <out.smrg> <k> <r> <s> <start_width> <max_occ> <w>
 *         <max_chain_gap> <mask_level> <drop_ratio>
 *       mem_chain + mem_chain_flt as for chain (filter on), then per chain
 *       mem_chain2aln_short and, when it declines, mem_chain2aln
 *       (software/bwamem.c:1452-1460); every read's regions written as SMRG (and the
 *       wall time of the chain2aln loop alone on stderr: "chain2aln_seconds=..."):
 *       "SMRG0001", u64 n_reads, per read u32 n then n x {i64 rb, re;
 *       i32 qb, qe, score, truesc, sub, csub, sub_n, w, seedcov, secondary}.
 *   kswa  <tasks.smat> <out.smar>
 *       the reference's own ksw_align2 (software/ksw.c:342) on every task
 *       (SMAT: as SMKT with per task {u64 q_off, t_off; i32 qlen, tlen, xtra, pad}),
 *       results as SMAR: "SMAR0001", u64 n, n x i32 {score, te, qe, score2, te2, tb, qb}.
 *   mem   <prefix> <reads.fq> <n_threads> <batch_size> <pe> [<pg>]
 *       The body of the reference's main_mem (software/fastmap.c:193-230) on the
 *       unmodified pipeline: bwa_print_sam_hdr, then bseq_read chunks through
 *       mem_process_seqs (software/bwamem.c:1614: kt_for_batch -> worker1_batched
 *       -> mem_align1_core_batched, then mem_sam_pe / mem_reg2sam_se), SAM on
 *       stdout.  The index is loaded as bwa_idx_load does (software/bwa.c:312-333)
 *       minus bwa_idx_load_bwt's FPGA upload (software/bwa.c:283-307), and the
 *       per-worker buffers main_mem allocates for the HARP path
 *       (software/fastmap.c:208-210; sw_handshake as the manager allocates it,
 *       :324) are allocated the same way.  With batch_size <= 2 every batch takes
 *       bwt_smem1_batched's CPU path (software/bwt.c:603, 686-717): this is
 *       `bwa mem -t N -b 1` of the reference, the golden SAM for the GPU build.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <pthread.h>
#include <sys/time.h>

#include <zlib.h>
#include "bwt.h"
#include "bwamem.h"
#include "bwa.h"
#include "bntseq.h"
#include "kseq.h"
#include "utils.h"
#include "ksw.h"
#include "smem_formats.h"
KSEQ_DECLARE(gzFile)

/* defined in software/bwamem.c:244 (not exported by software/bwamem.h) */
extern const bwtintv_v *smem_next2(smem_i *itr, int split_len, int split_width, int start_width);
/* defined in software/bwtindex.c:187 */
extern int bwa_index(int argc, char *argv[]);

static double now_s(void)
{
	struct timeval tv;
	gettimeofday(&tv, 0);
	return tv.tv_sec + tv.tv_usec * 1e-6;
}

typedef struct {
	int k, split_width, start_width;
	float split_factor;
} opts_t;

/* The seeding loop exactly as mem_chain()/mem_insert_seed() drive it. Emits
 * each returned list through cb (may be NULL). Returns number of calls. */
static int seed_one(const bwt_t *bwt, smem_i *itr, const opts_t *o, int len, const uint8_t *q,
		FILE *out, uint64_t *n_intv)
{
	const bwtintv_v *a;
	int n_calls = 0, split_len;
	long pos = 0;
	uint32_t zero = 0;
	if (out) { pos = ftell(out); fwrite(&zero, 4, 1, out); }
	if (len < o->k) goto done; /* software/bwamem.c:600 */
	split_len = (int)(o->k * o->split_factor + .499);
	split_len = split_len < len ? split_len : len;
	smem_set_query(itr, len, q);
	while ((a = smem_next2(itr, split_len, o->split_width, o->start_width)) != 0) {
		++n_calls;
		if (n_intv) *n_intv += a->n;
		if (out) {
			uint32_t n = (uint32_t)a->n;
			size_t i;
			fwrite(&n, 4, 1, out);
			for (i = 0; i < a->n; ++i) {
				uint64_t v[4] = { a->a[i].x[0], a->a[i].x[1], a->a[i].x[2], a->a[i].info };
				fwrite(v, 8, 4, out);
			}
		}
	}
done:
	if (out) {
		long end = ftell(out);
		uint32_t nc = (uint32_t)n_calls;
		fseek(out, pos, SEEK_SET);
		fwrite(&nc, 4, 1, out);
		fseek(out, end, SEEK_SET);
	}
	(void)bwt;
	return n_calls;
}

static int parse_opts(char **argv, opts_t *o)
{
	o->k = atoi(argv[0]);
	o->split_factor = (float)atof(argv[1]);
	o->split_width = atoi(argv[2]);
	o->start_width = atoi(argv[3]);
	return 0;
}

static int cmd_smem(int argc, char **argv)
{
	bwt_t *bwt;
	smrd_reads_t r;
	smem_i *itr;
	opts_t o;
	FILE *out;
	uint64_t i;
	if (argc < 8) { fprintf(stderr, "usage: smem <bwt> <reads> <out> <k> <r> <s> <start_width>\n"); return 1; }
	parse_opts(argv + 4, &o);
	bwt = bwt_restore_bwt(argv[1]);
	if (smrd_load(argv[2], &r) != 0) { fprintf(stderr, "cannot load reads %s\n", argv[2]); return 1; }
	out = fopen(argv[3], "wb");
	if (!out) return 1;
	smgo_write_header(out, r.n_reads);
	itr = smem_itr_init(bwt);
	for (i = 0; i < r.n_reads; ++i)
		seed_one(bwt, itr, &o, r.len[i], r.codes + r.off[i], out, 0);
	smem_itr_destroy(itr);
	fclose(out);
	smrd_free(&r);
	bwt_destroy(bwt);
	return 0;
}

typedef struct {
	const bwt_t *bwt;
	const smrd_reads_t *r;
	const opts_t *o;
	uint64_t beg, end, n_intv;
} bench_job_t;

static void *bench_worker(void *data)
{
	bench_job_t *j = (bench_job_t*)data;
	smem_i *itr = smem_itr_init(j->bwt);
	uint64_t i;
	for (i = j->beg; i < j->end; ++i)
		seed_one(j->bwt, itr, j->o, j->r->len[i], j->r->codes + j->r->off[i], 0, &j->n_intv);
	smem_itr_destroy(itr);
	return 0;
}

static int cmd_bench(int argc, char **argv)
{
	bwt_t *bwt;
	smrd_reads_t r;
	opts_t o;
	int t, n_threads;
	uint64_t n, n_intv = 0;
	double t0, t1;
	pthread_t *tid;
	bench_job_t *jobs;
	if (argc < 9) { fprintf(stderr, "usage: bench <bwt> <reads> <threads> <max_reads> <k> <r> <s> <sw>\n"); return 1; }
	parse_opts(argv + 5, &o);
	bwt = bwt_restore_bwt(argv[1]);
	if (smrd_load(argv[2], &r) != 0) return 1;
	n_threads = atoi(argv[3]);
	n = (uint64_t)atoll(argv[4]);
	if (n == 0 || n > r.n_reads) n = r.n_reads;
	tid = (pthread_t*)calloc(n_threads, sizeof(pthread_t));
	jobs = (bench_job_t*)calloc(n_threads, sizeof(bench_job_t));
	t0 = now_s();
	for (t = 0; t < n_threads; ++t) {
		jobs[t].bwt = bwt; jobs[t].r = &r; jobs[t].o = &o;
		jobs[t].beg = n * t / n_threads; jobs[t].end = n * (t + 1) / n_threads;
		pthread_create(&tid[t], 0, bench_worker, &jobs[t]);
	}
	for (t = 0; t < n_threads; ++t) { pthread_join(tid[t], 0); n_intv += jobs[t].n_intv; }
	t1 = now_s();
	printf("reads=%llu seconds=%.6f threads=%d reads_per_s=%.3f intervals=%llu\n",
			(unsigned long long)n, t1 - t0, n_threads, n / (t1 - t0), (unsigned long long)n_intv);
	free(tid); free(jobs); smrd_free(&r); bwt_destroy(bwt);
	return 0;
}

static int cmd_sa(int argc, char **argv)
{
	bwt_t *bwt;
	FILE *in, *out;
	char magic[8];
	uint64_t n_reads, r;
	int k, max_occ;
	if (argc < 7) { fprintf(stderr, "usage: sa <bwt> <sa> <in.smgo> <out.smsa> <k> <max_occ>\n"); return 1; }
	k = atoi(argv[5]);
	max_occ = atoi(argv[6]);
	bwt = bwt_restore_bwt(argv[1]);
	bwt_restore_sa(argv[2], bwt);
	in = fopen(argv[3], "rb");
	out = fopen(argv[4], "wb");
	if (!in || !out) return 1;
	if (fread(magic, 1, 8, in) != 8 || memcmp(magic, SMGO_MAGIC, 8) != 0) return 1;
	if (fread(&n_reads, 8, 1, in) != 1) return 1;
	smsa_write_header(out, n_reads);
	for (r = 0; r < n_reads; ++r) {
		uint32_t n_calls, c, n_occ = 0;
		long pos = ftell(out);
		if (fread(&n_calls, 4, 1, in) != 1) return 1;
		fwrite(&n_occ, 4, 1, out);
		for (c = 0; c < n_calls; ++c) {
			uint32_t n, i;
			if (fread(&n, 4, 1, in) != 1) return 1;
			for (i = 0; i < n; ++i) {
				uint64_t v[4];
				int slen;
				bwtint_t j;
				if (fread(v, 8, 4, in) != 4) return 1;
				slen = (uint32_t)v[3] - (int)(v[3] >> 32);
				if (slen < k || v[2] > (uint64_t)max_occ) continue;
				for (j = 0; j < v[2]; ++j) {
					uint64_t p = bwt_sa(bwt, v[0] + j);
					fwrite(&p, 8, 1, out);
					++n_occ;
				}
			}
		}
		{
			long end = ftell(out);
			fseek(out, pos, SEEK_SET);
			fwrite(&n_occ, 4, 1, out);
			fseek(out, end, SEEK_SET);
		}
	}
	fclose(in);
	fclose(out);
	bwt_destroy(bwt);
	return 0;
}

/* mem_seed_t / mem_chain_t / mem_chain_v are private to software/bwamem.c
 * (:317-327); these are layout-identical declarations to read its results */
typedef struct { int64_t rbeg; int32_t qbeg, len; } h_seed_t;
typedef struct { int n, m; int64_t pos; h_seed_t *seeds; } h_chain_t;
typedef struct { size_t n, m; h_chain_t *a; } h_chain_v;
extern h_chain_v mem_chain(const mem_opt_t *opt, const bwt_t *bwt, int64_t l_pac, int len, const uint8_t *seq);
extern int mem_chain_flt(const mem_opt_t *opt, int n_chn, h_chain_t *chains);

static int cmd_chain(int argc, char **argv)
{
	bwt_t *bwt;
	smrd_reads_t r;
	mem_opt_t *opt;
	FILE *out;
	uint64_t i;
	int filter;
	if (argc < 15) {
		fprintf(stderr, "usage: chain <bwt> <sa> <reads> <out> <k> <r> <s> <sw> <max_occ> <w> <gap> <mask> <drop> <filter>\n");
		return 1;
	}
	opt = mem_opt_init();
	opt->min_seed_len = atoi(argv[5]);
	opt->split_factor = (float)atof(argv[6]);
	opt->split_width = atoi(argv[7]);
	if (atoi(argv[8]) == 2) opt->flag |= MEM_F_NO_EXACT;
	opt->max_occ = atoi(argv[9]);
	opt->w = atoi(argv[10]);
	opt->max_chain_gap = atoi(argv[11]);
	opt->mask_level = (float)atof(argv[12]);
	opt->chain_drop_ratio = (float)atof(argv[13]);
	filter = atoi(argv[14]);
	bwt = bwt_restore_bwt(argv[1]);
	bwt_restore_sa(argv[2], bwt);
	if (smrd_load(argv[3], &r) != 0) return 1;
	out = fopen(argv[4], "wb");
	if (!out) return 1;
	smch_write_header(out, r.n_reads);
	for (i = 0; i < r.n_reads; ++i) {
		h_chain_v c = mem_chain(opt, bwt, (int64_t)(bwt->seq_len >> 1), r.len[i], r.codes + r.off[i]);
		uint32_t nc, j;
		if (filter) c.n = mem_chain_flt(opt, (int)c.n, c.a);
		nc = (uint32_t)c.n;
		fwrite(&nc, 4, 1, out);
		for (j = 0; j < nc; ++j) {
			uint32_t n = (uint32_t)c.a[j].n;
			int k;
			fwrite(&c.a[j].pos, 8, 1, out);
			fwrite(&n, 4, 1, out);
			for (k = 0; k < c.a[j].n; ++k) {
				fwrite(&c.a[j].seeds[k].rbeg, 8, 1, out);
				fwrite(&c.a[j].seeds[k].qbeg, 4, 1, out);
				fwrite(&c.a[j].seeds[k].len, 4, 1, out);
			}
		}
		for (j = 0; j < c.m && j < c.n; ++j) free(c.a[j].seeds);
		free(c.a);
	}
	fclose(out);
	smrd_free(&r);
	free(opt);
	bwt_destroy(bwt);
	return 0;
}

extern int mem_chain2aln_short(const mem_opt_t *opt, int64_t l_pac, const uint8_t *pac, int l_query,
		const uint8_t *query, const h_chain_t *c, mem_alnreg_v *av);
extern void mem_chain2aln(const mem_opt_t *opt, int64_t l_pac, const uint8_t *pac, int l_query, const uint8_t *query,
		const h_chain_t *c, mem_alnreg_v *av);

static int cmd_aln(int argc, char **argv)
{
	bwt_t *bwt;
	smrd_reads_t r;
	mem_opt_t *opt;
	FILE *out, *fp;
	uint64_t i;
	int64_t l_pac;
	uint8_t *pac;
	double t_aln = 0.0;
	uint64_t n_regs = 0;
	if (argc < 15) {
		fprintf(stderr, "usage: aln <bwt> <sa> <pac> <reads> <out> <k> <r> <s> <sw> <max_occ> <w> <gap> <mask> <drop>\n");
		return 1;
	}
	opt = mem_opt_init();
	opt->min_seed_len = atoi(argv[6]);
	opt->split_factor = (float)atof(argv[7]);
	opt->split_width = atoi(argv[8]);
	if (atoi(argv[9]) == 2) opt->flag |= MEM_F_NO_EXACT;
	opt->max_occ = atoi(argv[10]);
	opt->w = atoi(argv[11]);
	opt->max_chain_gap = atoi(argv[12]);
	opt->mask_level = (float)atof(argv[13]);
	opt->chain_drop_ratio = (float)atof(argv[14]);
	bwt = bwt_restore_bwt(argv[1]);
	bwt_restore_sa(argv[2], bwt);
	l_pac = (int64_t)(bwt->seq_len >> 1);
	pac = calloc(l_pac / 4 + 1, 1);
	fp = fopen(argv[3], "rb");
	if (!fp || fread(pac, 1, (l_pac + 3) / 4, fp) != (size_t)((l_pac + 3) / 4)) return 1;
	fclose(fp);
	if (smrd_load(argv[4], &r) != 0) return 1;
	out = fopen(argv[5], "wb");
	if (!out) return 1;
	fwrite("SMRG0001", 1, 8, out);
	fwrite(&r.n_reads, 8, 1, out);
	for (i = 0; i < r.n_reads; ++i) {
		const uint8_t *q = r.codes + r.off[i];
		h_chain_v c = mem_chain(opt, bwt, l_pac, r.len[i], q);
		mem_alnreg_v av = { 0, 0, 0 };
		uint32_t j, n;
		c.n = mem_chain_flt(opt, (int)c.n, c.a);
		t_aln -= now_s();
		for (j = 0; j < c.n; ++j)   /* software/bwamem.c:1452-1460 */
			if (mem_chain2aln_short(opt, l_pac, pac, r.len[i], q, &c.a[j], &av) > 0)
				mem_chain2aln(opt, l_pac, pac, r.len[i], q, &c.a[j], &av);
		t_aln += now_s();
		n_regs += av.n;
		n = (uint32_t)av.n;
		fwrite(&n, 4, 1, out);
		for (j = 0; j < n; ++j) {
			const mem_alnreg_t *a = &av.a[j];
			int32_t v[10] = { a->qb, a->qe, a->score, a->truesc, a->sub, a->csub, a->sub_n, a->w, a->seedcov,
				a->secondary };
			fwrite(&a->rb, 8, 1, out);
			fwrite(&a->re, 8, 1, out);
			fwrite(v, 4, 10, out);
		}
		free(av.a);
		for (j = 0; j < c.m && j < c.n; ++j) free(c.a[j].seeds);
		free(c.a);
	}
	fclose(out);
	/* the chains -> regions loop alone, one thread: the alignment stage's CPU baseline */
	fprintf(stderr, "chain2aln_seconds=%.6f reads=%llu regions=%llu\n", t_aln, (unsigned long long)r.n_reads,
			(unsigned long long)n_regs);
	smrd_free(&r);
	free(pac);
	free(opt);
	bwt_destroy(bwt);
	return 0;
}

/* ksw <tasks.smkt> <out.smkr>: the reference's own ksw_extend2 on every task */
extern int ksw_extend2(int qlen, const uint8_t *query, int tlen, const uint8_t *target, int m, const int8_t *mat,
		int o_del, int e_del, int o_ins, int e_ins, int w, int end_bonus, int zdrop, int h0, int *_qle, int *_tle,
		int *_gtle, int *_gscore, int *_max_off);

typedef struct { uint64_t q_off, t_off; int32_t qlen, tlen, w, end_bonus, zdrop, h0; } ksw_task_t;

static int cmd_ksw(int argc, char **argv)
{
	char magic[8];
	uint64_t n, qb, tb, i;
	int8_t mat[28];
	int32_t pen[4];
	ksw_task_t *T;
	uint8_t *q, *t;
	FILE *fp, *out;
	if (argc < 3) { fprintf(stderr, "usage: ksw <tasks.smkt> <out.smkr>\n"); return 1; }
	fp = fopen(argv[1], "rb");
	if (!fp) return 1;
	if (fread(magic, 1, 8, fp) != 8 || memcmp(magic, SMKT_MAGIC, 8) != 0) return 1;
	if (fread(&n, 8, 1, fp) != 1 || fread(&qb, 8, 1, fp) != 1 || fread(&tb, 8, 1, fp) != 1) return 1;
	if (fread(mat, 1, 28, fp) != 28 || fread(pen, 4, 4, fp) != 4) return 1;
	T = malloc(sizeof(ksw_task_t) * (n ? n : 1));
	q = malloc(qb ? qb : 1);
	t = malloc(tb ? tb : 1);
	if (fread(T, sizeof(ksw_task_t), n, fp) != n || fread(q, 1, qb, fp) != qb || fread(t, 1, tb, fp) != tb) return 1;
	fclose(fp);
	out = fopen(argv[2], "wb");
	if (!out) return 1;
	fwrite(SMKR_MAGIC, 1, 8, out);
	fwrite(&n, 8, 1, out);
	for (i = 0; i < n; ++i) {
		int32_t r[6];
		r[0] = ksw_extend2(T[i].qlen, q + T[i].q_off, T[i].tlen, t + T[i].t_off, 5, mat, pen[0], pen[1], pen[2], pen[3],
				T[i].w, T[i].end_bonus, T[i].zdrop, T[i].h0, &r[1], &r[2], &r[3], &r[4], &r[5]);
		fwrite(r, 4, 6, out);
	}
	fclose(out);
	free(T); free(q); free(t);
	return 0;
}

typedef struct { uint64_t q_off, t_off; int32_t qlen, tlen, xtra, pad; } kswa_task_t;

static int cmd_kswa(int argc, char **argv)
{
	char magic[8];
	uint64_t n, qb, tb, i;
	int8_t mat[28];
	int32_t pen[4];
	kswa_task_t *T;
	uint8_t *q, *t;
	FILE *fp, *out;
	if (argc < 3) { fprintf(stderr, "usage: kswa <tasks.smat> <out.smar>\n"); return 1; }
	fp = fopen(argv[1], "rb");
	if (!fp) return 1;
	if (fread(magic, 1, 8, fp) != 8 || memcmp(magic, "SMAT0001", 8) != 0) return 1;
	if (fread(&n, 8, 1, fp) != 1 || fread(&qb, 8, 1, fp) != 1 || fread(&tb, 8, 1, fp) != 1) return 1;
	if (fread(mat, 1, 28, fp) != 28 || fread(pen, 4, 4, fp) != 4) return 1;
	T = malloc(sizeof(kswa_task_t) * (n ? n : 1));
	q = malloc(qb ? qb : 1);
	t = malloc(tb ? tb : 1);
	if (fread(T, sizeof(kswa_task_t), n, fp) != n || fread(q, 1, qb, fp) != qb || fread(t, 1, tb, fp) != tb) return 1;
	fclose(fp);
	out = fopen(argv[2], "wb");
	if (!out) return 1;
	fwrite("SMAR0001", 1, 8, out);
	fwrite(&n, 8, 1, out);
	for (i = 0; i < n; ++i) {
		kswr_t r = ksw_align2(T[i].qlen, q + T[i].q_off, T[i].tlen, t + T[i].t_off, 5, mat, pen[0], pen[1], pen[2], pen[3],
				T[i].xtra, 0);
		int32_t v[7] = { r.score, r.te, r.qe, r.score2, r.te2, r.tb, r.qb };
		fwrite(v, 4, 7, out);
	}
	fclose(out);
	free(T); free(q); free(t);
	return 0;
}

/* the HARP-path globals of software/fastmap.c:27-29 and software/main.c:28 (their
 * definitions are linked from the reference objects; allocated here as
 * main_mem and the manager thread do) */
extern unsigned long int **worker_mem;
extern volatile unsigned char *sw_handshake;
extern char *bwa_pg;

static int cmd_mem(int argc, char **argv)
{
	mem_opt_t *opt;
	bwt_t *bwt;
	bntseq_t *bns;
	uint8_t *pac;
	char *tmp;
	gzFile fp;
	kseq_t *ks;
	bseq1_t *seqs;
	int i, n;
	int64_t n_processed = 0;
	if (argc < 6) { fprintf(stderr, "usage: mem <prefix> <reads.fq> <threads> <batch> <pe> [pg]\n"); return 1; }
	opt = mem_opt_init();
	opt->n_threads = atoi(argv[3]);
	opt->batch_size = atoi(argv[4]) > 1? atoi(argv[4]) : 1;
	if (atoi(argv[5])) opt->flag |= MEM_F_PE;
	bwa_pg = argc > 6? argv[6] : "@PG\tID:bwa\tPN:bwa\tVN:0.7.8-r455";
	tmp = calloc(strlen(argv[1]) + 5, 1);
	strcat(strcpy(tmp, argv[1]), ".bwt");
	bwt = bwt_restore_bwt(tmp);
	strcat(strcpy(tmp, argv[1]), ".sa");
	bwt_restore_sa(tmp, bwt);
	free(tmp);
	bns = bns_restore(argv[1]);
	pac = calloc(bns->l_pac / 4 + 1, 1);
	err_fread_noeof(pac, 1, bns->l_pac / 4 + 1, bns->fp_pac);
	err_fclose(bns->fp_pac);
	bns->fp_pac = 0;
	fp = gzopen(argv[2], "r");
	if (!fp) return 1;
	ks = kseq_init(fp);
	bwa_print_sam_hdr(bns, 0);
	worker_mem = (unsigned long int **)malloc(sizeof(unsigned long int *) * opt->n_threads);
	for (i = 0; i < opt->n_threads; ++i)
		worker_mem[i] = (unsigned long int *)malloc(sizeof(unsigned long int) * 1024 * 1024 + 1);
	sw_handshake = (unsigned char *)calloc(opt->n_threads + 1, 1);
	while ((seqs = bseq_read(opt->chunk_size * opt->n_threads, &n, ks, 0)) != 0) {
		if ((opt->flag & MEM_F_PE) && (n & 1)) n = n >> 1 << 1;
		for (i = 0; i < n; ++i) { free(seqs[i].comment); seqs[i].comment = 0; }
		mem_process_seqs(opt, bwt, bns, pac, n_processed, n, seqs, 0);
		n_processed += n;
		for (i = 0; i < n; ++i) {
			err_fputs(seqs[i].sam, stdout);
			free(seqs[i].name); free(seqs[i].comment); free(seqs[i].seq); free(seqs[i].qual); free(seqs[i].sam);
		}
		free(seqs);
	}
	for (i = 0; i < opt->n_threads; ++i) free(worker_mem[i]);
	free(worker_mem);
	free((void*)sw_handshake);
	kseq_destroy(ks);
	gzclose(fp);
	free(pac);
	bns_destroy(bns);
	bwt_destroy(bwt);
	free(opt);
	fflush(stdout);
	return 0;
}

int main(int argc, char **argv)
{
	if (argc < 2) {
		fprintf(stderr, "usage: ref_harness index|smem|bench|sa ...\n");
		return 1;
	}
	if (strcmp(argv[1], "index") == 0) {
		char *av[7];
		if (argc < 4) return 1;
		av[0] = "index"; av[1] = "-a"; av[2] = "is"; av[3] = "-p"; av[4] = argv[3]; av[5] = argv[2]; av[6] = 0;
		return bwa_index(6, av);
	}
	if (strcmp(argv[1], "smem") == 0) return cmd_smem(argc - 1, argv + 1);
	if (strcmp(argv[1], "bench") == 0) return cmd_bench(argc - 1, argv + 1);
	if (strcmp(argv[1], "sa") == 0) return cmd_sa(argc - 1, argv + 1);
	if (strcmp(argv[1], "chain") == 0) return cmd_chain(argc - 1, argv + 1);
	if (strcmp(argv[1], "ksw") == 0) return cmd_ksw(argc - 1, argv + 1);
	if (strcmp(argv[1], "aln") == 0) return cmd_aln(argc - 1, argv + 1);
	if (strcmp(argv[1], "mem") == 0) return cmd_mem(argc - 1, argv + 1);
	if (strcmp(argv[1], "kswa") == 0) return cmd_kswa(argc - 1, argv + 1);
	fprintf(stderr, "unknown command %s\n", argv[1]);
	return 1;
}
