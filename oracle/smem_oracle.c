/*
 * smem_oracle.c — TEST INFRASTRUCTURE ONLY.  CPU restatement of the
 * reference SMEM seeding path (see smem_oracle.h for the function map).
 * Written from the reference's behaviour; every step cites the line it
 * follows.  Used as the parity checker and as the "port" CPU baseline.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <sys/time.h>
#include "smem_oracle.h"

/* ---------------------------------------------------------------- index */

/* byte -> four 8-bit base counts (software/bwt.c:60-69) */
static void gen_cnt_table(uint32_t t[256])
{
	int b, s;
	for (b = 0; b < 256; ++b) {
		uint32_t packed = 0;
		for (s = 0; s < 4; ++s) {                 /* the 4 symbols of the byte */
			int sym = (b >> (2 * s)) & 3;
			packed += 1u << (sym * 8);
		}
		t[b] = packed;
	}
}

orc_bwt_t *orc_bwt_load(const char *fn)
{
	/* .bwt = primary, L2[1..4], then bwt words (software/bwt.c:899-918) */
	FILE *fp = fopen(fn, "rb");
	orc_bwt_t *b;
	long sz;
	if (!fp) return 0;
	fseek(fp, 0, SEEK_END);
	sz = ftell(fp);
	fseek(fp, 0, SEEK_SET);
	b = (orc_bwt_t*)calloc(1, sizeof(*b));
	b->bwt_size = (uint64_t)(sz - 40) / 4;
	b->bwt = (uint32_t*)malloc(b->bwt_size * 4 + 64);
	if (fread(&b->primary, 8, 1, fp) != 1 || fread(b->L2 + 1, 8, 4, fp) != 4
			|| fread(b->bwt, 4, b->bwt_size, fp) != b->bwt_size) {
		fclose(fp); free(b->bwt); free(b); return 0;
	}
	fclose(fp);
	b->L2[0] = 0;
	b->seq_len = b->L2[4];
	b->owns = 1;
	gen_cnt_table(b->cnt_table);
	return b;
}

orc_bwt_t *orc_bwt_wrap(const uint32_t *bwt, uint64_t bwt_size, uint64_t primary, const uint64_t L2[5])
{
	orc_bwt_t *b = (orc_bwt_t*)calloc(1, sizeof(*b));
	b->bwt = (uint32_t*)bwt;
	b->bwt_size = bwt_size;
	b->primary = primary;
	memcpy(b->L2, L2, sizeof(b->L2));
	b->seq_len = L2[4];
	gen_cnt_table(b->cnt_table);
	return b;
}

void orc_bwt_free(orc_bwt_t *b)
{
	if (!b) return;
	if (b->owns) free(b->bwt);
	free(b);
}

void orc_free(void *p) { free(p); }

/* ------------------------------------------------------------------ occ */

/* Occ(c, k) for the 4 bases: counts of each base in BWT[0..k] with the $ row
 * removed (software/bwt.c:187-204).  Bucket = 128 symbols: 4 x u64
 * checkpoint followed by 8 x u32 words of 16 MSB-first 2-bit symbols
 * (software/bwt.h:72-73). */
void orc_occ4(const orc_bwt_t *b, uint64_t k, uint64_t cnt[4])
{
	const uint32_t *bucket, *w;
	uint32_t acc = 0, last;
	int i, nfull;
	if (k == (uint64_t)-1) { cnt[0] = cnt[1] = cnt[2] = cnt[3] = 0; return; }
	k -= (k >= b->primary);                        /* $ is not stored */
	bucket = b->bwt + ((k >> 7) << 4);
	memcpy(cnt, bucket, 32);
	w = bucket + 8;
	nfull = (int)((k & 127) >> 4);
	for (i = 0; i < nfull; ++i) {
		uint32_t x = w[i];
		acc += b->cnt_table[x & 0xff] + b->cnt_table[(x >> 8) & 0xff]
			+ b->cnt_table[(x >> 16) & 0xff] + b->cnt_table[x >> 24];
	}
	/* keep the (k&15)+1 leading symbols of the partial word; the masked tail
	 * reads as A and is subtracted from the A count */
	last = w[nfull] & ~((1u << ((~k & 15) << 1)) - 1);
	acc += b->cnt_table[last & 0xff] + b->cnt_table[(last >> 8) & 0xff]
		+ b->cnt_table[(last >> 16) & 0xff] + b->cnt_table[last >> 24];
	acc -= (uint32_t)(~k & 15);
	cnt[0] += acc & 0xff;
	cnt[1] += (acc >> 8) & 0xff;
	cnt[2] += (acc >> 16) & 0xff;
	cnt[3] += acc >> 24;
}

/* bidirectional extension of ik in all four directions (software/bwt.c:416-429) */
void orc_extend(const orc_bwt_t *b, const orc_intv_t *ik, orc_intv_t ok[4], int is_back)
{
	uint64_t tk[4], tl[4];
	int c, a = !is_back;               /* coordinate searched through the BWT */
	uint64_t k = ik->x[a] - 1;
	orc_occ4(b, k, tk);                /* bwt_2occ4 == two bwt_occ4 (software/bwt.c:213-214) */
	orc_occ4(b, k + ik->x[2], tl);
	for (c = 0; c < 4; ++c) {
		ok[c].x[a] = b->L2[c] + 1 + tk[c];
		ok[c].x[2] = tl[c] - tk[c];
	}
	/* the other coordinate: +1 if the interval covers the $ row, then the
	 * cumulative sizes in reverse-complement base order */
	ok[3].x[is_back] = ik->x[is_back] + (ik->x[a] <= b->primary && ik->x[a] + ik->x[2] - 1 >= b->primary);
	ok[2].x[is_back] = ok[3].x[is_back] + ok[3].x[2];
	ok[1].x[is_back] = ok[2].x[is_back] + ok[2].x[2];
	ok[0].x[is_back] = ok[1].x[is_back] + ok[1].x[2];
}

/* -------------------------------------------------------------- vectors */

typedef struct { size_t n, m; orc_intv_t *a; } ivec_t;

static void iv_push(ivec_t *v, const orc_intv_t *x)
{
	if (v->n == v->m) {
		v->m = v->m ? v->m << 1 : 16;
		v->a = (orc_intv_t*)realloc(v->a, v->m * sizeof(orc_intv_t));
	}
	v->a[v->n++] = *x;
}

static void iv_reverse(ivec_t *v)
{
	size_t i;
	for (i = 0; i < v->n / 2; ++i) {
		orc_intv_t t = v->a[i];
		v->a[i] = v->a[v->n - 1 - i];
		v->a[v->n - 1 - i] = t;
	}
}

typedef struct {
	ivec_t matches, sub, fwd, prev, curr, merged;
	orc_stats_t st;
} worker_t;

/* orc_seed_trace: the Occ64 bucket index of every load the GPU kernel makes,
 * in extend order (bit 31: the second bucket of the same extend) */
typedef struct { uint32_t *p; uint64_t n, cap; } trace_t;
static __thread trace_t *g_trace;

static void trace_put(uint32_t v)
{
	if (g_trace->n < g_trace->cap) g_trace->p[g_trace->n] = v;
	g_trace->n++;
}

/* returns the Occ64 bucket loads of the extend (0 when not used) */
static int count_extend(const orc_bwt_t *b, const orc_intv_t *ik, int is_back, int used, orc_stats_t *st)
{
	uint64_t k = ik->x[!is_back] - 1, l = k + ik->x[2];
	uint64_t kk = k - (k >= b->primary), ll = l - (l >= b->primary);
	uint64_t nb = (k == (uint64_t)-1) ? 1 : 1 + ((kk >> 7) != (ll >> 7));
	int nb64 = (k == (uint64_t)-1) ? 1 : 1 + ((kk >> 6) != (ll >> 6));
	st->n_ext_ref++;
	st->n_bkt_ref += nb;
	if (used) {
		st->n_ext++;
		st->n_bkt += nb;
		st->n_bkt64 += nb64;
		if (g_trace) {
			if (k == (uint64_t)-1) trace_put((uint32_t)(ll >> 6));
			else {
				trace_put((uint32_t)(kk >> 6));
				if (nb64 == 2) trace_put((uint32_t)(ll >> 6) | 0x80000000u);
			}
		}
	}
	return used ? nb64 : 0;
}

/* ------------------------------------------------------------ bwt_smem1 */

/* SMEMs covering position x (software/bwt.c:776-835). Fills mem in start
 * order, returns the end of the longest exact match starting at x. */
/* list entries per lane the GPU kernel keeps in LDS (smem_kernels.hip NLIST,
 * 11 in the product build; ORC_LIST_LDS overrides): the n_*_hi / n_fwd_spill
 * counters model the kernel's arena traffic (an entry at index >= NL) */
static int list_lds(void)
{
	static int v = -1;
	if (v < 0) { const char *e = getenv("ORC_LIST_LDS"); v = e ? atoi(e) : 11; }
	return v;
}

static int smem1(const orc_bwt_t *b, int len, const uint8_t *q, int x, int min_intv, ivec_t *mem, worker_t *w)
{
	const int NL = list_lds();
	orc_intv_t ik, ok[4];
	ivec_t *prev = &w->prev, *curr = &w->curr, *t;
	int i, j, c, ret;
	uint64_t ik_prev2 = 0;
	int had_u1 = 0, has_u1 = 0;
	/* text-mode model: tm = ik came from a text compare (x1 unknown), tm_pos = its text
	 * position is known; for the backward list's entry 0 (the only one that can have
	 * size 1: sizes strictly grow along a list) p0_lazy = x0 unknown, p0_pos likewise */
	int tm = 0, tm_pos = 0, p0_lazy = 0, p0_pos = 0, c0_lazy = 0, c0_pos = 0, in_run = 0;

	mem->n = 0;
	w->st.n_smem1++;
	if (q[x] > 3) return x + 1;
	if (min_intv < 1) min_intv = 1;
	/* bwt_set_intv (software/bwt.h:80) */
	ik.x[0] = b->L2[q[x]] + 1;
	ik.x[2] = b->L2[q[x] + 1] - b->L2[q[x]];
	ik.x[1] = b->L2[3 - q[x]] + 1;
	ik.info = (uint64_t)(x + 1);

	/* forward extension, pushing ik each time the interval shrinks
	 * (software/bwt.c:791-805) */
	w->fwd.n = 0;
	for (i = x + 1; i < len; ++i) {
		if (q[i] > 3) { iv_push(&w->fwd, &ik); break; }      /* ambiguous base */
		c = 3 - q[i];
		orc_extend(b, &ik, ok, 0);
		{
			int nb64 = count_extend(b, &ik, 0, 1, &w->st);
			if (ik.x[2] == 1) {  /* text mode: q[i] against the text after the occurrence */
				w->st.n_tm_saved += nb64;
				if (!tm_pos) { w->st.n_tm_sa++; tm_pos = 1; w->st.n_tm_runs++; }
				w->st.n_tm_bases++;
			}
		}
		w->st.n_ext_fwd++;
		w->st.n_ext_len[i + 1 - x < 32 ? i + 1 - x : 32]++;
		if (i - x <= 12) w->st.n_ext_fwd_k12++;
		if (ik.x[2] == 1) { w->st.n_ext_u1_fwd++; if (i == x + 1 || ik_prev2 != 1) w->st.n_run_u1++; }
		ik_prev2 = ik.x[2];
		if (ok[c].x[2] != ik.x[2]) {
			if (tm) w->st.n_tm_isa++;  /* the pushed interval's exact x1 */
			iv_push(&w->fwd, &ik);
			if (ok[c].x[2] < (uint64_t)min_intv) break;
		}
		tm = ik.x[2] == 1;
		ik = ok[c];
		ik.info = (uint64_t)(i + 1);
	}
	if (i == len) { if (tm) w->st.n_tm_isa++; iv_push(&w->fwd, &ik); }
	w->st.n_fwd_push += w->fwd.n;
	if ((int)w->fwd.n > NL) w->st.n_fwd_spill += w->fwd.n - NL;  /* the LDS ring spills its oldest entries */
	iv_reverse(&w->fwd);                 /* longest match first (software/bwt.c:806) */
	ret = (int)w->fwd.a[0].info;

	/* backward extension of every surviving interval (software/bwt.c:810-829) */
	prev->n = 0;
	for (j = 0; j < (int)w->fwd.n; ++j) iv_push(prev, &w->fwd.a[j]);
	/* prev[0] is the forward phase's last push: exact, at the forward run's text position
	 * when the forward phase compared text (its x0 never changed) */
	p0_lazy = 0;
	p0_pos = w->fwd.n > 0 && w->fwd.a[0].x[2] == 1 && tm_pos;
	in_run = p0_pos;
	for (i = x - 1; i >= -1; --i) {
		c = i < 0 ? -1 : (q[i] < 4 ? q[i] : -1);
		curr->n = 0;
		c0_lazy = c0_pos = 0;
		had_u1 = has_u1; has_u1 = 0;
		if (c >= 0) {
			w->st.n_bwd_step++;
			w->st.n_step_hist[prev->n < 16 ? prev->n : 16]++;
		}
		for (j = 0; j < (int)prev->n; ++j) {
			orc_intv_t *p = &prev->a[j];
			if (i < x - 1 && j >= NL) w->st.n_bwd_read_hi++;
			if (c >= 0 && j >= NL) w->st.n_bwd_task_hi++;
			orc_extend(b, p, ok, 1);
			{
				int nb64 = count_extend(b, p, 1, c >= 0, &w->st);
				if (c >= 0 && p->x[2] == 1) {  /* text mode: q[i] against the base before the occurrence */
					w->st.n_tm_saved += nb64;
					if (!p0_pos) w->st.n_tm_sa++;
					if (!in_run) w->st.n_tm_runs++;
					w->st.n_tm_bases++;
				}
			}
			if (c >= 0) { int sl = (int)(uint32_t)p->info - i; w->st.n_ext_len[sl < 32 ? sl : 32]++; }
			if (c >= 0 && p->x[2] == 1) {
				w->st.n_ext_u1_bwd++;
				if (!had_u1) w->st.n_run_u1++;
				has_u1 = 1;
			}
			if (c < 0 || ok[c].x[2] < (uint64_t)min_intv) {
				/* p cannot be extended: it is a MEM unless a longer one was
				 * already kept at this i, or it is contained in the last one */
				if (curr->n == 0 && (mem->n == 0 || (uint64_t)(i + 1) < mem->a[mem->n - 1].info >> 32)) {
					orc_intv_t e = *p;
					if (j == 0 && p0_lazy) w->st.n_tm_isa++;  /* the emitted SMEM's exact x0 */
					e.info |= (uint64_t)(i + 1) << 32;
					iv_push(mem, &e);
				}
			} else if (curr->n == 0 || ok[c].x[2] != curr->a[curr->n - 1].x[2]) {
				if ((int)curr->n >= NL) w->st.n_bwd_push_hi++;
				ok[c].info = p->info;
				if (curr->n == 0) {  /* the new entry 0: lazy when a text compare made it */
					c0_lazy = p->x[2] == 1;
					c0_pos = p->x[2] == 1;
				}
				iv_push(curr, &ok[c]);
			}
		}
		if (curr->n == 0) break;
		t = curr; curr = prev; prev = t;
		p0_lazy = c0_lazy; p0_pos = c0_pos;
		in_run = p0_pos;
	}
	iv_reverse(mem);                     /* sorted by start (software/bwt.c:830) */
	return ret;
}

/* ------------------------------------------------------------ smem_next2 */

/* one iterator step (software/bwamem.c:244-305); returns NULL when done */
static const ivec_t *smem_next2(const orc_bwt_t *b, const uint8_t *q, int len, int *start,
		int split_len, int split_width, int start_width, worker_t *w)
{
	int i, j, max = 0, max_i = 0, ori_start;
	w->matches.n = w->sub.n = 0;
	if (*start >= len || *start < 0) return 0;
	while (*start < len && q[*start] > 3) ++*start;       /* skip ambiguous bases */
	if (*start == len) return 0;
	ori_start = *start;
	*start = smem1(b, len, q, ori_start, start_width, &w->matches, w);
	if (w->matches.n == 0) return &w->matches;
	for (i = 0; i < (int)w->matches.n; ++i) {            /* first longest match */
		const orc_intv_t *p = &w->matches.a[i];
		int l = (int)((uint32_t)p->info - (p->info >> 32));
		if (max < l) max = l, max_i = i;
	}
	if (split_len > 0 && max >= split_len && w->matches.a[max_i].x[2] <= (uint64_t)split_width) {
		/* re-seed from the middle of a long unique SMEM (software/bwamem.c:272-278) */
		const orc_intv_t *p = &w->matches.a[max_i];
		int mid = (int)(((uint32_t)p->info + (p->info >> 32)) >> 1);
		smem1(b, len, q, mid, (int)(p->x[2] + 1), &w->sub, w);
		/* ordered merge keyed by (start, len-end) (software/bwamem.c:280-301) */
		w->merged.n = 0;
		i = j = 0;
		while (i < (int)w->matches.n && j < (int)w->sub.n) {
			const orc_intv_t *a = &w->matches.a[i], *s = &w->sub.a[j];
			int64_t xi = (int64_t)(a->info >> 32 << 32 | (uint64_t)(len - (uint32_t)a->info));
			int64_t xj = (int64_t)(s->info >> 32 << 32 | (uint64_t)(len - (uint32_t)s->info));
			if (xi < xj) { iv_push(&w->merged, a); ++i; }
			else {
				if ((int)((uint32_t)s->info - (s->info >> 32)) >= max >> 1 && (uint32_t)s->info > (uint32_t)ori_start)
					iv_push(&w->merged, s);
				++j;
			}
		}
		for (; i < (int)w->matches.n; ++i) iv_push(&w->merged, &w->matches.a[i]);
		for (; j < (int)w->sub.n; ++j) {
			const orc_intv_t *s = &w->sub.a[j];
			if ((int)((uint32_t)s->info - (s->info >> 32)) >= max >> 1 && (uint32_t)s->info > (uint32_t)ori_start)
				iv_push(&w->merged, s);
		}
		w->matches.n = 0;
		for (i = 0; i < (int)w->merged.n; ++i) iv_push(&w->matches, &w->merged.a[i]);
	}
	return &w->matches;
}

/* -------------------------------------------------------------- driver */

typedef struct { uint8_t *p; size_t n, m; } bbuf_t;

static void bb_put(bbuf_t *b, const void *src, size_t n)
{
	if (b->n + n > b->m) {
		b->m = (b->n + n) * 2 + 4096;
		b->p = (uint8_t*)realloc(b->p, b->m);
	}
	memcpy(b->p + b->n, src, n);
	b->n += n;
}

typedef struct {
	const orc_bwt_t *b;
	const uint8_t *codes;
	const int64_t *offs;
	const orc_opt_t *opt;
	int64_t beg, end;
	int want_out;
	bbuf_t out;
	uint32_t *n_intv_pr, *n_calls_pr;
	uint64_t *bytes_pr;
	worker_t w;
} job_t;

/* the mem_chain guard + mem_insert_seed loop (software/bwamem.c:600,453-460) */
static void seed_range(job_t *jb)
{
	int64_t r;
	worker_t *w = &jb->w;
	const orc_opt_t *o = jb->opt;
	for (r = jb->beg; r < jb->end; ++r) {
		const uint8_t *q = jb->codes + jb->offs[r];
		int len = (int)(jb->offs[r + 1] - jb->offs[r]);
		int start = 0, split_len;
		uint32_t n_calls = 0, n_intv = 0;
		size_t hdr = jb->out.n;
		uint64_t bkt0 = w->st.n_bkt;
		const ivec_t *a;
		if (jb->want_out) bb_put(&jb->out, &n_calls, 4);
		if (len >= o->min_seed_len) {
			split_len = (int)(o->min_seed_len * o->split_factor + .499);
			split_len = split_len < len ? split_len : len;
			w->st.n_bases += (uint64_t)len;
			while ((a = smem_next2(jb->b, q, len, &start, split_len, o->split_width, o->start_width, w)) != 0) {
				++n_calls;
				n_intv += (uint32_t)a->n;
				if (jb->want_out) {
					uint32_t n = (uint32_t)a->n;
					bb_put(&jb->out, &n, 4);
					bb_put(&jb->out, a->a, a->n * sizeof(orc_intv_t));
				}
			}
		}
		if (jb->want_out) memcpy(jb->out.p + hdr, &n_calls, 4);
		w->st.n_calls += n_calls;
		w->st.n_intv += n_intv;
		if (jb->n_intv_pr) jb->n_intv_pr[r] = n_intv;
		if (jb->n_calls_pr) jb->n_calls_pr[r] = n_calls;
		if (jb->bytes_pr) /* algorithmic bytes: DESIGN.md "roofline" */
			jb->bytes_pr[r] = 64 * (w->st.n_bkt - bkt0) + (len >= o->min_seed_len ? (uint64_t)len : 0) + 32ull * n_intv;
	}
}

static void *job_main(void *data) { seed_range((job_t*)data); return 0; }

static void free_worker(worker_t *w)
{
	free(w->matches.a); free(w->sub.a); free(w->fwd.a); free(w->prev.a); free(w->curr.a); free(w->merged.a);
}

static void add_stats(orc_stats_t *d, const orc_stats_t *s)
{
	d->n_calls += s->n_calls; d->n_intv += s->n_intv; d->n_smem1 += s->n_smem1;
	d->n_ext += s->n_ext; d->n_ext_ref += s->n_ext_ref; d->n_bkt += s->n_bkt;
	d->n_bkt_ref += s->n_bkt_ref; d->n_bases += s->n_bases; d->n_bkt64 += s->n_bkt64;
	d->n_ext_fwd += s->n_ext_fwd; d->n_ext_u1_fwd += s->n_ext_u1_fwd; d->n_ext_u1_bwd += s->n_ext_u1_bwd;
	d->n_run_u1 += s->n_run_u1; d->n_ext_fwd_k12 += s->n_ext_fwd_k12;
	{ int k; for (k = 0; k < 33; ++k) d->n_ext_len[k] += s->n_ext_len[k]; }
	d->n_fwd_push += s->n_fwd_push; d->n_bwd_push_hi += s->n_bwd_push_hi; d->n_bwd_read_hi += s->n_bwd_read_hi;
	d->n_fwd_spill += s->n_fwd_spill;
	d->n_bwd_step += s->n_bwd_step; d->n_bwd_task_hi += s->n_bwd_task_hi;
	d->n_tm_saved += s->n_tm_saved; d->n_tm_sa += s->n_tm_sa; d->n_tm_isa += s->n_tm_isa;
	d->n_tm_runs += s->n_tm_runs; d->n_tm_bases += s->n_tm_bases;
	{ int k; for (k = 0; k < 17; ++k) d->n_step_hist[k] += s->n_step_hist[k]; }
}

int orc_seed(const orc_bwt_t *b, int64_t n_reads, const uint8_t *codes, const int64_t *offs,
		const orc_opt_t *opt, int n_threads,
		uint8_t **out, uint64_t *out_len,
		uint32_t *n_intv_per_read, uint32_t *n_calls_per_read, uint64_t *bytes_per_read,
		orc_stats_t *stats)
{
	int t;
	job_t *jobs;
	pthread_t *tid;
	if (n_threads < 1) n_threads = 1;
	if (n_threads > n_reads && n_reads > 0) n_threads = (int)n_reads;
	jobs = (job_t*)calloc(n_threads, sizeof(job_t));
	tid = (pthread_t*)calloc(n_threads, sizeof(pthread_t));
	for (t = 0; t < n_threads; ++t) {
		job_t *j = &jobs[t];
		j->b = b; j->codes = codes; j->offs = offs; j->opt = opt;
		j->beg = n_reads * t / n_threads;
		j->end = n_reads * (t + 1) / n_threads;
		j->want_out = out != 0;
		j->n_intv_pr = n_intv_per_read; j->n_calls_pr = n_calls_per_read; j->bytes_pr = bytes_per_read;
		if (n_threads > 1) pthread_create(&tid[t], 0, job_main, j);
	}
	if (n_threads == 1) seed_range(&jobs[0]);
	else for (t = 0; t < n_threads; ++t) pthread_join(tid[t], 0);
	if (stats) memset(stats, 0, sizeof(*stats));
	if (out) {
		bbuf_t all = {0, 0, 0};
		uint64_t nr = (uint64_t)n_reads;
		bb_put(&all, "SMGO0001", 8);
		bb_put(&all, &nr, 8);
		for (t = 0; t < n_threads; ++t) bb_put(&all, jobs[t].out.p, jobs[t].out.n);
		*out = all.p;
		if (out_len) *out_len = all.n;
	}
	for (t = 0; t < n_threads; ++t) {
		if (stats) add_stats(stats, &jobs[t].w.st);
		free(jobs[t].out.p);
		free_worker(&jobs[t].w);
	}
	free(jobs); free(tid);
	return 0;
}

/* The Occ64 bucket trace of seeding reads [0, n_reads) on one thread (a
 * replay input: tools/replay_ceiling.hip); read r's loads are
 * out[read_off[r] .. read_off[r + 1]).  Returns the total, which may exceed
 * cap (then only the first cap were written). */
int64_t orc_seed_trace(const orc_bwt_t *b, int64_t n_reads, const uint8_t *codes, const int64_t *offs,
		const orc_opt_t *opt, uint32_t *out, uint64_t cap, uint64_t *read_off)
{
	job_t jb;
	trace_t tr = {out, 0, cap};
	int64_t r;
	memset(&jb, 0, sizeof(jb));
	jb.b = b; jb.codes = codes; jb.offs = offs; jb.opt = opt;
	g_trace = &tr;
	for (r = 0; r < n_reads; ++r) {
		read_off[r] = tr.n;
		jb.beg = r; jb.end = r + 1;
		seed_range(&jb);
	}
	read_off[n_reads] = tr.n;
	g_trace = 0;
	free_worker(&jb.w);
	return (int64_t)tr.n;
}

double orc_seed_timed(const orc_bwt_t *b, int64_t n_reads, const uint8_t *codes, const int64_t *offs,
		const orc_opt_t *opt, int n_threads, orc_stats_t *stats)
{
	struct timeval t0, t1;
	gettimeofday(&t0, 0);
	orc_seed(b, n_reads, codes, offs, opt, n_threads, 0, 0, 0, 0, 0, stats);
	gettimeofday(&t1, 0);
	return (t1.tv_sec - t0.tv_sec) + (t1.tv_usec - t0.tv_usec) * 1e-6;
}

/* ------------------------------------------------------- SA lookup (bwt_sa) */

orc_sa_t *orc_sa_load(const char *fn)
{
	/* .sa: primary, L2[1..4], sa_intv, seq_len, sa[1 .. n_sa-1] (software/bwt.c:852-897) */
	uint64_t hdr[7];
	orc_sa_t *s;
	FILE *fp = fopen(fn, "rb");
	if (!fp) return 0;
	if (fread(hdr, 8, 7, fp) != 7) { fclose(fp); return 0; }
	s = (orc_sa_t*)calloc(1, sizeof(orc_sa_t));
	s->sa_intv = hdr[5];
	s->seq_len = hdr[6];
	s->n_sa = (s->seq_len + s->sa_intv) / s->sa_intv;
	s->sa = (uint64_t*)malloc(8 * s->n_sa);
	s->sa[0] = (uint64_t)-1;
	if (fread(s->sa + 1, 8, s->n_sa - 1, fp) != s->n_sa - 1) { fclose(fp); free(s->sa); free(s); return 0; }
	fclose(fp);
	s->owns = 1;
	return s;
}

orc_sa_t *orc_sa_wrap(const uint64_t *sa, uint64_t n_sa, uint64_t sa_intv, uint64_t seq_len)
{
	orc_sa_t *s = (orc_sa_t*)calloc(1, sizeof(orc_sa_t));
	s->sa = (uint64_t*)sa;
	s->n_sa = n_sa;
	s->sa_intv = sa_intv;
	s->seq_len = seq_len;
	return s;
}

void orc_sa_free(orc_sa_t *s)
{
	if (!s) return;
	if (s->owns) free(s->sa);
	free(s);
}

/* bwt_invPsi (software/bwt.c:71-77): the LF step.  x = k with the $ row
 * removed, c = BWT symbol at x (bwt_B0, software/bwt.h:78), result =
 * L2[c] + Occ(c, k) (bwt_occ, software/bwt.c:125-146); row primary maps to 0 */
static uint64_t inv_psi(const orc_bwt_t *b, uint64_t k)
{
	uint64_t x = k - (k > b->primary), cnt[4];
	uint32_t w = b->bwt[((x >> 7) << 4) + 8 + ((x & 127) >> 4)];
	int c = (int)(w >> ((~x & 15) << 1) & 3);
	if (k == b->primary) return 0;
	orc_occ4(b, k, cnt);  /* == bwt_occ(k, c) for c; k == seq_len gives the totals */
	return b->L2[c] + cnt[c];
}

uint64_t orc_sa_lookup(const orc_bwt_t *b, const orc_sa_t *s, uint64_t k)
{
	uint64_t sa = 0, mask = s->sa_intv - 1;
	while (k & mask) {
		++sa;
		k = inv_psi(b, k);
	}
	return sa + s->sa[k / s->sa_intv];  /* sa[0] = -1 (software/bwt.c:110-113) */
}

typedef struct {
	const orc_bwt_t *b;
	const orc_sa_t *s;
	const uint64_t *k;
	uint64_t *out;
	uint64_t beg, end;
} sa_job_t;

static void *sa_job(void *data)
{
	sa_job_t *j = (sa_job_t*)data;
	uint64_t i;
	for (i = j->beg; i < j->end; ++i) j->out[i] = orc_sa_lookup(j->b, j->s, j->k[i]);
	return 0;
}

void orc_sa_batch(const orc_bwt_t *b, const orc_sa_t *s, const uint64_t *k, uint64_t n, uint64_t *out, int n_threads)
{
	int t;
	sa_job_t *jobs;
	pthread_t *tid;
	if (n_threads < 1) n_threads = 1;
	jobs = (sa_job_t*)calloc(n_threads, sizeof(sa_job_t));
	tid = (pthread_t*)calloc(n_threads, sizeof(pthread_t));
	for (t = 0; t < n_threads; ++t) {
		jobs[t].b = b; jobs[t].s = s; jobs[t].k = k; jobs[t].out = out;
		jobs[t].beg = n * t / n_threads; jobs[t].end = n * (t + 1) / n_threads;
		pthread_create(&tid[t], 0, sa_job, &jobs[t]);
	}
	for (t = 0; t < n_threads; ++t) pthread_join(tid[t], 0);
	free(jobs); free(tid);
}

