/*
 * aln_oracle.c — TEST INFRASTRUCTURE ONLY.  Plain-C restatement of the step
 * after chaining in mem_align1_core (software/bwamem.c:1452-1460): every
 * chain of a read, in order, becomes alignment regions (mem_alnreg_t):
 *
 *   mem_chain2aln_short  software/bwamem.c:805-852
 *     ksw_align2         software/ksw.c:342-364   (forward pass, then the
 *                                                 reverse pass for the start)
 *     ksw_u8 / ksw_i16   software/ksw.c:110-229 / 231-333 (striped local SW)
 *   mem_chain2aln        software/bwamem.c:1040-1188
 *     ksw_extend2        software/ksw.c:379-476   (orc_ksw_extend, ksw_oracle.c)
 *   cal_max_gap          software/bwamem.c:854-861
 *   bns_get_seq          software/bntseq.c:355-376 (_get_pac, software/bntseq.h)
 *
 * The striped local SW is restated as the scalar computation its vector code
 * performs: the query is cut into p blocks of slen columns (p = 16 bytes or
 * 8 words per vector), padded to p * slen columns scoring 0; per target row a
 * first pass carries F only inside each block and sets E from that H, then
 * the lazy-F loop carries F across blocks until it can no longer raise an H
 * (software/ksw.c:176-188).  The row maximum (padding included) feeds the
 * suboptimal-hit list b and the best row; the query end is the smallest
 * column holding the maximum of the best row.  Pinned against the compiled
 * reference's own regions (oracle/_ref/ref_harness aln and the .smrg.gz fixtures in tests/golden).
 * Only tests/ and bench.py's CPU leg use it; the product never links it.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "smem_oracle.h"

#define SHORT_EXT 50   /* MEM_SHORT_EXT, software/bwamem.c:801 */
#define SHORT_LEN 200  /* MEM_SHORT_LEN */
#define BAND_TRY  2    /* MAX_BAND_TRY */
#define XBYTE  0x10000 /* KSW_X*, software/ksw.h:6-9 */
#define XSTOP  0x20000
#define XSUBO  0x40000
#define XSTART 0x80000

typedef struct { int score, te, qe, score2, te2, tb, qb; } swr_t;  /* kswr_t */

static int imax(int a, int b) { return a > b ? a : b; }
static int subs(int a, int b) { return a > b ? a - b : 0; }   /* unsigned saturating subtract */

/* the byte variant's bias and the largest score (ksw_qinit, software/ksw.c:78-85) */
void orc_sw_shift_top(const int8_t *mat, int *shift, int *top)
{
	uint8_t sh = 127, md = 0;
	int k;
	for (k = 0; k < 25; ++k) {
		if (mat[k] < (int8_t)sh) sh = (uint8_t)mat[k];
		if (mat[k] > (int8_t)md) md = (uint8_t)mat[k];
	}
	*top = md;
	*shift = (uint8_t)(256 - sh);
}

/* one ksw_u8 (p = 16) or ksw_i16 (p = 8) run; xtra as there */
extern __thread uint64_t orc_cells_ext, orc_cells_sw;  /* ksw_oracle.c */

static swr_t sw_pass(int p, int qlen, const uint8_t *query, int tlen, const uint8_t *target, const int8_t *mat,
		int o_del, int e_del, int o_ins, int e_ins, int xtra)
{
	const int slen = (qlen + p - 1) / p, qp = slen * p, oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
	const int minsc = (xtra & XSUBO) ? xtra & 0xffff : 0x10000;
	const int endsc = (xtra & XSTOP) ? xtra & 0xffff : 0x10000;
	const int u8 = p == 16;
	swr_t r = { 0, -1, -1, -1, -1, -1, -1 };
	int *H0, *H1, *E, *Hm, *tmp, f[16], gmax = 0, te = -1, i, j, l, k, shift, top;
	int8_t *prof;
	uint64_t *b = 0;
	int n_b = 0, m_b = 0;
	orc_sw_shift_top(mat, &shift, &top);
	H0 = calloc(qp + 1, sizeof(int)); H1 = calloc(qp + 1, sizeof(int));
	E = calloc(qp + 1, sizeof(int)); Hm = calloc(qp + 1, sizeof(int));
	prof = malloc((size_t)5 * (qp + 1));
	for (k = 0; k < 5; ++k)
		for (j = 0; j < qp; ++j) prof[k * qp + j] = j < qlen ? mat[k * 5 + query[j]] : 0;
	for (i = 0; i < tlen; ++i) {
		const int8_t *s = prof + target[i] * qp;
		int rmax = 0;
		orc_cells_sw += (uint64_t)qlen;
		/* pass 1: F inside each block of slen columns */
		for (l = 0; l < p; ++l) {
			int fl = 0;
			for (j = 0; j < slen; ++j) {
				const int q = j + l * slen;
				int h = q ? H0[q - 1] : 0;
				if (u8) {
					h += s[q] + shift;
					if (h > 255) h = 255;
					h = subs(h, shift);
				} else h += s[q];
				h = imax(h, E[q]);
				h = imax(h, fl);
				rmax = imax(rmax, h);
				H1[q] = h;
				E[q] = imax(subs(E[q], e_del), subs(h, oe_del));
				fl = imax(subs(fl, e_ins), subs(h, oe_ins));
			}
			f[l] = fl;
		}
		/* lazy F: shift one block right, sweep, until no F exceeds H - oe_ins */
		for (k = 0; k < 16; ++k) {
			for (l = p - 1; l > 0; --l) f[l] = f[l - 1];
			f[0] = 0;
			for (j = 0; j < slen; ++j) {
				int done = 1;
				for (l = 0; l < p; ++l) {
					const int q = j + l * slen;
					const int h = imax(H1[q], f[l]);
					H1[q] = h;
					f[l] = subs(f[l], e_ins);
					if (f[l] > subs(h, oe_ins)) done = 0;
				}
				if (done) goto end_lazy;
			}
		}
end_lazy:
		if (rmax >= minsc) {  /* the suboptimal list (software/ksw.c:191-199) */
			if (n_b == 0 || (int32_t)b[n_b - 1] + 1 != i) {
				if (n_b == m_b) {
					m_b = m_b ? m_b << 1 : 8;
					b = realloc(b, 8 * m_b);
				}
				b[n_b++] = (uint64_t)rmax << 32 | i;
			} else if ((int)(b[n_b - 1] >> 32) < rmax) b[n_b - 1] = (uint64_t)rmax << 32 | i;
		}
		if (rmax > gmax) {
			gmax = rmax, te = i;
			memcpy(Hm, H1, sizeof(int) * qp);
			if ((u8 && gmax + shift >= 255) || gmax >= endsc) break;
		}
		tmp = H0, H0 = H1, H1 = tmp;
	}
	r.score = u8 ? (gmax + shift < 255 ? gmax : 255) : gmax;
	r.te = te;
	if (!u8 || r.score != 255) {
		int mx = -1;
		for (k = 0; k < qp; ++k) {  /* vector memory order: lane k % p, slot k / p */
			const int q = k / p + k % p * slen;
			if (Hm[q] > mx) mx = Hm[q], r.qe = q;
			else if (Hm[q] == mx && q < r.qe) r.qe = q;
		}
		if (n_b) {
			const int d = (r.score + top - 1) / top, low = te - d, high = te + d;
			for (k = 0; k < n_b; ++k) {
				const int e = (int32_t)b[k];
				if ((e < low || e > high) && (int)(b[k] >> 32) > r.score2) r.score2 = b[k] >> 32, r.te2 = e;
			}
		}
	}
	free(b); free(H0); free(H1); free(E); free(Hm); free(prof);
	return r;
}

/* ksw_align2 (software/ksw.c:342-364) */
static swr_t sw_align(int qlen, const uint8_t *query, int tlen, const uint8_t *target, const orc_aln_opt_t *o, int xtra);

/* ksw_align2 of one problem, for the tests: out = kswr_t {score, te, qe, score2, te2, tb, qb} */
void orc_ksw_align2(int qlen, const uint8_t *query, int tlen, const uint8_t *target, const int8_t *mat, int o_del,
		int e_del, int o_ins, int e_ins, int xtra, int32_t out[7])
{
	orc_aln_opt_t o;
	swr_t r;
	memset(&o, 0, sizeof(o));
	memcpy(o.mat, mat, 25);
	o.o_del = o_del, o.e_del = e_del, o.o_ins = o_ins, o.e_ins = e_ins;
	r = sw_align(qlen, query, tlen, target, &o, xtra);
	out[0] = r.score, out[1] = r.te, out[2] = r.qe, out[3] = r.score2, out[4] = r.te2, out[5] = r.tb, out[6] = r.qb;
}

static swr_t sw_align(int qlen, const uint8_t *query, int tlen, const uint8_t *target, const orc_aln_opt_t *o, int xtra)
{
	const int p = (xtra & XBYTE) ? 16 : 8;
	swr_t r = sw_pass(p, qlen, query, tlen, target, o->mat, o->o_del, o->e_del, o->o_ins, o->e_ins, xtra), rr;
	uint8_t *rq, *rt;
	int i;
	if ((xtra & XSTART) == 0 || ((xtra & XSUBO) && r.score < (xtra & 0xffff)) || r.qe < 0) return r;
	rq = malloc(r.qe + 1);
	rt = malloc(tlen > 0 ? tlen : 1);
	for (i = 0; i <= r.qe; ++i) rq[i] = query[r.qe - i];
	for (i = 0; i < tlen; ++i) rt[i] = i <= r.te ? target[r.te - i] : target[i];
	rr = sw_pass(p, r.qe + 1, rq, tlen, rt, o->mat, o->o_del, o->e_del, o->o_ins, o->e_ins, XSTOP | r.score);
	free(rq); free(rt);
	if (r.score == rr.score) r.tb = r.te - rr.te, r.qb = r.qe - rr.qe;
	return r;
}

static inline int pac_get(const uint8_t *pac, int64_t l) { return pac[l >> 2] >> ((~l & 3) << 1) & 3; }

/* bns_get_seq (software/bntseq.c:355-376): [beg, end) of the forward-reverse
 * text; nothing when it bridges the strands */
static uint8_t *get_seq(int64_t l_pac, const uint8_t *pac, int64_t beg, int64_t end, int64_t *len)
{
	uint8_t *seq;
	int64_t k, l = 0;
	if (end < beg) { int64_t t = beg; beg = end; end = t; }
	if (end > l_pac << 1) end = l_pac << 1;
	if (beg < 0) beg = 0;
	if (!(beg >= l_pac || end <= l_pac)) { *len = 0; return malloc(1); }
	*len = end - beg;
	seq = malloc(end - beg + 1);
	if (beg >= l_pac) {
		const int64_t beg_f = (l_pac << 1) - 1 - end, end_f = (l_pac << 1) - 1 - beg;
		for (k = end_f; k > beg_f; --k) seq[l++] = 3 - pac_get(pac, k);
	} else
		for (k = beg; k < end; ++k) seq[l++] = pac_get(pac, k);
	return seq;
}

static int max_gap(const orc_aln_opt_t *o, int qlen)  /* cal_max_gap */
{
	const int l_del = (int)((double)(qlen * o->a - o->o_del) / o->e_del + 1.);
	const int l_ins = (int)((double)(qlen * o->a - o->o_ins) / o->e_ins + 1.);
	int l = l_del > l_ins ? l_del : l_ins;
	l = l > 1 ? l : 1;
	return l < o->w << 1 ? l : o->w << 1;
}

typedef struct { int n, m; orc_alnreg_t *a; } regv_t;

static orc_alnreg_t *reg_push(regv_t *v)
{
	if (v->n == v->m) {
		v->m = v->m ? v->m << 1 : 8;
		v->a = realloc(v->a, sizeof(orc_alnreg_t) * v->m);
	}
	memset(&v->a[v->n], 0, sizeof(orc_alnreg_t));
	return &v->a[v->n++];
}

/* mem_chain2aln_short (software/bwamem.c:805-852): 0 when it added a region */
static int chain2aln_short(const orc_aln_opt_t *o, int64_t l_pac, const uint8_t *pac, int l_query,
		const uint8_t *query, const orc_seed_t *sd, int n, regv_t *av)
{
	int i, qb = l_query, qe = 0, seedcov = 0, xtra;
	int64_t rb = l_pac << 1, re = 0, rlen;
	uint8_t *rseq;
	swr_t x;
	orc_alnreg_t *a;
	if (n == 0) return -1;
	for (i = 0; i < n; ++i) {
		const orc_seed_t *s = &sd[i];
		qb = qb < s->qbeg ? qb : s->qbeg;
		qe = qe > s->qbeg + s->len ? qe : s->qbeg + s->len;
		rb = rb < s->rbeg ? rb : s->rbeg;
		re = re > s->rbeg + s->len ? re : s->rbeg + s->len;
		seedcov += s->len;
	}
	qb -= SHORT_EXT; qe += SHORT_EXT;
	if (qb <= 10 || qe >= l_query - 10) return 1;
	rb -= SHORT_EXT; re += SHORT_EXT;
	rb = rb > 0 ? rb : 0;
	re = re < l_pac << 1 ? re : l_pac << 1;
	if (rb < l_pac && l_pac < re) {
		if (sd[0].rbeg < l_pac) re = l_pac;
		else rb = l_pac;
	}
	if ((re - rb) - (qe - qb) > SHORT_EXT || (qe - qb) - (re - rb) > SHORT_EXT) return 1;
	if (qe - qb >= o->w * 4 || re - rb >= o->w * 4) return 1;
	if (qe - qb >= SHORT_LEN || re - rb >= SHORT_LEN) return 1;
	rseq = get_seq(l_pac, pac, rb, re, &rlen);
	xtra = XSUBO | XSTART | ((qe - qb) * o->a < 250 ? XBYTE : 0) | (o->min_seed_len * o->a);
	x = sw_align(qe - qb, query + qb, (int)(re - rb), rseq, o, xtra);
	free(rseq);
	if (x.tb < SHORT_EXT >> 1 || x.te > re - rb - (SHORT_EXT >> 1)) return 1;
	a = reg_push(av);
	a->rb = rb + x.tb; a->re = rb + x.te + 1;
	a->qb = qb + x.qb; a->qe = qb + x.qe + 1;
	a->score = x.score;
	a->csub = x.score2;
	a->seedcov = seedcov;
	return 0;
}

static int cmp_u64(const void *a, const void *b)
{
	const uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
	return x < y ? -1 : x > y;
}

/* shape statistics of the extensions chain2aln makes, per thread (test
 * infrastructure: how the DP work of the alignment stage is distributed):
 * [b][0] calls, [b][1] in-band cells, by qlen bucket b = 0: <= 16, 1: <= 32,
 * 2: <= 64, 3: <= 128, 4: <= 256, 5: longer */
__thread uint64_t orc_ext_shape[6][2];

void orc_ext_shapes(uint64_t out[12], int reset)
{
	memcpy(out, orc_ext_shape, sizeof(orc_ext_shape));
	if (reset) memset(orc_ext_shape, 0, sizeof(orc_ext_shape));
}

/* which seeds chain2aln extends, per thread (test infrastructure: how much
 * work a region computed ahead per chain would save): [0] seeds extended that
 * are their chain's first in the order (the longest), [1] other seeds
 * extended, [2] first seeds not extended (contained in an earlier chain's
 * region), [3] seeds of the chains chain2aln runs on */
__thread uint64_t orc_seed_use[4];

void orc_seed_uses(uint64_t out[4], int reset)
{
	memcpy(out, orc_seed_use, sizeof(orc_seed_use));
	if (reset) memset(orc_seed_use, 0, sizeof(orc_seed_use));
}

static int extend(const orc_aln_opt_t *o, int qlen, const uint8_t *q, int tlen, const uint8_t *t, int w,
		int end_bonus, int h0, orc_ksw_result_t *res)
{
	int b = qlen <= 16 ? 0 : qlen <= 32 ? 1 : qlen <= 64 ? 2 : qlen <= 128 ? 3 : qlen <= 256 ? 4 : 5, r;
	uint64_t c0 = orc_cells_ext;
	orc_ksw_task_t T;
	orc_ksw_opt_t ko;
	memset(&T, 0, sizeof(T));
	T.qlen = qlen, T.tlen = tlen, T.w = w, T.end_bonus = end_bonus, T.zdrop = o->zdrop, T.h0 = h0;
	memcpy(ko.mat, o->mat, 25);
	ko.o_del = o->o_del, ko.e_del = o->e_del, ko.o_ins = o->o_ins, ko.e_ins = o->e_ins;
	r = orc_ksw_extend(&T, q, t, &ko, res);
	orc_ext_shape[b][0] += 1, orc_ext_shape[b][1] += orc_cells_ext - c0;
	return r;
}

/* mem_chain2aln (software/bwamem.c:1040-1188) */
static void chain2aln(const orc_aln_opt_t *o, int64_t l_pac, const uint8_t *pac, int l_query, const uint8_t *query,
		const orc_seed_t *sd, int n, regv_t *av)
{
	int i, k, aw[2];
	int64_t rlen, rmax[2];
	uint8_t *rseq, *qs, *rs;
	uint64_t *srt;
	if (n == 0) return;
	rmax[0] = l_pac << 1; rmax[1] = 0;
	for (i = 0; i < n; ++i) {
		const orc_seed_t *t = &sd[i];
		const int64_t b = t->rbeg - (t->qbeg + max_gap(o, t->qbeg));
		const int64_t e = t->rbeg + t->len + ((l_query - t->qbeg - t->len) + max_gap(o, l_query - t->qbeg - t->len));
		rmax[0] = rmax[0] < b ? rmax[0] : b;
		rmax[1] = rmax[1] > e ? rmax[1] : e;
	}
	rmax[0] = rmax[0] > 0 ? rmax[0] : 0;
	rmax[1] = rmax[1] < l_pac << 1 ? rmax[1] : l_pac << 1;
	if (rmax[0] < l_pac && l_pac < rmax[1]) {
		if (sd[0].rbeg < l_pac) rmax[1] = l_pac;
		else rmax[0] = l_pac;
	}
	rseq = get_seq(l_pac, pac, rmax[0], rmax[1], &rlen);
	srt = malloc(n * 8);
	for (i = 0; i < n; ++i) srt[i] = (uint64_t)sd[i].len << 32 | i;
	qsort(srt, n, 8, cmp_u64);  /* keys are distinct: any sort gives ks_introsort_64's order */
	qs = malloc(l_query + 1);
	orc_seed_use[3] += n;
	rs = malloc(rlen + 1);
	for (k = n - 1; k >= 0; --k) {
		const orc_seed_t *s = &sd[(uint32_t)srt[k]];
		orc_alnreg_t *a;
		orc_ksw_result_t x;
		for (i = 0; i < av->n; ++i) {  /* contained in a region made before? */
			const orc_alnreg_t *p = &av->a[i];
			int64_t rd;
			int qd, w, g;
			if (s->rbeg < p->rb || s->rbeg + s->len > p->re || s->qbeg < p->qb || s->qbeg + s->len > p->qe) continue;
			qd = s->qbeg - p->qb; rd = s->rbeg - p->rb;
			g = max_gap(o, (int)(qd < rd ? qd : rd));
			w = g < o->w ? g : o->w;
			if (qd - rd < w && rd - qd < w) break;
			qd = p->qe - (s->qbeg + s->len); rd = p->re - (s->rbeg + s->len);
			g = max_gap(o, (int)(qd < rd ? qd : rd));
			w = g < o->w ? g : o->w;
			if (qd - rd < w && rd - qd < w) break;
		}
		if (i < av->n) {  /* then only extend when a long overlapping seed disagrees */
			for (i = k + 1; i < n; ++i) {
				const orc_seed_t *t;
				if (srt[i] == 0) continue;
				t = &sd[(uint32_t)srt[i]];
				if (t->len < s->len * .95) continue;
				if (s->qbeg <= t->qbeg && s->qbeg + s->len - t->qbeg >= s->len >> 2 &&
						t->qbeg - s->qbeg != t->rbeg - s->rbeg) break;
				if (t->qbeg <= s->qbeg && t->qbeg + t->len - s->qbeg >= s->len >> 2 &&
						s->qbeg - t->qbeg != s->rbeg - t->rbeg) break;
			}
			if (i == n) {
				srt[k] = 0;
				orc_seed_use[2] += k == n - 1;
				continue;
			}
		}
		orc_seed_use[k == n - 1 ? 0 : 1] += 1;
		a = reg_push(av);
		a->w = aw[0] = aw[1] = o->w;
		a->score = a->truesc = -1;
		if (s->qbeg) {  /* left: reversed query and reference */
			const int64_t tmp = s->rbeg - rmax[0];
			for (i = 0; i < s->qbeg; ++i) qs[i] = query[s->qbeg - 1 - i];
			for (i = 0; i < tmp; ++i) rs[i] = rseq[tmp - 1 - i];
			for (i = 0; i < BAND_TRY; ++i) {
				const int prev = a->score;
				aw[0] = o->w << i;
				extend(o, s->qbeg, qs, (int)tmp, rs, aw[0], o->pen_clip5, s->len * o->a, &x);
				a->score = x.score;
				if (a->score == prev || x.max_off < (aw[0] >> 1) + (aw[0] >> 2)) break;
			}
			if (x.gscore <= 0 || x.gscore <= a->score - o->pen_clip5) {
				a->qb = s->qbeg - x.qle, a->rb = s->rbeg - x.tle;
				a->truesc = a->score;
			} else {
				a->qb = 0, a->rb = s->rbeg - x.gtle;
				a->truesc = x.gscore;
			}
		} else a->score = a->truesc = s->len * o->a, a->qb = 0, a->rb = s->rbeg;
		if (s->qbeg + s->len != l_query) {  /* right */
			const int qe = s->qbeg + s->len, sc0 = a->score;
			const int64_t re = s->rbeg + s->len - rmax[0];
			for (i = 0; i < BAND_TRY; ++i) {
				const int prev = a->score;
				aw[1] = o->w << i;
				extend(o, l_query - qe, query + qe, (int)(rmax[1] - rmax[0] - re), rseq + re, aw[1], o->pen_clip3, sc0,
						&x);
				a->score = x.score;
				if (a->score == prev || x.max_off < (aw[1] >> 1) + (aw[1] >> 2)) break;
			}
			if (x.gscore <= 0 || x.gscore <= a->score - o->pen_clip3) {
				a->qe = qe + x.qle, a->re = rmax[0] + re + x.tle;
				a->truesc += a->score - sc0;
			} else {
				a->qe = l_query, a->re = rmax[0] + re + x.gtle;
				a->truesc += x.gscore - sc0;
			}
		} else a->qe = l_query, a->re = s->rbeg + s->len;
		for (i = 0, a->seedcov = 0; i < n; ++i) {
			const orc_seed_t *t = &sd[i];
			if (t->qbeg >= a->qb && t->qbeg + t->len <= a->qe && t->rbeg >= a->rb && t->rbeg + t->len <= a->re)
				a->seedcov += t->len;
		}
		a->w = aw[0] > aw[1] ? aw[0] : aw[1];
	}
	free(srt); free(rseq); free(qs); free(rs);
}

int orc_aln_read(const orc_aln_opt_t *o, int64_t l_pac, const uint8_t *pac, int l_query, const uint8_t *query,
		int n_chains, const orc_aln_chain_t *chains, const orc_seed_t *seeds, orc_alnreg_t **out)
{
	regv_t av = { 0, 0, 0 };
	int c;
	for (c = 0; c < n_chains; ++c) {
		const orc_seed_t *sd = seeds + chains[c].seed_off;
		if (chain2aln_short(o, l_pac, pac, l_query, query, sd, chains[c].n, &av) > 0)
			chain2aln(o, l_pac, pac, l_query, query, sd, chains[c].n, &av);
	}
	*out = av.a;
	return av.n;
}

int orc_aln_batch(const orc_aln_opt_t *o, int64_t l_pac, const uint8_t *pac, int64_t n_reads, const uint8_t *codes,
		const uint64_t *offs, const orc_aln_chain_t *chains, const uint64_t *chain_off, const orc_seed_t *seeds,
		orc_alnreg_t **regs, uint64_t *reg_off)
{
	int64_t r;
	uint64_t n = 0, m = 0;
	orc_alnreg_t *all = malloc(sizeof(orc_alnreg_t));
	reg_off[0] = 0;
	for (r = 0; r < n_reads; ++r) {
		orc_alnreg_t *a = 0;
		const int k = orc_aln_read(o, l_pac, pac, (int)(offs[r + 1] - offs[r]), codes + offs[r],
				(int)(chain_off[r + 1] - chain_off[r]), chains + chain_off[r], seeds, &a);
		if (n + k > m) {
			m = (n + k) * 2 + 16;
			all = realloc(all, sizeof(orc_alnreg_t) * m);
			if (!all) { free(a); return -1; }
		}
		if (k) memcpy(all + n, a, sizeof(orc_alnreg_t) * k);
		free(a);
		n += k;
		reg_off[r + 1] = n;
	}
	*regs = all;
	return 0;
}
