/*
 * ksw_oracle.c — TEST INFRASTRUCTURE ONLY.  Plain-C restatement of the
 * banded Smith-Waterman extension BWA-MEM runs from each seed, §8(f) row 4:
 *
 *   ksw_extend2   software/ksw.c:379-476  (called by mem_chain2aln,
 *                                          software/bwamem.c:1136, 1164)
 *
 * Row i of the target against the query columns inside a band [lo, hi) that
 * starts as [0, qlen), is clipped to [i - w, i + w + 1) and then re-fitted
 * around the row's best cell; affine gaps (E vertical, F horizontal), local
 * scores floored at 0, an end bonus only through the to-end score, z-drop.
 * The column array keeps, for every column, the H of the previous row one
 * column to the left and the E of this row — the reference's layout, which
 * the band update reads.  Pinned against the compiled reference's own
 * ksw_extend2 (oracle/_ref/ref_harness ksw, tests/golden/ksw_*.gz).  Only
 * tests/ and bench.py's CPU leg use it; the product never links it.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "smem_oracle.h"

typedef struct { int32_t hprev, e; } col_t;

/* DP cells computed (in-band cells of ksw_extend2, the whole qlen x tlen
 * matrix of every ksw_align2 pass), per thread: the algorithmic work the GPU's
 * DP kernels are measured against (bench.py: cells/s) */
__thread uint64_t orc_cells_ext, orc_cells_sw;

void orc_cells(uint64_t out[2], int reset)
{
	out[0] = orc_cells_ext, out[1] = orc_cells_sw;
	if (reset) orc_cells_ext = orc_cells_sw = 0;
}

static int imax(int a, int b) { return a > b ? a : b; }

int orc_ksw_extend(const orc_ksw_task_t *T, const uint8_t *query, const uint8_t *target, const orc_ksw_opt_t *o,
                   orc_ksw_result_t *res)
{
	const int qlen = T->qlen, tlen = T->tlen;
	const int oe_del = o->o_del + o->e_del, oe_ins = o->o_ins + o->e_ins;
	int h0 = T->h0 > 0 ? T->h0 : 0;
	int w = T->w, top = 0, lo, hi, row;
	int best = h0, best_i = -1, best_j = -1, end_i = -1, end_score = -1, off_max = 0;
	col_t *c;
	int8_t *prof;
	int j, k;
	if (qlen < 1) return -1;
	c = (col_t*)calloc((size_t)qlen + 1, sizeof(col_t));
	prof = (int8_t*)malloc((size_t)qlen * 5);
	if (!c || !prof) { free(c); free(prof); return -1; }
	/* score of target symbol k against every query column */
	for (k = 0; k < 5; ++k)
		for (j = 0; j < qlen; ++j) prof[k * qlen + j] = o->mat[k * 5 + query[j]];
	/* row -1: a gap opened from h0 along the query, while it stays above e_ins */
	c[0].hprev = h0;
	c[1].hprev = h0 > oe_ins ? h0 - oe_ins : 0;
	for (j = 2; j <= qlen && c[j - 1].hprev > o->e_ins; ++j) c[j].hprev = c[j - 1].hprev - o->e_ins;
	/* the band can never be wider than the longest gap a full match pays for */
	for (k = 0; k < 25; ++k) top = imax(top, o->mat[k]);
	{
		int lim = (int)((double)(qlen * top + T->end_bonus - o->o_ins) / o->e_ins + 1.);
		lim = imax(lim, 1);
		if (w > lim) w = lim;
		lim = (int)((double)(qlen * top + T->end_bonus - o->o_del) / o->e_del + 1.);
		lim = imax(lim, 1);
		if (w > lim) w = lim;
	}
	lo = 0, hi = qlen;
	for (row = 0; row < tlen; ++row) {
		const int8_t *s = prof + (size_t)target[row] * qlen;
		int hleft = h0 - (o->o_del + o->e_del * (row + 1));  /* column -1 of this row */
		int f = 0, rmax = 0, rcol = -1, stop;
		if (hleft < 0) hleft = 0;
		if (lo < row - w) lo = row - w;
		if (hi > row + w + 1) hi = row + w + 1;
		if (hi > qlen) hi = qlen;
		if (hi > lo) orc_cells_ext += (uint64_t)(hi - lo);
		for (j = lo; j < hi; ++j) {
			int h = c[j].hprev + s[j], e = c[j].e, t;
			c[j].hprev = hleft;                       /* H(row, j-1) for the next row */
			if (h < e) h = e;
			if (h < f) h = f;
			hleft = h;
			if (h >= rmax) rmax = h, rcol = j;        /* the last column of the row maximum */
			t = imax(h - oe_del, 0);
			c[j].e = imax(e - o->e_del, t);            /* E of the next row */
			t = imax(h - oe_ins, 0);
			f = imax(f - o->e_ins, t);                 /* F of the next column */
		}
		c[hi].hprev = hleft;
		c[hi].e = 0;
		stop = lo < hi ? hi : lo;                     /* where the column scan stopped */
		if (stop == qlen) {                           /* reached the query end */
			if (hleft >= end_score) end_i = row;
			end_score = imax(end_score, hleft);
		}
		if (rmax == 0) break;
		if (rmax > best) {
			best = rmax, best_i = row, best_j = rcol;
			off_max = imax(off_max, abs(rcol - row));
		} else if (T->zdrop > 0) {
			const int di = row - best_i, dj = rcol - best_j;
			const int drop = di > dj ? best - rmax - (di - dj) * o->e_del : best - rmax - (dj - di) * o->e_ins;
			if (drop > T->zdrop) break;
		}
		/* refit the band: back to the nearest zero at or before the best
		 * column, forward to the first zero two columns past it */
		for (j = rcol; j >= lo && c[j].hprev; --j) {}
		lo = j + 1;
		for (j = rcol + 2; j <= hi && c[j].hprev; ++j) {}
		hi = j;
	}
	free(c);
	free(prof);
	res->score = best;
	res->qle = best_j + 1;
	res->tle = best_i + 1;
	res->gtle = end_i + 1;
	res->gscore = end_score;
	res->max_off = off_max;
	return 0;
}

int orc_ksw_batch(int64_t n, const orc_ksw_task_t *tasks, const uint8_t *q, const uint8_t *t, const orc_ksw_opt_t *o,
                  orc_ksw_result_t *out)
{
	int64_t i;
	for (i = 0; i < n; ++i)
		if (orc_ksw_extend(&tasks[i], q + tasks[i].q_off, t + tasks[i].t_off, o, &out[i]) != 0) return -1;
	return 0;
}
