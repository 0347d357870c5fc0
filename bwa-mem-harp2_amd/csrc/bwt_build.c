/*
 * bwt_build.c — index provisioning for the SMEM engine.
 *
 * Builds the BWA FM-index (.bwt) of a reference genome from scratch:
 *   text   = forward pac + reverse complement   (software/bntseq.c:303-309)
 *   SA     = suffix array of text$ by SA-IS (own implementation, induced sorting)
 *   BWT    = text[SA[i]-1] with the $ row removed, primary = rank of suffix 0
 *            (same convention as software/is.c:208-223)
 *   layout = 128-symbol buckets: 4 x u64 cumulative Occ then 8 x u32 words of
 *            16 MSB-first 2-bit symbols, plus one trailing count block
 *            (software/bwtindex.c:128-150, software/bwt.h:72-73)
 *   file   = primary, L2[1..4], words   (software/bwt.c:841-850)
 * The result is byte-identical to `bwa index -a is` (tests/test_oracle.py::
 * test_index_builder_matches_reference / test_index_builder_small_vs_reference).
 *
 * Indices are 32-bit: text length (2 x genome) must stay below 2^32 - 2.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "smem_gpu.h"

#define EMPTY 0xFFFFFFFFu

/* ------------------------------------------------------------- SA-IS */

typedef struct {
	const void *T;
	int cs;           /* 1: uint8 text, 4: uint32 text */
} text_t;

static inline uint32_t chr(const text_t *t, uint64_t i)
{
	return t->cs == 1 ? ((const uint8_t*)t->T)[i] : ((const uint32_t*)t->T)[i];
}

#define TGET(tb, i) (((tb)[(i) >> 3] >> ((i) & 7)) & 1)    /* 1 = S-type */
#define TSET(tb, i, v) do { if (v) (tb)[(i) >> 3] |= (uint8_t)(1u << ((i) & 7)); \
                            else (tb)[(i) >> 3] &= (uint8_t)~(1u << ((i) & 7)); } while (0)
#define IS_LMS(tb, i) ((i) > 0 && TGET(tb, i) && !TGET(tb, (i) - 1))

static void bucket_bounds(const text_t *t, uint32_t n, uint32_t K, uint32_t *bkt, int ends)
{
	uint32_t i, sum = 0;
	memset(bkt, 0, sizeof(uint32_t) * K);
	for (i = 0; i < n; ++i) bkt[chr(t, i)]++;
	for (i = 0; i < K; ++i) {
		sum += bkt[i];
		bkt[i] = ends ? sum : sum - bkt[i];
	}
}

static void induce(const text_t *t, uint32_t *SA, uint32_t n, uint32_t K, const uint8_t *tb, uint32_t *bkt)
{
	uint32_t i, j;
	bucket_bounds(t, n, K, bkt, 0);              /* L-type: bucket heads, left to right */
	for (i = 0; i < n; ++i) {
		j = SA[i];
		if (j != EMPTY && j > 0 && !TGET(tb, j - 1)) SA[bkt[chr(t, j - 1)]++] = j - 1;
	}
	bucket_bounds(t, n, K, bkt, 1);              /* S-type: bucket tails, right to left */
	for (i = n; i-- > 0;) {
		j = SA[i];
		if (j != EMPTY && j > 0 && TGET(tb, j - 1)) SA[--bkt[chr(t, j - 1)]] = j - 1;
	}
}

/* SA of t[0..n-1]; t[n-1] must be a unique smallest symbol (0). */
static int sais_core(const text_t *t, uint32_t *SA, uint32_t n, uint32_t K)
{
	uint8_t *tb;
	uint32_t *bkt, i, j, n1 = 0, name, prev;
	if (n == 1) { SA[0] = 0; return 0; }
	tb = (uint8_t*)calloc((n >> 3) + 1, 1);
	bkt = (uint32_t*)malloc(sizeof(uint32_t) * K);
	if (!tb || !bkt) { free(tb); free(bkt); return -1; }
	/* classify */
	TSET(tb, n - 1, 1);
	for (i = n - 1; i-- > 0;) {
		uint32_t a = chr(t, i), b = chr(t, i + 1);
		TSET(tb, i, a < b || (a == b && TGET(tb, i + 1)));
	}
	/* stage 1: sort LMS substrings */
	bucket_bounds(t, n, K, bkt, 1);
	for (i = 0; i < n; ++i) SA[i] = EMPTY;
	for (i = 1; i < n; ++i)
		if (IS_LMS(tb, i)) SA[--bkt[chr(t, i)]] = i;
	induce(t, SA, n, K, tb, bkt);
	/* compact sorted LMS positions into SA[0..n1) */
	for (i = 0; i < n; ++i)
		if (IS_LMS(tb, SA[i])) SA[n1++] = SA[i];
	/* name LMS substrings; names go to SA[n1 + pos/2] */
	for (i = n1; i < n; ++i) SA[i] = EMPTY;
	name = 0; prev = EMPTY;
	for (i = 0; i < n1; ++i) {
		uint32_t pos = SA[i], d;
		int diff = 0;
		if (prev == EMPTY) diff = 1;
		else {
			for (d = 0;; ++d) {
				if (chr(t, pos + d) != chr(t, prev + d) || TGET(tb, pos + d) != TGET(tb, prev + d)) { diff = 1; break; }
				if (d > 0 && (IS_LMS(tb, pos + d) || IS_LMS(tb, prev + d))) break;
			}
		}
		if (diff) { ++name; prev = pos; }
		SA[n1 + (pos >> 1)] = name - 1;
	}
	/* gather the reduced string into the tail of SA */
	for (i = n, j = n; i-- > n1;)
		if (SA[i] != EMPTY) SA[--j] = SA[i];
	/* stage 2: sort the reduced problem */
	{
		uint32_t *s1 = SA + n - n1, *SA1 = SA;
		if (name < n1) {
			text_t t1 = { s1, 4 };
			uint32_t *tmp = (uint32_t*)malloc(sizeof(uint32_t) * n1);
			uint32_t *s1c = (uint32_t*)malloc(sizeof(uint32_t) * n1);
			if (!tmp || !s1c) { free(tmp); free(s1c); free(tb); free(bkt); return -1; }
			memcpy(s1c, s1, sizeof(uint32_t) * n1);
			t1.T = s1c;
			if (sais_core(&t1, tmp, n1, name)) { free(tmp); free(s1c); free(tb); free(bkt); return -1; }
			memcpy(SA1, tmp, sizeof(uint32_t) * n1);
			free(tmp); free(s1c);
		} else {
			for (i = 0; i < n1; ++i) SA1[s1[i]] = i;
		}
		/* map reduced ranks back to text positions (reuse s1 as the LMS list) */
		for (i = 1, j = 0; i < n; ++i)
			if (IS_LMS(tb, i)) s1[j++] = i;
		for (i = 0; i < n1; ++i) SA1[i] = s1[SA1[i]];
	}
	/* stage 3: place sorted LMS suffixes at bucket tails and induce */
	for (i = n1; i < n; ++i) SA[i] = EMPTY;
	bucket_bounds(t, n, K, bkt, 1);
	for (i = n1; i-- > 0;) {
		j = SA[i];
		SA[i] = EMPTY;
		SA[--bkt[chr(t, j)]] = j;
	}
	induce(t, SA, n, K, tb, bkt);
	free(tb); free(bkt);
	return 0;
}

/* --------------------------------------------------------- public API */

static int build_core(const uint8_t *fwd, uint64_t n_fwd, int sa_intv, smem_index_t *idx, smem_sa_t *sa_out)
{
	uint64_t n, i, j, k, n_occ, c[4];
	uint8_t *text;
	uint32_t *SA, *packed, *out;
	uint64_t primary = 0;
	if (!fwd || !idx || n_fwd == 0) return SMEM_E_ARG;
	n = 2 * n_fwd;
	if (n + 1 >= 0xFFFFFFFEull) return SMEM_E_ARG;
	memset(idx, 0, sizeof(*idx));
	/* text$ with symbols shifted to 1..4 and sentinel 0 */
	text = (uint8_t*)malloc(n + 1);
	SA = (uint32_t*)malloc(sizeof(uint32_t) * (n + 1));
	if (!text || !SA) { free(text); free(SA); return SMEM_E_NOMEM; }
	for (i = 0; i < n_fwd; ++i) {
		if (fwd[i] > 3) { free(text); free(SA); return SMEM_E_ARG; }
		text[i] = (uint8_t)(fwd[i] + 1);
		text[n - 1 - i] = (uint8_t)(3 - fwd[i] + 1);
	}
	text[n] = 0;
	{
		text_t t = { text, 1 };
		if (sais_core(&t, SA, (uint32_t)(n + 1), 5)) { free(text); free(SA); return SMEM_E_NOMEM; }
	}
	/* SA[0] is the sentinel suffix; rows 0..n of the BWT matrix */
	if (sa_out) {
		/* sampled SA as bwt_cal_sa leaves it (software/bwt.c:80-102):
		 * sa[r] = SA[r * intv], sa[0] = -1 */
		memset(sa_out, 0, sizeof(*sa_out));
		sa_out->sa_intv = (uint64_t)sa_intv;
		sa_out->seq_len = n;
		sa_out->n_sa = (n + (uint64_t)sa_intv) / (uint64_t)sa_intv;
		sa_out->sa = (uint64_t*)malloc(8 * (sa_out->n_sa + 1));
		if (!sa_out->sa) { free(text); free(SA); return SMEM_E_NOMEM; }
		for (i = 0; i < sa_out->n_sa; ++i) sa_out->sa[i] = SA[i * (uint64_t)sa_intv];
		sa_out->sa[0] = (uint64_t)-1;
		sa_out->sa[sa_out->n_sa] = 0;  /* pad: 16-B loads of the last sample stay in bounds */
		sa_out->owns = 1;
	}
	memset(idx->L2, 0, sizeof(idx->L2));
	for (i = 0; i < n; ++i) idx->L2[text[i]]++;      /* text[i] in 1..4 -> L2[1..4] counts */
	for (i = 2; i <= 4; ++i) idx->L2[i] += idx->L2[i - 1];
	packed = (uint32_t*)calloc((n + 15) >> 4, 4);
	if (!packed) { free(text); free(SA); return SMEM_E_NOMEM; }
	for (i = 0, j = 0; i <= n; ++i) {
		uint32_t s = SA[i], b;
		if (s == 0) { primary = i; continue; }
		b = (uint32_t)(text[s - 1] - 1);
		packed[j >> 4] |= b << ((15 - (j & 15)) << 1);
		++j;
	}
	free(SA); free(text);
	/* interleave Occ checkpoints (software/bwtindex.c:128-150) */
	n_occ = (n + 127) / 128 + 1;
	idx->bwt_size = ((n + 15) >> 4) + n_occ * 8;
	out = (uint32_t*)calloc(idx->bwt_size + 16, 4);   /* +16: a full bucket can always be loaded */
	if (!out) { free(packed); return SMEM_E_NOMEM; }
	c[0] = c[1] = c[2] = c[3] = 0;
	for (i = 0, k = 0; i < n; ++i) {
		if ((i & 127) == 0) { memcpy(out + k, c, 32); k += 8; }
		if ((i & 15) == 0) out[k++] = packed[i >> 4];
		c[(packed[i >> 4] >> ((15 - (i & 15)) << 1)) & 3]++;
	}
	memcpy(out + k, c, 32);
	k += 8;
	free(packed);
	if (k != idx->bwt_size) { free(out); return SMEM_E_INTERNAL; }
	idx->bwt = out;
	idx->primary = primary;
	idx->seq_len = n;
	idx->owns = 1;
	if (sa_out) {
		sa_out->primary = primary;
		memcpy(sa_out->L2, idx->L2, sizeof(idx->L2));
	}
	return SMEM_OK;
}

int smem_bwt_build(const uint8_t *fwd, uint64_t n_fwd, smem_index_t *idx)
{
	return build_core(fwd, n_fwd, 0, idx, 0);
}

int smem_bwt_build_sa(const uint8_t *fwd, uint64_t n_fwd, int sa_intv, smem_index_t *idx, smem_sa_t *sa)
{
	int rc;
	if (!sa || sa_intv <= 0 || (sa_intv & (sa_intv - 1))) return SMEM_E_ARG;  /* power of 2 (software/bwt.c:87) */
	rc = build_core(fwd, n_fwd, sa_intv, idx, sa);
	if (rc != SMEM_OK) smem_sa_free(sa);
	return rc;
}

/* .sa file (software/bwt.c:852-863 / 877-897): primary, L2[1..4], sa_intv,
 * seq_len, then sa[1 .. n_sa-1] */
int smem_sa_write(const char *fn, const smem_sa_t *sa)
{
	FILE *fp;
	if (!sa || !sa->sa || sa->n_sa == 0) return SMEM_E_ARG;
	fp = fopen(fn, "wb");
	if (!fp) return SMEM_E_IO;
	if (fwrite(&sa->primary, 8, 1, fp) != 1 || fwrite(sa->L2 + 1, 8, 4, fp) != 4 || fwrite(&sa->sa_intv, 8, 1, fp) != 1
			|| fwrite(&sa->seq_len, 8, 1, fp) != 1 || fwrite(sa->sa + 1, 8, sa->n_sa - 1, fp) != sa->n_sa - 1) {
		fclose(fp);
		return SMEM_E_IO;
	}
	return fclose(fp) == 0 ? SMEM_OK : SMEM_E_IO;
}

int smem_sa_read(const char *fn, smem_sa_t *sa)
{
	FILE *fp;
	if (!sa) return SMEM_E_ARG;
	memset(sa, 0, sizeof(*sa));
	fp = fopen(fn, "rb");
	if (!fp) return SMEM_E_IO;
	if (fread(&sa->primary, 8, 1, fp) != 1 || fread(sa->L2 + 1, 8, 4, fp) != 4 || fread(&sa->sa_intv, 8, 1, fp) != 1
			|| fread(&sa->seq_len, 8, 1, fp) != 1 || sa->sa_intv == 0) {
		fclose(fp);
		return SMEM_E_IO;
	}
	sa->n_sa = (sa->seq_len + sa->sa_intv) / sa->sa_intv;
	sa->sa = (uint64_t*)malloc(8 * (sa->n_sa + 1));
	if (!sa->sa) { fclose(fp); return SMEM_E_NOMEM; }
	sa->sa[0] = (uint64_t)-1;
	sa->sa[sa->n_sa] = 0;
	if (fread(sa->sa + 1, 8, sa->n_sa - 1, fp) != sa->n_sa - 1) { fclose(fp); free(sa->sa); sa->sa = 0; return SMEM_E_IO; }
	fclose(fp);
	sa->owns = 1;
	return SMEM_OK;
}

void smem_sa_free(smem_sa_t *sa)
{
	if (!sa) return;
	if (sa->owns) free(sa->sa);
	memset(sa, 0, sizeof(*sa));
}

int smem_bwt_write(const char *fn, const smem_index_t *idx)
{
	FILE *fp = fopen(fn, "wb");
	if (!fp) return SMEM_E_IO;
	if (fwrite(&idx->primary, 8, 1, fp) != 1 || fwrite(idx->L2 + 1, 8, 4, fp) != 4
			|| fwrite(idx->bwt, 4, idx->bwt_size, fp) != idx->bwt_size) { fclose(fp); return SMEM_E_IO; }
	return fclose(fp) == 0 ? SMEM_OK : SMEM_E_IO;
}

int smem_bwt_read(const char *fn, smem_index_t *idx)
{
	/* software/bwt.c:899-918 */
	FILE *fp = fopen(fn, "rb");
	long sz;
	memset(idx, 0, sizeof(*idx));
	if (!fp) return SMEM_E_IO;
	fseek(fp, 0, SEEK_END);
	sz = ftell(fp);
	fseek(fp, 0, SEEK_SET);
	if (sz < 40 + 64) { fclose(fp); return SMEM_E_IO; }
	idx->bwt_size = (uint64_t)(sz - 40) >> 2;
	idx->bwt = (uint32_t*)calloc(idx->bwt_size + 16, 4);
	if (!idx->bwt) { fclose(fp); return SMEM_E_NOMEM; }
	if (fread(&idx->primary, 8, 1, fp) != 1 || fread(idx->L2 + 1, 8, 4, fp) != 4
			|| fread(idx->bwt, 4, idx->bwt_size, fp) != idx->bwt_size) {
		fclose(fp); free(idx->bwt); idx->bwt = 0; return SMEM_E_IO;
	}
	fclose(fp);
	idx->L2[0] = 0;
	idx->seq_len = idx->L2[4];
	idx->owns = 1;
	return SMEM_OK;
}

void smem_index_free(smem_index_t *idx)
{
	if (!idx) return;
	if (idx->owns) free(idx->bwt);
	memset(idx, 0, sizeof(*idx));
}
