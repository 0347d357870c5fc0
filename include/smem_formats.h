/*
 * smem_formats.h — on-disk formats shared by the oracle harnesses, the C host
 * driver and the Python bindings.  Header-only, plain C99.
 *
 * Reads file ("SMRD0001"), little-endian:
 *   char     magic[8]      = "SMRD0001"
 *   uint64_t n_reads
 *   uint64_t n_bases        total bases over all reads
 *   int32_t  len[n_reads]
 *   uint8_t  codes[n_bases] nt4 codes as produced by nst_nt4_table
 *                           (software/bntseq.c:44): 0..3 = A,C,G,T, >3 = ambiguous
 *
 * SMEM stream file ("SMGO0001") — the exact sequence of lists returned by
 * smem_next2() (software/bwamem.c:244-305) while mem_insert_seed()
 * (software/bwamem.c:453-460) drives it:
 *   char     magic[8]      = "SMGO0001"
 *   uint64_t n_reads
 *   per read:  uint32_t n_calls
 *              per call: uint32_t n ; n x { uint64_t x0, x1, x2, info }
 *
 * SA positions file ("SMSA0001") — for every interval of an SMGO stream, in
 * order, that mem_insert_seed() turns into seeds (seed length >= k and
 * x2 <= max_occ, software/bwamem.c:467), bwt_sa(bwt, x0 + j) for j < x2
 * (software/bwamem.c:469-474, software/bwt.c:104-114):
 *   char     magic[8]      = "SMSA0001"
 *   uint64_t n_reads
 *   per read:  uint32_t n_occ ; n_occ x uint64_t position (forward-reverse coordinate)
 *
 * Chains file ("SMCH0001") — per read, the chains mem_chain() returns
 * (software/bwamem.c:593-614; kbtree in-order, software/kbtree.h:336-358),
 * optionally after mem_chain_flt() (software/bwamem.c:629-690):
 *   char     magic[8]      = "SMCH0001"
 *   uint64_t n_reads
 *   per read:  uint32_t n_chains
 *              per chain: int64_t pos ; uint32_t n ;
 *                         n x { int64_t rbeg ; int32_t qbeg ; int32_t len }  (mem_seed_t)
 *
 * SW extension tasks file ("SMKT0001") — ksw_extend2 calls
 * (software/ksw.c:379) with m = 5:
 *   char     magic[8]      = "SMKT0001"
 *   uint64_t n_tasks, q_bytes, t_bytes
 *   int8_t   mat[25] ; int8_t pad[3] ; int32_t o_del, e_del, o_ins, e_ins
 *   n_tasks x { uint64_t q_off, t_off ; int32_t qlen, tlen, w, end_bonus, zdrop, h0 }
 *   uint8_t  q[q_bytes] ; uint8_t t[t_bytes]        codes 0..4
 * SW extension results file ("SMKR0001"):
 *   char     magic[8]      = "SMKR0001"
 *   uint64_t n_tasks
 *   n_tasks x { int32_t score (the return value), qle, tle, gtle, gscore, max_off }
 */
#ifndef SMEM_FORMATS_H
#define SMEM_FORMATS_H

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define SMRD_MAGIC "SMRD0001"
#define SMGO_MAGIC "SMGO0001"
#define SMSA_MAGIC "SMSA0001"
#define SMCH_MAGIC "SMCH0001"
#define SMKT_MAGIC "SMKT0001"
#define SMKR_MAGIC "SMKR0001"

typedef struct {
	uint64_t n_reads, n_bases;
	int32_t *len;
	uint64_t *off;     /* n_reads + 1 prefix offsets (computed on load) */
	uint8_t *codes;
} smrd_reads_t;

static inline void smrd_free(smrd_reads_t *r)
{
	if (!r) return;
	free(r->len); free(r->off); free(r->codes);
	memset(r, 0, sizeof(*r));
}

/* returns 0 on success */
static inline int smrd_load(const char *fn, smrd_reads_t *r)
{
	char magic[8];
	uint64_t i;
	FILE *fp = fopen(fn, "rb");
	memset(r, 0, sizeof(*r));
	if (!fp) return -1;
	if (fread(magic, 1, 8, fp) != 8 || memcmp(magic, SMRD_MAGIC, 8) != 0) { fclose(fp); return -2; }
	if (fread(&r->n_reads, 8, 1, fp) != 1 || fread(&r->n_bases, 8, 1, fp) != 1) { fclose(fp); return -3; }
	r->len = (int32_t*)malloc(sizeof(int32_t) * (r->n_reads ? r->n_reads : 1));
	r->off = (uint64_t*)malloc(sizeof(uint64_t) * (r->n_reads + 1));
	r->codes = (uint8_t*)malloc(r->n_bases ? r->n_bases : 1);
	if (fread(r->len, 4, r->n_reads, fp) != r->n_reads) { fclose(fp); smrd_free(r); return -4; }
	if (fread(r->codes, 1, r->n_bases, fp) != r->n_bases) { fclose(fp); smrd_free(r); return -5; }
	fclose(fp);
	r->off[0] = 0;
	for (i = 0; i < r->n_reads; ++i) r->off[i + 1] = r->off[i] + (uint64_t)r->len[i];
	if (r->off[r->n_reads] != r->n_bases) { smrd_free(r); return -6; }
	return 0;
}

static inline int smgo_write_header(FILE *fp, uint64_t n_reads)
{
	if (fwrite(SMGO_MAGIC, 1, 8, fp) != 8) return -1;
	if (fwrite(&n_reads, 8, 1, fp) != 1) return -1;
	return 0;
}

static inline int smch_write_header(FILE *fp, uint64_t n_reads)
{
	if (fwrite(SMCH_MAGIC, 1, 8, fp) != 8) return -1;
	if (fwrite(&n_reads, 8, 1, fp) != 1) return -1;
	return 0;
}

static inline int smsa_write_header(FILE *fp, uint64_t n_reads)
{
	if (fwrite(SMSA_MAGIC, 1, 8, fp) != 8) return -1;
	if (fwrite(&n_reads, 8, 1, fp) != 1) return -1;
	return 0;
}

#endif
