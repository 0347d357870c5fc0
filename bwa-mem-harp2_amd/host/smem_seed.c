/*
 * smem_seed.c — C host driver of the SMEM engine, shaped like the reference
 * path it replaces:
 *
 *   mem_process_seqs (software/bwamem.c:1614-1640)
 *     kt_for_batch(n_threads, worker1_batched, ..., batch_size)   software/kthread_batch.c:46
 *       mem_chain_batched(...)                                      software/bwamem.c:542-591
 *         mem_insert_seed_batched -> smem_next2_batched -> FPGA      software/bwamem.c:357-451
 *
 * Here each kt_for_batch_gpu worker hands its whole batch to
 * smem_gpu_collect() (include/smem_gpu.h) and then walks the returned
 * lists in order — exactly where mem_insert_seed's chaining body
 * (software/bwamem.c:462-499) would consume them.  This CLI writes the
 * lists as an SMGO stream (include/smem_formats.h) so they can be compared
 * byte for byte with the reference harness.
 *
 * usage: smem_seed [-t threads] [-b batch] [-g n_gpus] [-e] [-k 19] [-r 1.5] [-s 10]
 *                  <in.bwt> <reads.smrd> <out.smgo>
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <sys/time.h>
#include "smem_gpu.h"
#include "smem_formats.h"
#include "kt_batch.h"

typedef struct {
	uint8_t *rec;          /* SMGO record of the read: n_calls, then lists */
	size_t n;
} read_out_t;

typedef struct {
	smem_gpu_t **gpus;
	int n_gpus;
	const smrd_reads_t *reads;
	const smem_opt_t *opt;
	read_out_t *out;
	volatile int err;
} shared_t;

static void worker(void *data, int start, int batch, int tid)
{
	shared_t *s = (shared_t*)data;
	smem_gpu_t *g = s->gpus[tid % s->n_gpus];
	const uint8_t **seq;
	int *len;
	smem_batch_t *b = 0;
	int i, rc;
	if (batch <= 0) return;
	seq = (const uint8_t**)malloc(sizeof(*seq) * batch);
	len = (int*)malloc(sizeof(int) * batch);
	for (i = 0; i < batch; ++i) {
		seq[i] = s->reads->codes + s->reads->off[start + i];
		len[i] = s->reads->len[start + i];
	}
	rc = smem_gpu_collect(g, batch, seq, len, s->opt, &b);
	if (rc) {
		fprintf(stderr, "[smem_seed] smem_gpu_collect failed: %s\n", smem_strerror(rc));
		s->err = rc;
		free(seq); free(len);
		return;
	}
	for (i = 0; i < batch; ++i) {
		const smem_intv_t *iv;
		const uint32_t *cn;
		int ni, nc, c, pos = 0;
		size_t bytes;
		uint8_t *p;
		smem_batch_read(b, i, &iv, &ni, &cn, &nc);
		bytes = 4 + 4 * (size_t)nc + sizeof(smem_intv_t) * (size_t)ni;
		p = (uint8_t*)malloc(bytes);
		s->out[start + i].rec = p;
		s->out[start + i].n = bytes;
		memcpy(p, &nc, 4); p += 4;
		for (c = 0; c < nc; ++c) {      /* one smem_next2 list at a time, in order */
			memcpy(p, &cn[c], 4); p += 4;
			memcpy(p, iv + pos, sizeof(smem_intv_t) * cn[c]);
			p += sizeof(smem_intv_t) * cn[c];
			pos += (int)cn[c];
		}
	}
	free(seq); free(len);
}

int main(int argc, char **argv)
{
	int c, n_threads = 1, batch = 4096, n_gpus = 1, i, rc;
	smem_opt_t opt;
	smem_index_t idx;
	smrd_reads_t reads;
	shared_t sh;
	FILE *fp;
	struct timeval t0, t1;
	smem_opt_default(&opt);
	while ((c = getopt(argc, argv, "t:b:g:ek:r:s:")) >= 0) {
		switch (c) {
		case 't': n_threads = atoi(optarg); break;
		case 'b': batch = atoi(optarg); break;
		case 'g': n_gpus = atoi(optarg); break;
		case 'e': opt.start_width = 2; break;   /* MEM_F_NO_EXACT */
		case 'k': opt.min_seed_len = atoi(optarg); break;
		case 'r': opt.split_factor = (float)atof(optarg); break;
		case 's': opt.split_width = atoi(optarg); break;
		default: return 1;
		}
	}
	if (optind + 3 > argc) {
		fprintf(stderr, "usage: smem_seed [-t threads] [-b batch] [-g n_gpus] [-e] [-k 19] [-r 1.5] [-s 10] <in.bwt> <reads.smrd> <out.smgo>\n");
		return 1;
	}
	if ((rc = smem_bwt_read(argv[optind], &idx)) != 0) { fprintf(stderr, "cannot read %s\n", argv[optind]); return 1; }
	if (smrd_load(argv[optind + 1], &reads) != 0) { fprintf(stderr, "cannot read %s\n", argv[optind + 1]); return 1; }
	if (n_gpus > smem_gpu_device_count()) n_gpus = smem_gpu_device_count();
	if (n_gpus < 1) { fprintf(stderr, "[smem_seed] no HIP device\n"); return 2; }
	memset(&sh, 0, sizeof(sh));
	sh.gpus = (smem_gpu_t**)calloc(n_gpus, sizeof(smem_gpu_t*));
	sh.n_gpus = n_gpus;
	for (i = 0; i < n_gpus; ++i) {
		rc = smem_gpu_init(&sh.gpus[i], i, idx.bwt, idx.bwt_size, idx.primary, idx.L2);
		if (rc) { fprintf(stderr, "[smem_seed] smem_gpu_init(%d): %s\n", i, smem_strerror(rc)); return 2; }
	}
	smem_index_free(&idx);
	sh.reads = &reads;
	sh.opt = &opt;
	sh.out = (read_out_t*)calloc(reads.n_reads ? reads.n_reads : 1, sizeof(read_out_t));
	gettimeofday(&t0, 0);
	kt_for_batch_gpu(n_threads, worker, &sh, (int)reads.n_reads, batch);
	gettimeofday(&t1, 0);
	if (sh.err) return 3;
	fprintf(stderr, "[smem_seed] %llu reads in %.3f s (%d threads, %d GPUs, batch %d)\n",
			(unsigned long long)reads.n_reads, (t1.tv_sec - t0.tv_sec) + 1e-6 * (t1.tv_usec - t0.tv_usec),
			n_threads, n_gpus, batch);
	fp = fopen(argv[optind + 2], "wb");
	if (!fp) return 1;
	smgo_write_header(fp, reads.n_reads);
	for (i = 0; i < (int)reads.n_reads; ++i) {
		fwrite(sh.out[i].rec, 1, sh.out[i].n, fp);
		free(sh.out[i].rec);
	}
	fclose(fp);
	for (i = 0; i < n_gpus; ++i) smem_gpu_shutdown(sh.gpus[i]);
	free(sh.gpus); free(sh.out); smrd_free(&reads);
	return 0;
}
