/*
 * oracle_cli.c — TEST INFRASTRUCTURE ONLY.  Command-line front end of the C
 * restatement (smem_oracle.c), mirroring oracle/_ref/ref_harness's `smem`
 * and `bench` commands so their outputs can be compared byte for byte.
 *
 *   smem_oracle smem  <in.bwt> <reads.smrd> <out.smgo> <k> <r> <s> <start_width> [threads]
 *   smem_oracle bench <in.bwt> <reads.smrd> <threads> <max_reads> <k> <r> <s> <start_width>
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "smem_oracle.h"
#include "smem_formats.h"

static void parse_opt(char **a, orc_opt_t *o)
{
	o->min_seed_len = atoi(a[0]);
	o->split_factor = (float)atof(a[1]);
	o->split_width = atoi(a[2]);
	o->start_width = atoi(a[3]);
}

int main(int argc, char **argv)
{
	orc_bwt_t *b;
	smrd_reads_t r;
	orc_opt_t o;
	orc_stats_t st;
	int64_t *offs;
	uint64_t i;
	if (argc < 2) { fprintf(stderr, "usage: smem_oracle smem|bench ...\n"); return 1; }
	if (strcmp(argv[1], "smem") == 0 && argc >= 9) {
		uint8_t *out; uint64_t out_len; FILE *fp;
		int threads = argc > 9 ? atoi(argv[9]) : 1;
		parse_opt(argv + 5, &o);
		if (!(b = orc_bwt_load(argv[2]))) return 1;
		if (smrd_load(argv[3], &r)) return 1;
		offs = (int64_t*)malloc(8 * (r.n_reads + 1));
		for (i = 0; i <= r.n_reads; ++i) offs[i] = (int64_t)r.off[i];
		orc_seed(b, (int64_t)r.n_reads, r.codes, offs, &o, threads, &out, &out_len, 0, 0, 0, &st);
		fp = fopen(argv[4], "wb");
		fwrite(out, 1, out_len, fp);
		fclose(fp);
		fprintf(stderr, "reads=%llu calls=%llu intv=%llu smem1=%llu ext=%llu ext_ref=%llu bkt=%llu bkt_ref=%llu\n",
				(unsigned long long)r.n_reads, (unsigned long long)st.n_calls, (unsigned long long)st.n_intv,
				(unsigned long long)st.n_smem1, (unsigned long long)st.n_ext, (unsigned long long)st.n_ext_ref,
				(unsigned long long)st.n_bkt, (unsigned long long)st.n_bkt_ref);
		orc_free(out); free(offs); smrd_free(&r); orc_bwt_free(b);
		return 0;
	}
	if (strcmp(argv[1], "bench") == 0 && argc >= 10) {
		int threads = atoi(argv[4]);
		uint64_t n = (uint64_t)atoll(argv[5]);
		double t;
		parse_opt(argv + 6, &o);
		if (!(b = orc_bwt_load(argv[2]))) return 1;
		if (smrd_load(argv[3], &r)) return 1;
		if (n == 0 || n > r.n_reads) n = r.n_reads;
		offs = (int64_t*)malloc(8 * (r.n_reads + 1));
		for (i = 0; i <= r.n_reads; ++i) offs[i] = (int64_t)r.off[i];
		t = orc_seed_timed(b, (int64_t)n, r.codes, offs, &o, threads, &st);
		printf("reads=%llu seconds=%.6f threads=%d reads_per_s=%.3f intervals=%llu\n",
				(unsigned long long)n, t, threads, n / t, (unsigned long long)st.n_intv);
		free(offs); smrd_free(&r); orc_bwt_free(b);
		return 0;
	}
	fprintf(stderr, "bad command\n");
	return 1;
}
