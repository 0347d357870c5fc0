/*
 * smem_gpu.h — C ABI of the MI355X SMEM seeding engine (libsmemgpu.so).
 *
 * Drop-in boundary for BWA-MEM's seeding loop.  In the
 * reference, every kt_for_batch worker (software/kthread_batch.c:29-59)
 * runs mem_chain_batched -> mem_insert_seed_batched -> smem_next2_batched ->
 * bwt_smem1_batched (software/bwamem.c:542-591,357-451,110-241,
 * software/bwt.c:444-774), which packs <=128 reads per FPGA hand-shake
 * through the HARP manager thread (software/fastmap.c:320-429) and the AAL
 * glue (software/HelloALINLB.cpp:254-485).  This library replaces that whole
 * chain: one call seeds a batch of reads on the GPU and returns, per read,
 * exactly the sequence of interval lists smem_next2() (software/bwamem.c:244)
 * returns under mem_insert_seed() (software/bwamem.c:453-460) — bit-exact,
 * in order — so the caller's chaining body (software/bwamem.c:462-499) runs
 * unchanged.
 *
 * Plain C types only.  All entry points return 0 (SMEM_OK) or a negative
 * SMEM_E_* code; on a negative code the caller may fall back to its own CPU
 * path, mirroring the reference's reject -> CPU semantics
 * (software/bwt.c:686-717).  No entry point silently computes on the CPU.
 *
 * Failure contract: every entry point that runs work on a device returns
 * only once all of that work has finished or been abandoned (its streams
 * are synchronised on every return path), so no copy of the call lands in
 * host memory after the caller has resumed, whatever the code.  A HIP
 * runtime failure (SMEM_E_DEVICE) marks the device faulted: every later
 * call on it returns SMEM_E_DEVICE at once without enqueuing anything, so a
 * caller that takes its CPU path on SMEM_E_DEVICE computes exactly what the
 * reference computes.  Allocation failures are SMEM_E_NOMEM and leave the
 * device usable.  SMEM_GPU_FAIL=<stage>:<k>[:sticky] (stage: upload, seed,
 * sa, chain, aln, fetch, any) injects SMEM_E_DEVICE into every k-th call of
 * the stage after its work is enqueued, to test that contract.
 */
#ifndef SMEM_GPU_H
#define SMEM_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SMEM_OK           0
#define SMEM_E_ARG       -1   /* bad argument / shape */
#define SMEM_E_NOMEM     -2   /* host or device allocation failed */
#define SMEM_E_IO        -3   /* file I/O */
#define SMEM_E_DEVICE    -4   /* no usable HIP device or a HIP runtime error */
#define SMEM_E_INTERNAL  -5
#define SMEM_E_CAPACITY  -6   /* batch larger than the capacity it was created with */

/* bi-interval; identical layout to bwtintv_t (software/bwt.h:60-62):
 * x[0] forward SA start, x[1] reverse-complement SA start, x[2] size,
 * info = (query begin << 32) | query end (end exclusive). */
typedef struct { uint64_t x[3], info; } smem_intv_t;

/* FM-index in host memory.  The leading fields follow bwt_t
 * (software/bwt.h:46-51): primary, L2[5], seq_len, bwt_size, bwt. */
typedef struct {
	uint64_t primary;     /* S^-1(0): BWT row of the $ suffix */
	uint64_t L2[5];       /* cumulative base counts, L2[0] = 0 */
	uint64_t seq_len;     /* = L2[4] */
	uint64_t bwt_size;    /* number of uint32 words (Occ checkpoints interleaved) */
	uint32_t *bwt;        /* interleaved BWT + Occ, software/bwtindex.c:128-150 layout */
	int owns;             /* bwt was allocated by this library */
} smem_index_t;

/* Sampled suffix array for bwt_sa (software/bwt.c:80-114): sa[r] =
 * SA[r * sa_intv] for r < n_sa = (seq_len + sa_intv) / sa_intv, sa[0] =
 * (uint64_t)-1 as bwt_cal_sa leaves it.  primary / L2 / seq_len are those of
 * the .bwt it belongs to (the .sa header, software/bwt.c:852-863).  sa holds
 * n_sa + 1 words (one zero pad). */
typedef struct {
	uint64_t primary;
	uint64_t L2[5];
	uint64_t seq_len;
	uint64_t sa_intv;
	uint64_t n_sa;
	uint64_t *sa;
	int owns;
} smem_sa_t;

/* the mem_opt_t fields the seeding loop reads (software/bwamem.h:44-48,
 * software/bwamem.c:456-458) */
typedef struct {
	int min_seed_len;     /* -k, default 19 */
	float split_factor;   /* -r, default 1.5 */
	int split_width;      /* -s, default 10 */
	int start_width;      /* 1, or 2 when MEM_F_NO_EXACT (-e) */
} smem_opt_t;

typedef struct smem_gpu smem_gpu_t;       /* one device + its resident index */
typedef struct smem_batch smem_batch_t;   /* one worker's reads / results / scratch on one device */

/* defaults of mem_opt_init() (software/bwamem.c:58-65) */
void smem_opt_default(smem_opt_t *opt);

/* ---------------------------------------------------------------- index */
/* Build the .bwt of genome codes (0..3, forward strand only; the reverse
 * complement is appended as bns_fasta2bntseq(for_only=0) does).  Output is
 * byte-identical to `bwa index -a is` (software/bwtindex.c:187). */
int  smem_bwt_build(const uint8_t *fwd_codes, uint64_t n_fwd, smem_index_t *idx);
/* Same .bwt, built on a HIP device by prefix doubling + radix sort
 * (seconds for Gbp genomes); 2 x n_fwd must stay below 2^32 - 1. */
int  smem_bwt_build_gpu(int device, const uint8_t *fwd_codes, uint64_t n_fwd, smem_index_t *idx);
/* .bwt file I/O (software/bwt.c:841-850, 899-918) */
int  smem_bwt_read(const char *fn, smem_index_t *idx);
int  smem_bwt_write(const char *fn, const smem_index_t *idx);
void smem_index_free(smem_index_t *idx);
/* smem_bwt_build + the sampled SA bwa index writes beside it (`bwa index`
 * .sa, sa_intv = 32 there, software/bwtindex.c:280); sa_intv a power of 2 */
int  smem_bwt_build_sa(const uint8_t *fwd_codes, uint64_t n_fwd, int sa_intv, smem_index_t *idx, smem_sa_t *sa);
/* the same on a HIP device (prefix doubling, as smem_bwt_build_gpu) */
int  smem_bwt_build_gpu_sa(int device, const uint8_t *fwd_codes, uint64_t n_fwd, int sa_intv, smem_index_t *idx,
                           smem_sa_t *sa);
/* The bucketed builder with 64-bit suffix positions (both strands up to 2^34
 * symbols: a human-size genome).  smem_bwt_build_gpu(_sa) switch to it by
 * themselves once 2 * n_fwd no longer fits 32 bits; called directly it runs
 * at any size (tests compare it with the CPU builder).  sa may be NULL. */
int  smem_bwt_build_gpu_large(int device, const uint8_t *fwd_codes, uint64_t n_fwd, int sa_intv, smem_index_t *idx,
                              smem_sa_t *sa);
/* .sa file I/O (software/bwt.c:852-897) */
int  smem_sa_read(const char *fn, smem_sa_t *sa);
int  smem_sa_write(const char *fn, const smem_sa_t *sa);
void smem_sa_free(smem_sa_t *sa);

/* --------------------------------------------------------------- device */
/* Number of visible HIP devices (0 on a machine without a GPU). */
int  smem_gpu_device_count(void);

/* Upload the index to `device` and keep it resident in HBM.  Replaces the
 * FPGA index upload in bwa_idx_load_bwt (software/bwa.c:286-307) and the
 * AAL buffer setup (software/HelloALINLB.cpp:344-451).  The words are copied;
 * the caller's arrays may be freed afterwards.  Limits: seq_len < 2^34 and
 * an index below 4 GiB (both strands of ~8.5 Gbp); SMEM_E_ARG otherwise. */
int  smem_gpu_init(smem_gpu_t **gpu, int device, const uint32_t *bwt, uint64_t bwt_size,
                   uint64_t primary, const uint64_t L2[5]);
void smem_gpu_shutdown(smem_gpu_t *gpu);

/* Multi-GPU: the index replicated on `n` devices, one smem_gpu_t each
 * (reads shard across GPUs, no collective).  devices[i] (NULL:
 * 0 .. n-1) may repeat a device (two contexts on one GPU).  sa / pac (NULL:
 * none) are made resident as smem_gpu_load_sa / smem_gpu_load_pac do.  The
 * uploads run side by side, one host thread per device.  Replaces, for all
 * devices at once, the single FPGA upload of software/bwa.c:286-307.  On
 * failure every device opened so far is shut down and gpus[] is zeroed. */
int  smem_gpu_init_devices(smem_gpu_t **gpus, int n, const int *devices, const uint32_t *bwt, uint64_t bwt_size,
                           uint64_t primary, const uint64_t L2[5], const smem_sa_t *sa, const uint8_t *pac,
                           int64_t l_pac);
/* The same with the device work on one host thread per device: the call
 * checks its arguments and returns; the uploads (and the .sa densification)
 * run while the caller goes on (bwa mem reads its first chunk).  Every entry
 * point that touches a device waits for its upload first; smem_gpu_wait_ready
 * waits explicitly.  A failed upload faults the handle (smem_gpu_fault 3):
 * every call on it is refused with SMEM_E_DEVICE, the caller's CPU path.  bwt,
 * sa->sa and pac must stay valid until the device is ready (the smem_sa_t
 * itself is copied). */
int  smem_gpu_init_devices_async(smem_gpu_t **gpus, int n, const int *devices, const uint32_t *bwt, uint64_t bwt_size,
                                 uint64_t primary, const uint64_t L2[5], const smem_sa_t *sa, const uint8_t *pac,
                                 int64_t l_pac);
/* Waits until everything the device does in the background has finished:
 * the upload chain, the .sa densification and any smem_gpu_reserve_slots
 * sizing (batches need not wait: their SA lookups use the uploaded samples
 * until the densification is done). */
int  smem_gpu_wait_ready(smem_gpu_t *gpu);
/* The steps of smem_gpu_init_devices_async one by one, so that each starts
 * as soon as its input is in memory (bwa_idx_load reads .bwt, then .sa, then
 * .pac): open_async checks the device and uploads the index in the
 * background; load_sa_async / load_pac_async queue behind it.  Same waiting
 * and fault rules. */
int  smem_gpu_open_async(smem_gpu_t **gpu, int device, const uint32_t *bwt, uint64_t bwt_size, uint64_t primary,
                         const uint64_t L2[5]);
int  smem_gpu_load_sa_async(smem_gpu_t *gpu, const smem_sa_t *sa);
int  smem_gpu_load_pac_async(smem_gpu_t *gpu, const uint8_t *pac, int64_t l_pac);
/* "0,2,5" -> devices[] = {0, 2, 5}; NULL or "" -> every visible device.
 * Returns the count, or a negative code (bad list, more than max_devices,
 * no device for the empty spec). */
int  smem_gpu_parse_devices(const char *spec, int *devices, int max_devices);

/* ------------------------------------------------------------ one shot */
/* Thread-safe; may be called concurrently from kt_for_batch workers (each
 * calling thread gets its own buffers, created on first use and freed by
 * smem_gpu_shutdown; the streams come from the device's admission pool, see
 * smem_gpu_set_max_active).  seq[i] are nt4 codes (0..3, >3 ambiguous),
 * len[i] their lengths; the results stay valid until the same thread calls
 * smem_gpu_collect again.  Read them with smem_batch_read(*batch_out, i, ...). */
int  smem_gpu_collect(smem_gpu_t *gpu, int n_reads, const uint8_t *const *seq, const int *len,
                      const smem_opt_t *opt, smem_batch_t **batch_out);
/* The same with the batch chosen by worker slot (slot >= 0: the kt_for_batch
 * tid of software/kthread_batch.c:38, which the reference maps to its
 * per-worker FPGA buffer through get_thread_id, software/bwt.c:51-58; the slot's
 * batch is reused by whichever thread holds the slot next, so the short-lived
 * threads bwa mem starts per chunk do not each leave a batch behind; two
 * threads must not use one slot at once; slot < 0: the calling thread's batch,
 * as smem_gpu_collect).  flags: SMEM_COLLECT_NO_FETCH -- results stay in HBM
 * for smem_batch_sa / _chain / _chain2aln, and smem_batch_fetch_mask copies
 * only what the caller reads. */
#define SMEM_COLLECT_NO_FETCH 1
int  smem_gpu_collect_ex(smem_gpu_t *gpu, int slot, int n_reads, const uint8_t *const *seq, const int *len,
                         const smem_opt_t *opt, int flags, smem_batch_t **batch_out);
/* Pre-size worker slots [0, n_slots) of smem_gpu_collect_ex for batches of up
 * to reads_per_slot reads of up to max_len bases, with the later stages'
 * scratch and pinned result buffers sized at generous per-read estimates, and
 * load the code object of every kernel file (hipFuncGetAttributes: a kernel's
 * code object otherwise loads on its first launch); SMEM_GPU_WARMUP=full runs
 * one warm-up pass of every stage over a few reads cut from the resident .pac
 * instead.  Replaces the
 * per-worker buffers main_mem allocates before the first chunk
 * (software/fastmap.c:207-210).  Runs on a background host thread: the call
 * returns at once, and the first smem_gpu_collect* on the device waits for it.
 * A batch larger than reserved is re-created on first use, as without it. */
int  smem_gpu_reserve_slots(smem_gpu_t *gpu, int n_slots, int reads_per_slot, int max_len);
/* Reads one seeding launch holds in flight on the device at once: the
 * persistent grid's read owners (CUs x lanes per CU x owners per wave / 64;
 * 92,160 for the default kernel on MI355X).  A worker batch of at least this
 * many reads fills the device by itself (the binding's batch plan).
 * Needs no open device work: the CU count comes from the device's attributes. */
int  smem_gpu_grid_reads(const smem_gpu_t *gpu);
/* Admission, the HARP manager's role (software/fastmap.c:320-429): at most n
 * calls run work on the device at once, each on one of n leased stream pairs
 * (a device carries at most 2n streams however many workers share it); the
 * others wait for a pair instead of being rejected.  Default 8, or
 * SMEM_GPU_MAX_ACTIVE at smem_gpu_init; 0 restores the default. */
int  smem_gpu_set_max_active(smem_gpu_t *gpu, int n);
/* The admission limit in force (what smem_gpu_set_max_active / SMEM_GPU_MAX_ACTIVE
 * set): the batches a device runs at once, for a caller's batch plan. */
int  smem_gpu_get_max_active(const smem_gpu_t *gpu);
/* 0: the device has not faulted; 1: a HIP runtime failure faulted it (the
 * HIP runtime may also have printed its own diagnostics -- on a queue abort,
 * a dump of the queue's packets on stdout); 2: an injected sticky fault
 * (SMEM_GPU_FAIL); 3: smem_gpu_init_devices_async could not upload the index
 * (a refusal, e.g. an allocation that does not fit; an upload that failed on a
 * HIP runtime error reports 1).  msg (may be NULL) gets the first failure's text. */
int  smem_gpu_fault(const smem_gpu_t *gpu, char *msg, int msg_len);
/* Memory held: a batch's device and pinned host buffers (they grow to the
 * largest batch seen); a device's resident index (Occ64, densified SA and the
 * uploaded samples, .pac) and the batches it keeps (worker slots, per-thread
 * batches, the streaming pool) -- what a maintainer sizes -t / -b against. */
int  smem_batch_memory(const smem_batch_t *b, uint64_t *device_bytes, uint64_t *pinned_bytes);
int  smem_gpu_memory(smem_gpu_t *gpu, uint64_t *index_bytes, uint64_t *batch_bytes, uint64_t *pinned_bytes,
                     int *n_batches);

/* ------------------------------------------------------------ streaming */
/* bwa mem's chunk loop (software/fastmap.c:213-228, mem_process_seqs ->
 * kt_for_batch, software/bwamem.c:1614-1640, software/kthread_batch.c:29-59)
 * over one device, for read sets larger than one batch.  Reads [0, n_reads)
 * (nt4 codes, offs[n_reads + 1] into codes) are cut into chunks of at most
 * chunk_reads; n_workers host threads each own a batch (pinned staging
 * buffers, a HIP stream, device buffers) and run whole chunks: stage + H2D,
 * seeding + compaction, D2H into pinned host memory, then fn(ctx, chunk,
 * first_read, n, batch) on that worker's thread, where smem_batch_read /
 * smem_batch_results give the chunk's results (valid until fn returns).
 * Chunks are claimed in order; callbacks of different workers may overlap
 * and complete out of order (the chunk index orders them).  flags:
 * SMEM_STREAM_PAIRS -- n_reads must be even and chunk boundaries are kept
 * even, so both mates of a pair (reads 2k, 2k+1, interleaved as
 * software/bwamem.c:1600-1609 reads them) land in one chunk;
 * SMEM_STREAM_PACKED -- each interval crosses PCIe as a 16-B smem_pintv_t
 * (reads < 8192 bp), read with smem_batch_results_packed + smem_pintv_unpack
 * in the callback; SMEM_STREAM_RELEASE -- free the workers' batches when the
 * call returns.  Otherwise the handle keeps at most n_workers of them for
 * the next call (each holds ~1 GB of pinned host memory per 1M-read chunk;
 * a later call with fewer workers shrinks the pool, smem_gpu_shutdown frees
 * it).  fn may be NULL; a non-zero return from fn stops the stream and is
 * returned. */
typedef int (*smem_chunk_fn)(void *ctx, int64_t chunk, int64_t first_read, int n_reads, const smem_batch_t *b);
#define SMEM_STREAM_PAIRS   1   /* interleaved mates: chunks keep pairs whole */
#define SMEM_STREAM_PACKED  2   /* results as 16-B smem_pintv_t (smem_batch_results_packed): half the D2H */
#define SMEM_STREAM_RELEASE 4   /* do not keep the workers' batches (pinned buffers) for the next call */
typedef struct {
	double wall_s;           /* first chunk claimed -> last chunk delivered */
	uint64_t n_reads, n_chunks, n_intv;
	uint64_t h2d_bytes;      /* reads + offsets copied host -> device */
	uint64_t d2h_bytes;      /* intervals + list sizes + offsets copied device -> host */
	int workers;
	double stage_s, run_s, fetch_s;  /* summed over chunks: staging + H2D issue, smem_batch_run, smem_batch_fetch */
} smem_stream_stats_t;
int  smem_gpu_seed_stream(smem_gpu_t *gpu, int64_t n_reads, const uint8_t *codes, const uint64_t *offs,
                          const smem_opt_t *opt, int chunk_reads, int n_workers, int flags, smem_chunk_fn fn,
                          void *ctx, smem_stream_stats_t *stats);

/* ------------------------------------------------------- batch (explicit) */
int  smem_batch_create(smem_gpu_t *gpu, int max_reads, uint64_t max_bases, int max_len, smem_batch_t **b);
void smem_batch_destroy(smem_batch_t *b);
/* stage reads: per-read pointers (bseq1_t style) or one concatenated array
 * with offsets[n_reads+1]; copied host -> device on the batch stream */
int  smem_batch_set_reads(smem_batch_t *b, int n_reads, const uint8_t *const *seq, const int *len);
int  smem_batch_set_reads_packed(smem_batch_t *b, int n_reads, const uint8_t *codes, const uint64_t *offsets);
/* run the seeding loop on the resident reads; results stay in HBM */
int  smem_batch_run(smem_batch_t *b, const smem_opt_t *opt);
/* copy results device -> host (pinned): every stage that has run */
int  smem_batch_fetch(smem_batch_t *b);
/* copy only the named outputs: the interval lists (smem_batch_read /
 * _results), the SA positions (smem_batch_sa_results), the chains and seeds
 * (smem_batch_chain_results), the regions (smem_batch_aln_results).  Naming a
 * stage that has not run on this batch is SMEM_E_ARG.  A view whose output was
 * not copied by the last fetch returns SMEM_E_ARG. */
#define SMEM_FETCH_INTV    1
#define SMEM_FETCH_SA      2
#define SMEM_FETCH_CHAINS  4
#define SMEM_FETCH_REGS    8
#define SMEM_FETCH_ALL    15
int  smem_batch_fetch_mask(smem_batch_t *b, int mask);
/* per-read view of fetched results: the concatenation of all smem_next2
 * lists in order (n_intv intervals) and the size of each list (n_calls) */
int  smem_batch_read(const smem_batch_t *b, int i, const smem_intv_t **intv, int *n_intv,
                     const uint32_t **call_n, int *n_calls);
/* whole-batch views of fetched results: intv_off/call_off have n_reads+1 entries */
int  smem_batch_results(const smem_batch_t *b, const smem_intv_t **intv, const uint64_t **intv_off,
                        const uint32_t **call_n, const uint64_t **call_off);

/* 16-B wire form of a bwtintv_t (SMEM_STREAM_PACKED): x0, x1, x2 low words;
 * w = x0 bits 32-33 | x1 bits 32-33 << 2 | x2 bits 32-33 << 4 | query begin << 6
 * | query end << 19 (13 bits each) */
typedef struct { uint32_t x0, x1, x2, w; } smem_pintv_t;
#define SMEM_PINTV_MAX_LEN 8191
static inline void smem_pintv_unpack(const smem_pintv_t *p, smem_intv_t *o)
{
	o->x[0] = (uint64_t)(p->w & 3) << 32 | p->x0;
	o->x[1] = (uint64_t)(p->w >> 2 & 3) << 32 | p->x1;
	o->x[2] = (uint64_t)(p->w >> 4 & 3) << 32 | p->x2;
	o->info = (uint64_t)(p->w >> 6 & 8191) << 32 | (p->w >> 19);
}
/* the packed view of a batch fetched in SMEM_STREAM_PACKED mode */
int  smem_batch_results_packed(const smem_batch_t *b, const smem_pintv_t **pintv, const uint64_t **intv_off,
                               const uint32_t **call_n, const uint64_t **call_off);

/* ------------------------------------------------------- SA lookup */
/* Keep the sampled SA of the uploaded index resident in HBM (the index's
 * .sa, software/bwt.c:877-897; bwa_idx_load's bwt_restore_sa).  SMEM_E_ARG
 * if it does not belong to the index.  Reads sa->sa[0 .. n_sa-1] only (the
 * reference's bwt->sa array as is).  The device copy is densified to every
 * 4th row by LF walks from these samples (8 B per 4 symbols of HBM); lookups
 * return exactly what bwt_sa does with the .sa's own interval.  The
 * densification runs in the background (~0.3 s at human size): the call
 * returns after the upload, and until the densification has finished
 * smem_batch_sa walks to the uploaded samples instead (the same positions,
 * more LF steps), so no batch waits for it (SMEM_GPU_SYNC_INIT=1: wait here;
 * SMEM_GPU_SA_RAW=1: always the uploaded samples).  The uploaded samples stay
 * resident beside the dense copy until smem_gpu_shutdown. */
int  smem_gpu_load_sa(smem_gpu_t *gpu, const smem_sa_t *sa);
/* After smem_batch_run: bwt_sa (software/bwt.c:104-114) of every seed
 * occurrence mem_insert_seed() generates from the lists — each interval with
 * seed length >= min_seed_len and x2 <= max_occ, rows x0 .. x0+x2-1
 * (software/bwamem.c:462-474) — on the GPU.  smem_batch_fetch then copies
 * them; smem_batch_sa_results gives the positions (forward-reverse
 * coordinates, the mem_seed_t rbeg) in interval order and occ_off[n_intv + 1]
 * indexed by flat interval (the numbering of smem_batch_results). */
int  smem_batch_sa(smem_batch_t *b, int min_seed_len, int max_occ);
int  smem_batch_sa_results(const smem_batch_t *b, const uint64_t **pos, const uint64_t **occ_off, uint64_t *n_occ);

/* ------------------------------------------------------- chaining */
/* mem_seed_t (software/bwamem.c:317-320) */
typedef struct {
	int64_t rbeg;          /* forward-reverse coordinate (bwt_sa) */
	int32_t qbeg, len;
} smem_seed_t;
/* one chain of mem_chain_t (software/bwamem.c:322-326): pos and its n seeds,
 * seeds[seed_off .. seed_off + n) of smem_batch_chain_results */
typedef struct {
	int64_t pos;
	uint64_t seed_off;
	int32_t n, pad;
} smem_chain_t;
/* the mem_opt_t fields chaining reads (software/bwamem.h:39-53) */
typedef struct {
	int w;                    /* band width, 100 */
	int max_chain_gap;        /* 10000 */
	float mask_level;         /* 0.50 */
	float chain_drop_ratio;   /* 0.50 */
	int filter;               /* 1: mem_chain_flt after mem_chain, as mem_align1_core does */
} smem_chain_opt_t;
void smem_chain_opt_default(smem_chain_opt_t *opt);
/* After smem_batch_sa: mem_chain (software/bwamem.c:593-614) of every read on
 * the GPU — the seed sequence of mem_insert_seed (software/bwamem.c:462-499),
 * test_and_merge into the kbtree of chains, in-order chain list — and, when
 * opt->filter, mem_chain_flt (software/bwamem.c:629-690).  l_pac is the
 * forward strand length (bns->l_pac).  The filter's drop margin uses the
 * min_seed_len given to smem_batch_sa.  smem_batch_fetch copies the chains;
 * smem_batch_chain_results returns them per read: chain_off[n_reads + 1]
 * into chains[], each chain's seeds contiguous in seeds[]. */
int  smem_batch_chain(smem_batch_t *b, int64_t l_pac, const smem_chain_opt_t *opt);
int  smem_batch_chain_results(const smem_batch_t *b, const smem_chain_t **chains, const uint64_t **chain_off,
                              const smem_seed_t **seeds, uint64_t *n_chains, uint64_t *n_seeds);

/* --------------------------------------------------- SW extension */
/* one ksw_extend2 call (software/ksw.c:379) as mem_chain2aln makes it
 * (software/bwamem.c:1136, 1164): query / target are offsets into the code
 * pools (0..4; the left extension's reversed sequences as the caller builds
 * them), m = 5 */
typedef struct {
	uint64_t q_off, t_off;
	int32_t qlen, tlen;       /* 1 <= qlen <= 255, tlen >= 0 */
	int32_t w, end_bonus, zdrop, h0;
} smem_ksw_task_t;
/* the return value and the five out-parameters of ksw_extend2 */
typedef struct {
	int32_t score, qle, tle, gtle, gscore, max_off;
} smem_ksw_result_t;
typedef struct {
	int8_t mat[25], pad[3];   /* bwa_fill_scmat (software/bwa.c:84-93) */
	int32_t o_del, e_del, o_ins, e_ins;
} smem_ksw_opt_t;
/* mem_opt_init's scoring (software/bwamem.c:50-52): a 1, b 4, gaps 6 + 1 */
void smem_ksw_opt_default(smem_ksw_opt_t *opt);
/* ksw_extend2 of every task on the GPU, results in task order: the same
 * values the reference returns.  Host buffers in and out; kernel_ms (may be
 * NULL) gets the kernel's HIP-event time.  SMEM_E_ARG for a task outside the
 * limits above or gap penalties with e < 1 or o < 0 (the caller extends
 * those on the CPU, as the reference's reject path would). */
int  smem_ksw_extend(smem_gpu_t *gpu, int n, const smem_ksw_task_t *tasks, const uint8_t *q, uint64_t q_bytes,
                     const uint8_t *t, uint64_t t_bytes, const smem_ksw_opt_t *opt, smem_ksw_result_t *out,
                     double *kernel_ms);

/* one ksw_align2 call (software/ksw.c:342) as mem_chain2aln_short makes it
 * (software/bwamem.c:835-836): xtra = KSW_XSUBO | KSW_XSTART | (KSW_XBYTE when
 * qlen * a < 250) | min_seed_len * a; query / target offsets into code pools */
typedef struct {
	uint64_t q_off, t_off;
	int32_t qlen, tlen;       /* 1 <= qlen <= 256, 0 <= tlen <= 256 */
	int32_t xtra, pad;        /* KSW_XBYTE 0x10000, KSW_XSTOP 0x20000, KSW_XSUBO 0x40000, KSW_XSTART 0x80000 */
} smem_ksw_atask_t;
/* kswr_t (software/ksw.h:13-15) */
typedef struct {
	int32_t score, te, qe, score2, te2, tb, qb;
} smem_ksw_aresult_t;
/* ksw_align2 (striped local SW: ksw_u8 with KSW_XBYTE, else ksw_i16; the start
 * pass with KSW_XSTART) of every task on the GPU, one wave per problem: the
 * kswr_t the reference returns.  The device routine is the one
 * smem_chain2aln / smem_batch_chain2aln run for mem_chain2aln_short. */
int  smem_ksw_align2(smem_gpu_t *gpu, int n, const smem_ksw_atask_t *tasks, const uint8_t *q, uint64_t q_bytes,
                     const uint8_t *t, uint64_t t_bytes, const smem_ksw_opt_t *opt, smem_ksw_aresult_t *out,
                     double *kernel_ms);

/* ------------------------------------------- chains -> alignment regions */
/* mem_alnreg_t (software/bwamem.h:62-74); hash / sub / sub_n / secondary are
 * left 0 here, as mem_chain2aln leaves them (mem_mark_primary sets them later) */
typedef struct {
	int64_t rb, re;
	int32_t qb, qe, score, truesc, sub, csub, sub_n, w, seedcov, secondary;
	uint64_t hash;
} smem_alnreg_t;
/* the mem_opt_t fields mem_chain2aln reads (software/bwamem.h:33-45) */
typedef struct {
	smem_ksw_opt_t sc;        /* matrix and gap penalties */
	int a;                    /* match score, 1 */
	int w;                    /* band width, 100 */
	int zdrop;                /* 100 */
	int pen_clip5, pen_clip3; /* 5, 5 */
	int min_seed_len;         /* 19 */
} smem_aln_opt_t;
void smem_aln_opt_default(smem_aln_opt_t *opt);
/* The loop of mem_align1_core over every read's chains (software/bwamem.c:1452-1460):
 * mem_chain2aln_short, then mem_chain2aln when it declines (software/bwamem.c:805-852,
 * 1040-1188), on the GPU, one wave per read.  Replaces the host-side calls at
 * software/bwamem.c:1421-1422 / 1457-1458.  Inputs are host buffers in the layout
 * smem_batch_chain_results returns (chains[chain_off[r] .. chain_off[r+1]) of read r,
 * seeds[n_seeds] indexed by smem_chain_t.seed_off) plus the reads (nt4 codes, offs[n+1])
 * and the 2-bit forward-strand .pac (software/bntseq.c:303-309, l_pac bases).
 * regs must hold one region per chain seed (sum of chains' n); reg_off[n_reads + 1]
 * gets each read's regions, in the order the reference appends them.  Reads longer
 * than 1024 bp give SMEM_E_ARG. */
int  smem_chain2aln(smem_gpu_t *gpu, int n_reads, const uint8_t *codes, const uint64_t *offs,
                    const smem_chain_t *chains, const uint64_t *chain_off, const smem_seed_t *seeds, uint64_t n_seeds,
                    const uint8_t *pac, int64_t l_pac, const smem_aln_opt_t *opt, smem_alnreg_t *regs,
                    uint64_t *reg_off, double *kernel_ms);
/* (pac may be NULL when smem_gpu_load_pac made this l_pac's .pac resident.
 * Query codes must be 0..4 and no two chains may share seeds: SMEM_E_ARG.) */

/* Keep the 2-bit forward-strand .pac of the uploaded index resident in HBM
 * (bwa_idx_load's idx->pac, software/bwa.c:325-330); 2 * l_pac must equal the
 * index's seq_len.  Replacing a loaded .pac must not overlap a chains ->
 * regions call (smem_batch_chain2aln, smem_chain2aln) on the same handle:
 * such a call may still read the old copy. */
int  smem_gpu_load_pac(smem_gpu_t *gpu, const uint8_t *pac, int64_t l_pac);
/* Device-resident twin of smem_chain2aln: after smem_batch_chain (filter = 1,
 * as mem_align1_core_batched filters before extending, software/bwamem.c:1414-1422),
 * mem_chain2aln_short / mem_chain2aln of every chain of every read of the batch
 * over the reads, chains and seeds still in HBM and the resident .pac: no host
 * round trip, no per-call allocation once the batch has grown.  smem_batch_fetch
 * copies the regions; smem_batch_aln_results returns them with reg_off[n_reads + 1]. */
int  smem_batch_chain2aln(smem_batch_t *b, const smem_aln_opt_t *opt);
int  smem_batch_aln_results(const smem_batch_t *b, const smem_alnreg_t **regs, const uint64_t **reg_off,
                            uint64_t *n_regs);

/* ---------------------------------------------------------- telemetry */
typedef struct {
	double kernel_ms;        /* seeding kernel(s), HIP events on the batch stream */
	double compact_ms;       /* result compaction kernels */
	uint64_t n_intv;         /* intervals produced */
	uint64_t n_calls;        /* smem_next2 lists produced */
	uint32_t n_overflow;     /* reads re-run with a larger output capacity */
	int grid, block;         /* launch shape of the seeding kernel */
	double sa_ms;            /* smem_batch_sa kernels */
	uint64_t n_occ;          /* seed occurrences resolved by smem_batch_sa */
	double chain_ms;         /* smem_batch_chain kernels */
	uint64_t n_chains;       /* chains kept by smem_batch_chain */
	double aln_ms;           /* smem_batch_chain2aln kernels */
	uint64_t n_regs;         /* regions made by smem_batch_chain2aln */
	uint64_t t_start, t_end; /* the seeding launches' first wave start and last wave end, chip-wide
	                          * 100 MHz clock (s_memrealtime): comparable across batches and streams */
} smem_batch_stats_t;
int  smem_batch_stats(const smem_batch_t *b, smem_batch_stats_t *st);

/* tuning knobs (0 = default) — lanes per CU of the persistent seeding grid
 * (default: the kernel's own -- 960 for the 4-block seed_wp_kernel variants,
 * 768 otherwise) */
int  smem_gpu_set_lanes_per_cu(smem_gpu_t *gpu, int lanes_per_cu);
/* per-read output capacity (intervals) of batches created afterwards;
 * reads needing more go through the overflow pass (0 = len/2 + 32) */
int  smem_gpu_set_intv_cap(smem_gpu_t *gpu, int cap_per_read);
/* seeding-kernel variant, all bit-exact, kept for A/B measurement (the
 * product build has 0 = 49 (the default, seed_wp_kernel: see
 * smem_gpu_get_kernel_variant below for 40-51), 2 = 20 = 26, 9, 23, 24, 25, 27
 * and 28; the others need a library built with `make AB=1`, else SMEM_E_ARG):
 * 2 (the default of rounds 1-4) Occ64 buckets (32 B per 64 symbols, re-laid on the
 * device at init), per-lane fetch into two register slots with bucket reuse,
 * the first 11 entries of every list in LDS (the forward list as a ring of its
 * last 11 pushes); 11 the same with LDS-DMA slots and 7 list entries; 12 that
 * with 12 LDS entries at 2 blocks per CU; 13 the round-1 default (LDS-DMA
 * slots, 7 entries, forward list in the arena); 16-18 variant 11 with two
 * backward extends per lane per iteration (16; 17/18 at 2 blocks per CU with
 * 12/13 entries); 19 the default with two extends when both hit the slots;
 * 20 = 2; 21 register slots, 7 entries, 4 blocks per CU; 3 reference-layout buckets,
 * cooperative fetch, lists in global memory; 4 reference layout, per-lane
 * fetch; 5 as 2 with 12 list entries in LDS (2 blocks per CU); 6 as 2 with
 * lists in global memory; 9 the default with per-wave cycle stamps; 24 the next read claimed in the
 * uniform section (25 stamped); 27 wave priority in the extend arithmetic instead; 28 no wave priority
 * (smem_batch_debug); 10 the default on the Occ192 layout (64-B lines of
 * 192 symbols, built on first use: exact, 7 % slower at human size); 22
 * register slots on Occ192; 23 the default reading the bi-interval of every
 * extend result of at most k bases from the k-mer table (needs
 * smem_gpu_set_kmer_table) */
int  smem_gpu_set_kernel_variant(smem_gpu_t *gpu, int variant);
/* the seeding kernel variant the handle runs (0 given to the setter = the
 * default, 49: seed_wp_kernel -- the backward steps' entries extended by the
 * whole wave and pruned by ballot / prefix rank (software/bwt.c:812-826), 24
 * reads owned per wave, 18 list entries per read in LDS, 4 blocks per CU.
 * A/B: 40 32 reads / 20 entries / 3 blocks; 41 32 / 16; 42 24 / 24; 43 = 40
 * without wave priority; 44 24 / 16 / 4 blocks; 45 32 / 12; 46 28 / 14; 47, 48
 * two entries per worker lane; 50 20 / 22; 51 = 44 without wave priority; 2:
 * the lane-per-read seed_kernel of rounds 1-4).  SMEM_GPU_SEED_VARIANT in the
 * environment sets the default of every handle opened afterwards. */
int  smem_gpu_get_kernel_variant(const smem_gpu_t *gpu);
/* build (k = 1..15) or free (k = 0) the device table of the bi-intervals of
 * every string of 1..k bases, built on the device from the resident index:
 * 16 B x (4^(k+1) - 4) / 3 (k = 12: 358 MB, 14: 5.7 GB); a table of a string
 * is the interval bwt_extend reaches for it on any path (software/bwt.c:416-429) */
int  smem_gpu_set_kmer_table(smem_gpu_t *gpu, int k);
/* variant 9 (stamped diagnostic build): copy the per-wave cycle split
 * {advance, fetch, compute, iterations, active lanes, t0, t1, 0} of the last
 * run; returns the number of words copied or a negative code */
int  smem_batch_debug(const smem_batch_t *b, uint64_t *out, uint64_t n_words);
const char *smem_strerror(int code);
/* content hash (16 hex digits) of the sources this library was built from
 * (bwa-mem-harp2_amd/Makefile SRC_HASH): lets a caller prove that the .so it
 * loaded is the build of the sources beside it */
const char *smem_gpu_build_id(void);
/* hash of the seeding kernel's own sources and compile flags only
 * (csrc/smem_kernels.hip / .h): a counter profile of seed_kernel recorded on
 * another build of the runtime still describes this one when it matches */
const char *smem_gpu_kernel_id(void);

#ifdef __cplusplus
}
#endif
#endif
