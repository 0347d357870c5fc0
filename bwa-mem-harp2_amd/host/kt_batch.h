/*
 * kt_batch.h — batched work-stealing thread pool with the calling convention
 * of the reference's kt_for_batch (software/kthread_batch.c:46-59):
 *   func(data, start, batch_size, thread_index)
 * over [0, n) in chunks of batch_size.  Unlike the reference it publishes no
 * global thread table (software/kthread_batch.c:54 / software/bwt.c:51-58):
 * the worker index is passed to func, which is all a GPU-backed worker needs
 * to own its stream.
 */
#ifndef SMEM_KT_BATCH_H
#define SMEM_KT_BATCH_H

#ifdef __cplusplus
extern "C" {
#endif

void kt_for_batch_gpu(int n_threads, void (*func)(void *, int, int, int), void *data, int n, int batch_size);

#ifdef __cplusplus
}
#endif
#endif
