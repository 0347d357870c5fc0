/*
 * kt_batch.c — see kt_batch.h.  Each worker first takes the chunks
 * start = w*batch, w*batch + T*batch, ... (the reference's static
 * interleave, software/kthread_batch.c:57), then steals from the worker with
 * the lowest cursor (software/kthread_batch.c:19-27).
 */
#include <pthread.h>
#include <stdlib.h>
#include "kt_batch.h"

typedef struct pool_s pool_t;

typedef struct {
	pool_t *pool;
	int idx;
	long cursor;          /* next start this worker owns */
} worker_t;

struct pool_s {
	int n_threads, n, batch;
	worker_t *w;
	void (*func)(void *, int, int, int);
	void *data;
};

static long take(worker_t *w)
{
	return __sync_fetch_and_add(&w->cursor, (long)w->pool->n_threads * w->pool->batch);
}

static long steal(pool_t *p)
{
	int i, best = -1;
	long lo = 0x7fffffffffffffffL;
	for (i = 0; i < p->n_threads; ++i)
		if (p->w[i].cursor < lo) lo = p->w[i].cursor, best = i;
	if (best < 0) return -1;
	lo = take(&p->w[best]);
	return lo >= p->n ? -1 : lo;
}

static void *worker_main(void *arg)
{
	worker_t *w = (worker_t*)arg;
	pool_t *p = w->pool;
	long s;
	while ((s = take(w)) < p->n) {
		int bs = p->n - s > p->batch ? p->batch : (int)(p->n - s);
		p->func(p->data, (int)s, bs, w->idx);
	}
	while ((s = steal(p)) >= 0) {
		int bs = p->n - s > p->batch ? p->batch : (int)(p->n - s);
		p->func(p->data, (int)s, bs, w->idx);
	}
	return 0;
}

void kt_for_batch_gpu(int n_threads, void (*func)(void *, int, int, int), void *data, int n, int batch_size)
{
	pool_t p;
	pthread_t *tid;
	int i;
	if (n_threads < 1) n_threads = 1;
	if (batch_size < 1) batch_size = 1;
	p.n_threads = n_threads; p.n = n; p.batch = batch_size; p.func = func; p.data = data;
	p.w = (worker_t*)calloc(n_threads, sizeof(worker_t));
	tid = (pthread_t*)calloc(n_threads, sizeof(pthread_t));
	for (i = 0; i < n_threads; ++i) {
		p.w[i].pool = &p;
		p.w[i].idx = i;
		p.w[i].cursor = (long)i * batch_size;
	}
	if (n_threads == 1) worker_main(&p.w[0]);
	else {
		for (i = 0; i < n_threads; ++i) pthread_create(&tid[i], 0, worker_main, &p.w[i]);
		for (i = 0; i < n_threads; ++i) pthread_join(tid[i], 0);
	}
	free(tid);
	free(p.w);
}
