/*
 * chain_oracle.c — TEST INFRASTRUCTURE ONLY.  Plain-C restatement of the
 * reference's seed chaining and chain filter, the §8(f) row 3 stage:
 *
 *   seed loop of mem_insert_seed   software/bwamem.c:462-499
 *   test_and_merge                 software/bwamem.c:334-354
 *   kbtree(chn) put / interval /   software/kbtree.h:97-110 (getp_aux), 150-166 (intervalp),
 *   in-order traversal                      172-224 (split, putp), 336-358 (traverse);
 *                                  node order t from KB_DEFAULT_SIZE 512 (kbtree.h:52, 369)
 *   mem_chain                      software/bwamem.c:593-614
 *   mem_chain_weight               software/bwamem.c:501-521
 *   mem_chain_flt                  software/bwamem.c:629-690
 *   ks_introsort / combsort /      software/ksort.h:146-224 (flt_lt, software/bwamem.c:626)
 *   insertion sort
 *
 * Input is the seed sequence mem_insert_seed generates (every occurrence of
 * every kept interval, in order: software/bwamem.c:462-474); output is an
 * SMCH stream (include/smem_formats.h).  Pinned against chains produced by
 * the compiled reference (oracle/_ref/ref_harness chain, tests/golden/).
 * Only tests/ use it; the product never links it.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include "smem_oracle.h"

/* ------------------------------------------------------------ chain store */
typedef struct {
	int64_t pos;
	int n, m;
	orc_seed_t *s;
} chn_t;

/* B-tree of chain ids keyed by chains[id].pos; the node order of kbtree(chn)
 * at KB_DEFAULT_SIZE: t = ((512 - 4 - 8) / (8 + 24) + 1) >> 1 = 8, so at most
 * 15 keys and 16 children per node */
#define BT_T 8
#define BT_MAX (2 * BT_T - 1)

typedef struct bnode {
	int leaf, n;
	int id[BT_MAX];
	struct bnode *c[BT_MAX + 1];
} bnode_t;

typedef struct {
	bnode_t *root;
	chn_t *ch;
	int n_ch, m_ch;
} tree_t;

static inline int64_t kpos(const tree_t *t, const bnode_t *x, int i) { return t->ch[x->id[i]].pos; }

/* position in a node: the leftmost key equal to k (*eq = 1) or else the last
 * key below k (-1 if none; *eq = 0) */
static int node_find(const tree_t *t, const bnode_t *x, int64_t k, int *eq)
{
	int lo = 0, hi = x->n;
	*eq = 0;
	if (x->n == 0) return -1;
	while (lo < hi) {
		int mid = (lo + hi) >> 1;
		if (kpos(t, x, mid) < k) lo = mid + 1;
		else hi = mid;
	}
	if (lo == x->n) return x->n - 1;
	if (kpos(t, x, lo) == k) { *eq = 1; return lo; }
	return lo - 1;
}

/* nearest chain at or below k: an equal key met on the way down wins */
static int tree_lower(const tree_t *t, int64_t k)
{
	const bnode_t *x = t->root;
	int lower = -1;
	while (x) {
		int eq, i = node_find(t, x, k, &eq);
		if (i >= 0 && eq) return x->id[i];
		if (i >= 0) lower = x->id[i];
		if (x->leaf) break;
		x = x->c[i + 1];
	}
	return lower;
}

static bnode_t *node_new(int leaf)
{
	bnode_t *x = (bnode_t*)calloc(1, sizeof(bnode_t));
	x->leaf = leaf;
	return x;
}

/* split the full child y = x->c[i]: its upper 7 keys move to a new right
 * sibling, its middle key moves up into x at i */
static void node_split(bnode_t *x, int i, bnode_t *y)
{
	bnode_t *z = node_new(y->leaf);
	z->n = BT_T - 1;
	memcpy(z->id, y->id + BT_T, sizeof(int) * (BT_T - 1));
	if (!y->leaf) memcpy(z->c, y->c + BT_T, sizeof(bnode_t*) * BT_T);
	y->n = BT_T - 1;
	memmove(x->c + i + 2, x->c + i + 1, sizeof(bnode_t*) * (x->n - i));
	x->c[i + 1] = z;
	memmove(x->id + i + 1, x->id + i, sizeof(int) * (x->n - i));
	x->id[i] = y->id[BT_T - 1];
	++x->n;
}

static void tree_insert(tree_t *t, int id)
{
	const int64_t k = t->ch[id].pos;
	bnode_t *x = t->root;
	int eq, i;
	if (x->n == BT_MAX) { /* grow a new root above the full one */
		bnode_t *s = node_new(0);
		s->c[0] = x;
		node_split(s, 0, x);
		t->root = x = s;
	}
	while (!x->leaf) {
		i = node_find(t, x, k, &eq) + 1;
		if (x->c[i]->n == BT_MAX) {
			node_split(x, i, x->c[i]);
			if (k > kpos(t, x, i)) ++i;
		}
		x = x->c[i];
	}
	i = node_find(t, x, k, &eq);
	memmove(x->id + i + 2, x->id + i + 1, sizeof(int) * (x->n - i - 1));
	x->id[i + 1] = id;
	++x->n;
}

static void tree_inorder(const bnode_t *x, int *out, int *n)
{
	int i;
	for (i = 0; i < x->n; ++i) {
		if (!x->leaf) tree_inorder(x->c[i], out, n);
		out[(*n)++] = x->id[i];
	}
	if (!x->leaf) tree_inorder(x->c[x->n], out, n);
}

static void tree_free(bnode_t *x)
{
	int i;
	if (!x) return;
	if (!x->leaf) for (i = 0; i <= x->n; ++i) tree_free(x->c[i]);
	free(x);
}

/* test_and_merge (software/bwamem.c:334-354): 1 = seed absorbed by chain c
 * (contained, or appended), 0 = a new chain is needed */
static int try_merge(const orc_chain_opt_t *o, int64_t l_pac, chn_t *c, const orc_seed_t *p)
{
	const orc_seed_t *first = &c->s[0], *last = &c->s[c->n - 1];
	int64_t qend = last->qbeg + last->len, rend = last->rbeg + last->len, x, y;
	if (p->qbeg >= first->qbeg && p->qbeg + p->len <= qend && p->rbeg >= first->rbeg && p->rbeg + p->len <= rend)
		return 1;
	if ((last->rbeg < l_pac || first->rbeg < l_pac) && p->rbeg >= l_pac) return 0;
	x = p->qbeg - last->qbeg;
	y = p->rbeg - last->rbeg;
	if (y >= 0 && x - y <= o->w && y - x <= o->w && x - last->len < o->max_chain_gap && y - last->len < o->max_chain_gap) {
		if (c->n == c->m) {
			c->m <<= 1;
			c->s = (orc_seed_t*)realloc(c->s, sizeof(orc_seed_t) * c->m);
		}
		c->s[c->n++] = *p;
		return 1;
	}
	return 0;
}

/* ------------------------------------------------------------- filtering */
typedef struct { int beg, end, w, p, p2; } flt_t;  /* p, p2: chain index, -1 = none */

#define FLT_LT(a, b) ((a).w > (b).w)

static void flt_insertsort(flt_t *a, size_t n)
{
	size_t i, j;
	for (i = 1; i < n; ++i)
		for (j = i; j > 0 && FLT_LT(a[j], a[j - 1]); --j) {
			flt_t t = a[j]; a[j] = a[j - 1]; a[j - 1] = t;
		}
}

static void flt_combsort(flt_t *a, size_t n)
{
	const double shrink = 1.2473309501039786540366528676643;
	size_t gap = n, i;
	int swapped;
	do {
		if (gap > 2) {
			gap = (size_t)(gap / shrink);
			if (gap == 9 || gap == 10) gap = 11;
		}
		swapped = 0;
		for (i = 0; i + gap < n; ++i)
			if (FLT_LT(a[i + gap], a[i])) {
				flt_t t = a[i]; a[i] = a[i + gap]; a[i + gap] = t;
				swapped = 1;
			}
	} while (swapped || gap > 2);
	if (gap != 1) flt_insertsort(a, n);
}

/* ks_introsort(mem_flt) step for step: median-of-3 quicksort that leaves
 * ranges of <= 16 for one final insertion sort and falls back to combsort
 * when the depth budget (2 x ceil(log2 n)) runs out */
static void flt_sort(flt_t *a, size_t n)
{
	struct { size_t l, r; int d; } st[128];
	int top = 0, d;
	size_t s, t, i, j, k;
	flt_t rp, tmp;
	if (n < 1) return;
	if (n == 2) {
		if (FLT_LT(a[1], a[0])) { tmp = a[0]; a[0] = a[1]; a[1] = tmp; }
		return;
	}
	for (d = 2; (1ul << d) < n; ++d);
	d <<= 1;
	s = 0; t = n - 1;
	for (;;) {
		if (s < t) {
			if (--d == 0) {
				flt_combsort(a + s, t - s + 1);
				t = s;
				continue;
			}
			i = s; j = t; k = i + ((j - i) >> 1) + 1;
			if (FLT_LT(a[k], a[i])) {
				if (FLT_LT(a[k], a[j])) k = j;
			} else k = FLT_LT(a[j], a[i]) ? i : j;
			rp = a[k];
			if (k != t) { tmp = a[k]; a[k] = a[t]; a[t] = tmp; }
			for (;;) {
				do ++i; while (FLT_LT(a[i], rp));
				do --j; while (i <= j && FLT_LT(rp, a[j]));
				if (j <= i) break;
				tmp = a[i]; a[i] = a[j]; a[j] = tmp;
			}
			tmp = a[i]; a[i] = a[t]; a[t] = tmp;
			if (i - s > t - i) {
				if (i - s > 16) { st[top].l = s; st[top].r = i - 1; st[top].d = d; ++top; }
				s = t - i > 16 ? i + 1 : t;
			} else {
				if (t - i > 16) { st[top].l = i + 1; st[top].r = t; st[top].d = d; ++top; }
				t = i - s > 16 ? i - 1 : s;
			}
		} else {
			if (top == 0) {
				flt_insertsort(a, n);
				return;
			}
			--top; s = st[top].l; t = st[top].r; d = st[top].d;
		}
	}
}

/* mem_chain_weight (software/bwamem.c:501-521), the reference's second loop
 * included as written (it advances `end` by query coordinates) */
static int chain_weight(const chn_t *c)
{
	int64_t end;
	int j, w = 0, tmp;
	for (j = 0, end = 0; j < c->n; ++j) {
		const orc_seed_t *s = &c->s[j];
		if (s->qbeg >= end) w += s->len;
		else if (s->qbeg + s->len > end) w = (int)(w + (s->qbeg + s->len - end));
		end = end > s->qbeg + s->len ? end : s->qbeg + s->len;
	}
	tmp = w;
	for (j = 0, end = 0; j < c->n; ++j) {
		const orc_seed_t *s = &c->s[j];
		if (s->rbeg >= end) w += s->len;
		else if (s->rbeg + s->len > end) w = (int)(w + (s->rbeg + s->len - end));
		end = end > s->qbeg + s->len ? end : s->qbeg + s->len;
	}
	return w < tmp ? w : tmp;
}

/* mem_chain_flt (software/bwamem.c:629-690) over ch[0..n): reorders ch by
 * weight, drops chains, returns the new count */
static int chain_filter(const orc_chain_opt_t *o, int n_chn, chn_t *ch)
{
	flt_t *a;
	chn_t *sw;
	int i, j, n;
	if (n_chn <= 1) return n_chn;
	a = (flt_t*)malloc(sizeof(flt_t) * n_chn);
	for (i = 0; i < n_chn; ++i) {
		a[i].beg = ch[i].s[0].qbeg;
		a[i].end = ch[i].s[ch[i].n - 1].qbeg + ch[i].s[ch[i].n - 1].len;
		a[i].w = chain_weight(&ch[i]);
		a[i].p = i;
		a[i].p2 = -1;
	}
	flt_sort(a, n_chn);
	sw = (chn_t*)malloc(sizeof(chn_t) * n_chn);
	for (i = 0; i < n_chn; ++i) { sw[i] = ch[a[i].p]; a[i].p = i; }
	memcpy(ch, sw, sizeof(chn_t) * n_chn);
	free(sw);
	for (i = 1, n = 1; i < n_chn; ++i) {
		for (j = 0; j < n; ++j) {
			int b_max = a[j].beg > a[i].beg ? a[j].beg : a[i].beg;
			int e_min = a[j].end < a[i].end ? a[j].end : a[i].end;
			if (e_min > b_max) {
				int li = a[i].end - a[i].beg, lj = a[j].end - a[j].beg;
				int min_l = li < lj ? li : lj;
				if (e_min - b_max >= min_l * o->mask_level) {
					if (a[j].p2 < 0) a[j].p2 = a[i].p;
					if (a[i].w < a[j].w * o->drop_ratio && a[j].w - a[i].w >= o->min_seed_len << 1) break;
				}
			}
		}
		if (j == n) a[n++] = a[i];
	}
	for (i = 0; i < n; ++i) {
		if (ch[a[i].p].n > 0) ch[a[i].p].n = -ch[a[i].p].n;
		if (a[i].p2 >= 0 && ch[a[i].p2].n > 0) ch[a[i].p2].n = -ch[a[i].p2].n;
	}
	free(a);
	for (i = 0; i < n_chn; ++i) {
		if (ch[i].n >= 0) { free(ch[i].s); ch[i].s = 0; ch[i].n = ch[i].m = 0; }
		else ch[i].n = -ch[i].n;
	}
	for (i = n = 0; i < n_chn; ++i)
		if (ch[i].n > 0) ch[n++] = ch[i];
	return n;
}

/* ----------------------------------------------------------------- driver */
typedef struct {
	uint8_t *p;
	size_t n, m;
} obuf_t;

static void ob_put(obuf_t *b, const void *src, size_t n)
{
	if (b->n + n > b->m) {
		b->m = (b->n + n) * 2 + 256;
		b->p = (uint8_t*)realloc(b->p, b->m);
	}
	memcpy(b->p + b->n, src, n);
	b->n += n;
}

/* mem_chain's body over one read's seed sequence + the optional filter */
static void chain_read(const orc_seed_t *seeds, uint64_t n_seeds, int64_t l_pac, const orc_chain_opt_t *o, obuf_t *ob)
{
	tree_t t;
	uint64_t k;
	int *order, n_out = 0, i;
	chn_t *out;
	uint32_t nc;
	memset(&t, 0, sizeof(t));
	t.root = node_new(1);
	for (k = 0; k < n_seeds; ++k) {
		const orc_seed_t *s = &seeds[k];
		int lower;
		if (s->rbeg < l_pac && l_pac < s->rbeg + s->len) continue; /* bridging the two strands */
		lower = t.n_ch ? tree_lower(&t, s->rbeg) : -1;
		if (lower >= 0 && try_merge(o, l_pac, &t.ch[lower], s)) continue;
		if (t.n_ch == t.m_ch) {
			t.m_ch = t.m_ch ? t.m_ch * 2 : 16;
			t.ch = (chn_t*)realloc(t.ch, sizeof(chn_t) * t.m_ch);
		}
		t.ch[t.n_ch].pos = s->rbeg;
		t.ch[t.n_ch].n = 1;
		t.ch[t.n_ch].m = 4;
		t.ch[t.n_ch].s = (orc_seed_t*)malloc(sizeof(orc_seed_t) * 4);
		t.ch[t.n_ch].s[0] = *s;
		tree_insert(&t, t.n_ch);
		++t.n_ch;
	}
	order = (int*)malloc(sizeof(int) * (t.n_ch + 1));
	tree_inorder(t.root, order, &n_out);
	out = (chn_t*)malloc(sizeof(chn_t) * (t.n_ch + 1));
	for (i = 0; i < n_out; ++i) out[i] = t.ch[order[i]];
	if (o->filter) n_out = chain_filter(o, n_out, out);
	nc = (uint32_t)n_out;
	ob_put(ob, &nc, 4);
	for (i = 0; i < n_out; ++i) {
		uint32_t n = (uint32_t)out[i].n;
		ob_put(ob, &out[i].pos, 8);
		ob_put(ob, &n, 4);
		ob_put(ob, out[i].s, sizeof(orc_seed_t) * out[i].n);
		free(out[i].s);
	}
	free(out);
	free(order);
	free(t.ch);
	tree_free(t.root);
}

typedef struct {
	const orc_seed_t *seeds;
	const uint64_t *seed_off;
	int64_t beg, end, l_pac;
	const orc_chain_opt_t *o;
	obuf_t ob;
} cjob_t;

static void *chain_job(void *data)
{
	cjob_t *j = (cjob_t*)data;
	int64_t r;
	for (r = j->beg; r < j->end; ++r)
		chain_read(j->seeds + j->seed_off[r], j->seed_off[r + 1] - j->seed_off[r], j->l_pac, j->o, &j->ob);
	return 0;
}

int orc_chain(int64_t n_reads, const orc_seed_t *seeds, const uint64_t *seed_off, int64_t l_pac,
		const orc_chain_opt_t *o, int n_threads, uint8_t **out, uint64_t *out_len)
{
	cjob_t *jobs;
	pthread_t *tid;
	obuf_t all;
	int t;
	uint64_t nr = (uint64_t)n_reads;
	if (n_reads < 0 || !o || !out || !out_len) return -1;
	if (n_threads < 1) n_threads = 1;
	if (n_threads > n_reads) n_threads = n_reads > 0 ? (int)n_reads : 1;
	jobs = (cjob_t*)calloc(n_threads, sizeof(cjob_t));
	tid = (pthread_t*)calloc(n_threads, sizeof(pthread_t));
	for (t = 0; t < n_threads; ++t) {
		jobs[t].seeds = seeds; jobs[t].seed_off = seed_off; jobs[t].l_pac = l_pac; jobs[t].o = o;
		jobs[t].beg = n_reads * t / n_threads; jobs[t].end = n_reads * (t + 1) / n_threads;
		pthread_create(&tid[t], 0, chain_job, &jobs[t]);
	}
	memset(&all, 0, sizeof(all));
	ob_put(&all, "SMCH0001", 8);
	ob_put(&all, &nr, 8);
	for (t = 0; t < n_threads; ++t) {
		pthread_join(tid[t], 0);
		ob_put(&all, jobs[t].ob.p, jobs[t].ob.n);
		free(jobs[t].ob.p);
	}
	free(jobs); free(tid);
	*out = all.p;
	*out_len = all.n;
	return 0;
}
