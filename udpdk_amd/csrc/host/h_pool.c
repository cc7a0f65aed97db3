/*
 * h_pool.c — fork-join worker threads for the poll's per-socket host loops (burst admission and
 * ring publication in udpdk_poll_rx). The reference poller does this work on one core per
 * batch of BURST_SIZE mbufs (udpdk_poller.c:516-545); here one poll hands over up to a whole
 * GPU batch (1 M frames), so its per-socket loops run on [gpu] poll_threads threads, each over a
 * contiguous range of sockets (every socket's ring keeps a single producer).
 *
 * The workers are started on first use and stopped by udpdk_cleanup. h_pool_run(fn, ctx) runs
 * fn(ctx, part, parts) for every part < parts, part 0 on the calling thread, and returns when
 * all have finished.
 */
#include <pthread.h>
#include <stdint.h>

#include "host_state.h"

static struct {
    pthread_t th[H_MAX_WORKERS];
    uint32_t n;                   /* worker threads (parts = n + 1) */
    int started;
    pthread_mutex_t mu;
    pthread_cond_t go, done;
    uint64_t gen;                 /* job generation */
    uint64_t start_gen;           /* gen when the workers were started: the next job is theirs */
    uint32_t pending;             /* workers still running the current job */
    int stop;
    h_job_fn fn;
    void *ctx;
} g_pool = {.mu = PTHREAD_MUTEX_INITIALIZER, .go = PTHREAD_COND_INITIALIZER,
            .done = PTHREAD_COND_INITIALIZER};

static void *h_worker(void *arg)
{
    const uint32_t part = (uint32_t)(uintptr_t)arg;
    pthread_mutex_lock(&g_pool.mu);
    uint64_t seen = g_pool.start_gen;     /* not 0: after a restart gen still counts old jobs */
    for (;;) {
        while (g_pool.gen == seen && !g_pool.stop) pthread_cond_wait(&g_pool.go, &g_pool.mu);
        if (g_pool.stop) break;
        seen = g_pool.gen;
        const h_job_fn fn = g_pool.fn;
        void *ctx = g_pool.ctx;
        const uint32_t parts = g_pool.n + 1;
        pthread_mutex_unlock(&g_pool.mu);
        fn(ctx, part, parts);
        pthread_mutex_lock(&g_pool.mu);
        if (--g_pool.pending == 0) pthread_cond_signal(&g_pool.done);
    }
    pthread_mutex_unlock(&g_pool.mu);
    return NULL;
}

static void h_pool_start(void)
{
    uint32_t want = g_udpdk.poll_threads ? g_udpdk.poll_threads : H_POLL_THREADS_DEFAULT;
    if (want > H_MAX_WORKERS + 1) want = H_MAX_WORKERS + 1;
    g_pool.started = 1;
    g_pool.stop = 0;
    g_pool.n = 0;
    g_pool.start_gen = g_pool.gen;
    for (uint32_t t = 1; t < want; t++) {
        if (pthread_create(&g_pool.th[g_pool.n], NULL, h_worker, (void *)(uintptr_t)t)) break;
        g_pool.n++;
    }
}

uint32_t h_pool_parts(void)
{
    if (!g_pool.started) h_pool_start();
    return g_pool.n + 1;
}

void h_pool_run(h_job_fn fn, void *ctx)
{
    if (!g_pool.started) h_pool_start();
    if (g_pool.n) {
        pthread_mutex_lock(&g_pool.mu);
        g_pool.fn = fn;
        g_pool.ctx = ctx;
        g_pool.pending = g_pool.n;
        g_pool.gen++;
        pthread_cond_broadcast(&g_pool.go);
        pthread_mutex_unlock(&g_pool.mu);
    }
    fn(ctx, 0, g_pool.n + 1);
    if (g_pool.n) {
        pthread_mutex_lock(&g_pool.mu);
        while (g_pool.pending) pthread_cond_wait(&g_pool.done, &g_pool.mu);
        pthread_mutex_unlock(&g_pool.mu);
    }
}

void h_pool_stop(void)
{
    if (!g_pool.started) return;
    pthread_mutex_lock(&g_pool.mu);
    g_pool.stop = 1;
    pthread_cond_broadcast(&g_pool.go);
    pthread_mutex_unlock(&g_pool.mu);
    for (uint32_t t = 0; t < g_pool.n; t++) pthread_join(g_pool.th[t], NULL);
    g_pool.n = 0;
    g_pool.started = 0;
}
