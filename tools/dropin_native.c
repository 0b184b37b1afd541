/* dropin_native.c -- the drop-in's call shape from native threads (bench.py secondary.dropin,
 * "16_callers_native"): fishnet's workers are Rust tasks calling the C-ABI with no interpreter lock
 * between them (/root/reference/src/main.rs:263-343), so the Python threads of bench.py's own
 * 16-caller line measure the interpreter as much as the library.  T pthreads call
 * gn_evaluate_batch (GN_MODE_FULL, one lichess game per call) K times each on one context, after
 * a barrier; prints one JSON object: positions/s, calls/s, per-call p50 / p99, the coalescer's
 * launches, and a checksum of every call's records against a single-threaded pass.
 *
 * usage: dropin_native BIG.nnue SMALL.nnue GAMES.txt THREADS CALLS_PER_THREAD COALESCE
 * GAMES.txt: one game per line, its positions' FENs separated by '|'.
 * Built by fishnet_amd/build.py (build_dropin_native) against libgpu_nnue.so. */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/gpu_nnue.h"

typedef struct {
  char **fens;
  size_t n;
} Game;

static Game *games;
static size_t n_games;
static gn_ctx *ctx;
static int T, K;
static pthread_barrier_t go;
static double *lat;      /* [T * K] seconds */
static uint64_t *sums;   /* [T * K] record checksums */
static uint64_t *expect; /* [n_games] single-threaded checksums */
static int failed;

static double now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static uint64_t checksum(const gn_eval *e, size_t n) {
  const unsigned char *p = (const unsigned char *)e;
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < n * sizeof(gn_eval); ++i) h = (h ^ p[i]) * 1099511628211ull;
  return h;
}

static void *worker(void *arg) {
  const int t = (int)(intptr_t)arg;
  size_t cap = 0;
  for (size_t g = 0; g < n_games; ++g)
    if (games[g].n > cap) cap = games[g].n;
  gn_eval *out = malloc(cap * sizeof(gn_eval));
  pthread_barrier_wait(&go);
  for (int i = 0; i < K; ++i) {
    const Game *g = &games[((size_t)t * K + i) % n_games];
    const double t0 = now();
    const int rc = gn_evaluate_batch(ctx, (const char *const *)g->fens, g->n, out);
    lat[t * K + i] = now() - t0;
    if (rc) __atomic_store_n(&failed, rc, __ATOMIC_RELAXED);
    sums[t * K + i] = checksum(out, g->n);
  }
  free(out);
  return NULL;
}

static int cmp(const void *a, const void *b) {
  const double x = *(const double *)a, y = *(const double *)b;
  return x < y ? -1 : x > y;
}

int main(int argc, char **argv) {
  if (argc != 7) {
    fprintf(stderr, "usage: %s BIG SMALL GAMES THREADS CALLS_PER_THREAD COALESCE\n", argv[0]);
    return 2;
  }
  T = atoi(argv[4]), K = atoi(argv[5]);
  const int coalesce = atoi(argv[6]);
  FILE *f = fopen(argv[3], "r");
  if (!f || T <= 0 || K <= 0) return 2;
  size_t gcap = 1024;
  games = calloc(gcap, sizeof(Game));
  char *line = NULL;
  size_t lcap = 0;
  ssize_t len;
  while ((len = getline(&line, &lcap, f)) > 0) {
    if (line[len - 1] == '\n') line[--len] = 0;
    if (!len) continue;
    if (n_games == gcap) games = realloc(games, (gcap *= 2) * sizeof(Game));
    Game *g = &games[n_games++];
    size_t n = 1;
    for (ssize_t i = 0; i < len; ++i) n += line[i] == '|';
    g->fens = malloc(n * sizeof(char *));
    g->n = 0;
    for (char *tok = strtok(line, "|"); tok; tok = strtok(NULL, "|")) g->fens[g->n++] = strdup(tok);
  }
  free(line);
  fclose(f);
  const int dev = 0;
  if (gn_load_net(argv[1], argv[2], &dev, 1, &ctx)) {
    fprintf(stderr, "gn_load_net: %s\n", gn_last_error());
    return 1;
  }
  gn_set_option(ctx, GN_OPT_COALESCE, coalesce);
  /* the records every game's call must return: single-threaded, after a warmup */
  expect = malloc(n_games * sizeof(uint64_t));
  size_t cap = 0, npos = 0;
  for (size_t g = 0; g < n_games; ++g)
    if (games[g].n > cap) cap = games[g].n;
  gn_eval *out = malloc(cap * sizeof(gn_eval));
  for (size_t g = 0; g < n_games; ++g) {
    if (gn_evaluate_batch(ctx, (const char *const *)games[g].fens, games[g].n, out)) {
      fprintf(stderr, "gn_evaluate_batch: %s\n", gn_last_error());
      return 1;
    }
    expect[g] = checksum(out, games[g].n);
  }
  free(out);
  lat = calloc((size_t)T * K, sizeof(double));
  sums = calloc((size_t)T * K, sizeof(uint64_t));
  int64_t l0 = 0, c0 = 0, l1 = 0, c1 = 0;
  gn_get_option(ctx, GN_STAT_BATCH_LAUNCHES, &l0);
  gn_get_option(ctx, GN_STAT_BATCH_CALLS, &c0);
  pthread_barrier_init(&go, NULL, (unsigned)T + 1);
  pthread_t *th = malloc((size_t)T * sizeof(pthread_t));
  for (int t = 0; t < T; ++t) pthread_create(&th[t], NULL, worker, (void *)(intptr_t)t);
  pthread_barrier_wait(&go);
  const double t0 = now();
  for (int t = 0; t < T; ++t) pthread_join(th[t], NULL);
  const double wall = now() - t0;
  gn_get_option(ctx, GN_STAT_BATCH_LAUNCHES, &l1);
  gn_get_option(ctx, GN_STAT_BATCH_CALLS, &c1);
  size_t bad = 0;
  for (int t = 0; t < T; ++t)
    for (int i = 0; i < K; ++i) {
      const size_t g = ((size_t)t * K + i) % n_games;
      npos += games[g].n;
      bad += sums[t * K + i] != expect[g];
    }
  qsort(lat, (size_t)T * K, sizeof(double), cmp);
  const size_t m = (size_t)T * K;
  printf("{\"calls\": %zu, \"threads\": %d, \"coalesce\": %d, \"positions_per_s\": %.1f, \"calls_per_s\": %.1f, "
         "\"p50_ms\": %.4f, \"p99_ms\": %.4f, \"launches\": %lld, \"calls_served\": %lld, "
         "\"records_equal_to_single_thread\": %s, \"mismatching_calls\": %zu, \"failed_rc\": %d}\n",
         m, T, coalesce, (double)npos / wall, (double)m / wall, 1e3 * lat[m / 2], 1e3 * lat[(m * 99) / 100],
         (long long)(l1 - l0), (long long)(c1 - c0), bad ? "false" : "true", bad, failed);
  gn_free(ctx);
  return failed || bad ? 1 : 0;
}
