/*
 * synth.c -- deterministic synthetic workload generator (bench + tests).
 *
 * enwik8/enwik9 are not available offline, so the benchmark batches use the
 * calibrated English-like text of SURVEY.md 8(d), re-implemented here with a
 * splitmix64 generator so it is bit-stable on every host:
 *   - a 30,000-word vocabulary built once from seed 1234, word length
 *     1 + floor(Exp(mean 5)) letters drawn by English letter frequency;
 *   - words drawn Zipf(s = 1.1) with a per-stream seed;
 *   - 3 % capitalised, 1.5 % replaced by an integer < 100000;
 *   - 8 % of separators from {". ", ", ", "\n", " [[", "]] ", " | "}.
 * Secondary distributions: uniform random bytes and long runs.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define VOCAB 30000
#define MAX_WORD 40

static uint64_t sm64(uint64_t *s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static double u01(uint64_t *s) { return (double)(sm64(s) >> 11) * (1.0 / 9007199254740992.0); }

static char g_words[VOCAB][MAX_WORD + 1];
static unsigned char g_wlen[VOCAB];
static double g_zipf_cdf[VOCAB];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void build_vocab(void) {
  /* English letter frequencies (percent), a..z */
  static const double freq[26] = {8.2, 1.5, 2.8, 4.3, 12.7, 2.2, 2.0, 6.1, 7.0, 0.15,
                                  0.77, 4.0, 2.4, 6.7, 7.5, 1.9, 0.095, 6.0, 6.3, 9.1,
                                  2.8, 0.98, 2.4, 0.15, 2.0, 0.074};
  double cdf[26], acc = 0, tot = 0;
  uint64_t s = 1234;
  int i, k;
  for (i = 0; i < 26; i++) tot += freq[i];
  for (i = 0; i < 26; i++) { acc += freq[i] / tot; cdf[i] = acc; }
  for (i = 0; i < VOCAB; i++) {
    int len = 1 + (int)floor(-5.0 * log(1.0 - u01(&s)));
    if (len > MAX_WORD) len = MAX_WORD;
    for (k = 0; k < len; k++) {
      double u = u01(&s);
      int c = 0;
      while (c < 25 && u > cdf[c]) c++;
      g_words[i][k] = (char)('a' + c);
    }
    g_words[i][len] = 0;
    g_wlen[i] = (unsigned char)len;
  }
  acc = 0;
  for (i = 0; i < VOCAB; i++) acc += pow((double)(i + 1), -1.1);
  tot = acc;
  acc = 0;
  for (i = 0; i < VOCAB; i++) {
    acc += pow((double)(i + 1), -1.1) / tot;
    g_zipf_cdf[i] = acc;
  }
  g_zipf_cdf[VOCAB - 1] = 1.0;
}

static int zipf_pick(uint64_t *s) {
  double u = u01(s);
  int lo = 0, hi = VOCAB - 1;
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (g_zipf_cdf[mid] < u) lo = mid + 1; else hi = mid;
  }
  return lo;
}

/* Fill out[0..n) with English-like text for stream `seed`. */
void synth_text(uint64_t seed, unsigned char *out, size_t n) {
  static const char *seps[6] = {". ", ", ", "\n", " [[", "]] ", " | "};
  uint64_t s = seed * 0xD1B54A32D192ED03ull + 0x8BB84B93962EACC9ull;
  size_t pos = 0;
  pthread_once(&g_once, build_vocab);
  while (pos < n) {
    char tmp[64];
    int len, k;
    double u = u01(&s);
    if (u < 0.015) {
      len = snprintf(tmp, sizeof tmp, "%u", (unsigned)(sm64(&s) % 100000u));
    } else {
      int w = zipf_pick(&s);
      len = g_wlen[w];
      memcpy(tmp, g_words[w], (size_t)len);
      if (u01(&s) < 0.03) tmp[0] = (char)(tmp[0] - 'a' + 'A');
    }
    if (u01(&s) < 0.08) {
      const char *sp = seps[sm64(&s) % 6];
      size_t sl = strlen(sp);
      memcpy(tmp + len, sp, sl);
      len += (int)sl;
    } else {
      tmp[len++] = ' ';
    }
    for (k = 0; k < len && pos < n; k++) out[pos++] = (unsigned char)tmp[k];
  }
}

void synth_random(uint64_t seed, unsigned char *out, size_t n) {
  uint64_t s = seed ^ 0x5DEECE66Dull;
  size_t i = 0;
  while (i < n) {
    uint64_t v = sm64(&s);
    int k;
    for (k = 0; k < 8 && i < n; k++, v >>= 8) out[i++] = (unsigned char)v;
  }
}

/* Long runs: repeated short periods (exercise max-length overlapping copies). */
void synth_runs(uint64_t seed, unsigned char *out, size_t n) {
  uint64_t s = seed ^ 0x1234567ull;
  size_t i = 0;
  while (i < n) {
    unsigned period = 1 + (unsigned)(sm64(&s) % 7);
    size_t run = 200 + (size_t)(sm64(&s) % 2000);
    unsigned char pat[8];
    unsigned k;
    for (k = 0; k < period; k++) pat[k] = (unsigned char)sm64(&s);
    for (k = 0; run-- > 0 && i < n; k = (k + 1) % period) out[i++] = pat[k];
  }
}

typedef struct {
  int kind;
  uint64_t seed0;
  unsigned char *out;
  size_t stream_len, n, next;
  pthread_mutex_t mu;
} synth_job;

static void *synth_worker(void *arg) {
  synth_job *j = (synth_job *)arg;
  for (;;) {
    size_t i;
    pthread_mutex_lock(&j->mu);
    i = j->next++;
    pthread_mutex_unlock(&j->mu);
    if (i >= j->n) break;
    if (j->kind == 0) synth_text(j->seed0 + i, j->out + i * j->stream_len, j->stream_len);
    else if (j->kind == 1) synth_random(j->seed0 + i, j->out + i * j->stream_len, j->stream_len);
    else synth_runs(j->seed0 + i, j->out + i * j->stream_len, j->stream_len);
  }
  return NULL;
}

/* n streams of stream_len bytes each, stream i seeded seed0 + i. */
void synth_batch(int kind, uint64_t seed0, unsigned char *out, size_t stream_len, size_t n,
                 int threads) {
  synth_job j;
  pthread_t tid[64];
  int t;
  if (threads < 1) threads = 1;
  if (threads > 64) threads = 64;
  j.kind = kind;
  j.seed0 = seed0;
  j.out = out;
  j.stream_len = stream_len;
  j.n = n;
  j.next = 0;
  pthread_mutex_init(&j.mu, NULL);
  pthread_once(&g_once, build_vocab);
  for (t = 0; t < threads; t++) pthread_create(&tid[t], NULL, synth_worker, &j);
  for (t = 0; t < threads; t++) pthread_join(tid[t], NULL);
  pthread_mutex_destroy(&j.mu);
}
