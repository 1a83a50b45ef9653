/*
 * lzma_c_threads.c -- TEST / BENCH INFRASTRUCTURE: an unchanged multi-threaded
 * caller of the reference's one-call API.  THREADS pthreads each decode their
 * share of a stream set with LzmaDecode (LzmaDec.h:223-225, reentrant:
 * LzmaDec.c:972-1002), REPEAT times.  The same source is linked two ways:
 *   tests/c_host/build/lzma_c_threads  -> liblzmagpu.so (concurrent calls are
 *                                         coalesced into batch launches)
 *   oracle/_ref/lzma_c_threads_ref     -> the reference's LzmaDec.c compiled
 *                                         in place (oracle/Makefile.ref): the
 *                                         CPU baseline on the same host cores
 *
 *   lzma_c_threads THREADS SRC LENS PROPS OUT_SIZES REPEAT [MODE]
 * SRC: streams back to back; LENS / OUT_SIZES: uint64 per stream; PROPS: 5
 * bytes per stream.  MODE "one" (default): one LzmaDecode per stream; "buf":
 * the fork's zlib-like streaming shape per stream (LzmaDec_Allocate + Init,
 * then LzmaDec_DecodeToBuf with 1 KiB of input and 1 KiB of output per call,
 * 7zDec.c:567-648) -- each thread its own decoder, so concurrent calls run on
 * different CLzmaDec objects.  Prints one JSON line on STDERR (the fork's reference
 * decoder prints a debug line to stdout per call, LzmaDec.c:945): threads,
 * streams, decoded bytes, seconds, MB/s, failures, and the XOR of every
 * stream's (index-salted) CRC-32 so the two builds can be compared.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "lzma_gpu.h"

/* present when linked to liblzmagpu.so (the coalescer's batch counts), absent
 * in the reference build */
extern void LzmaGpu_CoalesceStats(uint64_t *batches, uint64_t *calls, uint64_t *max_batch,
                                  int reset) __attribute__((weak));
extern void LzmaGpu_CoalesceTimes(uint64_t *ns, uint64_t *batches, int reset)
    __attribute__((weak));

static void *SzAlloc(void *p, size_t size) { (void)p; return malloc(size ? size : 1); }
static void SzFree(void *p, void *address) { (void)p; free(address); }
static ISzAlloc g_Alloc = {SzAlloc, SzFree};

static unsigned crc32_of(const unsigned char *p, size_t n, unsigned salt) {
  unsigned c = 0xFFFFFFFFu ^ salt;
  size_t i;
  int k;
  for (i = 0; i < n; ++i) {
    c ^= p[i];
    for (k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
  }
  return c ^ 0xFFFFFFFFu;
}

static unsigned char *read_file(const char *path, size_t *n) {
  FILE *f = fopen(path, "rb");
  unsigned char *b;
  long sz;
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  b = (unsigned char *)malloc(sz > 0 ? (size_t)sz : 1);
  *n = fread(b, 1, (size_t)sz, f) == (size_t)sz ? (size_t)sz : 0;
  fclose(f);
  return b;
}

typedef struct {
  int tid, nthreads, repeat, buf_mode;
  size_t n;
  const unsigned char *src, *props;
  const uint64_t *off, *len, *out;
  uint64_t bytes, fails;
  unsigned crc;
} Work;

static void *worker(void *arg) {
  Work *w = (Work *)arg;
  size_t i, cap = 0;
  int r;
  unsigned char *buf = NULL;
  for (i = (size_t)w->tid; i < w->n; i += (size_t)w->nthreads)
    if (w->out[i] > cap) cap = w->out[i];
  buf = (unsigned char *)malloc(cap ? cap : 1);
  for (r = 0; r < w->repeat; ++r)
    for (i = (size_t)w->tid; i < w->n; i += (size_t)w->nthreads) {
      SizeT dl = w->out[i], sl = w->len[i];
      ELzmaStatus st;
      SRes res;
      if (!w->buf_mode) {
        res = LzmaDecode(buf, &dl, w->src + w->off[i], &sl, w->props + 5 * i, 5,
                         LZMA_FINISH_ANY, &st, &g_Alloc);
      } else {
        CLzmaDec dec;
        size_t ip = 0, op = 0;
        LzmaDec_Construct(&dec);
        res = LzmaDec_Allocate(&dec, w->props + 5 * i, 5, &g_Alloc);
        if (res == SZ_OK) {
          LzmaDec_Init(&dec);
          for (;;) {
            SizeT s1 = w->len[i] - ip, d1 = w->out[i] - op;
            if (s1 > 1024) s1 = 1024;
            if (d1 > 1024) d1 = 1024;
            res = LzmaDec_DecodeToBuf(&dec, buf + op, &d1, w->src + w->off[i] + ip, &s1,
                                      LZMA_FINISH_ANY, &st);
            ip += s1;
            op += d1;
            if (res != SZ_OK || st == LZMA_STATUS_FINISHED_WITH_MARK || op == w->out[i] ||
                (s1 == 0 && d1 == 0))
              break;
          }
          LzmaDec_Free(&dec, &g_Alloc);
        }
        dl = op;
      }
      if (res != SZ_OK || dl != w->out[i]) w->fails++;
      w->bytes += dl;
      if (r == 0) w->crc ^= crc32_of(buf, dl, (unsigned)i);
    }
  free(buf);
  return NULL;
}

int main(int argc, char **argv) {
  size_t ns = 0, nl = 0, np = 0, no = 0, n, i;
  int T, repeat, t;
  unsigned char *src, *props;
  uint64_t *len, *out, *off, bytes = 0, fails = 0;
  unsigned crc = 0;
  pthread_t *th;
  pthread_attr_t attr;
  Work *w;
  struct timespec a, b;
  double sec;
  if (argc != 7 && argc != 8) {
    fprintf(stderr, "usage: %s THREADS SRC LENS PROPS OUT_SIZES REPEAT [one|buf]\n", argv[0]);
    return 2;
  }
  T = atoi(argv[1]);
  repeat = atoi(argv[6]);
  src = read_file(argv[2], &ns);
  len = (uint64_t *)read_file(argv[3], &nl);
  props = read_file(argv[4], &np);
  out = (uint64_t *)read_file(argv[5], &no);
  if (!src || !len || !props || !out || T < 1 || repeat < 1) return 2;
  n = nl / 8;
  if (no / 8 != n || np != 5 * n) return 2;
  off = (uint64_t *)malloc((n ? n : 1) * 8);
  for (i = 0; i < n; ++i) off[i] = i ? off[i - 1] + len[i - 1] : 0;
  th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)T);
  w = (Work *)calloc((size_t)T, sizeof(Work));
  pthread_attr_init(&attr);
  pthread_attr_setstacksize(&attr, 256 * 1024);
  for (t = 0; t < T; ++t) {
    w[t].tid = t;
    w[t].nthreads = T;
    w[t].repeat = repeat;
    w[t].buf_mode = argc == 8 && strcmp(argv[7], "buf") == 0;
    w[t].n = n;
    w[t].src = src;
    w[t].props = props;
    w[t].off = off;
    w[t].len = len;
    w[t].out = out;
  }
  clock_gettime(CLOCK_MONOTONIC, &a);
  for (t = 0; t < T; ++t)
    if (pthread_create(&th[t], &attr, worker, &w[t]) != 0) return 3;
  for (t = 0; t < T; ++t) pthread_join(th[t], NULL);
  clock_gettime(CLOCK_MONOTONIC, &b);
  sec = (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
  for (t = 0; t < T; ++t) {
    bytes += w[t].bytes;
    fails += w[t].fails;
    crc ^= w[t].crc;
  }
  {
    uint64_t nb = 0, nc = 0, mx = 0, tns[8] = {0}, tb = 0;
    char ph[256] = "null";
    if (LzmaGpu_CoalesceStats) LzmaGpu_CoalesceStats(&nb, &nc, &mx, 0);
    if (LzmaGpu_CoalesceTimes) {
      /* host microseconds per one-call batch by phase (plan, stage, upload,
       * launch, wait, download, batch, call) */
      int k;
      size_t o = 0;
      LzmaGpu_CoalesceTimes(tns, &tb, 0);
      o += (size_t)snprintf(ph + o, sizeof ph - o, "[");
      for (k = 0; k < 8; ++k)
        o += (size_t)snprintf(ph + o, sizeof ph - o, "%s%.1f", k ? ", " : "",
                              tb ? (double)tns[k] / 1e3 / (double)(k == 7 && nc ? nc : tb) : 0.0);
      snprintf(ph + o, sizeof ph - o, "]");
    }
    fprintf(stderr,
            "{\"mode\": \"%s\", \"threads\": %d, \"streams\": %zu, \"repeat\": %d, \"bytes\": %llu, "
            "\"seconds\": %.6f, \"MBps\": %.2f, \"fails\": %llu, \"crc_xor\": \"%08x\", "
            "\"phase_us\": %s, "
            "\"batches\": %llu, \"batched_calls\": %llu, \"max_batch\": %llu}\n",
            (argc == 8 && strcmp(argv[7], "buf") == 0) ? "buf" : "one", T, n, repeat,
            (unsigned long long)bytes, sec, sec > 0 ? (double)bytes / sec / 1e6 : 0.0,
            (unsigned long long)fails, crc, ph, (unsigned long long)nb, (unsigned long long)nc,
            (unsigned long long)mx);
  }
  return 0;
}
