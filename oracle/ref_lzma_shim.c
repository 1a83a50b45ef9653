/*
 * ref_lzma_shim.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Thin ctypes-friendly wrapper around the *reference* LZMA SDK 9.20 LZMA
 * sources (LzmaDec.c Lzma2Dec.c LzmaEnc.c LzFind.c Lzma2Enc.c Alloc.c),
 * compiled in place from /root/reference by oracle/Makefile.ref into
 * oracle/_ref/libref_lzma.so -- the library that PINS the LZMA oracle.  It is
 * built with no stand-in of any kind (no -D defines beyond the encoder's
 * single-thread switch -D_7ZIP_ST, linked with -z defs: every symbol
 * resolved, nothing left to lazy binding).  The container code (7z / xz
 * readers, filters, CRCs) is in ref_shim.c -> oracle/_ref/libref.so.
 *
 * Used by tests/golden/make_golden*.py to (a) encode fixture streams with the
 * reference encoder and (b) record the reference decoder's exact
 * {res, status, destLen, srcLen} and output for every golden case, and by
 * bench.py's cpu_baseline leg (ref_lzma_decode_batch: the reference's own
 * LzmaDecode over a batch on host threads, "kind": "reference").
 *
 * Nothing in the product (lzma-sdk-zliblike_amd/) links or loads this.
 *
 * Reference interfaces driven here:
 *   LzmaEncode          LzmaEnc.h:72-74 / LzmaEnc.c:2248
 *   LzmaDecode          LzmaDec.h:223-225 / LzmaDec.c:972
 *   LzmaDec_Allocate + LzmaDec_DecodeToBuf   LzmaDec.c:950, 840
 *   LzmaDec_AllocateProbs + LzmaDec_DecodeToDic over a whole-output dic
 *                       LzmaDec.c:938, 719 (the 7zDec.c:127-171 pattern)
 *   Lzma2Enc_*          Lzma2Enc.h (single-threaded, -D_7ZIP_ST)
 *   Lzma2Dec_AllocateProbs + Lzma2Dec_Init + Lzma2Dec_DecodeToDic
 *                       Lzma2Dec.c:73,90,170 (the 7zDec.c:181-202 pattern;
 *                       Lzma2Decode one-call never calls Lzma2Dec_Init)
 *
 * The fork's printf in LzmaDec_AllocateProbs (LzmaDec.c:945) is silenced by
 * pointing fd 1 at /dev/null around each decoder call.
 */
#include <fcntl.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "Alloc.h"
#include "Lzma2Dec.h"
#include "Lzma2Enc.h"
#include "LzmaDec.h"
#include "LzmaEnc.h"

static void *shim_alloc(void *p, size_t n) { (void)p; return malloc(n ? n : 1); }
static void shim_free(void *p, void *a) { (void)p; free(a); }
static ISzAlloc g_shim_alloc = {shim_alloc, shim_free};

static int quiet_begin(void) {
  int saved, devnull;
  fflush(stdout);
  saved = dup(1);
  devnull = open("/dev/null", O_WRONLY);
  if (devnull >= 0) { dup2(devnull, 1); close(devnull); }
  return saved;
}

static void quiet_end(int saved) {
  fflush(stdout);
  if (saved >= 0) { dup2(saved, 1); close(saved); }
}

/* LzmaEncode with explicit lc/lp/pb/dict/level; props5 receives the 5-byte header. */
int ref_lzma_encode(unsigned char *dst, size_t *dst_len, const unsigned char *src,
                    size_t src_len, int level, unsigned dict_size, int lc, int lp,
                    int pb, int fb, int write_end_mark, unsigned char *props5) {
  CLzmaEncProps props;
  SizeT props_size = LZMA_PROPS_SIZE;
  SizeT dl = *dst_len;
  SRes res;
  LzmaEncProps_Init(&props);
  props.level = level;
  props.dictSize = dict_size;
  props.lc = lc;
  props.lp = lp;
  props.pb = pb;
  props.fb = fb;
  props.numThreads = 1;
  res = LzmaEncode(dst, &dl, src, src_len, &props, props5, &props_size,
                   write_end_mark, NULL, &g_shim_alloc, &g_shim_alloc);
  *dst_len = dl;
  return res;
}

/* LzmaDecode one-call.  *status is preset to -1 so "untouched" is visible. */
int ref_lzma_decode(unsigned char *dst, size_t *dst_len, const unsigned char *src,
                    size_t *src_len, const unsigned char *props, unsigned props_size,
                    int finish_mode, int *status) {
  ELzmaStatus st = (ELzmaStatus)-1;
  SizeT dl = *dst_len, sl = *src_len;
  int saved = quiet_begin();
  SRes res = LzmaDecode(dst, &dl, src, &sl, props, props_size,
                        (ELzmaFinishMode)finish_mode, &st, &g_shim_alloc);
  quiet_end(saved);
  *dst_len = dl;
  *src_len = sl;
  *status = (int)st;
  return res;
}

/*
 * zlib-like streaming decode through LzmaDec_DecodeToBuf, in the shape of the
 * fork's SzDecodeLzmaToFileWithBuf loop (7zDec.c:567-648): the input is fed in
 * chunks of at most in_chunk bytes, each call offers an output window of at
 * most out_chunk bytes (bounded by the remaining out_total), finish_mode is
 * passed on every call.  Per-call results are recorded into trace[] as
 * {res, status, srcLen, destLen} quadruples (at most max_calls).
 * Returns the number of calls made; *out_len / *in_used get the totals.
 */
int ref_lzma_stream_decode(const unsigned char *props, const unsigned char *src,
                           size_t src_total, unsigned char *out, size_t out_total,
                           size_t in_chunk, size_t out_chunk, int finish_mode,
                           long long *trace, int max_calls, size_t *out_len,
                           size_t *in_used) {
  CLzmaDec dec;
  size_t in_pos = 0, out_pos = 0;
  int calls = 0;
  int saved = quiet_begin();
  SRes ares;
  LzmaDec_Construct(&dec);
  ares = LzmaDec_Allocate(&dec, props, LZMA_PROPS_SIZE, &g_shim_alloc);
  quiet_end(saved);
  if (ares != SZ_OK) { *out_len = 0; *in_used = 0; return -(int)ares; }
  LzmaDec_Init(&dec);
  while (calls < max_calls) {
    SizeT sl = src_total - in_pos;
    SizeT dl = out_total - out_pos;
    ELzmaStatus st = (ELzmaStatus)-1;
    SRes res;
    if (sl > in_chunk) sl = in_chunk;
    if (dl > out_chunk) dl = out_chunk;
    res = LzmaDec_DecodeToBuf(&dec, out + out_pos, &dl, src + in_pos, &sl,
                              (ELzmaFinishMode)finish_mode, &st);
    trace[4 * calls + 0] = res;
    trace[4 * calls + 1] = (int)st;
    trace[4 * calls + 2] = (long long)sl;
    trace[4 * calls + 3] = (long long)dl;
    calls++;
    in_pos += sl;
    out_pos += dl;
    if (res != SZ_OK) break;
    if (st == LZMA_STATUS_FINISHED_WITH_MARK) break;
    if (out_pos == out_total) break;
    if (sl == 0 && dl == 0) break;
  }
  LzmaDec_Free(&dec, &g_shim_alloc);
  *out_len = out_pos;
  *in_used = in_pos;
  return calls;
}

typedef struct { ISeqInStream s; const unsigned char *p; size_t left; } ShimMemIn;
typedef struct { ISeqOutStream s; unsigned char *p; size_t cap, pos; int overflow; } ShimMemOut;

static SRes shim_mem_read(void *pp, void *buf, size_t *size) {
  ShimMemIn *in = (ShimMemIn *)pp;
  size_t n = *size < in->left ? *size : in->left;
  memcpy(buf, in->p, n);
  in->p += n;
  in->left -= n;
  *size = n;
  return SZ_OK;
}

static size_t shim_mem_write(void *pp, const void *buf, size_t size) {
  ShimMemOut *out = (ShimMemOut *)pp;
  if (out->pos + size > out->cap) { out->overflow = 1; return 0; }
  memcpy(out->p + out->pos, buf, size);
  out->pos += size;
  return size;
}

/* Single-threaded LZMA2 encode (Lzma2Enc.c built with -D_7ZIP_ST).
 * block_size > 0 makes the encoder emit a dictionary reset every block_size
 * input bytes (Lzma2Enc.c:310-361 block layout). */
int ref_lzma2_encode(unsigned char *dst, size_t *dst_len, const unsigned char *src,
                     size_t src_len, int level, unsigned dict_size, int lc, int lp,
                     int pb, size_t block_size, unsigned char *prop_byte) {
  CLzma2EncHandle enc = Lzma2Enc_Create(&g_shim_alloc, &g_shim_alloc);
  CLzma2EncProps props;
  ShimMemIn in;
  ShimMemOut out;
  SRes res;
  if (!enc) return SZ_ERROR_MEM;
  Lzma2EncProps_Init(&props);
  props.lzmaProps.level = level;
  props.lzmaProps.dictSize = dict_size;
  props.lzmaProps.lc = lc;
  props.lzmaProps.lp = lp;
  props.lzmaProps.pb = pb;
  props.lzmaProps.numThreads = 1;
  props.numBlockThreads = 1;
  props.numTotalThreads = 1;
  props.blockSize = block_size;
  res = Lzma2Enc_SetProps(enc, &props);
  if (res == SZ_OK) {
    *prop_byte = Lzma2Enc_WriteProperties(enc);
    in.s.Read = shim_mem_read;
    in.p = src;
    in.left = src_len;
    out.s.Write = shim_mem_write;
    out.p = dst;
    out.cap = *dst_len;
    out.pos = 0;
    out.overflow = 0;
    res = Lzma2Enc_Encode(enc, &out.s, &in.s, NULL);
    *dst_len = out.pos;
    if (res == SZ_OK && out.overflow) res = SZ_ERROR_OUTPUT_EOF;
  }
  Lzma2Enc_Destroy(enc);
  return res;
}

/*
 * LZMA2 decode with the dictionary == caller's output buffer.  Mirrors the
 * 7zDec.c:181-202 usage: AllocateProbs, set dic/dicBufSize, Lzma2Dec_Init,
 * one Lzma2Dec_DecodeToDic over the whole input.
 */
int ref_lzma2_decode(unsigned char *dst, size_t *dst_len, const unsigned char *src,
                     size_t *src_len, unsigned char prop, int finish_mode, int *status) {
  CLzma2Dec dec;
  ELzmaStatus st = (ELzmaStatus)-1;
  SizeT sl = *src_len;
  SRes res;
  int saved;
  Lzma2Dec_Construct(&dec);
  saved = quiet_begin();
  res = Lzma2Dec_AllocateProbs(&dec, prop, &g_shim_alloc);
  quiet_end(saved);
  if (res != SZ_OK) { *dst_len = 0; *src_len = 0; *status = -1; return res; }
  dec.decoder.dic = dst;
  dec.decoder.dicBufSize = *dst_len;
  Lzma2Dec_Init(&dec);
  res = Lzma2Dec_DecodeToDic(&dec, *dst_len, src, &sl, (ELzmaFinishMode)finish_mode, &st);
  *dst_len = dec.decoder.dicPos;
  *src_len = sl;
  *status = (int)st;
  Lzma2Dec_FreeProbs(&dec, &g_shim_alloc);
  return res;
}

/*
 * CPU baseline: the reference LzmaDecode (LzmaDec.c:972) over n streams on
 * `threads` host threads, 16 streams per work grab.  Streams i: src + src_off[i]
 * (src_len[i] bytes), props5 + 5 i, output dst + dst_off[i] (dst_cap[i] bytes).
 * The fork prints a line from LzmaDec_AllocateProbs (LzmaDec.c:945) on every
 * call: fd 1 points at /dev/null for the whole batch (the printf cost stays in
 * the timing -- it is the reference's own).  Returns the number of streams
 * whose result was not SZ_OK; res_out / dest_len_out may be NULL.
 */
typedef struct {
  const unsigned char *src, *props5;
  const uint64_t *src_off, *src_len, *dst_off, *dst_cap;
  unsigned char *dst;
  int fin;
  int32_t *res_out;
  uint64_t *dest_len_out;
  size_t n, next;
  pthread_mutex_t mu;
  int errors;
} ref_batch;

static void *ref_batch_worker(void *arg) {
  ref_batch *b = (ref_batch *)arg;
  int errs = 0;
  for (;;) {
    size_t i, end, k;
    pthread_mutex_lock(&b->mu);
    i = b->next;
    end = i + 16 < b->n ? i + 16 : b->n;
    b->next = end;
    pthread_mutex_unlock(&b->mu);
    if (i >= b->n) break;
    for (k = i; k < end; k++) {
      SizeT dl = (SizeT)b->dst_cap[k], sl = (SizeT)b->src_len[k];
      ELzmaStatus st;
      SRes r = LzmaDecode(b->dst + b->dst_off[k], &dl, b->src + b->src_off[k], &sl,
                          b->props5 + 5 * k, LZMA_PROPS_SIZE, (ELzmaFinishMode)b->fin, &st,
                          &g_shim_alloc);
      if (b->res_out) b->res_out[k] = r;
      if (b->dest_len_out) b->dest_len_out[k] = dl;
      if (r != SZ_OK) errs++;
    }
  }
  pthread_mutex_lock(&b->mu);
  b->errors += errs;
  pthread_mutex_unlock(&b->mu);
  return NULL;
}

int ref_lzma_decode_batch(const unsigned char *src, const uint64_t *src_off,
                          const uint64_t *src_len, const unsigned char *props5,
                          unsigned char *dst, const uint64_t *dst_off, const uint64_t *dst_cap,
                          int finish_mode, int32_t *res_out, uint64_t *dest_len_out, size_t n,
                          int threads) {
  ref_batch b;
  pthread_t tid[256];
  int t, saved;
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  b.src = src;
  b.src_off = src_off;
  b.src_len = src_len;
  b.props5 = props5;
  b.dst = dst;
  b.dst_off = dst_off;
  b.dst_cap = dst_cap;
  b.fin = finish_mode;
  b.res_out = res_out;
  b.dest_len_out = dest_len_out;
  b.n = n;
  b.next = 0;
  b.errors = 0;
  pthread_mutex_init(&b.mu, NULL);
  saved = quiet_begin();
  if (threads == 1) {
    ref_batch_worker(&b);
  } else {
    for (t = 0; t < threads; t++) pthread_create(&tid[t], NULL, ref_batch_worker, &b);
    for (t = 0; t < threads; t++) pthread_join(tid[t], NULL);
  }
  quiet_end(saved);
  pthread_mutex_destroy(&b.mu);
  return b.errors;
}

/*
 * CPU baseline for LZMA2 blocks (config 4): the 7zDec.c:181-202 pattern --
 * Lzma2Dec_AllocateProbs + Lzma2Dec_Init + Lzma2Dec_DecodeToDic over a flat
 * dictionary -- per block on `threads` host threads; fd 1 at /dev/null for the
 * whole batch (the per-call redirect of ref_lzma2_decode is not thread-safe).
 */
typedef struct {
  const unsigned char *src;
  const uint64_t *src_off, *src_len, *dst_off, *dst_cap;
  unsigned char *dst;
  unsigned char prop;
  int fin;
  int32_t *res_out;
  uint64_t *dest_len_out;
  size_t n, next;
  pthread_mutex_t mu;
  int errors;
} ref2_batch;

static void *ref2_batch_worker(void *arg) {
  ref2_batch *b = (ref2_batch *)arg;
  int errs = 0;
  /* one decoder per thread, its probabilities allocated once (the same prop
     for every block), re-initialised per block as 7zDec.c does per folder */
  CLzma2Dec dec;
  SRes ar;
  Lzma2Dec_Construct(&dec);
  ar = Lzma2Dec_AllocateProbs(&dec, b->prop, &g_shim_alloc);
  for (;;) {
    size_t k;
    pthread_mutex_lock(&b->mu);
    k = b->next++;
    pthread_mutex_unlock(&b->mu);
    if (k >= b->n) break;
    {
      ELzmaStatus st;
      SizeT sl = (SizeT)b->src_len[k];
      SRes r = ar;
      if (r == SZ_OK) {
        dec.decoder.dic = b->dst + b->dst_off[k];
        dec.decoder.dicBufSize = (SizeT)b->dst_cap[k];
        Lzma2Dec_Init(&dec);
        r = Lzma2Dec_DecodeToDic(&dec, (SizeT)b->dst_cap[k], b->src + b->src_off[k], &sl,
                                 (ELzmaFinishMode)b->fin, &st);
        if (b->dest_len_out) b->dest_len_out[k] = dec.decoder.dicPos;
      }
      if (b->res_out) b->res_out[k] = r;
      if (r != SZ_OK) errs++;
    }
  }
  Lzma2Dec_FreeProbs(&dec, &g_shim_alloc);
  pthread_mutex_lock(&b->mu);
  b->errors += errs;
  pthread_mutex_unlock(&b->mu);
  return NULL;
}

int ref_lzma2_decode_batch(const unsigned char *src, const uint64_t *src_off,
                           const uint64_t *src_len, unsigned char prop, unsigned char *dst,
                           const uint64_t *dst_off, const uint64_t *dst_cap, int finish_mode,
                           int32_t *res_out, uint64_t *dest_len_out, size_t n, int threads) {
  ref2_batch b;
  pthread_t tid[256];
  int t, saved;
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  b.src = src;
  b.src_off = src_off;
  b.src_len = src_len;
  b.prop = prop;
  b.dst = dst;
  b.dst_off = dst_off;
  b.dst_cap = dst_cap;
  b.fin = finish_mode;
  b.res_out = res_out;
  b.dest_len_out = dest_len_out;
  b.n = n;
  b.next = 0;
  b.errors = 0;
  pthread_mutex_init(&b.mu, NULL);
  saved = quiet_begin();
  if (threads == 1) {
    ref2_batch_worker(&b);
  } else {
    for (t = 0; t < threads; t++) pthread_create(&tid[t], NULL, ref2_batch_worker, &b);
    for (t = 0; t < threads; t++) pthread_join(tid[t], NULL);
  }
  quiet_end(saved);
  pthread_mutex_destroy(&b.mu);
  return b.errors;
}

/*
 * The 7zDec.c:127-171 (SzDecodeLzma) pattern: LzmaDec_AllocateProbs, dic = the
 * caller's whole output buffer (dicBufSize = out_total), LzmaDec_Init, then
 * LzmaDec_DecodeToDic(out_total, FINISH_END) over look windows of at most `win`
 * input bytes, each window starting where the previous call stopped reading.
 * Stops on an error, when the dictionary is full, or when a call neither reads
 * nor writes.  Per-call {res, status, srcLen, dicPos} into trace[] (at most
 * max_calls).  Returns the number of calls; *out_len = dicPos, *in_used.
 * *elapsed_ns (optional): wall time of the decode calls alone.
 */
#include <time.h>
int ref_lzma_dic_decode(const unsigned char *props, const unsigned char *src, size_t src_total,
                        unsigned char *out, size_t out_total, size_t win, long long *trace,
                        int max_calls, size_t *out_len, size_t *in_used,
                        long long *elapsed_ns) {
  CLzmaDec dec;
  size_t in_pos = 0;
  int calls = 0;
  struct timespec t0, t1;
  long long ns = 0;
  int saved = quiet_begin();
  SRes ares;
  LzmaDec_Construct(&dec);
  ares = LzmaDec_AllocateProbs(&dec, props, LZMA_PROPS_SIZE, &g_shim_alloc);
  if (ares != SZ_OK) { quiet_end(saved); *out_len = 0; *in_used = 0; return -(int)ares; }
  dec.dic = out;
  dec.dicBufSize = out_total;
  LzmaDec_Init(&dec);
  while (calls < max_calls) {
    SizeT sl = src_total - in_pos, pos0 = dec.dicPos;
    ELzmaStatus st = (ELzmaStatus)-1;
    SRes res;
    if (sl > win) sl = win;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    res = LzmaDec_DecodeToDic(&dec, out_total, src + in_pos, &sl, LZMA_FINISH_END, &st);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    ns += (long long)(t1.tv_sec - t0.tv_sec) * 1000000000LL + (t1.tv_nsec - t0.tv_nsec);
    if (trace) {
      trace[4 * calls + 0] = res;
      trace[4 * calls + 1] = (int)st;
      trace[4 * calls + 2] = (long long)sl;
      trace[4 * calls + 3] = (long long)dec.dicPos;
    }
    calls++;
    in_pos += sl;
    if (res != SZ_OK) break;
    if (dec.dicPos == dec.dicBufSize || (sl == 0 && dec.dicPos == pos0)) break;
  }
  LzmaDec_FreeProbs(&dec, &g_shim_alloc);
  quiet_end(saved);
  *out_len = dec.dicPos;
  *in_used = in_pos;
  if (elapsed_ns) *elapsed_ns = ns;
  return calls;
}
