/*
 * lzma2_walker.c -- TEST INFRASTRUCTURE (tests/test_c_host.py).
 *
 * Drives the REFERENCE's own LZMA2 chunk walker (Lzma2Dec.c, compiled in place
 * by oracle/Makefile.ref, its own LzmaDec.h / Types.h on the include path) on
 * top of liblzmagpu.so's LzmaDec_* -- the build a user of the reference gets
 * when they keep Lzma2Dec.c and link this library for the LZMA decoder.  The
 * walker writes stored chunks into CLzmaDec.dic itself and advances
 * dicPos / processedPos (Lzma2Dec.c:159-166) between the GPU decoder's calls,
 * so later LZMA chunks that match into stored bytes read what the host wrote:
 * the device mirror of the dictionary must notice (dropin_capi.hip).
 *
 *   lzma2_walker PROP STREAM_FILE OUT_SIZE IN_CHUNK DIC_CHUNK [OUT_CHUNK]
 *
 * 7zDec.c:181-202 (SzDecodeLzma2) shape: dic = the whole output buffer,
 * dicLimit advanced DIC_CHUNK bytes at a time (0: the whole output), input fed
 * IN_CHUNK bytes at a time.  Prints: res status dicPos inPos crc32 calls.
 * OUT_CHUNK > 0 (round 5): the XzDec shape instead -- the
 * decoder's own ring (Lzma2Dec_Allocate: dicBufSize = the dictionary size),
 * Lzma2Dec_DecodeToBuf into the output OUT_CHUNK bytes at a time; stored
 * chunks reach the ring in pieces on either side of its end (the walker wraps
 * dicPos to 0 between the GPU decoder's calls).  Prints the output position
 * in place of dicPos.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "Lzma2Dec.h"

static void *SzAlloc(void *p, size_t size) { (void)p; return malloc(size ? size : 1); }
static void SzFree(void *p, void *address) { (void)p; free(address); }
static ISzAlloc g_Alloc = {SzAlloc, SzFree};

static unsigned crc32_of(const unsigned char *p, size_t n) {
  unsigned c = 0xFFFFFFFFu;
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

int main(int argc, char **argv) {
  size_t ns = 0, out_size, in_chunk, dic_chunk, in_pos = 0, calls = 0;
  unsigned char *src, *out;
  unsigned prop;
  CLzma2Dec dec;
  SRes r;
  ELzmaStatus st = LZMA_STATUS_NOT_SPECIFIED;
  size_t out_chunk = 0, out_pos = 0;
  if (argc != 6 && argc != 7) {
    fprintf(stderr, "usage: %s PROP STREAM OUT_SIZE IN_CHUNK DIC_CHUNK [OUT_CHUNK]\n", argv[0]);
    return 2;
  }
  if (argc == 7) out_chunk = (size_t)strtoull(argv[6], NULL, 10);
  prop = (unsigned)strtoul(argv[1], NULL, 10);
  src = read_file(argv[2], &ns);
  out_size = (size_t)strtoull(argv[3], NULL, 10);
  in_chunk = (size_t)strtoull(argv[4], NULL, 10);
  dic_chunk = (size_t)strtoull(argv[5], NULL, 10);
  if (!src) return 2;
  out = (unsigned char *)malloc(out_size ? out_size : 1);
  memset(out, 0, out_size);
  Lzma2Dec_Construct(&dec);
  if (out_chunk) {
    r = Lzma2Dec_Allocate(&dec, (Byte)prop, &g_Alloc);
    if (r == SZ_OK) {
      Lzma2Dec_Init(&dec);
      for (;;) {
        SizeT sl = ns - in_pos, dl = out_size - out_pos;
        ELzmaFinishMode fin = LZMA_FINISH_END;
        if (sl > in_chunk) sl = in_chunk;
        if (dl > out_chunk) {
          dl = out_chunk;
          fin = LZMA_FINISH_ANY;
        }
        r = Lzma2Dec_DecodeToBuf(&dec, out + out_pos, &dl, src + in_pos, &sl, fin, &st);
        calls++;
        in_pos += sl;
        out_pos += dl;
        if (r != SZ_OK || st == LZMA_STATUS_FINISHED_WITH_MARK || (sl == 0 && dl == 0)) break;
      }
      Lzma2Dec_Free(&dec, &g_Alloc);
    }
    printf("%d %d %zu %zu %08x %zu\n", (int)r, (int)st, out_pos, in_pos, crc32_of(out, out_pos),
           calls);
    free(out);
    free(src);
    return 0;
  }
  r = Lzma2Dec_AllocateProbs(&dec, (Byte)prop, &g_Alloc);
  if (r == SZ_OK) {
    dec.decoder.dic = out;
    dec.decoder.dicBufSize = out_size;
    Lzma2Dec_Init(&dec);
    for (;;) {
      SizeT sl = ns - in_pos, pos0 = dec.decoder.dicPos, lim = out_size;
      ELzmaFinishMode fin = LZMA_FINISH_END;
      if (sl > in_chunk) sl = in_chunk;
      if (dic_chunk && out_size - pos0 > dic_chunk) {
        lim = pos0 + dic_chunk;
        fin = LZMA_FINISH_ANY;
      }
      r = Lzma2Dec_DecodeToDic(&dec, lim, src + in_pos, &sl, fin, &st);
      calls++;
      in_pos += sl;
      if (r != SZ_OK || st == LZMA_STATUS_FINISHED_WITH_MARK ||
          (sl == 0 && dec.decoder.dicPos == pos0))
        break;
    }
    Lzma2Dec_FreeProbs(&dec, &g_Alloc);
  }
  printf("%d %d %zu %zu %08x %zu\n", (int)r, (int)st, (size_t)dec.decoder.dicPos, in_pos,
         crc32_of(out, dec.decoder.dicPos), calls);
  free(out);
  free(src);
  return 0;
}
