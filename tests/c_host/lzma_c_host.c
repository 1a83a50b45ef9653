/*
 * lzma_c_host.c -- a C program written against the LZMA SDK's own decode API
 * (LzmaLib.h LzmaUncompress, LzmaDec.h LzmaDecode / LzmaDec_Allocate +
 * LzmaDec_Init + LzmaDec_DecodeToBuf, 7zCrc.h CrcGenerateTable / CrcCalc),
 * the way a user of the reference calls it -- compiled against
 * include/lzma_gpu.h and linked to liblzmagpu.so instead of LzmaDec.c.
 * TEST INFRASTRUCTURE: tests/test_c_host.py builds and runs it.
 *
 *   lzma_c_host PROPS_FILE STREAM_FILE OUT_SIZE IN_CHUNK OUT_CHUNK
 *
 * One line per API: name res status destLen srcLen crc32(output) [calls].
 * LzmaDec_DecodeToDic drives the 7zDec.c:127-171 loop (dic = the whole
 * output, look windows of IN_CHUNK input bytes, FINISH_END).
 * The streaming loop is the fork's SzDecodeLzmaToFileWithBuf shape
 * (7zDec.c:567-648): input fed IN_CHUNK bytes at a time, output windows of
 * OUT_CHUNK bytes, FINISH_ANY, until the output total or the end mark.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "lzma_gpu.h"

static void *SzAlloc(void *p, size_t size) { (void)p; return malloc(size ? size : 1); }
static void SzFree(void *p, void *address) { (void)p; free(address); }
static ISzAlloc g_Alloc = {SzAlloc, SzFree};

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
  size_t np = 0, ns = 0, out_size, in_chunk, out_chunk;
  unsigned char *props, *src, *out;
  if (argc != 6) {
    fprintf(stderr, "usage: %s PROPS STREAM OUT_SIZE IN_CHUNK OUT_CHUNK\n", argv[0]);
    return 2;
  }
  props = read_file(argv[1], &np);
  src = read_file(argv[2], &ns);
  out_size = (size_t)strtoull(argv[3], NULL, 10);
  in_chunk = (size_t)strtoull(argv[4], NULL, 10);
  out_chunk = (size_t)strtoull(argv[5], NULL, 10);
  if (!props || np != LZMA_PROPS_SIZE || !src) return 2;
  out = (unsigned char *)malloc(out_size ? out_size : 1);
  CrcGenerateTable();

  { /* LzmaLib.h: one call, FINISH_ANY */
    size_t dl = out_size, sl = ns;
    int r = LzmaUncompress(out, &dl, src, &sl, props, LZMA_PROPS_SIZE);
    printf("LzmaUncompress %d - %zu %zu %08x\n", r, dl, sl, (unsigned)CrcCalc(out, dl));
  }
  { /* LzmaDec.h: one call, FINISH_END */
    SizeT dl = out_size, sl = ns;
    ELzmaStatus st;
    SRes r;
    memset(out, 0, out_size);
    r = LzmaDecode(out, &dl, src, &sl, props, LZMA_PROPS_SIZE, LZMA_FINISH_END, &st, &g_Alloc);
    printf("LzmaDecode %d %d %zu %zu %08x\n", (int)r, (int)st, (size_t)dl, (size_t)sl,
           (unsigned)CrcCalc(out, dl));
  }
  { /* LzmaDec.h: zlib-like streaming over the ring dictionary */
    CLzmaDec dec;
    size_t in_pos = 0, out_pos = 0, calls = 0;
    SRes r;
    ELzmaStatus st = LZMA_STATUS_NOT_SPECIFIED;
    LzmaDec_Construct(&dec);
    r = LzmaDec_Allocate(&dec, props, LZMA_PROPS_SIZE, &g_Alloc);
    if (r == SZ_OK) {
      LzmaDec_Init(&dec);
      for (;;) {
        SizeT sl = ns - in_pos, dl = out_size - out_pos;
        if (sl > in_chunk) sl = in_chunk;
        if (dl > out_chunk) dl = out_chunk;
        r = LzmaDec_DecodeToBuf(&dec, out + out_pos, &dl, src + in_pos, &sl, LZMA_FINISH_ANY,
                                &st);
        calls++;
        in_pos += sl;
        out_pos += dl;
        if (r != SZ_OK || st == LZMA_STATUS_FINISHED_WITH_MARK || out_pos == out_size ||
            (sl == 0 && dl == 0))
          break;
      }
      LzmaDec_Free(&dec, &g_Alloc);
    }
    printf("LzmaDec_DecodeToBuf %d %d %zu %zu %08x %zu\n", (int)r, (int)st, out_pos, in_pos,
           (unsigned)CrcCalc(out, out_pos), calls);
  }
  { /* LzmaDec.h dictionary interface, the 7zDec.c:127-171 (SzDecodeLzma) shape:
       dic = the whole output buffer, DecodeToDic(FINISH_END) over look windows of
       IN_CHUNK input bytes */
    CLzmaDec dec;
    size_t in_pos = 0, calls = 0;
    SRes r;
    ELzmaStatus st = LZMA_STATUS_NOT_SPECIFIED;
    LzmaDec_Construct(&dec);
    dec.dicPos = 0;
    memset(out, 0, out_size);
    r = LzmaDec_AllocateProbs(&dec, props, LZMA_PROPS_SIZE, &g_Alloc);
    if (r == SZ_OK) {
      dec.dic = out;
      dec.dicBufSize = out_size;
      LzmaDec_Init(&dec);
      for (;;) {
        SizeT sl = ns - in_pos, pos0 = dec.dicPos;
        if (sl > in_chunk) sl = in_chunk;
        r = LzmaDec_DecodeToDic(&dec, out_size, src + in_pos, &sl, LZMA_FINISH_END, &st);
        calls++;
        in_pos += sl;
        if (r != SZ_OK || dec.dicPos == dec.dicBufSize || (sl == 0 && dec.dicPos == pos0)) break;
      }
      LzmaDec_FreeProbs(&dec, &g_Alloc);
    }
    printf("LzmaDec_DecodeToDic %d %d %zu %zu %08x %zu\n", (int)r, (int)st, (size_t)dec.dicPos,
           in_pos, (unsigned)CrcCalc(out, dec.dicPos), calls);
  }
  free(out);
  free(src);
  free(props);
  return 0;
}
