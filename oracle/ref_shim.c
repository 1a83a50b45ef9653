/*
 * ref_shim.c -- TEST INFRASTRUCTURE ONLY.
 *
 * ctypes wrappers around the reference's CONTAINER and filter code (xz and 7z
 * readers, x86 BCJ, CRC-64; the Bra / Delta / Bcj2 / CRC-32 functions are
 * called directly), compiled in place from /root/reference by
 * oracle/Makefile.ref into oracle/_ref/libref.so.  That library carries the
 * only stand-ins of the reference build, confined to it: 7zStream.c's
 * Windows-only TRUE constant (-DTRUE=1) and 7zFile.c's two Windows file
 * openers left to lazy binding (tests/native.py loads it RTLD_LAZY); neither
 * is on any path these wrappers drive.  The LZMA pin is oracle/_ref/
 * libref_lzma.so (ref_lzma_shim.c), built without them.
 *
 * Nothing in the product (lzma-sdk-zliblike_amd/) links or loads this.
 */
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "Alloc.h"
#include "LzmaDec.h"

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

/*
 * xz: XzUnpacker_Code (XzDec.c:604-870) over a whole
 * in-memory file, FINISH_END, in one call with an output buffer of *dst_len
 * bytes.  *done = XzUnpacker_IsStreamWasFinished (XzDec.c:872).  The CRC
 * tables (CrcGenerateTable, Crc64GenerateTable) are built on first use.
 */
#include "7zCrc.h"
#include "Bra.h"
#include "Xz.h"
#include "XzCrc64.h"

static void xz_tables(void) {
  static int done = 0;
  if (!done) { CrcGenerateTable(); Crc64GenerateTable(); done = 1; }
}

int ref_xz_decode(unsigned char *dst, size_t *dst_len, const unsigned char *src,
                  size_t *src_len, int *status, int *done) {
  CXzUnpacker u;
  SizeT dl = *dst_len, sl = *src_len;
  ECoderStatus st = CODER_STATUS_NOT_SPECIFIED;
  SRes res;
  int saved;
  xz_tables();
  saved = quiet_begin();
  XzUnpacker_Create(&u, &g_shim_alloc);
  res = XzUnpacker_Code(&u, dst, &dl, src, &sl, LZMA_FINISH_END, &st);
  *done = XzUnpacker_IsStreamWasFinished(&u) ? 1 : 0;
  XzUnpacker_Free(&u);
  quiet_end(saved);
  *dst_len = dl;
  *src_len = sl;
  *status = (int)st;
  return res;
}

/* x86 BCJ (Bra86.c:11) over a buffer: returns the bytes processed, state in/out. */
size_t ref_x86_convert(unsigned char *data, size_t size, unsigned ip, unsigned *state,
                       int encoding) {
  UInt32 s = *state;
  SizeT r = x86_Convert(data, size, ip, &s, encoding);
  *state = s;
  return r;
}

/* Crc64Calc (XzCrc64.c:30) */
unsigned long long ref_crc64(const unsigned char *data, size_t size) {
  xz_tables();
  return Crc64Calc(data, size);
}

/*
 * 7z archives: SzArEx_Open over an in-memory archive
 * through LookToRead (non-lookahead, as 7zMain.c:326 sets it up), then
 * SzArEx_Extract (7zIn.c:1322) for every file with a fresh folder cache
 * (blockIndex reset after an error, so each file's result stands alone).
 * Files that extract OK are appended to out; file_res / file_size per file;
 * names = the raw UTF-16LE FileNames buffer.  Returns SzArEx_Open's result.
 */
#include "7z.h"

typedef struct {
  ISeekInStream s;
  const Byte *data;
  size_t size, pos;
} ShimMemSeek;

static SRes shim_seek_read(void *pp, void *buf, size_t *size) {
  ShimMemSeek *m = (ShimMemSeek *)pp;
  size_t n = m->size - m->pos;
  if (n > *size) n = *size;
  memcpy(buf, m->data + m->pos, n);
  m->pos += n;
  *size = n;
  return SZ_OK;
}

static SRes shim_seek_seek(void *pp, Int64 *pos, ESzSeek origin) {
  ShimMemSeek *m = (ShimMemSeek *)pp;
  Int64 base = origin == SZ_SEEK_SET ? 0 : (origin == SZ_SEEK_CUR ? (Int64)m->pos : (Int64)m->size);
  Int64 np = base + *pos;
  if (np < 0) return SZ_ERROR_READ;
  m->pos = (size_t)np > m->size ? m->size : (size_t)np;
  *pos = np;
  return SZ_OK;
}

int ref_7z_extract(const unsigned char *arc, size_t size, unsigned char *out, size_t cap,
                   size_t *out_len, int *file_res, unsigned long long *file_size,
                   unsigned *n_files, unsigned max_files, unsigned char *names,
                   size_t names_cap, size_t *names_len) {
  ShimMemSeek ms;
  CLookToRead look;
  CSzArEx db;
  SRes res;
  UInt32 i, block = 0xFFFFFFFF;
  Byte *buf = 0;
  size_t buf_size = 0, pos = 0;
  int saved;
  xz_tables();
  ms.s.Read = shim_seek_read;
  ms.s.Seek = shim_seek_seek;
  ms.data = arc;
  ms.size = size;
  ms.pos = 0;
  LookToRead_CreateVTable(&look, False);
  look.realStream = &ms.s;
  LookToRead_Init(&look);
  saved = quiet_begin();
  SzArEx_Init(&db);
  res = SzArEx_Open(&db, &look.s, &g_shim_alloc, &g_shim_alloc);
  *n_files = 0;
  *names_len = 0;
  if (res == SZ_OK) {
    *n_files = db.db.NumFiles;
    if (db.FileNames.data && db.FileNames.size <= names_cap) {
      memcpy(names, db.FileNames.data, db.FileNames.size);
      *names_len = db.FileNames.size;
    }
    for (i = 0; i < db.db.NumFiles && i < max_files; i++) {
      size_t offset = 0, got = 0;
      SRes r = SzArEx_Extract(&db, &look.s, i, &block, &buf, &buf_size, &offset, &got,
                              &g_shim_alloc, &g_shim_alloc);
      file_res[i] = r;
      file_size[i] = db.db.Files[i].Size;
      if (r == SZ_OK && pos + got <= cap) {
        memcpy(out + pos, buf + offset, got);
        pos += got;
      }
      if (r != SZ_OK) block = 0xFFFFFFFF;
    }
  }
  free(buf);
  SzArEx_Free(&db, &g_shim_alloc);
  quiet_end(saved);
  *out_len = pos;
  return res;
}
