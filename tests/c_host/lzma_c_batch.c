/*
 * lzma_c_batch.c -- the batch extension from C: n LZMA streams decoded in one
 * launch, (a) from host buffers with LzmaGpu_DecodeBatchHost, (b) device-
 * resident with LzmaGpu_PlanBatchEx + LzmaGpu_DecodeBatchEx on buffers the
 * program allocates itself through the HIP runtime's C API (caller-owned
 * device memory, no allocation inside the decode call), (c) the same buffers
 * decoded time-sliced (LzmaGpu_PlanSliced + LzmaGpu_DecodeBatchSliced, one
 * round per call, LzmaGpu_SlicedActive between rounds).
 * TEST INFRASTRUCTURE: tests/test_c_host.py builds and runs it.
 *
 *   lzma_c_batch host|device|sliced SRC_FILE LENS_FILE PROPS_FILE CAP FINISH
 *
 * SRC_FILE: the streams back to back; LENS_FILE: n little-endian uint64
 * lengths; PROPS_FILE: n x 5 props bytes; every stream gets CAP output bytes.
 * Prints one line per stream: res status destLen srcLen crc32(output).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "lzma_gpu.h"

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

#define HIP_OK(x)                                                      \
  do {                                                                 \
    if ((x) != hipSuccess) {                                           \
      fprintf(stderr, "%s failed at line %d\n", #x, __LINE__);         \
      return 3;                                                        \
    }                                                                  \
  } while (0)

int main(int argc, char **argv) {
  size_t ns = 0, nl = 0, np = 0, n, i, cap, dst_bytes, off = 0;
  unsigned char *src, *lens_b, *props, *dst;
  uint64_t *lens;
  LzmaGpuStreamDesc *descs;
  LzmaGpuResult *res;
  int device;
  if (argc != 7) {
    fprintf(stderr, "usage: %s host|device|sliced SRC LENS PROPS CAP FINISH\n", argv[0]);
    return 2;
  }
  device = strcmp(argv[1], "device") == 0 ? 1 : strcmp(argv[1], "sliced") == 0 ? 2 : 0;
  src = read_file(argv[2], &ns);
  lens_b = read_file(argv[3], &nl);
  props = read_file(argv[4], &np);
  cap = (size_t)strtoull(argv[5], NULL, 10);
  if (!src || !lens_b || !props || nl % 8 != 0 || np != nl / 8 * 5) return 2;
  n = nl / 8;
  lens = (uint64_t *)lens_b;
  descs = (LzmaGpuStreamDesc *)calloc(n ? n : 1, sizeof *descs);
  res = (LzmaGpuResult *)calloc(n ? n : 1, sizeof *res);
  dst_bytes = n * cap;
  dst = (unsigned char *)malloc(dst_bytes ? dst_bytes : 1);
  for (i = 0; i < n; ++i) {
    descs[i].src_off = off;
    descs[i].src_len = lens[i];
    descs[i].dst_off = i * cap;
    descs[i].dst_cap = cap;
    memcpy(descs[i].props, props + 5 * i, 5);
    descs[i].props_size = 5;
    descs[i].finish_mode = (uint8_t)atoi(argv[6]);
    descs[i].kind = LZMA_GPU_KIND_LZMA;
    off += lens[i];
  }
  if (off != ns) return 2;
  CrcGenerateTable();
  if (!device) {
    SRes r = LzmaGpu_DecodeBatchHost(descs, n, src, ns, dst, dst_bytes, res);
    if (r != SZ_OK) {
      fprintf(stderr, "LzmaGpu_DecodeBatchHost: %d %s\n", (int)r, LzmaGpu_LastError());
      return 4;
    }
  } else if (device == 2) {
    /* time-sliced: 4 KiB of output per stream and round, rounds enqueued one
       at a time, the unfinished count read back between them */
    LzmaGpuSlicedPlan sp;
    uint32_t *order = (uint32_t *)malloc((n ? n : 1) * sizeof(uint32_t));
    void *d_src, *d_dst, *d_ws, *d_desc, *d_order, *d_res;
    unsigned r;
    size_t active, prev = n;
    hipStream_t stream;
    if (LzmaGpu_PlanSliced(descs, n, 4096, LZMA_GPU_SLICED_AUTO, order, &sp) != SZ_OK) return 4;
    HIP_OK(hipMalloc(&d_src, ns + 16));
    HIP_OK(hipMalloc(&d_dst, dst_bytes + 16));
    HIP_OK(hipMalloc(&d_ws, sp.workspace_bytes + 16));
    HIP_OK(hipMalloc(&d_desc, n * sizeof *descs + 16));
    HIP_OK(hipMalloc(&d_order, n * sizeof(uint32_t) + 16));
    HIP_OK(hipMalloc(&d_res, n * sizeof *res + 16));
    HIP_OK(hipStreamCreate(&stream));
    HIP_OK(hipMemcpy(d_src, src, ns, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_desc, descs, n * sizeof *descs, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_order, order, n * sizeof(uint32_t), hipMemcpyHostToDevice));
    for (r = 0; r < sp.rounds; ++r) {
      if (LzmaGpu_DecodeBatchSliced(&sp, (const LzmaGpuStreamDesc *)d_desc,
                                    (const uint32_t *)d_order, (const Byte *)d_src, (Byte *)d_dst,
                                    d_ws, (LzmaGpuResult *)d_res, r, 1, (void *)stream) != SZ_OK ||
          LzmaGpu_SlicedActive(&sp, d_ws, r + 1, &active, (void *)stream) != SZ_OK) {
        fprintf(stderr, "sliced round %u: %s\n", r, LzmaGpu_LastError());
        return 4;
      }
      if (active > prev) return 5; /* the unfinished count never rises */
      prev = active;
    }
    if (prev != 0) return 6;
    HIP_OK(hipMemcpy(res, d_res, n * sizeof *res, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(dst, d_dst, dst_bytes, hipMemcpyDeviceToHost));
    HIP_OK(hipStreamDestroy(stream));
    HIP_OK(hipFree(d_src));
    HIP_OK(hipFree(d_dst));
    HIP_OK(hipFree(d_ws));
    HIP_OK(hipFree(d_desc));
    HIP_OK(hipFree(d_order));
    HIP_OK(hipFree(d_res));
    free(order);
  } else {
    LzmaGpuPlan plan;
    uint32_t *order = (uint32_t *)malloc((n ? n : 1) * sizeof(uint32_t));
    void *d_src, *d_dst, *d_ws, *d_desc, *d_order, *d_res;
    hipStream_t stream;
    if (LzmaGpu_PlanBatchEx(descs, n, order, &plan) != SZ_OK) return 4;
    HIP_OK(hipMalloc(&d_src, ns + 16));
    HIP_OK(hipMalloc(&d_dst, dst_bytes + 16));
    HIP_OK(hipMalloc(&d_ws, plan.workspace_bytes + 16));
    HIP_OK(hipMalloc(&d_desc, n * sizeof *descs + 16));
    HIP_OK(hipMalloc(&d_order, n * sizeof(uint32_t) + 16));
    HIP_OK(hipMalloc(&d_res, n * sizeof *res + 16));
    HIP_OK(hipStreamCreate(&stream));
    HIP_OK(hipMemcpy(d_src, src, ns, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_desc, descs, n * sizeof *descs, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_order, order, n * sizeof(uint32_t), hipMemcpyHostToDevice));
    if (LzmaGpu_DecodeBatchEx(&plan, (const LzmaGpuStreamDesc *)d_desc, (const uint32_t *)d_order,
                              (const Byte *)d_src, (Byte *)d_dst, d_ws, (LzmaGpuResult *)d_res,
                              (void *)stream) != SZ_OK) {
      fprintf(stderr, "LzmaGpu_DecodeBatchEx: %s\n", LzmaGpu_LastError());
      return 4;
    }
    HIP_OK(hipStreamSynchronize(stream));
    HIP_OK(hipMemcpy(res, d_res, n * sizeof *res, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(dst, d_dst, dst_bytes, hipMemcpyDeviceToHost));
    HIP_OK(hipStreamDestroy(stream));
    HIP_OK(hipFree(d_src));
    HIP_OK(hipFree(d_dst));
    HIP_OK(hipFree(d_ws));
    HIP_OK(hipFree(d_desc));
    HIP_OK(hipFree(d_order));
    HIP_OK(hipFree(d_res));
    free(order);
  }
  for (i = 0; i < n; ++i)
    printf("%d %d %llu %llu %08x\n", (int)res[i].res, (int)res[i].status,
           (unsigned long long)res[i].dest_len, (unsigned long long)res[i].src_len,
           (unsigned)CrcCalc(dst + i * cap, (size_t)res[i].dest_len));
  free(dst);
  free(res);
  free(descs);
  free(props);
  free(lens_b);
  free(src);
  return 0;
}
